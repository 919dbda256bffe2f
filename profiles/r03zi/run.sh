#!/bin/bash
# r03zi: the driver's round-end commands on the final round-3 head: the -m gpu
# suite, smoke(), and bench.py with no flags (N=1 defaults).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03zi; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench.jsonl 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench.jsonl').readlines()[-1]); r=d['roofline']; o=d.get('overlap_cycles') or {}; c=d.get('cpu_baseline') or {}
print(round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],4), 'ms', 'kern', round(r['avg_launch_ms']*1e3,1), 'frac', round(r['frac'],4), 'traffic', r.get('traffic'), 'check', d['self_check'], 'overlap', round(o.get('ms_per_step',0),4), 'cpu', c.get('value'))"
echo all done
