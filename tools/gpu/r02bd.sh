#!/bin/bash
# r02bd: final validation of round 2's tree: full -m gpu suite, smoke, the
# driver's bench command.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02bd; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.jsonl 2> $O/bench.err || exit 1
python3 -c "import json; d=json.loads(open('$O/bench.jsonl').readlines()[-1]); r=d['roofline']; print(round(d['value']/1e9,3), round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms']*1e3,1), 'frac', round(r['frac'],4), 'traffic', r.get('traffic'), 'check', d['self_check'], 'cpu', d['cpu_baseline']['value'])"
echo all done
