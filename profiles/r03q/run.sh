#!/bin/bash
# r03q: config-3 overlapped launch, tile waves at priorities by progress rank
# (balance, new default) vs the request kernel's progress priorities
# (progress, round 3's product), alternating on one box; timeline of the
# balanced launch; fused / overlap parity tests; config-3 bench line.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03q; mkdir -p $O
timeout -k 10 300 python -u tools/exp_overlap.py 30 balance progress > $O/forms.jsonl 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
cat $O/forms.jsonl
timeout -k 10 200 python -u tools/trace_overlap.py 40 > $O/trace_overlap.jsonl 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "overlap or fused or split or config3" -x -q --timeout 300 --timeout-method thread > $O/pytest_fused.log 2>&1 || { tail -40 $O/pytest_fused.log; exit 1; }
tail -1 $O/pytest_fused.log
timeout -k 10 300 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 3 > $O/bench_c3.jsonl 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench_c3.jsonl').readlines()[-1]); r=d['roofline']; o=d.get('overlap_cycles') or {}
print('c3', round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms']*1e3,1), 'frac', round(r['frac'],4), 'check', d['self_check'], 'overlap', round(o.get('ms_per_step',0),4), round(o.get('frac',0),4))"
echo all done
