#!/bin/bash
# r03u: config 3 fused step, split-tile segments hosted by the first queue's
# waves after their own tile (first, new default) vs interleaved in the last
# queue's tiles (last, r03n-r03s), alternating; fused / overlap parity tests.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03u; mkdir -p $O
for i in 1 2; do
for h in first last; do
MIRSHA_AB=1 MIRSHA_FUSED_SPLIT_HOST=$h timeout -k 10 300 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 1 --no-pcie > $O/bench_c3_$h.$i.jsonl 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench_c3_$h.$i.jsonl').readlines()[-1]); o=d.get('overlap_cycles') or {}
print('$h', $i, 'fused step', round(d['ms_per_step'],4), 'kern', round(d['roofline']['avg_launch_ms'],4), 'frac', round(d['roofline']['frac'],4), 'overlap step', round(o.get('ms_per_step',0),4), d['self_check'])"
done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "overlap or fused or split or config3" -x -q --timeout 300 --timeout-method thread > $O/pytest_fused.log 2>&1 || { tail -40 $O/pytest_fused.log; exit 1; }
tail -1 $O/pytest_fused.log
echo all done
