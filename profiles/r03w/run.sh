#!/bin/bash
# r03w: config 3 fused step by split-tile segment host (MIRSHA_FUSED_SPLIT_HOST:
# 3 = interleaved in the last queue's tiles, product; 0 / 1 / 2 = queue q's
# waves after their own tile) and extra last-queue splits
# (MIRSHA_FUSED_EXTRA_SPLIT), alternating on one box; then the CU-block
# request kernel (config 3 sequential plan) at progress priorities (variant
# 10) vs by progress rank (12); fused / overlap parity tests.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03w; mkdir -p $O
for i in 1 2; do
for hx in 3:0 0:0 1:0 2:0 1:128; do
h=${hx%%:*}; x=${hx##*:}
MIRSHA_AB=1 MIRSHA_FUSED_SPLIT_HOST=$h MIRSHA_FUSED_EXTRA_SPLIT=$x timeout -k 10 300 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 1 --no-pcie > $O/bench_c3_h${h}x$x.$i.jsonl 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench_c3_h${h}x$x.$i.jsonl').readlines()[-1]); o=d.get('overlap_cycles') or {}
print('host $h extra $x', $i, 'fused step', round(d['ms_per_step'],4), 'kern', round(d['roofline']['avg_launch_ms'],4), 'frac', round(d['roofline']['frac'],4), 'overlap step', round(o.get('ms_per_step',0),4), d['self_check'])"
done
done
for i in 1 2; do
for v in 10 12; do
timeout -k 10 300 python -u bench.py --config 3 --pipeline sequential --variant $v --steps 20 --warmup 5 --cpu-seconds 1 --no-pcie > $O/bench_c3seq_v$v.$i.jsonl 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench_c3seq_v$v.$i.jsonl').readlines()[-1]); r=d['roofline']
print('variant $v', $i, 'step', round(d['ms_per_step'],4), 'request kernel', round(r['avg_launch_ms'],4), 'frac', round(r['frac'],4), d['self_check'])"
done
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "overlap or fused or split or config3" -x -q --timeout 300 --timeout-method thread > $O/pytest_fused.log 2>&1 || { tail -40 $O/pytest_fused.log; exit 1; }
tail -1 $O/pytest_fused.log
echo all done
