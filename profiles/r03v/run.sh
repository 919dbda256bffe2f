#!/bin/bash
# r03v: config 3 fused step with x more of the last queue's tiles split
# (MIRSHA_FUSED_EXTRA_SPLIT, first-queue segment hosts), x = 0 / 128 / 256,
# alternating; fused parity tests at the best setting.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03v; mkdir -p $O
for i in 1 2; do
for x in 0 128 256; do
MIRSHA_AB=1 MIRSHA_FUSED_EXTRA_SPLIT=$x timeout -k 10 300 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 1 --no-pcie > $O/bench_c3_x$x.$i.jsonl 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench_c3_x$x.$i.jsonl').readlines()[-1]); o=d.get('overlap_cycles') or {}
print('x$x', $i, 'fused step', round(d['ms_per_step'],4), 'kern', round(d['roofline']['avg_launch_ms'],4), 'frac', round(d['roofline']['frac'],4), 'overlap step', round(o.get('ms_per_step',0),4), d['self_check'])"
done
done
echo all done
