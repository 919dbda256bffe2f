#!/bin/bash
# r03s: config 3, fused-launch retirement counted per workgroup (product
# build) vs per wave (tools/scratch/bal: the r03q/r03r build), alternating.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03s; mkdir -p $O
for i in 1 2; do
for v in block wave; do
if [ $v = wave ]; then export MIRSHA_AB_LIB=tools/scratch/bal/libmirsha.so; else unset MIRSHA_AB_LIB; fi
timeout -k 10 300 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 1 --no-pcie > $O/bench_c3_$v.$i.jsonl 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench_c3_$v.$i.jsonl').readlines()[-1]); o=d.get('overlap_cycles') or {}
print('$v', $i, 'fused', round(d['ms_per_step'],4), 'kern', round(d['roofline']['avg_launch_ms'],4), 'overlap step', round(o.get('ms_per_step',0),4), 'kern', round(o.get('avg_launch_ms',0),4), 'frac', round(o.get('frac',0),4), d['self_check'])"
done
done
unset MIRSHA_AB_LIB
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "overlap or fused or split or config3" -x -q --timeout 300 --timeout-method thread > $O/pytest_fused.log 2>&1 || { tail -40 $O/pytest_fused.log; exit 1; }
tail -1 $O/pytest_fused.log
echo all done
