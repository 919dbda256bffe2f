#!/bin/bash
# r03z: fused-launch tiles loading by LDS-DMA (product build) vs the
# register-staged loader (tools/scratch/nodma: the r03x build), config 3,
# alternating; fused / overlap parity tests and a 60 s soak on the DMA build.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03z; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "overlap or fused or split or config3" -x -q --timeout 300 --timeout-method thread > $O/pytest_fused.log 2>&1 || { tail -40 $O/pytest_fused.log; exit 1; }
tail -1 $O/pytest_fused.log
for i in 1 2; do
for v in dma nodma; do
if [ $v = nodma ]; then export MIRSHA_AB_LIB=tools/scratch/nodma/libmirsha.so; else unset MIRSHA_AB_LIB; fi
timeout -k 10 300 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 1 --no-pcie > $O/bench_c3_$v.$i.jsonl 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench_c3_$v.$i.jsonl').readlines()[-1]); o=d.get('overlap_cycles') or {}
print('$v', $i, 'fused step', round(d['ms_per_step'],4), 'kern', round(d['roofline']['avg_launch_ms'],4), 'frac', round(d['roofline']['frac'],4), 'overlap step', round(o.get('ms_per_step',0),4), 'kern', round(o.get('avg_launch_ms',0),4), d['self_check'])"
done
done
unset MIRSHA_AB_LIB
timeout -k 10 150 python -u tests/soak_gpu.py --seconds 60 --seed 53 > $O/soak.log 2>&1 || { tail -20 $O/soak.log; exit 1; }
tail -1 $O/soak.log
echo all done
