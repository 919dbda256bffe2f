#!/bin/bash
# r03zb: LDS-DMA block loads in the request kernel too (product build) vs
# the request kernel's register-staged loads (tools/scratch/base: head
# 2a... with DMA only in the fused launch): the -m gpu suite on the DMA
# build, then config 2 (the driver's command) alternating x3 and config 3.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03zb; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for i in 1 2 3; do
for v in dma base; do
if [ $v = base ]; then export MIRSHA_AB_LIB=tools/scratch/base/libmirsha.so; else unset MIRSHA_AB_LIB; fi
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 1 --no-pcie > $O/bench_c2_$v.$i.jsonl 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench_c2_$v.$i.jsonl').readlines()[-1]); r=d['roofline']
print('$v', $i, 'step', round(d['ms_per_step'],4), 'request kernel', round(r['avg_launch_ms']*1e3,2), 'frac', round(r['frac'],4), 'probe', round(r.get('measured_peak',{}).get('frac',0),4), d['self_check'])"
done
done
unset MIRSHA_AB_LIB
timeout -k 10 300 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 1 --no-pcie > $O/bench_c3.jsonl 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench_c3.jsonl').readlines()[-1]); o=d.get('overlap_cycles') or {}
print('c3 fused', round(d['ms_per_step'],4), 'overlap', round(o.get('ms_per_step',0),4), d['self_check'])"
echo all done
