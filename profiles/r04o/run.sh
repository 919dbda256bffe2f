#!/bin/bash
# r04o: fused tile waves set their block priority right after the wait for the
# block's DMA (the overlapped launch's progress ranks then pay hipcc's LDS-DMA
# wait where it is free) and overlapped launches keep one block in flight.
# Same-box A/B against the r04n library (MIRSHA_AB_LIB, tools/scratch/r04nlib):
# config-3 fused steps and overlapped cycles; config-2 overlapped cycles; the
# fused parity tests.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04o; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "fused or full_size or pipeline or overlap" -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
export MIRSHA_AB=1
for i in 1 2 3; do
for lib in new old; do
if [ $lib = old ]; then export MIRSHA_AB_LIB=$PWD/tools/scratch/r04nlib/libmirsha.so; else unset MIRSHA_AB_LIB; fi
timeout -k 10 300 python -u bench.py --config 3 --pipeline fused --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie --no-config3-leg > $O/bench_c3_$lib.$i.jsonl 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
timeout -k 10 300 python -u bench.py --config 2 --pipeline overlap --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie --no-config3-leg > $O/bench_c2ovl_$lib.$i.jsonl 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench_c3_$lib.$i.jsonl').readlines()[-1]); r=d['roofline']; o=d.get('overlap_cycles') or {}
e=json.loads(open('$O/bench_c2ovl_$lib.$i.jsonl').readlines()[-1])
print('$lib', $i, 'c3 step', round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms'],4), 'ovl', round(o.get('ms_per_step',0),4), round(o.get('avg_launch_ms',0),4), 'check', d['self_check'], '| c2 ovl', round(e['ms_per_step'],4), round(e['roofline']['avg_launch_ms']*1e3,1), e['self_check'])"
done
done
echo all done
