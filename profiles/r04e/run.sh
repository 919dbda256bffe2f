#!/bin/bash
# r04e: the fused launch with the remapped identity made scalar again
# (readfirstlane) and the split-tile skip on the segment flags, vs the
# round-3 library; the CU-block request kernel's new product form (LDS-DMA,
# variant 0) vs the round-3 form (variant 12); fused / split / placement /
# CU-variant parity tests; diagnostics 14 (product form without its block
# loads; digests invalid) and 15 (without per-block priorities).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04e; mkdir -p $O
show() { python3 -c "
import json
d=json.loads(open('$1').readlines()[-1]); r=d['roofline']; o=d.get('overlap_cycles') or {}
print('$1', round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms'],4), d['self_check'], 'ovl', round(o.get('ms_per_step',0),4), round(o.get('avg_launch_ms',0),4))"; }
for i in 1 2; do
for v in new r03lib; do
if [ $v = new ]; then unset MIRSHA_AB_LIB; else export MIRSHA_AB_LIB=tools/scratch/$v/libmirsha.so; fi
timeout -k 10 300 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie > $O/c3_$v.$i.jsonl 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
show $O/c3_$v.$i.jsonl
done
done
unset MIRSHA_AB_LIB
export MIRSHA_AB=1
k=0
for v in 0 12 14 15 0; do
k=$((k+1))
MIRSHA_PROBE_WAVES=4 timeout -k 10 300 python -u bench.py --config 3 --pipeline sequential --variant $v --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie --no-overlap-extra > $O/c3seq_v$v.$k.jsonl 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
show $O/c3seq_v$v.$k.jsonl
python3 -c "
import json
d=json.loads(open('$O/c3seq_v$v.$k.jsonl').readlines()[-1]); m=d['roofline']['measured_peak']
print('   probe(4 waves/SIMD) cycles/wave-compression', round(m['cycles_per_wave_compression']), 'kernel frac of probe', round(m['frac'],3))"
done
unset MIRSHA_AB
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "split or placement or fused or overlap or config3 or cu" -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
echo all done
