#!/bin/bash
# r04f: bisect the fused config-3 step again (still 1.07 ms in r04e with the
# remapped identity readfirstlane'd).  First pass (results kept): C1 =
# without the remap block 0.80-0.81 ms, C2 = without the flag-based
# split-tile skip 1.07, C3 = without both 0.82, round-3 library 0.80: the
# remap block's mere presence.  Second pass: the remap rewritten with scalar
# control flow (readfirstlane on every LDS value) vs C1 vs round 3, then the
# fused / split / placement tests.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04f; mkdir -p $O
show() { python3 -c "
import json
d=json.loads(open('$1').readlines()[-1]); r=d['roofline']; o=d.get('overlap_cycles') or {}
print('$1', round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms'],4), d['self_check'], 'ovl', round(o.get('ms_per_step',0),4), round(o.get('avg_launch_ms',0),4))"; }
for i in 3 4; do
for v in new bisC1 r03lib; do
if [ $v = new ]; then unset MIRSHA_AB_LIB; else export MIRSHA_AB_LIB=tools/scratch/$v/libmirsha.so; fi
timeout -k 10 300 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie > $O/c3_$v.$i.jsonl 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
show $O/c3_$v.$i.jsonl
done
done
unset MIRSHA_AB_LIB
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "split or placement or fused or overlap or config3" -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
echo all done
