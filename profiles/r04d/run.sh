#!/bin/bash
# r04d: bisect the config-3 fused-step regression (1.07 ms vs round 3's 0.80):
# this build; A = without the placement remap's barrier; B = without the
# split-tile skip test; the round-3 library.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04d; mkdir -p $O
show() { python3 -c "
import json
d=json.loads(open('$1').readlines()[-1]); r=d['roofline']; o=d.get('overlap_cycles') or {}
print('$1', round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms'],4), d['self_check'], 'ovl', round(o.get('ms_per_step',0),4), round(o.get('avg_launch_ms',0),4))"; }
for i in 1 2; do
for v in new bisA bisB r03lib; do
if [ $v = new ]; then unset MIRSHA_AB_LIB; else export MIRSHA_AB_LIB=tools/scratch/$v/libmirsha.so; fi
timeout -k 10 300 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie > $O/c3_$v.$i.jsonl 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
show $O/c3_$v.$i.jsonl
done
done
echo all done
