#!/bin/bash
# r04f (3): fixed_prio / progress_prio take their priority through
# readfirstlane (scalar branches): fused config 3 vs the round-3 library and
# C1, the traced timeline, the config-3 sequential plan (CU kernel) and the
# config-2 driver command (the request kernel shares progress_prio).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04f; mkdir -p $O
show() { python3 -c "
import json
d=json.loads(open('$1').readlines()[-1]); r=d['roofline']; o=d.get('overlap_cycles') or {}
print('$1', round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms'],4), round(r['frac'],4), d['self_check'], 'ovl', round(o.get('ms_per_step',0),4), round(o.get('avg_launch_ms',0),4))"; }
for i in 5 6; do
for v in new r03lib; do
if [ $v = new ]; then unset MIRSHA_AB_LIB; else export MIRSHA_AB_LIB=tools/scratch/$v/libmirsha.so; fi
timeout -k 10 300 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie > $O/c3_$v.$i.jsonl 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
show $O/c3_$v.$i.jsonl
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie --no-config3-leg > $O/c2_$v.$i.jsonl 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
show $O/c2_$v.$i.jsonl
done
done
unset MIRSHA_AB_LIB
timeout -k 10 300 python -u bench.py --config 3 --pipeline sequential --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie --no-overlap-extra > $O/c3seq_new.jsonl 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
show $O/c3seq_new.jsonl
timeout -k 10 200 python -u tools/trace_queues.py > $O/trace_new2.txt 2>&1 || { tail $O/trace_new2.txt; exit 1; }
grep -v amdgpu.ids $O/trace_new2.txt
echo all done
