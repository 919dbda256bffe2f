#!/bin/bash
# r03r: config-3 overlapped cycles in the bench line, balance (default) vs
# progress priorities, alternating bench runs on one box.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03r; mkdir -p $O
for i in 1 2; do
for m in balance progress; do
MIRSHA_AB=1 MIRSHA_FUSED_OVERLAP_PRIO=$m timeout -k 10 300 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 1 --no-pcie > $O/bench_c3_$m.$i.jsonl 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench_c3_$m.$i.jsonl').readlines()[-1]); o=d.get('overlap_cycles') or {}
print('$m', $i, 'fused', round(d['ms_per_step'],4), 'overlap step', round(o.get('ms_per_step',0),4), 'kern', round(o.get('avg_launch_ms',0),4), 'frac', round(o.get('frac',0),4))"
done
done
echo all done
