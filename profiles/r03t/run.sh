#!/bin/bash
# r03t: the CU-block request kernel (config 3's sequential plan: 4,096 tiles,
# 4 waves per SIMD) at progress priorities (variant 10, product) vs
# priorities by progress rank (variant 12), alternating on one box.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03t; mkdir -p $O
for i in 1 2; do
for v in 10 12; do
timeout -k 10 300 python -u bench.py --config 3 --pipeline sequential --variant $v --steps 20 --warmup 5 --cpu-seconds 1 --no-pcie > $O/bench_c3seq_v$v.$i.jsonl 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench_c3seq_v$v.$i.jsonl').readlines()[-1]); r=d['roofline']
print('v$v', $i, 'step', round(d['ms_per_step'],4), 'request kernel', round(r['avg_launch_ms'],4), 'frac', round(r['frac'],4), d['self_check'])"
done
done
echo all done
