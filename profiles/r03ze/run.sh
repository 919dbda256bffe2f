#!/bin/bash
# r03ze: configs 5 and 1 bench lines on the final round-3 tree.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03ze; mkdir -p $O
timeout -k 10 400 python -u bench.py --config 5 --steps 5 --warmup 2 --cpu-seconds 3 > $O/bench_c5.jsonl 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
timeout -k 10 300 python -u bench.py --config 1 --steps 20 --warmup 5 --cpu-seconds 2 > $O/bench_c1.jsonl 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
for f in $O/bench_c5.jsonl $O/bench_c1.jsonl; do python3 -c "
import json
d=json.loads(open('$f').readlines()[-1]); r=d.get('roofline') or {}
print('$f', d['value'], d['ms_per_step'], r.get('frac'), d.get('self_check'), (d.get('cpu_baseline') or {}).get('value'))"; done
echo all done
