#!/bin/bash
# r03zf: cascade plan (one launch: config-2 requests + their batch chains):
# parity, then same-box A/B against the sequential plan (request kernel,
# then batch kernel), alternating.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03zf; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu \
  -k "cascade or pipeline_device_full_size or irregular_lists" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for r in 1 2; do
  for m in sequential cascade; do
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie --pipeline $m \
      > $O/bench_${m}_$r.jsonl 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
  done
done
for f in $O/bench_*.jsonl; do python3 -c "
import json
d=json.loads(open('$f').readlines()[-1]); r=d.get('roofline') or {}; o=d.get('overlap_cycles') or {}
print('$f', round(d['value']/1e9,3), round(d['ms_per_step'],4), r.get('kernel'), r.get('frac'), d.get('self_check'), o.get('ms_per_step'))"; done
echo all done
