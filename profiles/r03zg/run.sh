#!/bin/bash
# r03zg: config-2 overlapped cycles, A/B of the chain waves' grid position
# (MIRSHA_OVERLAP_CHAIN_AT, thousandths of the tile count: 0 = first, the
# product; 1000 = after every tile), alternating, plus parity at two positions.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03zg; mkdir -p $O
export MIRSHA_AB=1
for at in 500 1000; do
  MIRSHA_OVERLAP_CHAIN_AT=$at timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 \
    --timeout-method thread -m gpu -k "overlap" > $O/tests_$at.log 2>&1 || { tail -30 $O/tests_$at.log; exit 1; }
  tail -1 $O/tests_$at.log
done
for r in 1 2; do
  for at in 0 500 800 900 1000; do
    MIRSHA_OVERLAP_CHAIN_AT=$at timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --cpu-seconds 0 --no-pcie \
      --pipeline overlap > $O/bench_${at}_$r.jsonl 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
  done
done
for f in $O/bench_*.jsonl; do python3 -c "
import json
d=json.loads(open('$f').readlines()[-1]); r=d.get('roofline') or {}
print('$f', round(d['value']/1e9,3), round(d['ms_per_step'],4), r.get('kernel'), r.get('frac'), d.get('self_check'))"; done
echo all done
