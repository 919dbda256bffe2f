#!/bin/bash
# r03zk: config-3 fused step, A/B of which last-queue waves host the split
# tiles' segments (MIRSHA_FUSED_HOST_REVERSE=1: the last tile blocks'
# waves, i.e. those holding the latest positions; product 0: the first),
# alternating, after parity of the fused tests with the knob on.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03zk; mkdir -p $O
export MIRSHA_AB=1
MIRSHA_FUSED_HOST_REVERSE=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 \
  --timeout-method thread -m gpu -k "fused or full_size or overlap" > $O/tests_rev.log 2>&1 || { tail -30 $O/tests_rev.log; exit 1; }
tail -1 $O/tests_rev.log
for r in 1 2 3; do
  for v in 0 1; do
    MIRSHA_FUSED_HOST_REVERSE=$v timeout -k 10 300 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 \
      --no-pcie > $O/bench_${v}_$r.jsonl 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
  done
done
for f in $O/bench_*.jsonl; do python3 -c "
import json
d=json.loads(open('$f').readlines()[-1]); r=d.get('roofline') or {}; o=d.get('overlap_cycles') or {}
print('$f', round(d['ms_per_step'],4), r.get('frac'), d.get('self_check'), round(o.get('ms_per_step',0),4))"; done
echo all done
