#!/bin/bash
# r02v: per-block issue-priority tables for the request kernel (A/B, 3 reps).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02v; mkdir -p $O
for r in 1 2 3; do
  for lib in product p00000 p31000 p32000 p32110 p32101 p33100 p32210; do
    L=""; [ $lib = product ] || L=tools/scratch/$lib/libmirsha.so
    MIRSHA_AB_LIB=$L timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie > $O/ab_${lib}_$r.jsonl 2>> $O/ab.err || exit 1
  done
done
python3 tools/abview.py $O/ab_*.jsonl || true
echo all done
