#!/bin/bash
# r02y: issue-yield patterns of the request kernel's rounds (A/B, 3 reps):
# product (s_nop after every 4-cycle op) vs only after the rotates, only
# after the 3-input adds, after every second 4-cycle op.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02y2; mkdir -p $O
for r in 1 2 3; do
  for lib in product yhalf ythird yquarter yrothalf; do
    L=""; [ $lib = product ] || L=tools/scratch/$lib/libmirsha.so
    MIRSHA_AB_LIB=$L timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie > $O/ab_${lib}_$r.jsonl 2>> $O/ab.err || exit 1
  done
done
python3 tools/abview.py $O/ab_*.jsonl || true
echo all done
