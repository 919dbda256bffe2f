#!/bin/bash
# r05ai (A/B): config 5 with the round-3 library (e679b48, tools/ab_r03,
# removed after the run; loaded through MIRSHA_AB_LIB) vs the final one, on
# one box, alternated.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05ai3; mkdir -p $O
for r in 1 2; do
  MIRSHA_AB=1 MIRSHA_AB_LIB=tools/ab_r03/libmirsha.so timeout -k 10 400 python -u bench.py --config 5 --steps 5 --warmup 2 --cpu-seconds 1 --no-pcie >> $O/c5_r03lib.jsonl 2>> $O/err.txt || exit 1
  timeout -k 10 400 python -u bench.py --config 5 --steps 5 --warmup 2 --cpu-seconds 1 --no-pcie >> $O/c5_final.jsonl 2>> $O/err.txt || exit 1
done
echo done
