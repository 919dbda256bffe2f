#!/bin/bash
# r02g: tests, timeline with the high-priority prologue + DPP reductions, A/B.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02g; mkdir -p $O
true

for r in 1 2 3; do
  for lib in regloader old_dmaearly_wg4 old_reg_wg4 old_dmaearly old_reg; do
    L=""; [ $lib = product ] || L=tools/scratch/$lib/libmirsha.so
    MIRSHA_AB_LIB=$L timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie > $O/ab_${lib}_$r.jsonl 2>> $O/ab.err || exit 1
  done
  echo ab rep $r done
done
timeout -k 10 240 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.jsonl 2> $O/bench_driver.err || exit 1
echo all done
