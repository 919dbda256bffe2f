#!/bin/bash
# r02b: GPU tests on the LDS-DMA loader, driver bench command, same-box A/B
# against the register-staged loader and the round-1 form.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 240 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.jsonl 2> $O/bench_driver.err || exit 1
echo driver bench done
for r in 1 2 3; do
  for lib in product regloader r1form; do
    L=""; [ $lib = product ] || L=tools/scratch/$lib/libmirsha.so
    MIRSHA_AB_LIB=$L timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie > $O/ab_${lib}_$r.jsonl 2>> $O/ab.err || exit 1
  done
  echo ab rep $r done
done
echo all done
