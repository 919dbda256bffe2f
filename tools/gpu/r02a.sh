#!/bin/bash
# r02a: GPU tests, the driver's bench command, same-box A/B of the K-via-s_mov
# rounds + aligned loads against the round-1 form, then the rocprof passes.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02a; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 240 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.jsonl 2> $O/bench_driver.err || exit 1
echo driver bench done
for r in 1 2 3; do
  for lib in product r1form noaligned; do
    L=""; [ $lib = product ] || L=tools/scratch/$lib/libmirsha.so
    MIRSHA_AB_LIB=$L timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie > $O/ab_${lib}_$r.jsonl 2>> $O/ab.err || exit 1
  done
  echo ab rep $r done
done
timeout -k 10 120 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie > $O/bench_config3.jsonl 2>> $O/ab.err || exit 1
bash profiles/profile.sh r02a || exit 1
echo all done
