#!/bin/bash
# r02h: GPU tests (config-4 full scale, async lifetime, uneven absorb), A/B of
# the register loader's prologue / workgroup forms, timeline, driver bench.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02h; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --durations=8 > $O/gpu_tests.log 2>&1
rc=$?; tail -15 $O/gpu_tests.log; [ $rc -eq 0 ] || exit 1
MIRSHA_AB_LIB=tools/scratch/stamps/libmirsha.so timeout -k 10 180 python -u tools/stamp_run.py $O/stamps > $O/stamps.json 2> $O/stamps.err || { tail -20 $O/stamps.err; exit 1; }
cat $O/stamps.json
for r in 1 2 3; do
  for lib in product oldpro prio wg4 r1form; do
    L=""; [ $lib = product ] || L=tools/scratch/$lib/libmirsha.so
    MIRSHA_AB_LIB=$L timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie > $O/ab_${lib}_$r.jsonl 2>> $O/ab.err || exit 1
  done
  echo ab rep $r done
done
timeout -k 10 240 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.jsonl 2> $O/bench_driver.err || exit 1
timeout -k 10 240 python -u bench.py --config 4 --steps 10 --warmup 2 --cpu-seconds 3 > $O/bench_config4.jsonl 2>> $O/ab.err || exit 1
echo all done
