#!/bin/bash
# r02k: batch-pass forms for config 2 (chain kernel vs producer/consumer pairs
# for all 820 groups), 3 reps each, plus GPU tests of the validation changes.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02k; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit 1
for r in 1 2 3; do
  timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie > $O/ab_chain_$r.jsonl 2>> $O/ab.err || exit 1
  MIRSHA_PAIR_MAX_GROUPS=1024 timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie > $O/ab_pair_$r.jsonl 2>> $O/ab.err || exit 1
done
timeout -k 10 240 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 2 > $O/bench_driver.jsonl 2> $O/bench_driver.err || exit 1
echo all done
