#!/bin/bash
# r02i: GPU tests on the staged host path; benches of configs 1, 2 (driver
# command, PCIe legs), 3, 4.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02i; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -5 $O/gpu_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -u bench.py --config 1 > $O/bench_config1.jsonl 2> $O/c1.err || { tail $O/c1.err; exit 1; }
timeout -k 10 240 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.jsonl 2> $O/bench_driver.err || exit 1
timeout -k 10 200 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 3 > $O/bench_config3.jsonl 2>> $O/ab.err || exit 1
timeout -k 10 240 python -u bench.py --config 4 --steps 10 --warmup 2 --cpu-seconds 3 > $O/bench_config4.jsonl 2>> $O/ab.err || exit 1
echo all done
