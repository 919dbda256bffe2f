#!/bin/bash
# r02j: GPU tests; config-1 latency with and without the direct small-call
# path; driver bench (PCIe legs with host phases); config 4 host phases.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02j; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -5 $O/gpu_tests.log; [ $rc -eq 0 ] || exit 1
MIRSHA_DIRECT_SMALL=0 timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "nist or lengths or empty or slices" > $O/gpu_tests_nodirect.log 2>&1 || { tail $O/gpu_tests_nodirect.log; exit 1; }
tail -1 $O/gpu_tests_nodirect.log
timeout -k 10 200 python -u bench.py --config 1 > $O/bench_config1.jsonl 2> $O/c1.err || { tail $O/c1.err; exit 1; }
MIRSHA_DIRECT_SMALL=0 timeout -k 10 200 python -u bench.py --config 1 > $O/bench_config1_nodirect.jsonl 2>> $O/c1.err || exit 1
timeout -k 10 240 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 2 > $O/bench_driver.jsonl 2> $O/bench_driver.err || exit 1
timeout -k 10 240 python -u bench.py --config 4 --steps 10 --warmup 2 --cpu-seconds 0 > $O/bench_config4.jsonl 2>> $O/c1.err || exit 1
echo all done
