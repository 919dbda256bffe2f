#!/bin/bash
# r02o: pipelined host calls with a small first chunk and device-rebuilt
# offsets for gapless requests: pipelined-path tests, full GPU suite, host-call
# timeline, driver bench.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02o; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_host_pipeline.py -x -v --timeout 120 --timeout-method thread > $O/pipe_tests.log 2>&1
rc=$?; tail -4 $O/pipe_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit 1
MIRSHA_STAGE_TRACE=1 timeout -k 10 120 python -u tools/host_call_trace.py 5 > $O/host_trace.json 2> $O/host_trace.err || { tail $O/host_trace.err; exit 1; }
cat $O/host_trace.json
timeout -k 10 240 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 2 > $O/bench_driver.jsonl 2> $O/bench_driver.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_driver.jsonl'));print(d['value'],d['roofline']['frac'],json.dumps(d['pcie_inclusive']))"
echo all done
