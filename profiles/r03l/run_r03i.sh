#!/bin/bash
# r03i: config 5 at one rank's full shard (tests/test_gpu_config5.py).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03i; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_config5.py -x -v --timeout 300 --timeout-method thread --durations=3 > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -8 $O/pytest.log
