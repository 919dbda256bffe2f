#!/bin/bash
# r02bn: the -m gpu suite with the 15 s soak test included, as the driver runs it.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02bn; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python -u -m pytest tests/test_gpu_soak.py -m gpu -q --durations=1 > $O/soak_test.log 2>&1 || { tail -30 $O/soak_test.log; exit 1; }
grep -E "passed|s call" $O/soak_test.log
