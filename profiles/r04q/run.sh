#!/bin/bash
# r04q: a 300 s randomised soak on the final round-4 kernels (source key
# 1715c27c5fdacba4) and the multi-device tests.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04q; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py -q --timeout 120 --timeout-method thread > $O/pytest_multi.log 2>&1 || { tail -40 $O/pytest_multi.log; exit 1; }
tail -1 $O/pytest_multi.log
timeout -k 10 400 python -u tests/soak_gpu.py --seconds 300 --seed 131 > $O/soak.log 2>&1 || { tail -20 $O/soak.log; exit 1; }
tail -1 $O/soak.log
echo all done
