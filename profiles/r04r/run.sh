#!/bin/bash
# r04r: the lone-stretch knobs' parity test (every on/off combination) and
# the full GPU suite once more on the final tree.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04r; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
grep -c PASSED $O/pytest_gpu.log || true
echo all done
