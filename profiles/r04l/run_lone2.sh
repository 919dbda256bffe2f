#!/bin/bash
# r04l (lone 2): per-block time of the last queue's lone stretch in the full
# config-3 fused run (from the per-SIMD tile ends), lone form on.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04l5; mkdir -p $O
export MIRSHA_AB=1
timeout -k 10 200 python -u tools/trace_queues.py > $O/trace.txt 2>&1 || { tail $O/trace.txt; exit 1; }
grep -E "^queue [0-9]: [0-9]+ tiles|list groups|lone" $O/trace.txt
echo all done
