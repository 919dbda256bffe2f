#!/bin/bash
# r04l (lone): one tile wave per SIMD from the start (MIRSHA_FUSED_PACE=1,
# 1,006 config-3 tiles): how fast does a LONE wave run its 65 blocks, in the
# latency round form vs the throughput form?
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04l4; mkdir -p $O
export MIRSHA_AB=1 MIRSHA_FUSED_PACE=1
for lf in 1 0; do
MIRSHA_FUSED_LONE_FORM=$lf timeout -k 10 200 python -u tools/trace_queues.py 64384 > $O/trace_lf$lf.txt 2>&1 || { tail $O/trace_lf$lf.txt; exit 1; }
grep -E "^queue [0-9]: [0-9]+ tiles|list groups|lone-wave" $O/trace_lf$lf.txt
done
echo all done
