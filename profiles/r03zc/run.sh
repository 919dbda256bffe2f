#!/bin/bash
# r03zc: timelines of the final config-3 launches: the fused run
# (tools/trace_fused.py: queue ends, chain progress) and the overlapped run
# (tools/trace_overlap.py).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03zc; mkdir -p $O
timeout -k 10 200 python -u tools/trace_fused.py 3 0 > $O/trace_fused.jsonl 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
timeout -k 10 200 python -u tools/trace_overlap.py 40 > $O/trace_overlap.jsonl 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
echo all done
