#!/bin/bash
# r03e: fused config-3 timeline on the current head (queue ends, chain waits).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03e; mkdir -p $O
timeout -k 10 200 python -u tools/trace_fused.py 3 0 > $O/trace_c3.jsonl 2> $O/trace.err || { tail -20 $O/trace.err; exit 1; }
cat $O/trace_c3.jsonl
