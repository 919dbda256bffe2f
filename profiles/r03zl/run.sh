#!/bin/bash
# r03zl: per-XCD end times of the config-3 fused launch's last queue over
# consecutive runs (tools/trace_xcd.py).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03zl; mkdir -p $O
timeout -k 10 300 python -u tools/trace_xcd.py 6 > $O/trace_xcd.jsonl 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
cat $O/trace_xcd.jsonl
