#!/bin/bash
# r03h: config-3 launch forms on one box (tools/exp_overlap.py).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03h; mkdir -p $O
timeout -k 10 200 python -u tools/exp_overlap.py 20 > $O/forms.jsonl 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
cat $O/forms.jsonl
