#!/bin/bash
# r03m: fused config 3: the last queue's priority raised to 1 at block B (A/B).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03m; mkdir -p $O
for r in 1 2; do
for B in 0 15 30 45 55; do
  MIRSHA_AB=1 MIRSHA_FUSED_LAST_RAISE=$B timeout -k 10 200 python -u tools/exp_overlap.py 20 | sed "s/^/raise=$B /" >> $O/forms.txt 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
done
done
cat $O/forms.txt
