#!/bin/bash
# r03l: launch forms, block-batched first claims (product build) vs the
# static first-tile build (tools/scratch/static, HEAD~), alternating.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03l; mkdir -p $O
for i in 1 2; do
timeout -k 10 200 python -u tools/exp_overlap.py 30 | sed 's/^/batched /' >> $O/forms.txt 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
MIRSHA_AB_LIB=tools/scratch/static/libmirsha.so timeout -k 10 200 python -u tools/exp_overlap.py 30 | sed 's/^/static /' >> $O/forms.txt 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
done
cat $O/forms.txt
