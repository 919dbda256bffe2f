#!/bin/bash
# r02c: request-kernel timeline (stamps build) on config 2.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02c; mkdir -p $O
MIRSHA_AB_LIB=tools/scratch/stamps/libmirsha.so timeout -k 10 180 python -u tools/stamp_run.py $O/stamps > $O/stamps.json 2> $O/stamps.err || { tail -20 $O/stamps.err; exit 1; }
cat $O/stamps.json
