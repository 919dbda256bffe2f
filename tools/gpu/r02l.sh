#!/bin/bash
# r02l: current product after container restore: timeline (stamps build) of
# the request kernel, then profiles/profile.sh on the driver's command
# (kernel trace + stats, PMC passes).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02l; mkdir -p $O
MIRSHA_AB_LIB=tools/scratch/stamps/libmirsha.so timeout -k 10 180 python -u tools/stamp_run.py $O/stamps > $O/stamps.json 2> $O/stamps.err || { tail -20 $O/stamps.err; exit 1; }
cat $O/stamps.json
timeout -k 10 900 bash profiles/profile.sh r02l > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
cat gpurun_out/prof_r02l/bench_under_trace.jsonl | head -c 600; echo
echo all done
