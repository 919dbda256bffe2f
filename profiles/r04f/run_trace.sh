#!/bin/bash
# r04f (2): fused config-3 timelines (tools/trace_queues.py) of this build and
# of C1 (the build without the remap block).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04f; mkdir -p $O
timeout -k 10 200 python -u tools/trace_queues.py > $O/trace_new.txt 2>&1 || { tail $O/trace_new.txt; exit 1; }
cat $O/trace_new.txt
MIRSHA_AB_LIB=tools/scratch/bisC1/libmirsha.so timeout -k 10 200 python -u tools/trace_queues.py > $O/trace_c1.txt 2>&1 || { tail $O/trace_c1.txt; exit 1; }
cat $O/trace_c1.txt
