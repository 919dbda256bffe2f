#!/bin/bash
# r03zd: config-3 overlapped runs with every slot of a tile-block SIMD
# hosting one split-tile segment (product build) vs the last queue's waves
# hosting them (MIRSHA_FUSED_OVERLAP_SPLIT=last), alternating; fused /
# overlap parity tests, a 60 s soak, and the overlapped-launch timeline.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03zd; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "overlap or fused or split or config3" -x -q --timeout 300 --timeout-method thread > $O/pytest_fused.log 2>&1 || { tail -40 $O/pytest_fused.log; exit 1; }
tail -1 $O/pytest_fused.log
for i in 1 2 3; do
for v in all last; do
MIRSHA_AB=1 MIRSHA_FUSED_OVERLAP_SPLIT=$v timeout -k 10 300 python -u tools/exp_overlap.py 30 > $O/forms_$v.$i.jsonl 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
echo "$v $i $(cat $O/forms_$v.$i.jsonl)"
done
done
timeout -k 10 150 python -u tests/soak_gpu.py --seconds 60 --seed 61 > $O/soak.log 2>&1 || { tail -20 $O/soak.log; exit 1; }
tail -1 $O/soak.log
timeout -k 10 200 python -u tools/trace_overlap.py 40 > $O/trace_overlap.jsonl 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
echo all done
