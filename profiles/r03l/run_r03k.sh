#!/bin/bash
# r03k: block-batched first claims: fused/overlap parity, then launch forms.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03k; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dedup_async.py -x -q --timeout 120 --timeout-method thread -k "split or fused or full_size or overlap or watchdog or dedup or async or poll" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u tools/exp_overlap.py 20 > $O/forms.jsonl 2> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
cat $O/forms.jsonl
