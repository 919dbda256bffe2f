#!/bin/bash
# r02al: overlapped cycles (this cycle's request tiles + the previous cycle's
# batch chains in one launch): parity, then config-2 A/B of --pipeline overlap
# vs the sequential plan (auto), 3 reps interleaved.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02al; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "overlap" --timeout 120 --timeout-method thread > $O/pytest_overlap.log 2>&1 || { tail -30 $O/pytest_overlap.log; exit 1; }
tail -1 $O/pytest_overlap.log
for r in 1 2 3; do
  for m in auto overlap; do
    timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie --pipeline $m > $O/ab_${m}_$r.jsonl 2>> $O/ab.err || exit 1
  done
done
python3 tools/abview.py $O/ab_*.jsonl || true
for f in $O/ab_*.jsonl; do python3 -c "import json; d=json.loads(open('$f').readlines()[-1]); print('$f', d['roofline']['kernel'], round(d['value']/1e9,3), round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],3), 'check', d['self_check'])"; done
echo all done
