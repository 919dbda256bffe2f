#!/bin/bash
# r02ai: config-2 batch digests (52,429 BatchSize-20 lists = 820 groups of 64)
# by producer/consumer pairs (MIRSHA_PAIR_MAX_GROUPS=4096) vs the single-wave
# chain kernel (product: pairs only up to 512 groups); 3 reps interleaved.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02ai; mkdir -p $O
for r in 1 2 3; do
  for m in 512 4096; do
    MIRSHA_PAIR_MAX_GROUPS=$m timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie > $O/ab_pairmax${m}_$r.jsonl 2>> $O/ab.err || exit 1
  done
done
python3 tools/abview.py $O/ab_*.jsonl || true
echo all done
