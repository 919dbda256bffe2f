#!/bin/bash
# r02r: request-kernel issue priorities by progress, second box: head/tail tops
# h0t0 (all blocks at 0 after the prologue), h1t1, h2t2, h3t3, h2t3 and the
# product (h1t3), 4 interleaved reps.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02r; mkdir -p $O
for r in 1 2 3 4; do
  for lib in product h0t0 h1t1 h2t2 h3t3 h2t3; do
    L=""; [ $lib = product ] || L=tools/scratch/$lib/libmirsha.so
    MIRSHA_AB_LIB=$L timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie > $O/ab_${lib}_$r.jsonl 2>> $O/ab.err || exit 1
  done
done
python3 tools/abview.py $O/ab_*.jsonl || true
echo all done
