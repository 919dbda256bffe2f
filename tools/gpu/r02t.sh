#!/bin/bash
# r02t: priority schedule variants: top 3 (product), 0, 4, 5 and by tile
# fraction, config 2 (3 reps) and a 2 M-request config-5 stream (2 reps).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02t; mkdir -p $O
for r in 1 2 3; do
  for lib in product prio0 prio4 prio5 priofrac; do
    L=""; [ $lib = product ] || L=tools/scratch/$lib/libmirsha.so
    MIRSHA_AB_LIB=$L timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie > $O/ab_${lib}_$r.jsonl 2>> $O/ab.err || exit 1
  done
done
python3 tools/abview.py $O/ab_*.jsonl || true
for r in 1 2; do
  for lib in product prio0 priofrac; do
    L=""; [ $lib = product ] || L=tools/scratch/$lib/libmirsha.so
    MIRSHA_AB_LIB=$L timeout -k 10 200 python -u bench.py --config 5 --requests 2000000 --steps 5 --warmup 2 --cpu-seconds 0 > $O/c5_${lib}_$r.jsonl 2>> $O/c5.err || { tail $O/c5.err; exit 1; }
  done
done
python3 tools/abview.py $O/c5_*.jsonl || true
echo all done
