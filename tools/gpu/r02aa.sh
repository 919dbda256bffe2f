#!/bin/bash
# r02aa: persistent request waves (persist: per-tile block priorities;
# persistg: priorities from the progress over all the wave's tiles) vs the
# product one-wave-per-tile launch; parity suite on persistg first.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02aa; mkdir -p $O
MIRSHA_AB_LIB=tools/scratch/persistg/libmirsha.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_persistg.log 2>&1 || { tail -30 $O/pytest_persistg.log; exit 1; }
tail -1 $O/pytest_persistg.log
for r in 1 2 3; do
  for lib in product persist persistg; do
    L=""; [ $lib = product ] || L=tools/scratch/$lib/libmirsha.so
    MIRSHA_AB_LIB=$L timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie > $O/ab_${lib}_$r.jsonl 2>> $O/ab.err || exit 1
  done
done
python3 tools/abview.py $O/ab_*.jsonl || true
echo all done
