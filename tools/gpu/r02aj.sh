#!/bin/bash
# r02aj: lone-wave chains (compress_asm_lat: config-2 batch digests, lists
# kernel, low-occupancy request form) in the ILP round order (latilp) vs the
# product's no-yield throughput order; config 2, 3 reps interleaved; config-1
# latency for both.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02aj; mkdir -p $O
MIRSHA_AB_LIB=tools/scratch/latilp/libmirsha.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_latilp.log 2>&1 || { tail -30 $O/pytest_latilp.log; exit 1; }
tail -1 $O/pytest_latilp.log
for r in 1 2 3; do
  for lib in product latilp; do
    L=""; [ $lib = product ] || L=tools/scratch/$lib/libmirsha.so
    MIRSHA_AB_LIB=$L timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie > $O/ab_${lib}_$r.jsonl 2>> $O/ab.err || exit 1
  done
done
python3 tools/abview.py $O/ab_*.jsonl || true
for lib in product latilp; do
  L=""; [ $lib = product ] || L=tools/scratch/$lib/libmirsha.so
  MIRSHA_AB_LIB=$L timeout -k 10 200 python -u bench.py --config 1 > $O/c1_${lib}.jsonl 2>> $O/ab.err || exit 1
done
echo all done
