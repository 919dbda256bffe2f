#!/bin/bash
# r02ac: final-block tail form (compress_asm_tail + trimmed final-block loads)
# in the product.  New uniform-tile parity test first, then the full -m gpu
# suite, a same-box A/B against the no-tail build (3 reps interleaved), the
# L2 memory-side read requests by size (TCC_EA0_RDREQ_{32B,64B,128B}) for the
# calibration kernels and both request-kernel builds, and the driver's bench.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02ac; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "uniform_tiles" --timeout 120 --timeout-method thread > $O/pytest_uniform.log 2>&1 || { tail -30 $O/pytest_uniform.log; exit 1; }
tail -1 $O/pytest_uniform.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for lib in product notail; do
    L=""; [ $lib = product ] || L=tools/scratch/$lib/libmirsha.so
    MIRSHA_AB_LIB=$L timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie > $O/ab_${lib}_$r.jsonl 2>> $O/ab.err || exit 1
  done
done
python3 tools/abview.py $O/ab_*.jsonl || true
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
SZ="TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
timeout -s KILL 60 rocprofv3 --pmc $SZ --kernel-include-regex k_ --output-format csv -d $O/cal_sz -o run -- ./tools/fetch_calib > $O/cal_sz.log 2>&1
r=$?; echo "cal_sz rc=$r" >> $O/rc.txt; [ $r -ge 124 ] && exit $r
for lib in product notail; do
  L=""; [ $lib = product ] || L=tools/scratch/$lib/libmirsha.so
  MIRSHA_AB_LIB=$L timeout -s KILL 150 rocprofv3 --pmc $SZ --kernel-include-regex sha256_msgs --output-format csv -d $O/msgs_sz_$lib -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie > $O/msgs_sz_$lib.log 2>&1
  r=$?; echo "msgs_sz_$lib rc=$r" >> $O/rc.txt; [ $r -ge 124 ] && exit $r
  MIRSHA_AB_LIB=$L timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex sha256_msgs --output-format csv -d $O/msgs_req_$lib -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie > $O/msgs_req_$lib.log 2>&1
  r=$?; echo "msgs_req_$lib rc=$r" >> $O/rc.txt; [ $r -ge 124 ] && exit $r
done
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.jsonl 2> $O/bench.err || exit 1
echo all done
