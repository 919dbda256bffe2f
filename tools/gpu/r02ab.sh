#!/bin/bash
# r02ab: fresh-container rebuild validated on the GPU (full -m gpu suite,
# smoke, the driver's bench command), then the FETCH_SIZE calibration with the
# raw L2 memory-side request counters: the loader pattern (k_segments), the
# coalesced stream (k_stream16) and the request kernel itself, to price the
# gfx950 "x2" correction for this access pattern.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02ab; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.jsonl 2> $O/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -s KILL 60 rocprofv3 --list-avail > $O/counters.txt 2>&1
rc=$?; [ $rc -ge 124 ] && exit $rc
pass() {  # pass <name> <counters...>: one --pmc pass over the calibration kernels
  local n=$1; shift
  timeout -s KILL 60 rocprofv3 --pmc "$@" --kernel-include-regex k_ --output-format csv -d $O/cal_$n -o run -- ./tools/fetch_calib > $O/cal_$n.log 2>&1
  local r=$?
  echo "pass $n rc=$r" >> $O/cal_rc.txt
  [ $r -ge 124 ] && exit $r
  return 0
}
pass fetch FETCH_SIZE
pass rdreq TCC_EA0_RDREQ_sum
pass rd32 TCC_EA0_RDREQ_32B_sum
pass bubble TCC_BUBBLE_sum
pass req TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum
# the same raw counters on the request kernel under the driver's bench command
for c in TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum TCC_REQ_sum; do
  timeout -s KILL 150 rocprofv3 --pmc $c --kernel-include-regex sha256_msgs --output-format csv -d $O/msgs_$c -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie > $O/msgs_$c.log 2>&1
  r=$?; echo "msgs $c rc=$r" >> $O/cal_rc.txt; [ $r -ge 124 ] && exit $r
done
echo all done
