#!/bin/bash
# r05x: the round-5 tree after the buffer-headroom fix and the submit trace knob:
# pipelined-call order, metadata streams, drain on error): pytest -m gpu,
# smoke, the default bench line twice, and rocprofv3 --kernel-trace --stats of
# the default bench command.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r05x; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py >> $O/bench.jsonl 2>> $O/bench.err || exit 1
done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o c2 -- python3 $GRAFT_REPO_ROOT/bench.py > $O/bench_under_trace.jsonl 2> $O/prof.err || exit 1
echo done
