#!/bin/bash
# r05q (4): the tree with streaming stores in the library's staging packers
# and in the Go binding's packing (INTEGRATION.md streamPack): pytest -m gpu,
# smoke, the default bench line twice, and cgo_path plain/nt alternated.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05q4; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py >> $O/bench.jsonl 2>> $O/bench.err || exit 1
done
for r in 1 2 3 4 5 6; do
  timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 7 32 plain >> $O/cgo_plain.json 2>> $O/cgo.err || exit 1
  timeout -k 10 120 tests/c/build/cgo_path 1048576 256 15 7 32 nt >> $O/cgo_nt.json 2>> $O/cgo.err || exit 1
done
echo done
