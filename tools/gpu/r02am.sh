#!/bin/bash
# r02am: full -m gpu suite with the overlapped-cycles API, the driver's bench
# command (its line now carries the overlap_cycles figure), smoke.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02am; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.jsonl 2> $O/bench.err || exit 1
python3 -c "import json; d=json.loads(open('$O/bench.jsonl').readlines()[-1]); print(d['value'], d['roofline']['frac'], d['overlap_cycles'])"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
echo all done
