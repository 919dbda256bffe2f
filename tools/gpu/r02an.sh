#!/bin/bash
# r02an: the driver's bench command with the overlap figure measured right
# behind the timed region (r02am measured it after the CPU baseline, clock down).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02an; mkdir -p $O
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.jsonl 2> $O/bench.err || exit 1
python3 -c "import json; d=json.loads(open('$O/bench.jsonl').readlines()[-1]); print(d['value'], d['roofline']['frac'], d['overlap_cycles'])"
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
echo all done
