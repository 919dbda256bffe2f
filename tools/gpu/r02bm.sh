#!/bin/bash
# r02bm: the driver's bench command on the final bench.py (algorithmic bytes
# with off/len entries), config 3 line, smoke.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02bm; mkdir -p $O
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.jsonl 2> $O/bench.err || exit 1
timeout -k 10 300 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 5 > $O/bench_config3.jsonl 2>> $O/bench.err || exit 1
for f in $O/bench.jsonl $O/bench_config3.jsonl; do python3 -c "import json; d=json.loads(open('$f').readlines()[-1]); r=d['roofline']; print('$f', round(d['value']/1e6,1), round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms']*1e3,1), 'frac', round(r['frac'],4), 'traffic/alg', r.get('traffic_over_algorithmic'), 'check', d['self_check'])"; done
echo all done
