#!/bin/bash
# r02ay: fused tile tickets reset on device by the launch's last retiring wave
# (no host-predicted ticket bases): full -m gpu suite, smoke, driver bench,
# config-3 line, then profiles/profile.sh for configs 2 and 3 (PMC traffic of
# this build for profiles/traffic.json).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02ay; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.jsonl 2> $O/bench.err || exit 1
timeout -k 10 300 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 5 > $O/bench_config3.jsonl 2>> $O/bench.err || exit 1
for f in $O/bench.jsonl $O/bench_config3.jsonl; do python3 -c "import json; d=json.loads(open('$f').readlines()[-1]); print('$f', round(d['value']/1e6,1), round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],4), 'check', d['self_check'], 'ovl', {k: d['overlap_cycles'][k] for k in ('digests_per_s','ms_per_step','frac')} if d.get('overlap_cycles') else None)"; done
bash profiles/profile.sh r02ay > $O/prof2.log 2>&1 || { tail -5 $O/prof2.log; exit 1; }
bash profiles/profile.sh r02ay3 --config 3 > $O/prof3.log 2>&1 || { tail -5 $O/prof3.log; exit 1; }
echo all done
