#!/bin/bash
# r05p: round-5 kernels (variants 11-15 out of the product library; host code split;
# asynchronous arena submissions): the driver's commands (pytest -m gpu, smoke, the default
# bench line), a 60 s soak, then rocprofv3 kernel-trace + PMC passes
# (profiles/profile.sh) of config 2 (the driver's command), config 3 fused,
# config 3 sequential and config 2 overlapped cycles for the new source key.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05p; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.jsonl 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench.jsonl').readlines()[-1]); r=d['roofline']; c=d['config3'] or {}; o=d.get('overlap_cycles') or {}
print('c2', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms']*1e3,1), 'frac', round(r['frac'],4), d['self_check'], 'ovl', round(o.get('ms_per_step',0),4), 'key', d['roofline'].get('traffic_key'))
for k in ('fused','sequential'):
    l=c.get(k) or {}; o=l.get('overlap_cycles') or {}
    print('c3', k, round(l.get('ms_per_step',0),4), 'kern', round(l.get('avg_launch_ms',0),4), 'frac', round(l.get('frac',0),4), l.get('self_check'), 'ovl', round(o.get('ms_per_step',0),4), round(o.get('avg_launch_ms',0),4), round(o.get('frac',0),4))
m=d.get('multi_device') or {}
print('multi', m.get('devices'), round(m.get('ms_per_call',0),2), m.get('self_check'), m.get('error'))"
timeout -k 10 120 python -u tests/soak_gpu.py --seconds 60 --seed 113 > $O/soak.log 2>&1 || { tail -20 $O/soak.log; exit 1; }
tail -1 $O/soak.log
bash profiles/profile.sh r05p_c2 || exit 1
bash profiles/profile.sh r05p_c3 --config 3 || exit 1
bash profiles/profile.sh r05p_c3seq --config 3 --pipeline sequential || exit 1
bash profiles/profile.sh r05p_c2ovl --pipeline overlap || exit 1
echo all done
