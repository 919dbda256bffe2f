#!/bin/bash
# r04g: the round-4 kernels end to end -- the driver's commands (pytest -m gpu,
# smoke, the default bench line with its config-3 leg), a 120 s randomised
# soak (now with short-run split plans and the multi-device drop-in), then
# rocprofv3 kernel-trace + PMC passes (profiles/profile.sh) of config 2 (the
# driver's command), config 3 fused, config 3 sequential (the CU-block
# request kernel) and config 2 overlapped cycles.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04g; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.jsonl 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench.jsonl').readlines()[-1]); r=d['roofline']; c=d['config3'] or {}; o=d.get('overlap_cycles') or {}
print('c2', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms']*1e3,1), 'frac', round(r['frac'],4), d['self_check'], 'ovl', round(o.get('ms_per_step',0),4))
for k in ('fused','sequential'):
    l=c.get(k) or {}; o=l.get('overlap_cycles') or {}
    print('c3', k, round(l.get('ms_per_step',0),4), 'kern', round(l.get('avg_launch_ms',0),4), 'frac', round(l.get('frac',0),4), l.get('self_check'), 'ovl', round(o.get('ms_per_step',0),4), round(o.get('avg_launch_ms',0),4), round(o.get('frac',0),4))
cb=d['cpu_baseline']; print('leg s', round(c.get('leg_seconds',0),1), 'cpu', round(cb['value']/1e6,2), 'M/s go114', round(cb['go114_class']['value']/1e6,2), 'M/s')"
timeout -k 10 200 python -u tests/soak_gpu.py --seconds 120 --seed 71 > $O/soak.log 2>&1 || { tail -20 $O/soak.log; exit 1; }
tail -1 $O/soak.log
bash profiles/profile.sh r04g_c2 || exit 1
bash profiles/profile.sh r04g_c3 --config 3 || exit 1
bash profiles/profile.sh r04g_c3seq --config 3 --pipeline sequential || exit 1
bash profiles/profile.sh r04g_c2ovl --pipeline overlap || exit 1
echo all done
