#!/bin/bash
# r04i (2): the default bench line again after the multi_device leg's check
# moved to oracle samples (the first run compared against digests the steps
# had not yet produced: the leg runs before them).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04i2; mkdir -p $O
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.jsonl 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench.jsonl').readlines()[-1]); r=d['roofline']; c=d['config3'] or {}; o=d.get('overlap_cycles') or {}
print('c2', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms']*1e3,1), 'frac', round(r['frac'],4), d['self_check'], 'ovl', round(o.get('ms_per_step',0),4))
for k in ('fused','sequential'):
    l=c.get(k) or {}; o=l.get('overlap_cycles') or {}
    print('c3', k, round(l.get('ms_per_step',0),4), 'kern', round(l.get('avg_launch_ms',0),4), 'frac', round(l.get('frac',0),4), l.get('self_check'), 'ovl', round(o.get('ms_per_step',0),4), round(o.get('avg_launch_ms',0),4), round(o.get('frac',0),4))
m=d.get('multi_device') or {}
print('multi', m.get('devices'), round(m.get('ms_per_call',0),2), 'ms pinned', round((m.get('pageable') or {}).get('ms_per_call',0),2), 'ms pageable', m.get('self_check'), m.get('error'), [(x['device'], x['requests']) for x in m.get('per_device',[])])
p=d.get('pcie_inclusive') or {}; print('pcie', round(p.get('ms_per_call',0),2), round((p.get('pinned_arena') or {}).get('ms_per_call',0),2))
cb=d['cpu_baseline']; print('leg s', round(c.get('leg_seconds',0),1), 'cpu', round(cb['value']/1e6,2), 'M/s go114', round(cb['go114_class']['value']/1e6,2), 'M/s')"

echo all done
