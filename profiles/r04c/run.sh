#!/bin/bash
# r04c: is the default run's config-3 leg (fused step 1.07 ms in r04b) the leg
# or the round-4 kernel?  Standalone config-3 bench (fused plan) on this build
# and on the round-3 library (tools/scratch/r03lib, MIRSHA_AB_LIB), then the
# default bench again.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04c; mkdir -p $O
show() { python3 -c "
import json
d=json.loads(open('$1').readlines()[-1]); r=d['roofline']; o=d.get('overlap_cycles') or {}
print('$1', round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms'],4), 'frac', round(r['frac'],4), d['self_check'], 'ovl', round(o.get('ms_per_step',0),4), round(o.get('avg_launch_ms',0),4))"; }
for i in 1 2; do
timeout -k 10 300 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie > $O/c3_new.$i.jsonl 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
show $O/c3_new.$i.jsonl
MIRSHA_AB_LIB=tools/scratch/r03lib/libmirsha.so timeout -k 10 300 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie > $O/c3_r03.$i.jsonl 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
show $O/c3_r03.$i.jsonl
done
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 2 --no-pcie > $O/bench.jsonl 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench.jsonl').readlines()[-1]); c=d['config3'] or {}
for k in ('fused','sequential'):
    l=c.get(k) or {}; o=l.get('overlap_cycles') or {}
    print('leg', k, round(l.get('ms_per_step',0),4), 'kern', round(l.get('avg_launch_ms',0),4), l.get('self_check'), 'ovl', round(o.get('ms_per_step',0),4), round(o.get('avg_launch_ms',0),4))"
echo all done
