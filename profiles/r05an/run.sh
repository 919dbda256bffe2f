#!/bin/bash
# r05an: the final round-5 tree (after r05aj's aligned kernel-stored digests):
# the default bench line twice, then rocprofv3 kernel-trace + PMC passes of
# config 2 (profiles/profile.sh) for the rocprof/event agreement check.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r05an; mkdir -p $O
for i in 1 2; do
  timeout -k 10 400 python -u bench.py > $O/bench$i.jsonl 2> $O/bench$i.err || { tail $O/bench$i.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/bench$i.jsonl').readlines()[-1]); r=d['roofline']; g=d.get('cgo_path') or {}
print('c2', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms']*1e3,1), 'frac', round(r['frac'],4), 'self_check', d['self_check'], 'cgo', {k:(v.get('ms_per_call') if isinstance(v,dict) else v) for k,v in g.items() if isinstance(v,dict)})"
done
bash profiles/profile.sh r05an_c2 || exit 1
echo all done
