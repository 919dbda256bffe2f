#!/bin/bash
# r04i: the driver's commands on the round-4 head (kernel sources unchanged
# since r04g, key 91d043db9245f7a4): pytest -m gpu, smoke, the default bench
# line (config-3 leg with the overlapped cycles timed right after its steps;
# the new multi_device leg of the drop-in).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04i; mkdir -p $O
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
m=d.get('multi_device') or {}
print('multi', m.get('devices'), round(m.get('ms_per_call',0),2), 'ms pinned', round((m.get('pageable') or {}).get('ms_per_call',0),2), 'ms pageable', m.get('self_check'), m.get('error'), [(x['device'], x['requests']) for x in m.get('per_device',[])])
p=d.get('pcie_inclusive') or {}; print('pcie', round(p.get('ms_per_call',0),2), round((p.get('pinned_arena') or {}).get('ms_per_call',0),2))
cb=d['cpu_baseline']; print('leg s', round(c.get('leg_seconds',0),1), 'cpu', round(cb['value']/1e6,2), 'M/s go114', round(cb['go114_class']['value']/1e6,2), 'M/s')"

# dispatch gaps of back-to-back overlapped config-3 cycles (step 0.649 vs kernel 0.635 ms)
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/trace_c3ovl -o run -- python3 bench.py --config 3 --pipeline overlap --steps 30 --warmup 5 --cpu-seconds 0 --no-pcie --no-config3-leg --no-overlap-extra > $O/bench_c3ovl_trace.jsonl 2> $O/trace_c3ovl.err || { tail $O/trace_c3ovl.err; exit 1; }
python3 tools/dispatch_gaps.py $O/trace_c3ovl fused | tee $O/gaps_c3ovl.txt
python3 -c "
import json
d=json.loads(open('$O/bench_c3ovl_trace.jsonl').readlines()[-1]); print('c3 ovl under trace step', round(d['ms_per_step'],4), 'kern', round(d['roofline']['avg_launch_ms'],4))"
echo traced
echo all done
