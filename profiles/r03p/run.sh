#!/bin/bash
# r03p: the driver's commands on the restored head (session 2 of round 3): -m gpu suite, smoke, bench lines.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03p; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.jsonl 2> $O/bench.err || { tail $O/bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 3 > $O/bench_c3.jsonl 2>> $O/bench.err || { tail $O/bench.err; exit 1; }
for f in $O/bench.jsonl $O/bench_c3.jsonl; do python3 -c "
import json
d=json.loads(open('$f').readlines()[-1]); r=d['roofline']; o=d.get('overlap_cycles') or {}; c=d.get('cgo_path') or {}
print('$f', round(d['value']/1e6,1), round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms']*1e3,1), 'frac', round(r['frac'],4), 'check', d['self_check'], 'batch_ms', d.get('batch_kernel_avg_ms'), 'overlap', round(o.get('ms_per_step',0),4), round(o.get('frac',0),4), 'cgo', (c.get('parallel') or {}).get('ms'))"; done
timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 3 --cpu-seconds 3 > $O/bench_c4.jsonl 2>> $O/bench.err || { tail $O/bench.err; exit 1; }
timeout -k 10 200 python -u tools/trace_overlap.py 10 > $O/trace_overlap.jsonl 2>> $O/trace.err || { tail -20 $O/trace.err; exit 1; }
echo all done
