#!/bin/bash
# r03za: the round-3 kernels with LDS-DMA block loads in the fused launch: rocprofv3 kernel trace + PMC passes of the
# driver's bench command (config 2), config 3 (fused plan, with its overlapped
# leg) and config 2 overlapped cycles (profiles/profile.sh), then the driver's
# commands: the -m gpu suite, smoke, the default bench line; config 3 and 4
# bench lines.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03za; mkdir -p $O
bash profiles/profile.sh r03za_c2 || exit 1
bash profiles/profile.sh r03za_c3 --config 3 || exit 1
bash profiles/profile.sh r03za_c2ovl --pipeline overlap || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.jsonl 2> $O/bench.err || { tail $O/bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 3 > $O/bench_c3.jsonl 2>> $O/bench.err || { tail $O/bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 3 --cpu-seconds 3 > $O/bench_c4.jsonl 2>> $O/bench.err || { tail $O/bench.err; exit 1; }
for f in $O/bench.jsonl $O/bench_c3.jsonl $O/bench_c4.jsonl; do python3 -c "
import json
d=json.loads(open('$f').readlines()[-1]); r=d['roofline']; o=d.get('overlap_cycles') or {}
print('$f', round(d['value']/1e6,2), round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms']*1e3,1), 'frac', round(r['frac'],4), 'traffic', r.get('traffic'), 'check', d['self_check'], 'overlap', round(o.get('ms_per_step',0),4), round(o.get('frac',0),4), d.get('host_phases_ms'))"; done
echo all done
