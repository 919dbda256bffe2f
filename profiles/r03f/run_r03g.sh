#!/bin/bash
# r03g: config 3 overlapped cycles: progress priorities (product) vs queue
# priorities (A/B) for the tile waves; fused step as before.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03g; mkdir -p $O
for v in 0 1 0 1; do
  MIRSHA_AB=1 MIRSHA_FUSED_OVERLAP_QUEUE_PRIO=$v timeout -k 10 300 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie > $O/bench_c3_q$v.jsonl 2>> $O/bench.err || { tail $O/bench.err; exit 1; }
  python3 -c "
import json
d=json.loads(open('$O/bench_c3_q$v.jsonl').readlines()[-1]); r=d['roofline']; o=d.get('overlap_cycles') or {}
print('queueprio=$v c3 step', round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms']*1e3,1), 'frac', round(r['frac'],4), 'check', d['self_check'], 'overlap', round(o.get('ms_per_step',0),4), round(o.get('avg_launch_ms',0)*1e3,1), round(o.get('frac',0),4))"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "split or overlap" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
