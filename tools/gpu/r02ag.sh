#!/bin/bash
# r02ag: fused config 3, stolen (overflow) tiles at the last queue's priority
# (product) vs the taker's own priority (MIRSHA_FUSED_STEAL_PRIO=1); timelines.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02ag; mkdir -p $O
for r in 1 2; do
  for sp in 0 1; do
    MIRSHA_FUSED_STEAL_PRIO=$sp timeout -k 10 120 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie > $O/c3_steal${sp}_$r.jsonl 2>> $O/c3.err || exit 1
  done
done
for f in $O/c3_*.jsonl; do python3 -c "import json,sys; d=json.loads(open('$f').readlines()[-1]); print('$f', round(d['ms_per_step'],4), round(d['value']/1e6,1), 'frac', round(d['roofline']['frac'],3))"; done
MIRSHA_FUSED_STEAL_PRIO=1 timeout -k 10 200 python -u tools/trace_fused.py 3 4 > $O/trace_c3_steal1.jsonl 2> $O/trace.err || exit 1
echo all done
