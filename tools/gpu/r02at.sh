#!/bin/bash
# r02at: config-3 overlapped cycles through the sequential plan's overlap
# kernel (request tiles on all 1,024 SIMDs, the 524 VerifyBatch chains as lone
# waves first in the grid) vs the fused plan's overlap (tile queues + list
# pairs on 9 CUs); chain priority 0 (by fraction) and 2 (always 3).  Plus a
# kernel trace of the config-1 latency bench (what one small cycle launches).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02at; mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  timeout -k 10 150 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie > $O/c3_fused_$r.jsonl 2>> $O/ab.err || exit 1
  for m in 0 2; do
    MIRSHA_OVERLAP_CHAIN_PRIO=$m timeout -k 10 150 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie --pipeline sequential > $O/c3_seq_prio${m}_$r.jsonl 2>> $O/ab.err || exit 1
  done
done
for f in $O/c3_*.jsonl; do python3 -c "import json; d=json.loads(open('$f').readlines()[-1]); o=d.get('overlap_cycles') or {}; print('$f', 'step', round(d['ms_per_step'],4), 'ovl', round(o.get('ms_per_step',0),4), round(o.get('avg_launch_ms',0),4), round(o.get('frac',0),3))"; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/c1prof -o c1 -- python3 -u bench.py --config 1 > $O/c1.jsonl 2> $O/c1.err || exit 1
find $O/c1prof -name '*stats*' | head -5
echo all done
