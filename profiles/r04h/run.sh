#!/bin/bash
# r04h: fused-launch tail pairs (a SIMD's idle second-to-last-queue wave
# produces K + W for the last queue's remaining blocks).  (1) parity: the new
# tail-pair test and the fused tests that run config-3 shapes, split tiles,
# placement remap and irregular plans; (2) config-3 fused step A/B, pairs on
# vs MIRSHA_FUSED_TAIL_PAIRS=0, alternating; (3) a traced run of each.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04h; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "tail_pairs" -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
export MIRSHA_AB=1
for i in 1 2; do
for tp in 1 0; do
MIRSHA_FUSED_TAIL_PAIRS=$tp timeout -k 10 300 python -u bench.py --config 3 --pipeline fused --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie --no-overlap-extra --no-config3-leg > $O/bench_c3_tp$tp.$i.jsonl 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench_c3_tp$tp.$i.jsonl').readlines()[-1]); r=d['roofline']
print('tp$tp', $i, 'step', round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms'],4), 'frac', round(r['frac'],4), 'check', d['self_check'])"
done
done
for tp in 1 0; do
MIRSHA_FUSED_TAIL_PAIRS=$tp timeout -k 10 200 python -u tools/trace_queues.py > $O/trace_tp$tp.txt 2>&1 || { tail $O/trace_tp$tp.txt; exit 1; }
grep -E "queue|tail pairs" $O/trace_tp$tp.txt | head -12
done
echo all done
