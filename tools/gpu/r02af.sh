#!/bin/bash
# r02af: fused list chains as producer/consumer pairs (LDS flags) + tile queues by SIMD slot (HW_ID +
# LDS counter): fused parity, config-3 timelines per queue (paces 1, 2, 4) and
# a config-3 A/B over the pace.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02af; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "fused or pipeline" --timeout 120 --timeout-method thread > $O/pytest_fused.log 2>&1 || { tail -30 $O/pytest_fused.log; exit 1; }
tail -1 $O/pytest_fused.log
timeout -k 10 200 python -u tools/trace_fused.py 3 1 2 4 > $O/trace_c3.jsonl 2> $O/trace.err || { tail -5 $O/trace.err; exit 1; }
for r in 1 2; do
  for pace in 1 2 4; do
    MIRSHA_FUSED_PACE=$pace timeout -k 10 120 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie > $O/c3_pace${pace}_$r.jsonl 2>> $O/c3.err || exit 1
  done
done
for f in $O/c3_*.jsonl; do python3 -c "import json,sys; d=json.loads(open('$f').readlines()[-1]); print('$f', round(d['ms_per_step'],4), round(d['value']/1e6,1), 'frac', round(d['roofline']['frac'],3))"; done
echo all done
