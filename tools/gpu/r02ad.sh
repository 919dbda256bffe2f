#!/bin/bash
# r02ad: fused config-3 launch with tile queues (pace tile waves per SIMD, one
# per queue, queue 0 = earliest-needed tiles at issue priority 3).  Fused-plan
# parity first (paces 1/2/3/4), full -m gpu suite, then config-3 A/B over the
# pace (2 reps interleaved) and the driver's config-2 bench.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02ad; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "fused or pipeline" --timeout 120 --timeout-method thread > $O/pytest_fused.log 2>&1 || { tail -30 $O/pytest_fused.log; exit 1; }
tail -1 $O/pytest_fused.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for pace in 1 2 3 4; do
    MIRSHA_FUSED_PACE=$pace timeout -k 10 120 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie > $O/c3_pace${pace}_$r.jsonl 2>> $O/c3.err || exit 1
  done
done
for f in $O/c3_*.jsonl; do python3 -c "import json,sys; d=json.loads(open('$f').readlines()[-1]); print('$f', round(d['ms_per_step'],4), round(d['value']/1e6,1), 'frac', round(d['roofline']['frac'],3))"; done
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie > $O/bench_c2.jsonl 2> $O/bench.err || exit 1
echo all done
