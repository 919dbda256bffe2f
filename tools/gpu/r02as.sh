#!/bin/bash
# r02as: config 5 (arenas > 4 GiB): per-16-message-group 4 GiB windows at 8 waves/SIMD +
# 64-bit fallback vs the 64-bit form for every tile (MIRSHA_NO_BASED=1).
# Wide-arena parity both ways, full GPU suite, then config-5 A/B (1 GPU,
# 12.5 M requests, 2 reps interleaved).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02as; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "wide_arena" --timeout 200 --timeout-method thread > $O/pytest_wide.log 2>&1 || { tail -30 $O/pytest_wide.log; exit 1; }
tail -1 $O/pytest_wide.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for m in based wide; do
    E=""; [ $m = wide ] && E="MIRSHA_NO_BASED=1"
    env $E timeout -k 10 400 python -u bench.py --config 5 --steps 5 --warmup 2 --cpu-seconds 0 --no-pcie > $O/c5_${m}_$r.jsonl 2>> $O/c5.err || exit 1
  done
done
for f in $O/c5_*.jsonl; do python3 -c "import json; d=json.loads(open('$f').readlines()[-1]); print('$f', round(d['value']/1e6,1), round(d['ms_per_step'],3), 'frac', round(d['roofline']['frac'],4), 'check', d['self_check'])"; done
echo all done
