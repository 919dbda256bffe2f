#!/bin/bash
# r02ao: overlapped cycles on fused plans (config 3: the list pairs over the
# previous cycle's digests, no readiness waits): parity, then config-3 A/B of
# --pipeline overlap vs the fused plan (auto), 2 reps; config-2 overlap again.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02ao; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "overlap or fused" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for m in auto overlap; do
    timeout -k 10 120 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie --pipeline $m --no-overlap-extra > $O/c3_${m}_$r.jsonl 2>> $O/ab.err || exit 1
  done
done
for f in $O/c3_*.jsonl; do python3 -c "import json; d=json.loads(open('$f').readlines()[-1]); print('$f', d['roofline']['kernel'], round(d['value']/1e6,1), round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],3), 'check', d['self_check'])"; done
echo all done
