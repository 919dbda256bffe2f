#!/bin/bash
# r02au: fused plans whose list blocks also run tile waves
# (MIRSHA_FUSED_LIST_TILES 0 = product until now, 1 = SIMDs 2-3, 2 = all but
# the pair): parity (irregular shapes, config 3 full size incl. overlapped
# cycles), then config-3 fused step + overlapped-cycle figure, 2 reps interleaved.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02au; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "fused or overlap" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for m in 0 1 2; do
    MIRSHA_FUSED_LIST_TILES=$m timeout -k 10 150 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie > $O/c3_lt${m}_$r.jsonl 2>> $O/ab.err || exit 1
  done
done
for f in $O/c3_*.jsonl; do python3 -c "import json; d=json.loads(open('$f').readlines()[-1]); o=d.get('overlap_cycles') or {}; print('$f', 'step', round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],3), 'ovl', round(o.get('ms_per_step',0),4), round(o.get('avg_launch_ms',0),4), round(o.get('frac',0),3))"; done
echo all done
