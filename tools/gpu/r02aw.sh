#!/bin/bash
# r02aw: split fused form with the tile waves per CU capped by dynamic LDS
# (ceil(tiles / tile CUs)); parity of the fused forms, config-3 A/B vs the
# paced form, traces of both.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02aw; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "fused" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  timeout -k 10 150 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie > $O/c3_paced_$r.jsonl 2>> $O/ab.err || exit 1
  MIRSHA_FUSED_SPLIT=1 timeout -k 10 150 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie > $O/c3_split_$r.jsonl 2>> $O/ab.err || exit 1
done
for f in $O/c3_*.jsonl; do python3 -c "import json; d=json.loads(open('$f').readlines()[-1]); o=d.get('overlap_cycles') or {}; print('$f', 'step', round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],3), 'ovl', round(o.get('ms_per_step',0),4), round(o.get('avg_launch_ms',0),4), round(o.get('frac',0),3))"; done
MIRSHA_FUSED_SPLIT=1 timeout -k 10 200 python -u tools/trace_fused.py 3 4 > $O/trace_split.jsonl 2> $O/trace_split.err || exit 1
python3 -c "import json; d=json.loads(open('$O/trace_split.jsonl').readline()); print({k: d[k] for k in ['tiles_per_simd_pcts','tile_end_us_pcts','group_end_us','kernel_span_us']})"
echo all done
