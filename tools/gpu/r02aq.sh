#!/bin/bash
# r02aq: config-2 overlapped cycles, chain-wave priority schedule A/B
# (MIRSHA_OVERLAP_CHAIN_PRIO 0 = by fraction of the chain (product), 1 = 3 -
# block like the tiles, 2 = always 3, 3 = always 1), 2 reps interleaved.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02aq; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "overlap" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for m in 0 1 2 3; do
    MIRSHA_OVERLAP_CHAIN_PRIO=$m timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie --pipeline overlap > $O/ovl_prio${m}_$r.jsonl 2>> $O/ab.err || exit 1
  done
done
for f in $O/ovl_*.jsonl; do python3 -c "import json; d=json.loads(open('$f').readlines()[-1]); print('$f', round(d['value']/1e9,3), round(d['ms_per_step'],4), 'kern', round(d['roofline']['avg_launch_ms']*1e3,1), 'frac', round(d['roofline']['frac'],3))"; done
echo all done
