#!/bin/bash
# r02bj: config-3 overlapped cycles with every tile at one flat priority
# (MIRSHA_OVERLAP_FLAT_PRIO=p; the chains do not wait on this launch's tiles)
# vs the queue priorities, 2 reps interleaved.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02bj; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "overlap or list_tiles" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  timeout -k 10 150 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie > $O/c3_queue_$r.jsonl 2>> $O/ab.err || exit 1
  for p in 0 1; do
    MIRSHA_OVERLAP_FLAT_PRIO=$p timeout -k 10 150 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie > $O/c3_flat${p}_$r.jsonl 2>> $O/ab.err || exit 1
  done
done
for f in $O/c3_*.jsonl; do python3 -c "import json; d=json.loads(open('$f').readlines()[-1]); o=d.get('overlap_cycles') or {}; print('$f', 'step', round(d['ms_per_step'],4), 'ovl', round(o.get('ms_per_step',0),4), round(o.get('avg_launch_ms',0),4), round(o.get('frac',0),3))"; done
echo all done
