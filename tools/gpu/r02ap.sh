#!/bin/bash
# r02ap: validation of the current tree: full -m gpu suite, smoke, the driver's
# bench command, config-3 line (with its overlap figure), and a 2-rank
# rehearsal of the torchrun path (both ranks on device 0, gloo reductions).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02ap; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.jsonl 2> $O/bench.err || exit 1
timeout -k 10 300 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 5 > $O/bench_config3.jsonl 2>> $O/bench.err || exit 1
for f in $O/bench.jsonl $O/bench_config3.jsonl; do python3 -c "import json; d=json.loads(open('$f').readlines()[-1]); print('$f', round(d['value']/1e6,1), round(d['ms_per_step'],4), 'frac', round(d['roofline']['frac'],4), 'check', d['self_check'], 'ovl', {k: d['overlap_cycles'][k] for k in ('digests_per_s','ms_per_step','frac')} if d.get('overlap_cycles') else None)"; done
export MIRSHA_BENCH_DEVICE=0 MIRSHA_BENCH_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 10 --warmup 3 > $O/dist2_config2.jsonl 2> $O/dist2_config2.err || { tail -20 $O/dist2_config2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/dist2_config2.jsonl').readlines()[-1]); print('dist2', d['n_gpus'], round(d['value']/1e9,3), d['self_check'])"
echo all done
