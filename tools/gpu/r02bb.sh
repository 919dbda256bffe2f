#!/bin/bash
# r02bb: final checks of round 2's tree: the driver's bench command three
# times (spread), and a 2-rank rehearsal of the torchrun path (both ranks on
# device 0, gloo for the bench's own reductions).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02bb; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$r.jsonl 2>> $O/bench.err || exit 1
done
for f in $O/bench_*.jsonl; do python3 -c "import json; d=json.loads(open('$f').readlines()[-1]); r=d['roofline']; print('$f', round(d['value']/1e9,3), round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms']*1e3,1), 'frac', round(r['frac'],4), 'traffic', r.get('traffic'), 'check', d['self_check'])"; done
export MIRSHA_BENCH_DEVICE=0 MIRSHA_BENCH_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 > $O/dist2_config2.jsonl 2> $O/dist2_config2.err || { tail -20 $O/dist2_config2.err; exit 1; }
python3 -c "import json; d=json.loads(open('$O/dist2_config2.jsonl').readlines()[-1]); print('dist2', d['n_gpus'], round(d['value']/1e9,3), d['self_check'])"
echo all done
