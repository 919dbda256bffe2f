#!/bin/bash
# r03zh: rehearsal of bench.py's N>1 path on the final round-3 tree, on a
# one-GPU box: torchrun with 2 and 4 ranks, every rank on GPU 0
# (MIRSHA_BENCH_DEVICE=0), barriers and reductions over gloo
# (MIRSHA_BENCH_DIST_BACKEND=gloo; the driver's 8-GPU runs use RCCL).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03zh; mkdir -p $O
export MIRSHA_BENCH_DEVICE=0 MIRSHA_BENCH_DIST_BACKEND=gloo
run() {  # name nproc port args...
  local name=$1 np=$2 port=$3; shift 3
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $np --master-addr 127.0.0.1 \
    --master-port $port bench.py --gpus $np "$@" > $O/$name.jsonl 2> $O/$name.err || { tail -30 $O/$name.err; exit 1; }
}
run c2_n2 2 29611 --steps 20 --warmup 5
run c2_n4 4 29612 --steps 20 --warmup 5
run c3_n2 2 29613 --config 3 --steps 10 --warmup 3
run c5_n2 2 29614 --config 5 --requests 1000000 --steps 5 --warmup 2
run c4_n2 2 29615 --config 4 --steps 5 --warmup 2
for f in $O/*.jsonl; do python3 -c "
import json
d=json.loads(open('$f').readlines()[-1]); r=d.get('roofline') or {}
print('$f', d['n_gpus'], '%.4g' % d['value'], round(d['ms_per_step'],4), d.get('scaling'), r.get('frac'), d.get('self_check'), len(d.get('per_rank') or []))"; done
echo all done
