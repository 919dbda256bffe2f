#!/bin/bash
# r02u: (1) tail tiles in the no-yield round form (A/B, 3 reps); (2) rehearsal
# of bench.py's N>1 path on this one-GPU box: torchrun with 2 ranks sharing
# GPU 0, barriers/reductions over gloo (the driver uses RCCL on 2-8 GPUs),
# configs 2 and 5.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02u; mkdir -p $O
for r in 1 2 3; do
  for lib in product tl2k3 tl1k3 tl2k4 tl4k3; do
    L=""; [ $lib = product ] || L=tools/scratch/$lib/libmirsha.so
    MIRSHA_AB_LIB=$L timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie > $O/ab_${lib}_$r.jsonl 2>> $O/ab.err || exit 1
  done
done
python3 tools/abview.py $O/ab_*.jsonl || true
export MIRSHA_BENCH_DEVICE=0 MIRSHA_BENCH_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 10 --warmup 3 > $O/dist2_config2.jsonl 2> $O/dist2_config2.err || { tail -20 $O/dist2_config2.err; exit 1; }
cat $O/dist2_config2.jsonl | head -c 700; echo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --config 5 --requests 1000000 --steps 3 --warmup 1 > $O/dist2_config5.jsonl 2> $O/dist2_config5.err || { tail -20 $O/dist2_config5.err; exit 1; }
cat $O/dist2_config5.jsonl | head -c 900; echo
echo all done
