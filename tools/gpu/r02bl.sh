#!/bin/bash
# r02bl: request kernel's arena loads non-temporal (A/B build ntload,
# -DMIRSHA_AB_ARENA_POL=2) vs the product's default policy: configs 2 and 3,
# interleaved reps on one box.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02bl; mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie --no-overlap-extra > $O/c2_product_$r.jsonl 2>> $O/ab.err || exit 1
  MIRSHA_AB_LIB=tools/scratch/ntload/libmirsha.so timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie --no-overlap-extra > $O/c2_ntload_$r.jsonl 2>> $O/ab.err || exit 1
done
for r in 1 2; do
  timeout -k 10 150 python -u bench.py --config 3 --pipeline sequential --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie --no-overlap-extra > $O/c3seq_product_$r.jsonl 2>> $O/ab.err || exit 1
  MIRSHA_AB_LIB=tools/scratch/ntload/libmirsha.so timeout -k 10 150 python -u bench.py --config 3 --pipeline sequential --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie --no-overlap-extra > $O/c3seq_ntload_$r.jsonl 2>> $O/ab.err || exit 1
done
for f in $O/c*.jsonl; do python3 -c "import json; d=json.loads(open('$f').readlines()[-1]); r=d['roofline']; print('$f', round(d['ms_per_step'],4), 'kern_us', round(r['avg_launch_ms']*1e3,1), 'frac', round(r['frac'],4), 'lib', d.get('lib', ''))"; done
echo all done
