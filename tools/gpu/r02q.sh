#!/bin/bash
# r02q: request-kernel issue priorities by progress, head vs last-generation
# tops (same-box A/B, 3 reps), timeline of the product, config 4 host pool vs
# per-call thread spawn (4 reps).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02q; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "full_size or every_length or mixed or random" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 1
for r in 1 2 3; do
  for lib in product h0t0 h1t0 h1t2 h1t4 h0t3 h2t3; do
    L=""; [ $lib = product ] || L=tools/scratch/$lib/libmirsha.so
    MIRSHA_AB_LIB=$L timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie > $O/ab_${lib}_$r.jsonl 2>> $O/ab.err || exit 1
  done
done
python3 tools/abview.py $O/ab_*.jsonl || true
MIRSHA_AB_LIB=tools/scratch/stamps/libmirsha.so timeout -k 10 180 python -u tools/stamp_run.py $O/stamps > $O/stamps.json 2> $O/stamps.err || { tail -20 $O/stamps.err; exit 1; }
cat $O/stamps.json
for r in 1 2 3 4; do
  for lib in product spawn; do
    L=""; [ $lib = product ] || L=tools/scratch/$lib/libmirsha.so
    MIRSHA_AB_LIB=$L timeout -k 10 240 python -u bench.py --config 4 --steps 10 --warmup 2 --cpu-seconds 0 > $O/c4_${lib}_$r.jsonl 2>> $O/c4.err || { tail $O/c4.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c4_${lib}_$r.jsonl'));print('$lib',round(d['ms_per_step'],2),round(d['pcie_inclusive']['ms_per_call'],2))"
  done
done
echo all done
