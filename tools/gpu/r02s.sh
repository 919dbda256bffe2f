#!/bin/bash
# r02s: product with block-progress issue priorities (top 3): full GPU suite,
# A/B vs priority 0 (3 reps), timeline, driver bench, config 5, rocprof set.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02s; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit 1
for r in 1 2 3; do
  for lib in product prio0; do
    L=""; [ $lib = product ] || L=tools/scratch/$lib/libmirsha.so
    MIRSHA_AB_LIB=$L timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie > $O/ab_${lib}_$r.jsonl 2>> $O/ab.err || exit 1
  done
done
python3 tools/abview.py $O/ab_*.jsonl || true
MIRSHA_AB_LIB=tools/scratch/stamps/libmirsha.so timeout -k 10 180 python -u tools/stamp_run.py $O/stamps > $O/stamps.json 2> $O/stamps.err || { tail -20 $O/stamps.err; exit 1; }
cat $O/stamps.json
timeout -k 10 240 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 2 > $O/bench_driver.jsonl 2> $O/bench_driver.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_driver.jsonl'));print(d['value'],d['roofline']['frac'],json.dumps(d['pcie_inclusive'])[:300])"
timeout -k 10 400 python -u bench.py --config 5 --steps 3 --warmup 1 --cpu-seconds 3 > $O/bench_config5.jsonl 2> $O/c5.err || { tail $O/c5.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_config5.jsonl'));print(d['value'],d['roofline']['frac'],d['ms_per_step'])"
timeout -k 10 900 bash profiles/profile.sh r02s > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
echo all done
