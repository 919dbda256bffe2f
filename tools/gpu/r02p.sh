#!/bin/bash
# r02p: config 4 (host pool vs per-call thread spawn; large-message calls no
# longer pipelined), config 5 with the block-balanced sharder, driver bench
# with the median-of-10 PCIe leg, then the rocprof set of the driver's command.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02p; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_pipeline.py tests/test_gpu_dedup_async.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 1
# request kernel: issue priority falling with the wave's progress (A/B)
for r in 1 2 3; do
  for lib in product pblk3 pblk2 pblk1; do
    L=""; [ $lib = product ] || L=tools/scratch/$lib/libmirsha.so
    MIRSHA_AB_LIB=$L timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie > $O/ab_${lib}_$r.jsonl 2>> $O/ab.err || exit 1
  done
done
python3 tools/abview.py $O/ab_*.jsonl || true
MIRSHA_AB_LIB=tools/scratch/stampsp3/libmirsha.so timeout -k 10 180 python -u tools/stamp_run.py $O/stampsp3 > $O/stampsp3.json 2> $O/stamps.err || { tail -20 $O/stamps.err; exit 1; }
MIRSHA_AB_LIB=tools/scratch/stamps/libmirsha.so timeout -k 10 180 python -u tools/stamp_run.py $O/stamps > $O/stamps.json 2>> $O/stamps.err || { tail -20 $O/stamps.err; exit 1; }
for r in 1 2; do
  for lib in product spawn; do
    L=""; [ $lib = product ] || L=tools/scratch/$lib/libmirsha.so
    MIRSHA_AB_LIB=$L timeout -k 10 240 python -u bench.py --config 4 --steps 10 --warmup 2 --cpu-seconds 0 > $O/c4_${lib}_$r.jsonl 2>> $O/c4.err || { tail $O/c4.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/c4_${lib}_$r.jsonl'));print('$lib',d['ms_per_step'],d['pcie_inclusive']['ms_per_call'])"
  done
done
timeout -k 10 240 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 2 > $O/bench_driver.jsonl 2> $O/bench_driver.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_driver.jsonl'));print(d['value'],d['roofline']['frac'],json.dumps(d['pcie_inclusive']))"
timeout -k 10 400 python -u bench.py --config 5 --steps 3 --warmup 1 --cpu-seconds 5 > $O/bench_config5.jsonl 2> $O/c5.err || { tail $O/c5.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_config5.jsonl'));print(d['value'],d['roofline']['frac'],d['ms_per_step'])"
timeout -k 10 900 bash profiles/profile.sh r02p > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
echo all done
