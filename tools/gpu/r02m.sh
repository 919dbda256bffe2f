#!/bin/bash
# r02m: pipelined staged host calls (chunked H2D / kernel / D2H on three
# streams, persistent host pool) and the request kernel's copy-free rounds +
# uniform-length padding: new GPU tests, the full GPU suite, same-box A/B of
# the request kernel forms, driver bench (PCIe legs), config 1, then the r02l
# profile set (timeline + rocprof).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02m; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_pipeline.py -x -v --timeout 120 --timeout-method thread > $O/pipe_tests.log 2>&1
rc=$?; tail -12 $O/pipe_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -3 $O/gpu_tests.log; [ $rc -eq 0 ] || exit 1
for r in 1 2 3; do
  for lib in product movs ppad r02 occ6 pf5; do
    L=""; [ $lib = product ] || L=tools/scratch/$lib/libmirsha.so
    MIRSHA_AB_LIB=$L timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie > $O/ab_${lib}_$r.jsonl 2>> $O/ab.err || exit 1
  done
  echo ab rep $r done
done
python3 tools/abview.py $O/ab_*.jsonl || true
timeout -k 10 240 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 2 > $O/bench_driver.jsonl 2> $O/bench_driver.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_driver.jsonl'));print(d['value'],d['roofline']['frac'],json.dumps(d['pcie_inclusive']))"
timeout -k 10 200 python -u bench.py --config 1 > $O/bench_config1.jsonl 2> $O/c1.err || { tail $O/c1.err; exit 1; }
bash tools/gpu/r02l.sh > $O/r02l.log 2>&1 || { tail -5 $O/r02l.log; exit 1; }
tail -3 $O/r02l.log
echo all done
