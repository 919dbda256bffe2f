#!/bin/bash
# r02w: overlapped list pass (list stream): GPU test, then config 2 with and
# without --overlap-lists (3 reps each), driver command with the overlap.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02w; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_overlap.py tests/test_gpu_dedup_async.py tests/test_gpu_host_pipeline.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 1
for r in 1 2 3; do
  for ov in 0 1; do
    timeout -k 10 120 python -u bench.py --steps 50 --warmup 5 --cpu-seconds 0 --no-pcie --overlap-lists $ov > $O/ov${ov}_$r.jsonl 2>> $O/ab.err || exit 1
  done
done
for f in $O/ov*.jsonl; do python3 -c "import json;d=json.load(open('$f'));print('$f',round(d['ms_per_step']*1e3,1),round(d['roofline']['avg_launch_ms']*1e3,1),d['value']/1e9,d['self_check'])"; done
timeout -k 10 240 python -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 2 --overlap-lists 1 > $O/bench_driver_overlap.jsonl 2> $O/bench_driver.err || exit 1
python3 -c "import json;d=json.load(open('$O/bench_driver_overlap.jsonl'));print(d['value'],d['ms_per_step'],d['roofline']['frac'],d['self_check'])"
echo all done
