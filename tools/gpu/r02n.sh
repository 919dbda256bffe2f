#!/bin/bash
# r02n: host-call timeline (pipelined staged path, pageable + pinned), the
# pipelined-path GPU tests, timeline of the request kernel (stamps build with
# the prologue stamp after the priority raise), and the rocprof set of the
# driver's command for the current product (profiles/profile.sh).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02n; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_host_pipeline.py -x -q --timeout 120 --timeout-method thread > $O/pipe_tests.log 2>&1
rc=$?; tail -2 $O/pipe_tests.log; [ $rc -eq 0 ] || exit 1
MIRSHA_STAGE_TRACE=1 timeout -k 10 120 python -u tools/host_call_trace.py 5 > $O/host_trace.json 2> $O/host_trace.err || { tail $O/host_trace.err; exit 1; }
cat $O/host_trace.json
MIRSHA_AB_LIB=tools/scratch/stamps/libmirsha.so timeout -k 10 180 python -u tools/stamp_run.py $O/stamps > $O/stamps.json 2> $O/stamps.err || { tail -20 $O/stamps.err; exit 1; }
cat $O/stamps.json
timeout -k 10 900 bash profiles/profile.sh r02n > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }

# config 3: fused plan occupancy ramp (pace 2, second wave per SIMD joins after
# a fraction of the tiles), A/B against the default pace 1
for r in 1 2; do
  timeout -k 10 120 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie > $O/c3_base_$r.jsonl 2>> $O/c3.err || exit 1
  for f in 0.125 0.25 0.5; do
    MIRSHA_FUSED_PACE=2 MIRSHA_FUSED_RAMP=$f timeout -k 10 120 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie > $O/c3_ramp${f}_$r.jsonl 2>> $O/c3.err || exit 1
    MIRSHA_FUSED_PACE=2 MIRSHA_FUSED_RAMP=$f MIRSHA_FUSED_FLAGS=2 timeout -k 10 120 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie > $O/c3_ramp${f}y_$r.jsonl 2>> $O/c3.err || exit 1
  done
done
for f in $O/c3_*.jsonl; do python3 -c "import json,sys;d=json.load(open('$f'));print('$f',round(d['ms_per_step'],4))"; done
echo c3 done
echo all done
