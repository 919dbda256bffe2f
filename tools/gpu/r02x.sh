#!/bin/bash
# r02x: dedup heads queued before the byte-for-byte confirmation (overlap of
# host confirm and GPU hashing): dedup/async GPU tests incl. the collision
# path, full GPU suite, config 4 (3 reps), dedup timing on the box's CPUs.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02x; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dedup_async.py -x -v --timeout 150 --timeout-method thread > $O/dedup_tests.log 2>&1
rc=$?; tail -4 $O/dedup_tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; tail -2 $O/gpu_tests.log; [ $rc -eq 0 ] || exit 1
for r in 1 2 3; do
  timeout -k 10 240 python -u bench.py --config 4 --steps 10 --warmup 2 --cpu-seconds 0 > $O/c4_$r.jsonl 2>> $O/c4.err || { tail $O/c4.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/c4_$r.jsonl'));print(round(d['ms_per_step'],2),round(d['pcie_inclusive']['ms_per_call'],2),{k:round(v,2) for k,v in d['host_phases_ms'].items()})"
done
echo all done
