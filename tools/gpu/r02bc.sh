#!/bin/bash
# r02bc: dedup submissions validate the slice arrays inside the fingerprint
# walk (one pass over config 4's 15.7 M slices instead of two): dedup / async
# / C-ABI / mirror tests incl. the argument-error cases, then config 4 twice.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02bc; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_dedup_async.py tests/test_c_abi.py tests/test_gpu_host_pipeline.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --config 4 --steps 10 --warmup 2 --cpu-seconds 0 > $O/bench_config4_$r.jsonl 2>> $O/c4.err || { tail $O/c4.err; exit 1; }
done
for f in $O/bench_config4_*.jsonl; do python3 -c "import json; d=json.loads(open('$f').readlines()[-1]); print('$f', '%.4g' % d['value'], round(d['ms_per_step'],3), 'check', d.get('self_check'), d.get('host_phases_ms'))"; done
echo all done
