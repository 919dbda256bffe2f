#!/bin/bash
# r03c: config-3 request kernel forms: pair kernel at any size (6) vs CU-block (10).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03c; mkdir -p $O
for v in 10 11 10 11; do
timeout -k 10 200 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --pipeline sequential --no-pcie --no-overlap-extra --variant $v >> $O/c3seq_v$v.jsonl 2>> $O/bench.err || exit 1
done
for f in $O/c3seq_v*.jsonl; do python3 -c "
import json
for l in open('$f'):
    d=json.loads(l); r=d['roofline']; print('$f', round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms']*1e3,1), 'frac', round(r['frac'],4), d['self_check'], d.get('effective_clock_ghz'))"; done
echo all done
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_pipeline.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "host_pipeline or watchdog or cu" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
