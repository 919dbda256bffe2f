#!/bin/bash
# r03b: CU-block request kernel (config 3: 4,096 tiles, one 16-wave workgroup
# per CU, register prefetch) vs the one-wave LDS kernel (variant 5), same box;
# then the variant parity tests.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03b; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "cu or retired or watchdog or fused_plan_irregular or full_size" > $O/pytest_cu.log 2>&1 || { tail -30 $O/pytest_cu.log; exit 1; }
tail -1 $O/pytest_cu.log
for v in 0 5 0 5; do
timeout -k 10 200 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --pipeline sequential --no-pcie --no-overlap-extra --variant $v >> $O/c3seq_v$v.jsonl 2>> $O/bench.err || exit 1
done
for f in $O/c3seq_v*.jsonl; do python3 -c "
import json
for l in open('$f'):
    d=json.loads(l); r=d['roofline']; print('$f', round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms']*1e3,1), 'frac', round(r['frac'],4), d['self_check'])"; done
echo all done
