#!/bin/bash
# r04l: fused-launch lone-wave round form (g_simd_live) and the last queue staging two blocks ahead.
# the only live wave of their SIMD (g_simd_live).  (1) parity on every fused
# test; (2) config-3 fused step, lone form on vs MIRSHA_FUSED_LONE_FORM=0,
# alternating; (3) a traced run of each (queue ends, list-group ends).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04l7; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "fused or full_size or pipeline" -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
export MIRSHA_AB=1
for i in 1 2; do
for lf in 1 0; do
MIRSHA_FUSED_LONE_FORM=$lf timeout -k 10 300 python -u bench.py --config 3 --pipeline fused --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie --no-config3-leg > $O/bench_c3_lf$lf.$i.jsonl 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench_c3_lf$lf.$i.jsonl').readlines()[-1]); r=d['roofline']; o=d.get('overlap_cycles') or {}
print('lf$lf', $i, 'step', round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms'],4), 'frac', round(r['frac'],4), 'check', d['self_check'], 'ovl', round(o.get('ms_per_step',0),4), round(o.get('avg_launch_ms',0),4))"
done
done
for lf in 1 0; do
MIRSHA_FUSED_LONE_FORM=$lf timeout -k 10 200 python -u tools/trace_queues.py > $O/trace_lf$lf.txt 2>&1 || { tail $O/trace_lf$lf.txt; exit 1; }
grep -E "^queue [0-9]: [0-9]+ tiles|list groups|lone-wave" $O/trace_lf$lf.txt
done
echo all done
