#!/bin/bash
# r04b: CU-block request kernel, config 3 sequential plan: variant 12 (LDS-DMA
# one block ahead) vs 13 (LDS-DMA, next block read back mid-block), and the
# product form (0) once; an SQ PMC pass that also covers the clock probe (is
# SQ_WAIT_ANY the loads, or the round form's own yields?); the multi-device
# tests after the cut fix and variant-13 parity; the default bench line with
# its new config-3 leg.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04b; mkdir -p $O
export MIRSHA_AB=1
for i in 1 2; do
for v in 12 13; do
timeout -k 10 300 python -u bench.py --config 3 --pipeline sequential --variant $v --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie --no-overlap-extra > $O/bench_c3seq_v$v.$i.jsonl 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench_c3seq_v$v.$i.jsonl').readlines()[-1]); r=d['roofline']
print('v$v', $i, 'step', round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms'],4), 'frac', round(r['frac'],4), 'check', d['self_check'], 'probe', round(r['measured_peak']['cycles_per_wave_compression']))"
done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in 13; do
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-include-regex "sha256|clock_probe" --output-format csv -d $O/pmc_sq_v$v -o run -- python3 bench.py --config 3 --pipeline sequential --variant $v --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie --no-overlap-extra > $O/pmc_sq_v$v.log 2>&1 || { tail $O/pmc_sq_v$v.log; exit 1; }
done
export MIRSHA_TEST_AB_VARIANTS=13
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_parity.py tests/test_c_abi.py -k "multi or nist or every_length or uniform_tiles or random_lengths or full_size_configs or cgo" -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
unset MIRSHA_TEST_AB_VARIANTS MIRSHA_AB
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.jsonl 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench.jsonl').readlines()[-1]); r=d['roofline']; c=d['config3'] or {}
print('c2', round(d['value']/1e9,3), 'G/s', round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms']*1e3,1), 'frac', round(r['frac'],4), d['self_check'])
for k in ('fused','sequential'):
    l=c.get(k) or {}; o=l.get('overlap_cycles') or {}
    print('c3', k, round(l.get('ms_per_step',0),4), 'kern', round(l.get('avg_launch_ms',0),4), 'frac', round(l.get('frac',0),4), l.get('self_check'), 'ovl', round(o.get('ms_per_step',0),4), round(o.get('frac',0),4))
print('leg s', round(c.get('leg_seconds',0),1), 'cpu', d['cpu_baseline']['value'], d['cpu_baseline'].get('go114_class',{}).get('value'))"
echo all done
