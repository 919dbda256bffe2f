#!/bin/bash
# r04a: (1) config 3 sequential plan, request kernel = CU-block form, product
# (variant 0 -> the register-prefetching form) vs variant 12 (the fused
# launch's LDS-DMA loader, one block ahead), alternating, then one PMC pass
# per form; (2) the split-tile fix (run lengths shorter than the
# plan's), the placement probe / remap, the multi-device drop-in
# (tests/test_gpu_multi.py) and the variant-12 parity cases.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04a; mkdir -p $O
export MIRSHA_AB=1
for i in 1 2; do
for v in 0 12; do
timeout -k 10 300 python -u bench.py --config 3 --pipeline sequential --variant $v --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie --no-overlap-extra > $O/bench_c3seq_v$v.$i.jsonl 2>> $O/err.txt || { tail $O/err.txt; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench_c3seq_v$v.$i.jsonl').readlines()[-1]); r=d['roofline']
print('v$v', $i, 'step', round(d['ms_per_step'],4), 'kern', round(r['avg_launch_ms'],4), 'frac', round(r['frac'],4), 'check', d['self_check'])"
done
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in 0 12; do
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-include-regex sha256 --output-format csv -d $O/pmc_sq_v$v -o run -- python3 bench.py --config 3 --pipeline sequential --variant $v --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie --no-overlap-extra > $O/pmc_sq_v$v.log 2>&1 || { tail $O/pmc_sq_v$v.log; exit 1; }
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM TCC_HIT_sum TCC_MISS_sum --kernel-include-regex sha256 --output-format csv -d $O/pmc_mem_v$v -o run -- python3 bench.py --config 3 --pipeline sequential --variant $v --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie --no-overlap-extra > $O/pmc_mem_v$v.log 2>&1 || { tail $O/pmc_mem_v$v.log; exit 1; }
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_v0 -o run -- python3 bench.py --config 3 --pipeline sequential --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie --no-overlap-extra > $O/bench_under_trace_v0.jsonl 2> $O/trace_v0.err || { tail $O/trace_v0.err; exit 1; }
export MIRSHA_TEST_AB_VARIANTS=12
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_parity.py -k "multi or split or placement or fused_list_tiles or nist or every_length or uniform_tiles or random_lengths or full_size_configs" -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
echo all done
