#!/bin/bash
# r03a: the driver's exact commands on the round-2 head (GPUTEST_r02 never ran),
# then config 3's sequential plan under rocprofv3 (kernel trace + SQ counters).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03a; mkdir -p $O
timeout -k 10 900 python -m pytest tests -m gpu -x -q > $O/pytest_driver.log 2>&1 || { tail -30 $O/pytest_driver.log; exit 1; }
tail -1 $O/pytest_driver.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.jsonl 2> $O/bench.err || exit 1
timeout -k 10 300 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 2 --pipeline sequential --no-pcie > $O/bench_c3_seq.jsonl 2>> $O/bench.err || exit 1
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3seq_trace -o run -- python3 bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie --pipeline sequential --no-overlap-extra > $O/c3seq_under_trace.jsonl 2> $O/c3seq_trace.err || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-include-regex sha256 --output-format csv -d $O/c3seq_pmc_sq -o run -- python3 bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie --pipeline sequential --no-overlap-extra > $O/c3seq_pmc_sq.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-include-regex sha256 --output-format csv -d $O/c3seq_pmc_size -o run -- python3 bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie --pipeline sequential --no-overlap-extra > $O/c3seq_pmc_size.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM TCC_HIT_sum TCC_MISS_sum --kernel-include-regex sha256 --output-format csv -d $O/c3seq_pmc_mem -o run -- python3 bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 0 --no-pcie --pipeline sequential --no-overlap-extra > $O/c3seq_pmc_mem.log 2>&1 || exit 1
echo all done
