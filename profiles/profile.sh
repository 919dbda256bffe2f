#!/bin/bash
# rocprofv3 passes over the driver's own bench command (run on the GPU box from
# the repo root):
#   1. kernel trace + stats of exactly `bench.py --gpus 1 --steps 20 --warmup 5`
#      (plus any extra args): per-kernel average duration, to agree with the
#      bench line's HIP-event kernel time;
#   2..n. one --pmc pass each (counters never combined with other trace
#      domains), same command without the CPU baseline / PCIe legs.
# Usage: profiles/profile.sh <tag> [extra bench args...]
# Then locally: python3 profiles/summarize.py gpurun_out/prof_<tag> > .../summary.json
#               python3 profiles/update_traffic.py gpurun_out/prof_<tag>/summary.json --tag <tag> [--config N]
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r02}
shift || true
ARGS=("--gpus" "1" "--steps" "20" "--warmup" "5" "$@")
PARGS=("${ARGS[@]}" "--cpu-seconds" "0" "--no-pcie" "--no-config3-leg")
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py "${ARGS[@]}" > "$OUT/bench_under_trace.jsonl" 2> "$OUT/trace.err"
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex sha256 --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py "${PARGS[@]}" > "$OUT/pmc_fetch.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex sha256 --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py "${PARGS[@]}" > "$OUT/pmc_write.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-include-regex sha256 --output-format csv -d "$OUT/pmc_sq" -o run -- python3 bench.py "${PARGS[@]}" > "$OUT/pmc_sq.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM TCC_HIT_sum TCC_MISS_sum --kernel-include-regex sha256 --output-format csv -d "$OUT/pmc_mem" -o run -- python3 bench.py "${PARGS[@]}" > "$OUT/pmc_mem.log" 2>&1 || echo "pmc_mem pass failed (counter names?)" >> "$OUT/notes.txt"
timeout -s KILL 150 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum --kernel-include-regex sha256 --output-format csv -d "$OUT/pmc_size" -o run -- python3 bench.py "${PARGS[@]}" > "$OUT/pmc_size.log" 2>&1
python3 profiles/summarize.py "$OUT" > "$OUT/summary.json"
echo done
