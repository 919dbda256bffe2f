#!/bin/bash
# rocprofv3 passes for bench.py (run on the GPU box from the repo root):
#   1. kernel trace + stats   -> per-kernel average duration (must agree with bench.py's HIP-event timing)
#   2..n. one --pmc pass each (counters never combined with other trace domains)
# Usage: profiles/profile.sh <tag> [bench args...]
set -euo pipefail
cd /tmp && export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${1:-r01}
shift || true
# trace pass: bench.py's own default steps/warmup (the clock needs ~20 ms of
# load to settle), so its average duration is comparable with the bench line;
# counter passes: short runs.
TARGS=("--cpu-seconds" "0" "--no-pcie" "$@")
ARGS=("--steps" "20" "--warmup" "3" "--cpu-seconds" "0" "--no-pcie" "$@")
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py "${TARGS[@]}" > "$OUT/trace.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex sha256 --output-format csv -d "$OUT/pmc_fetch" -o run -- python3 bench.py "${ARGS[@]}" > "$OUT/pmc_fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex sha256 --output-format csv -d "$OUT/pmc_write" -o run -- python3 bench.py "${ARGS[@]}" > "$OUT/pmc_write.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-include-regex sha256 --output-format csv -d "$OUT/pmc_sq" -o run -- python3 bench.py "${ARGS[@]}" > "$OUT/pmc_sq.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM TCC_HIT_sum TCC_MISS_sum --kernel-include-regex sha256 --output-format csv -d "$OUT/pmc_mem" -o run -- python3 bench.py "${ARGS[@]}" > "$OUT/pmc_mem.log" 2>&1 || echo "pmc_mem pass failed (counter names?)" >> "$OUT/notes.txt"
echo done
