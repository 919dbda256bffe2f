#!/bin/bash
# Round-6 kernels: the default bench line twice (sampled events), then
# rocprof + PMC passes for config 3 (fused, sequential) and config 2's
# overlapped cycles (profiles/profile.sh), for profiles/traffic.json.
set -euo pipefail
OUT=gpurun_out/r06l
mkdir -p "$OUT"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench$i.jsonl" 2> "$OUT/bench$i.err"
done
timeout -k 10 600 bash profiles/profile.sh r06l_c3 --config 3 > "$OUT/prof_c3.log" 2>&1
timeout -k 10 600 bash profiles/profile.sh r06l_c3seq --config 3 --pipeline sequential > "$OUT/prof_c3seq.log" 2>&1
timeout -k 10 600 bash profiles/profile.sh r06l_c2ovl --pipeline overlap > "$OUT/prof_c2ovl.log" 2>&1
echo done
