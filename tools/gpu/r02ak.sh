#!/bin/bash
# r02ak: profile of the current product on the driver's command (kernel trace
# + stats, PMC passes incl. read requests by size) and the driver's bench line.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r02ak; mkdir -p $O
bash profiles/profile.sh r02ak || exit 1
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.jsonl 2> $O/bench.err || exit 1
timeout -k 10 300 python -u bench.py --config 3 --steps 20 --warmup 5 --cpu-seconds 5 > $O/bench_config3.jsonl 2>> $O/bench.err || exit 1
echo all done
