#!/bin/bash
# r04l (probe): tools/lone_probe -- a lone wave's per-block cost, piece by piece.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04l6; mkdir -p $O
timeout -k 10 120 ./tools/lone_probe 64 > $O/lone_probe.jsonl 2> $O/lone_probe.err || { cat $O/lone_probe.err; exit 1; }
cat $O/lone_probe.jsonl
echo all done
