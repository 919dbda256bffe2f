#!/bin/bash
# r03d: register-only compression rate vs waves per SIMD (clock probe, product round form).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 120 python -u - > $O/probe.txt 2>&1 <<'PY' || { cat $O/probe.txt; exit 1; }
import os
os.environ["MIRSHA_AB"] = "1"
from mirbft_amd import Engine
e = Engine(0)
for _ in range(3):
    for k in (8, 4, 2, 1, 5, 6):
        os.environ["MIRSHA_PROBE_WAVES"] = str(k)
        ghz, cyc = e.clock_probe(512)
        print(k, round(ghz, 3), round(cyc, 1), flush=True)
PY
cat $O/probe.txt
