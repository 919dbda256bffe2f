#!/bin/bash
# Config-3 issue-yield sweep: one library per yield form of
# the request kernels' rounds (gen_rounds_asm.py --yield: after every 1st /
# 2nd (product) / 3rd / 4th 4-cycle op, after the rotates only, none), built
# here into tools/ablib/y<form>/ from a copy of the product sources.
#   tools/yield_sweep.sh build        (CPU container)
#   tools/yield_sweep.sh run <out>    (GPU box: config-3 sequential plan =
#       sha256_msgs_cu_kernel at 4 waves/SIMD, and the clock probe at 4
#       waves/SIMD, every form twice, interleaved)
set -euo pipefail
cd "$(dirname "$0")/.."
FORMS=(2 1 3 4 rot none)
if [ "${1:-}" = "build" ]; then
    for f in "${FORMS[@]}"; do
        d=/tmp/ysweep_$f
        rm -rf "$d" && mkdir -p "$d/m/csrc" "$d/include"
        cp mirbft_amd/csrc/* "$d/m/csrc/" 2>/dev/null || true
        cp include/mirsha.h "$d/include/"
        python3 mirbft_amd/csrc/gen_rounds_asm.py --yield "$f" > "$d/m/csrc/sha256_rounds_asm.h"
        mkdir -p tools/ablib/y$f
        (cd "$d/m/csrc" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -shared \
            -o "$OLDPWD/tools/ablib/y$f/libmirsha.so" mirsha_kernels.hip mirsha_api.hip mirsha_staging.hip \
            mirsha_plan.hip mirsha_async.hip mirsha_multi.hip mirsha_scan.hip mirsha_host.cpp) &
    done
    wait
    ls -la tools/ablib/*/libmirsha.so
    exit 0
fi
OUT=${2:-gpurun_out/ysweep}
mkdir -p "$OUT"
for rep in 1 2; do
    for f in "${FORMS[@]}"; do
        MIRSHA_AB=1 MIRSHA_PROBE_WAVES=4 MIRSHA_AB_LIB=tools/ablib/y$f/libmirsha.so timeout -k 10 120 \
            python3 bench.py --config 3 --pipeline sequential --steps 40 --warmup 10 --no-pcie --cpu-seconds 0 \
            --no-overlap-extra --probe-iters 64 > "$OUT/y${f}_$rep.json" 2> "$OUT/y${f}_$rep.err"
        echo "$f $rep done"
    done
done
