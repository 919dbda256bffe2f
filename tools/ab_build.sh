#!/bin/bash
# Tools-only builds (never tracked, never loaded by tests, smoke() or the
# driver):
#   tools/ab_build.sh        the A/B round forms that tools/valu_microbench.hip
#                            times against the product's (bit-identical to
#                            FIPS 180-4, checked by tests/test_rounds_asm_sim.py)
#   tools/ab_build.sh lib    tools/ablib/libmirsha.so: the product sources with
#                            -DMIRSHA_AB_FORMS, i.e. plus the retired and
#                            diagnostic CU-block forms (variants 11-15; 14 skips
#                            its loads and its digests are NOT valid).  Loaded
#                            only through MIRSHA_AB_LIB=<path> (mirbft_amd/_lib.py)
#                            for same-box A/B timing.
set -euo pipefail
cd "$(dirname "$0")/.."
if [ "${1:-}" = "lib" ]; then
    mkdir -p tools/ablib
    make -s -C mirbft_amd/csrc OUT=../../tools/ablib EXTRA=-DMIRSHA_AB_FORMS ../../tools/ablib/libmirsha.so
    echo "tools/ablib/libmirsha.so built (A/B forms; MIRSHA_AB_LIB=tools/ablib/libmirsha.so MIRSHA_AB=1)"
    exit 0
fi
python3 mirbft_amd/csrc/gen_rounds_asm.py --ab > tools/sha256_rounds_asm_ab.h
echo "tools/sha256_rounds_asm_ab.h generated"
