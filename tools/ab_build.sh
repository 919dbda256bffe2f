#!/bin/bash
# Tools-only generated sources (not tracked): the A/B round forms that
# tools/valu_microbench.hip times against the product's (bit-identical to
# FIPS 180-4, checked by tests/test_rounds_asm_sim.py).  Product A/B builds of
# round 2 (-DMIRSHA_AB_* variants) are retired; their results are in
# profiles/r02* and DESIGN.md.
set -euo pipefail
cd "$(dirname "$0")/.."
python3 mirbft_amd/csrc/gen_rounds_asm.py --ab > tools/sha256_rounds_asm_ab.h
echo "tools/sha256_rounds_asm_ab.h generated"
