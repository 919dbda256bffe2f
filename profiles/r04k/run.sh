#!/bin/bash
# r04k: does one wave carrying two interleaved SHA-256 states issue better than
# two waves of one?  tools/ilp_asm_probe (the product's rounds_asm vs
# tools/gen_ilp2_asm.py's rounds2_asm, register-only) at 2/4/8 chains per
# SIMD; and tools/ilp_probe (compiler-generated rounds) for contrast.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04k; mkdir -p $O
timeout -k 10 120 ./tools/ilp_asm_probe 3000 > $O/ilp_asm_probe.jsonl 2> $O/ilp_asm_probe.err && timeout -k 10 120 ./tools/ilp_asm_probe 3000 yield > $O/yield_probe.jsonl 2> $O/ilp_asm_probe.err || { cat $O/ilp_asm_probe.err; exit 1; }
cat $O/yield_probe.jsonl
echo all done
