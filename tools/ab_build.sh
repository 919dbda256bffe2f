#!/bin/bash
# A/B builds of libmirsha.so from the product sources with measurement-only
# defines, into tools/scratch/<name>/ (git-ignored; travels to the GPU box).
# Select one at run time with MIRSHA_AB_LIB=tools/scratch/<name>/libmirsha.so.
#   r1form:    -DMIRSHA_AB_KSGPR -DMIRSHA_AB_NOALIGNED -DMIRSHA_AB_OLDPROLOGUE
#              (round constants in SGPRs, 5-dword chunks, round-1 prologue)
#   oldpro:    -DMIRSHA_AB_OLDPROLOGUE  (shuffle reductions, conditional metadata loads)
#   noprio:    -DMIRSHA_AB_NOPRIO       (request prologue at the default issue priority)
#   wg4:       -DMIRSHA_AB_WG4          (4-wave request workgroups)
#   stamps:    -DMIRSHA_AB_STAMPS       (per-tile timeline for tools/stamp_run.py)
#   ppad:      -DMIRSHA_AB_PRODUCER_PAD (loader-side padding for uniform-length tiles too)
#   occ6:      -DMIRSHA_AB_OCC6         (request kernel held to 6 waves/SIMD by LDS)
#   pf5:       -DMIRSHA_AB_PREFETCH     (next block chunks prefetched into registers, 5 waves/SIMD)
#   spawn:     -DMIRSHA_AB_SPAWN_THREADS (host passes on threads spawned per call instead of the pool)
#   yevery:    -DMIRSHA_AB_ROUNDS=rounds_asm_y_every (issue-yield s_nop after every 4-cycle op,
#              the round-1/2 form; other patterns: rounds_asm_y_* in tools/sha256_rounds_asm_ab.h)
#   latilp:    -DMIRSHA_AB_LAT_ROUNDS=rounds_asm_ilp (lone-wave chains: schedule woven into the rounds)
#   notail:    -DMIRSHA_AB_NOTAIL       (no final-block tail form: every block through compress_asm)
#   AB_ONLY="a b" builds only the named variants.
#   prioN:     -DMIRSHA_PRIO_TOP=N      (block b's rounds at issue priority max(0, N - b), clamped to 3; product 3)
set -euo pipefail
cd "$(dirname "$0")/.."
SRC=mirbft_amd/csrc
build() {
    local name=$1; shift
    if [ -n "${AB_ONLY:-}" ] && [[ " $AB_ONLY " != *" $name "* ]]; then return 0; fi
    mkdir -p tools/scratch/$name
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Itools "$@" -shared \
        -o tools/scratch/$name/libmirsha.so $SRC/mirsha_kernels.hip $SRC/mirsha_api.hip $SRC/mirsha_scan.hip $SRC/mirsha_host.cpp
}
build r1form -DMIRSHA_AB_KSGPR -DMIRSHA_AB_NOALIGNED -DMIRSHA_AB_OLDPROLOGUE &
build oldpro -DMIRSHA_AB_OLDPROLOGUE &
build noprio -DMIRSHA_AB_NOPRIO &
build wg4 -DMIRSHA_AB_WG4 &
build stamps -DMIRSHA_AB_STAMPS &
build ppad -DMIRSHA_AB_PRODUCER_PAD &
build occ6 -DMIRSHA_AB_OCC6 &
build pf5 -DMIRSHA_AB_PREFETCH &
build spawn -DMIRSHA_AB_SPAWN_THREADS &
build prio0 -DMIRSHA_PRIO_TOP=0 &
build yevery -DMIRSHA_AB_ROUNDS=rounds_asm_y_every &
build notail -DMIRSHA_AB_NOTAIL &
build latilp -DMIRSHA_AB_LAT_ROUNDS=rounds_asm_ilp &
wait
ls -la tools/scratch/*/libmirsha.so
