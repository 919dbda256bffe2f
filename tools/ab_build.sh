#!/bin/bash
# A/B builds of libmirsha.so from the product sources with measurement-only
# defines, into tools/scratch/<name>/ (git-ignored; travels to the GPU box).
# Select one at run time with MIRSHA_AB_LIB=tools/scratch/<name>/libmirsha.so.
#   r1form:    -DMIRSHA_AB_KSGPR -DMIRSHA_AB_NOALIGNED -DMIRSHA_AB_REGLOADER
#              (round constants in SGPRs, 5-dword chunks, register-staged loader)
#   regloader: -DMIRSHA_AB_REGLOADER                   (register-staged loader, no LDS-DMA)
#   stamps:    -DMIRSHA_AB_STAMPS                      (per-tile timeline for tools/stamp_run.py)
#   noprio:    -DMIRSHA_AB_NOPRIO                      (request-wave prologue at the default priority)
#   wg4:       -DMIRSHA_AB_WG4                         (4-wave request workgroups)
#   regloader is the register-staged loader; dmaearly issues the next block's
#   DMA before this block's rounds instead of between their halves; old_* use
#   the round-1 prologue (-DMIRSHA_AB_OLDPROLOGUE: shuffle reductions,
#   conditional metadata loads, default priority); *_wg4 4-wave workgroups.
set -euo pipefail
cd "$(dirname "$0")/.."
SRC=mirbft_amd/csrc
build() {
    local name=$1; shift
    mkdir -p tools/scratch/$name
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Itools "$@" -shared \
        -o tools/scratch/$name/libmirsha.so $SRC/mirsha_kernels.hip $SRC/mirsha_api.hip $SRC/mirsha_host.cpp
}
build r1form -DMIRSHA_AB_KSGPR -DMIRSHA_AB_NOALIGNED -DMIRSHA_AB_REGLOADER &
build regloader -DMIRSHA_AB_REGLOADER &
build stamps -DMIRSHA_AB_STAMPS &
build dmaearly -DMIRSHA_AB_DMA_EARLY &
build old_dmaearly_wg4 -DMIRSHA_AB_OLDPROLOGUE -DMIRSHA_AB_DMA_EARLY -DMIRSHA_AB_WG4 &
build old_reg_wg4 -DMIRSHA_AB_OLDPROLOGUE -DMIRSHA_AB_REGLOADER -DMIRSHA_AB_WG4 &
build old_dmaearly -DMIRSHA_AB_OLDPROLOGUE -DMIRSHA_AB_DMA_EARLY &
build old_reg -DMIRSHA_AB_OLDPROLOGUE -DMIRSHA_AB_REGLOADER &
wait
ls -la tools/scratch/*/libmirsha.so
