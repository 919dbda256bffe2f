#!/bin/bash
# A/B builds of libmirsha.so from the product sources with measurement-only
# defines, into tools/scratch/<name>/ (git-ignored; travels to the GPU box).
# Select one at run time with MIRSHA_AB_LIB=tools/scratch/<name>/libmirsha.so.
#   r1form:    -DMIRSHA_AB_KSGPR -DMIRSHA_AB_NOALIGNED  (round constants in SGPRs, 5-dword chunks)
#   noaligned: -DMIRSHA_AB_NOALIGNED                   (5-dword chunks only)
set -euo pipefail
cd "$(dirname "$0")/.."
SRC=mirbft_amd/csrc
build() {
    local name=$1; shift
    mkdir -p tools/scratch/$name
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Itools "$@" -shared \
        -o tools/scratch/$name/libmirsha.so $SRC/mirsha_kernels.hip $SRC/mirsha_api.hip $SRC/mirsha_host.cpp
}
build r1form -DMIRSHA_AB_KSGPR -DMIRSHA_AB_NOALIGNED &
build noaligned -DMIRSHA_AB_NOALIGNED &
wait
ls -la tools/scratch/*/libmirsha.so
