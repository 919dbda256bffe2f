// sha256_device.h — SHA-256 (FIPS 180-4) compression for gfx950, one message
// per lane.  Pure 32-bit integer VALU work: rotates lower to v_alignbit_b32,
// Ch/Maj to v_bitop3_b32, the Σ xors to v_xor3_b32, the sums to v_add3_u32.
// Replaces the block function of Go's crypto/sha256 that the reference's
// hash loop calls through `Hasher` (processor.go:21, :133-143).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sha256_rounds_asm.h"

namespace mirsha {

static constexpr uint32_t kK[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u,
    0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu,
    0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu,
    0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u,
    0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu,
    0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,
    0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u,
    0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u,
    0xc67178f2u};

static constexpr uint32_t kH0[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                    0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_rotateright32(x, n); }
// Three-input xor as ONE v_bitop3_b32 (truth table 0x96); hipcc otherwise
// splits it into two v_xor_b32.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t bsig0(uint32_t x) { return xor3(rotr(x, 2), rotr(x, 13), rotr(x, 22)); }
__device__ __forceinline__ uint32_t bsig1(uint32_t x) { return xor3(rotr(x, 6), rotr(x, 11), rotr(x, 25)); }
__device__ __forceinline__ uint32_t ssig0(uint32_t x) { return xor3(rotr(x, 7), rotr(x, 18), x >> 3); }
__device__ __forceinline__ uint32_t ssig1(uint32_t x) { return xor3(rotr(x, 17), rotr(x, 19), x >> 10); }
__device__ __forceinline__ uint32_t ch(uint32_t e, uint32_t f, uint32_t g) { return g ^ (e & (f ^ g)); }
// Majority is symmetric in its inputs, so truth table 0xE8 needs no operand-order care.
__device__ __forceinline__ uint32_t maj(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}

// One 64-byte block: st += F(st, w).  w[] holds the 16 big-endian message
// words on entry and is consumed as the rolling 16-word schedule window.
__device__ __forceinline__ void compress(uint32_t st[8], uint32_t w[16]) {
    uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
    uint32_t e = st[4], f = st[5], g = st[6], h = st[7];
#define MIRSHA_ROUND(a, b, c, d, e, f, g, h, j)                                              \
    {                                                                                        \
        if ((j) >= 16)                                                                       \
            w[(j)&15] += ssig1(w[((j)-2) & 15]) + w[((j)-7) & 15] + ssig0(w[((j)-15) & 15]);  \
        uint32_t t1 = h + bsig1(e) + ch(e, f, g) + kK[(j)] + w[(j)&15];                      \
        d += t1;                                                                             \
        h = t1 + bsig0(a) + maj(a, b, c);                                                    \
    }
#pragma unroll
    for (int j = 0; j < 64; j += 8) {
        MIRSHA_ROUND(a, b, c, d, e, f, g, h, j + 0);
        MIRSHA_ROUND(h, a, b, c, d, e, f, g, j + 1);
        MIRSHA_ROUND(g, h, a, b, c, d, e, f, j + 2);
        MIRSHA_ROUND(f, g, h, a, b, c, d, e, j + 3);
        MIRSHA_ROUND(e, f, g, h, a, b, c, d, j + 4);
        MIRSHA_ROUND(d, e, f, g, h, a, b, c, j + 5);
        MIRSHA_ROUND(c, d, e, f, g, h, a, b, j + 6);
        MIRSHA_ROUND(b, c, d, e, f, g, h, a, j + 7);
    }
#undef MIRSHA_ROUND
    st[0] += a; st[1] += b; st[2] += c; st[3] += d;
    st[4] += e; st[5] += f; st[6] += g; st[7] += h;
}

// The same compression with the 64 rounds in generated gfx950 assembly
// (sha256_rounds_asm.h): a..h + W[16] + 4 temporaries, no compiler-hoisted
// schedule partial sums.  Throughput form: an issue-yield `s_nop 0` after
// every second 4-cycle-class op (gen_rounds_asm.py, VARIANTS);
// the round constants are written into one scratch SGPR inside the asm, so a
// block loop keeps no 64 constant SGPRs live (SGPR count sets the waves per
// SIMD: MI355X_MICROARCH.md, residency).
__device__ __forceinline__ void compress_asm(uint32_t st[8], uint32_t w[16]) {
    uint32_t s[8];
#pragma unroll
    for (int i = 0; i < 8; i++) s[i] = st[i];
    rounds_asm(s, w);
#pragma unroll
    for (int i = 0; i < 8; i++) st[i] += s[i];
}

// compress_asm with work interleaved between its asm statements (hook(k)
// after statement k, see sha256_rounds_asm.h) and the state updated only on
// lanes with `live` set: every lane runs the rounds (a wave instruction costs
// the same at any exec mask), so a hook that stages data for the whole wave
// never runs under a divergent mask.
template <bool kNoYield = false, class H>
__device__ __forceinline__ void compress_asm_hooked(uint32_t st[8], uint32_t w[16], bool live, H hook) {
    uint32_t s[8];
#pragma unroll
    for (int i = 0; i < 8; i++) s[i] = st[i];
    if constexpr (kNoYield)
        rounds_asm_nonop(s, w, hook);
    else
        rounds_asm(s, w, hook);
#pragma unroll
    for (int i = 0; i < 8; i++) st[i] = live ? st[i] + s[i] : st[i];
}

// The wave-uniform scalars of a final block whose words 4..15 are all padding
// (FIPS 180-4 §5.1.1): u = message bytes in the block (at most 16; negative
// for the length-only block that follows a block ending in the 0x80 marker),
// L = message length.  Every field is passed through v_readfirstlane: the
// rotates have no scalar form and would otherwise stay VALU results, which
// the compiler hoists out of the block loop into VGPRs (the request kernel
// then spilled); called once per tile, before the loop.
__device__ __forceinline__ TailWords tail_words(int32_t u, uint32_t L) {
    auto sgpr = [](uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); };
    TailWords k;
    k.c4 = u == 16 ? 0x80000000u : 0u;
    k.c14 = L >> 29;
    k.c15 = L << 3;
    k.kw4 = kK[4] + k.c4;
    k.kw14 = kK[14] + k.c14;
    k.kw15 = kK[15] + k.c15;
    k.cs16 = sgpr(ssig1(k.c14));
    k.cs17 = sgpr(ssig1(k.c15));
    k.cs19 = sgpr(ssig0(k.c4));
    k.cs29 = sgpr(ssig0(k.c14));
    k.cs30 = sgpr(ssig0(k.c15) + k.c14);
    return k;
}

// compress_asm for such a final block: only w[0..3] are read (already padded).
__device__ __forceinline__ void compress_asm_tail(uint32_t st[8], uint32_t w[16], const TailWords& k) {
    uint32_t s[8];
#pragma unroll
    for (int i = 0; i < 8; i++) s[i] = st[i];
    rounds_asm_tail(s, w, k);
#pragma unroll
    for (int i = 0; i < 8; i++) st[i] += s[i];
}

// Latency form (no yields) for digest-list chains, which run at most one
// wave per SIMD: there the yields only lengthen the chain.
__device__ __forceinline__ void compress_asm_lat(uint32_t st[8], uint32_t w[16]) {
    uint32_t s[8];
#pragma unroll
    for (int i = 0; i < 8; i++) s[i] = st[i];
    rounds_asm_nonop(s, w);
#pragma unroll
    for (int i = 0; i < 8; i++) st[i] += s[i];
}

// Number of 64-byte compressions for an L-byte message: ceil((L + 9) / 64).
__device__ __host__ __forceinline__ uint32_t blocks_for_len(uint32_t L) { return (L + 72u) >> 6; }

// Big-endian word assembly straight from little-endian dwords at an arbitrary
// byte shift r (0..3): one v_perm_b32 does both the funnel shift and the byte
// swap.  lo = dword at the aligned address, hi = the next dword.
__device__ __forceinline__ uint32_t be_word(uint32_t hi, uint32_t lo, uint32_t sel) {
    return __builtin_amdgcn_perm(hi, lo, sel);
}
__device__ __forceinline__ uint32_t be_sel(uint32_t r) { return 0x00010203u + r * 0x01010101u; }

// FIPS 180-4 §5.1.1 padding applied to the 4 big-endian words at message byte
// position p (a 16-byte chunk of block `blk`, quarter q).  Only called for
// chunks that reach past the message end (p + 16 > L).
__device__ __forceinline__ void pad_chunk(uint32_t w[4], uint32_t p, uint32_t L, bool last_block,
                                          uint32_t q) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int64_t rem = (int64_t)L - (int64_t)(p + 4u * k);
        const uint32_t valid = rem <= 0 ? 0u : (rem >= 4 ? 4u : (uint32_t)rem);
        const uint32_t mask = valid == 4u ? 0xFFFFFFFFu : (valid == 0u ? 0u : ~(0xFFFFFFFFu >> (8u * valid)));
        uint32_t x = w[k] & mask;
        if (rem >= 0 && rem < 4) x |= 0x80u << (24u - 8u * (uint32_t)rem);
        w[k] = x;
    }
    if (last_block && q == 3u) {  // 64-bit big-endian bit length in words 14, 15
        w[2] = L >> 29;
        w[3] = L << 3;
    }
}

}  // namespace mirsha
