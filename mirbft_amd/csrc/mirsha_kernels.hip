// mirsha_kernels.hip — gfx950 kernels for MirBFT's Actions.Hash hot path.
//
//   sha256_msgs_kernel    request / generic messages packed in an arena
//                         (processor.go:129-143; one lane = one HashRequest)
//   sha256_lists_kernel   dependent second pass: digest of an ordered list of
//                         device-resident 32-byte digests (batch digests,
//                         sequence.go:154-157; VerifyBatch, batch_tracker.go:147-150;
//                         checkpoint chain, testengine/recorder.go:213-256)
//   gen_requests_kernel   synthetic request stream (bench/test utility, §8d)
//
// Layout: one wave (64 lanes) owns a tile of 64 messages, lane = message.
// In the LDS-staged form every lane is also a loader: per block, lane
// (j, q) = (lane>>2 + 16j, lane&3) fetches the 16-byte quarter q of message
// 16j + lane>>2 — 16 messages x 64 contiguous bytes per wave instruction —
// assembles big-endian words with one v_perm_b32 each, applies FIPS padding
// on the tail chunks, and writes them into the wave's private 4 KiB LDS tile,
// XOR-swizzled so both the ds_write_b128 (8-lane groups, 128 contiguous bytes)
// and the per-lane ds_read_b128 (16-lane groups) are bank-conflict free.
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstdio>

#include <hip/hip_ext.h>

#include "mirsha_kernels.h"
#include "sha256_device.h"

namespace mirsha {

// Wave-wide max / min, wave-uniform result (an SGPR).  DPP inside each 16-lane
// row (quad_perm xor 1 / xor 2, row_ror 4 / 8: four VALU ops, no LDS), then
// the four row results by v_readlane and a scalar reduction.  Called with all
// 64 lanes active (every call site is at a kernel's top, before divergence);
// a DPP source outside the row keeps the lane's own value.
// (The DPP moves' "old" operand is the op's identity, so hipcc folds each
// move into the max / min itself: v_max_u32_dpp, one VALU per step.)
template <bool kMax>
__device__ __forceinline__ uint32_t wave_reduce(uint32_t v) {
    auto op = [](uint32_t a, uint32_t b) { return kMax ? (a > b ? a : b) : (a < b ? a : b); };
    constexpr int id = kMax ? 0 : -1;
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0xB1, 0xF, 0xF, false));   // quad_perm [1,0,3,2]
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x4E, 0xF, 0xF, false));   // quad_perm [2,3,0,1]
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x124, 0xF, 0xF, false));  // row_ror:4
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x128, 0xF, 0xF, false));  // row_ror:8
    const uint32_t r0 = __builtin_amdgcn_readlane(v, 0), r1 = __builtin_amdgcn_readlane(v, 16);
    const uint32_t r2 = __builtin_amdgcn_readlane(v, 32), r3 = __builtin_amdgcn_readlane(v, 48);
    return op(op(r0, r1), op(r2, r3));
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v) { return wave_reduce<true>(v); }
__device__ __forceinline__ uint32_t wave_min(uint32_t v) { return wave_reduce<false>(v); }

// Raw 20 bytes (5 dwords) covering the 16-byte chunk q of block blk of a
// message at arena offset o: aligned down to 4 bytes, the byte shift is
// resolved later by v_perm.  Inactive chunks read at an out-of-range offset,
// which the buffer range check turns into zeros without a memory access.
struct RawChunk {
    uint32_t v[5];
    uint32_t sel;
};

__device__ __forceinline__ void issue_chunk(__amdgpu_buffer_rsrc_t rsrc, uint32_t records, uint32_t o,
                                            uint32_t blk, uint32_t q, bool active, RawChunk& c) {
    const uint32_t addr = o + 64u * blk + 16u * q;
    const uint32_t a = active ? (addr & ~3u) : 0xFFFFFFE0u;
    c.sel = be_sel(addr & 3u);
    // The range check covers a whole access: a 16-byte load straddling the end
    // of the arena would return 0 for its in-range bytes too.  The arena's last
    // chunk therefore takes 5 dword loads — in asm, because hipcc otherwise
    // merges adjacent buffer dword loads back into one dwordx4.
    if (a + 20u <= records || !active) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, a, 0, 0);
        c.v[0] = v[0]; c.v[1] = v[1]; c.v[2] = v[2]; c.v[3] = v[3];
        c.v[4] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, a + 16u, 0, 0);
    } else {
        asm volatile(
            "s_nop 4\n\t"
            "buffer_load_dword %0, %5, %6, 0 offen\n\t"
            "buffer_load_dword %1, %5, %6, 0 offen offset:4\n\t"
            "buffer_load_dword %2, %5, %6, 0 offen offset:8\n\t"
            "buffer_load_dword %3, %5, %6, 0 offen offset:12\n\t"
            "buffer_load_dword %4, %5, %6, 0 offen offset:16\n\t"
            "s_waitcnt vmcnt(0)"
            : "=&v"(c.v[0]), "=&v"(c.v[1]), "=&v"(c.v[2]), "=&v"(c.v[3]), "=&v"(c.v[4])
            : "v"(a), "s"(rsrc)
            : "memory");
    }
}

// The same raw chunk through 64-bit per-lane global addresses, for arenas
// beyond one buffer descriptor's 32-bit reach (> 4 GiB per launch, BASELINE
// config 5).  Same semantics: inactive chunks and dwords past `records`
// (arena_len rounded up to 4) read as zero without a memory access.
typedef uint32_t u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
__device__ __forceinline__ void issue_chunk_wide(const uint8_t* __restrict__ arena, uint64_t records, uint64_t o,
                                                 uint32_t blk, uint32_t q, bool active, RawChunk& c) {
    const uint64_t addr = o + 64ull * blk + 16u * q;
    const uint64_t a = addr & ~3ull;
    c.sel = be_sel((uint32_t)addr & 3u);
#pragma unroll
    for (int k = 0; k < 5; k++) c.v[k] = 0u;
    if (active) {
        const uint32_t* p = reinterpret_cast<const uint32_t*>(arena + a);
        if (a + 20u <= records) {
            const u32x4a4 v = *reinterpret_cast<const u32x4a4*>(p);
            c.v[0] = v[0]; c.v[1] = v[1]; c.v[2] = v[2]; c.v[3] = v[3];
            c.v[4] = p[4];
        } else {
#pragma unroll
            for (int k = 0; k < 5; k++)
                if (a + 4u * k + 4u <= records) c.v[k] = p[k];
        }
    }
}

// Big-endian SHA words of the chunk at message byte position p, with FIPS
// 180-4 §5.1.1 padding (0x80, zeros, 64-bit bit length in words 14/15 of the
// last block) applied branch-free on chunks that reach past the message end.
__device__ __forceinline__ void pad_words(uint32_t p, uint32_t L, bool last_block, uint32_t q, uint32_t out[4]) {
    if (p + 16u > L) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int32_t t = (int32_t)(L - (p + 4u * k));  // message bytes left at this word
            const uint32_t sh = (uint32_t)t << 3;          // only used when 0 <= t <= 3
            const uint32_t keep = ~(0xFFFFFFFFu >> sh);    // the t leading data bytes
            const uint32_t mark = 0x80000000u >> sh;       // the 0x80 byte right after them
            const uint32_t part = (out[k] & keep) | mark;
            out[k] = t >= 4 ? out[k] : (t < 0 ? 0u : part);
        }
        if (last_block && q == 3u) {
            out[2] = L >> 29;
            out[3] = L << 3;
        }
    }
}

// The same padding for a whole block of 16 words when the block position
// soff, the length L and `last` are wave-uniform (SGPRs): the keep / mark
// words are scalar, one v_bitop3 per word.
// kWords < 16: only the first kWords words (the final-block tail form keeps
// the rest, and the bit length, as scalars).
template <int kWords = 16>
__device__ __forceinline__ void pad_block_uniform(uint32_t w[16], uint32_t soff, uint32_t L, bool last) {
#pragma unroll
    for (int k = 0; k < kWords; k++) {
        const int32_t t = (int32_t)(L - (soff + 4u * k));  // message bytes left at word k
        const uint32_t sh = (uint32_t)t << 3;              // only used when 0 <= t <= 3
        uint32_t keep = t >= 4 ? 0xFFFFFFFFu : (t <= 0 ? 0u : ~(0xFFFFFFFFu >> sh));
        uint32_t mark = (t >= 0 && t < 4) ? 0x80000000u >> sh : 0u;
        if (k >= 14 && last) {  // 64-bit big-endian bit length
            keep = 0u;
            mark = k == 14 ? L >> 29 : L << 3;
        }
        keep = __builtin_amdgcn_readfirstlane(keep);
        mark = __builtin_amdgcn_readfirstlane(mark);
        w[k] = (w[k] & keep) | mark;
    }
}

__device__ __forceinline__ void finish_chunk(const RawChunk& c, uint32_t p, uint32_t L, bool last_block,
                                             uint32_t q, uint32_t out[4]) {
#pragma unroll
    for (int k = 0; k < 4; k++) out[k] = be_word(c.v[k + 1], c.v[k], c.sel);
    pad_words(p, L, last_block, q, out);
}

// Swizzled 16-byte slot of (message m, quarter q) inside a wave's 256-slot tile.
__device__ __forceinline__ uint32_t lds_slot(uint32_t m, uint32_t q) {
    return m * 4u + (q ^ ((m >> 2) & 3u));
}

__device__ __forceinline__ void store_digest(uint8_t* out, uint32_t msg, const uint32_t st[8]) {
    uint4* d = reinterpret_cast<uint4*>(out + 32ull * msg);
    d[0] = make_uint4(__builtin_bswap32(st[0]), __builtin_bswap32(st[1]), __builtin_bswap32(st[2]),
                      __builtin_bswap32(st[3]));
    d[1] = make_uint4(__builtin_bswap32(st[4]), __builtin_bswap32(st[5]), __builtin_bswap32(st[6]),
                      __builtin_bswap32(st[7]));
}

__device__ __forceinline__ void store_digest_buf(__amdgpu_buffer_rsrc_t ors, uint32_t msg, const uint32_t st[8]) {
    __builtin_amdgcn_raw_buffer_store_b128(
        (uint32_t __attribute__((ext_vector_type(4)))){__builtin_bswap32(st[0]), __builtin_bswap32(st[1]),
                                                        __builtin_bswap32(st[2]), __builtin_bswap32(st[3])},
        ors, 32u * msg, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(
        (uint32_t __attribute__((ext_vector_type(4)))){__builtin_bswap32(st[4]), __builtin_bswap32(st[5]),
                                                        __builtin_bswap32(st[6]), __builtin_bswap32(st[7])},
        ors, 32u * msg + 16u, 0, 0);
}

// Digest store with the sc1 cache policy: written through to memory (the line
// leaves this XCD's L2), so a list wave on any XCD can read it with sc1 loads
// once the storing wave has signalled (MI355X_MICROARCH.md, inter-workgroup
// visibility: stores and loads all sc1, one atomic add per storing wave).
constexpr int kSc1 = 1 << 4;  // gfx940+ cache-policy bit: buffer_* ... sc1

__device__ __forceinline__ void store_digest_sc1(__amdgpu_buffer_rsrc_t ors, uint32_t msg, const uint32_t st[8]) {
    __builtin_amdgcn_raw_buffer_store_b128(
        (uint32_t __attribute__((ext_vector_type(4)))){__builtin_bswap32(st[0]), __builtin_bswap32(st[1]),
                                                        __builtin_bswap32(st[2]), __builtin_bswap32(st[3])},
        ors, 32u * msg, 0, kSc1);
    __builtin_amdgcn_raw_buffer_store_b128(
        (uint32_t __attribute__((ext_vector_type(4)))){__builtin_bswap32(st[4]), __builtin_bswap32(st[5]),
                                                        __builtin_bswap32(st[6]), __builtin_bswap32(st[7])},
        ors, 32u * msg + 16u, 0, kSc1);
}

// Issue priority of a request wave, set before each block's rounds: block b
// runs at max(0, kPrioTop - b), so a wave that is behind wins issue over one
// that is ahead.  The SIMD's arbiter otherwise runs its waves in age order:
// the oldest finish first and the second generation inherits their spread,
// which left the last ~80 us of a config-2 launch draining from 8 to 0 waves
// per SIMD (profiles/r02n stamps).  Same-box A/B over two boxes
// (profiles/r02p, profiles/r02r), config 2 request kernel: top 3 189.9 /
// 190.1 us vs 193.8 / 193.3 us with every block at priority 0; tops 1 and 2
// and a high top for the launch's last generation only were in between or
// box-dependent.
constexpr uint32_t kPrioTop = 3;
__device__ __forceinline__ void progress_prio(uint32_t blk) {
    blk = (uint32_t)__builtin_amdgcn_readfirstlane((int)blk);  // scalar branches (see fixed_prio)
    const uint32_t p = blk < kPrioTop ? kPrioTop - blk : 0u;
    if (p >= 3u) __builtin_amdgcn_s_setprio(3);
    else if (p == 2u) __builtin_amdgcn_s_setprio(2);
    else if (p == 1u) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
}

// One wave hashes the tile of 64 messages at processing positions
// [64 t, 64 t + 64) (order[] maps a position to a message; NULL = identity).
// kLds: LDS-staged coalesced loader (else direct per-lane loads); kWide:
// 64-bit per-lane addresses for arenas beyond one buffer descriptor.
// Fixed issue priority of a fused-launch tile wave (its queue's), set before
// each block's rounds in place of progress_prio.
constexpr uint32_t kPrioProgress = 4;  // hash_tile<kFused>'s fprio: progress_prio instead of a fixed one
// The priority is wave-uniform; readfirstlane keeps the branches below scalar.
// When the compiler took it for a per-lane value, the branches became
// exec-mask regions and more than one s_setprio could execute (s_setprio
// ignores exec): fused config-3 runs then had some queue-0 waves at the
// lowest priority, ending with queue 3 (profiles/r04f, tools/trace_queues.py).
__device__ __forceinline__ void fixed_prio(uint32_t p) {
    p = (uint32_t)__builtin_amdgcn_readfirstlane((int)p);
    if (p >= 3u) __builtin_amdgcn_s_setprio(3);
    else if (p == 2u) __builtin_amdgcn_s_setprio(2);
    else if (p == 1u) __builtin_amdgcn_s_setprio(1);
    else __builtin_amdgcn_s_setprio(0);
}

// hash_tile<kFused>'s fprio: priority by rank of progress among the tile waves
// of the SIMD (FusedArgs::tile_prio_progress == 2, overlapped cycles).  Each
// wave publishes its block in its LDS word (g_bal_prog; an idle or finished
// wave's word is kBalDone) and, before each block, takes priority 3 minus the
// number of the SIMD's waves it is ahead of: the wave furthest behind wins
// issue.  With one fixed priority after a few blocks the arbiter's age order
// ran the SIMD's waves one after another instead (config 3's overlapped
// launch: waves ending at ~420 / 450 / 600 / 760 us, the last ~150 us at one
// wave per SIMD, tools/trace_overlap.py); by rank they end together
// (profiles/r03q, r03r: 706 -> 662 us).  The CU-block request kernel is
// better off without it (677 vs 646 us, profiles/r03w): there no segment
// host falls behind.
constexpr uint32_t kPrioBalance = 5;
constexpr uint32_t kBalDone = 0xFFFFFFFFu;
// [SIMD][hardware wave slot] (HW_ID's SIMD_ID and WAVE_ID fields: read with
// s_getreg where needed, so no register stays live across the block loop of
// the fused kernel, which sits at its 128-VGPR budget).
__shared__ uint32_t g_bal_prog[4 * 16];

// An LDS word read through inline asm: for an ordinary (or atomic) LDS
// access the compiler cannot prove distinct from a tile the wave's LDS-DMA is
// still filling, so it waits for every outstanding vector-memory op first
// (s_waitcnt vmcnt(0)), i.e. for the DMA of the next block(s) -- which turned
// the loads' prefetch into a full memory round trip per block (a lone wave:
// +750 cycles per block, tools/lone_probe.hip mode 7, profiles/r04l).  The
// word is never a DMA target; only the wave's own LDS ops are waited for.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(size_t)(const __attribute__((address_space(3))) void*)p;
}
__device__ __forceinline__ uint32_t lds_load_nodma(const uint32_t* p) {
    uint32_t v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(lds_addr(p)) : "memory");
    return v;
}

// Live waves per SIMD of a fused-launch workgroup (set to the waves per SIMD
// at launch, decremented as each wave leaves).  A tile wave that finds itself
// the only one left runs its blocks in the latency round form: the issue
// yields of the throughput form only stall a lone wave (tools/ilp_asm_probe,
// profiles/r04k: 7,424 vs 5,991 cycles per compression at one wave per SIMD,
// 5,314 vs 5,607 at four).
__shared__ uint32_t g_simd_live[4];
constexpr uint32_t kLoneSeen = 0xFFFFFFFFu;  // hash_tile's lone_sel once the wave has been seen alone
__device__ __forceinline__ bool simd_alone(uint32_t sel) {  // sel = SIMD + 1 (0: never)
    if (sel == 0u || sel == kLoneSeen) return sel != 0u;
    const uint32_t n = lds_load_nodma(&g_simd_live[sel - 1u]);
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)n) <= 1u;
}
__device__ __forceinline__ uint32_t bal_word() {
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    return ((hw >> 4) & 3u) * 16u + (hw & 15u);
}
__device__ __forceinline__ void balance_prio(uint32_t blk) {
    const uint32_t me = bal_word();
    // (atomics, not lds_load_nodma: the inline-asm form spilled the fused
    // kernel; the compiler's vmcnt wait stays on this overlapped-cycles path)
    __hip_atomic_store(g_bal_prog + me, blk, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const uint32_t* row = g_bal_prog + (me & ~15u);
    uint32_t ahead = 0;
#pragma unroll
    for (uint32_t k = 0; k < 16; k++)
        ahead += __hip_atomic_load(row + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < blk ? 1u : 0u;
    fixed_prio(3u - min(3u, (uint32_t)__builtin_amdgcn_readfirstlane((int)ahead)));
}
__device__ __forceinline__ void balance_done() {
    __hip_atomic_store(g_bal_prog + bal_word(), kBalDone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Software-pipelined block loop of a tile (kPf: launches of at most 4 waves
// per SIMD, which leave a wave 128 VGPRs), for tiles whose messages are all
// 4-byte aligned and whose loads all stay inside the arena.  Block b+1's
// words are staged WHILE block b's rounds run, between the round statements
// (compress_asm_hooked): after rounds 0-7 its raw chunks (loaded one block
// earlier) are byte-swapped and written to the wave's LDS tile and block b+2's
// chunks are loaded; after rounds 16-23 the transposed words are read back.
// So the transpose's LDS round trip and the loads hide behind this wave's own
// rounds: with 4 waves per SIMD started together (config 3) the waves reach
// their staging at the same time and the one-at-a-time form left the SIMD
// short of issuable waves there (643 us per config-3 launch, profiles/r03b).
template <bool kNoYield>
__device__ __forceinline__ void hash_tile_pipelined(__amdgpu_buffer_rsrc_t rsrc, const uint32_t vo[4],
                                                    const uint32_t sel[4], uint32_t L, uint32_t min_l, bool uni,
                                                    bool tail_ok, const TailWords& tw, uint32_t wave_nb,
                                                    uint32_t loop_nb, uint32_t nb, uint32_t lane, uint4* my,
                                                    uint32_t st[8]) {
    const uint32_t q = lane & 3u;
    uint32_t nx[4][4];  // raw chunks of the next block to stage
    auto load_raw = [&](uint32_t blk) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, vo[j], 64u * blk, 0);
            nx[j][0] = v[0]; nx[j][1] = v[1]; nx[j][2] = v[2]; nx[j][3] = v[3];
        }
    };
    // Words of block blk (raw chunks in nx) into the LDS tile; mixed tiles pad
    // per chunk here, uniform tiles after the read (pad_block_uniform).
    auto write_tile = [&](uint32_t blk) {
        const uint32_t soff = 64u * blk;
        const bool pad = soff + 64u > min_l;  // wave-uniform
#pragma unroll
        for (int j = 0; j < 4; j++) {
            uint32_t wq[4];
#pragma unroll
            for (int k = 0; k < 4; k++) wq[k] = be_word(k < 3 ? nx[j][k + 1] : 0u, nx[j][k], sel[j]);
            if (pad && !uni) {
                const uint32_t Lm = (uint32_t)__shfl((int)L, 16 * j + (int)(lane >> 2), 64);
                pad_words(soff + 16u * q, Lm, blk + 1u == blocks_for_len(Lm), q, wq);
            }
            my[lds_slot(16u * j + (lane >> 2), q)] = make_uint4(wq[0], wq[1], wq[2], wq[3]);
        }
        // LDS ops of a wave execute in order; the fences only keep the compiler
        // from moving the reads above the writes.
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    auto read_tile = [&](uint32_t w[16]) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const uint4 x = my[lds_slot(lane, (uint32_t)k)];
            w[4 * k + 0] = x.x; w[4 * k + 1] = x.y; w[4 * k + 2] = x.z; w[4 * k + 3] = x.w;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    auto pad_uniform = [&](uint32_t blk, uint32_t w[16]) {
        if (64u * blk + 64u > min_l && uni) {  // wave-uniform
            uint32_t wnb;  // opaque copy: no loop peeling to fold the test (see hash_tile)
            asm volatile("s_mov_b32 %0, %1" : "=s"(wnb) : "s"(wave_nb));
            pad_block_uniform(w, 64u * blk, min_l, wnb - blk == 1u);
        }
    };
    uint32_t w[16];
    load_raw(0u);
    write_tile(0u);
    if (1u < wave_nb) load_raw(1u);
    read_tile(w);
    for (uint32_t blk = 0; blk < loop_nb; blk++) {
        pad_uniform(blk, w);
        const bool next = blk + 1u < wave_nb;  // wave-uniform
        uint32_t wn[16];
        progress_prio(blk);
        compress_asm_hooked<kNoYield>(st, w, blk < nb, [&](int k) {
            if (k == 0 && next) {
                write_tile(blk + 1u);
                if (blk + 2u < wave_nb) load_raw(blk + 2u);
            } else if (k == 2 && next) {
                read_tile(wn);
            }
        });
#pragma unroll
        for (int i = 0; i < 16; i++) w[i] = wn[i];
    }
    if (tail_ok) {  // final block (<= 16 message bytes), staged during the loop's last block
        const uint32_t blk = wave_nb - 1u;
        pad_block_uniform<4>(w, 64u * blk, min_l, false);
        progress_prio(blk);
        if (blk < nb) compress_asm_tail(st, w, tw);
    }
}

// kFused (sha256_fused_paced_kernel's tile waves): blocks at the fixed
// priority fprio, digests stored with sc1 for list waves on other CUs.
// kPf (launches of at most 4 waves per SIMD, which leave 128 VGPRs per wave):
// the next block's chunks are staged while this block's rounds run
// (hash_tile_pipelined).
// Block range (the fused launch's split tiles, LDS loader only): blocks
// [b0, b1) of the tile, from the midstate in st (H0 when b0 == 0).  Returns
// kTileDone when the range reached the tile's end (the digest is then
// stored), kTilePaused when it did not (st_io then holds the midstate after
// block b1 - 1).  (A range that starts at or past the tile's end is never
// passed: the fused launch skips such split-tile segments itself.)
constexpr uint32_t kTilePaused = 0, kTileDone = 1;
// kDiag (diagnostic builds of the CU-block kernel only, variants 14 / 15,
// MIRSHA_AB=1; digests are NOT valid under 1): 1 = no block loads (the
// rounds run on the LDS tile's stale words), 2 = no per-block s_setprio.
template <bool kLds, bool kWide, bool kFused = false, bool kPf = false, bool kNoYield = false, bool kDma = false,
          bool kDmaPipe = false, int kDiag = 0>
__device__ __forceinline__ uint32_t hash_tile(const uint8_t* __restrict__ arena, uint64_t arena_len,
                                          const uint64_t* __restrict__ off, const uint32_t* __restrict__ len,
                                          const uint32_t* __restrict__ order, uint32_t n, uint8_t* __restrict__ out,
                                          uint4* my, uint32_t t, uint32_t lane, uint32_t fprio = 0,
                                          uint32_t b0 = 0u, uint32_t b1 = 0xFFFFFFFFu, uint32_t* st_io = nullptr,
                                          uint32_t lone_sel = 0u, uint4* my2 = nullptr,
                                          unsigned long long* lone_tr = nullptr) {
    auto block_prio = [&](uint32_t blk) {
        if constexpr (kDiag == 2) {
            return;
        } else if constexpr (kFused) {
            if (fprio == kPrioBalance)
                balance_prio(blk);
            else if (fprio == kPrioProgress)
                progress_prio(blk);
            else
                fixed_prio(fprio);
        } else {
            progress_prio(blk);
        }
    };
    // Prologue at the highest issue priority, back to 0 at the first
    // compression: a fresh wave is the youngest on its SIMD and at the default
    // priority gets the VALU only when every older wave stalls, so its
    // metadata loads and first block took ~20 us of a ~60-90 us wave life
    // (tools/stamp_run.py).  Same-box A/B (profiles/r02h): 196.4 us per
    // config-2 launch vs 201.9 us without.
    __builtin_amdgcn_s_setprio(3);
    const uint32_t slot = t * 64u + lane;
    const bool valid = slot < n;
    // Unconditional loads (n >= 1; an idle lane reads the last message's
    // entries), so the length and offset loads issue together.
    const uint32_t slot_c = valid ? slot : n - 1u;
    const uint32_t msg = order ? order[slot_c] : slot_c;
    const uint32_t L_ = len[msg];
    const uint64_t o_ = off[msg];
    const uint32_t L = valid ? L_ : 0u;
    const uint64_t o = valid ? o_ : 0u;
    const uint32_t nb = valid ? blocks_for_len(L) : 0u;
    // The tile's longest message, and from it (blocks_for_len is monotone) the
    // wave-uniform block count (SGPR: scalar block-loop tests).
    const uint32_t max_l = wave_max(valid ? L : 0u);
    const uint32_t wave_nb = blocks_for_len(max_l);

    // Bytes past arena_len inside the last dword are never part of a message
    // (they are masked by the padding logic), so the range rounds up to 4.
    const uint64_t records = (arena_len + 3u) & ~3ull;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)arena, (short)0, (int)(uint32_t)records, 0x00020000);
    auto issue = [&](uint64_t mo, uint32_t blk, uint32_t q, bool active, RawChunk& rc) {
        if constexpr (kWide)
            issue_chunk_wide(arena, records, mo, blk, q, active, rc);
        else
            issue_chunk(rsrc, (uint32_t)records, (uint32_t)mo, blk, q, active, rc);
    };

    uint32_t st[8];
#pragma unroll
    for (int i = 0; i < 8; i++) st[i] = (st_io && b0) ? st_io[i] : kH0[i];
    const bool finished = b1 >= wave_nb;

    if constexpr (kLds && !kWide) {
        // Loader roles: this lane fetches quarter q of messages m_j = 16j + lane/4.
        // Chunk addresses are loop-invariant VGPRs with the block in the
        // scalar offset.  There is no per-chunk activity test: a finished
        // message's chunk reads bytes nobody uses (in range) or zeros (out of
        // range).  A tile whose every load stays in the arena (all but the
        // arena's last tiles; a wave-uniform test) takes plain loads; the
        // others range-check each chunk (the 5-dword tail form of
        // issue_chunk).  The FIPS padding logic runs only on blocks that reach
        // past the wave's shortest message.
        const uint32_t q = lane & 3u;
        const uint64_t reach = valid ? o + 64ull * wave_nb + 20u : 0ull;
        const bool far = __builtin_amdgcn_ballot_w64(reach > records) == 0;
        // Every message of the tile 4-byte aligned (wave-uniform): a chunk's
        // words are its own 16 bytes, byte-swapped, so the fifth dword of the
        // funnel shift is never loaded (4 instead of 8 loads per block).
        const bool aligned = __builtin_amdgcn_ballot_w64(valid && (o & 3u) != 0u) == 0;
        // Wave-uniform (SGPR), so the padding test below is a scalar branch (as
        // a VGPR compare it became an exec-mask branch with the word assembly
        // duplicated).
        const uint32_t min_l = wave_min(valid ? L : 0xFFFFFFFFu);
        // Every valid message of the tile the same length (wave-uniform; the
        // common case: BASELINE configs 2 and 3, batch digest lists): the FIPS
        // padding words of a block are then the same for every lane, so they
        // are applied once per lane AFTER the LDS transpose, with the masks
        // computed on the scalar unit (16 VALU per padded block instead of the
        // per-chunk form's ~128 on the loader side).
        const bool uni = max_l == min_l;
        // Final-block tail form (compress_asm_tail) for uniform tiles whose
        // final block holds at most 16 message bytes; its scalars up front.
        const int32_t u_last = (int32_t)(min_l - 64u * (wave_nb - 1u));
        const bool tail_ok = uni && u_last <= 16;
        const TailWords tw = tail_words(u_last, min_l);
        uint32_t vo[4], sel[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const uint32_t a = (uint32_t)__shfl((int)(uint32_t)o, 16 * j + (int)(lane >> 2), 64) + 16u * q;
            vo[j] = a & ~3u;
            sel[j] = be_sel(a & 3u);
        }
        // One block of the tile into w[] (lane = message): loads, big-endian
        // words, per-chunk padding of mixed tiles, the LDS transpose.
        // trim (the tail-form final block): chunks wholly past the tile's
        // length are not loaded (zeros; words 4..15 are never read there),
        // so a config-2 request's final block fetches its 16 bytes, not 64.
        auto stage = [&](uint32_t blk, uint32_t w[16], uint32_t ln, bool trim) {
            const uint32_t soff = 64u * blk;
            const uint32_t qq = ln & 3u;
            const bool skip = trim && soff + 16u * qq >= min_l;
            RawChunk rc[4];
            if (far && !trim) {
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, vo[j], soff, 0);
                    rc[j].v[0] = v[0]; rc[j].v[1] = v[1]; rc[j].v[2] = v[2]; rc[j].v[3] = v[3];
                    rc[j].v[4] = 0u;
                }
                if (!aligned) {
#pragma unroll
                    for (int j = 0; j < 4; j++)
                        rc[j].v[4] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, vo[j], soff + 16u, 0);
                }
            } else if (far) {
                // a skipped chunk reads past the descriptor's range: zeros, no access
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const uint32_t a = skip ? 0xFFFFFFE0u : vo[j] + soff;
                    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, a, 0, 0);
                    rc[j].v[0] = v[0]; rc[j].v[1] = v[1]; rc[j].v[2] = v[2]; rc[j].v[3] = v[3];
                    rc[j].v[4] = aligned ? 0u : __builtin_amdgcn_raw_buffer_load_b32(rsrc, a + 16u, 0, 0);
                }
            } else {
#pragma unroll
                for (int j = 0; j < 4; j++)
                    issue_chunk(rsrc, (uint32_t)records, vo[j] + soff, 0u, 0u, !skip, rc[j]);
            }
            const bool pad = soff + 64u > min_l;  // wave-uniform
#pragma unroll
            for (int j = 0; j < 4; j++) {
                uint32_t wq[4];
#pragma unroll
                for (int k = 0; k < 4; k++) wq[k] = be_word(rc[j].v[k + 1], rc[j].v[k], sel[j]);
                if (pad && !uni) {
                    // Lengths fetched here (rare blocks), not kept live across the rounds.
                    const uint32_t Lm = (uint32_t)__shfl((int)L, 16 * j + (int)(ln >> 2), 64);
                    pad_words(soff + 16u * qq, Lm, blk + 1u == blocks_for_len(Lm), qq, wq);
                }
                // Unconditional: a slot of a finished message is never read.
                my[lds_slot(16u * j + (ln >> 2), qq)] = make_uint4(wq[0], wq[1], wq[2], wq[3]);
            }
            // Cross-lane hand-off inside one wave: LDS ops of a wave execute
            // in order; the fences only stop the compiler from reordering.
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint4 x = my[lds_slot(ln, (uint32_t)k)];
                w[4 * k + 0] = x.x; w[4 * k + 1] = x.y; w[4 * k + 2] = x.z; w[4 * k + 3] = x.w;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        };
        // A uniform tile's tail-form final block runs after the loop, not as a
        // branch inside it: two round copies joined inside the loop made the
        // register allocator spill (64 VGPRs is the 8-wave budget).
        const uint32_t loop_nb = tail_ok ? wave_nb - 1u : wave_nb;
        if constexpr (kPf && !kDma && !kDmaPipe) {
            if (far && aligned && b0 == 0u && finished) {
                hash_tile_pipelined<kNoYield>(rsrc, vo, sel, L, min_l, uni, tail_ok, tw, wave_nb, loop_nb, nb, lane, my,
                                              st);
                goto digest;
            }
        }
        const uint32_t loop_end = min(loop_nb, b1);
        // Fused launch, aligned in-range tiles: the block loop below with the
        // loads as LDS-DMA (buffer_load_dwordx4 ... lds), block b+1's issued as
        // soon as block b's words are read back, so they land while b's rounds
        // run.  The fused launch runs 4 waves per SIMD and fewer as its queues
        // end (the last queue runs its final stretch alone), where the
        // register-staged loader's load latency was exposed every block; the
        // register prefetch of hash_tile_pipelined does not fit its 128 VGPRs.
        // Lane l of piece j fetches slot 64 j + l of the swizzled tile
        // (lds_slot's inverse), so the transposed read back is the loader's.
        bool dma = false;
        if constexpr (kFused || kDma || kDmaPipe) dma = far && aligned;
        if (dma) {
            const uint32_t qd = (lane & 3u) ^ ((lane >> 4) & 3u);
            uint32_t vd[4];
#pragma unroll
            for (int j = 0; j < 4; j++)
                vd[j] = (uint32_t)__shfl((int)(uint32_t)o, 16 * j + (int)(lane >> 2), 64) + 16u * qd;
            // Two blocks in flight (kFused, my2 != nullptr: the last queue's
            // waves, which end their tiles alone on the SIMD, where one block
            // of lead did not cover the load latency): block b lands in tile
            // b & 1 (my, my2) and block b + 2's DMA follows b's read-back.
            const bool deep = kFused && my2 != nullptr;  // wave-uniform
            auto tile_of = [&](uint32_t blk) { return (deep && (blk & 1u)) ? my2 : my; };
            auto issue_dma = [&](uint32_t blk) {
                if constexpr (kDiag == 1) return;
                uint4* t = tile_of(blk);
#pragma unroll
                for (int j = 0; j < 4; j++)
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(
                        rsrc, (__attribute__((address_space(3))) void*)(t + 64 * j), 16, vd[j], 64u * blk, 0, 0);
            };
            // (bounds through readfirstlane: the block index is the DMA's
            // scalar offset, and a bound the compiler takes for divergent
            // turned every DMA into a waterfall loop)
            const uint32_t d0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)b0);
            const uint32_t d1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)loop_end);
            const uint32_t dmin = (uint32_t)__builtin_amdgcn_readfirstlane((int)min_l);
            // kDmaPipe (A/B): block b+1's words are read back from LDS in the
            // middle of block b's rounds (after statement 2; the wait for the
            // reads after statement 4, then block b+2's DMA), so neither the
            // DMA's landing nor the LDS round trip sits between two blocks.
            // 16 more live VGPRs (the next block's words): CU-block kernel only.
            auto read_words = [&](uint32_t x[16]) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the block landed in LDS
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint4 v = my[lds_slot(lane, (uint32_t)k)];
                    x[4 * k + 0] = v.x; x[4 * k + 1] = v.y; x[4 * k + 2] = v.z; x[4 * k + 3] = v.w;
                }
            };
            auto finish_words = [&](uint32_t blk, uint32_t x[16]) {
#pragma unroll
                for (int k = 0; k < 16; k++) x[k] = __builtin_bswap32(x[k]);
                if (64u * blk + 64u > dmin) {  // wave-uniform
                    uint32_t wnb;  // (opaque copy, as below)
                    asm volatile("s_mov_b32 %0, %1" : "=s"(wnb) : "s"(wave_nb));
                    if (uni) {
                        pad_block_uniform(x, 64u * blk, dmin, wnb - blk == 1u);
                    } else {
#pragma unroll
                        for (int k = 0; k < 4; k++)
                            pad_words(64u * blk + 16u * (uint32_t)k, L, blk + 1u == nb, (uint32_t)k, &x[4 * k]);
                    }
                }
            };
            if constexpr (kDmaPipe) {
                if (d0 < d1) {
                    uint32_t w[16];
                    issue_dma(d0);
                    read_words(w);
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    if (d0 + 1u < d1) issue_dma(d0 + 1u);
                    for (uint32_t blk = d0; blk < d1; blk++) {
                        finish_words(blk, w);
                        block_prio(blk);
                        const bool next = blk + 1u < d1, next2 = blk + 2u < d1;  // wave-uniform
                        uint32_t wn[16];
                        compress_asm_hooked(st, w, blk < nb, [&](int k) {
                            if (k == 2 && next) {
                                read_words(wn);
                            } else if (k == 4 && next) {
                                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads back: free the tile
                                if (next2) issue_dma(blk + 2u);
                            }
                        });
#pragma unroll
                        for (int i = 0; i < 16; i++) w[i] = wn[i];
                    }
                }
            }
            if (!kDmaPipe && d0 < d1) {
                issue_dma(d0);
                if (deep && d0 + 1u < d1) issue_dma(d0 + 1u);
            }
            for (uint32_t blk = kDmaPipe ? d1 : d0; blk < d1; blk++) {
                const uint32_t soff = 64u * blk;
                // block blk landed in LDS (deep: block blk + 1's 4 loads may stay in flight)
                if (deep && blk + 1u < d1)
                    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                else
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                // Fused tile waves set the block's priority here, right after the
                // wait for this block's DMA: kPrioBalance's LDS words are plain
                // LDS ops, before which hipcc waits for every in-flight LDS-DMA
                // (lds_load_nodma); here that wait is already paid (one block
                // in flight; the deep staging is off in overlapped launches).
                if constexpr (kFused) block_prio(blk);
                uint32_t w[16];
                const uint4* tb = tile_of(blk);
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    const uint4 x = tb[lds_slot(lane, (uint32_t)k)];
                    w[4 * k + 0] = x.x; w[4 * k + 1] = x.y; w[4 * k + 2] = x.z; w[4 * k + 3] = x.w;
                }
                // the reads are back before the next DMA overwrites the tile
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                if (blk + (deep ? 2u : 1u) < d1) issue_dma(blk + (deep ? 2u : 1u));
#pragma unroll
                for (int k = 0; k < 16; k++) w[k] = __builtin_bswap32(w[k]);
                if (soff + 64u > dmin) {  // wave-uniform
                    uint32_t wnb;  // (opaque copy, as below)
                    asm volatile("s_mov_b32 %0, %1" : "=s"(wnb) : "s"(wave_nb));
                    if (uni) {
                        pad_block_uniform(w, soff, dmin, wnb - blk == 1u);
                    } else {  // each lane pads its own message
#pragma unroll
                        for (int k = 0; k < 4; k++)
                            pad_words(soff + 16u * (uint32_t)k, L, blk + 1u == nb, (uint32_t)k, &w[4 * k]);
                    }
                }
                if constexpr (!kFused) block_prio(blk);
                if constexpr (kFused) {
                    // the SIMD's only live wave: latency round form (g_simd_live;
                    // the count only falls, so once alone the wave stops reading it)
                    if (lone_sel != 0u && simd_alone(lone_sel)) lone_sel = kLoneSeen;
                    if (lone_sel == kLoneSeen) {  // wave-uniform
                        if (lone_tr != nullptr) {  // traced runs: the first lone block (bits 53..62, flag 63)
                            if (lane == 0u) *lone_tr |= 1ull << 63 | (unsigned long long)min(blk, 1023u) << 53;
                            lone_tr = nullptr;
                        }
                        if (blk < nb) compress_asm_lat(st, w);
                    } else if (blk < nb) {
                        compress_asm(st, w);
                    }
                } else if (blk < nb) {
                    compress_asm(st, w);
                }
            }
        }
        for (uint32_t blk = dma ? loop_end : b0; blk < loop_end; blk++) {
            const uint32_t soff = 64u * blk;
            uint32_t w[16];
            stage(blk, w, lane, false);
            if (soff + 64u > min_l && uni) {  // wave-uniform
                // (the block count through an opaque s_mov: hipcc otherwise
                // peels the loop's last iteration to fold the test, a third
                // copy of the rounds.  An s_mov, not the s_sub_u32 of before:
                // SALU arithmetic writes SCC behind the compiler's back, and a
                // padding mask's s_cselect read the clobbered SCC -- a wrong
                // 0x80 marker at length 60, tests/test_gpu_parity.py uniform tiles)
                uint32_t wnb;
                asm volatile("s_mov_b32 %0, %1" : "=s"(wnb) : "s"(wave_nb));
                pad_block_uniform(w, soff, min_l, wnb - blk == 1u);
            }
            block_prio(blk);
            if (blk < nb) compress_asm(st, w);
        }
        // Final block of a uniform tile holding at most 16 message bytes
        // (u <= 16; u < 0: the length-only block after a full one): words
        // 4..15 are padding constants, and the tail rounds take them, and the
        // schedule terms they feed, as scalars (requests of a 16-byte header
        // plus a 2^k-byte payload: BASELINE configs 2 and 3).
        if (tail_ok && finished) {
            const uint32_t blk = wave_nb - 1u;
            uint32_t w[16];
            // (the lane index through an opaque copy: the LDS slot addresses
            // are then recomputed here instead of kept live, and spilled,
            // across the loop)
            uint32_t ln;
            asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
            stage(blk, w, ln, true);
            pad_block_uniform<4>(w, 64u * blk, min_l, false);
            block_prio(blk);
            if (blk < nb) compress_asm_tail(st, w, tw);
        }
    } else if constexpr (kLds) {
        // Wide arenas: the same LDS staging with per-chunk 64-bit addresses
        // and activity tests (one launch over > 4 GiB, BASELINE config 5).
        const uint32_t q = lane & 3u;
        uint32_t Lj[4], nbj[4];
        uint64_t oj[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int src = 16 * j + (int)(lane >> 2);
            Lj[j] = (uint32_t)__shfl((int)L, src, 64);
            oj[j] = (uint64_t)(uint32_t)__shfl((int)(uint32_t)o, src, 64);
            oj[j] |= (uint64_t)(uint32_t)__shfl((int)(uint32_t)(o >> 32), src, 64) << 32;
            nbj[j] = (uint32_t)__shfl((int)nb, src, 64);
        }
        for (uint32_t blk = 0; blk < wave_nb; blk++) {
            RawChunk rc[4];
#pragma unroll
            for (int j = 0; j < 4; j++) issue(oj[j], blk, q, blk < nbj[j], rc[j]);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                uint32_t wq[4];
                finish_chunk(rc[j], 64u * blk + 16u * q, Lj[j], blk + 1u == nbj[j], q, wq);
                my[lds_slot(16u * j + (lane >> 2), q)] = make_uint4(wq[0], wq[1], wq[2], wq[3]);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            uint32_t w[16];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint4 x = my[lds_slot(lane, (uint32_t)k)];
                w[4 * k + 0] = x.x; w[4 * k + 1] = x.y; w[4 * k + 2] = x.z; w[4 * k + 3] = x.w;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            progress_prio(blk);
            if (blk < nb) compress_asm(st, w);
        }
    } else {
        for (uint32_t blk = 0; blk < wave_nb; blk++) {
            const bool active = blk < nb;
            RawChunk rc[4];
#pragma unroll
            for (int q = 0; q < 4; q++) issue(o, blk, (uint32_t)q, active, rc[q]);
            uint32_t w[16];
#pragma unroll
            for (int q = 0; q < 4; q++)
                finish_chunk(rc[q], 64u * blk + 16u * q, L, blk + 1u == nb, (uint32_t)q, &w[4 * q]);
            progress_prio(blk);
            if (active) compress_asm(st, w);
        }
    }
digest:
    if (!finished) {  // a split tile's range: hand the midstate back
#pragma unroll
        for (int i = 0; i < 8; i++) st_io[i] = st[i];
        return kTilePaused;
    }
    if (valid) {
        if constexpr (kFused) {
            const __amdgpu_buffer_rsrc_t ors =
                __builtin_amdgcn_make_buffer_rsrc((void*)out, (short)0, (int)(32u * n), 0x00020000);
            store_digest_sc1(ors, msg, st);
        } else if constexpr (kLds && !kWide) {
            // 32-bit buffer offsets (launch_msgs sends n >= 2^27 to the wide
            // form): the message index stays one VGPR across the block loop
            // instead of a 64-bit address pair (the tail form spilled it).
            const __amdgpu_buffer_rsrc_t ors =
                __builtin_amdgcn_make_buffer_rsrc((void*)out, (short)0, (int)(32u * n), 0x00020000);
            store_digest_buf(ors, msg, st);
        } else {
            store_digest(out, msg, st);
        }
    }
    return kTileDone;
}

// One wave per workgroup: a workgroup's slot and LDS are released only when
// ALL its waves have finished, and the SIMD arbiter's age order finishes a
// workgroup's waves (one per SIMD) far apart, so 4-wave workgroups left SIMDs
// below their 8-wave occupancy (tools/stamp_run.py).  8 waves per SIMD bound
// the register budget to 64 VGPRs (the wide form keeps 6: 80 VGPRs, no spill).
constexpr uint32_t kMsgWaves = 1;
constexpr uint32_t kMsgOcc = 8, kTileSlots = 256;
template <bool kLds, bool kWide = false>
__global__ __launch_bounds__(64 * kMsgWaves, kWide ? 6 : kMsgOcc) void sha256_msgs_kernel(
    const uint8_t* __restrict__ arena, uint64_t arena_len, const uint64_t* __restrict__ off,
    const uint32_t* __restrict__ len, const uint32_t* __restrict__ order, uint32_t n,
    uint8_t* __restrict__ out) {
    __shared__ uint4 tile[kMsgWaves][kTileSlots];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t t = blockIdx.x * kMsgWaves + wv;
    if (t * 64u >= n) return;  // whole wave idle (wave-uniform)
    hash_tile<kLds, kWide>(arena, arena_len, off, len, order, n, out, tile[wv], t, lane);
}

// CU-block form of the request kernel, for launches of 1,025 to 4,096 tiles
// (at most 4 per SIMD; BASELINE config 3's 2^18 x 4 KB requests are exactly
// 4,096).  One-wave workgroups leave their placement to the dispatcher, and
// it stacks them unevenly: config 3's request waves lived 441 us on average
// in a 653 us launch (SQ_WAVE_CYCLES / SQ_WAVES, profiles/r03a), i.e. some
// SIMDs ran 5-6 tiles while others idled.  Here each CU gets ONE workgroup of
// 4k waves (kCuLds of LDS holds it alone on its CU), which the CU deals to
// its SIMDs in cyclic order: exactly k waves per SIMD.  Each wave's next
// block lands in its LDS tile by DMA while this block's rounds run (kMode 0).
constexpr uint32_t kCuLds = 96u * 1024u;
// kMode: 0 = the product form: block b+1's loads issued as LDS-DMA
// (buffer_load_dwordx4 ... lds) as soon as block b's words are read back,
// the fused launch's loader (config 3 sequential plan, same box:
// 0.632-0.634 vs 0.648 ms for the register-prefetching form, 1,424 vs
// 1,443 VALU per compression, profiles/r04a, r04b); A/B forms: 1 = the
// register-prefetching block loop (hash_tile_pipelined) with no-yield
// rounds (variant 11), 2 = the same with the product rounds (round 3's
// product form, variant 12), 3 = LDS-DMA with the next block's words read
// back mid-block (variant 13: 0.638 ms, slower).
template <int kMode>
__global__ __launch_bounds__(1024, 1) void sha256_msgs_cu_kernel(const uint8_t* __restrict__ arena,
                                                                 uint64_t arena_len,
                                                                 const uint64_t* __restrict__ off,
                                                                 const uint32_t* __restrict__ len,
                                                                 const uint32_t* __restrict__ order, uint32_t n,
                                                                 uint8_t* __restrict__ out) {
    extern __shared__ uint4 cu_lds[];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t t = blockIdx.x * (blockDim.x >> 6) + wv;
    if (t * 64u >= n) return;  // whole wave idle (wave-uniform)
    hash_tile<true, false, false, true, kMode == 1, kMode == 0 || kMode >= 4, kMode == 3,
              kMode == 4 ? 1 : kMode == 5 ? 2 : 0>(arena, arena_len, off, len, order, n, out, cu_lds + 256u * wv, t,
                                                     lane);
}

// ---- overlapped cycles: this cycle's request tiles + the previous cycle's
// batch chains in ONE launch ------------------------------------------------
// The state machine batches only request digests it already holds (results of
// earlier Ready() cycles: sequence.go:154-157 over client_tracker digests), so
// a stream of cycles pipelines: the launch that hashes cycle i's requests also
// runs cycle i-1's batch chains (compacted lists over its device-resident
// request digests, no readiness waits).  Chain waves come first in the grid
// and run at full occupancy beside the tile waves, at the throughput round
// form, instead of a second latency-bound launch of lone waves (36 us of a
// 221 us config-2 step).  Chain wave block b runs at priority
// 3 - floor(4 b / blocks): a chain is ~2x a request tile's length, so it keeps
// up with the tiles' progress priorities instead of starving behind the second
// generation.
__device__ __forceinline__ uint32_t ld_u32(__amdgpu_buffer_rsrc_t rs, uint32_t off, bool live);
__device__ __forceinline__ void load_digest(__amdgpu_buffer_rsrc_t rsrc, uint32_t id, bool live, uint4& x0,
                                            uint4& x1);
__device__ __forceinline__ void overlap_chain(const uint8_t* __restrict__ digests, uint32_t n_digests,
                                              const uint32_t* __restrict__ cidx, uint32_t n_entries,
                                              const uint32_t* __restrict__ cfirst, uint32_t n_lists,
                                              uint8_t* __restrict__ list_out, uint32_t g, uint32_t lane,
                                              uint32_t prio_mode) {
    __builtin_amdgcn_s_setprio(3);
    const uint32_t k = g * 64u + lane;
    const bool valid = k < n_lists;
    const uint32_t kc = valid ? k : n_lists - 1u;  // unconditional loads (n_lists >= 1)
    const uint32_t e0_ = cfirst[kc], e1_ = cfirst[kc + 1];
    const uint32_t e0 = valid ? e0_ : 0u;
    const uint32_t c = valid ? e1_ - e0_ : 0u;
    const uint32_t L = 32u * c;
    const uint32_t nb = valid ? blocks_for_len(L) : 0u;
    const uint32_t wave_nb = blocks_for_len(32u * wave_max(c));
    const __amdgpu_buffer_rsrc_t drs =
        __builtin_amdgcn_make_buffer_rsrc((void*)digests, (short)0, (int)(32u * n_digests), 0x00020000);
    const __amdgpu_buffer_rsrc_t irs =
        __builtin_amdgcn_make_buffer_rsrc((void*)cidx, (short)0, (int)(4u * n_entries), 0x00020000);
    uint32_t st[8];
#pragma unroll
    for (int i = 0; i < 8; i++) st[i] = kH0[i];
    // Indices one block ahead; the block's digests are loaded right before its
    // rounds (the other waves of the SIMD cover the latency; a digest prefetch
    // would cost 16 VGPRs of the 8-wave budget).
    uint32_t i0 = ld_u32(irs, 4u * e0, 0u < c), i1 = ld_u32(irs, 4u * (e0 + 1u), 1u < c);
    for (uint32_t blk = 0; blk < wave_nb; blk++) {
        const uint32_t d0 = 2u * blk;
        uint4 x[4];
        load_digest(drs, i0, d0 < c, x[0], x[1]);
        load_digest(drs, i1, d0 + 1u < c, x[2], x[3]);
        i0 = ld_u32(irs, 4u * (e0 + d0 + 2u), d0 + 2u < c);
        i1 = ld_u32(irs, 4u * (e0 + d0 + 3u), d0 + 3u < c);
        uint32_t w[16];
#pragma unroll
        for (int half = 0; half < 2; half++) {
            const uint32_t di = d0 + (uint32_t)half;
            const uint4 a = x[2 * half], b = x[2 * half + 1];
            w[8 * half + 0] = __builtin_bswap32(a.x) | (di == c ? 0x80000000u : 0u);
            w[8 * half + 1] = __builtin_bswap32(a.y); w[8 * half + 2] = __builtin_bswap32(a.z);
            w[8 * half + 3] = __builtin_bswap32(a.w); w[8 * half + 4] = __builtin_bswap32(b.x);
            w[8 * half + 5] = __builtin_bswap32(b.y); w[8 * half + 6] = __builtin_bswap32(b.z);
            w[8 * half + 7] = __builtin_bswap32(b.w);
        }
        if (blk + 1u == nb) {
            w[14] = L >> 29;
            w[15] = L << 3;
        }
        fixed_prio(prio_mode == 0u   ? 3u - min(3u, 4u * blk / wave_nb)
                   : prio_mode == 1u ? 3u - min(3u, blk)
                   : prio_mode == 2u ? 3u
                                     : 1u);
        if (blk < nb) compress_asm(st, w);
    }
    if (valid) {
        const __amdgpu_buffer_rsrc_t ors =
            __builtin_amdgcn_make_buffer_rsrc((void*)list_out, (short)0, (int)(32u * n_lists), 0x00020000);
        store_digest_buf(ors, k, st);
    }
}

// Occupancy bound 7 (72 VGPRs allowed): at the bound 8 the chain and tile
// roles spilled two VGPRs and five SGPRs to scratch (12 B per lane); at 7 the
// allocator fits them in 64 VGPRs with no spill, so the launch still runs 8
// waves per SIMD.
constexpr uint32_t kOverlapOcc = 7;
__global__ __launch_bounds__(64, kOverlapOcc) void sha256_msgs_overlap_kernel(OverlapArgs a) {
    __shared__ uint4 tile[kTileSlots];
    const uint32_t lane = threadIdx.x;
    if (blockIdx.x < a.list_waves) {
        overlap_chain(a.prev_digests, a.n_req_prev, a.cidx, a.n_entries, a.cfirst, a.n_lists, a.list_out,
                      blockIdx.x, lane, a.chain_prio);
        return;
    }
    const uint32_t t = blockIdx.x - a.list_waves;
    if (t * 64u >= a.n_req) return;
    hash_tile<true, false>(a.arena, a.arena_len, a.off, a.len, a.order, a.n_req, a.req_out, tile, t, lane);
}

// Low-occupancy form of the request kernel, for launches of at most one wave
// per SIMD (a few long messages: e.g. the distinct EpochChange payloads of a
// deduplicated cycle).  A lone wave's memory latency is not hidden by other
// waves, so each lane prefetches block b+1's chunks (direct per-lane loads)
// before compressing block b, and the rounds are the no-yield form (there is
// no other wave to yield the issue slot to).
__global__ __launch_bounds__(kBlockThreads) void sha256_msgs_lowocc_kernel(
    const uint8_t* __restrict__ arena, uint64_t arena_len, const uint64_t* __restrict__ off,
    const uint32_t* __restrict__ len, const uint32_t* __restrict__ order, uint32_t n, uint8_t* __restrict__ out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t t = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (t * 64u >= n) return;  // whole wave idle (wave-uniform)
    const uint32_t slot = t * 64u + lane;
    const bool valid = slot < n;
    const uint32_t msg = valid ? (order ? order[slot] : slot) : 0u;
    const uint32_t L = valid ? len[msg] : 0u;
    const uint32_t o = valid ? (uint32_t)off[msg] : 0u;
    const uint32_t nb = valid ? blocks_for_len(L) : 0u;
    const uint32_t wave_nb = wave_max(nb);
    const uint32_t records = (uint32_t)((arena_len + 3u) & ~3ull);
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc((void*)arena, (short)0, (int)records, 0x00020000);
    uint32_t st[8];
#pragma unroll
    for (int i = 0; i < 8; i++) st[i] = kH0[i];
    RawChunk cur[4];
#pragma unroll
    for (int q = 0; q < 4; q++) issue_chunk(rsrc, records, o, 0u, (uint32_t)q, 0u < nb, cur[q]);
    for (uint32_t blk = 0; blk < wave_nb; blk++) {
        // Next block's chunks first; past a lane's last block they are
        // inactive (range-checked zero reads, no memory access).
        RawChunk nxt[4];
#pragma unroll
        for (int q = 0; q < 4; q++) issue_chunk(rsrc, records, o, blk + 1u, (uint32_t)q, blk + 1u < nb, nxt[q]);
        uint32_t w[16];
#pragma unroll
        for (int q = 0; q < 4; q++)
            finish_chunk(cur[q], 64u * blk + 16u * q, L, blk + 1u == nb, (uint32_t)q, &w[4 * q]);
        // (the latency-ordered rounds_asm_ilp measured no faster here:
        // 3.03 ms per config-4 launch either way)
        if (blk < nb) compress_asm_lat(st, w);
#pragma unroll
        for (int q = 0; q < 4; q++) cur[q] = nxt[q];
    }
    if (valid) store_digest(out, msg, st);
}

// ---- producer / consumer pairs (wavefront-cooperative multi-block hashing) --
// When there are fewer 64-message groups than SIMDs, every group's wave runs
// alone on its SIMD and its time is one long dependent chain of compressions
// (a VerifyBatch of 500 digests is 251 of them), paced by what ONE wave can
// issue (~4 cycles per instruction).  A pair splits the compression's
// instruction stream over two waves of one 128-thread workgroup, which the
// dispatcher always places on two different SIMDs (tools/simd_probe.hip):
//   wave 0 (producer): loads block b+1, builds its 16 words, computes the
//     message schedule W[16..63] and K[j] + W[j] (~600 instructions) and
//     writes the 64 KW words to an LDS ring slot;
//   wave 1 (consumer): runs the 64 rounds of block b from the other slot
//     (rounds_kw8_asm: 14 instructions per round, ~900 per block).
// One workgroup barrier per block hands the slots over.
constexpr uint32_t kPairThreads = 128;

struct PairRing {
    uint4 kw[2][16][64];  // [slot][quad of 4 KW words][lane]: 16 B per lane, conflict-free b128 access
};

// Message schedule + round constants of one block into a ring slot.
__device__ __forceinline__ void produce_kw(uint32_t w[16], uint4 (*slot)[64], uint32_t lane) {
#pragma unroll
    for (int q = 0; q < 16; q++) {
        uint32_t kw[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const int j = 4 * q + i;
            if (j >= 16) w[j & 15] += ssig1(w[(j - 2) & 15]) + w[(j - 7) & 15] + ssig0(w[(j - 15) & 15]);
            kw[i] = kK[j] + w[j & 15];
        }
        slot[q][lane] = make_uint4(kw[0], kw[1], kw[2], kw[3]);
    }
}

// 64 rounds of one block from a ring slot; st += F only for a live block.
__device__ __forceinline__ void consume_kw(uint4 (*slot)[64], uint32_t lane, uint32_t st[8], bool live) {
    uint32_t s[8];
#pragma unroll
    for (int i = 0; i < 8; i++) s[i] = st[i];
    uint4 a = slot[0][lane], b = slot[1][lane];
#pragma unroll
    for (int c = 0; c < 8; c++) {
        uint4 na = a, nb = b;
        if (c < 7) {
            na = slot[2 * c + 2][lane];
            nb = slot[2 * c + 3][lane];
        }
        rounds_kw8_asm(s, a, b);
        a = na;
        b = nb;
    }
    if (live) {
#pragma unroll
        for (int i = 0; i < 8; i++) st[i] += s[i];
    }
}

__device__ __forceinline__ uint32_t ld_u32(__amdgpu_buffer_rsrc_t rs, uint32_t off, bool live);
__device__ __forceinline__ void load_digest(__amdgpu_buffer_rsrc_t rsrc, uint32_t id, bool live, uint4& x0,
                                            uint4& x1);

// Producer-side sources of block words, called for blocks 0, 1, 2, ... in
// order; each keeps the next block's loads in flight.
struct ArenaBlocks {  // message bytes at any alignment in an arena (< 4 GiB)
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t records, o, L, nb;
    RawChunk cur[4];
    __device__ void start(const uint8_t* arena, uint64_t arena_len, uint32_t off_, uint32_t L_, uint32_t nb_) {
        records = (uint32_t)((arena_len + 3u) & ~3ull);
        rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)arena, (short)0, (int)records, 0x00020000);
        o = off_;
        L = L_;
        nb = nb_;
#pragma unroll
        for (int q = 0; q < 4; q++) issue_chunk(rsrc, records, o, 0u, (uint32_t)q, 0u < nb, cur[q]);
    }
    __device__ void block(uint32_t blk, uint32_t w[16]) {
        RawChunk nxt[4];
#pragma unroll
        for (int q = 0; q < 4; q++) issue_chunk(rsrc, records, o, blk + 1u, (uint32_t)q, blk + 1u < nb, nxt[q]);
#pragma unroll
        for (int q = 0; q < 4; q++) finish_chunk(cur[q], 64u * blk + 16u * q, L, blk + 1u == nb, (uint32_t)q, &w[4 * q]);
#pragma unroll
        for (int q = 0; q < 4; q++) cur[q] = nxt[q];
    }
};

struct ListBlocks {  // concat(digests[cidx[e]]) of a compacted list (no null entries)
    __amdgpu_buffer_rsrc_t drs, irs;
    uint32_t e0, c, L, nb;
    uint4 cur[4];
    uint32_t nx0, nx1;
    __device__ void start(const uint8_t* digests, uint32_t n_digests, const uint32_t* cidx, uint32_t n_entries,
                          uint32_t e0_, uint32_t c_, uint32_t nb_) {
        drs = __builtin_amdgcn_make_buffer_rsrc((void*)digests, (short)0, (int)(32u * n_digests), 0x00020000);
        irs = __builtin_amdgcn_make_buffer_rsrc((void*)cidx, (short)0, (int)(4u * n_entries), 0x00020000);
        e0 = e0_;
        c = c_;
        L = 32u * c;
        nb = nb_;
        nx0 = ld_u32(irs, 4u * (e0 + 2u), 2u < c);
        nx1 = ld_u32(irs, 4u * (e0 + 3u), 3u < c);
        const uint32_t i0 = ld_u32(irs, 4u * e0, 0u < c), i1 = ld_u32(irs, 4u * (e0 + 1u), 1u < c);
        load_digest(drs, i0, 0u < c, cur[0], cur[1]);
        load_digest(drs, i1, 1u < c, cur[2], cur[3]);
    }
    __device__ void block(uint32_t blk, uint32_t w[16]) {
        uint4 nxt[4];
        load_digest(drs, nx0, 2u * blk + 2u < c, nxt[0], nxt[1]);
        load_digest(drs, nx1, 2u * blk + 3u < c, nxt[2], nxt[3]);
        const uint32_t nn0 = ld_u32(irs, 4u * (e0 + 2u * blk + 4u), 2u * blk + 4u < c);
        const uint32_t nn1 = ld_u32(irs, 4u * (e0 + 2u * blk + 5u), 2u * blk + 5u < c);
#pragma unroll
        for (int half = 0; half < 2; half++) {
            const uint32_t di = 2u * blk + (uint32_t)half;  // digest ordinal in the message
            const uint4 x0 = cur[2 * half], x1 = cur[2 * half + 1];
            // past the end the loads returned zeros; only the 0x80 marker is added
            w[8 * half + 0] = __builtin_bswap32(x0.x) | (di == c ? 0x80000000u : 0u);
            w[8 * half + 1] = __builtin_bswap32(x0.y); w[8 * half + 2] = __builtin_bswap32(x0.z);
            w[8 * half + 3] = __builtin_bswap32(x0.w); w[8 * half + 4] = __builtin_bswap32(x1.x);
            w[8 * half + 5] = __builtin_bswap32(x1.y); w[8 * half + 6] = __builtin_bswap32(x1.z);
            w[8 * half + 7] = __builtin_bswap32(x1.w);
        }
        if (blk + 1u == nb) {
            w[14] = L >> 29;
            w[15] = L << 3;
        }
#pragma unroll
        for (int i = 0; i < 4; i++) cur[i] = nxt[i];
        nx0 = nn0;
        nx1 = nn1;
    }
};

// The pair loop shared by both sources: the producer stays one block ahead.
template <class Src>
__device__ __forceinline__ void pair_loop(Src& src, PairRing& ring, bool producer, uint32_t lane, uint32_t nb,
                                          uint32_t st[8]) {
    const uint32_t wave_nb = wave_max(nb);  // same in both waves: they serve the same 64 messages
#pragma unroll
    for (int i = 0; i < 8; i++) st[i] = kH0[i];
    if (producer && wave_nb) {
        uint32_t w[16];
        src.block(0u, w);
        produce_kw(w, ring.kw[0], lane);
    }
    __syncthreads();
    for (uint32_t blk = 0; blk < wave_nb; blk++) {
        if (producer) {
            if (blk + 1u < wave_nb) {
                uint32_t w[16];
                src.block(blk + 1u, w);
                produce_kw(w, ring.kw[(blk + 1u) & 1u], lane);
            }
        } else {
            consume_kw(ring.kw[blk & 1u], lane, st, blk < nb);
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(kPairThreads) void sha256_msgs_pair_kernel(
    const uint8_t* __restrict__ arena, uint64_t arena_len, const uint64_t* __restrict__ off,
    const uint32_t* __restrict__ len, const uint32_t* __restrict__ order, uint32_t n, uint8_t* __restrict__ out) {
    __shared__ PairRing ring;
    const uint32_t lane = threadIdx.x & 63u;
    const bool producer = threadIdx.x < 64u;
    const uint32_t slot = blockIdx.x * 64u + lane;
    const bool valid = slot < n;
    const uint32_t msg = valid ? (order ? order[slot] : slot) : 0u;
    const uint32_t L = valid ? len[msg] : 0u;
    const uint32_t nb = valid ? blocks_for_len(L) : 0u;
    ArenaBlocks src;
    if (producer) src.start(arena, arena_len, valid ? (uint32_t)off[msg] : 0u, L, nb);
    uint32_t st[8];
    pair_loop(src, ring, producer, lane, nb, st);
    if (!producer && valid) store_digest(out, msg, st);
}

__global__ __launch_bounds__(kPairThreads) void sha256_chain_pair_kernel(
    const uint8_t* __restrict__ digests, uint32_t n_digests, const uint32_t* __restrict__ cidx, uint32_t n_entries,
    const uint32_t* __restrict__ cfirst, uint32_t n_lists, uint8_t* __restrict__ out) {
    __shared__ PairRing ring;
    const uint32_t lane = threadIdx.x & 63u;
    const bool producer = threadIdx.x < 64u;
    const uint32_t k = blockIdx.x * 64u + lane;
    const bool valid = k < n_lists;
    const uint32_t e0 = valid ? cfirst[k] : 0u;
    const uint32_t c = valid ? cfirst[k + 1] - e0 : 0u;
    const uint32_t nb = valid ? blocks_for_len(32u * c) : 0u;
    ListBlocks src;
    if (producer) src.start(digests, n_digests, cidx, n_entries, e0, c, nb);
    uint32_t st[8];
    pair_loop(src, ring, producer, lane, nb, st);
    if (!producer && valid) store_digest(out, k, st);
}

// Dependent pass: message k = concat(digests[idx[e]] for e in [first[k], first[k+1]))
// skipping idx == kNullIndex (a null request's empty digest, client_tracker.go:840-847).
// One lane per list.  These waves run few per SIMD, so every global read on
// the chain is an unconditional, range-checked buffer load (no branch + wait
// per element): indices are prefetched two blocks ahead, digests one block
// ahead.  If any list of the wave holds null entries, the whole wave first
// compacts its lists into `scratch` (same positions as idx) and reads there.
// aux bit 31 (volatile) keeps hipcc from merging adjacent dword loads into a
// dwordx2/x4, whose range check would zero in-range entries that share an
// access with out-of-range ones at the end of the array (lowers to sc0 sc1:
// L1 bypass, L2-served).
constexpr int kNoMerge = (int)(1u << 31);
__device__ __forceinline__ uint32_t ld_u32(__amdgpu_buffer_rsrc_t rs, uint32_t off, bool live) {
    return __builtin_amdgcn_raw_buffer_load_b32(rs, live ? off : 0xFFFFFFF0u, 0, kNoMerge);
}

// Digest `id` through a range-checked descriptor: a dead slot (or an index
// past n_digests) reads zeros instead of faulting, without a branch.
__device__ __forceinline__ void load_digest(__amdgpu_buffer_rsrc_t rsrc, uint32_t id, bool live, uint4& x0,
                                            uint4& x1) {
    const uint32_t o = live ? 32u * id : 0xFFFFFFE0u;
    const auto a = __builtin_amdgcn_raw_buffer_load_b128(rsrc, o, 0, 0);
    const auto b = __builtin_amdgcn_raw_buffer_load_b128(rsrc, o + 16u, 0, 0);
    x0 = make_uint4(a[0], a[1], a[2], a[3]);
    x1 = make_uint4(b[0], b[1], b[2], b[3]);
}

// Hash this lane's list whose non-null entries are read through `brs` at
// [e0, e0 + c).  Returns true if a null marker was met (only possible on the
// optimistic pass, where brs is the caller's idx and c = e1 - e0).
__device__ __forceinline__ bool hash_list(__amdgpu_buffer_rsrc_t drs, __amdgpu_buffer_rsrc_t brs, uint32_t e0,
                                          uint32_t c, bool valid, uint32_t st[8]) {
    const uint32_t L = 32u * c;
    const uint32_t nb = valid ? blocks_for_len(L) : 0u;
    const uint32_t wave_nb = wave_max(nb);
#pragma unroll
    for (int i = 0; i < 8; i++) st[i] = kH0[i];
    bool saw_null = false;

    // Pipeline registers: digests of block b (cur), indices of block b+1 (nx).
    uint4 cur[4];
    uint32_t nx0 = ld_u32(brs, 4u * (e0 + 2u), 2u < c), nx1 = ld_u32(brs, 4u * (e0 + 3u), 3u < c);
    {
        const uint32_t i0 = ld_u32(brs, 4u * e0, 0u < c), i1 = ld_u32(brs, 4u * (e0 + 1u), 1u < c);
        saw_null |= (0u < c && i0 == kNullIndex) || (1u < c && i1 == kNullIndex);
        load_digest(drs, i0, 0u < c, cur[0], cur[1]);
        load_digest(drs, i1, 1u < c, cur[2], cur[3]);
    }
    for (uint32_t blk = 0; blk < wave_nb; blk++) {
        // Issue block b+1's digests and block b+2's indices before compressing b.
        const bool l0 = 2u * blk + 2u < c, l1 = 2u * blk + 3u < c;
        saw_null |= (l0 && nx0 == kNullIndex) || (l1 && nx1 == kNullIndex);
        uint4 nxt[4];
        load_digest(drs, nx0, l0, nxt[0], nxt[1]);
        load_digest(drs, nx1, l1, nxt[2], nxt[3]);
        const uint32_t nn0 = ld_u32(brs, 4u * (e0 + 2u * blk + 4u), 2u * blk + 4u < c);
        const uint32_t nn1 = ld_u32(brs, 4u * (e0 + 2u * blk + 5u), 2u * blk + 5u < c);
        if (blk < nb) {
            uint32_t w[16];
#pragma unroll
            for (int half = 0; half < 2; half++) {
                const uint32_t di = 2u * blk + (uint32_t)half;  // digest ordinal in the message
                const uint4 x0 = cur[2 * half], x1 = cur[2 * half + 1];
                // Past the end the loads returned zeros; only the 0x80 marker is added.
                w[8 * half + 0] = __builtin_bswap32(x0.x) | (di == c ? 0x80000000u : 0u);
                w[8 * half + 1] = __builtin_bswap32(x0.y); w[8 * half + 2] = __builtin_bswap32(x0.z);
                w[8 * half + 3] = __builtin_bswap32(x0.w); w[8 * half + 4] = __builtin_bswap32(x1.x);
                w[8 * half + 5] = __builtin_bswap32(x1.y); w[8 * half + 6] = __builtin_bswap32(x1.z);
                w[8 * half + 7] = __builtin_bswap32(x1.w);
            }
            if (blk + 1u == nb) {
                w[14] = L >> 29;
                w[15] = L << 3;
            }
            compress_asm_lat(st, w);
        }
#pragma unroll
        for (int i = 0; i < 4; i++) cur[i] = nxt[i];
        nx0 = nn0;
        nx1 = nn1;
    }
    return saw_null;
}

__global__ __launch_bounds__(kBlockThreads) void sha256_lists_kernel(
    const uint8_t* __restrict__ digests, uint32_t n_digests, const uint32_t* __restrict__ idx,
    uint32_t n_entries, const uint32_t* __restrict__ first, uint32_t n_lists, uint32_t* __restrict__ scratch,
    uint8_t* __restrict__ out) {
    const __amdgpu_buffer_rsrc_t drs =
        __builtin_amdgcn_make_buffer_rsrc((void*)digests, (short)0, (int)(32u * n_digests), 0x00020000);
    const __amdgpu_buffer_rsrc_t irs =
        __builtin_amdgcn_make_buffer_rsrc((void*)idx, (short)0, (int)(4u * n_entries), 0x00020000);
    const uint32_t k = blockIdx.x * kBlockThreads + threadIdx.x;
    const bool valid = k < n_lists;
    const uint32_t e0 = valid ? first[k] : 0u;
    const uint32_t e1 = valid ? first[k + 1] : 0u;

    // Optimistic pass: assume no null request in the list (the common case;
    // no counting prologue on the latency chain).  Nulls are detected as the
    // indices stream in; if any lane of the wave met one, the whole wave
    // compacts its lists into scratch and hashes again (wave-uniform branch).
    uint32_t st[8];
    const bool saw_null = hash_list(drs, irs, e0, e1 - e0, valid, st);
    if (__any(saw_null)) {
        uint32_t m = 0;
        for (uint32_t e = e0; e < e1; e++) {
            const uint32_t v = idx[e];
            if (v != kNullIndex) scratch[e0 + m++] = v;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const __amdgpu_buffer_rsrc_t srs =
            __builtin_amdgcn_make_buffer_rsrc((void*)scratch, (short)0, (int)(4u * n_entries), 0x00020000);
        (void)hash_list(drs, srs, e0, m, valid, st);
    }
    if (valid) store_digest(out, k, st);
}

// Pipelined dependent pass: one SEGMENT of every list's chain.  Lists are
// compacted (no null entries).  Segment [ob, oe) hashes the full 2-digest
// blocks of digest ordinals ob .. min(oe, c) (ob, oe even) starting from the
// midstate in `state` (H0 when ob == 0); a list whose last digest falls in
// the segment (c <= oe) is finalised (partial block + FIPS padding) and its
// digest written to out, otherwise the midstate is written back.  Lists with
// c <= ob (ob > 0) were finalised by an earlier segment and are skipped.
// The waves raise their issue priority: they run beside the next request
// chunk and must keep near-alone speed on their SIMD.
// kUni (uni = B > 0): identity lists of B entries -- list k is digests
// [k B, min(k B + B, n_entries)), the BatchSize batches over consecutive
// requests of a plan (mirsha_plan.hip detects them) -- so bounds and indices
// are computed, not loaded: the chain's first digest loads issue at once
// instead of after two dependent loads (cfirst, then cidx).
// With B even every full list's final block is padding only (32 B digests,
// 64 B blocks): a wave whose lists all hold B entries runs that block as 64
// rounds over the precomputed K[j] + W[j] of `pad` (rounds_kw8_asm, ~900
// instead of ~1,450 instructions on the chain's critical path).
template <bool kUni>
__global__ __launch_bounds__(kBlockThreads) void sha256_chain_kernel(
    const uint8_t* __restrict__ digests, uint32_t n_digests, const uint32_t* __restrict__ cidx,
    uint32_t n_entries, const uint32_t* __restrict__ cfirst, uint32_t n_lists, uint32_t ob, uint32_t oe,
    uint32_t* __restrict__ state, uint8_t* __restrict__ out, uint32_t uni, PadBlockKW pad) {
    __builtin_amdgcn_s_setprio(3);
    const __amdgpu_buffer_rsrc_t drs =
        __builtin_amdgcn_make_buffer_rsrc((void*)digests, (short)0, (int)(32u * n_digests), 0x00020000);
    const __amdgpu_buffer_rsrc_t irs =
        __builtin_amdgcn_make_buffer_rsrc((void*)cidx, (short)0, (int)(4u * n_entries), 0x00020000);
    const uint32_t k = blockIdx.x * kBlockThreads + threadIdx.x;
    const bool valid = k < n_lists;
    uint32_t e0, c;
    if constexpr (kUni) {
        e0 = valid ? k * uni : 0u;
        c = valid ? min(uni, n_entries - e0) : 0u;
    } else {
        e0 = valid ? cfirst[k] : 0u;
        c = valid ? cfirst[k + 1] - e0 : 0u;
    }
    // digest index of ordinal o of this list (0 for a dead slot: never read live)
    auto index = [&](uint32_t o, bool lv) -> uint32_t {
        if constexpr (kUni)
            return e0 + o;
        else
            return ld_u32(irs, 4u * (e0 + o), lv);
    };
    const bool active = valid && (ob == 0u || c > ob);
    const bool fin = active && c <= oe;
    const uint32_t full_end = fin ? (c & ~1u) : oe;  // exclusive ordinal of the full blocks
    const uint32_t nblk = active ? (full_end - ob) / 2u + (fin ? 1u : 0u) : 0u;
    const uint32_t wave_nb = wave_max(nblk);
    const uint32_t L = 32u * c;
    // wave-uniform: every lane finishes a full list of B (even) entries here
    const bool pad_wave = kUni && pad.use && __all(fin && c == uni);

    uint32_t st[8];
    if (ob == 0u || !active) {
#pragma unroll
        for (int i = 0; i < 8; i++) st[i] = kH0[i];
    } else {
        const uint4* sp = reinterpret_cast<const uint4*>(state + 8ull * k);
        const uint4 s0 = sp[0], s1 = sp[1];
        st[0] = s0.x; st[1] = s0.y; st[2] = s0.z; st[3] = s0.w;
        st[4] = s1.x; st[5] = s1.y; st[6] = s1.z; st[7] = s1.w;
    }

    // Same prefetch pipeline as hash_list: digests one block ahead, indices two.
    auto live = [&](uint32_t t, uint32_t slot) { return t < nblk && ob + 2u * t + slot < c; };
    uint4 cur[4];
    uint32_t nx0 = index(ob + 2u, live(1, 0)), nx1 = index(ob + 3u, live(1, 1));
    {
        const uint32_t i0 = index(ob, live(0, 0));
        const uint32_t i1 = index(ob + 1u, live(0, 1));
        load_digest(drs, i0, live(0, 0), cur[0], cur[1]);
        load_digest(drs, i1, live(0, 1), cur[2], cur[3]);
    }
    for (uint32_t t = 0; t < wave_nb; t++) {
        uint4 nxt[4];
        load_digest(drs, nx0, live(t + 1, 0), nxt[0], nxt[1]);
        load_digest(drs, nx1, live(t + 1, 1), nxt[2], nxt[3]);
        const uint32_t nn0 = index(ob + 2u * t + 4u, live(t + 2, 0));
        const uint32_t nn1 = index(ob + 2u * t + 5u, live(t + 2, 1));
        if (pad_wave && t + 1u == wave_nb) {  // the padding-only final block
            uint32_t s[8];
#pragma unroll
            for (int i = 0; i < 8; i++) s[i] = st[i];
#pragma unroll
            for (int g = 0; g < 8; g++)
                rounds_kw8_asm(s, make_uint4(pad.kw[8 * g], pad.kw[8 * g + 1], pad.kw[8 * g + 2], pad.kw[8 * g + 3]),
                               make_uint4(pad.kw[8 * g + 4], pad.kw[8 * g + 5], pad.kw[8 * g + 6], pad.kw[8 * g + 7]));
#pragma unroll
            for (int i = 0; i < 8; i++) st[i] += s[i];
        } else if (t < nblk) {
            uint32_t w[16];
#pragma unroll
            for (int half = 0; half < 2; half++) {
                const uint32_t di = ob + 2u * t + (uint32_t)half;
                const uint4 x0 = cur[2 * half], x1 = cur[2 * half + 1];
                w[8 * half + 0] = __builtin_bswap32(x0.x) | (fin && di == c ? 0x80000000u : 0u);
                w[8 * half + 1] = __builtin_bswap32(x0.y); w[8 * half + 2] = __builtin_bswap32(x0.z);
                w[8 * half + 3] = __builtin_bswap32(x0.w); w[8 * half + 4] = __builtin_bswap32(x1.x);
                w[8 * half + 5] = __builtin_bswap32(x1.y); w[8 * half + 6] = __builtin_bswap32(x1.z);
                w[8 * half + 7] = __builtin_bswap32(x1.w);
            }
            if (fin && t + 1u == nblk) {
                w[14] = L >> 29;
                w[15] = L << 3;
            }
            compress_asm_lat(st, w);
        }
#pragma unroll
        for (int i = 0; i < 4; i++) cur[i] = nxt[i];
        nx0 = nn0;
        nx1 = nn1;
    }
    if (fin) {
        store_digest(out, k, st);
    } else if (active) {
        uint4* sp = reinterpret_cast<uint4*>(state + 8ull * k);
        sp[0] = make_uint4(st[0], st[1], st[2], st[3]);
        sp[1] = make_uint4(st[4], st[5], st[6], st[7]);
    }
}

// ---- fused request -> list pass: ONE launch ---------------------------------
//
// The batch / VerifyBatch / checkpoint lists (sequence.go:154-157,
// batch_tracker.go:147-150) are sequential SHA chains over request digests
// produced in the same launch.  Request TILES (64 messages) are claimed in
// order from a ticket; the processing order is the needed-at ordinal of the
// lists, so every chain's early digests are produced first.  A list GROUP (64
// lists, one lane each) hashes its lists in chunks of kFusedChunkBlocks
// blocks; chunk j of group g may start once every tile that feeds it has
// stored its digests: counter[cbase[g] + j] reaches epoch * expected[...]
// (each feeding tile adds 1 per run, after its sc1 digest stores completed).
// Digests are read back with sc1 loads (MI355X_MICROARCH.md, inter-workgroup
// visibility).  List waves wait only on tile waves, which never wait, so the
// launch cannot deadlock; a 2 s watchdog per wait raises the error flag
// instead of hanging if that invariant is ever broken.
//
// Tile tickets start every run at 0: each wave of the launch retires once
// (fused_retire), and the last one resets them, after every claim of the run
// (each wave's claims complete before its retire count), so no host bookkeeping depends on
// how many waves claimed or where the dispatcher placed them.
__device__ __forceinline__ uint64_t claim(unsigned long long* ctr, uint32_t lane) {
    unsigned long long v = 0;
    if (lane == 0) v = __hip_atomic_fetch_add(ctr, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, 0, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), 0, 64);
    return ((uint64_t)hi << 32) | lo;
}

// Retire count per workgroup, not per wave: a wave counts itself in LDS and
// the workgroup's last wave adds 1 to the device-scope word (adds on one word
// serialise near 88 per us, MI355X_MICROARCH.md: the ~4,000 waves of a
// balanced overlapped launch, ending within tens of us, queued behind each
// other for their adds before they could end).  A workgroup's waves count
// only after their claims returned, and its last wave adds only after every
// wave of the workgroup counted, so the last add of the grid still follows
// every claim of the run.
__device__ __forceinline__ void fused_retire(unsigned long long* ctl, uint32_t lane, uint32_t* waves_retired) {
    if (lane != 0u) return;
    const uint32_t waves = blockDim.x >> 6;
    if (__hip_atomic_fetch_add(waves_retired, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) + 1u != waves)
        return;
    // Relaxed: every claim returned its value (the wave branched on it)
    // before the counts above, and device-scope atomics are performed at one
    // point past the XCDs' L2s (an acq_rel add cost each of config 3's ~4,000
    // waves an L2 writeback: +70 us, profiles/r02ay).
    const unsigned long long old =
        __hip_atomic_fetch_add(ctl + kCtlDone, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old + 1ull == gridDim.x) {
        for (uint32_t q = 0; q < kFusedMaxQueues; q++)
            __hip_atomic_store(ctl + kCtlTileTicket + 16u * q, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(ctl + kCtlDone, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

__device__ __forceinline__ uint64_t poll_counter(const unsigned long long* ctr) {
    return __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // global_load_dwordx2 sc1
}

// The plan's sticky error word (host-mapped memory, so every later host call
// on the plan sees it without a synchronisation): set on any watchdog expiry.
__device__ __forceinline__ void raise_error(unsigned long long* err) {
    __hip_atomic_store(err, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Blocks until *ctr >= target (wave-uniform).  Returns false on watchdog
// expiry (`watchdog` ticks of the 100 MHz clock; FusedArgs::watchdog).
__device__ __noinline__ bool wait_counter(const unsigned long long* ctr, uint64_t target,
                                          unsigned long long* err, uint64_t watchdog) {
    if (target == 0) return true;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (true) {
        const uint64_t v = poll_counter(ctr);
        if (__shfl((int)(v >= target), 0, 64)) return true;
        __builtin_amdgcn_s_sleep(8);  // ~512 cycles between polls
        if (__builtin_amdgcn_s_memrealtime() - t0 > watchdog) {
            if (__lane_id() == 0) raise_error(err);
            return false;
        }
    }
}

// Digest `id` via sc1 loads (L1 bypass: another CU wrote it this launch).
__device__ __forceinline__ void load_digest_sc1(__amdgpu_buffer_rsrc_t rsrc, uint32_t id, bool live, uint4& x0,
                                                uint4& x1) {
    const uint32_t o = live ? 32u * id : 0xFFFFFFE0u;
    const auto a = __builtin_amdgcn_raw_buffer_load_b128(rsrc, o, 0, kSc1);
    const auto b = __builtin_amdgcn_raw_buffer_load_b128(rsrc, o + 16u, 0, kSc1);
    x0 = make_uint4(a[0], a[1], a[2], a[3]);
    x1 = make_uint4(b[0], b[1], b[2], b[3]);
}

// Chain form of a list group for the paced kernel: a lane's list is consumed
// a whole readiness chunk (kFusedChunkBlocks blocks = kChunkDigests digests) at
// a time, double-buffered in registers, so one chunk's digest loads (sc1,
// served from MALL/HBM under full request load: several us) are in flight
// while the previous chunk is compressed.  Indices are static and loaded a
// chunk ahead.  (2-block chunks: the launch's 1024-thread tile blocks hold the
// kernel to 128 VGPRs.)
constexpr uint32_t kChunkDigests = 2u * kFusedChunkBlocks;
__device__ __forceinline__ void load_chunk_idx(__amdgpu_buffer_rsrc_t irs, uint32_t e0, uint32_t c, uint32_t chunk,
                                               uint32_t ix[kChunkDigests]) {
#pragma unroll
    for (uint32_t i = 0; i < kChunkDigests; i++) {
        const uint32_t o = kChunkDigests * chunk + i;
        ix[i] = ld_u32(irs, 4u * (e0 + o), o < c);
    }
}

__device__ __forceinline__ void load_chunk_digests(__amdgpu_buffer_rsrc_t drs, const uint32_t ix[kChunkDigests],
                                                   uint32_t c, uint32_t chunk, bool go, uint4 d[2 * kChunkDigests]) {
#pragma unroll
    for (uint32_t i = 0; i < kChunkDigests; i++)
        load_digest_sc1(drs, ix[i], go && kChunkDigests * chunk + i < c, d[2 * i], d[2 * i + 1]);
}

// Producer/consumer hand-off of a fused list pair (one per list block, two
// waves on two SIMDs): the producer builds each block's words from the list's
// digests (readiness waits, sc1 loads), computes the schedule and K + W into
// ring slot seq & 1 and publishes seq + 1; the consumer runs the rounds from
// that slot and frees it.  LDS flags with workgroup-scope acquire / release
// (no s_barrier: the list block's other waves have exited); the waits carry
// the same 2 s watchdog as the readiness waits.
// Fail closed: a producer whose readiness wait expired sets `aborted` and
// publishes produced = kRingAbort, so its consumer stops at once and stores
// no digest of this or any later group (the caller sees the plan's error
// word: mirsha_pipeline_status and every later call on the plan fail).
struct FusedPairRing {
    uint4 kw[2][16][64];
    uint32_t produced, consumed;  // blocks handed over / freed, over all groups of the block
    uint32_t aborted;
};
constexpr uint32_t kRingAbort = 0xFFFFFFFFu;

__device__ __forceinline__ bool lds_wait_ge(const uint32_t* p, uint32_t target, unsigned long long* err) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) {  // 2 s at 100 MHz
            if (__lane_id() == 0) raise_error(err);
            return false;
        }
    }
    return true;
}

__device__ __forceinline__ void lds_publish(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Shape of list group g for this lane's list.
struct FusedListShape {
    uint32_t k, e0, c, L, nb, wave_nb;
    bool valid;
    __device__ FusedListShape(const FusedArgs& a, uint32_t g, uint32_t lane) {
        k = g * 64u + lane;
        valid = k < a.n_lists;
        e0 = valid ? a.cfirst[k] : 0u;
        c = valid ? a.cfirst[k + 1] - e0 : 0u;
        L = 32u * c;
        nb = valid ? blocks_for_len(L) : 0u;
        wave_nb = wave_max(nb);
    }
};

// Consumer side of group g: the rounds of every block from the ring.
// Returns false (no digest stored) once the producer has aborted.
__device__ __forceinline__ bool fused_list_consume(const FusedArgs& a, FusedPairRing& ring, uint32_t g,
                                                   uint32_t lane, uint32_t& seq) {
    const FusedListShape sh(a, g, lane);
    uint32_t st[8];
#pragma unroll
    for (int i = 0; i < 8; i++) st[i] = kH0[i];
    for (uint32_t blk = 0; blk < sh.wave_nb; blk++, seq++) {
        if (!lds_wait_ge(&ring.produced, seq + 1u, a.err)) return false;
        if (__hip_atomic_load(&ring.aborted, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return false;
        consume_kw(ring.kw[seq & 1u], lane, st, blk < sh.nb);
        lds_publish(&ring.consumed, seq + 1u);
    }
    if (a.trace && lane == 0) a.trace[3u * a.n_tiles + a.n_counters + g] = __builtin_amdgcn_s_memrealtime();
    if (sh.valid) store_digest(a.list_out, sh.k, st);
    return true;
}

__device__ __forceinline__ bool fused_abort(FusedPairRing& ring) {
    __hip_atomic_store(&ring.aborted, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    lds_publish(&ring.produced, kRingAbort);
    return false;
}

// Producer side of group g: readiness waits and digest loads a chunk ahead,
// then each block's schedule + K + W into the ring.  Returns false (after
// fused_abort) when a wait expired: nothing past that point is handed over.
__device__ __forceinline__ bool fused_list_produce(const FusedArgs& a, __amdgpu_buffer_rsrc_t drs,
                                                   __amdgpu_buffer_rsrc_t irs, FusedPairRing& ring, uint32_t g,
                                                   uint32_t lane, uint32_t& seq) {
    const FusedListShape sh(a, g, lane);
    const uint32_t e0 = sh.e0, c = sh.c, L = sh.L, wave_nb = sh.wave_nb;
    const uint32_t nchunks = (wave_nb + kFusedChunkBlocks - 1u) / kFusedChunkBlocks;
    const uint32_t cb = a.cbase[g];
    auto target = [&](uint32_t chunk) -> uint64_t { return (uint64_t)a.epoch * a.expected[cb + chunk]; };
    auto stamp = [&](uint32_t at) {
        if (a.trace && lane == 0) a.trace[at] = __builtin_amdgcn_s_memrealtime();
    };
    if (nchunks == 0) return true;
    uint32_t ixc[kChunkDigests], ixn[kChunkDigests];
    load_chunk_idx(irs, e0, c, 0u, ixc);
    load_chunk_idx(irs, e0, c, 1u, ixn);
    if (!wait_counter(a.counters + cb, target(0), a.err, a.watchdog)) return fused_abort(ring);
    uint4 dc[2 * kChunkDigests];
    load_chunk_digests(drs, ixc, c, 0u, true, dc);
    uint64_t pollv = 1u < nchunks ? poll_counter(a.counters + cb + 1u) : 0u;
    for (uint32_t chunk = 0; chunk < nchunks; chunk++) {
        stamp(3u * a.n_tiles + cb + chunk);
        // Next chunk's digests now if its tiles are done (poll issued one chunk ago).
        const uint32_t nc = chunk + 1u;
        bool have_next = false;
        uint4 dn[2 * kChunkDigests];
        if (nc < nchunks) {
            have_next = (bool)__shfl((int)(pollv >= target(nc)), 0, 64);
            load_chunk_digests(drs, ixn, c, nc, have_next, dn);
        }
        uint32_t ixnn[kChunkDigests];
        load_chunk_idx(irs, e0, c, chunk + 2u, ixnn);
        if (!have_next && nc + 1u < nchunks) pollv = 0;
        if (have_next && nc + 1u < nchunks) pollv = poll_counter(a.counters + cb + nc + 1u);
        else if (nc < nchunks) pollv = poll_counter(a.counters + cb + nc);
#pragma unroll
        for (uint32_t j = 0; j < kFusedChunkBlocks; j++) {
            const uint32_t blk = kFusedChunkBlocks * chunk + j;
            if (blk < wave_nb) {  // wave-uniform: dead lanes hand over words the consumer ignores
                uint32_t w[16];
#pragma unroll
                for (int half = 0; half < 2; half++) {
                    const uint32_t di = 2u * blk + (uint32_t)half;
                    const uint4 x0 = dc[4 * j + 2 * half], x1 = dc[4 * j + 2 * half + 1];
                    w[8 * half + 0] = __builtin_bswap32(x0.x) | (di == c ? 0x80000000u : 0u);
                    w[8 * half + 1] = __builtin_bswap32(x0.y); w[8 * half + 2] = __builtin_bswap32(x0.z);
                    w[8 * half + 3] = __builtin_bswap32(x0.w); w[8 * half + 4] = __builtin_bswap32(x1.x);
                    w[8 * half + 5] = __builtin_bswap32(x1.y); w[8 * half + 6] = __builtin_bswap32(x1.z);
                    w[8 * half + 7] = __builtin_bswap32(x1.w);
                }
                if (blk + 1u == sh.nb) {
                    w[14] = L >> 29;
                    w[15] = L << 3;
                }
                // slot seq & 1 was last filled with block seq - 2: free once seq - 1 blocks are consumed
                if (seq >= 2u && !lds_wait_ge(&ring.consumed, seq - 1u, a.err)) return fused_abort(ring);
                produce_kw(w, ring.kw[seq & 1u], lane);
                lds_publish(&ring.produced, seq + 1u);
                seq++;
            }
        }
        stamp(3u * a.n_tiles + a.n_counters + a.n_groups + cb + chunk);
        if (nc < nchunks) {
            if (!have_next) {  // exposed: wait for the next chunk's tiles, then load it
                if (!wait_counter(a.counters + cb + nc, target(nc), a.err, a.watchdog)) return fused_abort(ring);
                load_chunk_digests(drs, ixn, c, nc, true, dn);
                if (nc + 1u < nchunks) pollv = poll_counter(a.counters + cb + nc + 1u);
            }
#pragma unroll
            for (uint32_t i = 0; i < 2 * kChunkDigests; i++) dc[i] = dn[i];
#pragma unroll
            for (uint32_t i = 0; i < kChunkDigests; i++) ixn[i] = ixnn[i];
        }
    }
    return true;
}

// Midstate of split tile s between two segments, [s][word][lane], written
// through (sc1) and read with sc1 loads by the next segment's host on any
// XCD after its flag wait (MI355X_MICROARCH.md, inter-workgroup visibility).
__device__ __forceinline__ void store_midstate_sc1(uint32_t* seg_state, uint32_t s, uint32_t lane,
                                                   const uint32_t st[8]) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(seg_state + 512ull * s), (short)0,
                                                                        2048, 0x00020000);
#pragma unroll
    for (int i = 0; i < 8; i++) __builtin_amdgcn_raw_buffer_store_b32(st[i], rs, 4u * (64u * i + lane), 0, kSc1);
}

__device__ __forceinline__ void load_midstate_sc1(const uint32_t* seg_state, uint32_t s, uint32_t lane,
                                                  uint32_t st[8]) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)(seg_state + 512ull * s), (short)0,
                                                                        2048, 0x00020000);
#pragma unroll
    for (int i = 0; i < 8; i++) st[i] = __builtin_amdgcn_raw_buffer_load_b32(rs, 4u * (64u * i + lane), 0, kSc1);
}

// Block = 4 x pace waves (pace per SIMD; wave w on SIMD w % 4), one block per
// CU (kPacedLds of LDS).  List blocks [0, list_blocks) run a chain pair on
// SIMDs 0 and 1; their other waves exit at once or, with list_tiles, serve
// the tile queues like a tile block's (FusedArgs::list_tiles).  Tile
// blocks fill the other CUs with `pace` tile waves per SIMD, one per tile
// QUEUE: the wave of slot q = w / 4 serves queue q (tiles in needed-at order,
// queue 0 the earliest) at issue priority prio_of(q), so on every SIMD the
// wave holding the earliest-needed tile wins issue and finishes first while
// the later queues soak up the remaining issue slots (the SIMD stays full, the
// chains get their digests in needed-at order); a wave whose queue is empty
// takes tiles from the last queue.  The tile waves run the request kernel's
// LDS-staged, yield-form hash_tile.
constexpr uint32_t kPacedMaxThreads = 256u * kPacedMaxPace;
__device__ __forceinline__ uint32_t prio_of(uint32_t q, uint32_t nq) {
    return q == 0u ? 3u : nq - 1u - q;  // 4 queues: 3 2 1 0; 2 queues: 3 0
}

__global__ __launch_bounds__(kPacedMaxThreads) void sha256_fused_paced_kernel(FusedArgs a) {
    extern __shared__ uint4 paced_lds[];
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t wv = threadIdx.x >> 6;
    const __amdgpu_buffer_rsrc_t drs =
        __builtin_amdgcn_make_buffer_rsrc((void*)a.list_digests, (short)0, (int)(32u * a.n_req), 0x00020000);
    // Identity = (simd, slot): the wave's SIMD (HW_ID) and its rank among the
    // block's waves on that SIMD.  A workgroup's waves are dealt to the CU's
    // SIMDs in cyclic order (MI355X_MICROARCH.md, LDS section), so a block of
    // 4P waves puts exactly P on every SIMD: one tile wave per queue per SIMD
    // (the static first tiles below), slot-0 waves on SIMDs 0 and 1 for a list
    // block's pair, the last slot hosting split-tile segments.  Every role
    // derives from the identity, so any other placement is remapped, not
    // failed: after the count, the waves at slot >= P (extras) take the
    // identities no wave holds (SIMDs with fewer than P waves), in order, and
    // every (simd, slot) of the block is held by exactly one wave -- some then
    // share a physical SIMD, which is slower but complete.  (Round 3 failed
    // such a run closed; plans probe the placement at creation and fall back
    // to the sequential plan when it is not cyclic, mirsha_plan.hip.)
    // FusedArgs::test_placement (MIRSHA_AB=1 MIRSHA_TEST_PLACEMENT=remap)
    // makes every wave read SIMD 0, so the remap runs on real hardware.
    __shared__ uint32_t simd_waves[4];
    __shared__ uint32_t extra_ticket, waves_counted;
    __shared__ uint32_t waves_retired;
    static_assert(kPacedRingOff + sizeof(FusedPairRing) <= kPacedLds && kPacedRingOff >= 4096u * kPacedMaxPace * 4u,
                  "paced LDS: staging tiles, then the pair ring");
    FusedPairRing& ring = *reinterpret_cast<FusedPairRing*>(reinterpret_cast<uint8_t*>(paced_lds) + kPacedRingOff);
    const bool list_block = blockIdx.x < a.list_waves;  // list_waves carries the number of LIST BLOCKS
    if (threadIdx.x < 4u) simd_waves[threadIdx.x] = 0u;
    if (threadIdx.x == 0u) waves_retired = extra_ticket = waves_counted = 0u;
    if (threadIdx.x < 64u) g_bal_prog[threadIdx.x] = kBalDone;  // tile progress (kPrioBalance)
    if (threadIdx.x < 4u) g_simd_live[threadIdx.x] = blockDim.x >> 8;  // P live waves per SIMD
    if (list_block && threadIdx.x == 0u) ring.produced = ring.consumed = ring.aborted = 0u;
    __syncthreads();
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    const uint32_t P = blockDim.x >> 8;
    uint32_t simd = a.test_placement ? 0u : (hw >> 4) & 3u;
    uint32_t slot = 0u;
    if (lane == 0u) {
        slot = atomicAdd(&simd_waves[simd], 1u);
        __hip_atomic_fetch_add(&waves_counted, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    // Everything below is scalar (readfirstlane on every LDS-read value): a
    // remap written with per-lane values made the compiler treat the whole
    // identity as divergent, and with this block present -- never executed
    // -- the fused config-3 step went 0.80 -> 1.07 ms (profiles/r04d-r04f
    // bisected it to this block).
    slot = (uint32_t)__builtin_amdgcn_readfirstlane(__shfl((int)slot, 0, 64));
    if (slot >= P) {  // scalar branch: an extra wave takes the next identity no wave holds
        // Only extras wait for the whole block's count (no barrier): every
        // wave of the block is resident, so the count completes.
        while ((uint32_t)__builtin_amdgcn_readfirstlane((int)__hip_atomic_load(
                   &waves_counted, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) < 4u * P)
            __builtin_amdgcn_s_sleep(1);
        uint32_t e = 0u;
        if (lane == 0u) e = atomicAdd(&extra_ticket, 1u);
        e = (uint32_t)__builtin_amdgcn_readfirstlane(__shfl((int)e, 0, 64));
        uint32_t ns = simd, nsl = slot;
        for (uint32_t s4 = 0; s4 < 4u; s4++) {
            const uint32_t have = min((uint32_t)__builtin_amdgcn_readfirstlane((int)simd_waves[s4]), P);
            const uint32_t miss = P - have;
            if (e < miss) {
                ns = s4;
                nsl = have + e;
                break;
            }
            e -= miss;
        }
        simd = ns;
        slot = nsl;
    }
    bool own = true, tiles = true;
    if (list_block && (slot != 0u || simd > 1u)) {  // not the pair: a tile wave, or idle
        tiles = !(a.list_tiles == 0u || (a.list_tiles == 1u && simd <= 1u));
    } else if (list_block) {  // groups blockIdx.x, + list blocks, ...: producer on SIMD 0, consumer on SIMD 1
        __builtin_amdgcn_s_setprio(3);
        uint32_t seq = 0u;
        if (simd == 0u) {
            const __amdgpu_buffer_rsrc_t irs =
                __builtin_amdgcn_make_buffer_rsrc((void*)a.cidx, (short)0, (int)(4u * a.n_entries), 0x00020000);
            for (uint32_t g = blockIdx.x; g < a.n_groups; g += a.list_waves)
                if (!fused_list_produce(a, drs, irs, ring, g, lane, seq)) break;
        } else {
            for (uint32_t g = blockIdx.x; g < a.n_groups; g += a.list_waves)
                if (!fused_list_consume(a, ring, g, lane, seq)) break;
        }
        tiles = a.list_tiles != 0u;
        own = false;  // chains done: tiles left in the last queue (the overflow)
    }
    uint4* my = paced_lds + 256u * wv;  // the wave's 4 KiB staging tile
    const uint32_t last = a.n_queues - 1u;
    const uint32_t q = min(slot, last);
    // Split tiles (FusedArgs::n_split): this wave hosts segment `seg` if it is
    // the last queue's wave on a tile-block SIMD with a segment assigned; it
    // runs the segment when its own first tile reaches block seg_at.
    constexpr uint32_t kNoSeg = 0xFFFFFFFFu;
    uint32_t seg = kNoSeg, seg_at = 0u;
    if (a.n_split && !list_block && slot == last) {
        const uint32_t h = (blockIdx.x - a.list_waves) * 4u + simd;
        if (h < a.n_split * a.seg_per_tile) {
            seg = h;
            seg_at = (h % a.seg_per_tile) * a.seg_nominal_nb / a.seg_per_tile;
        }
    }
    // The first tile of a wave in its own queue is static: queue q holds one
    // tile per wave of slot q (a_qw[q]), the wave's index among them below.
    // Claims on one ticket word saturate near 88 per us (MI355X_MICROARCH.md,
    // dequeue), so ~1,000 waves per queue claiming at launch waited up to
    // ~11 us; only the rest (steals, surplus tiles) go through the tickets.
    uint32_t static_idx = 0xFFFFFFFFu;
    if (!list_block) {
        static_idx = (blockIdx.x - a.list_waves) * 4u + simd;
    } else if (tiles && own) {
        const uint32_t lbs = a.list_tiles == 1u ? 2u : (q == 0u ? 2u : 4u);  // list-block tile waves of slot q
        static_idx = a.tile_blocks * 4u + blockIdx.x * lbs + (lbs == 2u ? simd - 2u : simd);
    }
    uint64_t t = 0;
    bool have = false;    // a claimed own tile in progress
    uint32_t ob0 = 0u;    // its next block
    uint32_t qq = q;
    uint32_t st[8];
    // A host's own tile's midstate while it runs its segment: in the tile
    // block's unused pair-ring LDS (2 KiB per SIMD's host wave), not registers.
    uint32_t* own_st = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(paced_lds) + kPacedRingOff) + 512u * simd;
    // The last queue's waves of a tile block stage two blocks ahead (hash_tile
    // my2): a second 4 KiB tile per SIMD after the parked midstates.
    uint4* deep_tile = (a.deep_last && !list_block && slot == last)
                           ? reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(paced_lds) + kPacedDeepOff) + 256u * simd
                           : nullptr;
    while (true) {
        if (!have && tiles) {
            qq = own ? q : last;
            uint64_t c;
            if (own && static_idx < a.q_waves[qq]) {
                c = a.q_first[qq] + static_idx;
                static_idx = 0xFFFFFFFFu;
            } else {
                static_idx = 0xFFFFFFFFu;
                c = claim(a.ctl + kCtlTileTicket + 16u * qq, lane) + a.q_first[qq] + a.q_waves[qq];
            }
            if (c >= a.q_end[qq]) {
                if (own && qq != last) {
                    own = false;
                    continue;
                }
                tiles = false;
            } else {
                t = c;
                have = true;
                ob0 = 0u;
                if (a.trace && lane == 0) {
                    uint32_t xcc;
                    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
                    a.trace[3 * t] = __builtin_amdgcn_s_memrealtime();
                    a.trace[3 * t + 2] = (unsigned long long)hw | ((unsigned long long)(xcc & 0xFFu) << 32) |
                                         ((unsigned long long)qq << 40) | ((unsigned long long)slot << 44) |
                                         ((unsigned long long)simd << 48) |
                                         ((unsigned long long)(list_block ? 1u : 0u) << 52);
                }
            }
        }
        // The next range of work: this wave's segment (at its turn), else its own tile.
        const bool is_seg = seg != kNoSeg && (!have || ob0 >= seg_at);
        if (!is_seg && !have) break;
        uint32_t wt, b0, b1, pr, s_i = 0u, k_i = 0u;
        if (is_seg) {
            s_i = seg / a.seg_per_tile;
            k_i = seg % a.seg_per_tile;
            const uint32_t S = a.seg_per_tile, nbs = a.seg_nb[s_i];
            wt = a.split_first + s_i;
            b0 = k_i * nbs / S;
            b1 = k_i + 1u == S ? 0xFFFFFFFFu : (k_i + 1u) * nbs / S;
            pr = 3u;  // a segment chain is sequential: run it at the top issue priority
#pragma unroll
            for (int i = 0; i < 8; i++) own_st[64 * i + lane] = st[i];
            // Segment k_i - 1 of this split tile done (this run)?  Fail closed on expiry.
            // (inline, not wait_counter: a call here spilled the live tile state)
            bool ok = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0ull;
            const uint64_t target = a.seg_epoch * S + k_i, t0 = __builtin_amdgcn_s_memrealtime();
            uint32_t fin = 0u;  // the tile already finished (an earlier segment published the run's end)
            while (ok) {
                const uint64_t f = poll_counter(a.seg_flags + 16u * s_i);
                if (__shfl((int)(f >= target), 0, 64)) {
                    fin = (uint32_t)__shfl((int)(f >= a.seg_epoch * S + S), 0, 64);
                    break;
                }
                __builtin_amdgcn_s_sleep(8);
                if (__builtin_amdgcn_s_memrealtime() - t0 > a.watchdog) {
                    if (lane == 0u) raise_error(a.err);
                    ok = false;
                }
            }
            // fail closed: this split tile's later segments and digest are never written;
            // fin: the run's messages are shorter than the plan's and an earlier
            // segment stored the digest: nothing to do, nothing to publish
            if (!ok || fin) {
                seg = kNoSeg;
#pragma unroll
                for (int i = 0; i < 8; i++) st[i] = own_st[64 * i + lane];
                continue;
            }
            if (b0) load_midstate_sc1(a.seg_state, s_i, lane, st);
        } else {
            wt = (uint32_t)t;
            b0 = ob0;
            b1 = seg != kNoSeg ? seg_at : 0xFFFFFFFFu;
            // (overlapped cycles: no chain waits on these tiles, so no queue
            // order to keep -- priorities by progress rank, kPrioBalance)
            pr = a.tile_prio_progress == 2u ? kPrioBalance
                 : a.tile_prio_progress     ? kPrioProgress
                                            : prio_of(a.steal_own_prio ? q : qq, a.n_queues);
        }
        const bool done = hash_tile<true, false, true>(a.arena, a.arena_len, a.off, a.len, a.order, a.n_req,
                                                       a.req_out, my, wt, lane, pr, b0, b1, st,
                                                       (a.lone_form && slot == last) ? simd + 1u : 0u, deep_tile,
                                                       (a.trace && !is_seg) ? a.trace + 3 * t + 2 : nullptr) ==
                          kTileDone;
        if (!done && !is_seg) {  // own tile paused at seg_at
            ob0 = seg_at;
            continue;
        }
        if (!done) store_midstate_sc1(a.seg_state, s_i, lane, st);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (done) {
            if (!is_seg && a.trace && lane == 0) a.trace[3 * t + 1] = __builtin_amdgcn_s_memrealtime();
            const uint32_t j0 = a.tadj_first[wt], j1 = a.tadj_first[wt + 1];
            for (uint32_t j = j0 + lane; j < j1; j += 64u)
                __hip_atomic_fetch_add(a.counters + a.tadj[j], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (is_seg) {
            // segment done; a segment that finished the tile (the last, or an
            // earlier one when the run's messages are shorter than the plan's
            // cut) publishes the run's end, which the later segments skip on
            if (lane == 0u)
                __hip_atomic_store(a.seg_flags + 16u * s_i,
                                   a.seg_epoch * a.seg_per_tile + (done ? a.seg_per_tile : k_i + 1u),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            seg = kNoSeg;
#pragma unroll
            for (int i = 0; i < 8; i++) st[i] = own_st[64 * i + lane];
        } else {
            have = false;
            if (lane == 0u) balance_done();  // no longer behind anyone (kPrioBalance)
        }
    }
    // this wave is no longer live on its SIMD (g_simd_live: a tile wave left alone switches round forms)
    if (lane == 0u) __hip_atomic_fetch_sub(&g_simd_live[simd], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    fused_retire(a.ctl, lane, &waves_retired);
}

// Placement probe (fused plan creation): blocks of the fused launch's shape
// (4P waves, kPacedLds of LDS: one block per CU) count their waves per SIMD;
// a block whose count is not P on every SIMD sets *broken.  With test != 0
// every wave reads SIMD 0 (tests: the plan's sequential fallback).
__global__ __launch_bounds__(kPacedMaxThreads) void placement_probe_kernel(uint32_t* broken, uint32_t test) {
    __shared__ uint32_t cnt[4];
    if (threadIdx.x < 4u) cnt[threadIdx.x] = 0u;
    __syncthreads();
    uint32_t hw;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    const uint32_t simd = test ? 0u : (hw >> 4) & 3u;
    if ((threadIdx.x & 63u) == 0u) atomicAdd(&cnt[simd], 1u);
    __syncthreads();
    if (threadIdx.x == 0u) {
        const uint32_t P = blockDim.x >> 8;
        if (cnt[0] != P || cnt[1] != P || cnt[2] != P || cnt[3] != P) atomicOr(broken, 1u);
    }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// Same stream as oracle_gen_requests (oracle/sha256_oracle.c): one thread per
// 8-byte word of the packed (16 + data_len)-byte messages.
__global__ void gen_requests_kernel(uint64_t seed, uint64_t first, uint64_t count, uint32_t data_len,
                                    uint8_t* __restrict__ arena) {
    const uint64_t stride = 16ull + data_len;
    const uint64_t words_per_msg = (data_len + 7u) / 8u + 2u;
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= count * words_per_msg) return;
    const uint64_t r = gid / words_per_msg, wi = gid % words_per_msg;
    const uint64_t i = first + r;
    uint8_t* m = arena + r * stride;
    uint64_t v;
    uint32_t nbytes = 8, base;
    if (wi == 0) { v = i % 16u; base = 0; }
    else if (wi == 1) { v = i / 16u; base = 8; }
    else {
        const uint32_t j = (uint32_t)(wi - 2);
        v = splitmix64(splitmix64(seed ^ i) + j);
        base = 16u + 8u * j;
        if (8u * j + 8u > data_len) nbytes = data_len - 8u * j;
    }
    for (uint32_t b = 0; b < nbytes; b++) m[base + b] = (uint8_t)(v >> (8 * b));
}

// BASELINE config 5 (mixed 64 B - 64 KB requests): data length
// of request i, integer-only so host (oracle_mixed_data_len), numpy and
// device agree bit for bit: log-uniform over the octaves of [64, 65536),
// uniform inside an octave.
constexpr uint64_t kLenTag = 0x4C454E4754480000ull;
__device__ __forceinline__ uint32_t mixed_data_len(uint64_t seed, uint64_t i) {
    const uint64_t x = splitmix64(seed ^ i ^ kLenTag) >> 40;
    const uint64_t t = 10u * x;
    const uint64_t e = t >> 24, m = t & 0xFFFFFFu;
    return (uint32_t)((64ull << e) + (((64ull << e) * m) >> 24));
}

__global__ void mixed_lengths_kernel(uint64_t seed, uint64_t first, uint64_t count, uint32_t* __restrict__ len) {
    const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r < count) len[r] = 16u + mixed_data_len(seed, first + r);
}

// One wave per message (grid-stride), lanes over its 8-byte words; byte
// stores because messages are packed at any byte alignment.
__global__ void gen_mixed_kernel(uint64_t seed, uint64_t first, uint64_t count, const uint64_t* __restrict__ off,
                                 uint8_t* __restrict__ arena) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t r = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < count; r += waves) {
        const uint64_t i = first + r;
        const uint32_t L = 16u + mixed_data_len(seed, i);
        const uint64_t key = splitmix64(seed ^ i);
        uint8_t* m = arena + off[r];
        for (uint32_t w = lane; 8u * w < L; w += 64u) {
            const uint64_t v = w == 0 ? i % 16u : (w == 1 ? i / 16u : splitmix64(key + (w - 2u)));
            const uint32_t nbytes = L - 8u * w < 8u ? L - 8u * w : 8u;
            for (uint32_t b = 0; b < nbytes; b++) m[8u * w + b] = (uint8_t)(v >> (8 * b));
        }
    }
}

// ---- launching ------------------------------------------------------------
LaunchEvents& next_launch_events() {
    thread_local LaunchEvents ev;
    return ev;
}

// Every kernel of the library is launched here: with the thread's pending
// timing events bound to the dispatch (hipExtLaunchKernel) when a timed
// launch set them, else a plain launch.  Errors are left for the caller's
// hipGetLastError, as with <<<...>>>.
template <typename... P, typename... A>
void launch_k(void (*k)(P...), dim3 grid, dim3 block, uint32_t shmem, hipStream_t s, A... args) {
    LaunchEvents& ev = next_launch_events();
    if (ev.start && ev.stop) {
        const hipEvent_t e0 = ev.start, e1 = ev.stop;
        ev = LaunchEvents{};
        hipExtLaunchKernelGGL(k, grid, block, shmem, s, e0, e1, 0u, static_cast<P>(args)...);
    } else {
        k<<<grid, block, shmem, s>>>(static_cast<P>(args)...);
    }
}

// ---- clock probe (bench diagnostics; no digest depends on it) ---------------
// Every SIMD runs kProbeWavesPerSimd waves of back-to-back throughput-form
// compressions on registers (the request kernel's rounds, no memory traffic);
// lane 0 of each wave records the shader-clock cycles (s_memtime) of its loop
// and the 100 MHz reference time (s_memrealtime) at its start and end.  Cycles
// over ticks is the clock the chip holds under this VALU load
// (MI355X_MICROARCH.md, DVFS item 6); the launch span (first start to last
// end) x clock / (iters x waves per SIMD) is the SIMD cost of one
// wave-compression: the achievable ceiling of the request kernel.
__global__ __launch_bounds__(256) void clock_probe_kernel(uint32_t iters, unsigned long long* __restrict__ stamps,
                                                          uint32_t* __restrict__ sink) {
    uint32_t st[8], w[16];
#pragma unroll
    for (int i = 0; i < 8; i++) st[i] = kH0[i] ^ threadIdx.x;
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = kK[i] + blockIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t b = 0; b < iters; b++) compress_asm(st, w);  // w keeps W[48..63]: fresh input
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    const uint32_t gw = blockIdx.x * 4u + (threadIdx.x >> 6);
    if ((threadIdx.x & 63u) == 0u) {
        stamps[3ull * gw] = t1 - t0;
        stamps[3ull * gw + 1ull] = r0;
        stamps[3ull * gw + 2ull] = r1;
    }
    sink[blockIdx.x * 256u + threadIdx.x] = st[0] ^ st[7];
}

hipError_t launch_clock_probe(uint32_t blocks, uint32_t iters, unsigned long long* stamps, uint32_t* sink,
                              hipStream_t s) {
    launch_k(clock_probe_kernel, blocks, 256, 0, s, iters, stamps, sink);
    return hipGetLastError();
}

// ---- host-side launchers --------------------------------------------------

const char* ab_getenv(const char* name) {
    const char* ab = getenv("MIRSHA_AB");
    return (ab && ab[0] == '1') ? getenv(name) : nullptr;
}

uint32_t pair_max_groups() {
    static const uint32_t v = [] {
        // Round 4 moved MIRSHA_PAIR behind MIRSHA_AB=1: say so once
        // to a caller still setting it alone, rather than ignoring it silently.
        if ((getenv("MIRSHA_PAIR") || getenv("MIRSHA_PAIR_MAX_GROUPS")) && !ab_getenv("MIRSHA_PAIR_MAX_GROUPS") &&
            !ab_getenv("MIRSHA_PAIR"))
            fprintf(stderr, "mirsha: MIRSHA_PAIR / MIRSHA_PAIR_MAX_GROUPS are A/B knobs, read only with MIRSHA_AB=1; "
                            "ignored\n");
        const char* e = ab_getenv("MIRSHA_PAIR");
        if (e && e[0] == '0') return 0u;
        const char* m = ab_getenv("MIRSHA_PAIR_MAX_GROUPS");
        return m ? (uint32_t)strtoul(m, nullptr, 10) : kPairMaxGroups;
    }();
    return v;
}

// Compute units of the current device (cached per device; relaxed atomics:
// mirsha_hash_batch_multi launches from one thread per device).
uint32_t cu_count() {
    static std::atomic<uint32_t> cached[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256u;
    uint32_t v = cached[dev].load(std::memory_order_relaxed);
    if (!v) {
        int a = 0;
        if (hipDeviceGetAttribute(&a, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || a <= 0) a = 256;
        v = (uint32_t)a;
        cached[dev].store(v, std::memory_order_relaxed);
    }
    return v;
}

// The dynamic-LDS limit of kernel `fn` (one of 8 forms) raised on the
// current device, once per (device, form): per-device flags, set with atomics
// (mirsha_hash_batch_multi launches from one thread per device).
hipError_t dyn_lds_attr(const void* fn, int form, uint32_t bytes) {
    static std::atomic<uint8_t> done[64][8] = {};
    int dev = 0;
    if (hipError_t e = hipGetDevice(&dev)) return e;
    if (dev >= 0 && dev < 64 && done[dev][form].load(std::memory_order_acquire)) return hipSuccess;
    if (hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes)) return e;
    if (dev >= 0 && dev < 64) done[dev][form].store(1, std::memory_order_release);
    return hipSuccess;
}

hipError_t launch_msgs(const uint8_t* arena, uint64_t arena_len, const uint64_t* off,
                       const uint32_t* len, const uint32_t* order, uint32_t n, uint8_t* out,
                       int variant, hipStream_t s) {
    if (n == 0) return hipSuccess;
    const uint32_t tiles = (n + 63u) / 64u;
    const uint32_t grid = (tiles + kWavesPerBlock - 1u) / kWavesPerBlock;
    const uint32_t mgrid = (tiles + kMsgWaves - 1u) / kMsgWaves;
    if (arena_len > kMaxBufferArena || n >= kMaxBufferMsgs) {  // 64-bit addressing (LDS loader)
        launch_k(sha256_msgs_kernel<true, true>, mgrid, 64 * kMsgWaves, 0, s, arena, arena_len, off, len, order, n, out);
        return hipGetLastError();
    }
    if (variant == kVariantPair || (variant == kVariantLds && tiles <= pair_max_groups())) {
        launch_k(sha256_msgs_pair_kernel, tiles, kPairThreads, 0, s, arena, arena_len, off, len, order, n, out);
        return hipGetLastError();
    }
    if (variant == kVariantLowOcc || (variant == kVariantLds && tiles <= kLowOccTiles)) {
        launch_k(sha256_msgs_lowocc_kernel, grid, kBlockThreads, 0, s, arena, arena_len, off, len, order, n, out);
        return hipGetLastError();
    }
    if (variant == kVariantCu || variant_is_ab_form(variant) ||
        (variant == kVariantLds && tiles <= kCuMaxWavesPerSimd * 4u * cu_count())) {
        // k waves per SIMD, one workgroup of 4k waves per CU
        const uint32_t k = (tiles + 4u * cu_count() - 1u) / (4u * cu_count());
        const uint32_t wg_waves = 4u * std::min(k, kCuMaxWavesPerSimd);
        const uint32_t cgrid = (tiles + wg_waves - 1u) / wg_waves;
#ifdef MIRSHA_AB_FORMS
        // tools/ab_build.sh lib: the retired and diagnostic forms (11-15)
        const int form = variant == kVariantCuNoYield ? 1 : variant == kVariantCuPrefetch ? 2
                         : variant == kVariantCuDmaPipe ? 3 : variant == kVariantCuDiagNoLoads ? 4
                         : variant == kVariantCuDiagNoPrio ? 5 : 0;
        const void* fns[6] = {(const void*)sha256_msgs_cu_kernel<0>, (const void*)sha256_msgs_cu_kernel<1>,
                              (const void*)sha256_msgs_cu_kernel<2>, (const void*)sha256_msgs_cu_kernel<3>,
                              (const void*)sha256_msgs_cu_kernel<4>, (const void*)sha256_msgs_cu_kernel<5>};
        const int slots[6] = {0, 1, 2, 5, 6, 7};  // dyn_lds_attr forms (3: fused, 4: placement probe)
        if (hipError_t e = dyn_lds_attr(fns[form], slots[form], kCuLds)) return e;
        if (form == 4)
            launch_k(sha256_msgs_cu_kernel<4>, cgrid, 64u * wg_waves, kCuLds, s, arena, arena_len, off, len, order, n, out);
        else if (form == 5)
            launch_k(sha256_msgs_cu_kernel<5>, cgrid, 64u * wg_waves, kCuLds, s, arena, arena_len, off, len, order, n, out);
        else if (form == 1)
            launch_k(sha256_msgs_cu_kernel<1>, cgrid, 64u * wg_waves, kCuLds, s, arena, arena_len, off, len, order, n, out);
        else if (form == 2)
            launch_k(sha256_msgs_cu_kernel<2>, cgrid, 64u * wg_waves, kCuLds, s, arena, arena_len, off, len, order, n, out);
        else if (form == 3)
            launch_k(sha256_msgs_cu_kernel<3>, cgrid, 64u * wg_waves, kCuLds, s, arena, arena_len, off, len, order, n, out);
        else
#endif
        {
            if (hipError_t e = dyn_lds_attr((const void*)sha256_msgs_cu_kernel<0>, 0, kCuLds)) return e;
            launch_k(sha256_msgs_cu_kernel<0>, cgrid, 64u * wg_waves, kCuLds, s, arena, arena_len, off, len, order, n, out);
        }
        return hipGetLastError();
    }
    if (variant == kVariantDirect)
        launch_k(sha256_msgs_kernel<false>, mgrid, 64 * kMsgWaves, 0, s, arena, arena_len, off, len, order, n, out);
    else
        launch_k(sha256_msgs_kernel<true>, mgrid, 64 * kMsgWaves, 0, s, arena, arena_len, off, len, order, n, out);
    return hipGetLastError();
}

hipError_t launch_msgs_overlap(const OverlapArgs& a, hipStream_t s) {
    const uint32_t tiles = (a.n_req + 63u) / 64u;
    if (a.list_waves + tiles == 0) return hipSuccess;
    if (a.arena_len > kMaxBufferArena || a.n_req >= kMaxBufferMsgs || (a.list_waves && a.n_lists == 0))
        return hipErrorInvalidValue;
    launch_k(sha256_msgs_overlap_kernel, a.list_waves + tiles, 64, 0, s, a);
    return hipGetLastError();
}

hipError_t launch_lists(const uint8_t* digests, uint32_t n_digests, const uint32_t* idx, uint32_t n_entries,
                        const uint32_t* first, uint32_t n_lists, uint32_t* scratch, uint8_t* out, hipStream_t s) {
    if (n_lists == 0) return hipSuccess;
    const uint32_t grid = (n_lists + kBlockThreads - 1u) / kBlockThreads;
    launch_k(sha256_lists_kernel, grid, kBlockThreads, 0, s, digests, n_digests, idx, n_entries, first, n_lists, scratch,
                                                      out);
    return hipGetLastError();
}

PadBlockKW pad_block_kw(uint64_t L) {
    auto rotr = [](uint32_t x, int n) { return (x >> n) | (x << (32 - n)); };
    uint32_t w[64] = {0x80000000u};
    w[14] = (uint32_t)(L >> 29);  // FIPS 180-4 §5.1.1: the 64-bit bit length, big-endian
    w[15] = (uint32_t)(L << 3);
    for (int j = 16; j < 64; j++) {
        const uint32_t s0 = rotr(w[j - 15], 7) ^ rotr(w[j - 15], 18) ^ (w[j - 15] >> 3);
        const uint32_t s1 = rotr(w[j - 2], 17) ^ rotr(w[j - 2], 19) ^ (w[j - 2] >> 10);
        w[j] = w[j - 16] + s0 + w[j - 7] + s1;
    }
    PadBlockKW p{};
    for (int j = 0; j < 64; j++) p.kw[j] = kK[j] + w[j];
    p.use = 1u;
    return p;
}

hipError_t launch_chain(const uint8_t* digests, uint32_t n_digests, const uint32_t* cidx, uint32_t n_entries,
                        const uint32_t* cfirst, uint32_t n_lists, uint32_t ob, uint32_t oe, uint32_t* state,
                        uint8_t* out, hipStream_t s, uint32_t uniform) {
    if (n_lists == 0) return hipSuccess;
    const uint32_t grid = (n_lists + kBlockThreads - 1u) / kBlockThreads;
    if (uniform) {
        // identity lists: list k = entries [k B, ...) must lie inside n_entries
        if ((uint64_t)(n_lists - 1u) * uniform >= n_entries || (uint64_t)n_lists * uniform < n_entries)
            return hipErrorInvalidValue;
        PadBlockKW pad{};
        if ((uniform & 1u) == 0u) {
            pad = pad_block_kw(32ull * uniform);
            const char* e = ab_getenv("MIRSHA_CHAIN_PAD");  // A/B: the generic final block
            pad.use = !(e && e[0] == '0');
        }
        launch_k(sha256_chain_kernel<true>, grid, kBlockThreads, 0, s, digests, n_digests, cidx, n_entries, cfirst,
                 n_lists, ob, oe, state, out, uniform, pad);
    } else {
        launch_k(sha256_chain_kernel<false>, grid, kBlockThreads, 0, s, digests, n_digests, cidx, n_entries, cfirst,
                 n_lists, ob, oe, state, out, 0u, PadBlockKW{});
    }
    return hipGetLastError();
}

hipError_t launch_chain_pair(const uint8_t* digests, uint32_t n_digests, const uint32_t* cidx, uint32_t n_entries,
                             const uint32_t* cfirst, uint32_t n_lists, uint8_t* out, hipStream_t s) {
    if (n_lists == 0) return hipSuccess;
    const uint32_t groups = (n_lists + 63u) / 64u;
    launch_k(sha256_chain_pair_kernel, groups, kPairThreads, 0, s, digests, n_digests, cidx, n_entries, cfirst, n_lists, out);
    return hipGetLastError();
}

hipError_t launch_fused_paced(const FusedArgs& a, uint32_t grid, uint32_t pace, hipStream_t s) {
    if (grid == 0) return hipSuccess;
    if (pace < 1 || pace > kPacedMaxPace || a.n_queues != pace) return hipErrorInvalidValue;
    if (hipError_t e = dyn_lds_attr((const void*)sha256_fused_paced_kernel, 3, kPacedLds)) return e;
    launch_k(sha256_fused_paced_kernel, grid, 256u * pace, kPacedLds, s, a);
    return hipGetLastError();
}

hipError_t launch_placement_probe(uint32_t grid, uint32_t pace, uint32_t* broken, uint32_t test, hipStream_t s) {
    if (grid == 0) return hipSuccess;
    if (pace < 1 || pace > kPacedMaxPace) return hipErrorInvalidValue;
    if (hipError_t e = dyn_lds_attr((const void*)placement_probe_kernel, 4, kPacedLds)) return e;
    launch_k(placement_probe_kernel, grid, 256u * pace, kPacedLds, s, broken, test);
    return hipGetLastError();
}

hipError_t launch_mixed_lengths(uint64_t seed, uint64_t first, uint64_t count, uint32_t* len, hipStream_t s) {
    if (count == 0) return hipSuccess;
    launch_k(mixed_lengths_kernel, (unsigned)((count + 255u) / 256u), 256, 0, s, seed, first, count, len);
    return hipGetLastError();
}

// ---- streaming checkpoint chains (testengine NodeState.ActiveHash) ---------
// Running SHA-256 states, one per application node: the checkpoint value of
// testengine/recorder.go:213-256 is Sum() of a hash that every committed
// request digest is written into (ActiveHash.Write, :223), reset at each
// checkpoint (Set, :187).  State per chain: midstate h[8], the pending
// digest of an odd count (its 8 big-endian words) and the digest count.
// Writes are 32-byte digests, so a block is always two whole digests.
__device__ __forceinline__ void load_digest_words(const uint8_t* __restrict__ digests, uint32_t p, bool live,
                                                  uint32_t w[8]) {
    if (live) {
        const uint4* d = reinterpret_cast<const uint4*>(digests + 32ull * p);
        const uint4 a = d[0], b = d[1];
        w[0] = __builtin_bswap32(a.x); w[1] = __builtin_bswap32(a.y);
        w[2] = __builtin_bswap32(a.z); w[3] = __builtin_bswap32(a.w);
        w[4] = __builtin_bswap32(b.x); w[5] = __builtin_bswap32(b.y);
        w[6] = __builtin_bswap32(b.z); w[7] = __builtin_bswap32(b.w);
    } else {
#pragma unroll
        for (int i = 0; i < 8; i++) w[i] = 0u;
    }
}

// One lane per chain with new digests pos[afirst[k] .. afirst[k+1]) (in write
// order).  With `odd` = a digest pending from earlier writes, the lane
// completes (odd + m) / 2 blocks: block t = digest q ‖ digest q+1 with
// q = 2t - odd (q = -1: the pending digest).
__global__ __launch_bounds__(kBlockThreads) void chains_absorb_kernel(
    const uint8_t* __restrict__ digests, const uint32_t* __restrict__ pos, const uint32_t* __restrict__ act,
    const uint32_t* __restrict__ afirst, uint32_t n_active, uint32_t* __restrict__ h, uint32_t* __restrict__ pend,
    uint64_t* __restrict__ cnt) {
    const uint32_t k = blockIdx.x * kBlockThreads + threadIdx.x;
    const bool valid = k < n_active;
    const uint32_t c = valid ? act[k] : 0u;
    const uint32_t e0 = valid ? afirst[k] : 0u;
    const uint32_t m = valid ? afirst[k + 1] - e0 : 0u;
    uint32_t st[8], pw[8];
    uint64_t n = 0;
    if (valid) {
#pragma unroll
        for (int i = 0; i < 8; i++) {
            st[i] = h[8ull * c + i];
            pw[i] = pend[8ull * c + i];
        }
        n = cnt[c];
    }
    const uint32_t odd = (uint32_t)(n & 1u);
    const uint32_t blocks = (odd + m) / 2u;
    const uint32_t steps = wave_max(blocks);
    for (uint32_t t = 0; t < steps; t++) {
        const bool live = t < blocks;
        const int32_t q = (int32_t)(2u * t) - (int32_t)odd;
        uint32_t w[16];
        if (q < 0) {
#pragma unroll
            for (int i = 0; i < 8; i++) w[i] = pw[i];
        } else {
            // Guarded like the second load below: past this lane's own block
            // count the index would run beyond its range in pos.
            load_digest_words(digests, live ? pos[e0 + (uint32_t)q] : 0u, live, w);
        }
        load_digest_words(digests, live ? pos[e0 + (uint32_t)(q + 1)] : 0u, live, w + 8);
        if (live) compress_asm_lat(st, w);
    }
    if (valid) {
        if ((odd + m) & 1u) {
            if (m) load_digest_words(digests, pos[e0 + m - 1u], true, pw);  // else the old pending stays
        }
#pragma unroll
        for (int i = 0; i < 8; i++) {
            h[8ull * c + i] = st[i];
            pend[8ull * c + i] = pw[i];
        }
        cnt[c] = n + m;
    }
}

// Sum(nil) of chains which[0..k): the final padded block (pending digest, if
// any, then 0x80 and the 64-bit bit length) from a copy of the midstate.
__global__ __launch_bounds__(kBlockThreads) void chains_sum_kernel(const uint32_t* __restrict__ which, uint32_t k_n,
                                                                   const uint32_t* __restrict__ h,
                                                                   const uint32_t* __restrict__ pend,
                                                                   const uint64_t* __restrict__ cnt,
                                                                   uint8_t* __restrict__ out) {
    const uint32_t k = blockIdx.x * kBlockThreads + threadIdx.x;
    const bool valid = k < k_n;
    const uint32_t c = valid ? which[k] : 0u;
    uint32_t st[8], w[16];
    const uint64_t n = valid ? cnt[c] : 0u;
    const bool odd = (n & 1u) != 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
        st[i] = valid ? h[8ull * c + i] : 0u;
        w[i] = odd ? pend[8ull * c + i] : 0u;
        w[8 + i] = 0u;
    }
    w[odd ? 8 : 0] = 0x80000000u;
    const uint64_t bits = n * 256u;
    w[14] = (uint32_t)(bits >> 32);
    w[15] = (uint32_t)bits;
    compress_asm_lat(st, w);
    if (valid) store_digest(out, k, st);
}

__global__ __launch_bounds__(kBlockThreads) void chains_reset_kernel(const uint32_t* __restrict__ which, uint32_t k_n,
                                                                     uint32_t* __restrict__ h,
                                                                     uint64_t* __restrict__ cnt) {
    const uint32_t k = blockIdx.x * kBlockThreads + threadIdx.x;
    if (k >= k_n) return;
    const uint32_t c = which[k];
#pragma unroll
    for (int i = 0; i < 8; i++) h[8ull * c + i] = kH0[i];
    cnt[c] = 0u;
}

hipError_t launch_chains_absorb(const uint8_t* digests, const uint32_t* pos, const uint32_t* act, const uint32_t* afirst,
                                uint32_t n_active, uint32_t* h, uint32_t* pend, uint64_t* cnt, hipStream_t s) {
    if (n_active == 0) return hipSuccess;
    launch_k(chains_absorb_kernel, (n_active + kBlockThreads - 1u) / kBlockThreads, kBlockThreads, 0, s, 
        digests, pos, act, afirst, n_active, h, pend, cnt);
    return hipGetLastError();
}

hipError_t launch_chains_sum(const uint32_t* which, uint32_t k, const uint32_t* h, const uint32_t* pend,
                             const uint64_t* cnt, uint8_t* out, hipStream_t s) {
    if (k == 0) return hipSuccess;
    launch_k(chains_sum_kernel, (k + kBlockThreads - 1u) / kBlockThreads, kBlockThreads, 0, s, which, k, h, pend, cnt, out);
    return hipGetLastError();
}

hipError_t launch_chains_reset(const uint32_t* which, uint32_t k, uint32_t* h, uint64_t* cnt, hipStream_t s) {
    if (k == 0) return hipSuccess;
    launch_k(chains_reset_kernel, (k + kBlockThreads - 1u) / kBlockThreads, kBlockThreads, 0, s, which, k, h, cnt);
    return hipGetLastError();
}

hipError_t launch_gen_mixed(uint64_t seed, uint64_t first, uint64_t count, const uint64_t* off, uint8_t* arena,
                            hipStream_t s) {
    if (count == 0) return hipSuccess;
    const uint64_t blocks = std::min<uint64_t>((count + 3u) / 4u, 65536u);
    launch_k(gen_mixed_kernel, (unsigned)blocks, 256, 0, s, seed, first, count, off, arena);
    return hipGetLastError();
}

hipError_t launch_gen_requests(uint64_t seed, uint64_t first, uint64_t count, uint32_t data_len,
                               uint8_t* arena, hipStream_t s) {
    if (count == 0) return hipSuccess;
    const uint64_t words = count * ((data_len + 7u) / 8u + 2u);
    const uint64_t grid = (words + 255u) / 256u;
    launch_k(gen_requests_kernel, (unsigned)grid, 256, 0, s, seed, first, count, data_len, arena);
    return hipGetLastError();
}

}  // namespace mirsha
