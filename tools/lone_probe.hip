// lone_probe.hip -- where does a LONE wave's block time go?  One wave per SIMD
// (one 4-wave workgroup per CU) hashes 64 messages of 4112 B laid out as
// config 3's, 64 blocks each, adding the fused launch's per-block pieces one
// at a time (profiles/r04l: a lone last-queue wave takes ~3.4 us per block
// against ~2.5 us for the latency round form's rounds alone):
//   0  rounds only (latency form), words from registers
//   1  + the words read back from a static LDS tile (4 x ds_read_b128) + bswap
//   2  + the block loaded by LDS-DMA one block ahead (the fused launch's loader)
//   3  + two blocks ahead (two tiles, s_waitcnt vmcnt(4))
//   4  mode 3 + the per-block s_setprio and LDS live-count read of the fused loop
//   5  mode 3 with the throughput round form (issue yields)
//   6  mode 3 + the per-block s_setprio only;  7  mode 3 + the LDS live-count read only
//   8  mode 3 in the fused loop's shape: both round forms in the loop, chosen by a
//      cached flag, each under a per-lane block-count test
// Prints SIMD cycles per block at the clock s_memtime / s_memrealtime reports.
//
// Build: hipcc --offload-arch=gfx950 -O3 -I mirbft_amd/csrc -o tools/lone_probe tools/lone_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "sha256_device.h"

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                 \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

using namespace mirsha;

constexpr uint32_t kStride = 4112u;

__device__ __forceinline__ uint32_t slot_of(uint32_t m, uint32_t q) { return m * 4u + (q ^ ((m >> 2) & 3u)); }

__shared__ uint32_t g_live[4];

template <int MODE>
__global__ __launch_bounds__(256, 1) void lone(const uint8_t* __restrict__ arena, uint32_t arena_len,
                                               uint32_t* __restrict__ out, unsigned long long* clk, int nblk) {
    __shared__ uint4 tiles[4][2][256];  // [wave][tile][slot]: 4 KiB per tile
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    if (threadIdx.x < 4u) g_live[threadIdx.x] = 1u;
    __syncthreads();
    uint4* my = tiles[wv][0];
    uint4* my2 = tiles[wv][1];
    const uint32_t wave = blockIdx.x * 4u + wv;
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)arena, (short)0, (int)arena_len, 0x00020000);
    const uint32_t qd = (lane & 3u) ^ ((lane >> 4) & 3u);
    uint32_t vd[4];
#pragma unroll
    for (int j = 0; j < 4; j++) vd[j] = (wave * 64u + 16u * j + (lane >> 2)) * kStride + 16u * qd;
    constexpr bool deep = MODE >= 3;
    auto tile_of = [&](uint32_t b) { return (deep && (b & 1u)) ? my2 : my; };
    auto issue = [&](uint32_t b) {
        uint4* t = tile_of(b);
#pragma unroll
        for (int j = 0; j < 4; j++)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)(t + 64 * j), 16,
                                                     vd[j], 64u * b, 0, 0);
    };
    uint32_t st[8];
#pragma unroll
    for (int i = 0; i < 8; i++) st[i] = kH0[i] + lane;
    uint32_t wr[16];
#pragma unroll
    for (int i = 0; i < 16; i++) wr[i] = lane * 131u + (uint32_t)i;
    if constexpr (MODE == 1) {  // a static tile
#pragma unroll
        for (int k = 0; k < 4; k++) my[slot_of(lane, (uint32_t)k)] = make_uint4(lane, k, 7u, 9u);
        __builtin_amdgcn_s_waitcnt(0);
    }
    const uint32_t n = (uint32_t)nblk;
    uint32_t lone_sel = wv + 1u;                     // (mode 8)
    const bool live_flag = g_live[wv] <= 1u;          // (mode 8: alone from the start)
    const uint32_t nb_lane = n + (lane & 1u);         // (mode 8: a per-lane block count, >= n)
    if constexpr (MODE >= 2) {
        issue(0u);
        if (deep && 1u < n) issue(1u);
    }
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (uint32_t b = 0; b < n; b++) {
        uint32_t w[16];
        if constexpr (MODE == 0) {
#pragma unroll
            for (int i = 0; i < 16; i++) w[i] = wr[i] ^ st[i & 7];
        } else {
            if constexpr (MODE >= 2) {
                if (deep && b + 1u < n)
                    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                else
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            const uint4* tb = tile_of(b);
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint4 x = tb[slot_of(lane, (uint32_t)k)];
                w[4 * k + 0] = x.x; w[4 * k + 1] = x.y; w[4 * k + 2] = x.z; w[4 * k + 3] = x.w;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            if constexpr (MODE >= 2) {
                const uint32_t nx = b + (deep ? 2u : 1u);
                if (nx < n) issue(nx);
            }
#pragma unroll
            for (int k = 0; k < 16; k++) w[k] = __builtin_bswap32(w[k]);
        }
        bool alone = true;
        if constexpr (MODE == 4 || MODE == 6) __builtin_amdgcn_s_setprio(0);
        if constexpr (MODE == 4 || MODE == 7) {
            const uint32_t lv = __hip_atomic_load(&g_live[wv], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            alone = (uint32_t)__builtin_amdgcn_readfirstlane((int)lv) <= 1u;
        }
        if constexpr (MODE == 8) {  // the fused loop's shape: both round forms, a per-lane block count
            if (lone_sel != 0u && live_flag) lone_sel = 0xFFFFFFFFu;
            if (lone_sel == 0xFFFFFFFFu) {
                if (b < nb_lane) compress_asm_lat(st, w);
            } else if (b < nb_lane) {
                compress_asm(st, w);
            }
        } else if (MODE == 5 || !alone) {
            compress_asm(st, w);
        } else {
            compress_asm_lat(st, w);
        }
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) acc ^= st[i];
    out[blockIdx.x * 256u + threadIdx.x] = acc;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = c1 - c0;
        clk[1] = r1 - r0;
    }
}

template <int MODE>
static void run(const uint8_t* d_arena, uint32_t arena_len, uint32_t* d_out, unsigned long long* d_clk, int cus,
                int nblk) {
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    lone<MODE><<<cus, 256>>>(d_arena, arena_len, d_out, d_clk, nblk);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    unsigned long long clk[2] = {0, 0};
    for (int rep = 0; rep < 7; rep++) {
        CHECK(hipEventRecord(a));
        lone<MODE><<<cus, 256>>>(d_arena, arena_len, d_out, d_clk, nblk);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) {
            best = ms;
            CHECK(hipMemcpy(clk, d_clk, sizeof(clk), hipMemcpyDeviceToHost));
        }
    }
    const double ghz = clk[1] ? (double)clk[0] / ((double)clk[1] * 10.0) : 0.0;
    // one wave per SIMD: its own loop cycles are the SIMD's
    printf("{\"mode\": %d, \"blocks\": %d, \"ms\": %.4f, \"clock_ghz\": %.3f, \"cycles_per_block\": %.0f, "
           "\"us_per_block\": %.3f}\n",
           MODE, nblk, best, ghz, (double)clk[0] / nblk, (double)clk[1] / nblk / 100.0);
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
}

int main(int argc, char** argv) {
    const int nblk = argc > 1 ? atoi(argv[1]) : 64;
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const size_t bytes = (size_t)cus * 4 * 64 * kStride;
    uint8_t* d_arena;
    uint32_t* d_out;
    unsigned long long* d_clk;
    CHECK(hipMalloc(&d_arena, bytes));
    CHECK(hipMemset(d_arena, 0x5A, bytes));
    CHECK(hipMalloc(&d_out, (size_t)cus * 256 * 4));
    CHECK(hipMalloc(&d_clk, 16));
    for (int rep = 0; rep < 2; rep++) {
        run<0>(d_arena, (uint32_t)bytes, d_out, d_clk, cus, nblk);
        run<1>(d_arena, (uint32_t)bytes, d_out, d_clk, cus, nblk);
        run<2>(d_arena, (uint32_t)bytes, d_out, d_clk, cus, nblk);
        run<3>(d_arena, (uint32_t)bytes, d_out, d_clk, cus, nblk);
        run<4>(d_arena, (uint32_t)bytes, d_out, d_clk, cus, nblk);
        run<5>(d_arena, (uint32_t)bytes, d_out, d_clk, cus, nblk);
        run<6>(d_arena, (uint32_t)bytes, d_out, d_clk, cus, nblk);
        run<7>(d_arena, (uint32_t)bytes, d_out, d_clk, cus, nblk);
        run<8>(d_arena, (uint32_t)bytes, d_out, d_clk, cus, nblk);
    }
    CHECK(hipFree(d_arena));
    CHECK(hipFree(d_out));
    CHECK(hipFree(d_clk));
    return 0;
}
