// ilp_asm_probe.hip -- the product's hand-scheduled rounds (rounds_asm, one
// state per lane) against two states interleaved instruction by instruction in
// one wave (tools/gen_ilp2_asm.py: rounds2_asm with the product's issue
// yields, rounds2_asm_noyield without), register-only compressions, W waves
// per SIMD (W workgroups of 4 waves per CU, pinned by their LDS reservation).
// Config 3's request kernel runs 4 waves x 1 state per SIMD; 2 waves x 2
// states carries the same four chains.  Prints cycles per chain-compression
// per SIMD at the clock measured by s_memtime / s_memrealtime.
//
// Build: python3 tools/gen_ilp2_asm.py > tools/sha256_ilp2_asm.h &&
//        hipcc --offload-arch=gfx950 -O3 -I mirbft_amd/csrc -o tools/ilp_asm_probe tools/ilp_asm_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "sha256_rounds_asm.h"
#include "sha256_ilp2_asm.h"

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                 \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

// mode 0: rounds_asm (1 state); 1: rounds2_asm (2 states, yields); 2: rounds2_asm_noyield;
// 3: rounds_asm_nonop (1 state, latency form)
template <int MODE, int W>
__global__ __launch_bounds__(256, W) void probe(uint32_t* out, unsigned long long* clk, int iters) {
    extern __shared__ uint32_t pad[];
    constexpr int S = (MODE == 1 || MODE == 2) ? 2 : 1;
    uint32_t st[S][8], w[S][16];
#pragma unroll
    for (int k = 0; k < S; k++) {
#pragma unroll
        for (int i = 0; i < 8; i++) st[k][i] = threadIdx.x * 0x9E3779B9u + 977u * (uint32_t)i + 31u * (uint32_t)k;
#pragma unroll
        for (int i = 0; i < 16; i++) w[k][i] = blockIdx.x * 0x85EBCA6Bu + 131u * (uint32_t)i + (uint32_t)k;
    }
    const unsigned long long c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; it++) {
        uint32_t s[S][8];
#pragma unroll
        for (int k = 0; k < S; k++)
#pragma unroll
            for (int i = 0; i < 8; i++) s[k][i] = st[k][i];
        if constexpr (MODE == 0) {
            mirsha::rounds_asm(s[0], w[0]);
        } else if constexpr (MODE == 3) {
            mirsha::rounds_asm_nonop(s[0], w[0]);
        } else if constexpr (MODE == 1) {
            rounds2_asm(s[0], w[0], s[1], w[1]);
        } else {
            rounds2_asm_noyield(s[0], w[0], s[1], w[1]);
        }
#pragma unroll
        for (int k = 0; k < S; k++) {
#pragma unroll
            for (int i = 0; i < 8; i++) st[k][i] += s[k][i];
#pragma unroll
            for (int i = 0; i < 16; i++) w[k][i] ^= st[k][i & 7];  // next block depends on this one
        }
    }
    const unsigned long long c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < S; k++)
#pragma unroll
        for (int i = 0; i < 8; i++) acc ^= st[k][i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = c1 - c0;
        clk[1] = r1 - r0;
    }
    if (acc == 0x12345678u) pad[0] = acc;  // keep the LDS reservation
}

template <int MODE, int W>
static void run(const char* name, uint32_t* d_out, unsigned long long* d_clk, int cus, int iters) {
    constexpr int S = (MODE == 1 || MODE == 2) ? 2 : 1;
    const int lds = (160 * 1024) / W - 1024;  // at most W workgroups per CU
    CHECK(hipFuncSetAttribute((const void*)probe<MODE, W>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    const int grid = cus * W;
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    probe<MODE, W><<<grid, 256, lds>>>(d_out, d_clk, 16);  // warm
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    unsigned long long clk[2] = {0, 0};
    for (int rep = 0; rep < 5; rep++) {
        CHECK(hipEventRecord(a));
        probe<MODE, W><<<grid, 256, lds>>>(d_out, d_clk, iters);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        if (ms < best) {
            best = ms;
            CHECK(hipMemcpy(clk, d_clk, sizeof(clk), hipMemcpyDeviceToHost));
        }
    }
    // one SIMD runs W waves x S chains of `iters` compressions
    const double ghz = clk[1] ? (double)clk[0] / ((double)clk[1] * 10.0) : 0.0;  // memrealtime is 100 MHz
    // SIMD cycles per 64-lane compression: the launch's time at the clock block 0
    // measured (s_memtime / s_memrealtime) over the W x S x iters compressions
    // each SIMD ran (block 0's own loop time is NOT the SIMD's: the arbiter
    // issues oldest-first, so the first workgroup finishes well before the rest)
    const double cyc_per_chain_comp = best * 1e-3 * ghz * 1e9 / ((double)W * S * iters);
    const double comps = (double)grid * 256.0 * S * iters;
    printf("{\"form\": \"%s\", \"waves_per_simd\": %d, \"states_per_wave\": %d, \"chains_per_simd\": %d, \"ms\": %.4f, "
           "\"gcomp_per_s\": %.3f, \"clock_ghz\": %.3f, \"simd_cycles_per_64_compressions\": %.0f}\n",
           name, W, S, W * S, best, comps / (best * 1e-3) / 1e9, ghz, cyc_per_chain_comp);
    CHECK(hipEventDestroy(a));
    CHECK(hipEventDestroy(b));
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 3000;
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    uint32_t* d_out;
    unsigned long long* d_clk;
    CHECK(hipMalloc(&d_out, (size_t)cus * 8 * 256 * 4));
    CHECK(hipMalloc(&d_clk, 16));
    if (argc > 2) {  // yield vs latency round form at 1-4 waves per SIMD
        for (int rep = 0; rep < 2; rep++) {
            run<0, 1>("rounds_asm", d_out, d_clk, cus, iters);
            run<3, 1>("rounds_asm_nonop", d_out, d_clk, cus, iters);
            run<0, 2>("rounds_asm", d_out, d_clk, cus, iters);
            run<3, 2>("rounds_asm_nonop", d_out, d_clk, cus, iters);
            run<0, 3>("rounds_asm", d_out, d_clk, cus, iters);
            run<3, 3>("rounds_asm_nonop", d_out, d_clk, cus, iters);
            run<0, 4>("rounds_asm", d_out, d_clk, cus, iters);
            run<3, 4>("rounds_asm_nonop", d_out, d_clk, cus, iters);
        }
        return 0;
    }
    for (int rep = 0; rep < 2; rep++) {
        run<0, 4>("rounds_asm", d_out, d_clk, cus, iters);
        run<1, 2>("rounds2_asm", d_out, d_clk, cus, iters);
        run<2, 2>("rounds2_asm_noyield", d_out, d_clk, cus, iters);
        run<0, 8>("rounds_asm", d_out, d_clk, cus, iters);
        run<1, 4>("rounds2_asm", d_out, d_clk, cus, iters);
        run<2, 4>("rounds2_asm_noyield", d_out, d_clk, cus, iters);
        run<0, 2>("rounds_asm", d_out, d_clk, cus, iters);
        run<1, 1>("rounds2_asm", d_out, d_clk, cus, iters);
        run<2, 1>("rounds2_asm_noyield", d_out, d_clk, cus, iters);
        run<3, 1>("rounds_asm_nonop", d_out, d_clk, cus, iters);
    }
    CHECK(hipFree(d_out));
    CHECK(hipFree(d_clk));
    return 0;
}
