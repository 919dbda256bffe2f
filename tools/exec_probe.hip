// exec_probe.hip -- does a wave64 VALU op with part of EXEC off issue faster
// on gfx950?  (verdict r5 item 1: DESIGN.md §5.1 / §5.3 assumed "a wave costs
// the same with fewer lanes"; this measures it.)
//
// Every SIMD runs W waves (W = 1, 2, 4, 8: one 256-thread workgroup per CU
// per W) of back-to-back SHA-256 compressions on registers -- the request
// kernel's rounds (compress_asm, issue-yield form) or the chains' latency
// form (compress_asm_lat) -- with EXEC set by a lane test around the loop:
//   mask 0  all 64 lanes                      mask 1  lanes 0..31 (low half)
//   mask 2  lanes 0..15                        mask 3  even lanes (32, both halves)
//   mask 4  lanes 32..63 (high half)
// Reported per (form, mask, W): SIMD cycles per wave-compression from the
// launch span (first start .. last end of s_memrealtime, at the clock
// s_memtime / s_memrealtime shows), and per lane-compression (÷ active lanes).
// Prints one JSON line per case.
//
// Build: hipcc --offload-arch=gfx950 -O3 -I mirbft_amd/csrc -o tools/exec_probe tools/exec_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "sha256_device.h"

#define CHECK(x)                                                   \
    do {                                                           \
        hipError_t e = (x);                                        \
        if (e != hipSuccess) {                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); \
            exit(1);                                               \
        }                                                          \
    } while (0)

using namespace mirsha;

__device__ __forceinline__ bool lane_on(int mask, uint32_t lane) {
    switch (mask) {
        case 1: return lane < 32u;
        case 2: return lane < 16u;
        case 3: return (lane & 1u) == 0u;
        case 4: return lane >= 32u;
        default: return true;
    }
}

template <int FORM, int MASK>
__global__ __launch_bounds__(256) void probe(uint32_t iters, unsigned long long* __restrict__ stamps,
                                             uint32_t* __restrict__ sink) {
    uint32_t st[8], w[16];
#pragma unroll
    for (int i = 0; i < 8; i++) st[i] = kH0[i] ^ threadIdx.x;
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = kK[i] + blockIdx.x;
    const uint32_t lane = threadIdx.x & 63u;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    if (lane_on(MASK, lane)) {
        for (uint32_t b = 0; b < iters; b++) {
            if constexpr (FORM == 0)
                compress_asm(st, w);
            else
                compress_asm_lat(st, w);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
    const uint32_t gw = blockIdx.x * 4u + (threadIdx.x >> 6);
    if (lane == 0u) {
        stamps[3ull * gw] = t1 - t0;
        stamps[3ull * gw + 1ull] = r0;
        stamps[3ull * gw + 2ull] = r1;
    }
    sink[blockIdx.x * 256u + threadIdx.x] = st[0] ^ st[7];
}

using Kern = void (*)(uint32_t, unsigned long long*, uint32_t*);

template <int FORM>
Kern pick(int mask) {
    switch (mask) {
        case 1: return probe<FORM, 1>;
        case 2: return probe<FORM, 2>;
        case 3: return probe<FORM, 3>;
        case 4: return probe<FORM, 4>;
        default: return probe<FORM, 0>;
    }
}

static const int kActive[5] = {64, 32, 16, 32, 32};
static const char* kMaskName[5] = {"full64", "low32", "low16", "even32", "high32"};

int main(int argc, char** argv) {
    const uint32_t iters = argc > 1 ? (uint32_t)atoi(argv[1]) : 64u;
    const int reps = argc > 2 ? atoi(argv[2]) : 3;
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const uint32_t cus = (uint32_t)prop.multiProcessorCount;
    const uint32_t max_blocks = cus * 8u;
    unsigned long long* stamps;
    uint32_t* sink;
    CHECK(hipMalloc(&stamps, 24ull * 4u * max_blocks));
    CHECK(hipMalloc(&sink, 4ull * 256u * max_blocks));
    std::vector<unsigned long long> h(3ull * 4u * max_blocks);
    // warm the clock: a second of full-occupancy throughput rounds
    for (int i = 0; i < 8; i++) hipLaunchKernelGGL(pick<0>(0), dim3(max_blocks), dim3(256), 0, 0, 256u, stamps, sink);
    CHECK(hipDeviceSynchronize());
    for (int form = 0; form < 2; form++)
        for (uint32_t wps : {1u, 2u, 4u, 8u})
            for (int mask = 0; mask < 5; mask++)
                for (int rep = 0; rep < reps; rep++) {
                    const uint32_t blocks = cus * wps, waves = 4u * blocks;
                    Kern k = form == 0 ? pick<0>(mask) : pick<1>(mask);
                    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, iters, stamps, sink);
                    CHECK(hipGetLastError());
                    CHECK(hipDeviceSynchronize());
                    CHECK(hipMemcpy(h.data(), stamps, 24ull * waves, hipMemcpyDeviceToHost));
                    std::vector<double> ghz(waves), percomp(waves);
                    unsigned long long first = ~0ull, last = 0;
                    for (uint32_t w = 0; w < waves; w++) {
                        const unsigned long long c = h[3 * w], a = h[3 * w + 1], b = h[3 * w + 2];
                        ghz[w] = b > a ? 0.1 * (double)c / (double)(b - a) : 0.0;
                        percomp[w] = (double)c / iters;
                        first = std::min(first, a);
                        last = std::max(last, b);
                    }
                    std::nth_element(ghz.begin(), ghz.begin() + waves / 2, ghz.end());
                    std::nth_element(percomp.begin(), percomp.begin() + waves / 2, percomp.end());
                    const double clk = ghz[waves / 2];
                    const double span_us = (double)(last - first) / 100.0;
                    const double span_cycles = span_us * 1e3 * clk;
                    const double per_wave_comp = span_cycles / ((double)iters * wps);
                    printf("{\"form\": \"%s\", \"mask\": \"%s\", \"active_lanes\": %d, \"waves_per_simd\": %u, "
                           "\"rep\": %d, \"iters\": %u, \"clock_ghz\": %.4f, \"span_us\": %.2f, "
                           "\"simd_cycles_per_wave_compression\": %.1f, \"simd_cycles_per_lane_compression\": %.2f, "
                           "\"wave_loop_cycles_per_compression_median\": %.1f}\n",
                           form == 0 ? "throughput" : "latency", kMaskName[mask], kActive[mask], wps, rep, iters,
                           clk, span_us, per_wave_comp, per_wave_comp / kActive[mask], percomp[waves / 2]);
                    fflush(stdout);
                }
    CHECK(hipFree(stamps));
    CHECK(hipFree(sink));
    return 0;
}
