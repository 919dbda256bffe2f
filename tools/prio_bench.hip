// prio_bench.hip — can a latency-bound SHA-256 chain wave keep near-alone
// speed on a SIMD that also runs 3..7 throughput (request) waves?
//
// Blocks 0..255 (one per CU, 4 waves = one per SIMD) are "chain" waves: NC
// sequential compressions, optionally at s_setprio 3.  Blocks 256.. are
// "request" waves running NR compressions each.  Reports the chain waves'
// in-kernel cycles per compression (s_memtime) against the chain-alone run.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/prio_bench tools/prio_bench.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../mirbft_amd/csrc/sha256_device.h"

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                 \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

// kCode: 0 = chain and request waves run the SAME compression code; 1 = the
// request waves run a different copy (compiler C++ rounds); 2 = the chain runs
// 4 distinct inlined copies per loop iteration (~45 KB of code), requests the
// asm copy -- instruction-cache footprint probes.
template <int kPrio, int kCode>
__global__ __launch_bounds__(256) void pb(unsigned* out, unsigned long long* clk, int nc, int nr) {
    const bool chain = blockIdx.x < 256;
    if (chain && kPrio) __builtin_amdgcn_s_setprio(3);
    uint32_t st[8], w[16];
#pragma unroll
    for (int i = 0; i < 8; i++) st[i] = mirsha::kH0[i] ^ threadIdx.x ^ blockIdx.x;
    const int n = chain ? nc : nr;
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    if (kCode == 2 && chain) {
        for (int b = 0; b < n; b += 4) {
#pragma unroll
            for (int u = 0; u < 4; u++) {
#pragma unroll
                for (int i = 0; i < 16; i++) w[i] = st[i & 7] + i + u;
                mirsha::compress_asm(st, w);
            }
        }
    } else {
        for (int b = 0; b < n; b++) {
#pragma unroll
            for (int i = 0; i < 16; i++) w[i] = st[i & 7] + i;
            if (kCode == 1 && !chain)
                mirsha::compress(st, w);
            else
                mirsha::compress_asm(st, w);
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = st[0] ^ st[7];
    if ((threadIdx.x & 63) == 0) {
        const int wv = blockIdx.x * 4 + (threadIdx.x >> 6);
        clk[2 * wv] = t1 - t0;
        clk[2 * wv + 1] = r1 - r0;
    }
}

template <int kPrio, int kCode = 0>
void run(int extra_per_simd, int nc, int nr, unsigned* d_out, unsigned long long* d_clk) {
    const int grid = 256 * (1 + extra_per_simd);
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    pb<kPrio, kCode><<<grid, 256>>>(d_out, d_clk, nc, nr);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    pb<kPrio, kCode><<<grid, 256>>>(d_out, d_clk, nc, nr);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> clk(2 * grid * 4);
    CHECK(hipMemcpy(clk.data(), d_clk, sizeof(unsigned long long) * clk.size(), hipMemcpyDeviceToHost));
    std::vector<double> cc, rc;
    double ghz = 0;
    for (int w = 0; w < grid * 4; w++) {
        const double cyc = (double)clk[2 * w];
        ghz += cyc / (double)clk[2 * w + 1] * 0.1;
        if (w < 1024) cc.push_back(cyc / nc); else rc.push_back(cyc / nr);
    }
    ghz /= grid * 4;
    std::sort(cc.begin(), cc.end());
    std::sort(rc.begin(), rc.end());
    printf("{\"code\": %d, \"prio\": %d, \"req_waves_per_simd\": %d, \"nc\": %d, \"nr\": %d, \"ms\": %.4f, \"clock_ghz\": %.3f, "
           "\"chain_cyc_per_comp_med\": %.1f, \"chain_cyc_per_comp_max\": %.1f, \"req_cyc_per_comp_med\": %.1f}\n",
           kCode, kPrio, extra_per_simd, nc, nr, ms, ghz, cc[cc.size() / 2], cc.back(),
           rc.empty() ? 0.0 : rc[rc.size() / 2]);
    fflush(stdout);
}

int main() {
    unsigned* d_out;
    unsigned long long* d_clk;
    CHECK(hipMalloc(&d_out, sizeof(unsigned) * 256 * 9 * 256));
    CHECK(hipMalloc(&d_clk, sizeof(unsigned long long) * 2 * 256 * 9 * 4));
    const int nc = 200;
    run<0>(0, nc, 0, d_out, d_clk);
    for (int extra : {1, 3, 7}) {
        // request waves run longer than the chain so the chain never runs alone
        run<0>(extra, nc, 400, d_out, d_clk);
        run<1>(extra, nc, 400, d_out, d_clk);
    }
    run<1, 1>(1, nc, 400, d_out, d_clk);
    run<1, 1>(3, nc, 400, d_out, d_clk);
    run<1, 2>(0, nc, 0, d_out, d_clk);
    run<1, 2>(1, nc, 400, d_out, d_clk);
    run<1, 2>(3, nc, 400, d_out, d_clk);
    return 0;
}
