// compress_bench.hip -- end-to-end cycles per SHA-256 compression for the
// instruction-order variants of tools/gen_compress_variants.py, pure
// registers, at 8 / 4 / 2 waves per SIMD.  Every variant's output is checked
// word for word against the production form (variant 0).
//
// Build: python tools/gen_compress_variants.py > tools/compress_variants.h &&
//        hipcc --offload-arch=gfx950 -O3 -o tools/compress_bench tools/compress_bench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "compress_variants.h"

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                 \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

static constexpr uint32_t kH0[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                    0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

template <int V>
__global__ __launch_bounds__(256) void loop(uint32_t* out, unsigned long long* clk, int nblk) {
    uint32_t st[8], w[16];
    uint32_t dm = threadIdx.x, ds = blockIdx.x;
#pragma unroll
    for (int i = 0; i < 8; i++) st[i] = kH0[i] ^ (threadIdx.x + 977u * blockIdx.x);
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int b = 0; b < nblk; b++) {
#pragma unroll
        for (int i = 0; i < 16; i++) w[i] = st[i & 7] + i;
        uint32_t s[8];
#pragma unroll
        for (int i = 0; i < 8; i++) s[i] = st[i];
        cv_run<V>(s, w, dm, ds);
#pragma unroll
        for (int i = 0; i < 8; i++) st[i] += s[i];
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
    for (int i = 0; i < 8; i++) out[gid * 8 + i] = st[i];
    if (dm == 0xFFFFFFFFu) out[0] = 0;  // keep dm live
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

static std::vector<uint32_t> ref_out;

template <int V>
void run1(int wps, uint32_t* d_out, unsigned long long* d_clk) {
    const int nblk = 256;
    const int grid = 256 * wps;  // 256 CUs x wps blocks of 4 waves = wps waves per SIMD
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    loop<V><<<grid, 256>>>(d_out, d_clk, nblk);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
        CHECK(hipEventRecord(e0));
        loop<V><<<grid, 256>>>(d_out, d_clk, nblk);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    std::vector<unsigned long long> clk(2 * grid);
    CHECK(hipMemcpy(clk.data(), d_clk, sizeof(unsigned long long) * 2 * grid, hipMemcpyDeviceToHost));
    double ghz = 0;
    for (int b = 0; b < grid; b++) ghz += (double)clk[2 * b] / (double)clk[2 * b + 1] * 0.1;
    ghz /= grid;
    const size_t nout = (size_t)grid * 256 * 8;
    std::vector<uint32_t> out(nout);
    CHECK(hipMemcpy(out.data(), d_out, nout * 4, hipMemcpyDeviceToHost));
    bool ok = true;
    if (V == 0) {
        if (ref_out.size() < nout) ref_out = out;
    } else {
        for (size_t i = 0; i < nout; i++)
            if (out[i] != ref_out[i]) { ok = false; break; }
    }
    const double comps = (double)grid * 256 * nblk;
    const double per_simd_wave = comps / 64.0 / 1024.0;
    printf("{\"variant\": \"%s\", \"wps\": %d, \"ms\": %.4f, \"clock_ghz\": %.3f, \"gcompress_per_s\": %.2f, "
           "\"cycles_per_wave_compress\": %.1f, \"match\": %s}\n",
           kCvNames[V], wps, best, ghz, comps / (best * 1e-3) / 1e9, best * 1e-3 * ghz * 1e9 / per_simd_wave,
           ok ? "true" : "false");
    fflush(stdout);
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
}

template <int V>
void run_all(uint32_t* d_out, unsigned long long* d_clk) {
    if constexpr (V < CV_COUNT) {
        for (int wps : {8, 4}) run1<V>(wps, d_out, d_clk);
        run_all<V + 1>(d_out, d_clk);
    }
}

int main() {
    uint32_t* d_out;
    unsigned long long* d_clk;
    CHECK(hipMalloc(&d_out, sizeof(uint32_t) * 256 * 8 * 256 * 8));
    CHECK(hipMalloc(&d_clk, sizeof(unsigned long long) * 2 * 256 * 8));
    // variant 0 at wps 8 first fills the reference outputs (largest grid)
    run_all<0>(d_out, d_clk);
    return 0;
}
