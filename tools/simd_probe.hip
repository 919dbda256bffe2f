// simd_probe.hip -- where do the waves of one workgroup land?  Reads HW_ID
// (s_getreg, gfx9 layout: wave [3:0], simd [5:4], cu [11:8], sh [12], se
// [15:13]) per wave and reports, for each workgroup shape, how often two waves
// of the same workgroup share a SIMD.  Input for the split-wave chain kernel
// (a producer wave and a consumer wave must sit on different SIMDs).
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/simd_probe tools/simd_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <vector>

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                 \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

__global__ void probe(uint32_t* out, uint32_t* xcc) {
    extern __shared__ uint32_t pad[];
    const uint32_t hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));   // HW_REG_HW_ID, 32 bits
    const uint32_t xc = __builtin_amdgcn_s_getreg(20 | (15 << 11));  // HW_REG_XCC_ID (gfx940+), 16 bits
    if ((threadIdx.x & 63) == 0) {
        const uint32_t w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
        out[w] = hw;
        xcc[w] = xc;
        pad[0] = hw;  // keep the LDS reservation
    }
    // stay resident a while so the dispatcher cannot reuse SIMDs
    uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < 2000) {
    }
}

static void run(int threads, int blocks, int lds) {
    const int wpb = threads / 64;
    const int nw = blocks * wpb;
    uint32_t *d, *dx;
    CHECK(hipMalloc(&d, 4 * nw));
    CHECK(hipMalloc(&dx, 4 * nw));
    probe<<<blocks, threads, lds>>>(d, dx);
    CHECK(hipDeviceSynchronize());
    std::vector<uint32_t> h(nw), hx(nw);
    CHECK(hipMemcpy(h.data(), d, 4 * nw, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(hx.data(), dx, 4 * nw, hipMemcpyDeviceToHost));
    int shared_pairs = 0, pairs = 0, same_cu = 0;
    std::map<int, int> simd_of_wave0;
    std::map<std::pair<int, int>, int> by_index;  // (wave index in block, simd) -> count
    for (int b = 0; b < blocks; b++) {
        for (int i = 0; i < wpb; i++) {
            const uint32_t a = h[b * wpb + i];
            by_index[{i, (int)((a >> 4) & 3)}]++;
            for (int j = i + 1; j < wpb; j++) {
                const uint32_t c = h[b * wpb + j];
                pairs++;
                const bool cu_same = ((a >> 8) & 0xFF) == ((c >> 8) & 0xFF) && ((a >> 13) & 7) == ((c >> 13) & 7) &&
                                     hx[b * wpb + i] == hx[b * wpb + j];
                same_cu += cu_same;
                shared_pairs += cu_same && ((a >> 4) & 3) == ((c >> 4) & 3);
            }
        }
    }
    printf("{\"threads\": %d, \"blocks\": %d, \"lds\": %d, \"wave_pairs\": %d, \"same_cu\": %d, \"same_simd\": %d, "
           "\"simd_by_wave_index\": \"",
           threads, blocks, lds, pairs, same_cu, shared_pairs);
    for (auto& kv : by_index) printf("w%d:s%d=%d ", kv.first.first, kv.first.second, kv.second);
    printf("\"}\n");
    CHECK(hipFree(d));
    CHECK(hipFree(dx));
}

int main() {
    run(128, 256, 0);
    run(128, 1024, 0);
    run(128, 256, 80 * 1024);
    run(256, 256, 80 * 1024);
    run(256, 1024, 0);
    run(512, 256, 80 * 1024);
    return 0;
}
