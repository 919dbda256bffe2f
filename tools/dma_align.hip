// dma_align.hip -- probe: H2D rate of 32 MiB copies from page-locked memory
// (hipHostMalloc, as mirsha_host_alloc) by source / destination alignment.
// The Go binding's chunks start at request boundaries (272-byte granularity
// at config 2), the host API's at fixed MiB offsets.  Prints one JSON line:
// per case the median GB/s of 9 copies of 10 back-to-back chunks.
//   hipcc --offload-arch=gfx950 -O2 -o tools/dma_align tools/dma_align.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    const size_t chunk = 32ull << 20, nch = 10, bytes = chunk * nch + (1 << 20);
    void *h = nullptr, *d = nullptr;
    if (hipHostMalloc(&h, bytes, hipHostMallocDefault) != hipSuccess) return 2;
    if (hipMalloc(&d, bytes) != hipSuccess) return 3;
    memset(h, 1, bytes);
    hipStream_t s;
    (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    struct Case {
        const char* name;
        size_t src_off, dst_off, step;
    } cases[] = {
        {"aligned_4k", 0, 0, chunk},
        {"src16_dst16", 16, 16, chunk},
        {"src272_dst272", 272, 272, chunk},
        {"src272_dst0", 272, 0, chunk},
        {"request_cut_272", 0, 0, chunk - chunk % 272},  // chunks of whole 272-B requests
        {"src4_dst4", 4, 4, chunk},
        {"src1_dst1", 1, 1, chunk},
    };
    printf("{");
    bool first = true;
    for (const Case& c : cases) {
        std::vector<double> t;
        for (int r = 0; r < 10; r++) {
            const double t0 = now();
            for (size_t k = 0; k < nch; k++) {
                const size_t o = k * c.step;
                (void)hipMemcpyAsync((char*)d + c.dst_off + o, (const char*)h + c.src_off + o, c.step,
                                     hipMemcpyHostToDevice, s);
            }
            (void)hipStreamSynchronize(s);
            if (r) t.push_back(now() - t0);
        }
        std::sort(t.begin(), t.end());
        printf("%s\"%s\": %.1f", first ? "" : ", ", c.name, (double)c.step * nch / t[t.size() / 2] / 1e9);
        first = false;
        fflush(stdout);
    }
    // D2H of digest-sized copies (a 32 MiB chunk of config 2 returns 3.9 MB),
    // alone and while a 32 MiB H2D runs on another stream.
    hipStream_t s2;
    (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (size_t sz : {1ull << 20, 4ull << 20, 16ull << 20, 64ull << 20})
        for (int busy = 0; busy < 2; busy++) {
            std::vector<double> t;
            for (int r = 0; r < 10; r++) {
                if (busy) (void)hipMemcpyAsync(d, h, chunk, hipMemcpyHostToDevice, s2);
                (void)hipEventRecord(e0, s);
                (void)hipMemcpyAsync((char*)h + chunk, (const char*)d + chunk, sz, hipMemcpyDeviceToHost, s);
                (void)hipEventRecord(e1, s);
                (void)hipStreamSynchronize(s);
                (void)hipStreamSynchronize(s2);
                float ms = 0;
                (void)hipEventElapsedTime(&ms, e0, e1);
                if (r) t.push_back(ms * 1e-3);
            }
            std::sort(t.begin(), t.end());
            printf(", \"d2h_%zuMiB%s_gbs\": %.1f", sz >> 20, busy ? "_during_h2d" : "", sz / t[t.size() / 2] / 1e9);
            fflush(stdout);
        }
    printf("}\n");
    (void)hipHostFree(h);
    (void)hipFree(d);
    return 0;
}
