// numa_h2d.hip -- probe: H2D / D2H bandwidth of page-locked host memory
// placed on each NUMA node, for the GPU this process uses.  The host API's
// page-locked arenas (mirsha_host_alloc) are DMA'd at PCIe rate; if the node
// the pages live on matters, the library should place them next to the GPU.
// Prints one JSON line: the GPU's PCI bus id and NUMA node (sysfs), then per
// node {h2d_gbs, d2h_gbs} for a 256 MiB copy (median of 9), with and without
// 15 threads streaming through host memory at the same time (the Go
// binding's packing goroutines).
//   hipcc --offload-arch=gfx950 -O2 -o tools/numa_h2d tools/numa_h2d.hip -lpthread
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include <immintrin.h>

static long mbind_(void* addr, unsigned long len, int mode, const unsigned long* mask, unsigned long maxnode,
                   unsigned flags) {
    return syscall(SYS_mbind, addr, len, mode, mask, maxnode, flags);
}

static int n_nodes() {
    int n = 0;
    for (;; n++) {
        std::string p = "/sys/devices/system/node/node" + std::to_string(n);
        if (access(p.c_str(), F_OK) != 0) break;
    }
    return n;
}

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static std::atomic<bool> g_stop{false};
static void* streamer(void* arg) {
    // read + write a private 64 MiB buffer in a loop (memory traffic like packing)
    const size_t n = 64ull << 20;
    uint8_t* a = (uint8_t*)malloc(n);
    uint8_t* b = (uint8_t*)malloc(n);
    memset(a, 1, n);
    memset(b, 2, n);
    while (!g_stop.load(std::memory_order_relaxed)) memcpy(b, a, n);
    free(a);
    free(b);
    (void)arg;
    return nullptr;
}

int main(int argc, char** argv) {
    const int dev = argc > 1 ? atoi(argv[1]) : 0;
    const size_t bytes = 256ull << 20;
    if (hipSetDevice(dev) != hipSuccess) return 2;
    char bus[64] = {0};
    (void)hipDeviceGetPCIBusId(bus, sizeof bus, dev);
    for (char* p = bus; *p; p++) *p = (char)tolower(*p);
    int gpu_node = -1;
    {
        std::string path = std::string("/sys/bus/pci/devices/") + bus + "/numa_node";
        FILE* f = fopen(path.c_str(), "r");
        if (f) {
            if (fscanf(f, "%d", &gpu_node) != 1) gpu_node = -1;
            fclose(f);
        }
    }
    void* d = nullptr;
    if (hipMalloc(&d, bytes) != hipSuccess) return 3;
    hipStream_t s;
    (void)hipStreamCreate(&s);
    const int nn = n_nodes();
    printf("{\"device\": %d, \"pci_bus_id\": \"%s\", \"gpu_numa_node\": %d, \"nodes\": %d, \"per_node\": [", dev, bus,
           gpu_node, nn);
    for (int node = 0; node < nn; node++) {
        void* h = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (h == MAP_FAILED) return 4;
        unsigned long mask[16] = {0};
        mask[node / 64] = 1ul << (node % 64);
        const long mb = mbind_(h, bytes, 2 /* MPOL_BIND */, mask, 1024, 0);
        memset(h, 7, bytes);  // fault the pages in on that node
        if (hipHostRegister(h, bytes, hipHostRegisterDefault) != hipSuccess) return 5;
        double res[2][2];  // [quiet / loaded][h2d / d2h]
        for (int loaded = 0; loaded < 2; loaded++) {
            std::vector<pthread_t> th;
            if (loaded) {
                g_stop = false;
                th.resize(15);
                for (auto& t : th) pthread_create(&t, nullptr, streamer, nullptr);
                usleep(200000);
            }
            for (int dir = 0; dir < 2; dir++) {
                std::vector<double> t;
                for (int r = 0; r < 10; r++) {
                    const double t0 = now();
                    if (dir == 0)
                        (void)hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s);
                    else
                        (void)hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s);
                    (void)hipStreamSynchronize(s);
                    if (r) t.push_back(now() - t0);
                }
                std::sort(t.begin(), t.end());
                res[loaded][dir] = bytes / t[t.size() / 2] / 1e9;
            }
            if (loaded) {
                g_stop = true;
                for (auto& t : th) pthread_join(t, nullptr);
            }
        }
        printf("%s{\"node\": %d, \"mbind\": %ld, \"h2d_gbs\": %.1f, \"d2h_gbs\": %.1f, \"h2d_gbs_loaded\": %.1f, "
               "\"d2h_gbs_loaded\": %.1f}",
               node ? ", " : "", node, mb, res[0][0], res[0][1], res[1][0], res[1][1]);
        fflush(stdout);
        (void)hipHostUnregister(h);
        munmap(h, bytes);
    }
    // hipHostMalloc's own placement (what mirsha_host_alloc hands out)
    {
        void* h = nullptr;
        if (hipHostMalloc(&h, bytes, hipHostMallocDefault) != hipSuccess) return 6;
        memset(h, 7, bytes);
        int where = -1;
        {
            long r = syscall(SYS_get_mempolicy, &where, nullptr, 0, h, 3 /* MPOL_F_NODE | MPOL_F_ADDR */);
            if (r != 0) where = -1;
        }
        double bw[2];
        for (int dir = 0; dir < 2; dir++) {
            std::vector<double> t;
            for (int r = 0; r < 10; r++) {
                const double t0 = now();
                if (dir == 0)
                    (void)hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s);
                else
                    (void)hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s);
                (void)hipStreamSynchronize(s);
                if (r) t.push_back(now() - t0);
            }
            std::sort(t.begin(), t.end());
            bw[dir] = bytes / t[t.size() / 2] / 1e9;
        }
        printf("], \"hipHostMalloc\": {\"first_page_node\": %d, \"h2d_gbs\": %.1f, \"d2h_gbs\": %.1f}", where, bw[0],
               bw[1]);
        // Full duplex?  H2D of the whole buffer on one stream while D2H of
        // 1/8 of it (the digests' share of a chunk) runs on another.
        void* h2 = nullptr;
        void* d2 = nullptr;
        hipStream_t s2;
        (void)hipStreamCreate(&s2);
        if (hipHostMalloc(&h2, bytes / 8, hipHostMallocDefault) == hipSuccess && hipMalloc(&d2, bytes / 8) == hipSuccess) {
            std::vector<double> t;
            for (int r = 0; r < 10; r++) {
                const double t0 = now();
                (void)hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s);
                (void)hipMemcpyAsync(h2, d2, bytes / 8, hipMemcpyDeviceToHost, s2);
                (void)hipStreamSynchronize(s);
                (void)hipStreamSynchronize(s2);
                if (r) t.push_back(now() - t0);
            }
            std::sort(t.begin(), t.end());
            const double both = t[t.size() / 2];
            printf(", \"duplex\": {\"h2d_plus_eighth_d2h_ms\": %.3f, \"h2d_alone_ms\": %.3f, \"serial_estimate_ms\": %.3f}",
                   both * 1e3, bytes / (bw[0] * 1e9) * 1e3, (bytes / (bw[0] * 1e9) + bytes / 8 / (bw[1] * 1e9)) * 1e3);
        }
        // Freshly written buffers: 15 threads write the whole buffer (plain
        // stores, or non-temporal stores that bypass the caches), then the
        // H2D starts at once: does DMA of lines still dirty in CPU caches
        // run slower?
        for (int nt = 0; nt < 2; nt++) {
            std::vector<double> t;
            for (int r = 0; r < 10; r++) {
                std::vector<std::thread> th;
                const size_t per = bytes / 15 / 64 * 64;
                for (int k = 0; k < 15; k++)
                    th.emplace_back([&, k] {
                        uint8_t* p = (uint8_t*)h + per * k;
                        const size_t len = k == 14 ? bytes - per * 14 : per;
                        if (!nt) {
                            memset(p, r + k, len);
                        } else {
                            const __m128i v = _mm_set1_epi8((char)(r + k));
                            for (size_t x = 0; x + 16 <= len; x += 16) _mm_stream_si128((__m128i*)(p + x), v);
                            _mm_sfence();
                        }
                    });
                for (auto& x : th) x.join();
                const double t0 = now();
                (void)hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s);
                (void)hipStreamSynchronize(s);
                if (r) t.push_back(now() - t0);
            }
            std::sort(t.begin(), t.end());
            printf(", \"%s\": {\"h2d_gbs\": %.1f}", nt ? "fresh_nontemporal" : "fresh_plain", bytes / t[t.size() / 2] / 1e9);
        }
        (void)hipHostFree(h);
    }
    printf("}\n");
    return 0;
}
