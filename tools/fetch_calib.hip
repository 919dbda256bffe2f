// fetch_calib.hip — calibrate rocprofv3 FETCH_SIZE on gfx950 against known
// byte counts for the access patterns the hash kernels use
// (MI355X_MICROARCH.md §HBM: "calibrate on a known byte count in your own
// access pattern before trusting an absolute").
//
//   k_stream16: fully coalesced 16 B/lane streaming read of B bytes
//   k_segments: the sha256_msgs_kernel loader pattern — per wave instruction
//               16 messages x 64 contiguous bytes (4 lanes x 16 B each), 272-B
//               messages, every byte read exactly once (B = n x 272)
//   k_lane272:  the direct-variant pattern — each lane reads its own 272-B
//               message 16 B at a time (uncoalesced across lanes)
// Run under: rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_ -- ./fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                          \
    do {                                                                  \
        hipError_t e = (x);                                               \
        if (e != hipSuccess) {                                            \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));        \
            exit(1);                                                      \
        }                                                                 \
    } while (0)

__global__ void k_stream16(const uint4* __restrict__ p, size_t n16, unsigned* out) {
    unsigned acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// One wave per 64 messages; block b of every message read as 16-B quarters
// by lane (j, q) = (16 j + lane / 4, lane % 4), exactly like the LDS loader.
__global__ void k_segments(const uint8_t* __restrict__ p, unsigned n_msgs, unsigned* out) {
    const unsigned lane = threadIdx.x & 63u, wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    unsigned acc = 0;
    for (unsigned blk = 0; blk < 5; blk++) {
        for (unsigned j = 0; j < 4; j++) {
            const unsigned m = wave * 64u + 16u * j + (lane >> 2);
            const unsigned pos = 64u * blk + 16u * (lane & 3u);
            if (m < n_msgs && pos < 272u) {
                const uint4 v = *reinterpret_cast<const uint4*>(p + 272ull * m + pos);
                acc ^= v.x ^ v.y ^ v.z ^ v.w;
            }
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_lane272(const uint8_t* __restrict__ p, unsigned n_msgs, unsigned* out) {
    const unsigned m = blockIdx.x * blockDim.x + threadIdx.x;
    unsigned acc = 0;
    if (m < n_msgs)
        for (unsigned pos = 0; pos < 272u; pos += 16u) {
            const uint4 v = *reinterpret_cast<const uint4*>(p + 272ull * m + pos);
            acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const unsigned n = 1u << 20;
    const size_t bytes = 272ull * n;
    uint8_t* d;
    unsigned* o;
    CHECK(hipMalloc(&d, bytes));
    CHECK(hipMalloc(&o, 64));
    CHECK(hipMemset(d, 1, bytes));
    for (int r = 0; r < 3; r++) {
        k_stream16<<<2048, 256>>>(reinterpret_cast<const uint4*>(d), bytes / 16, o);
        k_segments<<<(n / 64 + 3) / 4, 256>>>(d, n, o);
        k_lane272<<<n / 256, 256>>>(d, n, o);
    }
    CHECK(hipDeviceSynchronize());
    printf("{\"bytes_per_launch\": %zu}\n", bytes);
    return 0;
}
