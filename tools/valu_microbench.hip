// valu_microbench.hip — measured issue rate of the int32 VALU instructions the
// SHA-256 rounds use, on gfx950, plus the in-kernel shader clock.
//
// Each lane runs ITERS x 64 instructions of ONE kind over 8 independent
// chains (no dependency stalls at 8 waves/SIMD); the grid fills every SIMD
// with 8 waves.  Reports ns per wave-instruction per SIMD and cycles at the
// measured clock (s_memtime / s_memrealtime x 100 MHz).
//
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/valu_mb tools/valu_microbench.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e = (x);                                                        \
        if (e != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                 \
            exit(1);                                                               \
        }                                                                          \
    } while (0)

constexpr int ITERS = 2048;

#define REP8(S) S(0) S(1) S(2) S(3) S(4) S(5) S(6) S(7)

// 8 chains, each instruction depends only on its own chain's previous value.
#define BODY(OPSTR)                                                                            \
    asm volatile(OPSTR(0) OPSTR(1) OPSTR(2) OPSTR(3) OPSTR(4) OPSTR(5) OPSTR(6) OPSTR(7)       \
                 : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]),     \
                   "+v"(x[6]), "+v"(x[7])                                                      \
                 : "v"(y), "s"(k), "v"(z));

#define OP_ADD(i) "v_add_u32_e32 %" #i ", %" #i ", %8\n\t"
#define OP_ADD3(i) "v_add3_u32 %" #i ", %" #i ", %9, %8\n\t"
#define OP_ALIGN(i) "v_alignbit_b32 %" #i ", %" #i ", %" #i ", 7\n\t"
#define OP_BITOP3(i) "v_bitop3_b32 %" #i ", %" #i ", %8, %" #i " bitop3:0x96\n\t"
#define OP_BFI(i) "v_bfi_b32 %" #i ", %" #i ", %8, %" #i "\n\t"
#define OP_XOR(i) "v_xor_b32_e32 %" #i ", %" #i ", %8\n\t"
#define OP_LSHR(i) "v_lshrrev_b32_e32 %" #i ", 3, %" #i "\n\t"
#define OP_FMA(i) "v_fma_f32 %" #i ", %" #i ", %8, %8\n\t"
#define OP_ADD3V(i) "v_add3_u32 %" #i ", %" #i ", %8, %10\n\t"
#define OP_BITOP3V(i) "v_bitop3_b32 %" #i ", %" #i ", %8, %10 bitop3:0xca\n\t"
#define OP_ALIGN2(i) "v_alignbit_b32 %" #i ", %" #i ", %8, 7\n\t"
#define OP_LSHLOR(i) "v_lshl_or_b32 %" #i ", %" #i ", 7, %8\n\t"
#define OP_OR3(i) "v_or3_b32 %" #i ", %" #i ", %8, %10\n\t"
#define OP_LSHLADD(i) "v_lshl_add_u32 %" #i ", %" #i ", 3, %8\n\t"
#define OP_ANDOR(i) "v_and_or_b32 %" #i ", %" #i ", %8, %10\n\t"
#define OP_PERM(i) "v_perm_b32 %" #i ", %" #i ", %8, %10\n\t"
#define OP_ALIGNBYTE(i) "v_alignbyte_b32 %" #i ", %" #i ", %" #i ", 1\n\t"
#define OP_XAD(i) "v_xad_u32 %" #i ", %" #i ", %8, %10\n\t"
#define OP_ADDLSHL(i) "v_add_lshl_u32 %" #i ", %" #i ", %8, 3\n\t"
#define OP_LSHLREV(i) "v_lshlrev_b32_e32 %" #i ", 7, %" #i "\n\t"
#define OP_ADD3SV(i) "v_add3_u32 %" #i ", %" #i ", %9, %8\n\t" "v_add_u32_e32 %" #i ", %" #i ", %8\n\t"
// T2: independent simple/complex alternation (chains 0..7 all different)
#define T2BODY "v_add_u32_e32 %0, %0, %8\n\tv_alignbit_b32 %1, %1, %1, 7\n\tv_add_u32_e32 %2, %2, %8\n\tv_alignbit_b32 %3, %3, %3, 7\n\tv_add_u32_e32 %4, %4, %8\n\tv_alignbit_b32 %5, %5, %5, 7\n\tv_add_u32_e32 %6, %6, %8\n\tv_alignbit_b32 %7, %7, %7, 7\n\t"
// T3: dependent adds (one chain per statement position, consecutive instructions dependent)
#define T3BODY "v_add_u32_e32 %0, %0, %8\n\tv_add_u32_e32 %0, %0, %8\n\tv_add_u32_e32 %0, %0, %8\n\tv_add_u32_e32 %0, %0, %8\n\tv_add_u32_e32 %1, %1, %8\n\tv_add_u32_e32 %1, %1, %8\n\tv_add_u32_e32 %1, %1, %8\n\tv_add_u32_e32 %1, %1, %8\n\t"
// T4: simple pairs then complex pairs: add a, add b, align c, align d
#define T4BODY "v_add_u32_e32 %0, %0, %8\n\tv_add_u32_e32 %1, %1, %8\n\tv_alignbit_b32 %2, %2, %2, 7\n\tv_alignbit_b32 %3, %3, %3, 7\n\tv_add_u32_e32 %4, %4, %8\n\tv_add_u32_e32 %5, %5, %8\n\tv_alignbit_b32 %6, %6, %6, 7\n\tv_alignbit_b32 %7, %7, %7, 7\n\t"
// T5: dependent bitop3 chain
#define T5BODY "v_bitop3_b32 %0, %0, %8, %10 bitop3:0x96\n\tv_bitop3_b32 %0, %0, %8, %10 bitop3:0x96\n\tv_bitop3_b32 %0, %0, %8, %10 bitop3:0x96\n\tv_bitop3_b32 %0, %0, %8, %10 bitop3:0x96\n\tv_bitop3_b32 %1, %1, %8, %10 bitop3:0x96\n\tv_bitop3_b32 %1, %1, %8, %10 bitop3:0x96\n\tv_bitop3_b32 %1, %1, %8, %10 bitop3:0x96\n\tv_bitop3_b32 %1, %1, %8, %10 bitop3:0x96\n\t"
// T6: 3 simple (add, bitop3, xor) independent, then 1 complex
#define T6BODY "v_add_u32_e32 %0, %0, %8\n\tv_bitop3_b32 %1, %1, %8, %10 bitop3:0x96\n\tv_xor_b32_e32 %2, %2, %8\n\tv_alignbit_b32 %3, %3, %3, 7\n\tv_add_u32_e32 %4, %4, %8\n\tv_bitop3_b32 %5, %5, %8, %10 bitop3:0x96\n\tv_xor_b32_e32 %6, %6, %8\n\tv_alignbit_b32 %7, %7, %7, 7\n\t"
#define RAWBODY(STR) asm volatile(STR : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]) : "v"(y), "s"(k), "v"(z));
#define OP_LSHR7(i) "v_lshrrev_b32_e32 %" #i ", 7, %" #i "\n\t"
#define OP_LSHL3(i) "v_lshlrev_b32_e32 %" #i ", 3, %" #i "\n\t"
#define OP_LSHLV(i) "v_lshlrev_b32_e32 %" #i ", %8, %" #i "\n\t"
#define OP_OR(i) "v_or_b32_e32 %" #i ", %" #i ", %8\n\t"
#define OP_SUB(i) "v_sub_u32_e32 %" #i ", %" #i ", %8\n\t"
#define OP_MIXAA(i) "v_alignbit_b32 %" #i ", %" #i ", %" #i ", 7\n\t" "v_add_u32_e32 %" #i ", %" #i ", %8\n\t"

template <int KIND>
__global__ __launch_bounds__(256) void mb(unsigned* out, unsigned long long* clk) {
    unsigned x[8];
    const unsigned y = threadIdx.x * 2654435761u;
    const unsigned k = 0x9E3779B9u;
    const unsigned z = threadIdx.x * 40503u + 7u;
#pragma unroll
    for (int i = 0; i < 8; i++) x[i] = threadIdx.x + i;
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS; it++) {
        // 8 statements x 8 instructions = 64 instructions per iteration
#pragma unroll
        for (int u = 0; u < 8; u++) {
            if constexpr (KIND == 0) BODY(OP_ADD)
            if constexpr (KIND == 1) BODY(OP_ADD3)
            if constexpr (KIND == 2) BODY(OP_ALIGN)
            if constexpr (KIND == 3) BODY(OP_BITOP3)
            if constexpr (KIND == 4) BODY(OP_BFI)
            if constexpr (KIND == 5) BODY(OP_XOR)
            if constexpr (KIND == 6) BODY(OP_LSHR)
            if constexpr (KIND == 7) BODY(OP_FMA)
            if constexpr (KIND == 8) BODY(OP_ADD3V)
            if constexpr (KIND == 9) BODY(OP_BITOP3V)
            if constexpr (KIND == 10) BODY(OP_ALIGN2)
            if constexpr (KIND == 11) BODY(OP_LSHLOR)
            if constexpr (KIND == 12) BODY(OP_OR3)
            if constexpr (KIND == 13) BODY(OP_LSHLADD)
            if constexpr (KIND == 14) BODY(OP_ANDOR)
            if constexpr (KIND == 15) BODY(OP_PERM)
            if constexpr (KIND == 16) BODY(OP_ALIGNBYTE)
            if constexpr (KIND == 17) BODY(OP_XAD)
            if constexpr (KIND == 18) BODY(OP_ADDLSHL)
            if constexpr (KIND == 19) BODY(OP_LSHLREV)
            if constexpr (KIND == 20) BODY(OP_ADD3SV)
            if constexpr (KIND == 21) BODY(OP_MIXAA)
            if constexpr (KIND == 22) RAWBODY(T2BODY)
            if constexpr (KIND == 23) RAWBODY(T3BODY)
            if constexpr (KIND == 24) RAWBODY(T4BODY)
            if constexpr (KIND == 25) RAWBODY(T5BODY)
            if constexpr (KIND == 26) RAWBODY(T6BODY)
            if constexpr (KIND == 27) BODY(OP_LSHR7)
            if constexpr (KIND == 28) BODY(OP_LSHL3)
            if constexpr (KIND == 29) BODY(OP_LSHLV)
            if constexpr (KIND == 30) BODY(OP_OR)
            if constexpr (KIND == 31) BODY(OP_SUB)
        }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    unsigned acc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) acc ^= x[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

template <int KIND>
void run(const char* name, int blocks, unsigned* d_out, unsigned long long* d_clk) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    mb<KIND><<<blocks, 256>>>(d_out, d_clk);  // warm-up
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
        CHECK(hipEventRecord(e0));
        mb<KIND><<<blocks, 256>>>(d_out, d_clk);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    unsigned long long* clk = (unsigned long long*)malloc(sizeof(unsigned long long) * 2 * blocks);
    CHECK(hipMemcpy(clk, d_clk, sizeof(unsigned long long) * 2 * blocks, hipMemcpyDeviceToHost));
    double ghz = 0;
    for (int b = 0; b < blocks; b++) ghz += (double)clk[2 * b] / (double)clk[2 * b + 1] * 0.1;
    ghz /= blocks;
    free(clk);
    const double waves = blocks * 4.0;
    const double insts = waves * ITERS * 64.0 * ((KIND == 20 || KIND == 21) ? 2 : 1);  // wave-instructions
    const double per_simd = insts / 1024.0;             // 256 CUs x 4 SIMDs
    const double ns = best * 1e6 / per_simd;            // ns per wave-instruction per SIMD
    printf("{\"op\": \"%s\", \"ms\": %.4f, \"ns_per_wave_inst_per_simd\": %.4f, \"clock_ghz\": %.3f, "
           "\"cycles_per_wave_inst\": %.3f, \"lane_ops_per_s_T\": %.2f}\n",
           name, best, ns, ghz, ns * ghz, insts * 64.0 / (best * 1e-3) / 1e12);
}

#include "../mirbft_amd/csrc/sha256_device.h"
#include "sha256_rounds_asm_ab.h"

// Pure-register SHA-256 compression loop (generated-asm rounds): the
// achievable per-compression cost with no memory traffic at all.
template <int V>
__device__ __forceinline__ void compress_variant(uint32_t st[8], uint32_t w[16]) {
    uint32_t s[8];
#pragma unroll
    for (int i = 0; i < 8; i++) s[i] = st[i];
    if constexpr (V == 0) mirsha::rounds_asm(s, w);
    if constexpr (V == 1) mirsha::rounds_asm_bfi(s, w);
    if constexpr (V == 2) mirsha::rounds_asm_add2(s, w);
    if constexpr (V == 3) mirsha::rounds_asm_lit(s, w);
    if constexpr (V == 4) mirsha::rounds_asm_add2lit(s, w);
    if constexpr (V == 5) mirsha::rounds_asm_ilp(s, w);
#pragma unroll
    for (int i = 0; i < 8; i++) st[i] += s[i];
}

template <int kAsm>
__global__ __launch_bounds__(256) void sha_loop(unsigned* out, unsigned long long* clk, int nblk) {
    uint32_t st[8], w[16];
#pragma unroll
    for (int i = 0; i < 8; i++) st[i] = mirsha::kH0[i] ^ threadIdx.x;
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int b = 0; b < nblk; b++) {
#pragma unroll
        for (int i = 0; i < 16; i++) w[i] = st[i & 7] + i;
        if constexpr (kAsm >= 0) compress_variant<kAsm>(st, w); else mirsha::compress(st, w);
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    out[blockIdx.x * blockDim.x + threadIdx.x] = st[0] ^ st[7];
    if (threadIdx.x == 0) {
        clk[2 * blockIdx.x] = t1 - t0;
        clk[2 * blockIdx.x + 1] = r1 - r0;
    }
}

template <int kAsm>
void run_sha1(int blocks, unsigned* d_out, unsigned long long* d_clk, int wpb) {
    const int nblk = 256;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int grid = blocks * wpb / 8;
    sha_loop<kAsm><<<grid, 256>>>(d_out, d_clk, nblk);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 5; rep++) {
        CHECK(hipEventRecord(e0));
        sha_loop<kAsm><<<grid, 256>>>(d_out, d_clk, nblk);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }
    unsigned long long* clk = (unsigned long long*)malloc(sizeof(unsigned long long) * 2 * grid);
    CHECK(hipMemcpy(clk, d_clk, sizeof(unsigned long long) * 2 * grid, hipMemcpyDeviceToHost));
    double ghz = 0;
    for (int b = 0; b < grid; b++) ghz += (double)clk[2 * b] / (double)clk[2 * b + 1] * 0.1;
    ghz /= grid;
    free(clk);
    const double comps = (double)grid * 256 * nblk;
    const double per_simd_wave_blocks = comps / 64.0 / 1024.0;
    printf("{\"op\": \"sha256_compress_%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"clock_ghz\": %.3f, "
           "\"gcompress_per_s\": %.2f, \"cycles_per_wave_compress\": %.1f}\n",
           kAsm == 0 ? "asm" : kAsm == 1 ? "asm_bfi" : kAsm == 2 ? "asm_add2" : kAsm == 3 ? "asm_lit" : kAsm == 4 ? "asm_add2lit" : kAsm == 5 ? "asm_ilp" : "cxx", wpb, best, ghz, comps / (best * 1e-3) / 1e9,
           best * 1e-3 * ghz * 1e9 / per_simd_wave_blocks);
}

void run_sha(int blocks, unsigned* d_out, unsigned long long* d_clk) {
    for (int wps : {8, 2, 1}) {
        run_sha1<0>(blocks, d_out, d_clk, wps);
        run_sha1<5>(blocks, d_out, d_clk, wps);
        run_sha1<-1>(blocks, d_out, d_clk, wps);
    }
}

int main() {
    const int blocks = 256 * 8;  // 8 blocks of 4 waves per CU = 8 waves/SIMD
    unsigned* d_out;
    unsigned long long* d_clk;
    CHECK(hipMalloc(&d_out, sizeof(unsigned) * blocks * 256));
    CHECK(hipMalloc(&d_clk, sizeof(unsigned long long) * 2 * blocks));
    run<0>("v_add_u32", blocks, d_out, d_clk);
    run<1>("v_add3_u32(sgpr)", blocks, d_out, d_clk);
    run<2>("v_alignbit_b32", blocks, d_out, d_clk);
    run<3>("v_bitop3_b32", blocks, d_out, d_clk);
    run<4>("v_bfi_b32", blocks, d_out, d_clk);
    run<5>("v_xor_b32", blocks, d_out, d_clk);
    run<6>("v_lshrrev_b32", blocks, d_out, d_clk);
    run<7>("v_fma_f32", blocks, d_out, d_clk);
    run<8>("v_add3_u32(3 vgpr)", blocks, d_out, d_clk);
    run<9>("v_bitop3_b32(3 vgpr)", blocks, d_out, d_clk);
    run<10>("v_alignbit_b32(2 vgpr)", blocks, d_out, d_clk);
    run<11>("v_lshl_or_b32", blocks, d_out, d_clk);
    run<12>("v_or3_b32", blocks, d_out, d_clk);
    run<13>("v_lshl_add_u32", blocks, d_out, d_clk);
    run<14>("v_and_or_b32", blocks, d_out, d_clk);
    run<15>("v_perm_b32", blocks, d_out, d_clk);
    run<16>("v_alignbyte_b32", blocks, d_out, d_clk);
    run<17>("v_xad_u32", blocks, d_out, d_clk);
    run<18>("v_add_lshl_u32", blocks, d_out, d_clk);
    run<19>("v_lshlrev_b32", blocks, d_out, d_clk);
    run<20>("mix add3(sgpr)+add", blocks, d_out, d_clk);
    run<21>("mix alignbit+add", blocks, d_out, d_clk);
    run<22>("T2 add|align alternating, independent", blocks, d_out, d_clk);
    run<23>("T3 dependent adds", blocks, d_out, d_clk);
    run<24>("T4 add,add,align,align independent", blocks, d_out, d_clk);
    run<25>("T5 dependent bitop3", blocks, d_out, d_clk);
    run<26>("T6 add,bitop3,xor,align independent", blocks, d_out, d_clk);
    run<27>("v_lshrrev_b32 7", blocks, d_out, d_clk);
    run<28>("v_lshlrev_b32 3", blocks, d_out, d_clk);
    run<29>("v_lshlrev_b32 vgpr", blocks, d_out, d_clk);
    run<30>("v_or_b32", blocks, d_out, d_clk);
    run<31>("v_sub_u32", blocks, d_out, d_clk);
    if (getenv("MB_SHA")) run_sha(blocks, d_out, d_clk);
    return 0;
}
