#!/usr/bin/env python3
"""Generates tools/rot_bench.hip: issue cost on gfx950 of the candidate
single-instruction ROTATE forms and the left-shift substitutes, next to the
two reference classes measured by tools/gen_valu_mix.py (v_lshrrev_b32 /
v_add_u32 / v_bitop3_b32 at ~2 cycles per wave-instruction, v_alignbit_b32 /
v_add3_u32 / v_lshlrev_b32 at ~4).

Why: a SHA-256 round spends 6 of its 14 instructions on rotates
(v_alignbit_b32, 4-cycle class), and one 4-cycle instruction in a stream
drags the 2-cycle ones with it (valu_mix: align1+add7 = 3.7 cycles/inst).  A
rotate in the 2-cycle class -- e.g. v_lshrrev_b64 of a duplicated pair (x:x),
whose low half is rotr(x, n) -- would take the compression from ~5,500 to
~3,600 cycles per wave.

Usage: python tools/gen_rot_bench.py && hipcc --offload-arch=gfx950 -O3 \
         -o tools/rot_bench tools/rot_bench.hip && tools/rot_bench
"""
import os
import sys

NP = 8  # 64-bit pair chains: operands %0..%7 (printed v[a:a+1])
NX = 8  # 32-bit chains: operands %8..%15; %16 = y (vgpr), %17 = k (sgpr), %18 = z (vgpr)

OPS = {
    # references
    "add": "v_add_u32_e32 %{x}, %{x}, %16",
    "lshr": "v_lshrrev_b32_e32 %{x}, 25, %{x}",
    "lshl": "v_lshlrev_b32_e32 %{x}, 7, %{x}",
    "lshl_v": "v_lshlrev_b32_e32 %{x}, %16, %{x}",
    "lshr_v": "v_lshrrev_b32_e32 %{x}, %16, %{x}",
    "align": "v_alignbit_b32 %{x}, %{x}, %{x}, 7",
    "bitop3": "v_bitop3_b32 %{x}, %{x}, %16, %18 bitop3:0x96",
    # 64-bit shifts of a pair
    "lshr64": "v_lshrrev_b64 %{p}, 7, %{p}",
    "lshr64_25": "v_lshrrev_b64 %{p}, 25, %{p}",
    "lshl64": "v_lshlrev_b64 %{p}, 7, %{p}",
    "lshladd64": "v_lshl_add_u64 %{p}, %{p}, 3, %{p}",
    "pk_mov": "v_pk_mov_b32 %{p}, %{p}, %{p} op_sel:[1,0]",
    "pk_add_f32": "v_pk_add_f32 %{p}, %{p}, %{p}",
    # left-shift substitutes
    "bfrev": "v_bfrev_b32_e32 %{x}, %{x}",
    "sdwa_mov_w1": "v_mov_b32_sdwa %{x}, %{x} dst_sel:WORD_1 dst_unused:UNUSED_PAD src0_sel:WORD_0",
    "sdwa_lshl": "v_lshlrev_b32_sdwa %{x}, %16, %{x} dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD",
    "sdwa_add": "v_add_u32_sdwa %{x}, %{x}, %16 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0",
    "mul_lo": "v_mul_lo_u32 %{x}, %{x}, %16",
    "mul_hi": "v_mul_hi_u32 %{x}, %{x}, %16",
    "add_self": "v_add_u32_e32 %{x}, %{x}, %{x}",
    "bfe": "v_bfe_u32 %{x}, %{x}, 3, 20",
    "mov": "v_mov_b32_e32 %{x}, %16",
    "xor": "v_xor_b32_e32 %{x}, %{x}, %16",
}


def seq_single(op):
    return [op] * 64


def seq_alt(*ops):
    out = []
    while len(out) < 64:
        out += list(ops)
    return out[:64]


PATTERNS = [(op, seq_single(op)) for op in OPS]
# --mix: 3 slow + 2 fast per group of 5 (3.2 cycles/inst if the classes simply add)
MIX5 = [
    ("mov", "align", "align", "align", "bitop3"),
    ("add", "align", "align", "align", "bitop3"),
    ("xor", "align", "align", "align", "bitop3"),
    ("lshr", "align", "align", "align", "bitop3"),
    ("mov", "align", "align", "align", "mov"),
    ("bitop3", "align", "align", "align", "bitop3"),
    ("align", "mov", "align", "bitop3", "align"),
    ("align", "align", "align", "add", "add"),
    ("align", "align", "align", "mov", "mov"),
    ("align", "align", "align", "lshr", "lshr"),
    ("align", "align", "align", "xor", "xor"),
    ("mov", "lshr64", "lshr64", "lshr64", "bitop3"),
    ("add", "lshr64", "lshr64", "lshr64", "bitop3"),
    ("lshr64", "lshr64", "lshr64", "bitop3", "add"),
]
if "--mix" in sys.argv:
    PATTERNS = [("+".join(m), seq_alt(*m)) for m in MIX5]
    PATTERNS += [
        ("align+mov", seq_alt("align", "mov")),
        ("align+mov+mov", seq_alt("align", "mov", "mov")),
        ("align+lshr", seq_alt("align", "lshr")),
        ("align+xor", seq_alt("align", "xor")),
        ("align+add+mov", seq_alt("align", "add", "mov")),
    ]
PATTERNS += [
    ("lshr64+add", seq_alt("lshr64", "add")),
    ("lshr64+bitop3", seq_alt("lshr64", "bitop3")),
    ("lshr64x3+bitop3+add", seq_alt("lshr64", "lshr64", "lshr64", "bitop3", "add")),
    ("pk_mov+lshr64", seq_alt("pk_mov", "lshr64")),
    ("mov+lshr64x3+bitop3", seq_alt("mov", "lshr64", "lshr64", "lshr64", "bitop3")),
    ("sdwa_mov_w1+add", seq_alt("sdwa_mov_w1", "add")),
    ("bfrev+lshr", seq_alt("bfrev", "lshr")),
    ("lshl_v+add", seq_alt("lshl_v", "add")),
    ("align+add", seq_alt("align", "add")),
]


def render(seq):
    return [OPS[op].replace("{p}", str(i % NP)).replace("{x}", str(NP + i % NX)) for i, op in enumerate(seq)]


def main():
    here = os.path.dirname(os.path.abspath(__file__))
    kernels, runs = [], []
    for pid, (name, seq) in enumerate(PATTERNS):
        body = "\\n\\t".join(render(seq))
        kernels.append(
            f'template <> __device__ __forceinline__ void body<{pid}>(unsigned long long* p, unsigned* x, unsigned y, unsigned k, unsigned z) {{\n'
            f'    asm volatile("{body}\\n\\t"\n'
            '                 : "+v"(p[0]), "+v"(p[1]), "+v"(p[2]), "+v"(p[3]), "+v"(p[4]), "+v"(p[5]), "+v"(p[6]), "+v"(p[7]),\n'
            '                   "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7])\n'
            '                 : "v"(y), "s"(k), "v"(z) : "vcc");\n}\n')
        runs.append(f'        run<{pid}>("{name}", 64, wps, d_out, d_clk);')
    src = f'''// GENERATED by tools/gen_rot_bench.py -- do not edit.
// Issue cost of gfx950 rotate / left-shift candidates (see the generator's docstring).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CHECK(x) do {{ hipError_t e = (x); if (e != hipSuccess) {{ fprintf(stderr, "%s: %s\\n", #x, hipGetErrorString(e)); exit(1); }} }} while (0)
constexpr int ITERS = 1024;
template <int P> __device__ __forceinline__ void body(unsigned long long* p, unsigned* x, unsigned y, unsigned k, unsigned z);
{"".join(kernels)}
template <int P>
__global__ __launch_bounds__(256) void mb(unsigned* out, unsigned long long* clk) {{
    unsigned long long p[8];
    unsigned x[8];
    const unsigned y = threadIdx.x * 2654435761u, k = 0x9E3779B9u ^ blockIdx.x, z = threadIdx.x * 40503u + 7u;
#pragma unroll
    for (int i = 0; i < 8; i++) {{ x[i] = threadIdx.x + i; p[i] = 0x0123456789ABCDEFull * (threadIdx.x + i + 1); }}
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS; it++) {{
        body<P>(p, x, y, k, z);
        body<P>(p, x, y, k, z);
        body<P>(p, x, y, k, z);
        body<P>(p, x, y, k, z);
    }}
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    unsigned acc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) acc ^= x[i] ^ (unsigned)p[i] ^ (unsigned)(p[i] >> 32);
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
    if (threadIdx.x == 0) {{ clk[2 * blockIdx.x] = t1 - t0; clk[2 * blockIdx.x + 1] = r1 - r0; }}
}}
template <int P>
void run(const char* name, int n_real, int wps, unsigned* d_out, unsigned long long* d_clk) {{
    const int blocks = 256 * wps;  // 4 waves per block, one per SIMD: wps waves per SIMD
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    mb<P><<<blocks, 256>>>(d_out, d_clk);
    CHECK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int rep = 0; rep < 3; rep++) {{
        CHECK(hipEventRecord(e0));
        mb<P><<<blocks, 256>>>(d_out, d_clk);
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
    }}
    static unsigned long long clk[2 * 256 * 16];
    CHECK(hipMemcpy(clk, d_clk, sizeof(unsigned long long) * 2 * blocks, hipMemcpyDeviceToHost));
    double ghz = 0;
    for (int b = 0; b < blocks; b++) ghz += (double)clk[2 * b] / (double)clk[2 * b + 1] * 0.1;
    ghz /= blocks;
    const double insts = (double)ITERS * 4 * n_real;
    const double cpi_wall = best * 1e-3 * ghz * 1e9 / (insts * wps);
    printf("{{\\"pattern\\": \\"%s\\", \\"wps\\": %d, \\"ms\\": %.4f, \\"clock_ghz\\": %.3f, \\"cyc_per_inst_wall\\": %.3f}}\\n",
           name, wps, best, ghz, cpi_wall);
    fflush(stdout);
    CHECK(hipEventDestroy(e0)); CHECK(hipEventDestroy(e1));
}}
int main() {{
    unsigned* d_out; unsigned long long* d_clk;
    CHECK(hipMalloc(&d_out, sizeof(unsigned) * 256 * 16 * 256));
    CHECK(hipMalloc(&d_clk, sizeof(unsigned long long) * 2 * 256 * 16));
    const int wlist[2] = {{8, 2}};
    for (int wi = 0; wi < 2; wi++) {{
        const int wps = wlist[wi];
{chr(10).join(runs)}
    }}
    return 0;
}}
'''
    with open(os.path.join(here, "rot_bench.hip"), "w") as f:
        f.write(src)
    print(f"wrote {len(runs)} patterns")


if __name__ == "__main__":
    main()
