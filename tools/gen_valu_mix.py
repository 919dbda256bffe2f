#!/usr/bin/env python3
"""Generates tools/valu_mix.hip: issue-cost microbenchmarks for gfx950 VALU
instruction *sequences* (not single opcodes): how a stream's cost depends on
which opcode classes it mixes and in what grouping, at 1/2/4/8 waves per SIMD.

Why: tools/valu_microbench.hip found two cost classes among the int32 ops the
SHA-256 rounds use (~2.2 cycles per wave-instruction: v_add_u32, v_xor_b32,
v_lshrrev_b32, v_bitop3_b32; ~4.1: v_alignbit_b32, v_add3_u32, v_lshlrev_b32,
v_perm_b32 ...) and mixed streams costing more than the sum.  The grouping
that minimises a round's cost decides how the round asm is generated.

Usage: python tools/gen_valu_mix.py && hipcc --offload-arch=gfx950 -O3 \
         -o tools/valu_mix tools/valu_mix.hip && tools/valu_mix
"""
import os

NCH = 16  # independent chains (operands %0..%15); %16 = y (vgpr), %17 = k (sgpr), %18 = z (vgpr)

# opcode templates over chain register c
OPS = {
    "add": "v_add_u32_e32 %{c}, %{c}, %16",
    "adds": "v_add_u32_e32 %{c}, %17, %{c}",          # SGPR src0
    "addlit": "v_add_u32_e32 %{c}, 0x428a2f98, %{c}",   # literal src0
    "sub": "v_sub_u32_e32 %{c}, %{c}, %16",
    "xor": "v_xor_b32_e32 %{c}, %{c}, %16",
    "and": "v_and_b32_e32 %{c}, %{c}, %16",
    "or": "v_or_b32_e32 %{c}, %{c}, %16",
    "xnor": "v_xnor_b32_e32 %{c}, %{c}, %16",
    "not": "v_not_b32_e32 %{c}, %{c}",
    "mov": "v_mov_b32_e32 %{c}, %16",
    "lshr": "v_lshrrev_b32_e32 %{c}, 3, %{c}",
    "ashr": "v_ashrrev_i32_e32 %{c}, 3, %{c}",
    "lshl": "v_lshlrev_b32_e32 %{c}, 3, %{c}",
    "lshl_e64": "v_lshlrev_b32_e64 %{c}, 3, %{c}",
    "lshr_e64": "v_lshrrev_b32_e64 %{c}, 3, %{c}",
    "add_e64": "v_add_u32_e64 %{c}, %{c}, %16",
    "lshl16": "v_lshlrev_b16_e32 %{c}, 3, %{c}",
    "pk_add16": "v_pk_add_u16 %{c}, %{c}, %16",
    "pk_lshl16": "v_pk_lshlrev_b16 %{c}, 3, %{c}",
    "mul24": "v_mul_u32_u24_e32 %{c}, %{c}, %16",
    "max": "v_max_u32_e32 %{c}, %{c}, %16",
    "cnd": "v_cndmask_b32_e32 %{c}, %{c}, %16, vcc",
    "bitop3": "v_bitop3_b32 %{c}, %{c}, %16, %18 bitop3:0x96",
    "bitop3s": "v_bitop3_b32 %{c}, %{c}, %17, %18 bitop3:0x96",
    "bitop3_16": "v_bitop3_b16 %{c}, %{c}, %16, %18 bitop3:0x96",
    "align": "v_alignbit_b32 %{c}, %{c}, %{c}, 7",
    "align_s": "v_alignbit_b32 %{c}, %{c}, %{c}, %17",
    "alignbyte": "v_alignbyte_b32 %{c}, %{c}, %{c}, 1",
    "add3": "v_add3_u32 %{c}, %{c}, %16, %18",
    "add3s": "v_add3_u32 %{c}, %{c}, %17, %18",
    "bfe": "v_bfe_u32 %{c}, %{c}, 3, 20",
    "perm": "v_perm_b32 %{c}, %{c}, %16, %18",
    "lshladd": "v_lshl_add_u32 %{c}, %{c}, 3, %16",
    "lshlor": "v_lshl_or_b32 %{c}, %{c}, 3, %16",
    "or3": "v_or3_b32 %{c}, %{c}, %16, %18",
    "mad24": "v_mad_u32_u24 %{c}, %{c}, %16, %18",
    "lshl64": "v_lshlrev_b64 %{c2}, 3, %{c2}",
    "lshr64": "v_lshrrev_b64 %{c2}, 3, %{c2}",
    "fma": "v_fma_f32 %{c}, %{c}, %16, %18",
    "addf": "v_add_f32_e32 %{c}, %{c}, %16",
    "pk_addf": "v_pk_add_f32 %{c2}, %{c2}, %{c2}",
    "nop": "s_nop 0",
}


def seq_single(op):
    return [op] * 64


def seq_group(a, b, na, nb):
    out = []
    while len(out) < 64:
        out += [a] * na + [b] * nb
    return out[:64]


PATTERNS = []
for op in OPS:
    if op == "nop":
        continue
    PATTERNS.append((op, seq_single(op)))
for n in (1, 2, 4, 8, 16, 32):
    PATTERNS.append((f"align{n}+add{n}", seq_group("align", "add", n, n)))
for n in (1, 2, 4, 8, 16):
    PATTERNS.append((f"align{n}+xor{n}", seq_group("align", "xor", n, n)))
    PATTERNS.append((f"align{n}+bitop3_{n}", seq_group("align", "bitop3", n, n)))
    PATTERNS.append((f"add3_{n}+add{n}", seq_group("add3", "add", n, n)))
for (na, nb) in ((1, 3), (3, 1), (6, 10), (4, 8), (1, 7), (2, 14)):
    PATTERNS.append((f"align{na}+add{nb}", seq_group("align", "add", na, nb)))
PATTERNS.append(("bitop3+add alt", seq_group("bitop3", "add", 1, 1)))
PATTERNS.append(("lshr+add alt", seq_group("lshr", "add", 1, 1)))
PATTERNS.append(("lshr+bitop3 alt", seq_group("lshr", "bitop3", 1, 1)))
PATTERNS.append(("adds+add alt", seq_group("adds", "add", 1, 1)))
PATTERNS.append(("align+nop alt", seq_group("align", "nop", 1, 1)))
PATTERNS.append(("add+nop alt", seq_group("add", "nop", 1, 1)))


def render(seq):
    lines = []
    for i, op in enumerate(seq):
        c = i % NCH
        c2 = (i % (NCH // 2)) * 2
        t = OPS[op]
        if "{c2}" in t:
            # 64-bit register pair via the asm operand modifier is not available for
            # separate variables: use the pair of chains c2, c2+1 through explicit names
            t = t.replace("%{c2}", "v[%" + "{lo}:%" + "{hi}]")
        lines.append(t.replace("{c}", str(c)).replace("{c2}", str(c2)))
    return lines


def main():
    here = os.path.dirname(os.path.abspath(__file__))
    kernels = []
    runs = []
    for pid, (name, seq) in enumerate(PATTERNS):
        if any("{c2}" in OPS[o] for o in seq):
            continue  # 64-bit ops need register pairs: handled by the pair kernel below
        body = "\\n\\t".join(render(seq))
        kernels.append(f'template <> __device__ __forceinline__ void body<{pid}>(unsigned* x, unsigned y, unsigned k, unsigned z) {{\n'
                       f'    asm volatile("{body}\\n\\t"\n'
                       '                 : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]),\n'
                       '                   "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15])\n'
                       '                 : "v"(y), "s"(k), "v"(z) : "vcc");\n}\n')
        n_real = sum(1 for o in seq if o != "nop")
        runs.append(f'    run<{pid}>("{name}", {n_real}, wps, d_out, d_clk);')
    src = f'''// GENERATED by tools/gen_valu_mix.py -- do not edit.
// Issue cost of gfx950 VALU instruction sequences (see the generator's docstring).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#define CHECK(x) do {{ hipError_t e = (x); if (e != hipSuccess) {{ fprintf(stderr, "%s: %s\\n", #x, hipGetErrorString(e)); exit(1); }} }} while (0)
constexpr int ITERS = 1024;
template <int P> __device__ __forceinline__ void body(unsigned* x, unsigned y, unsigned k, unsigned z);
{"".join(kernels)}
template <int P>
__global__ __launch_bounds__(256) void mb(unsigned* out, unsigned long long* clk) {{
    unsigned x[16];
    const unsigned y = threadIdx.x * 2654435761u, k = 0x9E3779B9u ^ blockIdx.x, z = threadIdx.x * 40503u + 7u;
#pragma unroll
    for (int i = 0; i < 16; i++) x[i] = threadIdx.x + i;
    unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < ITERS; it++) {{
        body<P>(x, y, k, z);
        body<P>(x, y, k, z);
        body<P>(x, y, k, z);
        body<P>(x, y, k, z);
    }}
    unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    unsigned acc = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) acc ^= x[i];
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
    double cyc = 0, ghz = 0;
    for (int b = 0; b < blocks; b++) {{ cyc += (double)clk[2 * b]; ghz += (double)clk[2 * b] / (double)clk[2 * b + 1] * 0.1; }}
    cyc /= blocks; ghz /= blocks;
    // in-kernel cycles per wave-instruction per SIMD: each wave's own span x waves/SIMD / its instruction count
    const double insts = (double)ITERS * 4 * n_real;
    const double cpi = cyc / insts / wps;   // if the wps waves overlap perfectly
    const double cpi_wall = best * 1e-3 * ghz * 1e9 / (insts * wps);
    printf("{{\\"pattern\\": \\"%s\\", \\"wps\\": %d, \\"ms\\": %.4f, \\"clock_ghz\\": %.3f, \\"cyc_per_inst_inkernel\\": %.3f, \\"cyc_per_inst_wall\\": %.3f}}\\n",
           name, wps, best, ghz, cpi, cpi_wall);
    fflush(stdout);
    CHECK(hipEventDestroy(e0)); CHECK(hipEventDestroy(e1));
}}
int main(int argc, char** argv) {{
    unsigned* d_out; unsigned long long* d_clk;
    CHECK(hipMalloc(&d_out, sizeof(unsigned) * 256 * 16 * 256));
    CHECK(hipMalloc(&d_clk, sizeof(unsigned long long) * 2 * 256 * 16));
    const char* w = getenv("MB_WPS");
    int wlist[4] = {{8, 2, 1, 4}};
    int nw = w ? 1 : 4;
    if (w) wlist[0] = atoi(w);
    for (int wi = 0; wi < nw; wi++) {{
        const int wps = wlist[wi];
{chr(10).join(runs)}
    }}
    return 0;
}}
'''
    with open(os.path.join(here, "valu_mix.hip"), "w") as f:
        f.write(src)
    print(f"wrote {len(runs)} patterns")


if __name__ == "__main__":
    main()
