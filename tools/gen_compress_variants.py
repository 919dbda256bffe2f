#!/usr/bin/env python3
"""Generates tools/compress_variants.h: whole-compression A/B forms of the 64
SHA-256 rounds for tools/compress_bench.hip.

Question under test: in a mixed stream on gfx950, the 2-cycle-class VALU ops
(v_add_u32, v_bitop3_b32, v_lshrrev_b32, v_mov_b32) cost ~4 cycles each, like
the 4-cycle class (v_alignbit_b32, v_add3_u32, v_lshlrev_b32) -- but
tools/rot_bench showed "align+add+mov" at 6.4 cycles per repeat against 8.0
for "align+add", i.e. a v_mov_b32 between a simple and a complex op removes
the penalty.  These variants insert moves (or s_nop) at the measured
transitions, or regroup each round (rotates first, then the simple ops), and
time the compression end to end at 8 and 4 waves per SIMD.

All forms compute the same compression (the bench checks every output word
against the production form).

Usage: python tools/gen_compress_variants.py > tools/compress_variants.h
"""
import os
import re
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "mirbft_amd", "csrc"))
import gen_rounds_asm as g  # noqa: E402

COMPLEX = ("v_alignbit_b32", "v_add3_u32", "v_bfi_b32", "v_lshlrev_b32", "v_perm_b32")
SIMPLE = ("v_add_u32_e32", "v_bitop3_b32", "v_lshrrev_b32_e32", "v_xor_b32_e32")

# operand map for every variant: %0..%7 state, %8..%23 W, %24..%35 temps,
# %36 dummy mov target, %37 mov source (never written), %38..%45 K (SGPR)
NT = 12
DM, DS = 36, 37
K0 = 38


def cls(ins):
    m = ins.split()[0]
    if m.startswith("v_mov"):
        return "M"
    if m.startswith("s_"):
        return "N"
    if m in COMPLEX:
        return "C"
    if m in SIMPLE:
        return "S"
    raise ValueError(ins)


def remap_base(lines, kfirst=28):
    """gen_rounds_asm numbers K from %28 (block) or %36 (block_ilp); move them to K0.."""
    def f(m):
        i = int(m.group(1))
        return f"%{K0 + i - kfirst}" if kfirst <= i <= kfirst + 7 else f"%{i}"
    return [re.sub(r"%(\d+)", f, ln) for ln in lines]


MOV = f"v_mov_b32_e32 %{DM}, %{DS}"
SNOP_ = "s_nop 0"


def insert(lines, where, filler=MOV, n=1):
    out = []
    for i, ln in enumerate(lines):
        c = cls(ln)
        prev = cls(out[-1]) if out else None
        if where == "SC" and c == "C" and prev == "S":
            out += [filler] * n
        out.append(ln)
        if where == "afterC" and c == "C":
            out += [filler] * n
        if where == "afterS" and c == "S":
            out += [filler] * n
        if where == "all":
            out += [filler] * n
    return out


def operands(ins):
    parts = ins.split(None, 1)[1].replace(",", " ").split()
    return parts[0], [x for x in parts[1:] if x.startswith("%")]


def insert_cond(lines, pred, filler=SNOP_):
    """filler after instruction i when pred(lines[i], lines[i+1]) holds."""
    out = []
    for i, ln in enumerate(lines):
        out.append(ln)
        nxt = lines[i + 1] if i + 1 < len(lines) else None
        if nxt is not None and pred(ln, nxt):
            out.append(filler)
    return out


def c_then_dep(a, b):
    return cls(a) == "C" and operands(a)[0] in operands(b)[1]


def c_then_indep(a, b):
    return cls(a) == "C" and operands(a)[0] not in operands(b)[1]


def c_then_s(a, b):
    return cls(a) == "C" and cls(b) == "S"


def c_then_c(a, b):
    return cls(a) == "C" and cls(b) == "C"


def any_then_dep(a, b):
    return operands(a)[0] in operands(b)[1]


def insert_after(lines, mnemonics, filler):
    out = []
    for ln in lines:
        out.append(ln)
        if ln.split()[0] in mnemonics:
            out.append(filler)
    return out


def interleave_cs(lines):
    """Greedy reorder inside one block: after a complex op prefer an
    independent simple op whose inputs are ready (dependencies respected)."""
    remaining = list(lines)
    out = []
    written = {}
    def deps(ln):
        d, srcs = operands(ln)
        return d, srcs
    while remaining:
        # candidates: instructions with no unsatisfied dependency on earlier remaining ones
        pick = None
        last_c = bool(out) and cls(out[-1]) == "C"
        for i, ln in enumerate(remaining):
            d, srcs = deps(ln)
            blocked = False
            for prev in remaining[:i]:
                pd, ps = deps(prev)
                if pd in srcs or d in ps or pd == d:
                    blocked = True
                    break
            if blocked:
                continue
            if pick is None:
                pick = i
            if last_c and cls(ln) == "S":
                pick = i
                break
            if not last_c:
                break
        out.append(remaining.pop(pick))
    return out


def ilp_block(j0):
    return remap_base(g.block_ilp(j0), kfirst=36)


def grouped_block(j0, plain_adds, sc_mov):
    """Rotates first, then the simple ops.  plain_adds: K as a literal and
    every sum as v_add_u32 (all simple); else add3 with K in an SGPR."""
    op = g.op
    T = [op(24 + i) for i in range(NT)]
    lines = []
    for r in range(8):
        j = j0 + r
        a, b, c, d, e, f, gg, h = [op(g.STATE[(k - r) % 8]) for k in range(8)]
        wj = op(g.W[j & 15])
        if j >= 16:
            w2, w7, w15 = op(g.W[(j - 2) & 15]), op(g.W[(j - 7) & 15]), op(g.W[(j - 15) & 15])
            lines += [
                f"v_alignbit_b32 {T[0]}, {w15}, {w15}, 7",
                f"v_alignbit_b32 {T[1]}, {w15}, {w15}, 18",
                f"v_alignbit_b32 {T[2]}, {w2}, {w2}, 17",
                f"v_alignbit_b32 {T[3]}, {w2}, {w2}, 19",
                f"v_lshrrev_b32_e32 {T[4]}, 3, {w15}",
                f"v_lshrrev_b32_e32 {T[5]}, 10, {w2}",
                f"v_bitop3_b32 {T[0]}, {T[0]}, {T[1]}, {T[4]} bitop3:0x96",
                f"v_bitop3_b32 {T[2]}, {T[2]}, {T[3]}, {T[5]} bitop3:0x96",
            ]
            if plain_adds:
                lines += [f"v_add_u32_e32 {wj}, {wj}, {T[0]}", f"v_add_u32_e32 {wj}, {wj}, {T[2]}",
                          f"v_add_u32_e32 {wj}, {wj}, {w7}"]
            else:
                lines += [f"v_add_u32_e32 {wj}, {wj}, {w7}", f"v_add3_u32 {wj}, {wj}, {T[0]}, {T[2]}"]
        lines += [
            f"v_alignbit_b32 {T[0]}, {e}, {e}, 6",
            f"v_alignbit_b32 {T[1]}, {e}, {e}, 11",
            f"v_alignbit_b32 {T[2]}, {e}, {e}, 25",
            f"v_alignbit_b32 {T[3]}, {a}, {a}, 2",
            f"v_alignbit_b32 {T[4]}, {a}, {a}, 13",
            f"v_alignbit_b32 {T[5]}, {a}, {a}, 22",
        ]
        if not plain_adds:
            lines.append(f"v_add3_u32 {h}, {h}, %{K0 + r}, {wj}")
        lines += [
            f"v_bitop3_b32 {T[0]}, {T[0]}, {T[1]}, {T[2]} bitop3:0x96",
            f"v_bitop3_b32 {T[1]}, {e}, {f}, {gg} bitop3:0xca",
            f"v_bitop3_b32 {T[3]}, {T[3]}, {T[4]}, {T[5]} bitop3:0x96",
            f"v_bitop3_b32 {T[4]}, {a}, {b}, {c} bitop3:0xe8",
        ]
        if plain_adds:
            lines += [
                f"v_add_u32_e32 {h}, 0x{g.K[j]:08x}, {h}",
                f"v_add_u32_e32 {h}, {h}, {wj}",
                f"v_add_u32_e32 {h}, {h}, {T[0]}",
                f"v_add_u32_e32 {h}, {h}, {T[1]}",
                f"v_add_u32_e32 {d}, {d}, {h}",
                f"v_add_u32_e32 {h}, {h}, {T[3]}",
                f"v_add_u32_e32 {h}, {h}, {T[4]}",
            ]
        else:
            lines += [
                f"v_add3_u32 {h}, {h}, {T[0]}, {T[1]}",
                f"v_add_u32_e32 {d}, {d}, {h}",
                f"v_add3_u32 {h}, {h}, {T[3]}, {T[4]}",
            ]
    if sc_mov:
        lines = insert(lines, "SC")
    return lines


def base_block(j0):
    return remap_base(g.block(j0, "bitop3", "add3", "sgpr"))


SNOP = "s_nop 0"

VARIANTS = [
    ("base", lambda j0: base_block(j0)),
    ("snop_after_align", lambda j0: insert_after(base_block(j0), ("v_alignbit_b32",), SNOP)),
    ("snop_after_add3", lambda j0: insert_after(base_block(j0), ("v_add3_u32",), SNOP)),
    ("sleep0_after_c", lambda j0: insert(base_block(j0), "afterC", "s_sleep 0")),
    ("setprio_after_c", lambda j0: insert(base_block(j0), "afterC", "s_setprio 0")),
    ("interleave_snop_after_c", lambda j0: insert(interleave_cs(base_block(j0)), "afterC", SNOP)),
    ("interleave", lambda j0: interleave_cs(base_block(j0))),
    ("snop_after_c", lambda j0: insert(base_block(j0), "afterC", SNOP)),
    ("snop1_after_c", lambda j0: insert(base_block(j0), "afterC", "s_nop 1")),
    ("snop_c_dep", lambda j0: insert_cond(base_block(j0), c_then_dep)),
    ("snop_c_indep", lambda j0: insert_cond(base_block(j0), c_then_indep)),
    ("snop_c_s", lambda j0: insert_cond(base_block(j0), c_then_s)),
    ("snop_c_c", lambda j0: insert_cond(base_block(j0), c_then_c)),
    ("snop_any_dep", lambda j0: insert_cond(base_block(j0), any_then_dep)),
    ("snop_after_c_sc", lambda j0: insert(insert(base_block(j0), "afterC", SNOP), "SC", SNOP)),
    ("ilp_snop_after_c", lambda j0: insert(ilp_block(j0), "afterC", SNOP)),
    ("grouped_snop_after_c", lambda j0: insert(grouped_block(j0, False, False), "afterC", SNOP)),
    ("grouped_adds_snop_after_c", lambda j0: insert(grouped_block(j0, True, False), "afterC", SNOP)),
    ("ilp", lambda j0: ilp_block(j0)),
    ("ilp_mov_after_c", lambda j0: insert(ilp_block(j0), "afterC")),
    ("grouped_mov_after_c", lambda j0: insert(grouped_block(j0, False, False), "afterC")),
    ("grouped_adds_mov_after_c", lambda j0: insert(grouped_block(j0, True, False), "afterC")),
    ("mov_sc", lambda j0: insert(base_block(j0), "SC")),
    ("mov_after_c", lambda j0: insert(base_block(j0), "afterC")),
    ("snop_sc", lambda j0: insert(base_block(j0), "SC", "s_nop 0")),
]


def emit_fn(name, gen):
    out = [f"__device__ __forceinline__ void cv_{name}(uint32_t s[8], uint32_t w[16], uint32_t& dm, uint32_t ds) {{",
           "    uint32_t " + ", ".join(f"t{i}" for i in range(NT)) + ";"]
    counts = {"C": 0, "S": 0, "M": 0, "N": 0}
    for j0 in range(0, 64, 8):
        body = gen(j0)
        for ln in body:
            counts[cls(ln)] += 1
        out.append("    asm volatile(")
        for ln in body:
            out.append(f'        "{ln}\\n\\t"')
        outs = ", ".join([f'"+v"(s[{i}])' for i in range(8)] + [f'"+v"(w[{i}])' for i in range(16)]
                         + [f'"=&v"(t{i})' for i in range(NT)] + ['"+v"(dm)'])
        ins = ", ".join(['"v"(ds)'] + [f'"s"(0x{g.K[j0 + r]:08X}u)' for r in range(8)])
        out.append(f"        : {outs}")
        out.append(f"        : {ins});")
    out.append("}")
    return out, counts


def main():
    out = ["// GENERATED by tools/gen_compress_variants.py -- do not edit.", "#pragma once", "#include <stdint.h>", ""]
    names = []
    for name, gen in VARIANTS:
        fn, counts = emit_fn(name, gen)
        out.append(f"// {name}: per compression C={counts['C']} S={counts['S']} mov={counts['M']} nop={counts['N']}")
        out += fn
        out.append("")
        names.append(name)
    out.append(f"#define CV_COUNT {len(names)}")
    out.append("static const char* kCvNames[] = {" + ", ".join(f'"{n}"' for n in names) + "};")
    out.append("template <int V> __device__ __forceinline__ void cv_run(uint32_t s[8], uint32_t w[16], uint32_t& dm, uint32_t ds) {")
    for i, n in enumerate(names):
        out.append(f"    if constexpr (V == {i}) cv_{n}(s, w, dm, ds);")
    out.append("}")
    sys.stdout.write("\n".join(out) + "\n")


if __name__ == "__main__":
    main()
