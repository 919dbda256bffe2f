#!/usr/bin/env python3
"""Generate sha256_rounds_asm.h: the 64 SHA-256 rounds (FIPS 180-4 §6.2.2 step 3)
as hand-scheduled gfx950 VALU assembly, 8 rounds per inline-asm statement.

Why asm: hipcc's scheduler reassociates the message-schedule sums and hoists
partial sums for later rounds, which costs ~40 extra VGPRs (79 for a bare
compression loop, 112 in the full kernel => 4 waves/SIMD, and the kernel is
dependency-stall bound).  Here the register set is exactly a..h (8), the
16-word schedule window (16) and 4 temporaries; register names rotate in the
generator, so there are no moves.

Per round (14 VALU ops; + 10 for a schedule word when j >= 16):
  S1  = alignbit(e,e,6) ^ alignbit(e,e,11) ^ alignbit(e,e,25)   3 + bitop3(0x96)
  ch  = v_bfi_b32(e, f, g)                                      1
  h  += S1 + ch             (v_add3_u32)                        1
  h  += K[j] + W[j]         (v_add3_u32, K in an SGPR)          1
  d  += h                   (t1 -> new e)                       1
  S0  = alignbit(a,a,2) ^ alignbit(a,a,13) ^ alignbit(a,a,22)   3 + bitop3(0x96)
  maj = bitop3(a, b, c, 0xE8)                                   1
  h  += S0 + maj            (new a)                             1
Schedule: W[j] += s1(W[j-2]) + s0(W[j-15]) + W[j-7]   (2 alignbit + 1 shift + bitop3) x 2 + add3 + add

Issue yield after every 4-cycle-class op (rounds_asm): a `s_nop 0` after each
v_alignbit_b32 / v_add3_u32 lets the SIMD's age-ordered VALU arbiter pass to
another wave instead of waiting on this one's next instruction.  Measured on
the pure-register compression loop (tools/compress_bench.hip,
profiles/r01/compress_variants.jsonl): 5,498 -> 5,021 cycles per
wave-compression at 8 waves/SIMD (-8.7 %), 5,562 -> 5,097 at 4; a v_mov_b32
filler gives nearly the same (5,041), two fillers or `s_nop 1` lose, and a
filler after the 2-cycle-class ops loses.

Run:  python gen_rounds_asm.py > sha256_rounds_asm.h
      python gen_rounds_asm.py --ab > ../../tools/sha256_rounds_asm_ab.h   (tools only, not tracked)
"""

K = [
    0x428A2F98, 0x71374491, 0xB5C0FBCF, 0xE9B5DBA5, 0x3956C25B, 0x59F111F1, 0x923F82A4, 0xAB1C5ED5,
    0xD807AA98, 0x12835B01, 0x243185BE, 0x550C7DC3, 0x72BE5D74, 0x80DEB1FE, 0x9BDC06A7, 0xC19BF174,
    0xE49B69C1, 0xEFBE4786, 0x0FC19DC6, 0x240CA1CC, 0x2DE92C6F, 0x4A7484AA, 0x5CB0A9DC, 0x76F988DA,
    0x983E5152, 0xA831C66D, 0xB00327C8, 0xBF597FC7, 0xC6E00BF3, 0xD5A79147, 0x06CA6351, 0x14292967,
    0x27B70A85, 0x2E1B2138, 0x4D2C6DFC, 0x53380D13, 0x650A7354, 0x766A0ABB, 0x81C2C92E, 0x92722C85,
    0xA2BFE8A1, 0xA81A664B, 0xC24B8B70, 0xC76C51A3, 0xD192E819, 0xD6990624, 0xF40E3585, 0x106AA070,
    0x19A4C116, 0x1E376C08, 0x2748774C, 0x34B0BCB5, 0x391C0CB3, 0x4ED8AA4A, 0x5B9CCA4F, 0x682E6FF3,
    0x748F82EE, 0x78A5636F, 0x84C87814, 0x8CC70208, 0x90BEFFFA, 0xA4506CEB, 0xBEF9A3F7, 0xC67178F2,
]

# operand numbering inside one statement
STATE = list(range(0, 8))        # %0..%7   a..h at the block's first round
W = list(range(8, 24))           # %8..%23  W[0..15]
T = list(range(24, 28))          # %24..%27 temporaries (early-clobber outputs)
KOP = list(range(28, 36))        # %28..%35 K[j0..j0+7] in SGPRs


def op(i):
    return f"%{i}"


COMPLEX = ("v_alignbit_b32", "v_add3_u32", "v_bfi_b32")


def yield_after_complex(lines, which=COMPLEX, every=1):
    """An issue-yield s_nop 0 after every `every`-th op whose opcode is in `which`."""
    out, k = [], 0
    for ln in lines:
        out.append(ln)
        if ln.split()[0] in which:
            k += 1
            if k % every == 0:
                out.append("s_nop 0")
    return out


def block(j0, ch_mode="bfi", add_mode="add3", k_mode="sgpr", nops=False):
    """nops: False, True (after every 4-cycle op) or (opcodes, every) for
    A/B yield patterns."""
    """8 rounds from j0.  k_mode: "sgpr" = K[j] as 8 SGPR inputs %28..%35 (the
    compiler hoists all 64 constants out of a block loop: 64 live SGPRs);
    "smov" = K[j] written by s_mov_b32 into ONE scratch SGPR output %28 inside
    the statement, in the slot of the round's first issue-yield s_nop (the
    scalar move yields the VALU slot just like the nop); "lit" = VOP2 literal."""
    rounds = []
    for r in range(8):
        lines = []
        j = j0 + r
        a, b, c, d, e, f, g, h = [op(STATE[(k - r) % 8]) for k in range(8)]
        wj = op(W[j & 15])
        t0, t1, t2, t3 = (op(x) for x in T)
        if j >= 16:
            w2, w7, w15 = op(W[(j - 2) & 15]), op(W[(j - 7) & 15]), op(W[(j - 15) & 15])
            lines += [
                f"v_alignbit_b32 {t0}, {w15}, {w15}, 7",
                f"v_alignbit_b32 {t1}, {w15}, {w15}, 18",
                f"v_lshrrev_b32_e32 {t2}, 3, {w15}",
                f"v_bitop3_b32 {t0}, {t0}, {t1}, {t2} bitop3:0x96",
                f"v_alignbit_b32 {t1}, {w2}, {w2}, 17",
                f"v_alignbit_b32 {t2}, {w2}, {w2}, 19",
                f"v_lshrrev_b32_e32 {t3}, 10, {w2}",
                f"v_bitop3_b32 {t1}, {t1}, {t2}, {t3} bitop3:0x96",
            ]
            if add_mode == "add3":
                lines += [f"v_add3_u32 {wj}, {wj}, {t0}, {t1}", f"v_add_u32_e32 {wj}, {wj}, {w7}"]
            else:
                lines += [f"v_add_u32_e32 {wj}, {wj}, {t0}", f"v_add_u32_e32 {wj}, {wj}, {t1}",
                          f"v_add_u32_e32 {wj}, {wj}, {w7}"]
        lines += [
            f"v_alignbit_b32 {t0}, {e}, {e}, 6",
            f"v_alignbit_b32 {t1}, {e}, {e}, 11",
            f"v_alignbit_b32 {t2}, {e}, {e}, 25",
            f"v_bitop3_b32 {t0}, {t0}, {t1}, {t2} bitop3:0x96",
        ]
        if ch_mode == "bfi":
            lines.append(f"v_bfi_b32 {t1}, {e}, {f}, {g}")
        else:  # Ch(e,f,g) = e ? f : g, truth table 0xCA with src0=0xF0, src1=0xCC, src2=0xAA
            lines.append(f"v_bitop3_b32 {t1}, {e}, {f}, {g} bitop3:0xca")
        if add_mode == "add3":
            lines.append(f"v_add3_u32 {h}, {h}, {t0}, {t1}")
        else:
            lines += [f"v_add_u32_e32 {h}, {h}, {t0}", f"v_add_u32_e32 {h}, {h}, {t1}"]
        if k_mode in ("sgpr", "smov"):
            lines.append(f"v_add3_u32 {h}, {h}, {op(KOP[r]) if k_mode == 'sgpr' else op(KOP[0])}, {wj}")
        else:  # VOP2 with a 32-bit literal: h += K, h += W
            lines += [f"v_add_u32_e32 {h}, 0x{K[j]:08x}, {h}", f"v_add_u32_e32 {h}, {h}, {wj}"]
        lines += [
            f"v_add_u32_e32 {d}, {d}, {h}",
            f"v_alignbit_b32 {t0}, {a}, {a}, 2",
            f"v_alignbit_b32 {t1}, {a}, {a}, 13",
            f"v_alignbit_b32 {t2}, {a}, {a}, 22",
            f"v_bitop3_b32 {t0}, {t0}, {t1}, {t2} bitop3:0x96",
            f"v_bitop3_b32 {t1}, {a}, {b}, {c} bitop3:0xe8",
        ]
        if add_mode == "add3":
            lines.append(f"v_add3_u32 {h}, {h}, {t0}, {t1}")
        else:
            lines += [f"v_add_u32_e32 {h}, {h}, {t0}", f"v_add_u32_e32 {h}, {h}, {t1}"]
        if nops is True:
            lines = yield_after_complex(lines)
        elif nops:
            lines = yield_after_complex(lines, *nops)
        if k_mode == "smov":
            # K[j] into the scratch SGPR: in the slot of the round's first
            # yield with nops (after its first 4-cycle op), else up front.
            mov = f"s_mov_b32 {op(KOP[0])}, 0x{K[j]:08x}"
            if "s_nop 0" in lines:
                lines[lines.index("s_nop 0")] = mov
            else:
                lines.insert(0, mov)
        rounds += lines
    return rounds


def block_ilp(j0):
    """Latency-oriented order for waves that run alone on a SIMD (few long
    chains, e.g. batch digests): h+K+W first, the e- and a-side rotations
    interleaved, and the schedule word W[j+2] woven into round j, so no
    instruction waits on the one right before it."""
    R = [op(24 + i) for i in range(8)]
    Q = [op(32 + i) for i in range(4)]
    kop = lambda r: op(36 + r)
    lines = []
    for r in range(8):
        j = j0 + r
        a, b, c, d, e, f, g, h = [op(STATE[(k - r) % 8]) for k in range(8)]
        wj = op(W[j & 15])
        t = j + 2
        sched = 16 <= t <= 63
        if sched:
            wt, wt2, wt7, wt15 = op(W[t & 15]), op(W[(t - 2) & 15]), op(W[(t - 7) & 15]), op(W[(t - 15) & 15])
        S = lambda ins: lines.append(ins) if sched else None
        lines.append(f"v_add3_u32 {h}, {h}, {kop(r)}, {wj}")
        lines.append(f"v_alignbit_b32 {R[0]}, {e}, {e}, 6")
        if sched: S(f"v_alignbit_b32 {Q[0]}, {wt15}, {wt15}, 7")
        lines.append(f"v_alignbit_b32 {R[1]}, {e}, {e}, 11")
        if sched: S(f"v_alignbit_b32 {Q[1]}, {wt15}, {wt15}, 18")
        lines.append(f"v_alignbit_b32 {R[2]}, {e}, {e}, 25")
        if sched: S(f"v_lshrrev_b32_e32 {Q[2]}, 3, {wt15}")
        lines.append(f"v_bitop3_b32 {R[3]}, {e}, {f}, {g} bitop3:0xca")
        lines.append(f"v_alignbit_b32 {R[4]}, {a}, {a}, 2")
        if sched: S(f"v_bitop3_b32 {Q[0]}, {Q[0]}, {Q[1]}, {Q[2]} bitop3:0x96")
        lines.append(f"v_bitop3_b32 {R[0]}, {R[0]}, {R[1]}, {R[2]} bitop3:0x96")
        lines.append(f"v_alignbit_b32 {R[5]}, {a}, {a}, 13")
        if sched: S(f"v_alignbit_b32 {Q[1]}, {wt2}, {wt2}, 17")
        lines.append(f"v_add3_u32 {h}, {h}, {R[0]}, {R[3]}")
        lines.append(f"v_alignbit_b32 {R[6]}, {a}, {a}, 22")
        if sched: S(f"v_alignbit_b32 {Q[2]}, {wt2}, {wt2}, 19")
        lines.append(f"v_add_u32_e32 {d}, {d}, {h}")
        lines.append(f"v_bitop3_b32 {R[7]}, {a}, {b}, {c} bitop3:0xe8")
        if sched: S(f"v_lshrrev_b32_e32 {Q[3]}, 10, {wt2}")
        lines.append(f"v_bitop3_b32 {R[4]}, {R[4]}, {R[5]}, {R[6]} bitop3:0x96")
        if sched: S(f"v_bitop3_b32 {Q[1]}, {Q[1]}, {Q[2]}, {Q[3]} bitop3:0x96")
        lines.append(f"v_add3_u32 {h}, {h}, {R[4]}, {R[7]}")
        if sched:
            S(f"v_add3_u32 {wt}, {wt}, {Q[0]}, {Q[1]}")
            S(f"v_add_u32_e32 {wt}, {wt}, {wt7}")
    return lines


def emit_fn_ilp(name):
    out = [f"__device__ __forceinline__ void {name}(uint32_t s[8], uint32_t w[16]) {{",
           "    uint32_t r0, r1, r2, r3, r4, r5, r6, r7, q0, q1, q2, q3;"]
    for j0 in range(0, 64, 8):
        body = block_ilp(j0)
        out.append(f"    // rounds {j0}..{j0 + 7} (W[{j0 + 2}..{j0 + 9}] scheduled inside)")
        out.append("    asm volatile(")
        for ln in body:
            out.append(f'        "{ln}\\n\\t"')
        outs = ", ".join([f'"+v"(s[{i}])' for i in range(8)] + [f'"+v"(w[{i}])' for i in range(16)]
                         + [f'"=&v"(r{i})' for i in range(8)] + [f'"=&v"(q{i})' for i in range(4)])
        ins = ", ".join(f'"s"(0x{K[j0 + r]:08X}u)' for r in range(8))
        out.append(f"        : {outs}")
        out.append(f"        : {ins});")
    out.append("}")
    out.append("")
    return out


def block_kw():
    """Consumer rounds of the producer/consumer pair kernels: 8 rounds whose
    K[j] + W[j] arrive precomputed (%14..%21, from the producer wave through
    LDS), so no message schedule here: 14 instructions per round, ordered
    for a lone wave (h += KW first, the e- and a-side rotations interleaved)."""
    T = [op(8 + i) for i in range(6)]
    lines = []
    for r in range(8):
        a, b, c, d, e, f, g, h = [op((k - r) % 8) for k in range(8)]
        kw = op(14 + r)
        lines += [
            f"v_add_u32_e32 {h}, {h}, {kw}",
            f"v_alignbit_b32 {T[0]}, {e}, {e}, 6",
            f"v_alignbit_b32 {T[3]}, {a}, {a}, 2",
            f"v_alignbit_b32 {T[1]}, {e}, {e}, 11",
            f"v_alignbit_b32 {T[4]}, {a}, {a}, 13",
            f"v_alignbit_b32 {T[2]}, {e}, {e}, 25",
            f"v_alignbit_b32 {T[5]}, {a}, {a}, 22",
            f"v_bitop3_b32 {T[0]}, {T[0]}, {T[1]}, {T[2]} bitop3:0x96",
            f"v_bitop3_b32 {T[1]}, {e}, {f}, {g} bitop3:0xca",
            f"v_bitop3_b32 {T[3]}, {T[3]}, {T[4]}, {T[5]} bitop3:0x96",
            f"v_bitop3_b32 {T[4]}, {a}, {b}, {c} bitop3:0xe8",
            f"v_add3_u32 {h}, {h}, {T[0]}, {T[1]}",
            f"v_add_u32_e32 {d}, {d}, {h}",
            f"v_add3_u32 {h}, {h}, {T[3]}, {T[4]}",
        ]
    return lines


def tail_round(j):
    """Round j of a FINAL block whose words 4..15 are wave-uniform constants:
    W4 = c4 (0x80000000 when the block holds exactly 16 message bytes, else 0),
    W5..W13 = 0, W14 = c14, W15 = c15 (the 64-bit bit length).  Only W0..W3
    come from the message.  Constant terms of the schedule arrive summed in
    SGPRs (cs16 = s1(c14), cs17 = s1(c15), cs19 = s0(c4), cs29 = s0(c14),
    cs30 = s0(c15) + c14) and the rounds 4..15 add K[j] + W[j] as one scalar
    (kw4, kw14, kw15, or K[j] itself): 89 instead of 160 schedule ops and 12
    two-input adds instead of v_add3.  Named operands (%[x])."""
    a, b, c, d, e, f, g, h = [f"%[s{(k - j) % 8}]" for k in range(8)]
    W = lambda i: f"%[w{i & 15}]"
    t0, t1, t2, t3 = "%[t0]", "%[t1]", "%[t2]", "%[t3]"
    s0 = lambda x: [f"v_alignbit_b32 {t0}, {x}, {x}, 7", f"v_alignbit_b32 {t1}, {x}, {x}, 18",
                    f"v_lshrrev_b32_e32 {t2}, 3, {x}", f"v_bitop3_b32 {t0}, {t0}, {t1}, {t2} bitop3:0x96"]
    s1 = lambda x: [f"v_alignbit_b32 {t1}, {x}, {x}, 17", f"v_alignbit_b32 {t2}, {x}, {x}, 19",
                    f"v_lshrrev_b32_e32 {t3}, 10, {x}", f"v_bitop3_b32 {t1}, {t1}, {t2}, {t3} bitop3:0x96"]
    wj = W(j)
    lines = []
    if j == 16:
        lines += s0(W(1)) + [f"v_add3_u32 {wj}, {wj}, {t0}, %[cs16]"]
    elif j == 17:
        lines += s0(W(2)) + [f"v_add3_u32 {wj}, {wj}, {t0}, %[cs17]"]
    elif j == 18:  # + W11 = 0
        lines += s0(W(3)) + s1(W(16)) + [f"v_add3_u32 {wj}, {wj}, {t0}, {t1}"]
    elif j == 19:  # + W12 = 0, s0(W4) = cs19
        lines += s1(W(17)) + [f"v_add3_u32 {wj}, {wj}, {t1}, %[cs19]"]
    elif j in (20, 21, 22):  # s1(W[j-2]) + W4 / W14 / W15 (the other terms are zero)
        lines += s1(W(j - 2)) + [f"v_add_u32_e32 {wj}, %[{('c4', 'c14', 'c15')[j - 20]}], {t1}"]
    elif 23 <= j <= 28:  # s1(W[j-2]) + W[j-7]
        lines += s1(W(j - 2)) + [f"v_add_u32_e32 {wj}, {W(j - 7)}, {t1}"]
    elif j in (29, 30):  # + s0(W14) / s0(W15) + W14
        lines += s1(W(j - 2)) + [f"v_add3_u32 {wj}, {W(j - 7)}, {t1}, %[cs{j}]"]
    elif j == 31:  # s1(W29) + W24 + s0(W16) + W15
        lines += s0(W(16)) + s1(W(29)) + [f"v_add3_u32 {wj}, {W(24)}, {t0}, {t1}",
                                            f"v_add_u32_e32 {wj}, %[c15], {wj}"]
    lines += [
        f"v_alignbit_b32 {t0}, {e}, {e}, 6",
        f"v_alignbit_b32 {t1}, {e}, {e}, 11",
        f"v_alignbit_b32 {t2}, {e}, {e}, 25",
        f"v_bitop3_b32 {t0}, {t0}, {t1}, {t2} bitop3:0x96",
        f"v_bitop3_b32 {t1}, {e}, {f}, {g} bitop3:0xca",
        f"v_add3_u32 {h}, {h}, {t0}, {t1}",
    ]
    kmov = None
    if j < 4 or j >= 16:
        lines.append(f"v_add3_u32 {h}, {h}, %[kt], {wj}")
        kmov = f"s_mov_b32 %[kt], 0x{K[j]:08x}"
    elif j in (4, 14, 15):
        lines.append(f"v_add_u32_e32 {h}, %[kw{j}], {h}")
    else:  # W[j] = 0
        lines.append(f"v_add_u32_e32 {h}, %[kt], {h}")
        kmov = f"s_mov_b32 %[kt], 0x{K[j]:08x}"
    lines += [
        f"v_add_u32_e32 {d}, {d}, {h}",
        f"v_alignbit_b32 {t0}, {a}, {a}, 2",
        f"v_alignbit_b32 {t1}, {a}, {a}, 13",
        f"v_alignbit_b32 {t2}, {a}, {a}, 22",
        f"v_bitop3_b32 {t0}, {t0}, {t1}, {t2} bitop3:0x96",
        f"v_bitop3_b32 {t1}, {a}, {b}, {c} bitop3:0xe8",
        f"v_add3_u32 {h}, {h}, {t0}, {t1}",
    ]
    lines = yield_after_complex(lines, *TAIL_YIELD) if TAIL_YIELD else lines
    if kmov:
        if "s_nop 0" in lines:
            lines[lines.index("s_nop 0")] = kmov
        else:
            lines.insert(0, kmov)
    return lines


# issue-yield pattern of the tail form (the product's: after every second
# 4-cycle op); set_yield() changes it together with rounds_asm's (A/B builds).
TAIL_YIELD = (COMPLEX, 2)

# statements of the tail form: (first round, end round); the window words each
# one touches are derived from its text (at most 29 operands per statement)
TAIL_STATEMENTS = [(0, 8), (8, 16), (16, 24), (24, 28), (28, 32)]
TAIL_SCALARS = ["kw4", "kw14", "kw15", "c4", "c14", "c15", "cs16", "cs17", "cs19", "cs29", "cs30"]


def emit_fn_tail(name, normal_variant):
    ch, ad, km, nops = VARIANTS[normal_variant]
    out = ["template <class H = NoHook>",
           f"__device__ __forceinline__ void {name}(uint32_t s[8], uint32_t w[16], const TailWords& k, H hook = {{}}) {{",
           "    uint32_t t0, t1, t2, t3; uint32_t kt;"]
    stmt = 0
    import re
    defined = {f"w{i}" for i in range(4)}  # window words 4..15 are first WRITTEN (W20..W31)
    for j0, j1 in TAIL_STATEMENTS:
        if stmt:
            out.append(f"    hook({stmt - 1});")
        stmt += 1
        body = []
        for j in range(j0, j1):
            body += tail_round(j)
        text = "\n".join(body)
        used = set(re.findall(r"%\[(\w+)\]", text))
        fresh = set()  # words whose first access in this statement is a write: "=&v"
        for ln in body:
            names = re.findall(r"%\[(w\d+)\]", ln)
            for k, nm in enumerate(names):
                if nm in defined or nm in fresh:
                    continue
                assert k == 0 and ln.split(None, 1)[1].startswith(f"%[{nm}]"), f"{nm} read before written"
                fresh.add(nm)
        defined |= fresh
        out.append(f"    // rounds {j0}..{j1 - 1} (final-block form)")
        out.append("    asm volatile(")
        for ln in body:
            out.append(f'        "{ln}\\n\\t"')
        outs = [f'[s{i}] "+v"(s[{i}])' for i in range(8)]
        outs += [f'[w{i}] "{"=&v" if f"w{i}" in fresh else "+v"}"(w[{i}])' for i in range(16) if f"w{i}" in used]
        outs += [f'[t{i}] "=&v"(t{i})' for i in range(4) if f"t{i}" in used]
        if "kt" in used:
            outs.append('[kt] "=&s"(kt)')
        ins = [f'[{x}] "s"(k.{x})' for x in TAIL_SCALARS if x in used]
        out.append(f"        : {', '.join(outs)}")
        out.append(f"        : {', '.join(ins)});")
    # rounds 32..63: the ordinary statements (every window word is live)
    for j0 in range(32, 64, 8):
        out.append(f"    hook({stmt - 1});")
        stmt += 1
        body = block(j0, ch, ad, km, nops)
        out.append(f"    // rounds {j0}..{j0 + 7}")
        out.append("    asm volatile(")
        for ln in body:
            out.append(f'        "{ln}\\n\\t"')
        outs = ", ".join([f'"+v"(s[{i}])' for i in range(8)] + [f'"+v"(w[{i}])' for i in range(16)]
                         + ['"=&v"(t0)', '"=&v"(t1)', '"=&v"(t2)', '"=&v"(t3)', '"=&s"(kt)'])
        out.append(f"        : {outs}")
        out.append("        : );")
    out.append("}")
    out.append("")
    return out


def emit_fn_kw(name):
    out = [f"__device__ __forceinline__ void {name}(uint32_t s[8], uint4 k0, uint4 k1) {{",
           "    uint32_t t0, t1, t2, t3, t4, t5;",
           "    asm volatile("]
    for ln in block_kw():
        out.append(f'        "{ln}\\n\\t"')
    outs = ", ".join([f'"+v"(s[{i}])' for i in range(8)] + [f'"=&v"(t{i})' for i in range(6)])
    ins = ", ".join(f'"v"({v})' for v in ("k0.x", "k0.y", "k0.z", "k0.w", "k1.x", "k1.y", "k1.z", "k1.w"))
    out.append(f"        : {outs}")
    out.append(f"        : {ins});")
    out.append("}")
    out.append("")
    return out


# Product forms (sha256_rounds_asm.h): the request kernel's yield form and
# the latency form of the lone-wave chains.
VARIANTS = {
    # name: (ch_mode, add_mode, k_mode, nops)
    # request-kernel form: a yield after every SECOND 4-cycle op (the register
    # loop alone prefers one after every op, 5,021 vs 5,090 cycles per
    # wave-compression, but in the request kernel -- memory stalls, progress
    # priorities -- every second one measured 187.8-188.1 vs 189.1-189.5 us per
    # config-2 launch on two boxes, profiles/r02y)
    "rounds_asm": ("bitop3", "add3", "smov", (COMPLEX, 2)),
    "rounds_asm_nonop": ("bitop3", "add3", "sgpr", False),
}
# A/B forms for tools/ only (tools/sha256_rounds_asm_ab.h), bit-identical.
AB_VARIANTS = {
    "rounds_asm_ksgpr": ("bitop3", "add3", "sgpr", True),
    # yield patterns (A/B against the product's "after every second 4-cycle op")
    "rounds_asm_y_every": ("bitop3", "add3", "smov", True),  # the round-1/2 product form
    "rounds_asm_y_rot": ("bitop3", "add3", "smov", (("v_alignbit_b32",), 1)),
    "rounds_asm_y_add3": ("bitop3", "add3", "smov", (("v_add3_u32",), 1)),
    "rounds_asm_y_third": ("bitop3", "add3", "smov", (COMPLEX, 3)),
    "rounds_asm_y_quarter": ("bitop3", "add3", "smov", (COMPLEX, 4)),
    "rounds_asm_y_rothalf": ("bitop3", "add3", "smov", (("v_alignbit_b32",), 2)),
    "rounds_asm_bfi": ("bfi", "add3", "sgpr", False),
    "rounds_asm_add2": ("bitop3", "add", "sgpr", False),
    "rounds_asm_lit": ("bitop3", "add3", "lit", False),
    "rounds_asm_add2lit": ("bitop3", "add", "lit", False),
}


# --yield forms for A/B builds of the whole library (tools/yield_sweep.sh):
# the request kernels' issue-yield density at 4 waves per SIMD.
YIELD_FORMS = {
    "1": (COMPLEX, 1), "2": (COMPLEX, 2), "3": (COMPLEX, 3), "4": (COMPLEX, 4),
    "rot": (("v_alignbit_b32",), 1), "rot2": (("v_alignbit_b32",), 2), "none": False,
}


def set_yield(form):
    global TAIL_YIELD
    y = YIELD_FORMS[form]
    ch, ad, km, _ = VARIANTS["rounds_asm"]
    VARIANTS["rounds_asm"] = (ch, ad, km, y)
    TAIL_YIELD = y


def emit_fn(name, ch_mode, add_mode, k_mode, nops, rounds=(0, 64)):
    out = ["template <class H = NoHook>",
           f"__device__ __forceinline__ void {name}(uint32_t s[8], uint32_t w[16], H hook = {{}}) {{",
           "    uint32_t t0, t1, t2, t3;" + (" uint32_t kt;" if k_mode == "smov" else "")]
    for j0 in range(rounds[0], rounds[1], 8):
        if j0 != rounds[0]:
            out.append(f"    hook({(j0 - rounds[0]) // 8 - 1});")
        body = block(j0, ch_mode, add_mode, k_mode, nops)
        out.append(f"    // rounds {j0}..{j0 + 7}")
        out.append("    asm volatile(")
        for ln in body:
            out.append(f'        "{ln}\\n\\t"')
        outs = ", ".join([f'"+v"(s[{i}])' for i in range(8)] + [f'"+v"(w[{i}])' for i in range(16)]
                         + ['"=&v"(t0)', '"=&v"(t1)', '"=&v"(t2)', '"=&v"(t3)']
                         + (['"=&s"(kt)'] if k_mode == "smov" else []))
        if k_mode == "sgpr":
            ins = ", ".join(f'"s"(0x{K[j0 + r]:08X}u)' for r in range(8))
        else:
            ins = ""
        out.append(f"        : {outs}")
        out.append(f"        : {ins});")
    out.append("}")
    out.append("")
    return out


HEADER = [
    "// GENERATED by mirbft_amd/csrc/gen_rounds_asm.py — do not edit by hand.",
    "// 64 SHA-256 rounds (FIPS 180-4 §6.2.2) for gfx950, 8 per asm statement.",
]


def emit():
    out = HEADER + [
        "// rounds_asm: throughput form (issue-yield s_nop after each 4-cycle op, K[j]",
        "// by s_mov_b32 into one scratch SGPR in a yield slot, so no constants stay",
        "// live across a block loop); rounds_asm_nonop: latency form (lone waves).",
        "#pragma once",
        "#include <stdint.h>",
        "",
        "namespace mirsha {",
        "",
        "// s[0..7] = working variables a..h (updated in place: after 8 rounds the",
        "// names have rotated back), w[0..15] = schedule window (consumed).",
        "// hook(k) runs between asm statements k and k + 1 (k = 0, 1, ...): a caller",
        "// interleaves other work (e.g. staging the next block) with the rounds.",
        "struct NoHook {",
        "    __device__ __forceinline__ void operator()(int) const {}",
        "};",
        "#define MIRSHA_NOHOOK_DEFINED",
        "",
    ]
    for name, (ch, ad, km, nops) in VARIANTS.items():
        out += emit_fn(name, ch, ad, km, nops)
    out += [
        "// Wave-uniform constants of a final block whose words 4..15 are padding",
        "// (rounds_asm_tail; filled by tail_words() in sha256_device.h).",
        "struct TailWords {",
        "    uint32_t " + ", ".join(TAIL_SCALARS) + ";",
        "};",
        "// rounds_asm for a final block with only W0..W3 from the message (same",
        "// yield pattern): the schedule's constant terms and K[j] + W[j] of rounds",
        "// 4..15 are scalars (71 fewer schedule ops; 12 v_add3 become v_add).",
    ]
    out += emit_fn_tail("rounds_asm_tail", "rounds_asm")
    out.append("// 8 consumer rounds with K + W precomputed (pair kernels): names rotate")
    out.append("// back after 8 rounds, so the same statement serves every 8-round chunk.")
    out += emit_fn_kw("rounds_kw8_asm")
    out.append("}  // namespace mirsha")
    return "\n".join(out) + "\n"


def emit_ab():
    out = HEADER + [
        "// A/B timing forms for tools/ (valu_microbench.hip), bit-identical to the",
        "// product forms in mirbft_amd/csrc/sha256_rounds_asm.h.",
        "#pragma once",
        "#include <stdint.h>",
        "",
        "namespace mirsha {",
        "",
        "#ifndef MIRSHA_NOHOOK_DEFINED",
        "struct NoHook {",
        "    __device__ __forceinline__ void operator()(int) const {}",
        "};",
        "#endif",
        "",
    ]
    for name, (ch, ad, km, nops) in AB_VARIANTS.items():
        out += emit_fn(name, ch, ad, km, nops)
    out.append("// Latency-oriented order (lone waves): same instructions, 12 temporaries.")
    out += emit_fn_ilp("rounds_asm_ilp")
    out.append("}  // namespace mirsha")
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    import sys

    if "--yield" in sys.argv:  # A/B builds only; the product header is the default form
        set_yield(sys.argv[sys.argv.index("--yield") + 1])
    sys.stdout.write(emit_ab() if "--ab" in sys.argv else emit())
