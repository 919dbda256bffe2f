"""CPU check of the generated gfx950 round assembly (mirbft_amd/csrc/
sha256_rounds_asm.h): a small interpreter for the handful of VALU/SALU opcodes
the generator emits runs every product round function on random states and
blocks and compares with a pure-Python FIPS 180-4 compression (the primitive of
Go's crypto/sha256 behind the reference's Hasher, processor.go:21, :133-143).

This pins the instruction text itself, register rotation and operand binding
included, without a GPU; the -m gpu suite checks the compiled kernels.
"""
from __future__ import annotations

import os
import random
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "mirbft_amd", "csrc", "sha256_rounds_asm.h")
M = 0xFFFFFFFF

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


def rotr(x, n):
    return ((x >> n) | (x << (32 - n))) & M


def s0(x):
    return rotr(x, 7) ^ rotr(x, 18) ^ (x >> 3)


def s1(x):
    return rotr(x, 17) ^ rotr(x, 19) ^ (x >> 10)


def ref_rounds(s, w):
    """The 64 rounds on working state s (a..h) and block words w (no feed-forward)."""
    w = list(w)
    for j in range(16, 64):
        w.append((s1(w[j - 2]) + w[j - 7] + s0(w[j - 15]) + w[j - 16]) & M)
    a, b, c, d, e, f, g, h = s
    for j in range(64):
        t1 = (h + (rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25)) + ((e & f) ^ (~e & g)) + K[j] + w[j]) & M
        t2 = ((rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22)) + ((a & b) ^ (a & c) ^ (b & c))) & M
        a, b, c, d, e, f, g, h = (t1 + t2) & M, a, b, c, (d + t1) & M, e, f, g
    return [a, b, c, d, e, f, g, h]


# ---- a tiny interpreter ----------------------------------------------------
def _bitop3(a, b, c, table):
    r = 0
    for idx in range(8):
        if table >> idx & 1:
            r |= (a if idx & 4 else ~a) & (b if idx & 2 else ~b) & (c if idx & 1 else ~c)
    return r & M


def _val(tok, regs):
    tok = tok.strip()
    if tok.startswith("%"):
        return regs[tok]
    return int(tok, 0)


def run_asm(lines, regs):
    for ln in lines:
        parts = ln.split(None, 1)
        opc = parts[0]
        if opc == "s_nop":
            continue
        mod = None
        args = parts[1]
        if " bitop3:" in args:
            args, mod = args.split(" bitop3:")
        ops = [x.strip() for x in args.split(",")]
        dst, src = ops[0], [_val(x, regs) for x in ops[1:]]
        if opc == "v_alignbit_b32":
            v = (((src[0] << 32) | src[1]) >> (src[2] & 31)) & M
        elif opc == "v_lshrrev_b32_e32":
            v = src[1] >> (src[0] & 31)
        elif opc == "v_bitop3_b32":
            v = _bitop3(src[0], src[1], src[2], int(mod, 0))
        elif opc == "v_bfi_b32":
            v = ((src[0] & src[1]) | (~src[0] & src[2])) & M
        elif opc == "v_add3_u32":
            v = (src[0] + src[1] + src[2]) & M
        elif opc == "v_add_u32_e32":
            v = (src[0] + src[1]) & M
        elif opc == "s_mov_b32":
            v = src[0] & M
        else:
            raise AssertionError(f"opcode the interpreter does not know: {opc}")
        regs[dst] = v


# ---- header parsing ----------------------------------------------------------
GEN = os.path.join(ROOT, "mirbft_amd", "csrc", "gen_rounds_asm.py")


def _functions(path=HDR):
    text = open(path).read()
    fns = {}
    for m in re.finditer(r"__device__ __forceinline__ void (\w+)\(([^)]*)\) \{(.*?)\n\}\n", text, re.S):
        fns[m.group(1)] = (m.group(2), m.group(3))
    return fns


def _statements(body):
    """Each asm statement: (instruction lines, [(operand name or index, C expr, constraint)])."""
    out = []
    for m in re.finditer(r"asm volatile\((.*?)\);", body, re.S):
        blob = m.group(1)
        lines = [x.replace("\\n\\t", "") for x in re.findall(r'"([^"]*\\n\\t)"', blob)]
        tail = blob.split("\n        :", 1)[1]
        operands = []
        for sect in tail.split("\n        :"):
            for om in re.finditer(r'(?:\[(\w+)\]\s*)?"([=&+]*[vs])"\(([^)]+\)?)\)', sect):
                operands.append((om.group(1), om.group(3), om.group(2)))
        out.append((lines, operands))
    return out


def run_function(name, env, path=HDR):
    """Run generated function `name`; env maps C expressions (s[0], w[3], k.c4,
    k0.x ...) to values and is updated for the "+" / "=" operands."""
    _, body = _functions(path)[name]
    for lines, operands in _statements(body):
        regs = {}
        for i, (nm, expr, cons) in enumerate(operands):
            key = f"%[{nm}]" if nm else f"%{i}"
            lit = re.fullmatch(r"(0x[0-9A-Fa-f]+)u?", expr)
            regs[key] = int(lit.group(1), 16) if lit else env.get(expr, 0xDEADBEEF)
        run_asm(lines, regs)
        for i, (nm, expr, cons) in enumerate(operands):
            if "=" in cons or "+" in cons:
                env[expr] = regs[f"%[{nm}]" if nm else f"%{i}"]
    return env


def _rand_state(rng):
    return [rng.getrandbits(32) for _ in range(8)]


def test_rounds_asm_matches_fips():
    rng = random.Random(1)
    for name in ("rounds_asm", "rounds_asm_nonop"):
        for _ in range(4):
            s, w = _rand_state(rng), [rng.getrandbits(32) for _ in range(16)]
            env = {f"s[{i}]": s[i] for i in range(8)}
            env.update({f"w[{i}]": w[i] for i in range(16)})
            run_function(name, env)
            assert [env[f"s[{i}]"] for i in range(8)] == ref_rounds(s, w), name


def tail_words(c4, c14, c15):
    """The scalars of rounds_asm_tail, as tail_words() in sha256_device.h."""
    return {"k.kw4": (K[4] + c4) & M, "k.kw14": (K[14] + c14) & M, "k.kw15": (K[15] + c15) & M,
            "k.c4": c4, "k.c14": c14, "k.c15": c15, "k.cs16": s1(c14), "k.cs17": s1(c15),
            "k.cs19": s0(c4), "k.cs29": s0(c14), "k.cs30": (s0(c15) + c14) & M}


def test_rounds_asm_tail_matches_fips():
    rng = random.Random(2)
    cases = [(0x80000000, 0, 272 * 8), (0, 0, 64 * 8), (0x80000000, 0, 4112 * 8)]
    cases += [(rng.choice([0, 0x80000000]), rng.getrandbits(32), rng.getrandbits(32)) for _ in range(5)]
    for c4, c14, c15 in cases:
        s = _rand_state(rng)
        head = [rng.getrandbits(32) for _ in range(4)]
        block = head + [c4] + [0] * 9 + [c14, c15]
        env = {f"s[{i}]": s[i] for i in range(8)}
        env.update({f"w[{i}]": head[i] for i in range(4)})
        env.update({f"w[{i}]": rng.getrandbits(32) for i in range(4, 16)})  # not read by the tail form
        env.update(tail_words(c4, c14, c15))
        run_function("rounds_asm_tail", env)
        assert [env[f"s[{i}]"] for i in range(8)] == ref_rounds(s, block), (c4, c14, c15)


def test_rounds_kw8_asm_matches_fips():
    """The pair kernels' consumer: 8 rounds per call with K + W precomputed."""
    rng = random.Random(3)
    s, w = _rand_state(rng), [rng.getrandbits(32) for _ in range(16)]
    full = list(w)
    for j in range(16, 64):
        full.append((s1(full[j - 2]) + full[j - 7] + s0(full[j - 15]) + full[j - 16]) & M)
    env = {f"s[{i}]": s[i] for i in range(8)}
    for c in range(8):
        kw = [(K[8 * c + i] + full[8 * c + i]) & M for i in range(8)]
        env.update({f"k0.{x}": kw[i] for i, x in enumerate("xyzw")})
        env.update({f"k1.{x}": kw[4 + i] for i, x in enumerate("xyzw")})
        run_function("rounds_kw8_asm", env)
    assert [env[f"s[{i}]"] for i in range(8)] == ref_rounds(s, w)


def test_ab_round_forms_match_fips(tmp_path):
    """The A/B-only forms (gen_rounds_asm.py --ab, generated for tools/ only:
    yield patterns, K-in-SGPR, bfi / add2 / literal variants, the lone-wave
    ILP order) are bit-identical to FIPS 180-4 too."""
    AB_HDR = str(tmp_path / "sha256_rounds_asm_ab.h")
    with open(AB_HDR, "w") as f:
        subprocess.run([sys.executable, GEN, "--ab"], stdout=f, check=True)
    rng = random.Random(4)
    names = [n for n, (sig, _) in _functions(AB_HDR).items() if "uint32_t w[16]" in sig]
    assert "rounds_asm_ilp" in names and len(names) >= 8
    for name in names:
        s, w = _rand_state(rng), [rng.getrandbits(32) for _ in range(16)]
        env = {f"s[{i}]": s[i] for i in range(8)}
        env.update({f"w[{i}]": w[i] for i in range(16)})
        run_function(name, env, AB_HDR)
        assert [env[f"s[{i}]"] for i in range(8)] == ref_rounds(s, w), name
