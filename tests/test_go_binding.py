"""The Go binding (go/gpuhash.go, go/gpuhash_test.go) against the C-ABI, on
the CPU (verdict r5 item 4; there is no Go toolchain to compile it):

1. every C.mirsha_* call names a function include/mirsha.h declares, with the
   declared number of arguments, each argument a pointer or a scalar as the
   parameter is, of the declared C type where the Go side states it (a cast
   or a declared variable), and every C.MIRSHA_* / C.mirsha_* type it names
   is defined there;
2. every mirsha_* call the Go file makes is made by the C mirrors that run on
   the GPU (tests/c/cgo_sequence.c, tests/c/cgo_path.c);
3. the mirrored paths make the same calls in the same order: the chunked
   HashBatch (Go hashChunked through GPUHasher / GPUHasherMulti vs C
   hash_batch_chunked), gpuHash.Sum vs gpu_sum, and the SubmitBatch / Wait
   and lifecycle sequences inside cgo_sequence.c's main.

The checker is exercised on injected faults: a wrong arity, a wrong argument
type or kind, an unknown function, a swapped call order must each fail it."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GO = os.path.join(ROOT, "go", "gpuhash.go")
GO_TEST = os.path.join(ROOT, "go", "gpuhash_test.go")
HEADER = os.path.join(ROOT, "include", "mirsha.h")
C_SEQ = os.path.join(ROOT, "tests", "c", "cgo_sequence.c")
C_PATH = os.path.join(ROOT, "tests", "c", "cgo_path.c")


def _read(p):
    with open(p) as f:
        return f.read()


def strip_comments(src, go=False):
    """Drop // and /* */ comments outside string / char / raw-string literals."""
    out, i, n = [], 0, len(src)
    quotes = "\"'`" if go else "\"'"
    while i < n:
        c = src[i]
        if src.startswith("//", i):
            j = src.find("\n", i)
            i = n if j < 0 else j
        elif src.startswith("/*", i):
            j = src.find("*/", i + 2)
            i = n if j < 0 else j + 2
            out.append(" ")
        elif c in quotes:
            j = i + 1
            while j < n and src[j] != c:
                j += 2 if (src[j] == "\\" and c != "`") else 1
            out.append(src[i:j + 1])
            i = j + 1
        else:
            out.append(c)
            i += 1
    return "".join(out)


def split_args(s):
    """Top-level comma split of an argument list (brackets and strings respected)."""
    if not s.strip():
        return []
    args, depth, cur, i = [], 0, [], 0
    while i < len(s):
        c = s[i]
        if c in "\"'`":
            j = i + 1
            while j < len(s) and s[j] != c:
                j += 2 if (s[j] == "\\" and c != "`") else 1
            cur.append(s[i:j + 1])
            i = j + 1
            continue
        if c in "([{":
            depth += 1
        elif c in ")]}":
            depth -= 1
        if c == "," and depth == 0:
            args.append("".join(cur))
            cur = []
        else:
            cur.append(c)
        i += 1
    args.append("".join(cur))
    return [a.strip() for a in args]


def call_args(src, open_paren):
    """The text between src[open_paren] == '(' and its matching ')'."""
    depth, i = 0, open_paren
    while i < len(src):
        if src[i] in "\"'`":
            q, i = src[i], i + 1
            while src[i] != q:
                i += 2 if (src[i] == "\\" and q != "`") else 1
        elif src[i] == "(":
            depth += 1
        elif src[i] == ")":
            depth -= 1
            if depth == 0:
                return src[open_paren + 1:i]
        i += 1
    raise ValueError("unbalanced call")


def header_api(text):
    """{function: argument count}, {MIRSHA_* macros}, {typedef names}."""
    src = strip_comments(text)
    funcs = {}
    for m in re.finditer(r"\b(mirsha_\w+)\s*\(", src):
        pre = src[max(0, m.start() - 64):m.start()]
        if not re.search(r"(int|void|char|mirsha_ctx)\s*\**\s*$", pre):
            continue  # a use inside a macro or comment, not a declaration
        args = split_args(call_args(src, m.end() - 1))
        funcs[m.group(1)] = 0 if args == ["void"] else len(args)
    macros = set(re.findall(r"#define\s+(MIRSHA_\w+)", src))
    types = set(re.findall(r"typedef\s+struct\s+\w+\s+(mirsha_\w+)\s*;", src))
    return funcs, macros, types


def go_c_refs(text):
    """[(name, n_args)] of every C.mirsha_*(...) call, and the other C.* names."""
    src = strip_comments(text, go=True)
    calls = [(m.group(1), len(split_args(call_args(src, m.end() - 1))))
             for m in re.finditer(r"\bC\.(mirsha_\w+)\s*\(", src)]
    names = set(re.findall(r"\bC\.((?:MIRSHA|mirsha)_\w+)\b(?!\s*\()", src))
    return calls, names


def check_against_header(go_text, header_text):
    """Problems (empty when the binding matches the header)."""
    funcs, macros, types = header_api(header_text)
    calls, names = go_c_refs(go_text)
    bad = []
    for name, n in calls:
        if name not in funcs:
            bad.append(f"C.{name}: not declared in mirsha.h")
        elif funcs[name] != n:
            bad.append(f"C.{name}: {n} arguments, mirsha.h declares {funcs[name]}")
    for name in names:
        if name not in macros and name not in types:
            bad.append(f"C.{name}: no such macro or type in mirsha.h")
    return bad


# ---- argument kinds -----------------------------------------------------------

def header_params(text):
    """{function: [(is_pointer, base type)]} of every mirsha_* declaration."""
    src = strip_comments(text)
    out = {}
    for m in re.finditer(r"\b(mirsha_\w+)\s*\(", src):
        pre = src[max(0, m.start() - 64):m.start()]
        if not re.search(r"(int|void|char|mirsha_ctx)\s*\**\s*$", pre):
            continue
        params = []
        for a in split_args(call_args(src, m.end() - 1)):
            if a == "void":
                continue
            words = [w for w in re.findall(r"[A-Za-z_]\w*", a) if w != "const"]
            params.append(("*" in a, words[0] if words else None))
        out[m.group(1)] = params
    return out


def go_symbols(src):
    """{name: (is_pointer, C type or None)} from Go declarations: variables,
    parameters and struct fields of C.* / *C.* / unsafe.Pointer type."""
    sym = {}
    for m in re.finditer(r"\b(\w+)\s+(\*?)C\.(\w+)\b", src):
        sym[m.group(1)] = (bool(m.group(2)), m.group(3))
    for m in re.finditer(r"\b(\w+)\s+\*?unsafe\.Pointer\b", src):
        sym[m.group(1)] = (True, None)
    for m in re.finditer(r"\b(\w+)\s*:=\s*C\.(\w+)\(", src):
        sym[m.group(1)] = (False, m.group(2))
    for m in re.finditer(r"\b(\w+)\s*:=\s*\(\*C\.(\w+)\)\(", src):
        sym[m.group(1)] = (True, m.group(2))
    return sym


def arg_kind(expr, sym):
    """(is_pointer, C type or None) of a Go argument expression, or None."""
    e = expr.strip()
    m = re.fullmatch(r"C\.(\w+)\(.*\)", e, re.S)
    if m:
        return (False, m.group(1))
    m = re.fullmatch(r"\(\*C\.(\w+)\)\(.*\)", e, re.S)
    if m:
        return (True, m.group(1))
    if e.startswith("&"):
        return (True, None)
    if re.fullmatch(r"\d+", e):
        return (False, None)
    m = re.fullmatch(r"\*?(?:\w+\.)*(\w+)", e)
    if m and m.group(1) in sym:
        return sym[m.group(1)]
    return None


def check_arg_kinds(go_text, header_text):
    """Problems: a scalar where mirsha.h takes a pointer or the reverse, or a
    C scalar / pointee type that differs from the declared one."""
    params = header_params(header_text)
    src = strip_comments(go_text, go=True)
    sym = go_symbols(src)
    bad = []
    for m in re.finditer(r"\bC\.(mirsha_\w+)\s*\(", src):
        name = m.group(1)
        if name not in params:
            continue
        for i, (a, (ptr, base)) in enumerate(zip(split_args(call_args(src, m.end() - 1)), params[name])):
            k = arg_kind(a, sym)
            if k is None:
                continue
            if k[0] != ptr:
                bad.append(f"C.{name} argument {i + 1} ({a}): {'pointer' if k[0] else 'scalar'} for a "
                           f"{'pointer' if ptr else 'scalar'} parameter")
            elif k[1] and base and k[1] != base and not (ptr and base == "void"):
                bad.append(f"C.{name} argument {i + 1} ({a}): C.{k[1]} for {base}")
    return bad


# ---- call sequences ---------------------------------------------------------

def _body(src, start):
    """Body text of the function whose signature starts at `start`: from the
    first '{' at parenthesis depth 0 to its matching '}'."""
    depth, i = 0, start
    while True:
        c = src[i]
        if c == "(":
            depth += 1
        elif c == ")":
            depth -= 1
        elif c == "{" and depth == 0:
            break
        i += 1
    j, b = i, 0
    while True:
        if src[j] in "\"'`":
            q, j = src[j], j + 1
            while src[j] != q:
                j += 2 if (src[j] == "\\" and q != "`") else 1
        elif src[j] == "{":
            b += 1
        elif src[j] == "}":
            b -= 1
            if b == 0:
                return src[i + 1:j]
        j += 1


def go_functions(text):
    """{'Name' | 'Recv.Name': body} of every func in a Go file."""
    src = strip_comments(text, go=True)
    out = {}
    for m in re.finditer(r"^func\s+(?:\(\s*\w+\s+\*?(\w+)\s*\)\s*)?(\w+)\s*\(", src, re.M):
        key = f"{m.group(1)}.{m.group(2)}" if m.group(1) else m.group(2)
        out[key] = _body(src, m.end() - 1)
    return out


def go_sequence(funcs, key, hasher, depth=0):
    """mirsha_* calls of Go function `key` in source order, local calls
    inlined: plain functions, methods on g / h.g / pb.g (the hasher type
    `hasher`) and on e (the chunkEngine, resolved to `hasher`)."""
    if depth > 8:
        return []
    body, seq = funcs[key], []
    for m in re.finditer(r"(?:\b([A-Za-z_][\w\.]*)\.)?\b([A-Za-z_]\w*)\s*\(", body):
        qual, name = m.group(1), m.group(2)
        if qual == "C":
            if name.startswith("mirsha_"):
                seq.append(name)
        elif qual in ("g", "h.g", "pb.g", "e") and f"{hasher}.{name}" in funcs:
            seq += go_sequence(funcs, f"{hasher}.{name}", hasher, depth + 1)
        elif qual is None and name in funcs and name != key.split(".")[-1]:
            seq += go_sequence(funcs, name, hasher, depth + 1)
    return seq


def c_functions(text):
    """{name: body} of every function definition in a C file."""
    src = strip_comments(text)
    out = {}
    for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b(\w+)\s*\(([^;{}]*)\)\s*\{", src, re.M):
        out[m.group(1)] = _body(src, m.start(2) - 1)
    return out


def c_sequence(funcs, name, depth=0):
    if depth > 8:
        return []
    seq = []
    for m in re.finditer(r"\b([A-Za-z_]\w*)\s*\(", funcs[name]):
        f = m.group(1)
        if f.startswith("mirsha_"):
            seq.append(f)
        elif f in funcs and f != name:
            seq += c_sequence(funcs, f, depth + 1)
    return seq


def only(seq, vocab):
    return [s for s in seq if s in vocab]


def is_subsequence(small, big):
    it = iter(big)
    return all(any(x == y for y in it) for x in small)


SINGLE_CHUNK = {"mirsha_submit_batch", "mirsha_poll", "mirsha_wait"}
MULTI_CHUNK = {"mirsha_submit_arena_multi", "mirsha_poll_multi", "mirsha_wait_multi"}


def mirror_problems(go_text, seq_text, path_text):
    g = go_functions(go_text)
    cs, cp = c_functions(seq_text), c_functions(path_text)
    bad = []
    # the chunked HashBatch: identical call order in the Go body and its C twin
    for hasher, vocab in (("GPUHasher", SINGLE_CHUNK), ("GPUHasherMulti", MULTI_CHUNK)):
        gs = only(go_sequence(g, f"{hasher}.HashBatch", hasher), vocab)
        ps = only(c_sequence(cp, "hash_batch_chunked"), vocab)
        if gs != ps or len(gs) != 3:
            bad.append(f"{hasher}.HashBatch {gs} != cgo_path.c hash_batch_chunked {ps}")
    # gpuHash.Sum: grow the pinned arena, one-request mirsha_hash_batch
    vocab = {"mirsha_host_alloc", "mirsha_host_free", "mirsha_hash_batch"}
    gs = only(go_sequence(g, "gpuHash.Sum", "GPUHasher"), vocab)
    ps = only(c_sequence(cs, "gpu_sum"), vocab)
    if gs != ps:
        bad.append(f"gpuHash.Sum {gs} != cgo_sequence.c gpu_sum {ps}")
    # lifecycle and asynchronous forms: in order inside cgo_sequence.c main
    main = c_sequence(cs, "main")
    for key, hasher in (("NewGPUHasher", "GPUHasher"), ("GPUHasher.SubmitBatch", "GPUHasher"),
                        ("GPUHasher.Close", "GPUHasher"), ("NewGPUHasherMulti", "GPUHasherMulti"),
                        ("GPUHasherMulti.SubmitBatch", "GPUHasherMulti"), ("GPUHasherMulti.Close", "GPUHasherMulti")):
        gs = [s for s in go_sequence(g, key, hasher) if "last_error" not in s]  # g.fail: the panic path
        if not gs or not is_subsequence(gs, main):
            bad.append(f"{key} {gs} is not a call sequence of cgo_sequence.c main")
    # every call the binding makes is made on the GPU by one of the C mirrors
    made = set(main) | {s for f in cp for s in c_sequence(cp, f)} | {s for f in cs for s in c_sequence(cs, f)}
    made |= set(re.findall(r"\b(mirsha_\w+)\s*\(", strip_comments(seq_text + path_text)))  # CHECK macros
    for name, _ in go_c_refs(go_text)[0]:
        if name not in made:
            bad.append(f"C.{name}: no C mirror makes this call")
    return bad


# ---- tests ------------------------------------------------------------------

def test_go_files_exist_and_integration_points_at_them():
    for p in (GO, GO_TEST, os.path.join(ROOT, "go", "ntcopy_amd64.s")):
        assert os.path.exists(p), p
    doc = _read(os.path.join(ROOT, "INTEGRATION.md"))
    assert "go/gpuhash.go" in doc and "go/ntcopy_amd64.s" in doc
    assert "func ntCopy(dst, src unsafe.Pointer, n uintptr)" in _read(GO)
    assert "TEXT ·ntCopy(SB), NOSPLIT, $0-24" in _read(os.path.join(ROOT, "go", "ntcopy_amd64.s"))


def test_binding_calls_match_header():
    calls, _ = go_c_refs(_read(GO))
    assert len(calls) >= 25 and {"mirsha_submit_batch", "mirsha_submit_arena_multi", "mirsha_hash_batch"} <= {
        c for c, _ in calls}
    assert check_against_header(_read(GO), _read(HEADER)) == []


def test_binding_argument_kinds_match_header():
    assert check_arg_kinds(_read(GO), _read(HEADER)) == []
    # the checker sees most arguments (casts, &x, literals, declared names)
    params = header_params(_read(HEADER))
    src = strip_comments(_read(GO), go=True)
    sym = go_symbols(src)
    seen = total = 0
    for m in re.finditer(r"\bC\.(mirsha_\w+)\s*\(", src):
        for a in split_args(call_args(src, m.end() - 1)):
            total += 1
            seen += arg_kind(a, sym) is not None
    assert seen / total > 0.9, (seen, total)


@pytest.mark.parametrize("fault,needle", [
    # a 32-bit length where mirsha_submit_batch takes uint64_t arena_len
    (lambda s: s.replace("(*C.uint8_t)(arena), C.uint64_t(total),", "(*C.uint8_t)(arena), C.uint32_t(total),", 1),
     "C.uint32_t for uint64_t"),
    # the ticket by value where mirsha_poll takes int* done
    (lambda s: s.replace("C.mirsha_poll(g.ctx, t, &d)", "C.mirsha_poll(g.ctx, t, d)", 1), "scalar for a pointer"),
    # a pointer where mirsha_wait takes the ticket
    (lambda s: s.replace("C.mirsha_wait(g.ctx, t)", "C.mirsha_wait(g.ctx, &t)", 1), "pointer for a scalar"),
    # the wrong pointee type
    (lambda s: s.replace("(*C.uint64_t)(unsafe.Pointer(&off[0]))", "(*C.uint32_t)(unsafe.Pointer(&off[0]))", 1),
     "C.uint32_t for uint64_t"),
])
def test_argument_check_catches_injected_faults(fault, needle):
    bad = check_arg_kinds(fault(_read(GO)), _read(HEADER))
    assert any(needle in b for b in bad), bad


def test_c_mirrors_match_header():
    funcs, _, _ = header_api(_read(HEADER))
    for path in (C_SEQ, C_PATH):
        src = strip_comments(_read(path))
        for m in re.finditer(r"\b(mirsha_\w+)\s*\(", src):
            n = len(split_args(call_args(src, m.end() - 1)))
            assert funcs.get(m.group(1)) == n, (path, m.group(1), n)


def test_c_mirrors_make_the_same_calls_in_the_same_order():
    assert mirror_problems(_read(GO), _read(C_SEQ), _read(C_PATH)) == []


@pytest.mark.parametrize("fault,needle", [
    # one argument too few
    (lambda s: s.replace("C.mirsha_poll(g.ctx, t, &d)", "C.mirsha_poll(g.ctx, &d)"), "mirsha_poll: 2 arguments"),
    # one too many
    (lambda s: s.replace("C.mirsha_wait(g.ctx, t)", "C.mirsha_wait(g.ctx, t, 0)"), "mirsha_wait: 3 arguments"),
    # a function the header does not declare
    (lambda s: s.replace("C.mirsha_host_alloc(g.ctx", "C.mirsha_host_allocate(g.ctx", 1), "not declared"),
    # a constant it does not define
    (lambda s: s.replace("C.MIRSHA_SUBMIT_DEDUP", "C.MIRSHA_SUBMIT_DEDUPE", 1), "no such macro"),
])
def test_header_check_catches_injected_faults(fault, needle):
    bad = check_against_header(fault(_read(GO)), _read(HEADER))
    assert any(needle in b for b in bad), bad


def test_order_check_catches_a_swapped_call():
    go = _read(GO)
    # submit before polling the earlier chunks: the order differs from cgo_path.c
    a = "\t\tupto := copied\n\t\tfor upto < k-1 && e.done(tickets[upto]) {\n\t\t\tupto++\n\t\t}\n"
    b = "\t\tif k > 0 {\n\t\t\tlo, hi := cs[k-1].lo, cs[k-1].hi\n"
    assert a in go and b in go
    i, j = go.index(a), go.index(b)
    swapped = go[:i] + go[j:j + len(b)] + "\t\t\t_ = lo\n\t\t\t_ = hi\n\t\t}\n" + go[i:j] + go[j + len(b):]
    swapped = swapped.replace("tickets[k-1] = e.submit(", "tickets[k-1] = e.submit(", 1)
    # move the submit call itself ahead of the poll loop
    swapped = go.replace(a, "\t\tif k > 0 {\n\t\t\te.submit(arena, total, off, lens, dig)\n\t\t}\n" + a, 1)
    bad = mirror_problems(swapped, _read(C_SEQ), _read(C_PATH))
    assert any("hash_batch_chunked" in b for b in bad), bad


def test_order_check_catches_a_missing_mirror_call():
    seq = _read(C_SEQ).replace("CHECK(mirsha_submit_slices(ctx, ptr, slen, first, n_total, out1, "
                               "MIRSHA_SUBMIT_DEDUP, &t1));", "")
    seq = seq.replace("CHECK(mirsha_submit_slices(ctx, ptr, slen, first, 20, out2, 0, &t2));", "")
    bad = mirror_problems(_read(GO), seq, _read(C_PATH))
    assert any("GPUHasher.SubmitBatch" in b for b in bad), bad


def test_integration_md_go_snippets_match_header():
    """The Go snippets left in INTEGRATION.md (Processor wiring, overlapped
    device cycles) call the C-ABI with the declared names and arities too."""
    doc = _read(os.path.join(ROOT, "INTEGRATION.md"))
    blocks = re.findall(r"```go\n(.*?)```", doc, re.S)
    assert blocks
    code = "\n".join(blocks)
    assert check_against_header(code, _read(HEADER)) == []
    assert any(name == "mirsha_pipeline_overlap_device" for name, _ in go_c_refs(code)[0])


def test_go_test_file_uses_only_binding_api():
    """go/gpuhash_test.go calls the binding's exported API only (no C.*), with
    crypto/sha256 as the expected values."""
    src = strip_comments(_read(GO_TEST), go=True)
    assert "C." not in src
    for api in ("NewGPUHasher(", "HashBatch(", "SubmitBatch(", ".Wait()", "Hasher()", "NewGPUHasherMulti("):
        assert api in src, api
    assert '"crypto/sha256"' in src
