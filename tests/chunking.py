"""HashBatch's chunk planner restated for the tests (go/gpuhash.go planChunks,
tests/c/cgo_path.c hash_batch_chunked).  Test infrastructure."""
import numpy as np


def plan_chunks(lens, chunk_bytes):
    """Python twin of HashBatch's chunk planner (INTEGRATION.md planChunks,
    tests/c/cgo_path.c): [(first request, end request, whole blocks?)].
    Whole blocks of ceil(n / 4096) requests until a quarter, a half, then a
    whole budget is reached; a block over a whole budget is cut at request
    boundaries (no submission may outgrow one device arena)."""
    lens = np.asarray(lens, dtype=np.int64)
    n = lens.size
    if n == 0:
        return []
    br = -(-n // 4096)
    nb = -(-n // br)
    bpre = np.concatenate([[0], np.cumsum([lens[b * br:(b + 1) * br].sum() for b in range(nb)])])
    out, b0 = [], 0
    while b0 < nb:
        budget = chunk_bytes >> (2 - len(out)) if len(out) < 2 else chunk_bytes
        r0, r1 = b0 * br, min((b0 + 1) * br, n)
        if bpre[b0 + 1] - bpre[b0] > chunk_bytes:
            lo = r0
            while lo < r1:
                hi, s = lo + 1, lens[lo]
                while hi < r1 and s + lens[hi] <= chunk_bytes:
                    s += lens[hi]
                    hi += 1
                out.append((lo, hi, False))
                lo = hi
            b0 += 1
            continue
        b1 = b0 + 1
        while b1 < nb and bpre[b1] - bpre[b0] < budget and bpre[b1 + 1] - bpre[b1] <= chunk_bytes:
            b1 += 1
        out.append((r0, min(b1 * br, n), True))
        b0 = b1
    return out
