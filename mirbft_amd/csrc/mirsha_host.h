// mirsha_host.h — host-side helpers of the C-ABI (internal, not installed).
//
// The Go side hands one Ready() cycle's requests over as slice lists
// (HashRequest.Data, actions.go:157-164).  Before they reach the GPU they are
// packed into one pinned arena (the single host copy), optionally after a
// content-addressed dedup: during an epoch change every node hashes the SAME
// EpochChange payload once per acknowledging source (applyEpochChangeAckMsg,
// epoch_target.go:459-477, N sources x N origins per node), so identical
// requests are hashed once and their digest is copied to every duplicate, in
// origin order.
#pragma once
#include <stdint.h>

#include <functional>

namespace mirsha {
namespace host {

// Worker threads for a host pass over `bytes` bytes in `n` items: 1 below a
// few MiB, else min(hardware threads, 16, MIRSHA_HOST_THREADS if set).
int threads_for(uint64_t bytes, uint32_t n);

// fn(lo, hi) over contiguous index ranges covering [0, n), on `threads` threads.
void parallel_for(uint32_t n, int threads, const std::function<void(uint32_t, uint32_t)>& fn);

// 64-bit fingerprint of concat(ptr[s] for s in [s0, s1)): depends only on the
// concatenated bytes, not on how they are sliced.  NOT cryptographic: equal
// fingerprints are always confirmed byte for byte before two requests share
// a digest.  MIRSHA_DEDUP_WEAK_FP=1 (tests) makes every fingerprint 0 so that
// the confirm / collision path runs on every same-length pair.
uint64_t fingerprint(const uint8_t* const* ptr, const uint64_t* len, uint32_t s0, uint32_t s1);

// Byte equality of two slice-list concatenations of equal total length.
bool equal_concat(const uint8_t* const* ptr, const uint64_t* len, uint32_t a0, uint32_t a1, uint32_t b0,
                  uint32_t b1);

// rep[i] = the smallest j <= i whose request bytes equal request i's (i if
// none).  req_len[i] = total bytes of request i.  Returns the number of
// distinct requests (rep[i] == i).  = dedup_candidates + dedup_resolve.
uint32_t dedup_plan(const uint8_t* const* ptr, const uint64_t* len, const uint32_t* first, uint32_t n,
                    const uint64_t* req_len, uint32_t* rep);

// First half of dedup_plan: fingerprints fp[i] and tentative representatives
// tent[i] = the first request with the same (fingerprint, length).  Returns
// the number of heads (tent[i] == i); every head is a final representative,
// so their hashing may start before dedup_resolve confirms the rest.
uint32_t dedup_candidates(const uint8_t* const* ptr, const uint64_t* len, const uint32_t* first, uint32_t n,
                          const uint64_t* req_len, uint64_t* fp, uint32_t* tent);

// dedup_candidates with the call's slice validation folded into the same walk
// over the slice arrays (config 4: 15.7 M slices of 8-32 B, so the arrays are
// as large as the payload): per request its length req_len[i] and err[i]
// (0 ok, 1 slice_first not monotone or past ns, 2 a NULL slice with bytes,
// 3 longer than max_len).  Returns false (tent unset) if any err[i] != 0.
bool dedup_candidates_checked(const uint8_t* const* ptr, const uint64_t* len, const uint32_t* first, uint32_t n,
                              uint32_t ns, uint64_t max_len, uint64_t* req_len, uint8_t* err, uint64_t* fp,
                              uint32_t* tent, uint32_t* heads);

// Second half: confirms every tentative match byte for byte and resolves
// fingerprint collisions; fills rep[] as dedup_plan.  Returns distinct count.
uint32_t dedup_resolve(const uint8_t* const* ptr, const uint64_t* len, const uint32_t* first, uint32_t n,
                       const uint64_t* req_len, const uint64_t* fp, const uint32_t* tent, uint32_t* rep);

// Copies request which[k] (k < m) to dst + dst_off[k], in parallel.
void pack(const uint8_t* const* ptr, const uint64_t* len, const uint32_t* first, const uint32_t* which,
          uint32_t m, const uint64_t* dst_off, uint8_t* dst, int threads);

// Bytes [a, b) of the packed arena of n requests -- request i = concat of its
// slices [first[i], first[i+1]), placed at poff[i] (nondecreasing) -- into
// dst (dst[0] = byte a), split over `threads` threads by byte range.  With
// ptr == nullptr the source is the contiguous `base` instead (a parallel
// memcpy of base[a, b)).  Used to fill one pinned staging chunk while the
// previous chunk's DMA is in flight.
void pack_range(const uint8_t* base, const uint8_t* const* ptr, const uint64_t* len, const uint32_t* first,
                uint32_t n, const uint64_t* poff, uint64_t a, uint64_t b, uint8_t* dst, int threads);

}  // namespace host
}  // namespace mirsha
