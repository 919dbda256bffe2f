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
#include <unordered_map>
#include <vector>

namespace mirsha {
namespace host {

// Worker threads for a host pass over `bytes` bytes in `n` items: 1 below a
// few MiB, else min(hardware threads, 16, MIRSHA_HOST_THREADS if set).
int threads_for(uint64_t bytes, uint32_t n);

// fn(lo, hi) over contiguous index ranges covering [0, n), on `threads` threads.
void parallel_for(uint32_t n, int threads, const std::function<void(uint32_t, uint32_t)>& fn);

// out[i] = len[0] + ... + len[i-1]; returns the total.  Two passes over
// contiguous parts on the pool (part sums, then each part's offsets) when n is
// large (a config-2 cycle's 2^20 lengths: ~1 ms serially).
uint64_t exclusive_scan(const uint32_t* len, uint32_t n, uint64_t* out);

// Host threads of the process: min(hardware threads, 16), or MIRSHA_HOST_THREADS.
int max_threads();

// Pool of the calling thread's parallel_for: slot 0 = the process pool
// (max_threads() workers, the default); slots 1..kMaxPools-1 = pools of
// `threads` threads (workers + the caller), created on first use and kept,
// for callers that pack for several devices at once (mirsha_multi: one per
// device, each with its share of the host threads, so the devices' packing
// runs side by side instead of queueing for one pool).  threads_for() is
// capped at the selected pool's size.
constexpr int kMaxPools = 17;
void use_pool(int slot, int threads);

// 64-bit fingerprint of concat(ptr[s] for s in [s0, s1)): depends only on the
// concatenated bytes, not on how they are sliced.  NOT cryptographic: equal
// fingerprints are always confirmed byte for byte before two requests share
// a digest.  MIRSHA_DEDUP_WEAK_FP=1 (tests) makes every fingerprint 0 so that
// the confirm / collision path runs on every same-length pair.
uint64_t fingerprint(const uint8_t* const* ptr, const uint64_t* len, uint32_t s0, uint32_t s1);

// Byte equality of two slice-list concatenations of equal total length.
bool equal_concat(const uint8_t* const* ptr, const uint64_t* len, uint32_t a0, uint32_t a1, uint32_t b0,
                  uint32_t b1);

// Content-addressed dedup of n requests (slice lists), streamed over
// contiguous request ranges ("segments") in origin order, so the caller can
// start hashing the first segment's distinct requests while the rest is still
// being scanned:
//   for each segment [lo, hi):  scan(lo, hi); assign(lo, hi, heads); confirm(lo, hi);
//   then resolve(rep, &extra).
// scan: validation + a slicing-independent 64-bit fingerprint per request
// (one walk over its slice arrays, in parallel); a request whose
// (fingerprint, length) key matches a head of an EARLIER segment is compared
// with it byte for byte right there, while its bytes are cache-warm.  A
// request whose first 64 bytes match such a head is compared with it first:
// if equal, that one walk settles it (no fingerprint walk).
// assign: the remaining requests of the segment in origin order; the first
// request of a new key is a head (appended to `heads`): every head is a final
// representative, so it may be hashed at once.
// confirm: byte comparison of the segment's other tentative matches.
// resolve: rep[i] = the smallest j <= i whose bytes equal request i's (i if
// none); fingerprint collisions (a key match that the bytes refute, rare)
// become representatives too and are appended to `extra`.  Returns the number
// of distinct requests.  Equality is never decided by the fingerprint.
class DedupScan {
  public:
    DedupScan(const uint8_t* const* ptr, const uint64_t* len, const uint32_t* first, uint32_t n,
              uint64_t max_len);
    // Segment boundaries b[0] = 0 < ... < b.back() = n (~1/16 of the slices
    // each; one segment for small calls).
    std::vector<uint32_t> segments() const;
    // False if any request of [lo, hi) is malformed: err()[i] = 1 slice_first
    // not monotone or past its end, 2 a NULL slice with bytes, 3 longer than
    // max_len.
    bool scan(uint32_t lo, uint32_t hi);
    void assign(uint32_t lo, uint32_t hi, std::vector<uint32_t>& heads);
    void confirm(uint32_t lo, uint32_t hi);
    uint32_t resolve(uint32_t* rep, std::vector<uint32_t>* extra);
    const uint64_t* req_len() const { return req_len_.data(); }
    const uint8_t* err() const { return err_.data(); }

  private:
    static constexpr uint32_t kUnset = 0xFFFFFFFFu;
    static constexpr uint8_t kPending = 2;  // ok_: 0 refuted, 1 confirmed (or a head), 2 to confirm
    const uint8_t* const* ptr_;
    const uint64_t* len_;
    const uint32_t* first_;
    uint32_t n_, ns_;
    uint64_t max_len_;
    std::vector<uint64_t> req_len_, fp_;
    std::vector<uint32_t> tent_;
    std::vector<uint8_t> err_, ok_;
    std::unordered_map<uint64_t, uint32_t> head_;
    std::unordered_map<uint64_t, uint32_t> prefix_;  // first 64 bytes -> the first head with them
};

// The whole plan on the host (mirsha_dedup_plan): rep[] as DedupScan::resolve;
// returns the distinct count, or UINT32_MAX on malformed slice arrays (then
// *err_out = per-request codes if `err` is given).
uint32_t dedup_plan(const uint8_t* const* ptr, const uint64_t* len, const uint32_t* first, uint32_t n,
                    uint32_t* rep, const uint8_t** err_out, std::vector<uint8_t>* err);

// Copies request which[k] (k < m) to dst + dst_off[k], in parallel.  With
// `stream` the stores bypass the CPU caches (non-temporal, fenced before
// return): for page-locked staging a DMA reads next, which then runs at the
// link's rate instead of ~9% below it (profiles/r05o).  Not for buffers the
// CPU reads back.
void pack(const uint8_t* const* ptr, const uint64_t* len, const uint32_t* first, const uint32_t* which,
          uint32_t m, const uint64_t* dst_off, uint8_t* dst, int threads, bool stream = false);

// Bytes [a, b) of the packed arena of n requests -- request i = concat of its
// slices [first[i], first[i+1]), placed at poff[i] (nondecreasing) -- into
// dst (dst[0] = byte a), split over `threads` threads by byte range.  With
// ptr == nullptr the source is the contiguous `base` instead (a parallel
// memcpy of base[a, b)).  Used to fill one pinned staging chunk while the
// previous chunk's DMA is in flight.  `stream` as for pack.
void pack_range(const uint8_t* base, const uint8_t* const* ptr, const uint64_t* len, const uint32_t* first,
                uint32_t n, const uint64_t* poff, uint64_t a, uint64_t b, uint8_t* dst, int threads,
                bool stream = false);

}  // namespace host
}  // namespace mirsha
