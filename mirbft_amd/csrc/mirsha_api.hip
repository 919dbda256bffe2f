// mirsha_api.hip — host side of the C-ABI declared in include/mirsha.h.
//
// Owns device/pinned buffers (grow-only pools), the launch stream, length
// bucketing and request-range sharding.  Every entry point returns digests in
// ORIGIN order (processor.go:139 indexes Digests[i] by the request's position),
// unlike ProcessorWorkPool's completion-order collector (processor.go:349-356).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mirsha.h"
#include "mirsha_host.h"
#include "mirsha_kernels.h"
#include "sha256_device.h"

namespace {

constexpr uint64_t kStageChunk = 32ull << 20;  // pinned staging chunk for pageable request bytes
constexpr int kStageSlots = 3;                  // chunks in flight (packed while earlier ones DMA)
constexpr uint64_t kInlineArena = 1ull << 20;   // arenas up to this ride in the metadata copy
constexpr uint64_t kPinnedOutMax = 8ull << 20;  // digest results up to this come back via pinned staging

constexpr uint64_t kArenaSlack = 256;           // loader may touch up to 80 B past a message
constexpr uint32_t kFusedMaxListWaves = 64;      // list groups (64 chains each) a fused launch takes
constexpr uint32_t kFusedMaxListBlocks = 32;     // list CUs (one producer / consumer pair each)
constexpr uint32_t kFusedMinChainBlocks = 64;    // AUTO picks the fused launch from this chain length
constexpr uint32_t kFusedDefaultPace = 4;        // tile waves (= tile queues) per SIMD
constexpr uint32_t kFusedDefaultListTiles = 1;   // FusedArgs::list_tiles (fused_build; profiles/r02au, r02av)

struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t want = std::max(n, cap + cap / 2);
        hipError_t e = hipMalloc(&p, want);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            e = hipMalloc(&p, n);
            if (e != hipSuccess) { p = nullptr; return e; }
            want = n;
        }
        cap = want;
        return hipSuccess;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
    void release() { if (p) (void)hipFree(p); p = nullptr; cap = 0; }
};

struct PinnedBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        hipError_t e = hipHostMalloc(&p, n, hipHostMallocDefault);
        if (e != hipSuccess) { p = nullptr; return e; }
        cap = n;
        return hipSuccess;
    }
    template <class T> T* as() const { return static_cast<T*>(p); }
    void release() { if (p) (void)hipHostFree(p); p = nullptr; cap = 0; }
};

// One in-flight submission of the asynchronous API (mirsha_submit_slices):
// its own pinned staging and device buffers, so up to kAsyncSlots Ready()
// cycles can be packed / copied / hashed while the caller works on.
constexpr uint32_t kAsyncSlots = 4;
using Clock = std::chrono::steady_clock;
inline double ms_since(Clock::time_point t0) {
    return std::chrono::duration<double, std::milli>(Clock::now() - t0).count();
}

struct AsyncSlot {
    PinnedBuf stage;  // [arena bytes | off u64[m] | len u32[m] | order u32[m]]
    Clock::time_point t_queued;  // when its device work was queued
    PinnedBuf dig;    // m x 32 digests (D2H target)
    DevBuf dev;       // the same layout as stage, then m x 32 digests
    PinnedBuf stage2;  // a dedup submission's second launch (representatives
    DevBuf dev2;       // found after the first), queued behind the first
    hipEvent_t done = nullptr;
    uint64_t ticket = 0;
    bool busy = false;
    uint8_t* user_out = nullptr;
    uint32_t n = 0, m = 0;
    std::vector<uint32_t> rank;  // request -> row of `dig` (empty: identity)
    double prof[MIRSHA_PROF_PHASES] = {};  // this submission's host phases (published when it completes)
};

struct KernelTimer {
    std::vector<std::pair<hipEvent_t, hipEvent_t>> pending;
    std::vector<hipEvent_t> pool;
    uint64_t launches = 0;
    double ms = 0.0;
};

}  // namespace

struct mirsha_ctx {
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    int variant = mirsha::kVariantLds;
    bool timing = false;
    uint32_t time_mask = 0xFFFFFFFFu;  // kernels timed while timing is on
    std::string err;
    DevBuf d_arena, d_off, d_len, d_order, d_out, d_idx, d_first, d_out2, d_scratch;
    DevBuf d_scan;  // scratch of the offsets scan (pipelined gapless calls)
    // Staged host calls (see "staged host calls" below): a ring of pinned
    // chunks for pageable request bytes, one pinned metadata block (plus small
    // arenas) -> one H2D, and pinned digest staging for small results.
    PinnedBuf h_ring[kStageSlots];
    hipEvent_t ring_ev[kStageSlots] = {};
    bool ring_busy[kStageSlots] = {};
    PinnedBuf h_meta, h_outs;
    DevBuf d_meta;
    // Pipelined staged calls (run_pipelined): H2D and D2H each on their own
    // stream, so chunk k's digests return while chunk k+1's bytes go in.
    hipStream_t xin = nullptr, xout = nullptr;
    std::vector<hipEvent_t> xev;  // per-call events (grow-only pool)
    KernelTimer timers[6];         // msgs, lists, gen, chain, fused, overlap
    AsyncSlot slots[kAsyncSlots];
    uint64_t next_ticket = 1;  // ticket of the next submission
    uint64_t done_ticket = 0;  // every ticket <= this one has completed
    double prof[MIRSHA_PROF_PHASES] = {};  // host phases of the last slice submission (ms)
};

// Streaming checkpoint chains (see mirsha.h, mirsha_chains_create).
struct mirsha_chains {
    int device = 0;
    uint32_t n = 0;
    DevBuf d_h, d_pend, d_cnt;                        // state
    DevBuf d_dig, d_pos, d_act, d_afirst, d_which, d_out;  // per call
};

// A request -> batch-digest pipeline plan (see mirsha.h, mirsha_pipeline_create).
struct mirsha_pipeline {
    int device = 0;
    int mode = MIRSHA_PIPELINE_FUSED;
    uint32_t n_req = 0, n_lists = 0, n_entries = 0;
    // fused mode (one persistent launch, see mirsha_kernels.hip)
    std::vector<uint32_t> tadj_first, tadj, cbase, expected;
    uint32_t n_tiles = 0, n_groups = 0, n_counters = 0, grid = 0;
    uint32_t pace = 1, list_blocks = 0, tile_waves = 0;  // tile waves per SIMD; list blocks first in the grid
    uint32_t list_tiles = 0;  // FusedArgs::list_tiles
    uint32_t q_first[mirsha::kFusedMaxQueues + 1] = {};  // tile queues (fused_build)
    uint32_t q_end[mirsha::kFusedMaxQueues] = {};        // queue q = [q_first[q], q_end[q])
    uint32_t q_waves[mirsha::kFusedMaxQueues] = {};      // waves of each queue's slot
    uint32_t tile_blocks = 0;
    uint64_t epoch = 0;  // completed runs of a fused plan
    DevBuf d_tadj_first, d_tadj, d_cbase, d_expected, d_counters, d_ctl, d_trace;
    // Sticky error word of a fused plan, in host-mapped memory: the launch's
    // list waves set it on a readiness-watchdog expiry; every later call on the
    // plan reads it without a synchronisation and fails (fail closed).
    unsigned long long* h_err = nullptr;
    unsigned long long* d_err = nullptr;
    unsigned long long watchdog = mirsha::kFusedWatchdogTicks;
    // split tiles (FusedArgs::n_split)
    uint32_t n_split = 0, split_first = 0, seg_per_tile = 0, seg_nominal_nb = 0;
    std::vector<uint32_t> seg_nb;
    DevBuf d_seg_nb, d_seg_state, d_seg_flags;
    uint64_t seg_runs = 0;  // launches of the plan (segment flags are monotone over them)
    // Fused plans probe the block placement at creation (launch_placement_probe):
    // not cyclic -> the plan is built SEQUENTIAL instead (fallback = 1).
    int fallback = 0;
    uint32_t test_placement = 0;  // FusedArgs::test_placement (tests only)
    DevBuf d_probe;
    bool trace = false;
    std::vector<uint32_t> cidx, cfirst;      // compacted lists (no null entries)
    std::vector<uint32_t> order;             // request processing order
    DevBuf d_cidx, d_cfirst, d_order, d_state;
};

namespace {

int fail(mirsha_ctx* c, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (c) c->err = buf;
    return code;
}

#define HIP_TRY(c, expr)                                                                    \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess)                                                               \
            return fail((c), _e == hipErrorOutOfMemory ? MIRSHA_ENOMEM : MIRSHA_EHIP,       \
                        "%s: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, __LINE__); \
    } while (0)

hipEvent_t take_event(KernelTimer& t) {
    if (!t.pool.empty()) {
        hipEvent_t e = t.pool.back();
        t.pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

// Brackets one launch with events on the launch stream when timing is on.
template <class F>
int timed_launch_on(mirsha_ctx* c, int which, hipStream_t st, F&& launch) {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const bool timed = c->timing && ((c->time_mask >> which) & 1u);
    if (timed) {
        e0 = take_event(c->timers[which]);
        e1 = take_event(c->timers[which]);
        if (e0) (void)hipEventRecord(e0, st);
    }
    hipError_t e = launch();
    if (e != hipSuccess) return fail(c, MIRSHA_EHIP, "kernel launch: %s", hipGetErrorString(e));
    if (timed && e0 && e1) {
        (void)hipEventRecord(e1, st);
        c->timers[which].pending.emplace_back(e0, e1);
    }
    return MIRSHA_OK;
}

template <class F>
int timed_launch(mirsha_ctx* c, int which, F&& launch) {
    return timed_launch_on(c, which, c->stream, launch);
}

int use_device(mirsha_ctx* c) {
    HIP_TRY(c, hipSetDevice(c->device));
    return MIRSHA_OK;
}

uint32_t host_blocks(uint32_t L) { return (uint32_t)(((uint64_t)L + 72u) >> 6); }

// Stable sort of message indices by block count, longest first.
bool bucket_order(const uint32_t* len, uint32_t n, uint32_t* order) {
    if (n == 0) return true;
    uint32_t lo = UINT32_MAX, hi = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t b = host_blocks(len[i]);
        lo = std::min(lo, b);
        hi = std::max(hi, b);
    }
    if (lo == hi) {
        for (uint32_t i = 0; i < n; i++) order[i] = i;
        return true;
    }
    const uint64_t range = (uint64_t)hi - lo + 1;
    if (range <= (1u << 22)) {
        std::vector<uint32_t> count(range + 1, 0);
        for (uint32_t i = 0; i < n; i++) count[hi - host_blocks(len[i]) + 1]++;
        for (uint64_t k = 1; k <= range; k++) count[k] += count[k - 1];
        for (uint32_t i = 0; i < n; i++) order[count[hi - host_blocks(len[i])]++] = i;
    } else {
        for (uint32_t i = 0; i < n; i++) order[i] = i;
        std::stable_sort(order, order + n, [&](uint32_t a, uint32_t b) {
            return host_blocks(len[a]) > host_blocks(len[b]);
        });
    }
    return false;
}

int check_lists(mirsha_ctx* c, const uint32_t* idx, const uint32_t* first, uint32_t n_lists,
                uint32_t n_digests) {
    if (!first) return fail(c, MIRSHA_EINVAL, "list_first is NULL");
    if (n_digests > mirsha::kMaxListDigests) return fail(c, MIRSHA_ERANGE, "%u digests > %u", n_digests, mirsha::kMaxListDigests);
    if (first[0] != 0) return fail(c, MIRSHA_EINVAL, "list_first[0] must be 0");
    for (uint32_t b = 0; b < n_lists; b++)
        if (first[b + 1] < first[b]) return fail(c, MIRSHA_EINVAL, "list_first not monotone at %u", b);
    const uint32_t entries = first[n_lists];
    if (entries && !idx) return fail(c, MIRSHA_EINVAL, "idx is NULL");
    if (entries > mirsha::kMaxListEntries) return fail(c, MIRSHA_ERANGE, "%u list entries > %u", entries, mirsha::kMaxListEntries);
    std::atomic<uint32_t> bad{UINT32_MAX};
    mirsha::host::parallel_for(entries, mirsha::host::threads_for(4ull * entries, entries), [&](uint32_t a, uint32_t b) {
        for (uint32_t e = a; e < b; e++)
            if (idx[e] != MIRSHA_NULL_INDEX && idx[e] >= n_digests) {
                uint32_t cur = bad.load();
                while (e < cur && !bad.compare_exchange_weak(cur, e)) {}
                return;
            }
    });
    if (const uint32_t e = bad.load(); e != UINT32_MAX)
        return fail(c, MIRSHA_EINVAL, "idx[%u]=%u out of range (%u digests)", e, idx[e], n_digests);
    // 32 bytes per digest must fit a 32-bit message length.
    for (uint32_t b = 0; b < n_lists; b++)
        if ((uint64_t)(first[b + 1] - first[b]) * 32u > MIRSHA_MAX_MESSAGE_BYTES)
            return fail(c, MIRSHA_ERANGE, "list %u too long", b);
    return MIRSHA_OK;
}

// ---- staged host calls --------------------------------------------------------
//
// The synchronous host API (the Go drop-in's path: one call per Ready()
// cycle) moves the cycle's request bytes to HBM at PCIe rate and everything
// else in ONE copy each way:
//   - request bytes: DMA'd straight from a page-locked caller arena
//     (mirsha_host_alloc), else packed by host threads into a ring of pinned
//     chunks, each chunk's DMA overlapping the packing of the next; small
//     arenas ride in the metadata copy;
//   - metadata (offsets, lengths, bucket order, list indices): one pinned
//     block, one H2D;
//   - digests (requests, then lists, contiguous on the device): one D2H
//     (through pinned staging when small);
//   - one stream synchronisation per call.
// Round 1 made 3-6 separate copies from pageable vectors plus two
// synchronisations per call.

// The bytes to hash, as the packed arena [0, total).
struct ArenaSrc {
    const uint8_t* base = nullptr;        // contiguous: arena byte x = base[x]; or
    const uint8_t* const* ptr = nullptr;  // slice lists: request i = its slices, at poff[i]
    const uint64_t* slen = nullptr;
    const uint32_t* sfirst = nullptr;
    const uint64_t* poff = nullptr;
    uint32_t n = 0;
    uint64_t total = 0;
};

// A boolean A/B or diagnostic knob ("1" = set; only with MIRSHA_AB=1).
bool getenv_flag(const char* name) {
    const char* e = mirsha::ab_getenv(name);
    return e && e[0] == '1';
}

bool host_pinned(const void* p) {
    hipPointerAttribute_t a;
    if (!p || hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// memcpy by host threads (metadata and result copies): one thread per
// 256 KiB (a 3.7 MB chunk of digests got 3 threads at the 1 MiB grain of
// threads_for, ~25 GB/s, and the copy-out was 1.3 ms of a config-2 call).
void pmemcpy(void* dst, const void* src, uint64_t n) {
    const int t = n < (1u << 19) ? 1 : (int)std::min<uint64_t>(mirsha::host::threads_for(1ull << 40, 1u << 20), n >> 18);
    mirsha::host::pack_range(static_cast<const uint8_t*>(src), nullptr, nullptr, nullptr, 0, nullptr, 0, n,
                             static_cast<uint8_t*>(dst), t);
}

void fill(const ArenaSrc& src, uint64_t a, uint64_t b, uint8_t* dst) {
    mirsha::host::pack_range(src.base, src.ptr, src.slen, src.sfirst, src.n, src.poff, a, b, dst,
                             mirsha::host::threads_for(b - a, 1u << 20));
}

// Queues src's bytes into d_arena on c->stream (large arenas; small ones are
// inlined by the caller).  Returns after the last chunk's DMA is queued.
int h2d_arena(mirsha_ctx* c, const ArenaSrc& src, uint8_t* d_arena) {
    if (src.total == 0) return MIRSHA_OK;
    if (src.base && host_pinned(src.base)) {  // page-locked caller arena: one DMA from it
        HIP_TRY(c, hipMemcpyAsync(d_arena, src.base, src.total, hipMemcpyHostToDevice, c->stream));
        return MIRSHA_OK;
    }
    for (uint64_t a = 0, k = 0; a < src.total; a += kStageChunk, k++) {
        const int slot = (int)(k % kStageSlots);
        const uint64_t b = std::min(src.total, a + kStageChunk);
        if (!c->ring_ev[slot]) HIP_TRY(c, hipEventCreateWithFlags(&c->ring_ev[slot], hipEventDisableTiming));
        if (c->ring_busy[slot]) HIP_TRY(c, hipEventSynchronize(c->ring_ev[slot]));  // its previous DMA is done
        HIP_TRY(c, c->h_ring[slot].ensure(kStageChunk));
        fill(src, a, b, c->h_ring[slot].as<uint8_t>());
        HIP_TRY(c, hipMemcpyAsync(d_arena + a, c->h_ring[slot].p, b - a, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(c, hipEventRecord(c->ring_ev[slot], c->stream));
        c->ring_busy[slot] = true;
    }
    return MIRSHA_OK;
}

// Device bytes [0, total) -> host: [0, split) to dst_a, [split, total) to
// dst_b, through the pinned ring: chunk k+1's DMA runs while chunk k is
// copied out by host threads (the caller's buffers are usually pageable).
int d2h_split(mirsha_ctx* c, const uint8_t* d_src, uint64_t total, uint64_t split, uint8_t* dst_a, uint8_t* dst_b) {
    const uint64_t nch = (total + kStageChunk - 1) / kStageChunk;
    auto dst_at = [&](uint64_t x) { return x < split ? dst_a + x : dst_b + (x - split); };
    auto queue = [&](uint64_t k) -> int {
        const int slot = (int)(k % kStageSlots);
        const uint64_t a = k * kStageChunk, b = std::min(total, a + kStageChunk);
        if (!c->ring_ev[slot]) HIP_TRY(c, hipEventCreateWithFlags(&c->ring_ev[slot], hipEventDisableTiming));
        HIP_TRY(c, c->h_ring[slot].ensure(kStageChunk));
        HIP_TRY(c, hipMemcpyAsync(c->h_ring[slot].p, d_src + a, b - a, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipEventRecord(c->ring_ev[slot], c->stream));
        return MIRSHA_OK;
    };
    for (uint64_t k = 0; k < std::min<uint64_t>(nch, kStageSlots - 1); k++)
        if (int rc = queue(k)) return rc;
    for (uint64_t k = 0; k < nch; k++) {
        if (k + kStageSlots - 1 < nch)
            if (int rc = queue(k + kStageSlots - 1)) return rc;
        const int slot = (int)(k % kStageSlots);
        HIP_TRY(c, hipEventSynchronize(c->ring_ev[slot]));
        const uint64_t a = k * kStageChunk, b = std::min(total, a + kStageChunk);
        const uint8_t* src = c->h_ring[slot].as<uint8_t>();
        // split the chunk at the a/b boundary, copy each part with threads
        const uint64_t m = std::min(std::max(split, a), b);
        if (m > a) mirsha::host::pack_range(src - a, nullptr, nullptr, nullptr, 0, nullptr, a, m, dst_at(a),
                                            mirsha::host::threads_for(m - a, 1u << 20));
        if (b > m) mirsha::host::pack_range(src - a, nullptr, nullptr, nullptr, 0, nullptr, m, b, dst_at(m),
                                            mirsha::host::threads_for(b - m, 1u << 20));
    }
    return MIRSHA_OK;
}

// Layout of the per-call metadata block (pinned and on device).
struct MetaLayout {
    uint64_t off, len, order, idx, first, arena, end;
    MetaLayout(uint32_t n, bool ordered, uint32_t entries, uint32_t n_lists, uint64_t inline_arena) {
        auto al = [](uint64_t x) { return (x + 15u) & ~15ull; };
        off = 0;
        len = al(off + 8ull * n);
        order = al(len + 4ull * n);
        idx = al(order + (ordered ? 4ull * n : 0));
        first = al(idx + 4ull * entries);
        arena = al(first + (n_lists ? 4ull * (n_lists + 1) : 0));
        end = al(arena + inline_arena + (inline_arena ? kArenaSlack : 0));
    }
};

// Metadata of n messages into the pinned block: offsets rebased by `shift`,
// lengths, and whether the block counts differ (a bucket order is needed).
// One parallel pass.
bool meta_fill(const uint64_t* off, const uint32_t* len, uint32_t n, uint64_t shift, uint8_t* h, const MetaLayout& L) {
    std::atomic<uint32_t> lo_b{UINT32_MAX}, hi_b{0};
    uint64_t* ho = reinterpret_cast<uint64_t*>(h + L.off);
    uint32_t* hl = reinterpret_cast<uint32_t*>(h + L.len);
    mirsha::host::parallel_for(n, mirsha::host::threads_for(12ull * n, n), [&](uint32_t a, uint32_t b) {
        uint32_t lo = UINT32_MAX, hi = 0;
        for (uint32_t i = a; i < b; i++) {
            ho[i] = off[i] - shift;
            hl[i] = len[i];
            const uint32_t k = host_blocks(len[i]);
            lo = std::min(lo, k);
            hi = std::max(hi, k);
        }
        uint32_t cur = lo_b.load();
        while (lo < cur && !lo_b.compare_exchange_weak(cur, lo)) {}
        cur = hi_b.load();
        while (hi > cur && !hi_b.compare_exchange_weak(cur, hi)) {}
    });
    return n && lo_b.load() != hi_b.load();
}

hipError_t take_events(mirsha_ctx* c, size_t k) {
    while (c->xev.size() < k) {
        hipEvent_t e = nullptr;
        hipError_t r = hipEventCreateWithFlags(&e, hipEventDisableTiming);
        if (r != hipSuccess) return r;
        c->xev.push_back(e);
    }
    return hipSuccess;
}

// The pipelined form of a large synchronous call (messages packed in order
// in [0, total)).  The arena goes over PCIe in kStageChunk chunks on the xin
// stream (straight from a page-locked caller arena, else packed by the host
// pool into the pinned ring behind the previous chunks' DMA); as soon as a
// chunk has landed, the request kernel hashes every message that lies wholly
// inside the bytes received so far, and the xout stream brings those digests
// back while the next chunks are still coming in (PCIe is full duplex).  The
// lists kernel follows the last request chunk.  A call then costs about its
// H2D time plus one chunk's kernel and D2H, instead of H2D + kernels + D2H +
// host copy-out in sequence.
// Per-call metadata of the pipelined path: [len u32 | idx u32 | first u32 |
// order u32 (if the block counts differ) | off u64].  Only [0, copy) goes over
// PCIe: off is left out when the requests are gapless (rebuilt on the device
// by an exclusive scan of len), order when it is not needed.
struct PipeLayout {
    uint64_t len, idx, first, order, off, end, copy;
    PipeLayout(uint32_t n, uint32_t entries, uint32_t n_lists, bool ordered, bool gapless) {
        auto al = [](uint64_t x) { return (x + 15u) & ~15ull; };
        len = 0;
        idx = al(len + 4ull * n);
        first = al(idx + 4ull * entries);
        order = al(first + (n_lists ? 4ull * (n_lists + 1) : 0));
        off = al(order + (ordered ? 4ull * n : 0));
        end = al(off + 8ull * n);
        copy = gapless ? off : end;
    }
};

// The pipelined form of a large synchronous call (messages packed in order
// in [0, total)).  The arena goes over PCIe in chunks on the xin stream
// (straight from a page-locked caller arena, else packed by the host pool into
// the pinned ring behind the previous chunks' DMA; the first chunk is small so
// the DMA starts early); as soon as a chunk has landed, the request kernel
// hashes every message that lies wholly inside the bytes received so far, and
// the xout stream brings those digests back while the next chunks are still
// coming in (PCIe is full duplex).  The lists kernel follows the last request
// chunk.  A call then costs about its H2D time plus one chunk's kernel and
// D2H, instead of H2D + kernels + D2H + host copy-out in sequence.
// `gapless`: off[i] - shift = len[0] + ... + len[i-1].
constexpr uint64_t kFirstChunk = 8ull << 20;
int run_pipelined(mirsha_ctx* c, const ArenaSrc& src, const uint64_t* off, const uint32_t* len, uint32_t n,
                  uint64_t shift, bool gapless, const uint32_t* idx, const uint32_t* first, uint32_t n_lists,
                  uint8_t* req_out, uint8_t* list_out) {
    double t_pack = 0.0, t_wait = 0.0, t_out = 0.0;
    // MIRSHA_STAGE_TRACE=1: one line per call on stderr with the host time
    // (us since entry) at which each chunk was queued and each wait returned.
    const bool trace = getenv_flag("MIRSHA_STAGE_TRACE");
    const auto t_entry = Clock::now();
    std::string tl;
    auto mark = [&](const char* what, uint32_t k) {
        if (!trace) return;
        char b[48];
        snprintf(b, sizeof b, " %s%u@%.0f", what, k, ms_since(t_entry) * 1e3);
        tl += b;
    };
    const uint64_t total = src.total;
    const uint32_t entries = n_lists ? first[n_lists] : 0u;
    // Chunk k covers arena bytes [cb[k], cb[k+1]).
    std::vector<uint64_t> cb{0};
    for (uint64_t x = std::min(total, kFirstChunk); ; x = std::min(total, x + kStageChunk)) {
        cb.push_back(x);
        if (x == total) break;
    }
    const uint32_t nch = (uint32_t)cb.size() - 1;
    if (!c->xin) HIP_TRY(c, hipStreamCreateWithFlags(&c->xin, hipStreamNonBlocking));
    if (!c->xout) HIP_TRY(c, hipStreamCreateWithFlags(&c->xout, hipStreamNonBlocking));
    // events: in[k], kern[k], out[k] per chunk; meta; lists kernel; lists out
    HIP_TRY(c, take_events(c, 3ull * nch + 3));
    hipEvent_t* ev_in = c->xev.data();
    hipEvent_t* ev_kern = ev_in + nch;
    hipEvent_t* ev_out = ev_kern + nch;
    hipEvent_t ev_meta = ev_out[nch], ev_lk = ev_out[nch + 1], ev_lo = ev_out[nch + 2];
    HIP_TRY(c, c->d_arena.ensure(total + kArenaSlack));
    uint8_t* d_arena = c->d_arena.as<uint8_t>();
    const bool pinned_src = src.base && host_pinned(src.base);
    auto queue_in = [&](uint32_t k) -> int {
        const uint64_t a = cb[k], b = cb[k + 1];
        const uint8_t* from = pinned_src ? src.base + a : nullptr;
        if (!from) {
            const int slot = (int)(k % kStageSlots);
            if (k >= (uint32_t)kStageSlots) {  // the slot's previous chunk must have left it
                const auto w = Clock::now();
                HIP_TRY(c, hipEventSynchronize(ev_in[k - kStageSlots]));
                t_wait += ms_since(w);
            }
            HIP_TRY(c, c->h_ring[slot].ensure(kStageChunk));
            const auto p = Clock::now();
            fill(src, a, b, c->h_ring[slot].as<uint8_t>());
            t_pack += ms_since(p);
            from = c->h_ring[slot].as<uint8_t>();
        }
        HIP_TRY(c, hipMemcpyAsync(d_arena + a, from, b - a, hipMemcpyHostToDevice, c->xin));
        HIP_TRY(c, hipEventRecord(ev_in[k], c->xin));
        mark("in", k);
        return MIRSHA_OK;
    };
    if (int rc = queue_in(0)) return rc;

    // Metadata (behind chunk 0 on the same copy stream).  Chunk k hashes the
    // messages [cut[k], cut[k+1]): those ending within its bytes [0, cb[k+1]).
    const auto tp = Clock::now();
    std::vector<uint32_t> cut(nch + 1, 0);
    for (uint32_t k = 0; k + 1 < nch; k++) {
        const uint64_t bk = cb[k + 1];
        uint32_t lo = cut[k], hi = n;  // first i with end(i) > bk (ends are nondecreasing)
        while (lo < hi) {
            const uint32_t mid = lo + (hi - lo) / 2;
            if (off[mid] - shift + len[mid] <= bk) lo = mid + 1; else hi = mid;
        }
        cut[k + 1] = lo;
    }
    cut[nch] = n;
    // Lengths first (and whether the block counts differ), then the layout.
    HIP_TRY(c, c->h_meta.ensure(PipeLayout(n, entries, n_lists, true, false).end));
    uint8_t* h = c->h_meta.as<uint8_t>();
    std::atomic<uint32_t> lo_b{UINT32_MAX}, hi_b{0};
    mirsha::host::parallel_for(n, mirsha::host::threads_for(4ull * n, n), [&](uint32_t a, uint32_t b) {
        uint32_t* hl = reinterpret_cast<uint32_t*>(h);
        uint32_t lo = UINT32_MAX, hi = 0;
        for (uint32_t i = a; i < b; i++) {
            hl[i] = len[i];
            const uint32_t k = host_blocks(len[i]);
            lo = std::min(lo, k);
            hi = std::max(hi, k);
        }
        uint32_t cur = lo_b.load();
        while (lo < cur && !lo_b.compare_exchange_weak(cur, lo)) {}
        cur = hi_b.load();
        while (hi > cur && !hi_b.compare_exchange_weak(cur, hi)) {}
    });
    const bool ordered = lo_b.load() != hi_b.load();
    const PipeLayout L(n, entries, n_lists, ordered, gapless);
    HIP_TRY(c, c->d_meta.ensure(L.end));
    if (!gapless) {
        uint64_t* ho = reinterpret_cast<uint64_t*>(h + L.off);
        mirsha::host::parallel_for(n, mirsha::host::threads_for(8ull * n, n), [&](uint32_t a, uint32_t b) {
            for (uint32_t i = a; i < b; i++) ho[i] = off[i] - shift;
        });
    }
    if (ordered) {  // a bucket order per chunk, indices local to the chunk
        mirsha::host::parallel_for(nch, (int)nch, [&](uint32_t a, uint32_t b) {
            for (uint32_t k = a; k < b; k++)
                bucket_order(len + cut[k], cut[k + 1] - cut[k], reinterpret_cast<uint32_t*>(h + L.order) + cut[k]);
        });
    }
    if (entries) pmemcpy(h + L.idx, idx, 4ull * entries);
    if (n_lists) pmemcpy(h + L.first, first, 4ull * (n_lists + 1));
    HIP_TRY(c, hipMemcpyAsync(c->d_meta.p, h, L.copy, hipMemcpyHostToDevice, c->xin));
    HIP_TRY(c, hipEventRecord(ev_meta, c->xin));
    HIP_TRY(c, hipStreamWaitEvent(c->stream, ev_meta, 0));
    uint8_t* dm = c->d_meta.as<uint8_t>();
    if (gapless) {  // off = exclusive scan of len, on the device
        size_t tb = 0;
        HIP_TRY(c, mirsha::launch_offsets_scan(nullptr, tb, reinterpret_cast<const uint32_t*>(dm + L.len),
                                               reinterpret_cast<uint64_t*>(dm + L.off), n, c->stream));
        HIP_TRY(c, c->d_scan.ensure(std::max<size_t>(tb, 4)));
        HIP_TRY(c, mirsha::launch_offsets_scan(c->d_scan.p, tb, reinterpret_cast<const uint32_t*>(dm + L.len),
                                               reinterpret_cast<uint64_t*>(dm + L.off), n, c->stream));
    }
    c->prof[MIRSHA_PROF_PLAN] = ms_since(tp);
    mark("meta", 0);

    const uint64_t out_bytes = 32ull * ((uint64_t)n + n_lists);
    HIP_TRY(c, c->d_out.ensure(std::max<uint64_t>(out_bytes, 32)));
    uint8_t* d_req = c->d_out.as<uint8_t>();
    uint8_t* d_lst = d_req + 32ull * n;
    const bool direct_out = host_pinned(req_out);
    HIP_TRY(c, c->h_outs.ensure(std::max<uint64_t>(direct_out ? 32ull * n_lists : out_bytes, 32)));
    uint8_t* h_req = direct_out ? req_out : c->h_outs.as<uint8_t>();
    uint8_t* h_lst = direct_out ? c->h_outs.as<uint8_t>() : h_req + 32ull * n;

    uint32_t copied = 0;  // chunks whose digests are in req_out
    auto copy_out = [&](uint32_t k0, uint32_t k1) {  // chunks [k0, k1), one parallel copy
        if (!direct_out && cut[k1] > cut[k0]) {
            const auto w = Clock::now();
            pmemcpy(req_out + 32ull * cut[k0], h_req + 32ull * cut[k0], 32ull * (cut[k1] - cut[k0]));
            t_out += ms_since(w);
            mark("out", k1);
        }
    };
    for (uint32_t k = 0; k < nch; k++) {
        if (k > 0)
            if (int rc = queue_in(k)) return rc;
        const uint32_t i0 = cut[k], cnt = cut[k + 1] - i0;
        HIP_TRY(c, hipStreamWaitEvent(c->stream, ev_in[k], 0));
        if (cnt) {
            if (int rc = timed_launch(c, 0, [&] {
                    return mirsha::launch_msgs(d_arena, total, reinterpret_cast<const uint64_t*>(dm + L.off) + i0,
                                               reinterpret_cast<const uint32_t*>(dm + L.len) + i0,
                                               ordered ? reinterpret_cast<const uint32_t*>(dm + L.order) + i0 : nullptr,
                                               cnt, d_req + 32ull * i0, c->variant, c->stream);
                }))
                return rc;
        }
        HIP_TRY(c, hipEventRecord(ev_kern[k], c->stream));
        HIP_TRY(c, hipStreamWaitEvent(c->xout, ev_kern[k], 0));
        if (cnt) HIP_TRY(c, hipMemcpyAsync(h_req + 32ull * i0, d_req + 32ull * i0, 32ull * cnt, hipMemcpyDeviceToHost, c->xout));
        HIP_TRY(c, hipEventRecord(ev_out[k], c->xout));
        // digests that are already back go to the caller while later chunks pack
        uint32_t ready = copied;
        while (ready < k) {
            const hipError_t q = hipEventQuery(ev_out[ready]);
            if (q == hipErrorNotReady) {
                (void)hipGetLastError();  // NotReady is not an error; never let a later launch check see it
                break;
            }
            if (q != hipSuccess) return fail(c, MIRSHA_EHIP, "hipEventQuery: %s", hipGetErrorString(q));
            ready++;
        }
        copy_out(copied, ready);
        copied = ready;
    }
    if (n_lists) {
        HIP_TRY(c, c->d_scratch.ensure(sizeof(uint32_t) * std::max<uint32_t>(entries, 1)));
        if (int rc = timed_launch(c, 1, [&] {
                return mirsha::launch_lists(d_req, n, reinterpret_cast<const uint32_t*>(dm + L.idx), entries,
                                            reinterpret_cast<const uint32_t*>(dm + L.first), n_lists,
                                            c->d_scratch.as<uint32_t>(), d_lst, c->stream);
            }))
            return rc;
        HIP_TRY(c, hipEventRecord(ev_lk, c->stream));
        HIP_TRY(c, hipStreamWaitEvent(c->xout, ev_lk, 0));
        HIP_TRY(c, hipMemcpyAsync(h_lst, d_lst, 32ull * n_lists, hipMemcpyDeviceToHost, c->xout));
        HIP_TRY(c, hipEventRecord(ev_lo, c->xout));
    }
    // The rest: all but the last chunk are usually back by now (one copy for
    // them), then the last chunk and the lists.
    if (copied + 1 < nch) {
        const auto w = Clock::now();
        HIP_TRY(c, hipEventSynchronize(ev_out[nch - 2]));
        t_wait += ms_since(w);
        mark("w", nch - 2);
        copy_out(copied, nch - 1);
        copied = nch - 1;
    }
    if (copied < nch) {
        const auto w = Clock::now();
        HIP_TRY(c, hipEventSynchronize(ev_out[nch - 1]));
        t_wait += ms_since(w);
        mark("w", nch - 1);
        copy_out(copied, nch);
    }
    if (n_lists) {
        const auto w = Clock::now();
        HIP_TRY(c, hipEventSynchronize(ev_lo));
        t_wait += ms_since(w);
        memcpy(list_out, h_lst, 32ull * n_lists);
    }
    mark("end", nch);
    if (trace) fprintf(stderr, "mirsha stage trace: %u chunks%s\n", nch, tl.c_str());
    // The caller's stream also saw every kernel finish (ev_out waits on them).
    c->prof[MIRSHA_PROF_PACK] = t_pack;
    c->prof[MIRSHA_PROF_DEVICE] = t_wait;
    c->prof[MIRSHA_PROF_SCATTER] = t_out;
    c->prof[MIRSHA_PROF_CHUNKS] = nch;
    return MIRSHA_OK;
}

// One synchronous call: n messages (offsets minus `shift` are positions in the
// packed arena) and optionally n_lists digest lists over their digests.
// req_out / list_out are the caller's host buffers (n x 32, n_lists x 32).
// Largest block count of n messages (one parallel pass).
uint32_t max_blocks(const uint32_t* len, uint32_t n) {
    std::atomic<uint32_t> hi{0};
    mirsha::host::parallel_for(n, mirsha::host::threads_for(4ull * n, n), [&](uint32_t a, uint32_t b) {
        uint32_t m = 0;
        for (uint32_t i = a; i < b; i++) m = std::max(m, len[i]);
        uint32_t cur = hi.load();
        while (m > cur && !hi.compare_exchange_weak(cur, m)) {}
    });
    return host_blocks(hi.load());
}

// Each chunk of a pipelined call is its own launch, and a launch takes at
// least its longest message's chain (~2-2.5 us per block at one wave per
// SIMD).  Past 256 blocks (16 KiB) that floor exceeds a 32 MiB chunk's DMA
// (~0.55 ms) and chunked launches would serialise: 9 x 1.86 ms for config 4's
// 61.6 KB acks (profiles/r02p) instead of one 1.86 ms launch.
constexpr uint32_t kPipeMaxBlocks = 256;

// `layout`: kInOrder = the messages lie in [0, total) in index order (each
// starts at or after the previous one's end), which the pipelined form needs;
// kGapless = in order with no gaps (off[i] - shift = len[0] + ... + len[i-1]).
enum ArenaLayout { kAnyOrder = 0, kInOrder = 1, kGapless = 2 };
int run_staged(mirsha_ctx* c, const ArenaSrc& src, const uint64_t* off, const uint32_t* len, uint32_t n,
               uint64_t shift, ArenaLayout layout, const uint32_t* idx, const uint32_t* first, uint32_t n_lists,
               uint8_t* req_out, uint8_t* list_out) {
    if (n && layout != kAnyOrder && src.total > kStageChunk && !getenv_flag("MIRSHA_NO_PIPELINED_CALLS") &&
        max_blocks(len, n) <= kPipeMaxBlocks)
        return run_pipelined(c, src, off, len, n, shift, layout == kGapless && !getenv_flag("MIRSHA_NO_OFFSET_SCAN"),
                             idx, first, n_lists, req_out, list_out);
    // Host phases into c->prof (mirsha_ctx_host_profile): pack = queueing the
    // request bytes, plan = metadata block, device = queue -> sync, scatter =
    // digests to the caller.  (validate is filled by the caller.)
    auto t0 = Clock::now();
    c->prof[MIRSHA_PROF_CHUNKS] = 0;  // single-shot staging
    const uint32_t entries = n_lists ? first[n_lists] : 0u;
    const bool inl = src.total <= kInlineArena;
    // Large arenas first: their chunks DMA while the metadata is built.
    HIP_TRY(c, c->d_arena.ensure(inl ? 1 : src.total + kArenaSlack));
    if (!inl)
        if (int rc = h2d_arena(c, src, c->d_arena.as<uint8_t>())) return rc;
    c->prof[MIRSHA_PROF_PACK] = ms_since(t0);
    t0 = Clock::now();
    const MetaLayout L(n, true, entries, n_lists, inl ? src.total : 0);
    HIP_TRY(c, c->h_meta.ensure(L.end));
    HIP_TRY(c, c->d_meta.ensure(L.end));
    uint8_t* h = c->h_meta.as<uint8_t>();
    const bool ordered = meta_fill(off, len, n, shift, h, L);
    if (ordered) bucket_order(len, n, reinterpret_cast<uint32_t*>(h + L.order));
    if (entries) pmemcpy(h + L.idx, idx, 4ull * entries);
    if (n_lists) pmemcpy(h + L.first, first, 4ull * (n_lists + 1));
    if (inl && src.total) fill(src, 0, src.total, h + L.arena);
    c->prof[MIRSHA_PROF_PLAN] = ms_since(t0);
    t0 = Clock::now();
    // (A zero-copy form for small calls -- kernels reading the pinned block
    // and writing pinned digests over PCIe -- measured no faster: 47.6 vs
    // 44.5 us for a 17-request cycle, profiles/r02j.)
    HIP_TRY(c, hipMemcpyAsync(c->d_meta.p, h, L.end, hipMemcpyHostToDevice, c->stream));
    uint8_t* dm = c->d_meta.as<uint8_t>();
    const uint8_t* d_arena = inl ? dm + L.arena : c->d_arena.as<uint8_t>();
    // Digests: requests then lists, contiguous (one D2H).
    const uint64_t out_bytes = 32ull * ((uint64_t)n + n_lists);
    HIP_TRY(c, c->d_out.ensure(std::max<uint64_t>(out_bytes, 32)));
    uint8_t* d_req = c->d_out.as<uint8_t>();
    uint8_t* d_lst = d_req + 32ull * n;
    if (n) {
        if (int rc = timed_launch(c, 0, [&] {
                return mirsha::launch_msgs(d_arena, src.total, reinterpret_cast<const uint64_t*>(dm + L.off),
                                           reinterpret_cast<const uint32_t*>(dm + L.len),
                                           ordered ? reinterpret_cast<const uint32_t*>(dm + L.order) : nullptr, n,
                                           d_req, c->variant, c->stream);
            }))
            return rc;
    }
    if (n_lists) {
        // Lists index the request digests just computed, or with no requests
        // the arena itself as 32-byte digests (mirsha_digest_lists).
        const uint8_t* d_dig = n ? d_req : d_arena;
        const uint32_t n_dig = n ? n : (uint32_t)(src.total / 32u);
        HIP_TRY(c, c->d_scratch.ensure(sizeof(uint32_t) * std::max<uint32_t>(entries, 1)));
        if (int rc = timed_launch(c, 1, [&] {
                return mirsha::launch_lists(d_dig, n_dig, reinterpret_cast<const uint32_t*>(dm + L.idx), entries,
                                            reinterpret_cast<const uint32_t*>(dm + L.first), n_lists,
                                            c->d_scratch.as<uint32_t>(), d_lst, c->stream);
            }))
            return rc;
    }
    if (out_bytes <= kPinnedOutMax) {
        HIP_TRY(c, c->h_outs.ensure(std::max<uint64_t>(out_bytes, 32)));
        HIP_TRY(c, hipMemcpyAsync(c->h_outs.p, d_req, out_bytes, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        c->prof[MIRSHA_PROF_DEVICE] = ms_since(t0);
        t0 = Clock::now();
        if (n) memcpy(req_out, c->h_outs.p, 32ull * n);
        if (n_lists) memcpy(list_out, c->h_outs.as<uint8_t>() + 32ull * n, 32ull * n_lists);
    } else {
        // Large results: device -> pinned ring chunks -> caller, each chunk's
        // copy-out overlapping the next chunk's DMA.
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        for (bool& b : c->ring_busy) b = false;
        c->prof[MIRSHA_PROF_DEVICE] = ms_since(t0);
        t0 = Clock::now();
        if (int rc = d2h_split(c, d_req, out_bytes, 32ull * n, req_out, list_out)) return rc;
    }
    c->prof[MIRSHA_PROF_SCATTER] = ms_since(t0);
    for (bool& b : c->ring_busy) b = false;  // every queued chunk DMA has completed
    return MIRSHA_OK;
}

// Validates messages of a caller arena: the dense span [lo, hi) they cover,
// their total length, and their layout (in index order: off[i] >= off[i-1] +
// len[i-1]; gapless: equality).  One parallel pass.
int arena_span(mirsha_ctx* c, uint64_t arena_len, const uint64_t* off, const uint32_t* len, uint32_t n,
               uint64_t* lo_out, uint64_t* hi_out, uint64_t* total_out = nullptr, ArenaLayout* layout_out = nullptr) {
    // Threads over index ranges; the first bad message (lowest index) is reported.
    const int T = mirsha::host::threads_for(12ull * n, n);
    std::vector<uint64_t> los(T, UINT64_MAX), his(T, 0), tot(T, 0);
    std::vector<uint32_t> bad(T, UINT32_MAX);
    std::vector<uint8_t> ord(T, 1), tight(T, 1);
    const uint32_t step = (n + T - 1) / std::max(T, 1);
    mirsha::host::parallel_for(n, T, [&](uint32_t a, uint32_t b) {
        const int k = (int)(a / std::max<uint32_t>(step, 1));
        uint64_t lo = UINT64_MAX, hi = 0, t = 0;
        bool in = true, gl = true;
        for (uint32_t i = a; i < b; i++) {
            if (len[i] > MIRSHA_MAX_MESSAGE_BYTES || off[i] > arena_len || len[i] > arena_len - off[i]) {
                bad[k] = i;
                break;
            }
            lo = std::min<uint64_t>(lo, off[i]);
            hi = std::max<uint64_t>(hi, off[i] + len[i]);
            t += len[i];
            if (i && off[i] < off[i - 1] + len[i - 1]) in = false;
            if (i && off[i] != off[i - 1] + len[i - 1]) gl = false;
        }
        los[k] = lo;
        his[k] = hi;
        tot[k] = t;
        ord[k] = in;
        tight[k] = gl;
    });
    const uint32_t i = *std::min_element(bad.begin(), bad.end());
    if (i != UINT32_MAX) {
        if (len[i] > MIRSHA_MAX_MESSAGE_BYTES)
            return fail(c, MIRSHA_ERANGE, "message %u is %u bytes (max %u)", i, len[i], MIRSHA_MAX_MESSAGE_BYTES);
        return fail(c, MIRSHA_EINVAL, "message %u [%llu,+%u) outside arena of %llu bytes", i,
                    (unsigned long long)off[i], len[i], (unsigned long long)arena_len);
    }
    *lo_out = n ? *std::min_element(los.begin(), los.end()) : 0;
    *hi_out = n ? *std::max_element(his.begin(), his.end()) : 0;
    uint64_t t = 0;
    for (uint64_t x : tot) t += x;
    if (total_out) *total_out = t;
    if (layout_out) {
        auto all = [](const std::vector<uint8_t>& v) { return std::all_of(v.begin(), v.end(), [](uint8_t x) { return x != 0; }); };
        *layout_out = !all(ord) ? kAnyOrder : (all(tight) && (!n || off[0] == *lo_out) ? kGapless : kInOrder);
    }
    return MIRSHA_OK;
}

// A caller arena + offsets: the span itself when dense, else the messages
// packed back to back (sparse arenas do not ship their gaps).
int run_arena_call(mirsha_ctx* c, const uint8_t* arena, uint64_t arena_len, const uint64_t* off, const uint32_t* len,
                   uint32_t n, const uint32_t* idx, const uint32_t* first, uint32_t n_lists, uint8_t* req_out,
                   uint8_t* list_out) {
    const auto t0 = Clock::now();
    for (double& x : c->prof) x = 0.0;
    uint64_t lo = 0, hi = 0, total = 0;
    ArenaLayout layout = kAnyOrder;
    if (int rc = arena_span(c, arena_len, off, len, n, &lo, &hi, &total, &layout)) return rc;
    c->prof[MIRSHA_PROF_VALIDATE] = ms_since(t0);
    ArenaSrc src;
    if (hi - lo <= 2 * total + 4096) {  // dense: ship the span, offsets rebased on lo
        src.base = arena + lo;
        src.total = hi - lo;
        const int rc = run_staged(c, src, off, len, n, lo, layout, idx, first, n_lists, req_out, list_out);
        c->prof[MIRSHA_PROF_TOTAL] = ms_since(t0);
        return rc;
    }
    // sparse: one slice per message, packed back to back
    std::vector<uint64_t> roff(n);
    std::vector<const uint8_t*> sp(n);
    std::vector<uint64_t> sl(n);
    std::vector<uint32_t> sf(n + 1);
    uint64_t p = 0;
    for (uint32_t i = 0; i < n; i++) {
        sp[i] = arena + off[i];
        sl[i] = len[i];
        sf[i] = i;
        roff[i] = p;
        p += len[i];
    }
    sf[n] = n;
    src.ptr = sp.data();
    src.slen = sl.data();
    src.sfirst = sf.data();
    src.poff = roff.data();
    src.n = n;
    src.total = total;
    const int rc = run_staged(c, src, roff.data(), len, n, 0, kGapless, idx, first, n_lists, req_out, list_out);
    c->prof[MIRSHA_PROF_TOTAL] = ms_since(t0);
    return rc;
}

// ---- request -> batch-digest plan (sequential form) ------------------------
//
// The dependent pass (batch / VerifyBatch digests over request digests,
// sequence.go:154-157, batch_tracker.go:147-150) is a set of sequential SHA
// chains over the request digests.  The sequential plan runs the request
// kernel at full occupancy, then the list chains; the lists are compacted
// once per plan (null requests contribute no bytes and are dropped).
// Stream-level pipelining (chain segments on a second stream) and the
// in-kernel continuation form were measured slower at BASELINE sizes and
// removed (code in git history before round 2).
int pipeline_build(mirsha_ctx* c, mirsha_pipeline* p, uint32_t n_req, const uint32_t* idx, const uint32_t* first,
                   uint32_t n_lists, const uint32_t* len) {
    p->n_req = n_req;
    p->n_lists = n_lists;
    p->cfirst.assign(n_lists + 1, 0);
    p->cidx.clear();
    p->cidx.reserve(first[n_lists]);
    std::vector<uint8_t> listed(n_req, 0);
    for (uint32_t k = 0; k < n_lists; k++) {
        for (uint32_t e = first[k]; e < first[k + 1]; e++) {
            if (idx[e] == MIRSHA_NULL_INDEX) continue;  // empty digest: contributes no bytes
            p->cidx.push_back(idx[e]);
            listed[idx[e]] = 1;
        }
        p->cfirst[k + 1] = (uint32_t)p->cidx.size();
    }
    p->n_entries = (uint32_t)p->cidx.size();
    // Processing order: listed requests first, then longest-first by block
    // count (length bucketing inside a wave), stable.
    p->order.resize(n_req);
    for (uint32_t r = 0; r < n_req; r++) p->order[r] = r;
    std::stable_sort(p->order.begin(), p->order.end(), [&](uint32_t x, uint32_t y) {
        if (listed[x] != listed[y]) return listed[x] > listed[y];
        return len ? host_blocks(len[x]) > host_blocks(len[y]) : false;
    });
    HIP_TRY(c, p->d_cidx.ensure(sizeof(uint32_t) * std::max<uint32_t>(p->n_entries, 1)));
    HIP_TRY(c, p->d_cfirst.ensure(sizeof(uint32_t) * (n_lists + 1)));
    HIP_TRY(c, p->d_order.ensure(sizeof(uint32_t) * std::max<uint32_t>(n_req, 1)));
    HIP_TRY(c, p->d_state.ensure(32ull * std::max<uint32_t>(n_lists, 1)));
    // Copies on the context stream (not the legacy null stream); the host
    // vectors must outlive them, hence the synchronize.
    if (p->n_entries)
        HIP_TRY(c, hipMemcpyAsync(p->d_cidx.p, p->cidx.data(), sizeof(uint32_t) * p->n_entries, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(p->d_cfirst.p, p->cfirst.data(), sizeof(uint32_t) * (n_lists + 1), hipMemcpyHostToDevice, c->stream));
    if (n_req)
        HIP_TRY(c, hipMemcpyAsync(p->d_order.p, p->order.data(), sizeof(uint32_t) * n_req, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return MIRSHA_OK;
}

int pipeline_run(mirsha_ctx* c, mirsha_pipeline* p, const uint8_t* d_arena, uint64_t arena_len, const uint64_t* d_off,
                 const uint32_t* d_len, uint8_t* d_req_out, uint8_t* d_list_out) {
    const uint32_t* order = p->d_order.as<uint32_t>();
    if (p->n_req) {
        if (int rc = timed_launch(c, 0, [&] {
                return mirsha::launch_msgs(d_arena, arena_len, d_off, d_len, order, p->n_req, d_req_out, c->variant,
                                           c->stream);
            }))
            return rc;
    }
    if (p->n_lists == 0) return MIRSHA_OK;
    if ((p->n_lists + 63u) / 64u <= mirsha::pair_max_groups())
        return timed_launch(c, 1, [&] {  // few long chains: producer/consumer pairs
            return mirsha::launch_chain_pair(d_req_out, p->n_req, p->d_cidx.as<uint32_t>(), p->n_entries,
                                             p->d_cfirst.as<uint32_t>(), p->n_lists, d_list_out, c->stream);
        });
    return timed_launch(c, 1, [&] {
        return mirsha::launch_chain(d_req_out, p->n_req, p->d_cidx.as<uint32_t>(), p->n_entries,
                                    p->d_cfirst.as<uint32_t>(), p->n_lists, 0u, mirsha::kOpenEnd,
                                    p->d_state.as<uint32_t>(), d_list_out, c->stream);
    });
}


// ---- fused plan: one launch (sha256_fused_paced_kernel) ----------------------
//
// Host work per plan (once per shape): compacted lists, needed-at processing
// order, and for every (tile, list-group chunk) pair that feeds it one
// readiness counter increment; expected[ctr] = number of distinct feeding tiles.
int fused_build(mirsha_ctx* c, mirsha_pipeline* p, uint32_t n_req, const uint32_t* idx, const uint32_t* first,
                uint32_t n_lists, const uint32_t* len) {
    p->n_req = n_req;
    p->n_lists = n_lists;
    p->cfirst.assign(n_lists + 1, 0);
    p->cidx.clear();
    p->cidx.reserve(first[n_lists]);
    std::vector<uint32_t> needed(n_req, UINT32_MAX);
    for (uint32_t k = 0; k < n_lists; k++) {
        uint32_t ord = 0;
        for (uint32_t e = first[k]; e < first[k + 1]; e++) {
            if (idx[e] == MIRSHA_NULL_INDEX) continue;  // empty digest: contributes no bytes
            p->cidx.push_back(idx[e]);
            needed[idx[e]] = std::min(needed[idx[e]], ord);
            ord++;
        }
        p->cfirst[k + 1] = (uint32_t)p->cidx.size();
    }
    p->n_entries = (uint32_t)p->cidx.size();
    if (n_req > (1u << 26)) return fail(c, MIRSHA_ERANGE, "fused plan: %u requests > 2^26", n_req);
    // Processing order: needed-at ordinal ascending (unlisted last), then
    // block count descending (length bucketing inside a wave).
    p->order.resize(n_req);
    for (uint32_t r = 0; r < n_req; r++) p->order[r] = r;
    std::stable_sort(p->order.begin(), p->order.end(), [&](uint32_t x, uint32_t y) {
        if (needed[x] != needed[y]) return needed[x] < needed[y];
        return len ? host_blocks(len[x]) > host_blocks(len[y]) : false;
    });
    std::vector<uint32_t> pos_of(n_req);
    for (uint32_t i = 0; i < n_req; i++) pos_of[p->order[i]] = i;
    p->n_tiles = (n_req + 63u) / 64u;
    p->n_groups = (n_lists + 63u) / 64u;
    // Counters: group g owns chunks [cbase[g], cbase[g+1]).
    constexpr uint32_t K = mirsha::kFusedChunkBlocks;
    p->cbase.assign(p->n_groups + 1, 0);
    for (uint32_t g = 0; g < p->n_groups; g++) {
        uint32_t nbmax = 0;
        for (uint32_t k = 64u * g; k < std::min(n_lists, 64u * g + 64u); k++)
            nbmax = std::max(nbmax, host_blocks(32u * (p->cfirst[k + 1] - p->cfirst[k])));
        p->cbase[g + 1] = p->cbase[g] + (nbmax + K - 1u) / K;
    }
    p->n_counters = p->cbase[p->n_groups];
    std::vector<uint64_t> pairs;
    pairs.reserve(p->n_entries);
    for (uint32_t k = 0; k < n_lists; k++) {
        const uint32_t cb = p->cbase[k >> 6];
        for (uint32_t e = p->cfirst[k]; e < p->cfirst[k + 1]; e++) {
            const uint32_t o = e - p->cfirst[k];
            pairs.push_back(((uint64_t)(pos_of[p->cidx[e]] >> 6) << 32) | (cb + (o >> 1) / K));
        }
    }
    std::sort(pairs.begin(), pairs.end());
    pairs.erase(std::unique(pairs.begin(), pairs.end()), pairs.end());
    p->tadj_first.assign(p->n_tiles + 1, 0);
    p->tadj.resize(pairs.size());
    p->expected.assign(std::max<uint32_t>(p->n_counters, 1), 0);
    for (size_t i = 0; i < pairs.size(); i++) {
        p->tadj_first[(pairs[i] >> 32) + 1]++;
        p->tadj[i] = (uint32_t)pairs[i];
        p->expected[(uint32_t)pairs[i]]++;
    }
    for (uint32_t t = 0; t < p->n_tiles; t++) p->tadj_first[t + 1] += p->tadj_first[t];
    // Grid: one block per CU.  List blocks (one producer / consumer pair each
    // on two SIMDs of an otherwise empty CU: a chain is latency-bound; group
    // g on list block g mod list_blocks) + tile blocks on the remaining CUs with
    // `pace` tile waves per SIMD, one per tile queue: queue q = the q-th run of
    // W = 4 x tile_blocks tiles in needed-at order (the last queue takes the
    // rest), served at issue priority 3 for queue 0 down to 0 for the last.
    // MIRSHA_FUSED_PACE (1..4, A/B) overrides the default.
    hipDeviceProp_t prop;
    HIP_TRY(c, hipGetDeviceProperties(&prop, c->device));
    const uint32_t cus = (uint32_t)prop.multiProcessorCount;
    p->pace = kFusedDefaultPace;
    if (const char* e = mirsha::ab_getenv("MIRSHA_FUSED_PACE"))
        p->pace = std::min<uint32_t>(mirsha::kPacedMaxPace, std::max<uint32_t>(1u, (uint32_t)atoi(e)));
    // one list pair per group, up to kFusedMaxListBlocks CUs (more groups: each pair takes several)
    p->list_blocks = std::min<uint32_t>(std::min<uint32_t>(p->n_groups, kFusedMaxListBlocks), cus / 8u);
    // List blocks' other waves as tile waves (MIRSHA_FUSED_LIST_TILES, A/B):
    // config 3's 4,096 tiles otherwise leave 144 as a fifth tile on the 988
    // SIMDs of the tile blocks.
    p->list_tiles = kFusedDefaultListTiles;
    if (const char* e = mirsha::ab_getenv("MIRSHA_FUSED_LIST_TILES")) p->list_tiles = std::min<uint32_t>(2u, (uint32_t)atoi(e));
    if (p->list_blocks == 0) p->list_tiles = 0;
    const uint32_t LB = p->list_blocks, P = p->pace;
    // tile waves of one list block per slot s (pair: slot 0 on SIMDs 0 and 1)
    auto lb_slot = [&](uint32_t s) -> uint32_t {
        return p->list_tiles == 0u ? 0u : p->list_tiles == 1u ? 2u : (s == 0u ? 2u : 4u);
    };
    uint32_t lb_tiles = 0;
    for (uint32_t s = 0; s < P; s++) lb_tiles += lb_slot(s);
    const uint32_t tile_blocks = std::max<uint32_t>(
        1, std::min<uint32_t>(cus - LB, (p->n_tiles - std::min(p->n_tiles, LB * lb_tiles) + 4u * P - 1u) / (4u * P)));
    p->tile_waves = tile_blocks * 4u * P + LB * lb_tiles;
    p->grid = LB + tile_blocks;
    // Queue q = the next (waves of slot q) tiles in needed-at order; the last takes the rest.
    uint32_t at = 0;
    for (uint32_t q = 0; q < P; q++) {
        p->q_first[q] = std::min<uint32_t>(p->n_tiles, at);
        p->q_waves[q] = 4u * tile_blocks + LB * lb_slot(q);
        at += p->q_waves[q];
    }
    p->tile_blocks = tile_blocks;
    p->q_first[P] = p->n_tiles;
    for (uint32_t q = 0; q < P; q++) p->q_end[q] = p->q_first[q + 1];
    // Split tiles (FusedArgs::n_split): tiles beyond the tile waves' slots
    // would run as a fifth tile on some SIMDs (config 3: 72 of 4,096, ending
    // ~130 us after the rest, profiles/r02af).  Instead each is cut into
    // block-range segments, one per host SIMD (the last queue's wave of every
    // tile-block SIMD), so the overflow spreads over the whole grid.
    p->n_split = p->seg_per_tile = p->seg_nominal_nb = 0;
    p->seg_nb.clear();
    const uint32_t hosts = 4u * tile_blocks;
    if (len && p->n_tiles > p->tile_waves) {
        const uint32_t ns = p->n_tiles - p->tile_waves;
        auto tile_blocks_of = [&](uint32_t t) {
            uint32_t m = 0;
            for (uint32_t i = 64u * t; i < std::min(n_req, 64u * t + 64u); i++)
                m = std::max(m, host_blocks(len[p->order[i]]));
            return m;
        };
        // Segment k runs when its host's own tile reaches block k * nom / S:
        // nom = the median block count of the hosts' own tiles (the last
        // queue's).  Only a schedule: a host whose own tile is shorter runs
        // its segment after that tile.
        // Which tiles split: with 2+ queues the first ns of the last queue.
        // Their chains of segments end before the last queue's tiles (the
        // hosts ARE that queue's waves), so in needed-at order they go before
        // it: the lists' final stretch, computed after the last tiles land,
        // is then only the last queue's positions.  With one queue, the last.
        const uint32_t sf = P >= 2 ? p->q_first[P - 1] : p->n_tiles - ns;
        std::vector<uint32_t> own;
        for (uint32_t t = p->q_first[P - 1]; t < p->n_tiles; t++)
            if (t < sf || t >= sf + ns) own.push_back(tile_blocks_of(t));
        std::vector<uint32_t> snb;
        for (uint32_t t = sf; t < sf + ns; t++) snb.push_back(tile_blocks_of(t));
        const uint32_t smax = *std::max_element(snb.begin(), snb.end());
        const uint32_t S = std::min(hosts / ns, smax);
        if (S >= 2 && !own.empty()) {
            std::nth_element(own.begin(), own.begin() + own.size() / 2, own.end());
            p->n_split = ns;
            p->split_first = sf;
            p->seg_per_tile = S;
            p->seg_nominal_nb = std::max(1u, own[own.size() / 2]);
            p->seg_nb = snb;
            if (P >= 2) {
                p->q_first[P - 1] += ns;  // (q_end[P - 2] stays sf: the split tiles belong to no queue)
            } else {
                p->q_first[P] = p->n_tiles - ns;
                p->q_end[0] = p->n_tiles - ns;
            }
        }
    }
    // Device copies.
    auto up = [&](DevBuf& d, const void* h, size_t bytes) -> int {
        HIP_TRY(c, d.ensure(std::max<size_t>(bytes, 4)));
        if (bytes) {
            HIP_TRY(c, hipMemcpyAsync(d.p, h, bytes, hipMemcpyHostToDevice, c->stream));
            HIP_TRY(c, hipStreamSynchronize(c->stream));
        }
        return MIRSHA_OK;
    };
    if (int rc = up(p->d_cidx, p->cidx.data(), sizeof(uint32_t) * p->n_entries)) return rc;
    if (int rc = up(p->d_cfirst, p->cfirst.data(), sizeof(uint32_t) * (n_lists + 1))) return rc;
    if (int rc = up(p->d_order, p->order.data(), sizeof(uint32_t) * n_req)) return rc;
    if (int rc = up(p->d_tadj_first, p->tadj_first.data(), sizeof(uint32_t) * (p->n_tiles + 1))) return rc;
    if (int rc = up(p->d_tadj, p->tadj.data(), sizeof(uint32_t) * p->tadj.size())) return rc;
    if (int rc = up(p->d_cbase, p->cbase.data(), sizeof(uint32_t) * (p->n_groups + 1))) return rc;
    if (int rc = up(p->d_expected, p->expected.data(), sizeof(uint32_t) * p->expected.size())) return rc;
    HIP_TRY(c, p->d_counters.ensure(8ull * std::max<uint32_t>(p->n_counters, 1)));
    HIP_TRY(c, hipMemsetAsync(p->d_counters.p, 0, 8ull * std::max<uint32_t>(p->n_counters, 1), c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    HIP_TRY(c, p->d_ctl.ensure(8ull * mirsha::kCtlWords));
    HIP_TRY(c, hipMemsetAsync(p->d_ctl.p, 0, 8ull * mirsha::kCtlWords, c->stream));
    if (p->n_split) {
        if (int rc = up(p->d_seg_nb, p->seg_nb.data(), sizeof(uint32_t) * p->n_split)) return rc;
        HIP_TRY(c, p->d_seg_state.ensure(2048ull * p->n_split));
        HIP_TRY(c, p->d_seg_flags.ensure(128ull * p->n_split));
        HIP_TRY(c, hipMemsetAsync(p->d_seg_flags.p, 0, 128ull * p->n_split, c->stream));
    }
    p->seg_runs = 0;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (!p->h_err) {
        void* h = nullptr;
        HIP_TRY(c, hipHostMalloc(&h, 64, hipHostMallocMapped | hipHostMallocCoherent));
        p->h_err = static_cast<unsigned long long*>(h);
        void* d = nullptr;
        HIP_TRY(c, hipHostGetDevicePointer(&d, h, 0));
        p->d_err = static_cast<unsigned long long*>(d);
    }
    *reinterpret_cast<volatile unsigned long long*>(p->h_err) = 0ull;
    // Test-only (MIRSHA_AB=1): the readiness watchdog in 100 MHz ticks, e.g. 0
    // to force the fail-closed path (tests/test_gpu_parity.py).
    p->watchdog = mirsha::kFusedWatchdogTicks;
    if (const char* e = mirsha::ab_getenv("MIRSHA_TEST_FUSED_WATCHDOG")) p->watchdog = strtoull(e, nullptr, 10);
    p->epoch = 0;
    const char* tr = mirsha::ab_getenv("MIRSHA_FUSED_TRACE");
    p->trace = tr && atoi(tr) != 0;
    if (p->trace) {
        const size_t words = 3ull * p->n_tiles + 2ull * p->n_counters + p->n_groups;
        HIP_TRY(c, p->d_trace.ensure(8ull * std::max<size_t>(words, 1)));
        HIP_TRY(c, hipMemsetAsync(p->d_trace.p, 0, 8ull * std::max<size_t>(words, 1), c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
    }
    return MIRSHA_OK;
}

// The plan's sticky error word, read without a synchronisation: set by an
// earlier run's expired readiness wait, whose list digests were not written.
int fused_failed(mirsha_ctx* c, const mirsha_pipeline* p) {
    if (p->h_err && *reinterpret_cast<const volatile unsigned long long*>(p->h_err))
        return fail(c, MIRSHA_EHIP,
                    "fused pass: a list wave's readiness wait expired (watchdog); its list digests were not "
                    "written and the plan refuses further runs");
    return MIRSHA_OK;
}

// overlap_prev != NULL: overlapped cycles -- the chains hash the PREVIOUS
// cycle's request digests (complete: no readiness waits) while this launch's
// tiles hash the current cycle; overlap with overlap_prev == NULL: tiles only
// (the first cycle).
int fused_run(mirsha_ctx* c, mirsha_pipeline* p, const uint8_t* d_arena, uint64_t arena_len, const uint64_t* d_off,
              const uint32_t* d_len, uint8_t* d_req_out, uint8_t* d_list_out, bool overlap = false,
              const uint8_t* overlap_prev = nullptr) {
    if (p->n_tiles + p->n_groups == 0) return MIRSHA_OK;
    if (int rc = fused_failed(c, p)) return rc;
    mirsha::FusedArgs a{};
    a.arena = d_arena;
    a.off = d_off;
    a.len = d_len;
    a.order = p->d_order.as<uint32_t>();
    a.req_out = d_req_out;
    a.cidx = p->d_cidx.as<uint32_t>();
    a.cfirst = p->d_cfirst.as<uint32_t>();
    a.list_out = d_list_out;
    a.tadj_first = p->d_tadj_first.as<uint32_t>();
    a.tadj = p->d_tadj.as<uint32_t>();
    a.cbase = p->d_cbase.as<uint32_t>();
    a.expected = p->d_expected.as<uint32_t>();
    a.counters = p->d_counters.as<unsigned long long>();
    a.ctl = p->d_ctl.as<unsigned long long>();
    a.err = p->d_err;
    a.watchdog = p->watchdog;
    a.trace = p->trace ? p->d_trace.as<unsigned long long>() : nullptr;
    a.n_counters = p->n_counters;
    for (uint32_t q = 0; q <= mirsha::kFusedMaxQueues; q++) a.q_first[q] = p->q_first[std::min(q, p->pace)];
    for (uint32_t q = 0; q < mirsha::kFusedMaxQueues; q++) a.q_end[q] = q < p->pace ? p->q_end[q] : p->n_tiles;
    for (uint32_t q = 0; q < mirsha::kFusedMaxQueues; q++) a.q_waves[q] = q < p->pace ? p->q_waves[q] : 0u;
    a.tile_blocks = p->tile_blocks;
    a.n_queues = p->pace;
    a.steal_own_prio = getenv_flag("MIRSHA_FUSED_STEAL_PRIO") ? 1u : 0u;
    a.list_tiles = p->list_tiles;
    a.arena_len = (uint32_t)arena_len;
    a.n_req = p->n_req;
    a.n_entries = p->n_entries;
    a.n_lists = p->n_lists;
    a.epoch = overlap ? 0ull : p->epoch + 1ull;  // 0: every readiness target is 0 (no waits)
    a.list_digests = overlap ? overlap_prev : d_req_out;
    a.n_tiles = p->n_tiles;
    a.n_groups = (overlap && !overlap_prev) ? 0u : p->n_groups;
    a.list_waves = p->list_blocks;
    a.n_split = p->n_split;
    a.split_first = p->split_first;
    a.seg_per_tile = p->seg_per_tile;
    a.seg_nominal_nb = p->seg_nominal_nb;
    a.seg_epoch = p->seg_runs;
    // Overlapped cycles: no chain waits on these tiles, so no queue order to
    // keep: the SIMD's tile waves at priorities by progress rank (kPrioBalance).
    // A/B (MIRSHA_FUSED_OVERLAP_PRIO): queue = the fused launch's queue
    // priorities, progress = the request kernel's progress_prio.
    a.tile_prio_progress = overlap ? 2u : 0u;
    if (const char* e = mirsha::ab_getenv("MIRSHA_FUSED_OVERLAP_PRIO"))
        if (overlap) a.tile_prio_progress = strcmp(e, "queue") == 0 ? 0u : strcmp(e, "progress") == 0 ? 1u : 2u;
    a.test_placement = p->test_placement;
    // A tile wave left alone on its SIMD runs the latency round form
    // (FusedArgs::lone_form).  A/B: MIRSHA_FUSED_LONE_FORM=0.
    a.lone_form = 1u;
    if (const char* e = mirsha::ab_getenv("MIRSHA_FUSED_LONE_FORM")) a.lone_form = atoi(e) != 0 ? 1u : 0u;
    // The last queue's tile waves stage two blocks ahead (FusedArgs::deep_last).
    // A/B: MIRSHA_FUSED_DEEP_LAST=0.
    a.deep_last = overlap ? 0u : 1u;  // (overlapped launches: no lone stretch, and one DMA in flight keeps
                                      // the progress ranks' LDS wait free, hash_tile)
    if (const char* e = mirsha::ab_getenv("MIRSHA_FUSED_DEEP_LAST")) a.deep_last = atoi(e) != 0 ? 1u : 0u;
    a.seg_nb = p->d_seg_nb.as<uint32_t>();
    a.seg_state = p->d_seg_state.as<uint32_t>();
    a.seg_flags = p->d_seg_flags.as<unsigned long long>();
    if (int rc = timed_launch(c, 4, [&] { return mirsha::launch_fused_paced(a, p->grid, p->pace, c->stream); }))
        return rc;
    p->epoch++;
    p->seg_runs++;
    return MIRSHA_OK;
}

int fused_status(mirsha_ctx* c, mirsha_pipeline* p) {
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (p->mode != MIRSHA_PIPELINE_FUSED) return MIRSHA_OK;
    return fused_failed(c, p);
}

// AUTO: the fused launch pays when a few LONG chains would otherwise run after
// the request pass (VerifyBatch of hundreds of digests, BASELINE config 3:
// 1.49 -> 1.04 ms); many short lists (BatchSize 20, config 2) run better as
// the request kernel at full occupancy followed by the list kernel.
bool fused_pays(const uint32_t* idx, const uint32_t* first, uint32_t n_lists) {
    if (n_lists == 0 || (n_lists + 63u) / 64u > kFusedMaxListWaves) return false;
    uint32_t maxc = 0;
    for (uint32_t k = 0; k < n_lists; k++) {
        uint32_t c = 0;
        for (uint32_t e = first[k]; e < first[k + 1]; e++) c += idx[e] != MIRSHA_NULL_INDEX;
        maxc = std::max(maxc, c);
    }
    return host_blocks(32u * maxc) >= kFusedMinChainBlocks;
}

// The fused launch's static roles (first tiles, pair, segment hosts) are
// dealt by (SIMD, slot) and assume a workgroup's waves land P per SIMD
// (cyclic dealing).  The kernel remaps any other placement so a run stays
// complete, but stacked waves would run slower than the sequential plan: so
// a plan whose probe finds any block of the launch's shape placed otherwise
// is built SEQUENTIAL (mirsha_pipeline_fallback reports it).  Test knob
// (MIRSHA_AB=1): MIRSHA_TEST_PLACEMENT=broken makes the probe report a
// broken placement, =remap makes the fused kernel's waves all read SIMD 0
// (the in-kernel remap, plan stays fused).
void pipeline_free(mirsha_pipeline* p);

int fused_placement_ok(mirsha_ctx* c, mirsha_pipeline* p, bool& ok) {
    ok = true;
    if (p->grid == 0) return MIRSHA_OK;
    const char* t = mirsha::ab_getenv("MIRSHA_TEST_PLACEMENT");
    const uint32_t test = (t && strcmp(t, "broken") == 0) ? 1u : 0u;
    p->test_placement = (t && strcmp(t, "remap") == 0) ? 1u : 0u;
    DevBuf& flag = p->d_probe;
    HIP_TRY(c, flag.ensure(4));
    HIP_TRY(c, hipMemsetAsync(flag.p, 0, 4, c->stream));
    HIP_TRY(c, mirsha::launch_placement_probe(p->grid, p->pace, flag.as<uint32_t>(), test, c->stream));
    uint32_t broken = 0;
    HIP_TRY(c, hipMemcpyAsync(&broken, flag.p, 4, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    ok = broken == 0;
    return MIRSHA_OK;
}

int plan_build(mirsha_ctx* c, mirsha_pipeline* p, uint32_t n_req, const uint32_t* idx, const uint32_t* first,
               uint32_t n_lists, const uint32_t* len) {
    if (p->mode == MIRSHA_PIPELINE_AUTO)
        p->mode = fused_pays(idx, first, n_lists) ? MIRSHA_PIPELINE_FUSED : MIRSHA_PIPELINE_SEQUENTIAL;
    if (p->mode == MIRSHA_PIPELINE_FUSED) {
        if (int rc = fused_build(c, p, n_req, idx, first, n_lists, len)) return rc;
        bool ok = true;
        if (int rc = fused_placement_ok(c, p, ok)) return rc;
        if (ok) return MIRSHA_OK;
        pipeline_free(p);  // degrade: the two-kernel plan, which assumes no placement
        p->mode = MIRSHA_PIPELINE_SEQUENTIAL;
        p->fallback = 1;
    }
    return pipeline_build(c, p, n_req, idx, first, n_lists, len);
}

int plan_run(mirsha_ctx* c, mirsha_pipeline* p, const uint8_t* d_arena, uint64_t arena_len, const uint64_t* d_off,
             const uint32_t* d_len, uint8_t* d_req_out, uint8_t* d_list_out) {
    if (p->mode == MIRSHA_PIPELINE_FUSED) return fused_run(c, p, d_arena, arena_len, d_off, d_len, d_req_out, d_list_out);
    return pipeline_run(c, p, d_arena, arena_len, d_off, d_len, d_req_out, d_list_out);
}

int default_pipeline_mode() {
    const char* m = getenv("MIRSHA_PIPELINE_MODE");
    if (m && strcmp(m, "sequential") == 0) return MIRSHA_PIPELINE_SEQUENTIAL;
    if (m && strcmp(m, "fused") == 0) return MIRSHA_PIPELINE_FUSED;
    return MIRSHA_PIPELINE_AUTO;
}

void pipeline_free(mirsha_pipeline* p) {
    p->d_cidx.release();
    p->d_cfirst.release();
    p->d_order.release();
    p->d_state.release();
    p->d_tadj_first.release();
    p->d_tadj.release();
    p->d_cbase.release();
    p->d_expected.release();
    p->d_counters.release();
    p->d_ctl.release();
    p->d_trace.release();
    p->d_seg_nb.release();
    p->d_seg_state.release();
    p->d_seg_flags.release();
    p->d_probe.release();
    if (p->h_err) (void)hipHostFree(p->h_err);
    p->h_err = p->d_err = nullptr;
}


// Validates a slice-list request set and returns each request's total length.
// The first request with a per-request slice error (err[i]: 0 ok, 1 not
// monotone, 2 NULL slice, 3 too long), reported as the call's error.
int slice_errors(mirsha_ctx* c, const uint8_t* err, uint32_t n) {
    for (uint32_t i = 0; i < n; i++) {
        if (err[i] == 1) return fail(c, MIRSHA_EINVAL, "slice_first not monotone at request %u", i);
        if (err[i] == 2) return fail(c, MIRSHA_EINVAL, "request %u has a NULL slice", i);
        if (err[i] == 3) return fail(c, MIRSHA_ERANGE, "request %u exceeds %u bytes", i, MIRSHA_MAX_MESSAGE_BYTES);
    }
    return MIRSHA_OK;
}

// The call-level checks every slice submission makes first.
int slice_args(mirsha_ctx* c, const uint8_t* const* slice_ptr, const uint64_t* slice_len, const uint32_t* slice_first,
               uint32_t n, const uint8_t* out) {
    if (!slice_first || !out) return fail(c, MIRSHA_EINVAL, "NULL argument");
    if (slice_first[0] != 0) return fail(c, MIRSHA_EINVAL, "slice_first[0] must be 0");
    if (slice_first[n] && (!slice_ptr || !slice_len)) return fail(c, MIRSHA_EINVAL, "NULL slice arrays");
    return MIRSHA_OK;
}

int slice_lengths(mirsha_ctx* c, const uint8_t* const* slice_ptr, const uint64_t* slice_len,
                  const uint32_t* slice_first, uint32_t n, const uint8_t* out, std::vector<uint32_t>& len) {
    if (int rc = slice_args(c, slice_ptr, slice_len, slice_first, n, out)) return rc;
    const uint32_t ns = slice_first[n];
    len.resize(n);
    // err[i]: 0 ok, 1 not monotone, 2 NULL slice, 3 too long (first error reported)
    std::vector<uint8_t> err(n, 0);
    const uint64_t meta = 16ull * (ns > slice_first[0] ? ns : 0u);
    mirsha::host::parallel_for(n, mirsha::host::threads_for(meta, n), [&](uint32_t lo, uint32_t hi) {
        for (uint32_t i = lo; i < hi; i++) {
            if (slice_first[i + 1] < slice_first[i] || slice_first[i + 1] > ns) { err[i] = 1; continue; }
            uint64_t L = 0;
            for (uint32_t s = slice_first[i]; s < slice_first[i + 1]; s++) {
                if (slice_len[s] && !slice_ptr[s]) { err[i] = 2; break; }
                L += slice_len[s];
            }
            if (!err[i] && L > MIRSHA_MAX_MESSAGE_BYTES) err[i] = 3;
            len[i] = (uint32_t)L;
        }
    });
    return slice_errors(c, err.data(), n);
}

// Copies a completed submission's digests to the caller, in origin order.
int async_complete(mirsha_ctx* c, AsyncSlot& sl) {
    HIP_TRY(c, hipEventSynchronize(sl.done));
    const auto t_done = Clock::now();
    sl.prof[MIRSHA_PROF_DEVICE] = std::chrono::duration<double, std::milli>(t_done - sl.t_queued).count();
    const uint8_t* d = sl.dig.as<uint8_t>();
    if (sl.rank.empty()) {
        memcpy(sl.user_out, d, 32ull * sl.n);
    } else {
        for (uint32_t i = 0; i < sl.n; i++) memcpy(sl.user_out + 32ull * i, d + 32ull * sl.rank[i], 32);
    }
    sl.busy = false;
    c->done_ticket = std::max(c->done_ticket, sl.ticket);
    sl.prof[MIRSHA_PROF_SCATTER] = ms_since(t_done);
    sl.prof[MIRSHA_PROF_CHUNKS] = 0;
    // mirsha_ctx_host_profile: every phase of ONE submission, the most
    // recently completed (not one ticket's plan beside another's device time)
    for (int k = 0; k < MIRSHA_PROF_PHASES; k++) c->prof[k] = sl.prof[k];
    return MIRSHA_OK;
}

int async_wait_upto(mirsha_ctx* c, uint64_t ticket) {
    for (uint64_t t = c->done_ticket + 1; t <= ticket; t++) {
        AsyncSlot& sl = c->slots[(t - 1) % kAsyncSlots];
        if (sl.busy && sl.ticket == t)
            if (int rc = async_complete(c, sl)) return rc;
    }
    return MIRSHA_OK;
}

constexpr uint64_t align8(uint64_t x) { return (x + 7u) & ~7ull; }

int async_submit(mirsha_ctx* c, const uint8_t* const* slice_ptr, const uint64_t* slice_len,
                 const uint32_t* slice_first, uint32_t n, uint8_t* out, int flags, uint64_t* ticket_out,
                 uint32_t* n_unique_out) {
    if (flags & ~MIRSHA_SUBMIT_DEDUP) return fail(c, MIRSHA_EINVAL, "unknown submit flags 0x%x", flags);
    auto t0 = Clock::now();
    // Which requests reach the GPU: all, or one per distinct content.  With
    // dedup the requests are scanned in segments in origin order
    // (mirsha::host::DedupScan): the first segment's heads (distinct
    // contents, each a final representative) are packed and queued as soon as
    // that segment is scanned, and the GPU hashes them while the host scans
    // and confirms the rest -- a request matching an earlier head is compared
    // byte for byte in the same walk, while its bytes are cache-warm.
    // Representatives found later (new contents of later segments, and
    // fingerprint collisions, rare) follow in one second launch.
    const bool dedup = (flags & MIRSHA_SUBMIT_DEDUP) && n > 1;
    double ph[MIRSHA_PROF_PHASES] = {};
    std::vector<uint32_t> len;
    if (dedup) {
        if (int rc = slice_args(c, slice_ptr, slice_len, slice_first, n, out)) return rc;
        len.assign(n, 0u);
    } else if (n) {
        if (int rc = slice_lengths(c, slice_ptr, slice_len, slice_first, n, out, len)) return rc;
    }
    ph[MIRSHA_PROF_VALIDATE] = ms_since(t0);
    t0 = Clock::now();
    if (int rc = use_device(c)) return rc;
    AsyncSlot& sl = c->slots[(c->next_ticket - 1) % kAsyncSlots];
    if (sl.busy)
        if (int rc = async_wait_upto(c, sl.ticket)) return rc;  // ring full: retire the oldest
    sl.rank.clear();
    HIP_TRY(c, sl.dig.ensure(32ull * std::max<uint32_t>(n, 1)));
    if (!sl.done) HIP_TRY(c, hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
    ph[MIRSHA_PROF_PLAN] = ms_since(t0);
    // Packs requests `ids` (identity when null) into `stage`, and queues their
    // digests into rows [row0, row0 + m) of sl.dig.
    auto queue = [&](const uint32_t* ids, uint32_t m, uint32_t row0, PinnedBuf& stage, DevBuf& dev) -> int {
        const auto tq = Clock::now();
        std::vector<uint64_t> poff(m);
        std::vector<uint32_t> plen(m);
        uint64_t bytes = 0;
        for (uint32_t k = 0; k < m; k++) {
            const uint32_t i = ids ? ids[k] : k;
            poff[k] = bytes;
            plen[k] = len[i];
            bytes += len[i];
        }
        if (bytes + kArenaSlack > MIRSHA_MAX_DEVICE_ARENA_BYTES)
            return fail(c, MIRSHA_ERANGE, "submission of %llu bytes exceeds one device arena (%u); split it",
                        (unsigned long long)bytes, MIRSHA_MAX_DEVICE_ARENA_BYTES);
        const uint64_t o_off = align8(bytes + kArenaSlack);
        const uint64_t o_len = o_off + 8ull * m, o_ord = o_len + 4ull * m, o_end = align8(o_ord + 4ull * m);
        const uint64_t o_dig = o_end;
        HIP_TRY(c, stage.ensure(o_end));
        HIP_TRY(c, dev.ensure(o_dig + 32ull * std::max<uint32_t>(m, 1)));
        uint8_t* st = stage.as<uint8_t>();
        mirsha::host::pack(slice_ptr, slice_len, slice_first, ids, m, poff.data(), st,
                           mirsha::host::threads_for(bytes, m));
        memcpy(st + o_off, poff.data(), 8ull * m);
        memcpy(st + o_len, plen.data(), 4ull * m);
        const bool identity = bucket_order(plen.data(), m, reinterpret_cast<uint32_t*>(st + o_ord));
        uint8_t* dv = dev.as<uint8_t>();
        if (m) {
            HIP_TRY(c, hipMemcpyAsync(dv, st, o_end, hipMemcpyHostToDevice, c->stream));
            int rc = timed_launch(c, 0, [&] {
                return mirsha::launch_msgs(dv, bytes, reinterpret_cast<const uint64_t*>(dv + o_off),
                                           reinterpret_cast<const uint32_t*>(dv + o_len),
                                           identity ? nullptr : reinterpret_cast<const uint32_t*>(dv + o_ord), m,
                                           dv + o_dig, c->variant, c->stream);
            });
            if (rc) return rc;
            HIP_TRY(c, hipMemcpyAsync(sl.dig.as<uint8_t>() + 32ull * row0, dv + o_dig, 32ull * m,
                                      hipMemcpyDeviceToHost, c->stream));
        }
        ph[MIRSHA_PROF_PACK] += ms_since(tq);
        return MIRSHA_OK;
    };
    uint32_t m = n;
    if (!dedup) {
        if (int rc = queue(nullptr, n, 0, sl.stage, sl.dev)) return rc;
        sl.t_queued = Clock::now();
    } else {
        mirsha::host::DedupScan d(slice_ptr, slice_len, slice_first, n, MIRSHA_MAX_MESSAGE_BYTES);
        const std::vector<uint32_t> seg = d.segments();
        std::vector<uint32_t> first_heads, later;  // the first launch's rows, then the second's
        bool queued = false;
        for (size_t k = 0; k + 1 < seg.size(); k++) {
            const uint32_t lo = seg[k], hi = seg[k + 1];
            t0 = Clock::now();
            const bool ok = d.scan(lo, hi);
            ph[MIRSHA_PROF_VALIDATE] += ms_since(t0);
            if (!ok) {
                // the first launch still reads this slot's buffers: let it finish
                if (queued) HIP_TRY(c, hipStreamSynchronize(c->stream));
                return slice_errors(c, d.err(), n);
            }
            t0 = Clock::now();
            for (uint32_t i = lo; i < hi; i++) len[i] = (uint32_t)d.req_len()[i];
            d.assign(lo, hi, k == 0 ? first_heads : later);
            ph[MIRSHA_PROF_PLAN] += ms_since(t0);
            if (k == 0) {
                if (int rc = queue(first_heads.data(), (uint32_t)first_heads.size(), 0, sl.stage, sl.dev))
                    return rc;
                queued = true;
                sl.t_queued = Clock::now();
            }
            t0 = Clock::now();
            d.confirm(lo, hi);
            ph[MIRSHA_PROF_PLAN] += ms_since(t0);
        }
        t0 = Clock::now();
        std::vector<uint32_t> rep(n);
        const uint32_t distinct = d.resolve(rep.data(), &later);  // collisions appended to `later`
        const uint32_t m0 = (uint32_t)first_heads.size();
        m = m0 + (uint32_t)later.size();
        if (m != distinct) return fail(c, MIRSHA_EHIP, "dedup: %u representatives for %u contents", m, distinct);
        sl.rank.resize(n);
        for (uint32_t k = 0; k < m0; k++) sl.rank[first_heads[k]] = k;
        for (uint32_t k = 0; k < (uint32_t)later.size(); k++) sl.rank[later[k]] = m0 + k;
        bool identity = true;
        for (uint32_t i = 0; i < n; i++) {
            sl.rank[i] = sl.rank[rep[i]];
            identity &= sl.rank[i] == i;
        }
        if (identity) sl.rank.clear();  // all distinct, rows already in origin order
        ph[MIRSHA_PROF_PLAN] += ms_since(t0);
        if (!later.empty())
            if (int rc = queue(later.data(), (uint32_t)later.size(), m0, sl.stage2, sl.dev2)) return rc;
    }
    if (n_unique_out) *n_unique_out = m;
    HIP_TRY(c, hipEventRecord(sl.done, c->stream));
    sl.busy = true;
    sl.user_out = out;
    sl.n = n;
    sl.m = m;
    sl.ticket = c->next_ticket++;
    for (int k = 0; k < MIRSHA_PROF_PHASES; k++) sl.prof[k] = ph[k];
    if (ticket_out) *ticket_out = sl.ticket;
    return MIRSHA_OK;
}

}  // namespace

extern "C" {

int mirsha_version(void) { return (0 << 16) | 1; }

int mirsha_device_count(int* count) {
    if (!count) return MIRSHA_EINVAL;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        n = 0;
    }
    *count = n;
    return MIRSHA_OK;
}

int mirsha_ctx_create(int device, mirsha_ctx** out) {
    if (!out) return MIRSHA_EINVAL;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        (void)hipGetLastError();
        return MIRSHA_ENODEV;
    }
    if (device < 0 || device >= n) return MIRSHA_EINVAL;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return MIRSHA_EHIP;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return MIRSHA_ENODEV;  // gfx950 code objects only
    mirsha_ctx* c = new mirsha_ctx();
    c->device = device;
    if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return MIRSHA_EHIP;
    }
    c->stream = c->own;
    *out = c;
    return MIRSHA_OK;
}

void mirsha_ctx_destroy(mirsha_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->device);
    (void)hipStreamSynchronize(c->stream);
    for (auto& t : c->timers) {
        for (auto& pr : t.pending) { (void)hipEventDestroy(pr.first); (void)hipEventDestroy(pr.second); }
        for (auto e : t.pool) (void)hipEventDestroy(e);
    }
    c->d_arena.release(); c->d_off.release(); c->d_len.release(); c->d_order.release();
    c->d_out.release(); c->d_idx.release(); c->d_first.release(); c->d_out2.release(); c->d_scratch.release();
    c->d_scan.release();
    for (int k = 0; k < kStageSlots; k++) {
        c->h_ring[k].release();
        if (c->ring_ev[k]) (void)hipEventDestroy(c->ring_ev[k]);
    }
    c->h_meta.release();
    c->h_outs.release();
    c->d_meta.release();
    for (auto e : c->xev) (void)hipEventDestroy(e);
    if (c->xin) (void)hipStreamDestroy(c->xin);
    if (c->xout) (void)hipStreamDestroy(c->xout);
    for (auto& sl : c->slots) {
        sl.stage.release(); sl.dig.release(); sl.dev.release(); sl.stage2.release(); sl.dev2.release();
        if (sl.done) (void)hipEventDestroy(sl.done);
    }
    if (c->own) (void)hipStreamDestroy(c->own);
    delete c;
}

const char* mirsha_last_error(const mirsha_ctx* c) { return c ? c->err.c_str() : "null context"; }

int mirsha_ctx_set_stream(mirsha_ctx* c, void* s) {
    if (!c) return MIRSHA_EINVAL;
    c->stream = s ? static_cast<hipStream_t>(s) : c->own;
    return MIRSHA_OK;
}

void* mirsha_ctx_stream(mirsha_ctx* c) { return c ? static_cast<void*>(c->stream) : nullptr; }

int mirsha_ctx_set_variant(mirsha_ctx* c, int v) {
    if (!c || !mirsha::variant_valid(v)) return MIRSHA_EINVAL;
    c->variant = v;
    return MIRSHA_OK;
}

int mirsha_ctx_set_timing(mirsha_ctx* c, int enable) {
    if (!c) return MIRSHA_EINVAL;
    c->timing = enable != 0;
    return MIRSHA_OK;
}

int mirsha_ctx_kernel_time(mirsha_ctx* c, int which, uint64_t* launches, double* total_ms) {
    if (!c || which < 0 || which > 5) return MIRSHA_EINVAL;
    if (int rc = use_device(c)) return rc;
    KernelTimer& t = c->timers[which];
    for (auto& pr : t.pending) {
        HIP_TRY(c, hipEventSynchronize(pr.second));
        float ms = 0.f;
        HIP_TRY(c, hipEventElapsedTime(&ms, pr.first, pr.second));
        t.ms += ms;
        t.launches++;
        t.pool.push_back(pr.first);
        t.pool.push_back(pr.second);
    }
    t.pending.clear();
    if (launches) *launches = t.launches;
    if (total_ms) *total_ms = t.ms;
    return MIRSHA_OK;
}

int mirsha_ctx_set_timing_mask(mirsha_ctx* c, uint32_t mask) {
    if (!c) return MIRSHA_EINVAL;
    c->time_mask = mask;
    return MIRSHA_OK;
}

int mirsha_ctx_reset_timing(mirsha_ctx* c) {
    if (!c) return MIRSHA_EINVAL;
    for (int k = 0; k < 6; k++) {
        int rc = mirsha_ctx_kernel_time(c, k, nullptr, nullptr);
        if (rc) return rc;
        c->timers[k].launches = 0;
        c->timers[k].ms = 0.0;
    }
    return MIRSHA_OK;
}

int mirsha_sync(mirsha_ctx* c) {
    if (!c) return MIRSHA_EINVAL;
    if (int rc = use_device(c)) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return MIRSHA_OK;
}

int mirsha_hash_batch(mirsha_ctx* c, const uint8_t* arena, uint64_t arena_len, const uint64_t* off,
                      const uint32_t* len, uint32_t n, uint8_t* out) {
    if (!c) return MIRSHA_EINVAL;
    if (n == 0) return MIRSHA_OK;
    if (!off || !len || !out || (!arena && arena_len)) return fail(c, MIRSHA_EINVAL, "NULL argument");
    if (int rc = use_device(c)) return rc;
    return run_arena_call(c, arena, arena_len, off, len, n, nullptr, nullptr, 0, out, nullptr);
}


int mirsha_hash_slices(mirsha_ctx* c, const uint8_t* const* slice_ptr, const uint64_t* slice_len,
                       const uint32_t* slice_first, uint32_t n, uint8_t* out) {
    if (!c) return MIRSHA_EINVAL;
    if (n == 0) return MIRSHA_OK;
    const auto t0 = Clock::now();
    for (double& x : c->prof) x = 0.0;
    std::vector<uint32_t> len;
    if (int rc = slice_lengths(c, slice_ptr, slice_len, slice_first, n, out, len)) return rc;
    c->prof[MIRSHA_PROF_VALIDATE] = ms_since(t0);
    if (int rc = use_device(c)) return rc;
    // One packing pass, by threads, straight into pinned staging (the Go
    // side's single copy), chunk by chunk behind the DMA of the previous one.
    std::vector<uint64_t> poff(n);
    uint64_t p = 0;
    for (uint32_t i = 0; i < n; i++) {
        poff[i] = p;
        p += len[i];
    }
    ArenaSrc src;
    src.ptr = slice_ptr;
    src.slen = slice_len;
    src.sfirst = slice_first;
    src.poff = poff.data();
    src.n = n;
    src.total = p;
    const int rc = run_staged(c, src, poff.data(), len.data(), n, 0, kGapless, nullptr, nullptr, 0, out, nullptr);
    c->prof[MIRSHA_PROF_TOTAL] = ms_since(t0);
    return rc;
}

int mirsha_host_alloc(mirsha_ctx* c, uint64_t bytes, void** out) {
    if (!c || !out) return MIRSHA_EINVAL;
    *out = nullptr;
    if (int rc = use_device(c)) return rc;
    HIP_TRY(c, hipHostMalloc(out, std::max<uint64_t>(bytes, 1), hipHostMallocDefault));
    return MIRSHA_OK;
}

void mirsha_host_free(void* p) {
    if (p) (void)hipHostFree(p);
}

int mirsha_hash_slices_dedup(mirsha_ctx* c, const uint8_t* const* slice_ptr, const uint64_t* slice_len,
                             const uint32_t* slice_first, uint32_t n, uint8_t* out, uint32_t* n_unique_out) {
    if (!c) return MIRSHA_EINVAL;
    if (n_unique_out) *n_unique_out = 0;
    if (n == 0) return MIRSHA_OK;
    uint64_t t = 0;
    if (int rc = async_submit(c, slice_ptr, slice_len, slice_first, n, out, MIRSHA_SUBMIT_DEDUP, &t, n_unique_out))
        return rc;
    return async_wait_upto(c, t);
}

int mirsha_submit_slices(mirsha_ctx* c, const uint8_t* const* slice_ptr, const uint64_t* slice_len,
                         const uint32_t* slice_first, uint32_t n, uint8_t* out, int flags, uint64_t* ticket_out) {
    if (!c || !ticket_out) return MIRSHA_EINVAL;
    return async_submit(c, slice_ptr, slice_len, slice_first, n, out, flags, ticket_out, nullptr);
}

int mirsha_wait(mirsha_ctx* c, uint64_t ticket) {
    if (!c) return MIRSHA_EINVAL;
    if (ticket == 0 || ticket >= c->next_ticket) return fail(c, MIRSHA_EINVAL, "unknown ticket %llu", (unsigned long long)ticket);
    if (ticket <= c->done_ticket) return MIRSHA_OK;
    if (int rc = use_device(c)) return rc;
    return async_wait_upto(c, ticket);
}

int mirsha_poll(mirsha_ctx* c, uint64_t ticket, int* done) {
    if (!c || !done) return MIRSHA_EINVAL;
    if (ticket == 0 || ticket >= c->next_ticket) return fail(c, MIRSHA_EINVAL, "unknown ticket %llu", (unsigned long long)ticket);
    *done = 0;
    if (ticket <= c->done_ticket) {
        *done = 1;
        return MIRSHA_OK;
    }
    if (int rc = use_device(c)) return rc;
    for (uint64_t t = c->done_ticket + 1; t <= ticket; t++) {
        AsyncSlot& sl = c->slots[(t - 1) % kAsyncSlots];
        const hipError_t q = hipEventQuery(sl.done);
        if (q == hipErrorNotReady) {
            (void)hipGetLastError();  // not an error (see run_pipelined)
            return MIRSHA_OK;
        }
        if (q != hipSuccess) return fail(c, MIRSHA_EHIP, "hipEventQuery: %s", hipGetErrorString(q));
    }
    if (int rc = async_wait_upto(c, ticket)) return rc;
    *done = 1;
    return MIRSHA_OK;
}

int mirsha_hash_requests_then_batches(mirsha_ctx* c, const uint8_t* arena, uint64_t arena_len,
                                      const uint64_t* off, const uint32_t* len, uint32_t n_req,
                                      const uint32_t* idx, const uint32_t* first, uint32_t n_batches,
                                      uint8_t* req_out, uint8_t* batch_out) {
    if (!c) return MIRSHA_EINVAL;
    if (n_req && (!off || !len || !req_out || (!arena && arena_len))) return fail(c, MIRSHA_EINVAL, "NULL argument");
    if (n_batches && !batch_out) return fail(c, MIRSHA_EINVAL, "batch_digests_out is NULL");
    if (n_batches)
        if (int rc = check_lists(c, idx, first, n_batches, n_req)) return rc;
    if (int rc = use_device(c)) return rc;
    // Per-call plans cost host sorting and device allocations, so the host API
    // uses a plan only when asked (MIRSHA_PIPELINE_MODE=fused|auto); the
    // device API (mirsha_pipeline_create + *_device) amortises one plan.
    const char* pmode = getenv("MIRSHA_PIPELINE_MODE");
    const bool pipelined = pmode && (strcmp(pmode, "fused") == 0 || strcmp(pmode, "auto") == 0);
    uint64_t lo = 0, hi = 0, total = 0;
    if (pipelined) {
        if (int rc = arena_span(c, arena_len, off, len, n_req, &lo, &hi)) return rc;
        for (uint32_t i = 0; i < n_req; i++) total += len[i];
    }
    const uint64_t span = n_req ? hi - lo : 0;
    if (pipelined && n_batches && n_req && span + kArenaSlack <= MIRSHA_MAX_DEVICE_ARENA_BYTES &&
        span <= 2 * total + 4096) {
        HIP_TRY(c, c->d_out.ensure(32ull * std::max<uint32_t>(n_req, 1)));
        mirsha_pipeline p;
        p.device = c->device;
        p.mode = default_pipeline_mode();
        int rc = plan_build(c, &p, n_req, idx, first, n_batches, len);
        if (rc == MIRSHA_OK) {
            std::vector<uint64_t> roff(off, off + n_req);
            for (auto& x : roff) x -= lo;
            HIP_TRY(c, c->d_arena.ensure(span + kArenaSlack));
            HIP_TRY(c, c->d_off.ensure(sizeof(uint64_t) * n_req));
            HIP_TRY(c, c->d_len.ensure(sizeof(uint32_t) * n_req));
            HIP_TRY(c, c->d_out2.ensure(32ull * n_batches));
            if (span) HIP_TRY(c, hipMemcpyAsync(c->d_arena.p, arena + lo, span, hipMemcpyHostToDevice, c->stream));
            HIP_TRY(c, hipMemcpyAsync(c->d_off.p, roff.data(), sizeof(uint64_t) * n_req, hipMemcpyHostToDevice, c->stream));
            HIP_TRY(c, hipMemcpyAsync(c->d_len.p, len, sizeof(uint32_t) * n_req, hipMemcpyHostToDevice, c->stream));
            rc = plan_run(c, &p, c->d_arena.as<uint8_t>(), span, c->d_off.as<uint64_t>(), c->d_len.as<uint32_t>(),
                          c->d_out.as<uint8_t>(), c->d_out2.as<uint8_t>());
            if (rc == MIRSHA_OK) rc = fused_status(c, &p);
            if (rc == MIRSHA_OK) {
                HIP_TRY(c, hipMemcpyAsync(batch_out, c->d_out2.p, 32ull * n_batches, hipMemcpyDeviceToHost, c->stream));
                HIP_TRY(c, hipMemcpyAsync(req_out, c->d_out.p, 32ull * n_req, hipMemcpyDeviceToHost, c->stream));
                HIP_TRY(c, hipStreamSynchronize(c->stream));
            }
        }
        (void)hipStreamSynchronize(c->stream);
        pipeline_free(&p);
        return rc;
    }
    // Staged path: request bytes at PCIe rate, metadata and digests in one
    // copy each way, request kernel then list kernel.
    if (n_req == 0 && n_batches == 0) return MIRSHA_OK;
    if (n_req == 0) {  // lists of null requests only (every entry is MIRSHA_NULL_INDEX)
        ArenaSrc none;
        return run_staged(c, none, nullptr, nullptr, 0, 0, kAnyOrder, idx, first, n_batches, nullptr, batch_out);
    }
    return run_arena_call(c, arena, arena_len, off, len, n_req, idx, first, n_batches, req_out, batch_out);
}

int mirsha_pipeline_create(mirsha_ctx* c, uint32_t n_req, const uint32_t* len, const uint32_t* idx,
                           const uint32_t* list_first, uint32_t n_lists, mirsha_pipeline** out) {
    return mirsha_pipeline_create_mode(c, n_req, len, idx, list_first, n_lists, default_pipeline_mode(), out);
}

int mirsha_pipeline_create_mode(mirsha_ctx* c, uint32_t n_req, const uint32_t* len, const uint32_t* idx,
                                const uint32_t* list_first, uint32_t n_lists, int mode, mirsha_pipeline** out) {
    if (!c || !out) return MIRSHA_EINVAL;
    *out = nullptr;
    if (mode != MIRSHA_PIPELINE_SEQUENTIAL && mode != MIRSHA_PIPELINE_FUSED && mode != MIRSHA_PIPELINE_AUTO)
        return fail(c, MIRSHA_EINVAL, "bad pipeline mode %d (sequential 0, fused 1, auto 3)", mode);
    if (int rc = check_lists(c, idx, list_first, n_lists, n_req)) return rc;
    if (int rc = use_device(c)) return rc;
    mirsha_pipeline* p = new mirsha_pipeline();
    p->device = c->device;
    p->mode = mode;
    int rc = plan_build(c, p, n_req, idx, list_first, n_lists, len);
    if (rc != MIRSHA_OK) {
        pipeline_free(p);
        delete p;
        return rc;
    }
    *out = p;
    return MIRSHA_OK;
}

void mirsha_pipeline_destroy(mirsha_pipeline* p) {
    if (!p) return;
    (void)hipSetDevice(p->device);
    pipeline_free(p);
    delete p;
}

int mirsha_pipeline_mode(const mirsha_pipeline* p) { return p ? p->mode : MIRSHA_EINVAL; }

int mirsha_pipeline_fallback(const mirsha_pipeline* p) { return p ? p->fallback : MIRSHA_EINVAL; }

int mirsha_pipeline_trace(mirsha_ctx* c, mirsha_pipeline* p, uint64_t* out, uint64_t cap, uint64_t* words) {
    if (!c || !p || !words) return MIRSHA_EINVAL;
    *words = 0;
    if (p->mode != MIRSHA_PIPELINE_FUSED || !p->trace) return MIRSHA_OK;
    if (int rc = use_device(c)) return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    const uint64_t n = 3ull * p->n_tiles + 2ull * p->n_counters + p->n_groups;
    *words = n;
    if (out && cap) {
        HIP_TRY(c, hipMemcpyAsync(out, p->d_trace.p, 8ull * std::min(n, cap), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
    }
    return MIRSHA_OK;
}

int mirsha_pipeline_shape(const mirsha_pipeline* p, uint32_t* n_tiles, uint32_t* n_counters, uint32_t* n_groups) {
    if (!p || !n_tiles || !n_counters || !n_groups) return MIRSHA_EINVAL;
    *n_tiles = p->n_tiles;
    *n_counters = p->n_counters;
    *n_groups = p->n_groups;
    return MIRSHA_OK;
}

int mirsha_pipeline_segments(const mirsha_pipeline* p, uint32_t* n_segments, uint32_t* bounds, uint32_t cap) {
    if (!p || !n_segments) return MIRSHA_EINVAL;
    *n_segments = 1;
    if (bounds && cap >= 1) bounds[0] = 0;
    return MIRSHA_OK;
}

int mirsha_pipeline_split_tiles(const mirsha_pipeline* p, uint32_t* n_split, uint32_t* segments_per_tile) {
    if (!p || !n_split || !segments_per_tile) return MIRSHA_EINVAL;
    *n_split = p->n_split;
    *segments_per_tile = p->seg_per_tile;
    return MIRSHA_OK;
}

int mirsha_pipeline_status(mirsha_ctx* c, mirsha_pipeline* p) {
    if (!c || !p) return MIRSHA_EINVAL;
    if (int rc = use_device(c)) return rc;
    return fused_status(c, p);
}

int mirsha_hash_requests_then_batches_device(mirsha_ctx* c, mirsha_pipeline* p, const uint8_t* d_arena,
                                             uint64_t arena_len, const uint64_t* d_off, const uint32_t* d_len,
                                             uint8_t* d_req_out, uint8_t* d_batch_out) {
    if (!c || !p) return MIRSHA_EINVAL;
    if (p->device != c->device) return fail(c, MIRSHA_EINVAL, "pipeline built for device %d", p->device);
    if (p->n_req && (!d_off || !d_len || !d_req_out || (!d_arena && arena_len))) return fail(c, MIRSHA_EINVAL, "NULL argument");
    if (p->n_lists && !d_batch_out) return fail(c, MIRSHA_EINVAL, "NULL batch output");
    if (arena_len > MIRSHA_MAX_DEVICE_ARENA_BYTES) return fail(c, MIRSHA_ERANGE, "device arena too large");
    if (int rc = use_device(c)) return rc;
    return plan_run(c, p, d_arena, arena_len, d_off, d_len, d_req_out, d_batch_out);
}

int mirsha_pipeline_overlap_device(mirsha_ctx* c, mirsha_pipeline* p, const uint8_t* d_arena, uint64_t arena_len,
                                   const uint64_t* d_off, const uint32_t* d_len, uint8_t* d_req_out,
                                   const uint8_t* d_prev_req, uint8_t* d_prev_batch_out) {
    if (!c || !p) return MIRSHA_EINVAL;
    if (p->device != c->device) return fail(c, MIRSHA_EINVAL, "pipeline built for device %d", p->device);
    const bool tiles = d_req_out != nullptr && p->n_req;
    const bool chains = d_prev_req != nullptr && p->n_lists;
    if (tiles && (!d_off || !d_len || (!d_arena && arena_len))) return fail(c, MIRSHA_EINVAL, "NULL argument");
    if (chains && !d_prev_batch_out) return fail(c, MIRSHA_EINVAL, "NULL batch output");
    if (p->mode == MIRSHA_PIPELINE_FUSED) {
        // Long chains (VerifyBatch): the fused launch's tile queues and list
        // pairs, the pairs over the previous cycle's digests without waits.
        if (arena_len > MIRSHA_MAX_DEVICE_ARENA_BYTES) return fail(c, MIRSHA_ERANGE, "device arena too large");
        if (int rc = use_device(c)) return rc;
        if (tiles)
            return fused_run(c, p, d_arena, arena_len, d_off, d_len, d_req_out, chains ? d_prev_batch_out : nullptr,
                             true, chains ? d_prev_req : nullptr);
        if (!chains) return MIRSHA_OK;
        if (int rc = fused_failed(c, p)) return rc;
        return timed_launch(c, 1, [&] {  // flush: the last cycle's chains alone, producer/consumer pairs
            return mirsha::launch_chain_pair(d_prev_req, p->n_req, p->d_cidx.as<uint32_t>(), p->n_entries,
                                             p->d_cfirst.as<uint32_t>(), p->n_lists, d_prev_batch_out, c->stream);
        });
    }
    if (arena_len > mirsha::kMaxBufferArena) return fail(c, MIRSHA_ERANGE, "overlap: arena > %llu bytes",
                                                         (unsigned long long)mirsha::kMaxBufferArena);
    if (p->n_req >= mirsha::kMaxBufferMsgs) return fail(c, MIRSHA_ERANGE, "overlap: %u requests", p->n_req);
    if (int rc = use_device(c)) return rc;
    mirsha::OverlapArgs a{};
    a.arena = d_arena;
    a.arena_len = tiles ? arena_len : 0;
    a.off = d_off;
    a.len = d_len;
    a.order = p->d_order.as<uint32_t>();
    a.n_req = tiles ? p->n_req : 0u;
    a.req_out = d_req_out;
    a.prev_digests = d_prev_req;
    a.n_req_prev = p->n_req;
    a.cidx = p->d_cidx.as<uint32_t>();
    a.n_entries = p->n_entries;
    a.cfirst = p->d_cfirst.as<uint32_t>();
    a.n_lists = p->n_lists;
    a.list_out = d_prev_batch_out;
    a.list_waves = chains ? (p->n_lists + 63u) / 64u : 0u;
    if (const char* e = mirsha::ab_getenv("MIRSHA_OVERLAP_CHAIN_PRIO")) a.chain_prio = (uint32_t)atoi(e) & 3u;
    return timed_launch(c, 5, [&] { return mirsha::launch_msgs_overlap(a, c->stream); });
}

int mirsha_digest_lists(mirsha_ctx* c, const uint8_t* digests, uint32_t n_digests, const uint32_t* idx,
                        const uint32_t* first, uint32_t n_lists, uint8_t* out) {
    if (!c) return MIRSHA_EINVAL;
    if (n_lists == 0) return MIRSHA_OK;
    if (!out || (n_digests && !digests)) return fail(c, MIRSHA_EINVAL, "NULL argument");
    if (int rc = check_lists(c, idx, first, n_lists, n_digests)) return rc;
    if (int rc = use_device(c)) return rc;
    ArenaSrc src;  // the digests themselves are the arena the lists index
    src.base = digests;
    src.total = 32ull * n_digests;
    return run_staged(c, src, nullptr, nullptr, 0, 0, kAnyOrder, idx, first, n_lists, nullptr, out);
}

int mirsha_hash_batch_device(mirsha_ctx* c, const uint8_t* d_arena, uint64_t arena_len,
                             const uint64_t* d_off, const uint32_t* d_len, const uint32_t* d_order,
                             uint32_t n, uint8_t* d_out) {
    if (!c) return MIRSHA_EINVAL;
    if (n == 0) return MIRSHA_OK;
    if (!d_off || !d_len || !d_out || (!d_arena && arena_len)) return fail(c, MIRSHA_EINVAL, "NULL argument");
    if (int rc = use_device(c)) return rc;
    return timed_launch(c, 0, [&] {
        return mirsha::launch_msgs(d_arena, arena_len, d_off, d_len, d_order, n, d_out, c->variant,
                                   c->stream);
    });
}

int mirsha_digest_lists_device(mirsha_ctx* c, const uint8_t* d_digests, uint32_t n_digests, const uint32_t* d_idx,
                               const uint32_t* d_first, uint32_t n_lists, uint32_t n_entries, uint8_t* d_out) {
    if (!c) return MIRSHA_EINVAL;
    if (n_lists == 0) return MIRSHA_OK;
    if (!d_idx || !d_first || !d_out) return fail(c, MIRSHA_EINVAL, "NULL argument");
    if (n_digests > mirsha::kMaxListDigests) return fail(c, MIRSHA_ERANGE, "n_digests %u too large", n_digests);
    if (n_entries > mirsha::kMaxListEntries) return fail(c, MIRSHA_ERANGE, "n_entries %u too large", n_entries);
    if (int rc = use_device(c)) return rc;
    HIP_TRY(c, c->d_scratch.ensure(sizeof(uint32_t) * std::max<uint32_t>(n_entries, 1)));
    return timed_launch(c, 1, [&] {
        return mirsha::launch_lists(d_digests, n_digests, d_idx, n_entries, d_first, n_lists,
                                    c->d_scratch.as<uint32_t>(), d_out, c->stream);
    });
}

int mirsha_bucket_order(const uint32_t* len, uint32_t n, uint32_t* order_out) {
    if (n && (!len || !order_out)) return MIRSHA_EINVAL;
    return bucket_order(len, n, order_out) ? 1 : 0;
}

int mirsha_synth_mixed_lengths_device(mirsha_ctx* c, uint64_t seed, uint64_t first, uint64_t count,
                                      uint32_t* d_len) {
    if (!c) return MIRSHA_EINVAL;
    if (count && !d_len) return fail(c, MIRSHA_EINVAL, "NULL length buffer");
    if (int rc = use_device(c)) return rc;
    return timed_launch(c, 2, [&] { return mirsha::launch_mixed_lengths(seed, first, count, d_len, c->stream); });
}

int mirsha_synth_mixed_device(mirsha_ctx* c, uint64_t seed, uint64_t first, uint64_t count, const uint64_t* d_off,
                              uint8_t* d_arena) {
    if (!c) return MIRSHA_EINVAL;
    if (count && (!d_off || !d_arena)) return fail(c, MIRSHA_EINVAL, "NULL argument");
    if (int rc = use_device(c)) return rc;
    return timed_launch(c, 2, [&] { return mirsha::launch_gen_mixed(seed, first, count, d_off, d_arena, c->stream); });
}

int mirsha_synth_requests_device(mirsha_ctx* c, uint64_t seed, uint64_t first, uint64_t count, uint32_t data_len,
                                 uint8_t* d_arena) {
    if (!c) return MIRSHA_EINVAL;
    if (count && !d_arena) return fail(c, MIRSHA_EINVAL, "NULL arena");
    if (int rc = use_device(c)) return rc;
    return timed_launch(c, 2, [&] { return mirsha::launch_gen_requests(seed, first, count, data_len, d_arena, c->stream); });
}

int mirsha_chains_create(mirsha_ctx* c, uint32_t n, mirsha_chains** out) {
    if (!c || !out) return MIRSHA_EINVAL;
    *out = nullptr;
    if (n == 0) return fail(c, MIRSHA_EINVAL, "n_chains must be > 0");
    if (int rc = use_device(c)) return rc;
    auto* ch = new mirsha_chains();
    ch->device = c->device;
    ch->n = n;
    std::vector<uint32_t> h(8ull * n);
    for (uint32_t i = 0; i < n; i++)
        for (int j = 0; j < 8; j++) h[8ull * i + j] = mirsha::kH0[j];
    auto up = [&]() -> int {
        HIP_TRY(c, ch->d_h.ensure(32ull * n));
        HIP_TRY(c, ch->d_pend.ensure(32ull * n));
        HIP_TRY(c, ch->d_cnt.ensure(8ull * n));
        HIP_TRY(c, hipMemcpyAsync(ch->d_h.p, h.data(), 32ull * n, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(c, hipMemsetAsync(ch->d_pend.p, 0, 32ull * n, c->stream));
        HIP_TRY(c, hipMemsetAsync(ch->d_cnt.p, 0, 8ull * n, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        return MIRSHA_OK;
    };
    if (int rc = up()) {
        mirsha_chains_destroy(ch);
        return rc;
    }
    *out = ch;
    return MIRSHA_OK;
}

void mirsha_chains_destroy(mirsha_chains* ch) {
    if (!ch) return;
    (void)hipSetDevice(ch->device);
    for (DevBuf* b : {&ch->d_h, &ch->d_pend, &ch->d_cnt, &ch->d_dig, &ch->d_pos, &ch->d_act, &ch->d_afirst,
                      &ch->d_which, &ch->d_out})
        b->release();
    delete ch;
}

int mirsha_chains_absorb(mirsha_ctx* c, mirsha_chains* ch, const uint8_t* digests, const uint32_t* chain_of,
                         uint32_t m) {
    if (!c || !ch) return MIRSHA_EINVAL;
    if (m == 0) return MIRSHA_OK;
    if (!digests || !chain_of) return fail(c, MIRSHA_EINVAL, "NULL argument");
    if (ch->device != c->device) return fail(c, MIRSHA_EINVAL, "chains belong to another device");
    // Group the writes by chain, keeping their order (counting sort).
    std::vector<uint32_t> count(ch->n + 1, 0);
    for (uint32_t i = 0; i < m; i++) {
        if (chain_of[i] >= ch->n) return fail(c, MIRSHA_EINVAL, "chain_of[%u] = %u >= %u", i, chain_of[i], ch->n);
        count[chain_of[i] + 1]++;
    }
    std::vector<uint32_t> act, afirst(1, 0);
    for (uint32_t k = 0; k < ch->n; k++)
        if (count[k + 1]) {
            act.push_back(k);
            afirst.push_back(afirst.back() + count[k + 1]);
        }
    for (uint32_t k = 0; k < ch->n; k++) count[k + 1] += count[k];
    std::vector<uint32_t> pos(m);
    for (uint32_t i = 0; i < m; i++) pos[count[chain_of[i]]++] = i;
    if (int rc = use_device(c)) return rc;
    const uint32_t na = (uint32_t)act.size();
    HIP_TRY(c, ch->d_dig.ensure(32ull * m));
    HIP_TRY(c, ch->d_pos.ensure(4ull * m));
    HIP_TRY(c, ch->d_act.ensure(4ull * na));
    HIP_TRY(c, ch->d_afirst.ensure(4ull * (na + 1)));
    HIP_TRY(c, hipMemcpyAsync(ch->d_dig.p, digests, 32ull * m, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(ch->d_pos.p, pos.data(), 4ull * m, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(ch->d_act.p, act.data(), 4ull * na, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipMemcpyAsync(ch->d_afirst.p, afirst.data(), 4ull * (na + 1), hipMemcpyHostToDevice, c->stream));
    if (int rc = timed_launch(c, 1, [&] {
            return mirsha::launch_chains_absorb(ch->d_dig.as<uint8_t>(), ch->d_pos.as<uint32_t>(),
                                                ch->d_act.as<uint32_t>(), ch->d_afirst.as<uint32_t>(), na,
                                                ch->d_h.as<uint32_t>(), ch->d_pend.as<uint32_t>(),
                                                ch->d_cnt.as<uint64_t>(), c->stream);
        }))
        return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));  // host vectors above feed async copies
    return MIRSHA_OK;
}

namespace {
int chains_which(mirsha_ctx* c, mirsha_chains* ch, const uint32_t* which, uint32_t k) {
    if (!which) return fail(c, MIRSHA_EINVAL, "NULL argument");
    if (ch->device != c->device) return fail(c, MIRSHA_EINVAL, "chains belong to another device");
    for (uint32_t j = 0; j < k; j++)
        if (which[j] >= ch->n) return fail(c, MIRSHA_EINVAL, "which[%u] = %u >= %u", j, which[j], ch->n);
    if (int rc = use_device(c)) return rc;
    HIP_TRY(c, ch->d_which.ensure(4ull * k));
    HIP_TRY(c, hipMemcpyAsync(ch->d_which.p, which, 4ull * k, hipMemcpyHostToDevice, c->stream));
    return MIRSHA_OK;
}
}  // namespace

int mirsha_chains_sum(mirsha_ctx* c, mirsha_chains* ch, const uint32_t* which, uint32_t k, uint8_t* out) {
    if (!c || !ch) return MIRSHA_EINVAL;
    if (k == 0) return MIRSHA_OK;
    if (!out) return fail(c, MIRSHA_EINVAL, "NULL argument");
    if (int rc = chains_which(c, ch, which, k)) return rc;
    HIP_TRY(c, ch->d_out.ensure(32ull * k));
    if (int rc = timed_launch(c, 1, [&] {
            return mirsha::launch_chains_sum(ch->d_which.as<uint32_t>(), k, ch->d_h.as<uint32_t>(),
                                             ch->d_pend.as<uint32_t>(), ch->d_cnt.as<uint64_t>(),
                                             ch->d_out.as<uint8_t>(), c->stream);
        }))
        return rc;
    HIP_TRY(c, hipMemcpyAsync(out, ch->d_out.p, 32ull * k, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return MIRSHA_OK;
}

int mirsha_chains_reset(mirsha_ctx* c, mirsha_chains* ch, const uint32_t* which, uint32_t k) {
    if (!c || !ch) return MIRSHA_EINVAL;
    if (k == 0) return MIRSHA_OK;
    if (int rc = chains_which(c, ch, which, k)) return rc;
    if (int rc = timed_launch(c, 1, [&] {
            return mirsha::launch_chains_reset(ch->d_which.as<uint32_t>(), k, ch->d_h.as<uint32_t>(),
                                               ch->d_cnt.as<uint64_t>(), c->stream);
        }))
        return rc;
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return MIRSHA_OK;
}

int mirsha_ctx_host_profile(const mirsha_ctx* c, double* ms_out, int n) {
    if (!c || !ms_out || n < 0) return MIRSHA_EINVAL;
    for (int k = 0; k < n && k < MIRSHA_PROF_PHASES; k++) ms_out[k] = c->prof[k];
    return MIRSHA_PROF_PHASES;
}

int mirsha_clock_probe(mirsha_ctx* c, uint32_t iters, double* clock_ghz, double* cycles_per_wave_compression) {
    if (!c || !clock_ghz || !cycles_per_wave_compression || iters == 0) return MIRSHA_EINVAL;
    if (int rc = use_device(c)) return rc;
    hipDeviceProp_t prop;
    HIP_TRY(c, hipGetDeviceProperties(&prop, c->device));
    // One 256-thread workgroup = one wave per SIMD of a CU; kProbeWavesPerSimd per CU
    // (MIRSHA_AB=1 MIRSHA_PROBE_WAVES=k: k per SIMD, occupancy A/B).
    uint32_t wps = mirsha::kProbeWavesPerSimd;
    if (const char* e = mirsha::ab_getenv("MIRSHA_PROBE_WAVES")) wps = std::min(8u, std::max(1u, (uint32_t)atoi(e)));
    const uint32_t blocks = (uint32_t)prop.multiProcessorCount * wps;
    const uint32_t waves = 4u * blocks;
    DevBuf stamps, sink;
    HIP_TRY(c, stamps.ensure(24ull * waves));
    HIP_TRY(c, sink.ensure(4ull * 256u * blocks));
    int rc = timed_launch(c, 2, [&] {
        return mirsha::launch_clock_probe(blocks, iters, stamps.as<unsigned long long>(), sink.as<uint32_t>(),
                                          c->stream);
    });
    std::vector<unsigned long long> h(3ull * waves);
    if (rc == MIRSHA_OK) {
        hipError_t e = hipMemcpyAsync(h.data(), stamps.p, 24ull * waves, hipMemcpyDeviceToHost, c->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e != hipSuccess) rc = fail(c, MIRSHA_EHIP, "clock probe: %s", hipGetErrorString(e));
    }
    stamps.release();
    sink.release();
    if (rc) return rc;
    std::vector<double> ghz(waves);
    unsigned long long first = ~0ull, last = 0;
    for (uint32_t w = 0; w < waves; w++) {
        const unsigned long long r0 = h[3 * w + 1], r1 = h[3 * w + 2];
        ghz[w] = r1 > r0 ? 0.1 * (double)h[3 * w] / (double)(r1 - r0) : 0.0;
        first = std::min(first, r0);
        last = std::max(last, r1);
    }
    std::nth_element(ghz.begin(), ghz.begin() + waves / 2, ghz.end());
    *clock_ghz = ghz[waves / 2];
    // Span in shader cycles at that clock, per SIMD, per wave-compression.
    const double span_cycles = (double)(last - first) * 10.0 * *clock_ghz;
    *cycles_per_wave_compression = span_cycles / ((double)iters * wps);
    return MIRSHA_OK;
}

// Per-device contexts of mirsha_hash_batch_multi, kept across calls (a
// context owns streams, events and grown staging buffers: creating one per
// call per device cost a stream setup and a cold staging path every time).
// A device listed twice in one call takes two contexts.  Released by
// mirsha_multi_release (or at process exit).
namespace {
std::mutex g_multi_mu;
std::vector<mirsha_ctx*> g_multi_idle;
}  // namespace

static int multi_ctx_take(int device, mirsha_ctx** out) {
    {
        std::lock_guard<std::mutex> lk(g_multi_mu);
        for (size_t i = 0; i < g_multi_idle.size(); i++)
            if (g_multi_idle[i]->device == device) {
                *out = g_multi_idle[i];
                g_multi_idle.erase(g_multi_idle.begin() + (ptrdiff_t)i);
                return MIRSHA_OK;
            }
    }
    return mirsha_ctx_create(device, out);
}

static void multi_ctx_give(mirsha_ctx* c) {
    std::lock_guard<std::mutex> lk(g_multi_mu);
    g_multi_idle.push_back(c);
}

void mirsha_multi_release(void) {
    std::vector<mirsha_ctx*> v;
    {
        std::lock_guard<std::mutex> lk(g_multi_mu);
        v.swap(g_multi_idle);
    }
    for (mirsha_ctx* c : v) mirsha_ctx_destroy(c);
}

int mirsha_hash_batch_multi(const int* devices, int ndev, const uint8_t* arena, uint64_t arena_len,
                            const uint64_t* off, const uint32_t* len, uint32_t n, uint8_t* out) {
    if (ndev <= 0 || !devices) return MIRSHA_EINVAL;
    if (n == 0) return MIRSHA_OK;
    if (!off || !len || !out) return MIRSHA_EINVAL;
    // Contiguous request ranges balanced by compressions.
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; i++) total += host_blocks(len[i]);
    std::vector<uint32_t> cut(ndev + 1, n);
    cut[0] = 0;
    uint64_t acc = 0;
    int d = 1;
    for (uint32_t i = 0; i < n && d < ndev; i++) {
        acc += host_blocks(len[i]);
        while (d < ndev && acc * ndev >= total * (uint64_t)d) cut[d++] = i + 1;
    }
    std::vector<int> rcs(ndev, MIRSHA_OK);
    std::vector<std::thread> th;
    for (int k = 0; k < ndev; k++) {
        th.emplace_back([&, k] {
            const uint32_t a = cut[k], b = cut[k + 1];
            if (a >= b) return;
            mirsha_ctx* c = nullptr;
            int rc = multi_ctx_take(devices[k], &c);
            if (rc == MIRSHA_OK) rc = mirsha_hash_batch(c, arena, arena_len, off + a, len + a, b - a, out + 32ull * a);
            rcs[k] = rc;
            if (c) multi_ctx_give(c);
        });
    }
    for (auto& t : th) t.join();
    for (int k = 0; k < ndev; k++)
        if (rcs[k]) return rcs[k];
    return MIRSHA_OK;
}

}  // extern "C"

// ---- multi-device drop-in (mirsha_multi) ----------------------------------
// One context per listed device (its own stream, pinned staging ring and
// PCIe link) and one persistent worker thread per device with its own host
// packing pool (mirsha::host::use_pool: an equal share of the host threads),
// so the devices pack, copy and hash their ranges side by side.  A call cuts
// the requests into contiguous ranges of equal BYTES (each device's share of
// the PCIe traffic), rebases each range's slice_first, and runs the
// single-device entry point on it; digests land in origin order (each range
// writes its own rows of digests_out).  No collective: requests are
// independent (actions.go:22-23).

struct MultiWorker {
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    std::function<void()> job;
    bool has_job = false, quit = false;
};

struct mirsha_multi {
    std::vector<int> devices;
    std::vector<mirsha_ctx*> ctx;
    std::vector<MultiWorker*> workers;
    std::mutex done_mu;
    std::condition_variable done_cv;
    int pending = 0;
    std::string err;
    // per-device sub-range of the last call (request index bounds) and the
    // asynchronous tickets: multi ticket t -> per-device tickets
    std::vector<uint32_t> cut;
    uint64_t next_ticket = 1, done_ticket = 0;
    std::vector<std::vector<uint64_t>> dev_tickets;  // [(t - 1) % slots][k]; 0 = device k had no requests
    std::vector<std::vector<uint32_t>> sub_first;   // rebased slice_first per device (sync calls)
    std::vector<std::vector<std::vector<uint32_t>>> async_first;  // [slot][k]: kept until the ticket retires
};

namespace {

constexpr int kMultiAsyncSlots = 4;  // as a context's ring (mirsha_submit_slices)

void multi_worker_loop(MultiWorker* w, mirsha_multi* m, int slot, int threads) {
    mirsha::host::use_pool(slot, threads);
    for (;;) {
        std::function<void()> job;
        {
            std::unique_lock<std::mutex> g(w->mu);
            w->cv.wait(g, [&] { return w->has_job || w->quit; });
            if (w->quit) return;
            job.swap(w->job);
            w->has_job = false;
        }
        job();
        {
            std::lock_guard<std::mutex> g(m->done_mu);
            if (--m->pending == 0) m->done_cv.notify_all();
        }
    }
}

// Runs fn(k) for every device k on its worker; returns the first device's
// error (its message copied to m->err).
int multi_run(mirsha_multi* m, const std::function<int(int)>& fn) {
    const int nd = (int)m->ctx.size();
    std::vector<int> rcs(nd, MIRSHA_OK);
    {
        std::lock_guard<std::mutex> g(m->done_mu);
        m->pending = nd;
    }
    for (int k = 0; k < nd; k++) {
        MultiWorker* w = m->workers[k];
        std::lock_guard<std::mutex> g(w->mu);
        w->job = [&, k] { rcs[k] = fn(k); };
        w->has_job = true;
        w->cv.notify_one();
    }
    {
        std::unique_lock<std::mutex> g(m->done_mu);
        m->done_cv.wait(g, [&] { return m->pending == 0; });
    }
    for (int k = 0; k < nd; k++)
        if (rcs[k]) {
            char buf[640];
            snprintf(buf, sizeof(buf), "device %d (index %d): %s", m->devices[k], k, mirsha_last_error(m->ctx[k]));
            m->err = buf;
            return rcs[k];
        }
    return MIRSHA_OK;
}

int multi_fail(mirsha_multi* m, int code, const char* msg) {
    m->err = msg;
    return code;
}

// Validates the slice lists (as mirsha_hash_slices does) and cuts [0, n) into
// one contiguous range per device with equal bytes (ranges may be empty).
int multi_cut(mirsha_multi* m, const uint8_t* const* slice_ptr, const uint64_t* slice_len,
              const uint32_t* slice_first, uint32_t n, const uint8_t* out) {
    if (!slice_first || !out) return multi_fail(m, MIRSHA_EINVAL, "NULL argument");
    if (slice_first[0] != 0) return multi_fail(m, MIRSHA_EINVAL, "slice_first[0] must be 0");
    if (slice_first[n] && (!slice_ptr || !slice_len)) return multi_fail(m, MIRSHA_EINVAL, "NULL slice arrays");
    const uint32_t ns = slice_first[n];
    std::vector<uint64_t> sum(n);
    std::vector<uint8_t> err(n, 0);
    mirsha::host::parallel_for(n, mirsha::host::threads_for(16ull * ns, n), [&](uint32_t lo, uint32_t hi) {
        for (uint32_t i = lo; i < hi; i++) {
            if (slice_first[i + 1] < slice_first[i] || slice_first[i + 1] > ns) { err[i] = 1; continue; }
            uint64_t L = 0;
            for (uint32_t s = slice_first[i]; s < slice_first[i + 1]; s++) {
                if (slice_len[s] && !slice_ptr[s]) { err[i] = 2; break; }
                L += slice_len[s];
            }
            if (!err[i] && L > MIRSHA_MAX_MESSAGE_BYTES) err[i] = 3;
            sum[i] = L;
        }
    });
    for (uint32_t i = 0; i < n; i++) {
        char buf[128];
        if (!err[i]) continue;
        snprintf(buf, sizeof(buf), err[i] == 1 ? "slice_first not monotone at request %u"
                                   : err[i] == 2 ? "request %u has a NULL slice" : "request %u exceeds the message limit", i);
        return multi_fail(m, err[i] == 3 ? MIRSHA_ERANGE : MIRSHA_EINVAL, buf);
    }
    // prefix sums, then the cut points at equal shares of the bytes (ties:
    // requests of 0 bytes count as 1 so empty requests spread too)
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; i++) {
        total += std::max<uint64_t>(sum[i], 1);
        sum[i] = total;
    }
    const int nd = (int)m->ctx.size();
    m->cut.assign(nd + 1, n);
    m->cut[0] = 0;
    for (int k = 1; k < nd; k++) {
        // the request boundary nearest to k/nd of the bytes
        const uint64_t want = (total * (uint64_t)k + nd / 2) / nd;
        uint32_t i = (uint32_t)(std::lower_bound(sum.begin(), sum.end(), want) - sum.begin());  // sum[i] >= want
        if (i < n && (i == 0 ? want : want - sum[i - 1]) * 2 > (sum[i] - (i ? sum[i - 1] : 0))) i++;
        m->cut[k] = std::max(std::min(i, n), m->cut[k - 1]);
    }
    return MIRSHA_OK;
}

void rebase_first(const uint32_t* slice_first, uint32_t a, uint32_t b, std::vector<uint32_t>& f) {
    f.resize(b - a + 1);
    const uint32_t base = slice_first[a];
    for (uint32_t i = a; i <= b; i++) f[i - a] = slice_first[i] - base;
}

}  // namespace

extern "C" {

int mirsha_multi_create(const int* devices, int ndev, mirsha_multi** out) {
    if (!out) return MIRSHA_EINVAL;
    *out = nullptr;
    if (!devices || ndev <= 0 || ndev >= mirsha::host::kMaxPools) return MIRSHA_EINVAL;
    mirsha_multi* m = new mirsha_multi();
    for (int k = 0; k < ndev; k++) {
        mirsha_ctx* c = nullptr;
        const int rc = mirsha_ctx_create(devices[k], &c);
        if (rc != MIRSHA_OK) {
            for (mirsha_ctx* x : m->ctx) mirsha_ctx_destroy(x);
            delete m;
            return rc;
        }
        m->devices.push_back(devices[k]);
        m->ctx.push_back(c);
    }
    // Each worker packs with an equal share of the host threads (>= 2).
    const int share = std::max(2, mirsha::host::max_threads() / ndev);
    for (int k = 0; k < ndev; k++) {
        MultiWorker* w = new MultiWorker();
        w->th = std::thread(multi_worker_loop, w, m, k + 1, share);
        m->workers.push_back(w);
    }
    m->async_first.resize(kMultiAsyncSlots);
    m->dev_tickets.assign(kMultiAsyncSlots, std::vector<uint64_t>(ndev, 0));
    *out = m;
    return MIRSHA_OK;
}

void mirsha_multi_destroy(mirsha_multi* m) {
    if (!m) return;
    for (MultiWorker* w : m->workers) {
        {
            std::lock_guard<std::mutex> g(w->mu);
            w->quit = true;
        }
        w->cv.notify_one();
        w->th.join();
        delete w;
    }
    for (mirsha_ctx* c : m->ctx) mirsha_ctx_destroy(c);
    delete m;
}

const char* mirsha_multi_last_error(const mirsha_multi* m) { return m ? m->err.c_str() : "null multi context"; }

int mirsha_multi_devices(const mirsha_multi* m) { return m ? (int)m->ctx.size() : MIRSHA_EINVAL; }

mirsha_ctx* mirsha_multi_ctx(mirsha_multi* m, int k) {
    return (m && k >= 0 && k < (int)m->ctx.size()) ? m->ctx[k] : nullptr;
}

int mirsha_multi_last_cut(const mirsha_multi* m, uint32_t* first_out, int cap) {
    if (!m || !first_out || cap < 0) return MIRSHA_EINVAL;
    for (int k = 0; k < cap && k < (int)m->cut.size(); k++) first_out[k] = m->cut[k];
    return (int)m->cut.size();
}

int mirsha_hash_slices_multi(mirsha_multi* m, const uint8_t* const* slice_ptr, const uint64_t* slice_len,
                             const uint32_t* slice_first, uint32_t n, uint8_t* digests_out) {
    if (!m) return MIRSHA_EINVAL;
    m->err.clear();
    if (n == 0) return MIRSHA_OK;
    if (int rc = multi_cut(m, slice_ptr, slice_len, slice_first, n, digests_out)) return rc;
    const int nd = (int)m->ctx.size();
    m->sub_first.resize(nd);
    return multi_run(m, [&](int k) -> int {
        const uint32_t a = m->cut[k], b = m->cut[k + 1];
        if (a >= b) return MIRSHA_OK;
        rebase_first(slice_first, a, b, m->sub_first[k]);
        const uint32_t s0 = slice_first[a];
        return mirsha_hash_slices(m->ctx[k], slice_ptr + s0, slice_len + s0, m->sub_first[k].data(), b - a,
                                  digests_out + 32ull * a);
    });
}

int mirsha_hash_arena_multi(mirsha_multi* m, const uint8_t* arena, uint64_t arena_len, const uint64_t* off,
                            const uint32_t* len, uint32_t n, uint8_t* digests_out) {
    if (!m) return MIRSHA_EINVAL;
    m->err.clear();
    if (n == 0) return MIRSHA_OK;
    if (!off || !len || !digests_out || (!arena && arena_len)) return multi_fail(m, MIRSHA_EINVAL, "NULL argument");
    // equal-bytes cut over the request lengths (empty requests count 1)
    const int nd = (int)m->ctx.size();
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; i++) total += std::max<uint32_t>(len[i], 1u);
    m->cut.assign(nd + 1, n);
    m->cut[0] = 0;
    uint64_t acc = 0;
    int d = 1;
    for (uint32_t i = 0; i < n && d < nd; i++) {
        acc += std::max<uint32_t>(len[i], 1u);
        while (d < nd && acc * (uint64_t)nd >= total * (uint64_t)d) m->cut[d++] = i + 1;
    }
    return multi_run(m, [&](int k) -> int {
        const uint32_t a = m->cut[k], b = m->cut[k + 1];
        if (a >= b) return MIRSHA_OK;
        return mirsha_hash_batch(m->ctx[k], arena, arena_len, off + a, len + a, b - a, digests_out + 32ull * a);
    });
}

int mirsha_multi_host_alloc(mirsha_multi* m, uint64_t bytes, void** out) {
    if (!m || !out) return MIRSHA_EINVAL;
    *out = nullptr;
    // portable: page-locked for every device's DMA engine, not only device 0's
    if (hipSetDevice(m->devices[0]) != hipSuccess ||
        hipHostMalloc(out, std::max<uint64_t>(bytes, 1), hipHostMallocPortable) != hipSuccess) {
        (void)hipGetLastError();
        *out = nullptr;
        return multi_fail(m, MIRSHA_ENOMEM, "hipHostMalloc (portable) failed");
    }
    return MIRSHA_OK;
}

int mirsha_submit_slices_multi(mirsha_multi* m, const uint8_t* const* slice_ptr, const uint64_t* slice_len,
                               const uint32_t* slice_first, uint32_t n, uint8_t* digests_out, int flags,
                               uint64_t* ticket_out) {
    if (!m || !ticket_out) return MIRSHA_EINVAL;
    m->err.clear();
    if (flags & ~MIRSHA_SUBMIT_DEDUP) return multi_fail(m, MIRSHA_EINVAL, "unknown submit flags");
    // ring full: retire the oldest multi ticket first (its rebased arrays are reused)
    const uint64_t t = m->next_ticket;
    if (t > (uint64_t)kMultiAsyncSlots && m->done_ticket < t - kMultiAsyncSlots)
        if (int rc = mirsha_wait_multi(m, t - kMultiAsyncSlots)) return rc;
    const int nd = (int)m->ctx.size();
    if (n == 0) {
        m->cut.assign(nd + 1, 0u);
    } else if (int rc = multi_cut(m, slice_ptr, slice_len, slice_first, n, digests_out)) {
        return rc;
    }
    auto& firsts = m->async_first[(t - 1) % kMultiAsyncSlots];
    firsts.resize(nd);
    std::vector<uint64_t> dt(nd, 0);
    const int rc = multi_run(m, [&](int k) -> int {
        const uint32_t a = m->cut[k], b = m->cut[k + 1];
        if (a >= b) return MIRSHA_OK;
        rebase_first(slice_first, a, b, firsts[k]);
        const uint32_t s0 = slice_first[a];
        return mirsha_submit_slices(m->ctx[k], slice_ptr + s0, slice_len + s0, firsts[k].data(), b - a,
                                    digests_out + 32ull * a, flags, &dt[k]);
    });
    if (rc) {
        // a device refused its range: retire the ranges the others queued
        // before returning, so no digest lands in digests_out after the
        // failed call (the caller may free it)
        const std::string err = m->err;
        for (size_t k = 0; k < dt.size(); k++)
            if (dt[k]) (void)mirsha_wait(m->ctx[k], dt[k]);
        m->err = err;
        return rc;
    }
    m->dev_tickets[(t - 1) % kMultiAsyncSlots] = dt;
    m->next_ticket++;
    *ticket_out = t;
    return MIRSHA_OK;
}

int mirsha_wait_multi(mirsha_multi* m, uint64_t ticket) {
    if (!m) return MIRSHA_EINVAL;
    if (ticket == 0 || ticket >= m->next_ticket) return multi_fail(m, MIRSHA_EINVAL, "unknown ticket");
    if (ticket <= m->done_ticket) return MIRSHA_OK;
    // every device's latest ticket up to `ticket` (its own tickets retire in order)
    std::vector<uint64_t> upto(m->ctx.size(), 0);
    for (uint64_t t = m->done_ticket + 1; t <= ticket; t++)
        for (size_t k = 0; k < upto.size(); k++)
            upto[k] = std::max(upto[k], m->dev_tickets[(t - 1) % kMultiAsyncSlots][k]);
    const int rc = multi_run(m, [&](int k) -> int { return upto[k] ? mirsha_wait(m->ctx[k], upto[k]) : MIRSHA_OK; });
    if (rc) return rc;
    m->done_ticket = ticket;
    return MIRSHA_OK;
}

int mirsha_poll_multi(mirsha_multi* m, uint64_t ticket, int* done) {
    if (!m || !done) return MIRSHA_EINVAL;
    if (ticket == 0 || ticket >= m->next_ticket) return multi_fail(m, MIRSHA_EINVAL, "unknown ticket");
    *done = 0;
    if (ticket <= m->done_ticket) {
        *done = 1;
        return MIRSHA_OK;
    }
    std::vector<uint64_t> upto(m->ctx.size(), 0);
    for (uint64_t t = m->done_ticket + 1; t <= ticket; t++)
        for (size_t k = 0; k < upto.size(); k++)
            upto[k] = std::max(upto[k], m->dev_tickets[(t - 1) % kMultiAsyncSlots][k]);
    std::vector<int> d(m->ctx.size(), 1);
    for (size_t k = 0; k < upto.size(); k++)
        if (upto[k])
            if (int rc = mirsha_poll(m->ctx[k], upto[k], &d[k])) {
                m->err = mirsha_last_error(m->ctx[k]);
                return rc;
            }
    for (int x : d)
        if (!x) return MIRSHA_OK;
    m->done_ticket = ticket;
    *done = 1;
    return MIRSHA_OK;
}

int mirsha_multi_host_profile(const mirsha_multi* m, int k, double* ms_out, int n) {
    if (!m || k < 0 || k >= (int)m->ctx.size()) return MIRSHA_EINVAL;
    return mirsha_ctx_host_profile(m->ctx[k], ms_out, n);
}

}  // extern "C"
