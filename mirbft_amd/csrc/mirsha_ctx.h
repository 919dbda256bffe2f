// mirsha_ctx.h — internal state shared by the host-side translation units of
// the C-ABI (include/mirsha.h); not part of the ABI.
//
//   mirsha_api.hip      contexts, timing, device-pointer API, synthetic
//                       streams, checkpoint chains, clock probe
//   mirsha_staging.hip  synchronous host calls: staging, pipelined H2D /
//                       kernels / D2H (mirsha_hash_batch / _slices /
//                       _requests_then_batches, mirsha_digest_lists)
//   mirsha_plan.hip     request -> batch plans: sequential, fused (placement
//                       probe), overlapped cycles (mirsha_pipeline_*)
//   mirsha_async.hip    the asynchronous ring (mirsha_submit_* / wait / poll,
//                       dedup)
//   mirsha_multi.hip    the multi-device drop-in (mirsha_multi_*)
//
// Every entry point returns digests in ORIGIN order (processor.go:139 indexes
// Digests[i] by the request's position), unlike ProcessorWorkPool's
// completion-order collector (processor.go:349-356).
#pragma once
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

namespace mirsha_api {

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

// Grow-only buffers.  A growth frees (hipFree / hipHostFree synchronise the
// device: every queued copy and kernel of every stream must finish first),
// so a buffer grows to 1.5x its old capacity, not to the exact request: ring
// slots see chunks a few hundred bytes apart, and exact-fit growth cost a
// ~9 ms device drain inside a submission now and then (profiles/r05w).
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t n) {
        if (n <= cap) return hipSuccess;
        size_t want = std::max(n, cap + cap / 2);
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
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
        size_t want = std::max(n, cap + cap / 2);
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            e = hipHostMalloc(&p, n, hipHostMallocDefault);
            if (e != hipSuccess) { p = nullptr; return e; }
            want = n;
        }
        cap = want;
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
    hipEvent_t ev_in = nullptr, ev_kern = nullptr;  // arena submissions: H2D landed, kernel done
    uint64_t ticket = 0;
    bool busy = false;
    uint8_t* user_out = nullptr;
    bool direct = false;  // digests DMA'd straight into a page-locked user_out (nothing to copy at retire)
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


}  // namespace mirsha_api
using namespace mirsha_api;

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
    // Host scratch of the synchronous slice call (request lengths, packed
    // offsets), kept across calls: fresh vectors cost ~1-2 ms of page faults
    // and zeroing per 2^20 requests.
    std::vector<uint32_t> sl_len;
    std::vector<uint64_t> sl_poff;
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
    uint32_t uniform = 0;                    // B: identity lists of B entries (uniform_lists), else 0
    std::vector<uint32_t> order;             // request processing order
    DevBuf d_cidx, d_cfirst, d_order, d_state;
};

namespace mirsha_api {

int fail(mirsha_ctx* c, int code, const char* fmt, ...);

#define HIP_TRY(c, expr)                                                                    \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess)                                                               \
            return fail((c), _e == hipErrorOutOfMemory ? MIRSHA_ENOMEM : MIRSHA_EHIP,       \
                        "%s: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, __LINE__); \
    } while (0)

hipEvent_t take_event(KernelTimer& t);

// One launch (a launch function that launches at most one kernel), timed
// when timing is on for `which`: the two events ride on the kernel's own
// dispatch (mirsha::launch_k, hipExtLaunchKernel), so they carry its start
// and end timestamps and add no marker packets to the stream.
template <class F>
int timed_launch(mirsha_ctx* c, int which, F&& launch) {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    const bool timed = c->timing && ((c->time_mask >> which) & 1u);
    if (timed) {
        e0 = take_event(c->timers[which]);
        e1 = take_event(c->timers[which]);
        if (e0 && e1) mirsha::next_launch_events() = {e0, e1};
    }
    hipError_t e = launch();
    // unconsumed: the launch function launched nothing (an empty call)
    const bool bound = e0 && e1 && !mirsha::next_launch_events().start;
    mirsha::next_launch_events() = {};
    if (timed && (!bound || e != hipSuccess)) {
        if (e0) c->timers[which].pool.push_back(e0);
        if (e1) c->timers[which].pool.push_back(e1);
    }
    if (e != hipSuccess) return fail(c, MIRSHA_EHIP, "kernel launch: %s", hipGetErrorString(e));
    if (bound) c->timers[which].pending.emplace_back(e0, e1);
    return MIRSHA_OK;
}

int use_device(mirsha_ctx* c);

inline uint32_t host_blocks(uint32_t L) { return (uint32_t)(((uint64_t)L + 72u) >> 6); }

// Stable sort of message indices by block count, longest first; true if the
// order is the identity (one bucket).
bool bucket_order(const uint32_t* len, uint32_t n, uint32_t* order);

int check_lists(mirsha_ctx* c, const uint32_t* idx, const uint32_t* first, uint32_t n_lists, uint32_t n_digests);

// A boolean A/B or diagnostic knob ("1" = set; only with MIRSHA_AB=1).
inline bool getenv_flag(const char* name) {
    const char* e = mirsha::ab_getenv(name);
    return e && e[0] == '1';
}

inline bool host_pinned(const void* p) {
    hipPointerAttribute_t a;
    if (!p || hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

// Page-locked host memory a kernel on `device` may store into: allocated or
// registered with that device current, or portable (every device maps it).
// Anything else takes the D2H path.
inline bool kernel_writable_host(const void* p, int device) {
    hipPointerAttribute_t a;
    if (!p || hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeHost && (a.device == device || (a.allocationFlags & hipHostMallocPortable));
}

constexpr uint64_t align8(uint64_t x) { return (x + 7u) & ~7ull; }

// ---- mirsha_staging.hip
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
// `layout`: kInOrder = the messages lie in [0, total) in index order (each
// starts at or after the previous one's end), which the pipelined form needs;
// kGapless = in order with no gaps (off[i] - shift = len[0] + ... + len[i-1]).
enum ArenaLayout { kAnyOrder = 0, kInOrder = 1, kGapless = 2 };
int run_staged(mirsha_ctx* c, const ArenaSrc& src, const uint64_t* off, const uint32_t* len, uint32_t n,
               uint64_t shift, ArenaLayout layout, const uint32_t* idx, const uint32_t* first, uint32_t n_lists,
               uint8_t* req_out, uint8_t* list_out);
int arena_span(mirsha_ctx* c, uint64_t arena_len, const uint64_t* off, const uint32_t* len, uint32_t n,
               uint64_t* lo_out, uint64_t* hi_out, uint64_t* total_out = nullptr, ArenaLayout* layout_out = nullptr);
int run_arena_call(mirsha_ctx* c, const uint8_t* arena, uint64_t arena_len, const uint64_t* off, const uint32_t* len,
                   uint32_t n, const uint32_t* idx, const uint32_t* first, uint32_t n_lists, uint8_t* req_out,
                   uint8_t* list_out);
int slice_errors(mirsha_ctx* c, const uint8_t* err, uint32_t n);
int slice_args(mirsha_ctx* c, const uint8_t* const* slice_ptr, const uint64_t* slice_len, const uint32_t* slice_first,
               uint32_t n, const uint8_t* out);
int slice_lengths(mirsha_ctx* c, const uint8_t* const* slice_ptr, const uint64_t* slice_len,
                  const uint32_t* slice_first, uint32_t n, const uint8_t* out, std::vector<uint32_t>& len);

// ---- mirsha_plan.hip
int plan_build(mirsha_ctx* c, mirsha_pipeline* p, uint32_t n_req, const uint32_t* idx, const uint32_t* first,
               uint32_t n_lists, const uint32_t* len);
int plan_run(mirsha_ctx* c, mirsha_pipeline* p, const uint8_t* d_arena, uint64_t arena_len, const uint64_t* d_off,
             const uint32_t* d_len, uint8_t* d_req_out, uint8_t* d_list_out);
int fused_status(mirsha_ctx* c, mirsha_pipeline* p);
void pipeline_free(mirsha_pipeline* p);
int default_pipeline_mode();

}  // namespace mirsha_api
