// mirsha_staging.hip — the synchronous host API (the Go drop-in's path: one
// call per Ready() cycle): staging, the pipelined H2D / kernel / D2H form,
// slice validation, and mirsha_hash_batch / _slices /
// _requests_then_batches, mirsha_digest_lists.
#include "mirsha_ctx.h"

namespace mirsha_api {

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
                             mirsha::host::threads_for(b - a, 1u << 20), true);
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

// A synchronous call that fails after queueing copies returns only once the
// context's streams have drained: nothing may still read the caller's arena
// or write its outputs after the call returns.  Disarmed on success (every
// queued operation was waited for).
struct DrainOnError {
    mirsha_ctx* c;
    bool on = true;
    ~DrainOnError() {
        if (!on) return;
        (void)hipStreamSynchronize(c->stream);
        if (c->xin) (void)hipStreamSynchronize(c->xin);
        if (c->xout) (void)hipStreamSynchronize(c->xout);
    }
};

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
    // Chunk k covers arena bytes [cb[k], cb[k+1]): 8, 16, then 32 MiB, so the
    // link is busy early while the pool fills the next (larger) chunk.
    std::vector<uint64_t> cb{0};
    for (uint64_t x = 0, step = kFirstChunk; x < total; step = std::min(2 * step, kStageChunk)) {
        x = std::min(total, x + step);
        cb.push_back(x);
    }
    const uint32_t nch = (uint32_t)cb.size() - 1;
    if (!c->xin) HIP_TRY(c, hipStreamCreateWithFlags(&c->xin, hipStreamNonBlocking));
    if (!c->xout) HIP_TRY(c, hipStreamCreateWithFlags(&c->xout, hipStreamNonBlocking));
    // A failure after the first copy is queued returns only once the streams
    // have drained (DrainOnError).
    DrainOnError drain{c};
    // events: in[k], kern[k], out[k] per chunk; lists kernel; lists out
    HIP_TRY(c, take_events(c, 3ull * nch + 2));
    hipEvent_t* ev_in = c->xev.data();
    hipEvent_t* ev_kern = ev_in + nch;
    hipEvent_t* ev_out = ev_kern + nch;
    hipEvent_t ev_lk = ev_out[nch], ev_lo = ev_out[nch + 1];
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
    // Before the plan: every chunk of a page-locked arena (DMA queued only),
    // else as many as the ring holds, so the plan's host time runs under
    // their DMA instead of leaving the link idle.
    uint32_t queued = 0;
    auto queue_upto = [&](uint32_t m) -> int {
        for (; queued < m; queued++)
            if (int rc = queue_in(queued)) return rc;
        return MIRSHA_OK;
    };
    if (int rc = queue_upto(pinned_src ? nch : std::min<uint32_t>(nch, (uint32_t)kStageSlots))) return rc;

    // Metadata, on the kernel stream (not behind the chunks on xin).  Chunk k
    // hashes the messages [cut[k], cut[k+1]): those ending within its bytes
    // [0, cb[k+1]).
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
    // (The plan's passes run while the first chunks cross PCIe: spread wide,
    // ~32 bytes of work per request.)
    std::atomic<uint32_t> lo_b{UINT32_MAX}, hi_b{0};
    mirsha::host::parallel_for(n, mirsha::host::threads_for(32ull * n, n), [&](uint32_t a, uint32_t b) {
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
        mirsha::host::parallel_for(n, mirsha::host::threads_for(32ull * n, n), [&](uint32_t a, uint32_t b) {
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
    HIP_TRY(c, hipMemcpyAsync(c->d_meta.p, h, L.copy, hipMemcpyHostToDevice, c->stream));
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
        if (int rc = queue_upto(k + 1)) return rc;
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
    // The rest as it comes back: wait for the next chunk, copy it together
    // with every later chunk already back, while the remaining DMA runs.
    while (copied < nch) {
        const auto w = Clock::now();
        HIP_TRY(c, hipEventSynchronize(ev_out[copied]));
        t_wait += ms_since(w);
        mark("w", copied);
        uint32_t ready = copied + 1;
        while (ready < nch) {
            const hipError_t q = hipEventQuery(ev_out[ready]);
            if (q == hipErrorNotReady) {
                (void)hipGetLastError();
                break;
            }
            if (q != hipSuccess) return fail(c, MIRSHA_EHIP, "hipEventQuery: %s", hipGetErrorString(q));
            ready++;
        }
        copy_out(copied, ready);
        copied = ready;
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
    drain.on = false;  // every event waited for above
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
    DrainOnError drain{c};
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
    drain.on = false;
    return MIRSHA_OK;
}

// Validates messages of a caller arena: the dense span [lo, hi) they cover,
// their total length, and their layout (in index order: off[i] >= off[i-1] +
// len[i-1]; gapless: equality).  One parallel pass.
int arena_span(mirsha_ctx* c, uint64_t arena_len, const uint64_t* off, const uint32_t* len, uint32_t n,
               uint64_t* lo_out, uint64_t* hi_out, uint64_t* total_out, ArenaLayout* layout_out) {
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

// Validates a slice-list request set and returns each request's total length.
// The first request with a per-request slice error (err[i]: 0 ok, 1 not
// monotone, 2 NULL slice, 3 too long), reported as the call's error.
int slice_errors_at(mirsha_ctx* c, uint8_t code, uint32_t i) {
    if (code == 1) return fail(c, MIRSHA_EINVAL, "slice_first not monotone at request %u", i);
    if (code == 2) return fail(c, MIRSHA_EINVAL, "request %u has a NULL slice", i);
    if (code == 3) return fail(c, MIRSHA_ERANGE, "request %u exceeds %u bytes", i, MIRSHA_MAX_MESSAGE_BYTES);
    return MIRSHA_OK;
}

int slice_errors(mirsha_ctx* c, const uint8_t* err, uint32_t n) {
    for (uint32_t i = 0; i < n; i++)
        if (err[i]) return slice_errors_at(c, err[i], i);
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
    if (len.size() < n) len.resize(n);  // grow-only: a reused vector is not cleared
    // The first bad request of each thread's range, and its code (1 not
    // monotone, 2 NULL slice, 3 too long); the lowest index is reported.
    const uint64_t meta = 16ull * (ns > slice_first[0] ? ns : 0u);
    const int T = mirsha::host::threads_for(meta, n);
    std::vector<uint32_t> bad(std::max(T, 1), UINT32_MAX);
    std::vector<uint8_t> code(std::max(T, 1), 0);
    const uint32_t step = (n + (uint32_t)std::max(T, 1) - 1) / (uint32_t)std::max(T, 1);
    mirsha::host::parallel_for(n, T, [&](uint32_t lo, uint32_t hi) {
        const uint32_t k = lo / std::max<uint32_t>(step, 1);
        for (uint32_t i = lo; i < hi; i++) {
            uint8_t e = 0;
            uint64_t L = 0;
            if (slice_first[i + 1] < slice_first[i] || slice_first[i + 1] > ns) {
                e = 1;
            } else {
                for (uint32_t s = slice_first[i]; s < slice_first[i + 1]; s++) {
                    if (slice_len[s] && !slice_ptr[s]) { e = 2; break; }
                    L += slice_len[s];
                }
                if (!e && L > MIRSHA_MAX_MESSAGE_BYTES) e = 3;
            }
            if (e) {
                bad[k] = i;
                code[k] = e;
                return;
            }
            len[i] = (uint32_t)L;
        }
    });
    uint32_t first_bad = UINT32_MAX;
    uint8_t first_code = 0;
    for (size_t k = 0; k < bad.size(); k++)
        if (bad[k] < first_bad) {
            first_bad = bad[k];
            first_code = code[k];
        }
    if (first_bad == UINT32_MAX) return MIRSHA_OK;
    return slice_errors_at(c, first_code, first_bad);
}

}  // namespace mirsha_api

extern "C" {

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
    std::vector<uint32_t>& len = c->sl_len;
    if (int rc = slice_lengths(c, slice_ptr, slice_len, slice_first, n, out, len)) return rc;
    c->prof[MIRSHA_PROF_VALIDATE] = ms_since(t0);
    if (int rc = use_device(c)) return rc;
    // One packing pass, by threads, straight into pinned staging (the Go
    // side's single copy), chunk by chunk behind the DMA of the previous one.
    std::vector<uint64_t>& poff = c->sl_poff;
    if (poff.size() < n) poff.resize(n);
    const uint64_t p = mirsha::host::exclusive_scan(len.data(), n, poff.data());
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

}  // extern "C"
