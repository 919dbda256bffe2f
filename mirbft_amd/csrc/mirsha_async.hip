// mirsha_async.hip — the asynchronous, order-preserving ring
// (mirsha_submit_slices / mirsha_wait / mirsha_poll, content-addressed dedup):
// the hash stage of ProcessorWorkPool (processor.go:312-361, 447-470) without
// its completion-order output.
#include "mirsha_ctx.h"

namespace mirsha_api {

// Copies a completed submission's digests to the caller, in origin order.
int async_complete(mirsha_ctx* c, AsyncSlot& sl) {
    HIP_TRY(c, hipEventSynchronize(sl.done));
    const auto t_done = Clock::now();
    sl.prof[MIRSHA_PROF_DEVICE] = std::chrono::duration<double, std::milli>(t_done - sl.t_queued).count();
    const uint8_t* d = sl.dig.as<uint8_t>();
    if (sl.direct) {
        // mirsha_submit_batch into page-locked digests_out: already there
    } else if (sl.rank.empty()) {
        if (sl.n) memcpy(sl.user_out, d, 32ull * sl.n);
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
    std::vector<uint32_t>& len = c->sl_len;  // context scratch (single caller), grow-only
    if (dedup) {
        if (int rc = slice_args(c, slice_ptr, slice_len, slice_first, n, out)) return rc;
        if (len.size() < n) len.resize(n);  // each segment's lengths are set before it is queued
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
    sl.direct = false;
    HIP_TRY(c, sl.dig.ensure(32ull * std::max<uint32_t>(n, 1)));
    if (!sl.done) HIP_TRY(c, hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
    ph[MIRSHA_PROF_PLAN] = ms_since(t0);
    // Packs requests `ids` (identity when null) into `stage`, and queues their
    // digests into rows [row0, row0 + m) of sl.dig.
    auto queue = [&](const uint32_t* ids, uint32_t m, uint32_t row0, PinnedBuf& stage, DevBuf& dev) -> int {
        const auto tq = Clock::now();
        uint64_t bytes = 0;
        for (uint32_t k = 0; k < m; k++) bytes += len[ids ? ids[k] : k];
        if (bytes + kArenaSlack > MIRSHA_MAX_DEVICE_ARENA_BYTES)
            return fail(c, MIRSHA_ERANGE, "submission of %llu bytes exceeds one device arena (%u); split it",
                        (unsigned long long)bytes, MIRSHA_MAX_DEVICE_ARENA_BYTES);
        const uint64_t o_off = align8(bytes + kArenaSlack);
        const uint64_t o_len = o_off + 8ull * m, o_ord = o_len + 4ull * m, o_end = align8(o_ord + 4ull * m);
        const uint64_t o_dig = o_end;
        HIP_TRY(c, stage.ensure(o_end));
        HIP_TRY(c, dev.ensure(o_dig + 32ull * std::max<uint32_t>(m, 1)));
        uint8_t* st = stage.as<uint8_t>();
        // offsets and lengths straight into the staged metadata (no temporaries)
        uint64_t* poff = reinterpret_cast<uint64_t*>(st + o_off);
        uint32_t* plen = reinterpret_cast<uint32_t*>(st + o_len);
        uint64_t p = 0;
        for (uint32_t k = 0; k < m; k++) {
            const uint32_t i = ids ? ids[k] : k;
            poff[k] = p;
            plen[k] = len[i];
            p += len[i];
        }
        mirsha::host::pack(slice_ptr, slice_len, slice_first, ids, m, poff, st, mirsha::host::threads_for(bytes, m),
                           true);
        const bool identity = bucket_order(plen, m, reinterpret_cast<uint32_t*>(st + o_ord));
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


// mirsha_submit_batch: n requests of a caller arena (request i =
// arena[off[i], off[i] + len[i])), one slot of the ring.  The off / len
// arrays are read before the call returns.  A dense range [lo, hi) of a
// page-locked arena is DMA'd straight from it (no host copy: the caller must
// leave those bytes alone until the ticket retires); a pageable or sparse one
// is copied into the slot's pinned staging first (packed back to back when
// sparse), so the caller may reuse it at once.  Digests land in a page-locked
// digests_out by DMA, else in the slot's pinned rows, copied out when the
// ticket retires.  The Go binding's chunked HashBatch packs
// chunk k + 1 of a Ready() cycle while chunk k's DMA, kernel and D2H run.
int async_submit_arena(mirsha_ctx* c, const uint8_t* arena, uint64_t arena_len, const uint64_t* off,
                       const uint32_t* len, uint32_t n, uint8_t* out, uint64_t* ticket_out) {
    auto t0 = Clock::now();
    const auto t_entry = t0;
    double ph[MIRSHA_PROF_PHASES] = {};
    // MIRSHA_SUBMIT_TRACE=1 (with MIRSHA_AB=1): a submission slower than 2 ms
    // prints where its time went (ms since entry at each step) on stderr.
    double tr[6] = {}, tq[8] = {};
    auto trace_done = [&](const char* how) {
        const double tot = ms_since(t_entry);
        if (tot > 2.0 && getenv_flag("MIRSHA_SUBMIT_TRACE"))
            fprintf(stderr,
                    "mirsha submit trace: %.3f ms (%s): slot wait %.3f, meta buffer %.3f, validate %.3f, "
                    "buffers %.3f, pack %.3f, queue %.3f [ev_in %.3f meta %.3f wait %.3f scan %.3f kernel %.3f "
                    "ev_kern %.3f d2h %.3f done %.3f]\n",
                    tot, how, tr[0], tr[1], tr[2], tr[3], tr[4], tr[5], tq[0], tq[1], tq[2], tq[3], tq[4], tq[5],
                    tq[6], tq[7]);
    };
    // One pass over the n entries on the calling thread (up to 2^18
    // requests: a chunk of the Go binding's HashBatch is ~120k requests and
    // its goroutines pack the NEXT chunk meanwhile): bounds, the span [lo,
    // hi), total bytes, block-count range, whether the requests are gapless,
    // and the lengths into the metadata block.  Offsets cross PCIe only when
    // the requests are not gapless (else the device rebuilds them by a scan
    // of the lengths), the bucket order only when block counts differ: 4 B
    // per request instead of 16 in the common case (the metadata shares the
    // link with the request bytes and the digests).
    struct Part {
        uint64_t lo = UINT64_MAX, hi = 0, tot = 0;
        uint32_t bmin = UINT32_MAX, bmax = 0, bad = UINT32_MAX;
        bool gapless = true;
    };
    const int T = n < (1u << 18) ? 1
                                 : (int)std::min<uint32_t>((uint32_t)mirsha::host::max_threads(), n / (1u << 16));
    std::vector<Part> parts(T);
    const uint32_t step = n ? (n + (uint32_t)T - 1) / (uint32_t)T : 1;
    // Slot buffers: `stage2` = the metadata block [len u32 | order u32 | off
    // u64] (the device's copy has the same layout), `stage` = a copy of the
    // request bytes when they are not DMA'd from the caller, `dev` = [request
    // bytes + slack | metadata | digests].
    if (int rc = use_device(c)) return rc;
    AsyncSlot& sl = c->slots[(c->next_ticket - 1) % kAsyncSlots];
    if (sl.busy)
        if (int rc = async_wait_upto(c, sl.ticket)) return rc;  // ring full: retire the oldest
    tr[0] = ms_since(t_entry);
    const uint64_t o_len = 0, o_ord = align8(4ull * n), o_off = align8(o_ord + 4ull * n), o_end = o_off + 8ull * n;
    HIP_TRY(c, sl.stage2.ensure(std::max<uint64_t>(o_end, 8)));
    tr[1] = ms_since(t_entry);
    uint8_t* mb = sl.stage2.as<uint8_t>();
    uint32_t* slen = reinterpret_cast<uint32_t*>(mb + o_len);
    uint32_t* sord = reinterpret_cast<uint32_t*>(mb + o_ord);
    uint64_t* soff = reinterpret_cast<uint64_t*>(mb + o_off);
    // The metadata block is page-locked host memory: written once, never
    // read back by the host.
    mirsha::host::parallel_for(n, T, [&](uint32_t a, uint32_t b) {
        Part& q = parts[a / step];
        for (uint32_t i = a; i < b; i++) {
            const uint64_t o = off[i];
            const uint32_t L = len[i];
            if (L > MIRSHA_MAX_MESSAGE_BYTES || o > arena_len || L > arena_len - o) {
                q.bad = i;
                return;
            }
            slen[i] = L;
            if (i > a && o != off[i - 1] + len[i - 1]) q.gapless = false;
            q.lo = std::min(q.lo, o);
            q.hi = std::max(q.hi, o + L);
            q.tot += L;
            const uint32_t k = host_blocks(L);
            q.bmin = std::min(q.bmin, k);
            q.bmax = std::max(q.bmax, k);
        }
    });
    Part all;
    for (int k = 0; k < T; k++) {
        const Part& q = parts[k];
        all.bad = std::min(all.bad, q.bad);
        all.lo = std::min(all.lo, q.lo);
        all.hi = std::max(all.hi, q.hi);
        all.tot += q.tot;
        all.bmin = std::min(all.bmin, q.bmin);
        all.bmax = std::max(all.bmax, q.bmax);
        all.gapless = all.gapless && q.gapless;
        const uint32_t a = (uint32_t)k * step;  // part boundaries
        if (k > 0 && a < n && off[a] != off[a - 1] + len[a - 1]) all.gapless = false;
    }
    if (all.bad != UINT32_MAX) {
        const uint32_t i = all.bad;
        if (len[i] > MIRSHA_MAX_MESSAGE_BYTES)
            return fail(c, MIRSHA_ERANGE, "message %u is %u bytes (max %u)", i, len[i], MIRSHA_MAX_MESSAGE_BYTES);
        return fail(c, MIRSHA_EINVAL, "message %u [%llu,+%u) outside arena of %llu bytes", i,
                    (unsigned long long)off[i], len[i], (unsigned long long)arena_len);
    }
    const uint64_t lo = n ? all.lo : 0, hi = n ? all.hi : 0, total = all.tot;
    const uint64_t span = hi - lo;
    const bool dense = span <= 2 * total + 4096;
    const uint64_t bytes = dense ? span : total;
    if (bytes + kArenaSlack > MIRSHA_MAX_DEVICE_ARENA_BYTES)
        return fail(c, MIRSHA_ERANGE, "submission of %llu bytes exceeds one device arena (%u); split it",
                    (unsigned long long)bytes, MIRSHA_MAX_DEVICE_ARENA_BYTES);
    // gapless => in order from lo = off[0]: the device scan of the lengths is the offsets
    const bool gapless = n && dense && all.gapless;
    if (!gapless && dense) {
        mirsha::host::parallel_for(n, T, [&](uint32_t a, uint32_t b) {
            for (uint32_t i = a; i < b; i++) soff[i] = off[i] - lo;
        });
    } else if (!dense) {  // packed back to back: off = exclusive scan of len
        uint64_t p = 0;
        for (uint32_t i = 0; i < n; i++) {
            soff[i] = p;
            p += len[i];
        }
    }
    const bool identity = n == 0 || all.bmin == all.bmax || bucket_order(len, n, sord);
    // bytes of the metadata block that cross PCIe
    const uint64_t meta_copy = !gapless ? o_end : !identity ? o_ord + 4ull * n : 4ull * n;
    ph[MIRSHA_PROF_VALIDATE] = ms_since(t0);
    tr[2] = ms_since(t_entry);
    t0 = Clock::now();
    sl.rank.clear();
    for (hipEvent_t* e : {&sl.done, &sl.ev_in, &sl.ev_kern})
        if (!*e) HIP_TRY(c, hipEventCreateWithFlags(e, hipEventDisableTiming));
    // Request bytes in on xin, the kernel on the context stream; digests
    // stored by the kernel into a page-locked digests_out (metadata then on
    // xin too), else out on xout with the metadata on the kernel stream.
    // Submission k+1's DMA runs behind submission k's DMA, not behind its
    // kernel (PCIe is full duplex).
    if (!c->xin) HIP_TRY(c, hipStreamCreateWithFlags(&c->xin, hipStreamNonBlocking));
    if (!c->xout) HIP_TRY(c, hipStreamCreateWithFlags(&c->xout, hipStreamNonBlocking));
    const bool from_caller = dense && n && host_pinned(arena + lo);
    sl.direct = host_pinned(out);
    // A page-locked digests_out is written by the kernel itself (posted
    // writes over PCIe; visible when the kernel's completion is), and the
    // metadata follows the request bytes on xin: every SDMA copy of the
    // submission is then on one stream.  With copies on three streams (H2D,
    // metadata, D2H) the runtime now and then blocked a hipMemcpyAsync for
    // 8-15 ms (profiles/r05w: 13-22 ms calls of the chunked HashBatch); with
    // one copy stream no call stalled, at the same steady-state speed.
    uint8_t* kout = nullptr;
    if (sl.direct && n && (reinterpret_cast<uintptr_t>(out) & 15u) == 0 && kernel_writable_host(out, c->device)) {
        void* dp = nullptr;
        if (hipHostGetDevicePointer(&dp, out, 0) == hipSuccess)
            kout = static_cast<uint8_t*>(dp);
        else
            (void)hipGetLastError();
    }
    if (!sl.direct) HIP_TRY(c, sl.dig.ensure(32ull * std::max<uint32_t>(n, 1)));
    // device: [request bytes + slack | len u32 | order u32 | off u64 | digests]
    const uint64_t d_meta = align8(bytes + kArenaSlack), d_dig = d_meta + o_end;
    size_t scan_bytes = 0;
    if (gapless) {
        HIP_TRY(c, mirsha::launch_offsets_scan(nullptr, scan_bytes, nullptr, nullptr, n, c->stream));
        HIP_TRY(c, c->d_scan.ensure(std::max<size_t>(scan_bytes, 4)));
    }
    if (!from_caller) HIP_TRY(c, sl.stage.ensure(std::max<uint64_t>(bytes, 8)));
    HIP_TRY(c, sl.dev.ensure(d_dig + 32ull * n));
    uint8_t* st = sl.stage.as<uint8_t>();
    ph[MIRSHA_PROF_PLAN] = ms_since(t0);
    tr[3] = ms_since(t_entry);
    t0 = Clock::now();
    uint8_t* dv = sl.dev.as<uint8_t>();
    if (from_caller) {
        HIP_TRY(c, hipMemcpyAsync(dv, arena + lo, bytes, hipMemcpyHostToDevice, c->xin));
    } else if (dense) {
        mirsha::host::pack_range(arena + lo, nullptr, nullptr, nullptr, 0, nullptr, 0, bytes, st,
                                 mirsha::host::threads_for(bytes, 1u << 20), true);
    } else {
        std::vector<const uint8_t*> sp(n);
        std::vector<uint64_t> sz(n);
        std::vector<uint32_t> sf(n + 1);
        for (uint32_t i = 0; i < n; i++) {
            sp[i] = arena + off[i];
            sz[i] = len[i];
            sf[i] = i;
        }
        sf[n] = n;
        mirsha::host::pack(sp.data(), sz.data(), sf.data(), nullptr, n, soff, st, mirsha::host::threads_for(bytes, n),
                           true);
    }
    tr[4] = ms_since(t_entry);
    // Queue the copies and the kernel.  A failure part-way leaves work that
    // reads this slot's buffers in flight while the slot is not marked busy:
    // drain the three streams before reporting it.
    auto queue = [&]() -> int {
        if (n) {
            if (!from_caller && bytes) HIP_TRY(c, hipMemcpyAsync(dv, st, bytes, hipMemcpyHostToDevice, c->xin));
            // The metadata: behind the request bytes on xin when the kernel
            // stores the digests (one copy stream), else on the kernel stream.
            if (kout) HIP_TRY(c, hipMemcpyAsync(dv + d_meta, mb, meta_copy, hipMemcpyHostToDevice, c->xin));
            HIP_TRY(c, hipEventRecord(sl.ev_in, c->xin));
            tq[0] = ms_since(t_entry);
            if (!kout) HIP_TRY(c, hipMemcpyAsync(dv + d_meta, mb, meta_copy, hipMemcpyHostToDevice, c->stream));
            tq[1] = ms_since(t_entry);
            HIP_TRY(c, hipStreamWaitEvent(c->stream, sl.ev_in, 0));
            tq[2] = ms_since(t_entry);
            uint64_t* d_off = reinterpret_cast<uint64_t*>(dv + d_meta + o_off);
            const uint32_t* d_len = reinterpret_cast<const uint32_t*>(dv + d_meta + o_len);
            if (gapless)  // off = exclusive scan of len, on the device (c->d_scan: c->stream's scratch)
                HIP_TRY(c, mirsha::launch_offsets_scan(c->d_scan.p, scan_bytes, d_len, d_off, n, c->stream));
            tq[3] = ms_since(t_entry);
            if (int rc = timed_launch(c, 0, [&] {
                    return mirsha::launch_msgs(dv, bytes, d_off, d_len,
                                               identity ? nullptr
                                                        : reinterpret_cast<const uint32_t*>(dv + d_meta + o_ord),
                                               n, kout ? kout : dv + d_dig, c->variant, c->stream);
                }))
                return rc;
            tq[4] = ms_since(t_entry);
            if (kout) {  // the digests are in host memory when the kernel ends
                HIP_TRY(c, hipEventRecord(sl.done, c->stream));
                tq[7] = ms_since(t_entry);
                return MIRSHA_OK;
            }
            HIP_TRY(c, hipEventRecord(sl.ev_kern, c->stream));
            HIP_TRY(c, hipStreamWaitEvent(c->xout, sl.ev_kern, 0));
            tq[5] = ms_since(t_entry);
            HIP_TRY(c, hipMemcpyAsync(sl.direct ? out : sl.dig.as<uint8_t>(), dv + d_dig, 32ull * n,
                                      hipMemcpyDeviceToHost, c->xout));
            tq[6] = ms_since(t_entry);
        }
        HIP_TRY(c, hipEventRecord(sl.done, c->xout));
        tq[7] = ms_since(t_entry);
        return MIRSHA_OK;
    };
    if (int rc = queue()) {
        for (hipStream_t q : {c->xin, c->stream, c->xout}) (void)hipStreamSynchronize(q);
        return rc;
    }
    sl.t_queued = Clock::now();
    ph[MIRSHA_PROF_PACK] = ms_since(t0);
    tr[5] = ms_since(t_entry);
    trace_done("arena");
    sl.busy = true;
    sl.user_out = out;
    sl.n = n;
    sl.m = n;
    sl.ticket = c->next_ticket++;
    for (int k = 0; k < MIRSHA_PROF_PHASES; k++) sl.prof[k] = ph[k];
    *ticket_out = sl.ticket;
    return MIRSHA_OK;
}

}  // namespace mirsha_api

extern "C" {

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

int mirsha_submit_batch(mirsha_ctx* c, const uint8_t* arena, uint64_t arena_len, const uint64_t* off,
                        const uint32_t* len, uint32_t n, uint8_t* digests_out, uint64_t* ticket_out) {
    if (!c || !ticket_out) return MIRSHA_EINVAL;
    if (n && (!off || !len || !digests_out || (!arena && arena_len))) return fail(c, MIRSHA_EINVAL, "NULL argument");
    return async_submit_arena(c, arena, arena_len, off, len, n, digests_out, ticket_out);
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

}  // extern "C"
