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
