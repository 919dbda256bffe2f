// mirsha_multi.hip — several GPUs of one node from one process: the
// per-call mirsha_hash_batch_multi and the mirsha_multi drop-in.  Requests
// shard by contiguous range; no collective (actions.go:22-23).
#include "mirsha_ctx.h"

extern "C" {

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

// m->cut from inclusive prefix sums of the request bytes (empty requests
// counting 1): the request boundary nearest to k/nd of the bytes for every
// k, so each device's share is within half a request of the fair one.  Both
// the slice and the arena entry points cut this way.
void cut_nearest(mirsha_multi* m, const std::vector<uint64_t>& sum) {
    const uint32_t n = (uint32_t)sum.size();
    const uint64_t total = n ? sum[n - 1] : 0;
    const int nd = (int)m->ctx.size();
    m->cut.assign(nd + 1, n);
    m->cut[0] = 0;
    for (int k = 1; k < nd; k++) {
        const uint64_t want = (total * (uint64_t)k + nd / 2) / nd;
        uint32_t i = (uint32_t)(std::lower_bound(sum.begin(), sum.end(), want) - sum.begin());  // sum[i] >= want
        if (i < n && (i == 0 ? want : want - sum[i - 1]) * 2 > (sum[i] - (i ? sum[i - 1] : 0))) i++;
        m->cut[k] = std::max(std::min(i, n), m->cut[k - 1]);
    }
}

// Arena form: the same cut over the request lengths.
void arena_cut(mirsha_multi* m, const uint32_t* len, uint32_t n) {
    std::vector<uint64_t> sum(n);
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; i++) {
        total += std::max<uint32_t>(len[i], 1u);
        sum[i] = total;
    }
    cut_nearest(m, sum);
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
    cut_nearest(m, sum);
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
    arena_cut(m, len, n);  // equal bytes, nearest request boundary (as multi_cut)
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

int mirsha_submit_arena_multi(mirsha_multi* m, const uint8_t* arena, uint64_t arena_len, const uint64_t* off,
                              const uint32_t* len, uint32_t n, uint8_t* digests_out, uint64_t* ticket_out) {
    if (!m || !ticket_out) return MIRSHA_EINVAL;
    m->err.clear();
    if (n && (!off || !len || !digests_out || (!arena && arena_len))) return multi_fail(m, MIRSHA_EINVAL, "NULL argument");
    const uint64_t t = m->next_ticket;
    if (t > (uint64_t)kMultiAsyncSlots && m->done_ticket < t - kMultiAsyncSlots)
        if (int rc = mirsha_wait_multi(m, t - kMultiAsyncSlots)) return rc;
    arena_cut(m, len, n);
    const int nd = (int)m->ctx.size();
    std::vector<uint64_t> dt(nd, 0);
    const int rc = multi_run(m, [&](int k) -> int {
        const uint32_t a = m->cut[k], b = m->cut[k + 1];
        if (a >= b) return MIRSHA_OK;
        return mirsha_submit_batch(m->ctx[k], arena, arena_len, off + a, len + a, b - a, digests_out + 32ull * a,
                                   &dt[k]);
    });
    if (rc) {
        // as mirsha_submit_slices_multi: nothing lands after a failed call
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
