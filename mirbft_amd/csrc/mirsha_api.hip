// mirsha_api.hip — host side of the C-ABI declared in include/mirsha.h:
// contexts, timing, the device-pointer API, synthetic streams, streaming
// checkpoint chains and the clock probe.  The other host units are listed in
// mirsha_ctx.h.
#include "mirsha_ctx.h"

namespace mirsha_api {

int fail(mirsha_ctx* c, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (c) c->err = buf;
    return code;
}

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

int use_device(mirsha_ctx* c) {
    HIP_TRY(c, hipSetDevice(c->device));
    return MIRSHA_OK;
}

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

}  // namespace mirsha_api

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
    if (c->xin) (void)hipStreamSynchronize(c->xin);
    if (c->xout) (void)hipStreamSynchronize(c->xout);
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
        if (sl.ev_in) (void)hipEventDestroy(sl.ev_in);
        if (sl.ev_kern) (void)hipEventDestroy(sl.ev_kern);
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

}  // extern "C"
