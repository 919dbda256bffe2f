// mirsha_plan.hip — request -> batch-digest plans (mirsha_pipeline_*): the
// sequential plan, the fused launch with its placement probe, and
// overlapped cycles.
#include "mirsha_ctx.h"

namespace mirsha_api {

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
// B when the compacted lists are identity lists of B entries -- list k is
// entries [k B, min(k B + B, n)) and cidx[e] == e: BatchSize batches over
// consecutive requests (sequence.go:154-157 as the synthetic streams and the
// bench build them) -- else 0.  The chain kernel then computes bounds and
// indices instead of loading them (sha256_chain_kernel<true>).
uint32_t uniform_lists(const std::vector<uint32_t>& cidx, const std::vector<uint32_t>& cfirst) {
    const size_t n_lists = cfirst.size() - 1, n = cidx.size();
    if (n_lists == 0 || n == 0 || cfirst[1] == 0) return 0;
    const uint64_t B = cfirst[1];
    if ((n_lists - 1) * B >= n || n_lists * B < n) return 0;
    for (size_t k = 0; k < n_lists; k++)
        if (cfirst[k] != k * B) return 0;
    for (size_t e = 0; e < n; e++)
        if (cidx[e] != e) return 0;
    // A/B (MIRSHA_AB=1 MIRSHA_CHAIN_UNIFORM=0): the loaded-index form
    if (const char* e = mirsha::ab_getenv("MIRSHA_CHAIN_UNIFORM"))
        if (e[0] == '0') return 0;
    return (uint32_t)B;
}

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
    p->uniform = uniform_lists(p->cidx, p->cfirst);
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
                                    p->d_state.as<uint32_t>(), d_list_out, c->stream, p->uniform);
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

}  // namespace mirsha_api

extern "C" {

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

}  // extern "C"
