/*
 * mirsha.h — C-ABI of the MI355X (gfx950) Actions.Hash engine for MirBFT.
 *
 * This is the ONLY native boundary of the drop-in.  Plain pointers and sizes,
 * no torch / HIP types in the signatures (a hipStream_t is passed as void*).
 * It replaces the arithmetic of the reference's hash loop
 *
 *     for i, req := range actions.Hash {            // processor.go:133
 *         h := p.Hasher()                           // processor.go:134 (sha256.New)
 *         for _, data := range req.Data { h.Write(data) }   // :135-137
 *         actionResults.Digests[i] = &HashResult{Request: req, Digest: h.Sum(nil)} // :139-142
 *     }
 *
 * and the equivalent loops in ProcessorWorkPool (processor.go:312-361, whose
 * completion-order output is NOT reproduced: every entry point here returns
 * digests in ORIGIN order) and testengine's Recording (testengine/recorder.go:441-455).
 * The Go-side binding a maintainer adds is in INTEGRATION.md.
 *
 * Conventions
 *   - Return value: MIRSHA_OK (0) or a negative MIRSHA_E* code; the message is
 *     available from mirsha_last_error(ctx).  The reference converts processor
 *     failures into panics (processor.go:75,81,85,91); the Go wrapper does the same.
 *   - Digests are 32 bytes each, written to digests_out[32*i] for request i.
 *   - Host-pointer entry points are synchronous: outputs are complete on return.
 *     Device-pointer entry points (*_device) are asynchronous on the context's
 *     stream; call mirsha_sync() (or synchronise the stream) before reading.
 *   - A context is single-caller (not re-entrant), like the reference
 *     Processor (serialised by its caller, processor.go:447-449).  Each call
 *     makes the context's device current (cgo may migrate OS threads).
 */
#ifndef MIRSHA_H
#define MIRSHA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MIRSHA_OK 0
#define MIRSHA_EINVAL (-1)   /* bad argument (NULL pointer, range outside arena, ...) */
#define MIRSHA_EHIP (-2)     /* HIP runtime error */
#define MIRSHA_ENOMEM (-3)   /* device or pinned allocation failed */
#define MIRSHA_ERANGE (-4)   /* size limit exceeded (see per-function notes) */
#define MIRSHA_ENODEV (-5)   /* no usable gfx950 device */

/* Null request marker inside a digest index list: contributes an EMPTY digest
 * (0 bytes), as a null request's RequestAck.Digest does (client_tracker.go:840-847). */
#define MIRSHA_NULL_INDEX 0xFFFFFFFFu

/* Largest single message and largest arena one device launch addresses. */
#define MIRSHA_MAX_MESSAGE_BYTES 0xFFFFFF00u
#define MIRSHA_MAX_DEVICE_ARENA_BYTES 0xFFFFFF00u

typedef struct mirsha_ctx mirsha_ctx;

int mirsha_version(void); /* (major << 16) | minor */

/* Number of visible devices (hipGetDeviceCount). */
int mirsha_device_count(int* count);

/* Create / destroy a context bound to one device.  Replaces the per-request
 * `p.Hasher()` factory (processor.go:21, :58) with one long-lived engine. */
int mirsha_ctx_create(int device, mirsha_ctx** out);
void mirsha_ctx_destroy(mirsha_ctx* ctx);
const char* mirsha_last_error(const mirsha_ctx* ctx);

/* Launch on an external stream (e.g. the caller's current HIP stream) instead
 * of the context-owned one.  NULL restores the context's own stream. */
int mirsha_ctx_set_stream(mirsha_ctx* ctx, void* hip_stream);
void* mirsha_ctx_stream(mirsha_ctx* ctx);

/* Kernel form for sha256 over packed messages (A/B measurement):
 * 0 = LDS-staged coalesced loader + generated-asm rounds (default; a launch
 *     of at most 512 64-message groups takes the producer/consumer pair
 *     kernel -- schedule and rounds of each compression on two waves on two
 *     SIMDs -- and one of at most 1024 groups (one wave per SIMD) the
 *     low-occupancy kernel: prefetching direct loads, no-yield rounds;
 *     MIRSHA_AB=1 MIRSHA_PAIR=0 in the environment disables the pair forms,
 *     an A/B knob read only with MIRSHA_AB=1),
 *     A launch of 1,025..4,096 groups (at most 4 per SIMD) takes the CU-block
 *     kernel: one workgroup of 4k waves per CU, exactly k waves per SIMD,
 *     each wave's next block DMA'd into its LDS tile during this block.
 * 1 = direct per-lane loads, 4 = the low-occupancy kernel at any size,
 * 5 = the LDS kernel at any size, 6 = the pair kernel at any size,
 * 10 = the CU-block kernel at any size (groups beyond 4 per SIMD run in
 *     later workgroups, one CU at a time).
 * All of these are bit-exact.  Anything else is EINVAL: 2, 3, 7, 8 (round-1
 * A/B forms) are retired, and 11-15 (retired and diagnostic forms of the
 * CU-block kernel, one of which skips its loads) exist only in the tools A/B
 * build (tools/ab_build.sh lib), never in this library, whatever the
 * environment says. */
int mirsha_ctx_set_variant(mirsha_ctx* ctx, int variant);

/* Per-kernel device-time accounting with HIP events bound to each timed
 * launch's own dispatch (hipExtLaunchKernel): the kernel's start and end
 * timestamps, no marker packets (an event-bound launch still costs a few us
 * of stream time, so a benchmark times a sample of its launches).
 * kernel: 0 = message kernel, 1 = digest-list (batch) kernel, 2 = generator
 * and clock probe, 3 = batch-chain kernel, 4 = fused request -> batch kernel
 * (one persistent launch per run), 5 = overlapped-cycles kernel
 * (mirsha_pipeline_overlap_device).
 * set_timing_mask: bit k on = kernel k is timed while timing is enabled
 * (default: all). */
int mirsha_ctx_set_timing(mirsha_ctx* ctx, int enable);
int mirsha_ctx_set_timing_mask(mirsha_ctx* ctx, uint32_t mask);
int mirsha_ctx_kernel_time(mirsha_ctx* ctx, int kernel, uint64_t* launches, double* total_ms);
int mirsha_ctx_reset_timing(mirsha_ctx* ctx);

/* Wait for all work queued on the context's stream. */
int mirsha_sync(mirsha_ctx* ctx);

/* ---------------------------------------------------------------- host API */

/* processor.go:129-143 over n requests whose bytes are already concatenated:
 * request i = arena[off[i] .. off[i]+len[i]).  Any byte alignment.  Lengths
 * are bucketed by block count internally (longest first); the digest of
 * request i always lands at digests_out[32*i]. */
int mirsha_hash_batch(mirsha_ctx* ctx, const uint8_t* arena, uint64_t arena_len,
                      const uint64_t* off, const uint32_t* len, uint32_t n,
                      uint8_t* digests_out);

/* The same for HashRequest.Data [][]byte (actions.go:157-164) without a
 * caller-side copy: request i = concat(slice_ptr[s] for s in
 * [slice_first[i], slice_first[i+1])), slice_first has n+1 entries.
 * A multi-slice Write sequence hashes exactly its concatenation. */
int mirsha_hash_slices(mirsha_ctx* ctx, const uint8_t* const* slice_ptr,
                       const uint64_t* slice_len, const uint32_t* slice_first, uint32_t n,
                       uint8_t* digests_out);

/* Content-addressed dedup of one Ready() cycle.  During an
 * epoch change every node hashes the same EpochChange payload once per
 * acknowledging source (applyEpochChangeAckMsg, epoch_target.go:459-477, with
 * epochChangeHashData, stateless.go:311-340): N sources x N origins requests,
 * N distinct payloads.  Requests whose concatenated bytes are equal are hashed
 * ONCE; every duplicate still gets its own digest at digests_out[32*i], in
 * origin order (equality is confirmed byte for byte; the fingerprint only
 * groups candidates).  *n_unique_out (may be NULL) = distinct requests hashed.
 * At most MIRSHA_MAX_DEVICE_ARENA_BYTES of distinct bytes per call. */
int mirsha_hash_slices_dedup(mirsha_ctx* ctx, const uint8_t* const* slice_ptr,
                             const uint64_t* slice_len, const uint32_t* slice_first, uint32_t n,
                             uint8_t* digests_out, uint32_t* n_unique_out);

/* Host-only (no device, no context): the dedup plan the call above uses.
 * rep_out[i] = smallest j <= i whose request bytes equal request i's
 * (rep_out[i] == i for the first of each distinct content). */
int mirsha_dedup_plan(const uint8_t* const* slice_ptr, const uint64_t* slice_len,
                      const uint32_t* slice_first, uint32_t n, uint32_t* rep_out,
                      uint32_t* n_unique_out);

/* Page-locked host memory for the caller's request arena.  The cgo binding
 * packs each Ready() cycle's request bytes into one C arena before the call
 * (INTEGRATION.md); allocated here (once, reused every cycle) that arena is
 * DMA'd to the GPU at PCIe rate, where a malloc'ed one goes through the
 * runtime's pageable staging.  mirsha_host_free releases it. */
int mirsha_host_alloc(mirsha_ctx* ctx, uint64_t bytes, void** out);
void mirsha_host_free(void* p);

/* ---------------------------------------- asynchronous, order-preserving */
/* Replaces the hash stage of ProcessorWorkPool (processor.go:312-361,
 * 447-470) without its completion-order output: the caller
 * submits a Ready() cycle's requests, goes on with the WAL writes and network
 * sends the cycle also carries (actions.go:22-23 lets hashing run beside
 * them), then waits for the digests.
 *   mirsha_submit_slices packs the requests into the context's pinned staging
 *     before it returns (the caller may reuse the slices at once), queues the
 *     H2D copy, the kernel and the D2H copy, and returns a ticket (> 0).
 *     digests_out must stay valid until that ticket is waited for: the
 *     digests land there, in origin order, inside mirsha_wait / mirsha_poll.
 *     flags: 0 or MIRSHA_SUBMIT_DEDUP.  Up to 4 submissions are in flight;
 *     a fifth first retires the oldest.
 *   mirsha_wait blocks until every submission up to `ticket` is complete and
 *     its digests are written (submissions complete in submission order).
 *   mirsha_poll sets *done = 1 (and writes the digests) if every submission
 *     up to `ticket` is complete, else 0 without blocking. */
#define MIRSHA_SUBMIT_DEDUP 1
int mirsha_submit_slices(mirsha_ctx* ctx, const uint8_t* const* slice_ptr,
                         const uint64_t* slice_len, const uint32_t* slice_first, uint32_t n,
                         uint8_t* digests_out, int flags, uint64_t* ticket_out);
int mirsha_wait(mirsha_ctx* ctx, uint64_t ticket);
int mirsha_poll(mirsha_ctx* ctx, uint64_t ticket, int* done);
/* The same ring over a caller arena (mirsha_hash_batch's arguments): request
 * i = arena[off[i] .. off[i]+len[i]).  For the Go binding's chunked HashBatch
 * (replaces processor.go:133-143 for one Ready() cycle): the
 * caller packs chunk k+1 of the cycle into a page-locked arena
 * (mirsha_host_alloc) while chunk k, already submitted, is DMA'd, hashed and
 * its digests copied back.
 *   off / len are read before the call returns (Go memory is fine there).
 *   A page-locked arena is DMA'd straight from the caller's memory: its bytes
 *     [min off, max off+len) must not change until the ticket retires.  A
 *     pageable arena is copied into the context's staging before the call
 *     returns.
 *   digests_out: C memory, valid until the ticket retires (as
 *     mirsha_submit_slices).  A page-locked (mirsha_host_alloc) digests_out
 *     is written by the hashing kernel itself, with no copy: its rows are
 *     final when the ticket retires (mirsha_wait / mirsha_poll).
 *   At most MIRSHA_MAX_DEVICE_ARENA_BYTES of request bytes per submission
 *   (else MIRSHA_ERANGE; submit the cycle in chunks).  Shares the ring (4 in
 *   flight) and the tickets of mirsha_submit_slices: mirsha_wait / mirsha_poll. */
int mirsha_submit_batch(mirsha_ctx* ctx, const uint8_t* arena, uint64_t arena_len,
                        const uint64_t* off, const uint32_t* len, uint32_t n,
                        uint8_t* digests_out, uint64_t* ticket_out);

/* Host-side phases (milliseconds) of the context's last host-API call.
 * Slice submissions (mirsha_submit_slices / mirsha_hash_slices_dedup):
 * validate = slice lengths (dedup: the segmented scan -- validation plus a
 * fingerprint walk or a byte comparison per request); plan = dedup plan
 * (head assignment, the remaining byte-for-byte confirmations, resolution);
 * pack = gather into pinned staging + bucket order + queueing, over every
 * launch (dedup: the first segment's distinct requests are queued before the
 * rest is scanned, later ones in a second launch); device = first launch
 * queued -> complete (H2D, kernels, D2H, overlapping the dedup scan of the
 * later segments and any time the caller spent before waiting); scatter =
 * digests copied to the caller in origin order.
 * Synchronous calls (mirsha_hash_batch / _slices / _requests_then_batches /
 * mirsha_digest_lists): validate = arguments; pack = queueing the request
 * bytes (pinned arena: one DMA; else packing into pinned chunks behind their
 * DMA); plan = the metadata block; device = queue -> synchronised; scatter =
 * digests to the caller.  Large synchronous calls are pipelined (chunked
 * H2D, kernels and D2H overlap): there pack = host time spent packing, device
 * = host time spent waiting on the device, scatter = copying digests out, and
 * the phases overlap the DMA rather than add up.  total = the whole call.
 * Asynchronous submissions (mirsha_submit_slices): every phase belongs to the
 * most recently COMPLETED ticket (published when it retires: mirsha_wait,
 * mirsha_poll, or a later submission reusing its ring slot); total = 0.
 * Writes min(n, phases) entries; returns the number of phases. */
#define MIRSHA_PROF_VALIDATE 0
#define MIRSHA_PROF_PLAN 1
#define MIRSHA_PROF_PACK 2
#define MIRSHA_PROF_DEVICE 3
#define MIRSHA_PROF_SCATTER 4
#define MIRSHA_PROF_TOTAL 5
/* not a time: H2D chunks of the last synchronous call (0 = single-shot staging) */
#define MIRSHA_PROF_CHUNKS 6
#define MIRSHA_PROF_PHASES 7
int mirsha_ctx_host_profile(const mirsha_ctx* ctx, double* ms_out, int n);

/* Request digests, then the dependent batch digests computed ON DEVICE from
 * the device-resident request digests (no host round trip):
 *   batch b = SHA-256(concat(req_digest[idx[e]] for e in [batch_first[b], batch_first[b+1])))
 * idx[e] == MIRSHA_NULL_INDEX is a null request (0 bytes).  Mirrors
 * sequence.allocate (sequence.go:154-157) and batchTracker.applyForwardBatchMsg
 * (batch_tracker.go:147-150) feeding processResults (state_machine.go:394-397). */
int mirsha_hash_requests_then_batches(mirsha_ctx* ctx, const uint8_t* arena, uint64_t arena_len,
                                      const uint64_t* off, const uint32_t* len, uint32_t n_req,
                                      const uint32_t* idx, const uint32_t* batch_first,
                                      uint32_t n_batches, uint8_t* req_digests_out,
                                      uint8_t* batch_digests_out);

/* Digest lists over caller-provided 32-byte digests (host memory): batch /
 * VerifyBatch digests over known RequestAck digests, and the testengine
 * application checkpoint value = Sum of the running hash over the digests
 * committed since the last reset (testengine/recorder.go:213-256). */
int mirsha_digest_lists(mirsha_ctx* ctx, const uint8_t* digests, uint32_t n_digests,
                        const uint32_t* idx, const uint32_t* list_first, uint32_t n_lists,
                        uint8_t* digests_out);

/* -------------------------------------------------------------- device API */
/* All pointers are device pointers; asynchronous on the context stream.
 * Reads past arena_len return 0.  Any arena size: up to
 * MIRSHA_MAX_DEVICE_ARENA_BYTES one 32-bit buffer descriptor addresses it,
 * beyond that (BASELINE config 5: ~123 GB per GPU in one launch) the loader
 * switches to 64-bit per-lane addresses.  order (may be NULL) lists message
 * indices in processing order, e.g. from mirsha_bucket_order (longest first:
 * with mixed sizes this keeps the long chains off the launch's tail); NULL =
 * identity. */
int mirsha_hash_batch_device(mirsha_ctx* ctx, const uint8_t* d_arena, uint64_t arena_len,
                             const uint64_t* d_off, const uint32_t* d_len,
                             const uint32_t* d_order, uint32_t n, uint8_t* d_digests_out);

/* d_digests holds n_digests 32-byte digests (< 2^27; reads are range-checked,
 * an out-of-range index reads zeros).  n_entries = d_list_first[n_lists] (the
 * caller knows it; it sizes the library's scratch for lists that contain
 * MIRSHA_NULL_INDEX entries). */
int mirsha_digest_lists_device(mirsha_ctx* ctx, const uint8_t* d_digests, uint32_t n_digests,
                               const uint32_t* d_idx, const uint32_t* d_list_first, uint32_t n_lists,
                               uint32_t n_entries, uint8_t* d_digests_out);

/* -------------------------------------------- request -> batch pipeline */
/* The batch digests of a Ready() cycle form sequential SHA chains over the
 * request digests (batch b = SHA-256(d_0 || ... || d_{n-1}), sequence.go:154-157).
 * A pipeline plan overlaps the dependent pass with the request pass.  It is
 * built once from the (host) index lists and reused for every run with the
 * same shape (device API below); a plan is single-stream, like its context.
 * len (may be NULL) = request lengths, for length bucketing.
 *   MIRSHA_PIPELINE_FUSED: ONE launch.  Requests are hashed in the order in
 *     which the lists first need them, one tile wave per SIMD so tiles finish
 *     in that order; chain waves, alone on a few CUs, advance each list chunk
 *     by chunk as device-side readiness counters report the feeding request
 *     tiles done (no host round trip, no second stream).  Pays for a few long
 *     chains (VerifyBatch of hundreds of digests).
 *   MIRSHA_PIPELINE_SEQUENTIAL: request kernel at full occupancy, then the
 *     list kernel.  Best for many short lists (BatchSize 20).
 *   MIRSHA_PIPELINE_AUTO (default): FUSED when the longest list is >= 64
 *     blocks (~126 digests) and there are <= 64 list groups, else SEQUENTIAL;
 *     mirsha_pipeline_mode() reports the choice.
 * (Modes 2 and 4 -- chain segments on a second stream, and an in-kernel
 * continuation form -- were measured slower and are retired: EINVAL.)
 * mirsha_pipeline_create reads MIRSHA_PIPELINE_MODE (auto | fused |
 * sequential; default auto). */
#define MIRSHA_PIPELINE_SEQUENTIAL 0
#define MIRSHA_PIPELINE_FUSED 1
#define MIRSHA_PIPELINE_AUTO 3
/* Deprecated (round 1; kept one release so old callers still compile): the
 * retired modes.  mirsha_pipeline_create_mode returns MIRSHA_EINVAL for them. */
#define MIRSHA_PIPELINE_STREAMS 2
#define MIRSHA_PIPELINE_CONT 4
typedef struct mirsha_pipeline mirsha_pipeline;
int mirsha_pipeline_create(mirsha_ctx* ctx, uint32_t n_req, const uint32_t* len, const uint32_t* idx,
                           const uint32_t* list_first, uint32_t n_lists, mirsha_pipeline** out);
int mirsha_pipeline_create_mode(mirsha_ctx* ctx, uint32_t n_req, const uint32_t* len, const uint32_t* idx,
                                const uint32_t* list_first, uint32_t n_lists, int mode, mirsha_pipeline** out);
void mirsha_pipeline_destroy(mirsha_pipeline* p);
int mirsha_pipeline_mode(const mirsha_pipeline* p);
/* 1 if a FUSED (or AUTO -> fused) plan was built SEQUENTIAL instead because
 * the placement probe at creation found the device not dealing a
 * workgroup's waves evenly over the SIMDs (the fused launch deals its static
 * roles by SIMD; its kernel stays correct under any placement, but stacked
 * waves would run slower than the sequential plan); 0 otherwise. */
int mirsha_pipeline_fallback(const mirsha_pipeline* p);
/* Synchronises the context stream and reports a fused run whose readiness
 * watchdog expired (MIRSHA_EHIP; never expected, the launch is deadlock-free
 * by construction).  MIRSHA_OK otherwise.
 * Fail closed: a list pair whose wait expired stores no digest of its lists
 * (d_batch_out keeps its old bytes there) and sets the plan's sticky error
 * word (host-mapped memory); from then on every run on the plan
 * (mirsha_hash_requests_then_batches_device, mirsha_pipeline_overlap_device)
 * returns MIRSHA_EHIP without launching, and so does this call.  The device
 * calls are asynchronous: a run's own expiry is reported by the next call on
 * the plan or by this call after it.  Destroy the plan and create a new one.
 * (MIRSHA_AB=1 MIRSHA_TEST_FUSED_WATCHDOG=<ticks of 100 MHz> at plan creation
 * shortens the 2 s watchdog; tests only.) */
int mirsha_pipeline_status(mirsha_ctx* ctx, mirsha_pipeline* p);
/* Diagnostics of a fused plan created with MIRSHA_AB=1 MIRSHA_FUSED_TRACE=1 in the
 * environment: the last run's timeline (s_memrealtime ticks, 100 MHz) --
 * per tile [start, end, info] at [3t, 3t+1, 3t+2] (info = HW_ID | XCC_ID << 32
 * | queue << 40 | slot << 44), per readiness chunk the time its list wave
 * passed the wait at [3 n_tiles + c] and finished the chunk's blocks at
 * [3 n_tiles + n_counters + n_groups + c], per list group its end at
 * [3 n_tiles + n_counters + g].  *words = total length (0 when tracing is off). */
int mirsha_pipeline_trace(mirsha_ctx* ctx, mirsha_pipeline* p, uint64_t* out, uint64_t cap, uint64_t* words);
int mirsha_pipeline_shape(const mirsha_pipeline* p, uint32_t* n_tiles, uint32_t* n_counters, uint32_t* n_groups);
/* Deprecated (round 1's chain-segment mode, retired): kept one release so old
 * callers still link.  Every plan is one segment: *n_segments = 1 and, if
 * cap >= 1, bounds[0] = 0. */
int mirsha_pipeline_segments(const mirsha_pipeline* p, uint32_t* n_segments, uint32_t* bounds, uint32_t cap);
/* Split tiles of a fused plan: request tiles beyond the launch's tile-wave
 * slots, each run as *segments_per_tile sequential block-range segments
 * spread one per SIMD (0, 0 when none). */
int mirsha_pipeline_split_tiles(const mirsha_pipeline* p, uint32_t* n_split, uint32_t* segments_per_tile);
/* Device-resident run: request digests to d_req_out (origin order), batch
 * digests to d_batch_out; asynchronous on the context stream. */
int mirsha_hash_requests_then_batches_device(mirsha_ctx* ctx, mirsha_pipeline* p, const uint8_t* d_arena,
                                             uint64_t arena_len, const uint64_t* d_off, const uint32_t* d_len,
                                             uint8_t* d_req_out, uint8_t* d_batch_out);

/* Overlapped cycles.  The state machine batches request digests it already holds, i.e.
 * results of EARLIER Ready() cycles (sequence.go:154-157), so in a stream of
 * cycles ONE launch hashes this cycle's requests (d_arena.. -> d_req_out, origin
 * order, as mirsha_hash_requests_then_batches_device) together with the batch
 * digests of the previous cycle over ITS request digests d_prev_req (p's lists)
 * into d_prev_batch_out.  Sequential plans (many short lists, BatchSize 20):
 * the chains run beside the request tiles at full occupancy instead of in a
 * second launch of lone chain waves.  Fused plans (long VerifyBatch chains):
 * the fused launch with its list pairs reading complete digests, so they
 * never wait on tiles.  d_req_out == NULL: chains only (the last cycle's
 * flush); d_prev_req == NULL: requests only (the first cycle).  d_prev_req must stay intact until the launch ends
 * (the context stream orders it).  Asynchronous on the context stream. */
int mirsha_pipeline_overlap_device(mirsha_ctx* ctx, mirsha_pipeline* p, const uint8_t* d_arena, uint64_t arena_len,
                                   const uint64_t* d_off, const uint32_t* d_len, uint8_t* d_req_out,
                                   const uint8_t* d_prev_req, uint8_t* d_prev_batch_out);

/* Host helper: order[] = message indices sorted by SHA-256 block count,
 * longest first (stable), so a wave's 64 lanes run equal-length chains.
 * Returns 1 if the order is the identity (all lengths in one bucket), else 0. */
int mirsha_bucket_order(const uint32_t* len, uint32_t n, uint32_t* order_out);

/* ------------------------------------- streaming checkpoint chains (f4) */
/* Device-resident running SHA-256 states, one per application node: the
 * testengine application's checkpoint value is Sum() of a hash into which
 * every committed request digest is written (NodeState.Commit,
 * testengine/recorder.go:213-256: ActiveHash.Write :223, Sum :244) and which
 * restarts at each checkpoint (NodeState.Set, :186-207).
 *   mirsha_chains_absorb: ActiveHash.Write(digest) for m 32-byte digests, in
 *     order; digest i goes to chain chain_of[i].  A null request's digest is
 *     empty and its Write changes nothing: leave it out.
 *   mirsha_chains_sum: ActiveHash.Sum(nil) of chains which[0..k) into
 *     out[32*j]; like Go's Sum it leaves the states unchanged.
 *   mirsha_chains_reset: ActiveHash = Hasher() for chains which[0..k).
 * Synchronous; chain ids < n_chains (else MIRSHA_EINVAL). */
typedef struct mirsha_chains mirsha_chains;
int mirsha_chains_create(mirsha_ctx* ctx, uint32_t n_chains, mirsha_chains** out);
void mirsha_chains_destroy(mirsha_chains* chains);
int mirsha_chains_absorb(mirsha_ctx* ctx, mirsha_chains* chains, const uint8_t* digests, const uint32_t* chain_of,
                         uint32_t m);
int mirsha_chains_sum(mirsha_ctx* ctx, mirsha_chains* chains, const uint32_t* which, uint32_t k, uint8_t* out);
int mirsha_chains_reset(mirsha_ctx* ctx, mirsha_chains* chains, const uint32_t* which, uint32_t k);

/* ------------------------------------------------- multi-GPU (one process) */
/* Shards the n requests by contiguous range across ndev devices (balanced by
 * block count), one context per device, host gather into origin order.  No
 * collective: requests are independent (actions.go:22-23). */
int mirsha_hash_batch_multi(const int* devices, int ndev, const uint8_t* arena,
                            uint64_t arena_len, const uint64_t* off, const uint32_t* len,
                            uint32_t n, uint8_t* digests_out);
/* Contexts mirsha_hash_batch_multi keeps per device between calls: freed here
 * (optional; otherwise at process exit). */
void mirsha_multi_release(void);

/* The multi-GPU drop-in: a Go caller's Ready() cycle crosses PCIe at about
 * one link's rate per call (config 2: ~50 GB/s), so one device caps every
 * host-memory caller; the reference's pool scales with cores instead
 * (processor.go:401-410, HashWorkers = runtime.NumCPU()).  A mirsha_multi
 * holds one context per listed device (its own stream, pinned staging ring,
 * PCIe link) and one host worker per device with its own packing pool (an
 * equal share of the host threads).  Each call validates the slice lists,
 * cuts the requests into contiguous ranges of equal bytes (one per device;
 * ranges may be empty), and runs mirsha_hash_slices / mirsha_submit_slices
 * on every range in parallel; digests land at digests_out[32*i] in origin
 * order.  A device may be listed twice (two contexts on it: tests).  With
 * MIRSHA_SUBMIT_DEDUP each device deduplicates within its own range.
 * Single-caller, like a context.  At most 16 devices. */
typedef struct mirsha_multi mirsha_multi;
int mirsha_multi_create(const int* devices, int ndev, mirsha_multi** out);
void mirsha_multi_destroy(mirsha_multi* m);
const char* mirsha_multi_last_error(const mirsha_multi* m);
int mirsha_multi_devices(const mirsha_multi* m);
/* Context of device index k (0 <= k < ndev) for per-device settings and
 * diagnostics (mirsha_ctx_set_variant, timing); owned by m. */
mirsha_ctx* mirsha_multi_ctx(mirsha_multi* m, int k);
/* Request-range cut of the last call (every entry point cuts at the request
 * boundary nearest to k/ndev of the bytes): first_out[k] = first request of device
 * index k, first_out[ndev] = n.  Returns ndev + 1 (entries written: min(cap, ndev + 1)). */
int mirsha_multi_last_cut(const mirsha_multi* m, uint32_t* first_out, int cap);
int mirsha_hash_slices_multi(mirsha_multi* m, const uint8_t* const* slice_ptr,
                             const uint64_t* slice_len, const uint32_t* slice_first, uint32_t n,
                             uint8_t* digests_out);
/* The same over a caller arena (mirsha_hash_batch on every range): with a
 * page-locked arena from mirsha_multi_host_alloc every device DMAs its range
 * straight from it over its own link (the Go binding's GPUHasherMulti packs
 * one Ready() cycle into that arena with GOMAXPROCS goroutines). */
int mirsha_hash_arena_multi(mirsha_multi* m, const uint8_t* arena, uint64_t arena_len,
                            const uint64_t* off, const uint32_t* len, uint32_t n, uint8_t* digests_out);
/* Page-locked host memory usable by every device of m (portable); free with mirsha_host_free. */
int mirsha_multi_host_alloc(mirsha_multi* m, uint64_t bytes, void** out);
/* Asynchronous form (mirsha_submit_slices on every range): up to 4
 * submissions in flight; wait / poll cover every device's range of every
 * submission up to `ticket`.  The caller may reuse the slices when submit returns. */
int mirsha_submit_slices_multi(mirsha_multi* m, const uint8_t* const* slice_ptr,
                               const uint64_t* slice_len, const uint32_t* slice_first, uint32_t n,
                               uint8_t* digests_out, int flags, uint64_t* ticket_out);
/* mirsha_submit_batch over several devices: the requests cut into contiguous
 * ranges of equal bytes (as mirsha_hash_arena_multi), each range submitted to
 * its device's ring, DMA'd straight from a page-locked arena
 * (mirsha_multi_host_alloc) over that device's own link.  Tickets, wait and
 * poll as mirsha_submit_slices_multi. */
int mirsha_submit_arena_multi(mirsha_multi* m, const uint8_t* arena, uint64_t arena_len,
                              const uint64_t* off, const uint32_t* len, uint32_t n,
                              uint8_t* digests_out, uint64_t* ticket_out);
int mirsha_wait_multi(mirsha_multi* m, uint64_t ticket);
int mirsha_poll_multi(mirsha_multi* m, uint64_t ticket, int* done);
/* mirsha_ctx_host_profile of device index k's last call (its range only). */
int mirsha_multi_host_profile(const mirsha_multi* m, int k, double* ms_out, int n);

/* ------------------------------------------- benchmark / test utility only */
/* Device-side synthetic request stream, byte-identical to the
 * oracle generator: request i = LE64(i%16) || LE64(i/16) || data_len bytes of
 * splitmix64(splitmix64(seed ^ i) + j).  count messages packed densely. */
int mirsha_synth_requests_device(mirsha_ctx* ctx, uint64_t seed, uint64_t first, uint64_t count,
                                 uint32_t data_len, uint8_t* d_arena);
/* BASELINE config 5 stream (mixed 64 B - 64 KB): d_len[r] = message length
 * (16 + data_len) of request first + r, data_len log-uniform over the octaves
 * of [64, 65536) in integer arithmetic (identical to the oracle's
 * oracle_mixed_data_len); then the message bytes (same layout and data as
 * above) at d_arena + d_off[r], any byte alignment. */
int mirsha_synth_mixed_lengths_device(mirsha_ctx* ctx, uint64_t seed, uint64_t first, uint64_t count,
                                      uint32_t* d_len);
int mirsha_synth_mixed_device(mirsha_ctx* ctx, uint64_t seed, uint64_t first, uint64_t count,
                              const uint64_t* d_off, uint8_t* d_arena);

/* Clock probe (diagnostics; bench.py runs it right after its timed region):
 * every SIMD runs 8 waves of `iters` back-to-back register-only compressions
 * in the request kernel's round form.  *clock_ghz = median over waves of
 * shader cycles / 100 MHz reference ticks (the clock held under this load);
 * *cycles_per_wave_compression = launch span (first wave start to last wave
 * end, in shader cycles at that clock) / (iters x 8): the SIMD cycles one
 * 64-lane compression costs with no memory traffic at all (the measured
 * ceiling the request kernel is compared with).  Synchronous. */
int mirsha_clock_probe(mirsha_ctx* ctx, uint32_t iters, double* clock_ghz, double* cycles_per_wave_compression);

#ifdef __cplusplus
}
#endif
#endif /* MIRSHA_H */
