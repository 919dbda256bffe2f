// mirsha_kernels.h — internal launcher declarations (not part of the C-ABI).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mirsha {

constexpr uint32_t kWavesPerBlock = 4;
constexpr uint32_t kBlockThreads = 64 * kWavesPerBlock;
constexpr uint32_t kNullIndex = 0xFFFFFFFFu;

// sha256_msgs_kernel forms.  Default kVariantLds: the LDS-staged coalesced
// loader, whose small launches take latency forms (<= pair_max_groups()
// tiles: producer/consumer pairs; <= kLowOccTiles tiles, one wave per SIMD:
// the low-occupancy prefetching kernel).  The others force one form at any
// size (A/B, tests).  Numbers 2, 3, 7, 8 (round-1 A/B forms) are retired.
enum : int {
    kVariantLds = 0,
    kVariantDirect = 1,   // direct per-lane loads
    kVariantLowOcc = 4,
    kVariantLdsOnly = 5,
    kVariantPair = 6,
    kVariantCu = 10,      // CU-block form (one workgroup per CU, LDS-DMA loads one block ahead; <= 4 tiles per SIMD)
    // Forms of the CU-block kernel compiled ONLY into the tools A/B library
    // (tools/ab_build.sh lib, -DMIRSHA_AB_FORMS; never the product):
    kVariantCuNoYield = 11,  // register-prefetching block loop, no-yield rounds
    kVariantCuPrefetch = 12, // register-prefetching block loop (round 3's product form)
    kVariantCuDmaPipe = 13,  // LDS-DMA, the next block's words read back mid-block
    kVariantCuDiagNoLoads = 14,  // diagnostic: without its block loads (its digests are NOT valid)
    kVariantCuDiagNoPrio = 15,   // diagnostic: without its per-block issue priorities
};
const char* ab_getenv(const char* name);
inline bool variant_is_ab_form(int v) {
#ifdef MIRSHA_AB_FORMS
    return v >= kVariantCuNoYield && v <= kVariantCuDiagNoPrio;
#else
    (void)v;
    return false;  // the product library accepts bit-exact forms only
#endif
}
inline bool variant_valid(int v) {
    return v == kVariantLds || v == kVariantDirect || v == kVariantLowOcc || v == kVariantLdsOnly || v == kVariantPair ||
           v == kVariantCu || variant_is_ab_form(v);
}
constexpr uint32_t kCuMaxWavesPerSimd = 4;
uint32_t cu_count();
// Schedule A/B and diagnostic knobs are read from the environment only when
// MIRSHA_AB=1 is set too (never in production).  Every knob the product
// library reads keeps the digests bit-exact (tests/test_gpu_parity.py runs
// them); the one form that does not (variant 14) exists only in the tools
// A/B library.
constexpr uint32_t kLowOccTiles = 1024;   // 256 CUs x 4 SIMDs
// Small launches take a latency form: at most pair_max_groups() 64-message
// groups (default kPairMaxGroups: <= 2 pairs per CU, every wave alone on a
// SIMD) the producer/consumer pair kernels.  Environment (A/B):
// MIRSHA_PAIR=0 turns the automatic choice off, MIRSHA_PAIR_MAX_GROUPS=n
// moves the threshold.
constexpr uint32_t kPairMaxGroups = 512;
uint32_t pair_max_groups();

// Arenas up to kMaxBufferArena bytes use one 32-bit buffer descriptor; larger
// ones (any size) the 64-bit per-lane addressed loader.
constexpr uint64_t kMaxBufferArena = 0xFFFFFF00ull;
// ... and digests through one descriptor (32-bit offsets 32 i) up to 2^27 messages.
constexpr uint32_t kMaxBufferMsgs = 1u << 27;
// off[i] = len[0] + ... + len[i-1] (exclusive scan; mirsha_scan.hip).  With
// tmp == nullptr only sets tmp_bytes (the scratch size for n requests).
hipError_t launch_offsets_scan(void* tmp, size_t& tmp_bytes, const uint32_t* len, uint64_t* off, uint32_t n,
                               hipStream_t s);
// Timing events for the next kernel this thread launches (timed_launch):
// bound to that kernel's own dispatch through hipExtLaunchKernel, so they
// carry its start and end timestamps and add no marker packets to the stream
// (separate hipEventRecord markers around each launch cost ~2.7 us of stream
// time apiece on gfx950, profiles/r06g).  Consumed (reset) by the launch.
struct LaunchEvents {
    hipEvent_t start = nullptr, stop = nullptr;
};
LaunchEvents& next_launch_events();

hipError_t launch_msgs(const uint8_t* arena, uint64_t arena_len, const uint64_t* off,
                       const uint32_t* len, const uint32_t* order, uint32_t n, uint8_t* out,
                       int variant, hipStream_t s);
// scratch: device buffer with at least first[n_lists] entries (null compaction).
// Digest reads are range-checked against n_digests (out-of-range reads zeros).
constexpr uint32_t kMaxListDigests = (1u << 27) - 1u;
// Index reads are range-checked against n_entries (= first[n_lists]).
constexpr uint32_t kMaxListEntries = (1u << 30) - 1u;
hipError_t launch_lists(const uint8_t* digests, uint32_t n_digests, const uint32_t* idx, uint32_t n_entries,
                        const uint32_t* first, uint32_t n_lists, uint32_t* scratch, uint8_t* out, hipStream_t s);
// One segment [ob, oe) of every (compacted) list chain; oe = kOpenEnd finalises all.
// uniform = B > 0: the lists are identity lists of B entries (list k =
// entries [k B, min(k B + B, n_entries)), cidx[e] == e); cidx / cfirst unread.
constexpr uint32_t kOpenEnd = 0xFFFFFFFEu;
// K[j] + W[j] of a padding-only final block (0x80, zeros, the 64-bit bit
// length of a message of L bytes, L a multiple of 64): its whole message
// schedule is a constant (pad_block_kw, host side).
struct PadBlockKW {
    uint32_t kw[64];
    uint32_t use;  // 0: no constant-block path (odd B, or the A/B knob MIRSHA_CHAIN_PAD=0)
};
PadBlockKW pad_block_kw(uint64_t L);
hipError_t launch_chain(const uint8_t* digests, uint32_t n_digests, const uint32_t* cidx, uint32_t n_entries,
                        const uint32_t* cfirst, uint32_t n_lists, uint32_t ob, uint32_t oe, uint32_t* state,
                        uint8_t* out, hipStream_t s, uint32_t uniform = 0);
// Whole (compacted) list chains by producer/consumer pairs, one 128-thread
// workgroup per 64 lists; for at most kPairMaxGroups groups.
hipError_t launch_chain_pair(const uint8_t* digests, uint32_t n_digests, const uint32_t* cidx, uint32_t n_entries,
                             const uint32_t* cfirst, uint32_t n_lists, uint8_t* out, hipStream_t s);
// Overlapped cycles (see mirsha_kernels.hip): this cycle's request tiles and
// the previous cycle's compacted list chains in one launch.
struct OverlapArgs {
    const uint8_t* arena;
    uint64_t arena_len;
    const uint64_t* off;
    const uint32_t* len;
    const uint32_t* order;  // NULL = identity
    uint32_t n_req;         // this cycle's requests (0: chains only)
    uint8_t* req_out;
    const uint8_t* prev_digests;  // previous cycle's request digests
    uint32_t n_req_prev;
    const uint32_t* cidx;
    uint32_t n_entries;
    const uint32_t* cfirst;
    uint32_t n_lists;
    uint8_t* list_out;
    uint32_t list_waves;  // (n_lists + 63) / 64, or 0: no chains this launch
    uint32_t chain_prio;  // A/B (MIRSHA_OVERLAP_CHAIN_PRIO): 0 by fraction of the chain, 1 = 3 - block, 2 = 3, 3 = 1
};
hipError_t launch_msgs_overlap(const OverlapArgs& a, hipStream_t s);
// Fused request -> list pass (one persistent launch), see mirsha_kernels.hip.
constexpr uint32_t kFusedChunkBlocks = 2;  // list blocks (4 digests) per readiness chunk
// Tile queues of the fused launch: queue q holds tiles [q_first[q], q_first[q+1])
// in needed-at order and is served first by the tile waves of slot q on every
// SIMD, at issue priority prio_of(q) (earliest-needed tiles win issue).
constexpr uint32_t kFusedMaxQueues = 4;
// ctl words (u64, one 128-B line each): tile tickets at kCtlTileTicket + 16 q,
// retired-wave count (the launch's last wave resets the tickets)
constexpr uint32_t kCtlTileTicket = 0, kCtlDone = 80, kCtlWords = 96;
// Readiness-wait watchdog of the fused launch's list waves (100 MHz ticks): 2 s.
constexpr unsigned long long kFusedWatchdogTicks = 200000000ull;
struct FusedArgs {
    const uint8_t* arena;
    const uint64_t* off;
    const uint32_t* len;
    const uint32_t* order;
    uint8_t* req_out;
    const uint32_t* cidx;      // compacted list entries (no null requests)
    const uint32_t* cfirst;    // n_lists + 1
    uint8_t* list_out;
    const uint32_t* tadj_first;  // n_tiles + 1: counters each tile feeds
    const uint32_t* tadj;
    const uint32_t* cbase;       // n_groups + 1: first counter of each list group
    const uint32_t* expected;    // tiles feeding each counter
    unsigned long long* counters;
    unsigned long long* ctl;     // kCtlWords: tickets + retire count, one 128-B line each
    unsigned long long* err;     // the plan's sticky error word (host-mapped), set on a watchdog expiry
    unsigned long long watchdog; // readiness-wait limit, 100 MHz ticks (kFusedWatchdogTicks)
    // Optional timeline (s_memrealtime, 100 MHz), NULL = off: per tile [start, end,
    // info] at [3t, 3t+1, 3t+2] (info = HW_ID | XCC_ID << 32 | queue << 40 | slot << 44);
    // per readiness chunk the time its list wave passed the wait at
    // [3 n_tiles + ctr] and finished its blocks at [3 n_tiles + n_counters +
    // n_groups + ctr]; per list group its end at [3 n_tiles + n_counters + g].
    unsigned long long* trace;
    uint32_t n_counters;
    uint32_t q_first[kFusedMaxQueues + 1];
    uint32_t q_end[kFusedMaxQueues];  // queue q = [q_first[q], q_end[q]); split tiles lie in no queue
    uint32_t q_waves[kFusedMaxQueues];  // waves serving each queue first (static first tiles); tickets count beyond
    uint32_t tile_blocks;               // tile blocks in the grid (after the list blocks)
    uint32_t n_queues;  // = tile waves per SIMD (pace)
    uint32_t steal_own_prio;  // A/B (MIRSHA_FUSED_STEAL_PRIO=1): tiles taken from the last queue keep the taker's priority
    // Tile waves in LIST blocks (MIRSHA_FUSED_LIST_TILES): 0 = none (the pair
    // is alone on its CU), 1 = the waves on SIMDs 2-3, 2 = every wave but the
    // pair; with 1 and 2 the pair waves take last-queue tiles after their chains.
    uint32_t list_tiles;
    // Digests the list chains read: req_out (this run's tiles, readiness
    // waits) or, for overlapped cycles, the previous cycle's request digests
    // (epoch = 0: no waits).
    const uint8_t* list_digests;
    uint32_t arena_len, n_req, n_entries, n_lists;
    // Run number of the plan (1, 2, ...): counters are monotone over runs and a
    // chunk is ready at epoch x expected; 64-bit so it never wraps.
    unsigned long long epoch;
    uint32_t n_tiles, n_groups, list_waves;
    // Split tiles: n_split tiles the tile waves' slots cannot take (config 3's
    // 4,096 tiles on 4,024 slots), placed just before the last queue in
    // needed-at order (after it with one queue)
    // run as seg_per_tile sequential block-range segments, segment k of split
    // tile s hosted by the last queue's wave h = s * seg_per_tile + k of the
    // tile blocks (h = (block - list blocks) * 4 + SIMD), which runs it when
    // its own first tile reaches block k * seg_nominal_nb / seg_per_tile.  A
    // segment's midstate goes through seg_state ([s][8][64] words), its
    // completion through seg_flags[16 s] (monotone: run seg_epoch, segment k
    // done at seg_epoch * seg_per_tile + k + 1).  So no SIMD takes a fifth
    // tile: the overflow spreads as one short segment per SIMD.
    uint32_t n_split, split_first, seg_per_tile, seg_nominal_nb;  // split tiles [split_first, + n_split)
    // Tile priorities: 0 = their queue's (fused runs); 1 = the request
    // kernel's progress priorities; 2 = by progress rank among the SIMD's tile
    // waves (overlapped cycles: nothing waits on this run's tiles).
    uint32_t tile_prio_progress;
    // Test only (MIRSHA_AB=1 MIRSHA_TEST_PLACEMENT=remap): every wave reads
    // SIMD 0, so the in-kernel identity remap of a non-cyclic placement runs.
    uint32_t test_placement;
    // Tile waves switch to the latency round form (no issue yields) while they
    // are the only live wave of their SIMD (sha256_fused_paced_kernel; A/B:
    // MIRSHA_FUSED_LONE_FORM=0 keeps the throughput form throughout).
    uint32_t lone_form;
    // The last queue's waves of the tile blocks keep two blocks of loads in
    // flight (A/B: MIRSHA_FUSED_DEEP_LAST=0 keeps one).
    uint32_t deep_last;
    unsigned long long seg_epoch;
    const uint32_t* seg_nb;            // blocks of each split tile
    uint32_t* seg_state;
    unsigned long long* seg_flags;
};
// list_waves = number of list BLOCKS (first in the grid); one block per CU
// (kPacedLds of LDS: 16 waves' 4 KiB staging tiles, then a list block's pair
// ring; more than half the CU's LDS keeps any second block off the CU), `pace`
// tile waves per SIMD.
constexpr uint32_t kPacedRingOff = 64u * 1024u;
constexpr uint32_t kPacedLds = 97u * 1024u;
// Tile blocks: the last queue's second staging tiles (4 KiB per SIMD) after
// the parked midstates (2 KiB per SIMD at kPacedRingOff).
constexpr uint32_t kPacedDeepOff = kPacedRingOff + 8u * 1024u;
static_assert(kPacedDeepOff + 4u * 4096u <= kPacedLds, "paced LDS: deep staging tiles");
constexpr uint32_t kPacedMaxPace = 4;
hipError_t launch_fused_paced(const FusedArgs& a, uint32_t grid, uint32_t pace, hipStream_t s);
// Placement probe of the fused launch's block shape: *broken |= 1 when some
// block's 4P waves are not dealt P per SIMD (test != 0: report broken).
hipError_t launch_placement_probe(uint32_t grid, uint32_t pace, uint32_t* broken, uint32_t test, hipStream_t s);
// Streaming checkpoint chains (state: midstate h[8], pending digest words
// pend[8], digest count cnt per chain), see mirsha_kernels.hip.
hipError_t launch_chains_absorb(const uint8_t* digests, const uint32_t* pos, const uint32_t* act, const uint32_t* afirst,
                                uint32_t n_active, uint32_t* h, uint32_t* pend, uint64_t* cnt, hipStream_t s);
hipError_t launch_chains_sum(const uint32_t* which, uint32_t k, const uint32_t* h, const uint32_t* pend,
                             const uint64_t* cnt, uint8_t* out, hipStream_t s);
hipError_t launch_chains_reset(const uint32_t* which, uint32_t k, uint32_t* h, uint64_t* cnt, hipStream_t s);
hipError_t launch_gen_requests(uint64_t seed, uint64_t first, uint64_t count, uint32_t data_len,
                               uint8_t* arena, hipStream_t s);
hipError_t launch_mixed_lengths(uint64_t seed, uint64_t first, uint64_t count, uint32_t* len, hipStream_t s);
hipError_t launch_gen_mixed(uint64_t seed, uint64_t first, uint64_t count, const uint64_t* off, uint8_t* arena,
                            hipStream_t s);
// Clock probe: `blocks` 256-thread workgroups of `iters` register-only
// compressions each; stamps[3w] = shader cycles of wave w's loop, [3w+1],
// [3w+2] = its start and end in 100 MHz ticks (s_memrealtime).
constexpr uint32_t kProbeWavesPerSimd = 8;
hipError_t launch_clock_probe(uint32_t blocks, uint32_t iters, unsigned long long* stamps, uint32_t* sink,
                              hipStream_t s);

}  // namespace mirsha
