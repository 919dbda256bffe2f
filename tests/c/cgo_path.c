/*
 * cgo_path.c -- end-to-end cost of the Go binding's HashBatch
 *  at BASELINE config 2 size, from C (no Go toolchain here):
 * slices -> digests, with the binding's own packing included.
 *
 * Input: n client requests as the state machine hands them to the Processor
 * (state_machine.go:313-317: Data = [LE64(client), LE64(reqNo), payload]),
 * every slice its own heap allocation, as Go's [][]byte slices are.  A
 * persistent pool of `threads` workers stands in for GOMAXPROCS goroutines
 * (a goroutine start costs ~1 us; a pthread_create per chunk would not).
 * Legs, each the median of `reps` calls after three warm-up calls (a fresh
 * process's first few calls can block ~9 ms in an SDMA copy enqueue of the
 * HIP runtime, profiles/r05w; a consensus node calls HashBatch every cycle):
 *   serial    round 2's HashBatch: one goroutine packs every slice into the
 *             mirsha_host_alloc arena, then one mirsha_hash_batch;
 *   parallel  INTEGRATION.md's HashBatch: offsets first, then the cycle in
 *             chunks of ~chunk_mib MiB: the workers pack chunk k into the
 *             pinned arena (and copy the digests of chunks already back into
 *             the Go-owned result buffer), then mirsha_submit_batch queues its
 *             DMA + kernel + D2H (into a pinned digest buffer) and returns, so
 *             chunk k's transfer overlaps chunk k+1's packing; mirsha_wait on
 *             the last ticket, the remaining digests copied by the workers;
 *   onecall   round 4's HashBatch: the workers pack the whole cycle, then one
 *             mirsha_hash_batch (no overlap of packing and DMA);
 *   lib       mirsha_hash_slices on C arrays of the slice pointers: the
 *             library's own packing into its pinned ring, overlapped with the
 *             DMA (what a binding could use if the slices were C memory; Go's
 *             cgo rules forbid passing Go pointers stored in C memory);
 *   multi     GPUHasherMulti.HashBatch: `parallel` over every visible device
 *             (device 0 twice on a one-GPU box) with mirsha_submit_arena_multi.
 * Prints ONE JSON line; "sample" carries the first 4 digests for
 * tests/test_c_abi.py to compare with the oracle; every leg's digests are
 * compared with the serial leg's.  Exit 0 = ok.
 *
 * Usage: cgo_path [n] [data_len] [threads] [reps] [chunk_mib] [pack_stores: plain|nt] [big_every big_len]
 * (big_every > 0: every big_every-th request carries big_len payload bytes;
 * "sample_big" then holds the first such request's digest)
 */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <emmintrin.h>
#include <time.h>

#include "mirsha.h"

static mirsha_ctx* ctx = NULL;
static mirsha_multi* multi = NULL;

#define CHECK(call)                                                                                     \
    do {                                                                                                \
        int rc_ = (call);                                                                               \
        if (rc_ != MIRSHA_OK) {                                                                         \
            fprintf(stderr, "%s failed: %d: %s\n", #call, rc_,                                         \
                    multi ? mirsha_multi_last_error(multi) : ctx ? mirsha_last_error(ctx) : "");        \
            exit(2);                                                                                    \
        }                                                                                               \
    } while (0)

static double now_ms(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec * 1e-6;
}

static uint64_t splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* One HashRequest: its Data slices. */
typedef struct {
    const uint8_t* ptr[3];
    uint64_t len[3];
} Request;

/* ---- worker pool (GOMAXPROCS goroutines + sync.WaitGroup) ---- */
typedef void (*PartFn)(void* arg, int part, int parts);
typedef struct Pool Pool;
typedef struct {
    Pool* pool;
    int idx;
} PoolSeat;
struct Pool {
    pthread_t th[64];
    PoolSeat seat[64];
    int n;
    pthread_mutex_t mu;
    pthread_cond_t go, done;
    uint64_t gen;
    int pending, quit;
    PartFn fn;
    void* arg;
};

static void* pool_worker(void* a) {
    PoolSeat* s = (PoolSeat*)a;
    Pool* p = s->pool;
    uint64_t seen = 0;
    for (;;) {
        pthread_mutex_lock(&p->mu);
        while (p->gen == seen && !p->quit) pthread_cond_wait(&p->go, &p->mu);
        if (p->quit) {
            pthread_mutex_unlock(&p->mu);
            return NULL;
        }
        seen = p->gen;
        PartFn fn = p->fn;
        void* arg = p->arg;
        pthread_mutex_unlock(&p->mu);
        fn(arg, s->idx, p->n);
        pthread_mutex_lock(&p->mu);
        if (--p->pending == 0) pthread_cond_signal(&p->done);
        pthread_mutex_unlock(&p->mu);
    }
}

static void pool_init(Pool* p, int n) {
    memset(p, 0, sizeof(*p));
    p->n = n;
    pthread_mutex_init(&p->mu, NULL);
    pthread_cond_init(&p->go, NULL);
    pthread_cond_init(&p->done, NULL);
    for (int i = 0; i < n; i++) {
        p->seat[i] = (PoolSeat){p, i};
        if (pthread_create(&p->th[i], NULL, pool_worker, &p->seat[i]) != 0) exit(4);
    }
}

/* fn(arg, part, n) on every worker (go func() ... for each part); pool_wait
 * is the WaitGroup.Wait. */
static void pool_start(Pool* p, PartFn fn, void* arg) {
    pthread_mutex_lock(&p->mu);
    p->fn = fn;
    p->arg = arg;
    p->pending = p->n;
    p->gen++;
    pthread_cond_broadcast(&p->go);
    pthread_mutex_unlock(&p->mu);
}

static void pool_wait(Pool* p) {
    pthread_mutex_lock(&p->mu);
    while (p->pending) pthread_cond_wait(&p->done, &p->mu);
    pthread_mutex_unlock(&p->mu);
}

static void pool_run(Pool* p, PartFn fn, void* arg) {
    pool_start(p, fn, arg);
    pool_wait(p);
}

static void pool_stop(Pool* p) {
    pthread_mutex_lock(&p->mu);
    p->quit = 1;
    pthread_cond_broadcast(&p->go);
    pthread_mutex_unlock(&p->mu);
    for (int i = 0; i < p->n; i++) pthread_join(p->th[i], NULL);
}

static void part_range(uint32_t lo, uint32_t hi, int part, int parts, uint32_t* a, uint32_t* b) {
    const uint32_t n = hi - lo, step = (n + (uint32_t)parts - 1) / (uint32_t)parts;
    const uint32_t x = (uint32_t)part * step;
    *a = lo + (x < n ? x : n);
    *b = lo + (x + step < n ? x + step : n);
}

/* One pool job: pack requests [lo, hi) into the arena at off[i] (h.Write of
 * every Data slice, processor.go:135-137), and copy digest rows [dlo, dhi)
 * from the pinned digest buffer into the caller's. */
typedef struct {
    const Request* reqs;
    uint8_t* arena;
    uint64_t* off;
    uint32_t lo, hi;
    const uint8_t* dsrc;
    uint8_t* ddst;
    uint32_t dlo, dhi;
    /* chunked form: the chunk is blocks [blo, bhi) of br requests each; the
     * workers write off[i] of their blocks from the blocks' byte prefix bpre
     * (the offsets pass folded into the packing) */
    const uint64_t* bpre;
    const uint32_t* lens;
    uint32_t n, br, blo, bhi;
} ChunkJob;

/* pack_stores "nt": each worker gathers its requests in a 16 KiB window and
 * streams the window into the page-locked arena with non-temporal stores (a
 * Go binding would call a small assembly helper per window);
 * DMA of lines still dirty in CPU caches runs ~9% below the link
 * (profiles/r05o). */
static int g_nt = 0;
static void nt_copy(uint8_t* dst, const uint8_t* src, uint64_t n) {
    uint64_t h = (16 - ((uintptr_t)dst & 15)) & 15;
    if (h > n) h = n;
    memcpy(dst, src, h);
    dst += h, src += h, n -= h;
    for (; n >= 64; n -= 64, dst += 64, src += 64) {
        const __m128i x0 = _mm_loadu_si128((const __m128i*)src), x1 = _mm_loadu_si128((const __m128i*)(src + 16)),
                      x2 = _mm_loadu_si128((const __m128i*)(src + 32)), x3 = _mm_loadu_si128((const __m128i*)(src + 48));
        _mm_stream_si128((__m128i*)dst, x0);
        _mm_stream_si128((__m128i*)(dst + 16), x1);
        _mm_stream_si128((__m128i*)(dst + 32), x2);
        _mm_stream_si128((__m128i*)(dst + 48), x3);
    }
    for (; n >= 16; n -= 16, dst += 16, src += 16) _mm_stream_si128((__m128i*)dst, _mm_loadu_si128((const __m128i*)src));
    memcpy(dst, src, n);
}

static void chunk_part_nt(const ChunkJob* j, uint32_t a, uint32_t b) {
    enum { WIN = 16384 };
    _Alignas(64) uint8_t win[WIN];
    uint64_t fill = 0;
    uint8_t* at = a < b ? j->arena + j->off[a] : NULL; /* requests [a, b) are contiguous in the arena */
    for (uint32_t i = a; i < b; i++)
        for (int s = 0; s < 3; s++) {
            const uint64_t l = j->reqs[i].len[s];
            if (fill + l > WIN) {
                nt_copy(at, win, fill);
                at += fill;
                fill = 0;
            }
            if (l >= WIN) {
                nt_copy(at, j->reqs[i].ptr[s], l);
                at += l;
                continue;
            }
            memcpy(win + fill, j->reqs[i].ptr[s], l);
            fill += l;
        }
    if (fill) nt_copy(at, win, fill);
    _mm_sfence();
}

static void chunk_part(void* arg, int part, int parts) {
    const ChunkJob* j = (const ChunkJob*)arg;
    uint32_t a, b;
    if (j->bpre) {
        uint32_t ba, bb;
        part_range(j->blo, j->bhi, part, parts, &ba, &bb);
        a = ba * j->br < j->n ? ba * j->br : j->n;
        b = bb * j->br < j->n ? bb * j->br : j->n;
        if (ba >= bb) a = b = 0;
        uint64_t p = j->bpre[ba];
        for (uint32_t i = a; i < b; i++) {
            j->off[i] = p;
            p += j->lens[i];
        }
    } else {
        part_range(j->lo, j->hi, part, parts, &a, &b);
    }
    if (g_nt) {
        chunk_part_nt(j, a, b);
        a = b;
    }
    for (uint32_t i = a; i < b; i++) {
        uint8_t* dst = j->arena + j->off[i];
        for (int s = 0; s < 3; s++) {
            memcpy(dst, j->reqs[i].ptr[s], j->reqs[i].len[s]);
            dst += j->reqs[i].len[s];
        }
    }
    part_range(j->dlo, j->dhi, part, parts, &a, &b);
    if (b > a) memcpy(j->ddst + 32ull * a, j->dsrc + 32ull * a, 32ull * (b - a));
}

/* offsets and lengths of the cycle (Go: off[i], lens[i], serial); returns the total */
static uint64_t offsets(const Request* reqs, uint32_t n, uint64_t* off, uint32_t* lens) {
    uint64_t p = 0;
    for (uint32_t i = 0; i < n; i++) {
        off[i] = p;
        const uint64_t l = reqs[i].len[0] + reqs[i].len[1] + reqs[i].len[2];
        lens[i] = (uint32_t)l;
        p += l;
    }
    return p;
}

/* The chunked form's one pass before packing: lens[i] and the byte sum of
 * every block of br requests (at most MAX_BLOCKS blocks), by the pool; the
 * caller turns the sums into each block's starting offset.  The offsets
 * themselves are written by the packing workers (chunk_part). */
#define MAX_BLOCKS 4096
typedef struct {
    const Request* reqs;
    uint32_t n, br, nb;
    uint32_t* lens;
    uint64_t bpre[MAX_BLOCKS + 1];
} LenJob;

static void len_part(void* arg, int part, int parts) {
    LenJob* j = (LenJob*)arg;
    uint32_t ba, bb;
    part_range(0, j->nb, part, parts, &ba, &bb);
    for (uint32_t blk = ba; blk < bb; blk++) {
        const uint32_t a = blk * j->br, b = a + j->br < j->n ? a + j->br : j->n;
        uint64_t s = 0;
        for (uint32_t i = a; i < b; i++) {
            const uint64_t l = j->reqs[i].len[0] + j->reqs[i].len[1] + j->reqs[i].len[2];
            j->lens[i] = (uint32_t)l;
            s += l;
        }
        j->bpre[blk + 1] = s;
    }
}

static uint64_t lengths_parallel(const Request* reqs, uint32_t n, uint32_t* lens, Pool* pool, LenJob* j) {
    j->reqs = reqs;
    j->n = n;
    j->lens = lens;
    j->bpre[0] = 0;
    if (n == 0) { /* no blocks (and no division by a zero block size) */
        j->br = 1;
        j->nb = 0;
        return 0;
    }
    j->br = (n + MAX_BLOCKS - 1) / MAX_BLOCKS;
    j->nb = (n + j->br - 1) / j->br;
    pool_run(pool, len_part, j);
    for (uint32_t k = 0; k < j->nb; k++) j->bpre[k + 1] += j->bpre[k];
    return j->bpre[j->nb];
}

/* Round 2 / round 4 HashBatch: pack everything (1 or `pool` workers), one
 * mirsha_hash_batch.  {pack ms, call ms}. */
static void hash_batch_onecall(const Request* reqs, uint32_t n, uint8_t* arena, uint64_t* off, uint32_t* lens,
                               uint8_t* dig, Pool* pool, double* pack_ms, double* call_ms) {
    const double t0 = now_ms();
    const uint64_t total = offsets(reqs, n, off, lens);
    ChunkJob j = {reqs, arena, off, 0, n, NULL, NULL, 0, 0, NULL, NULL, 0, 0, 0, 0};
    if (pool)
        pool_run(pool, chunk_part, &j);
    else
        chunk_part(&j, 0, 1);
    const double t1 = now_ms();
    CHECK(mirsha_hash_batch(ctx, arena, total, off, lens, n, dig));
    *pack_ms = t1 - t0;
    *call_ms = now_ms() - t1;
}

/* INTEGRATION.md's HashBatch (single device, or a mirsha_multi when m != NULL):
 * offsets by the workers, then chunk k+1 packed by the workers WHILE the
 * caller submits chunk k (mirsha_submit_batch returns once its DMA, kernel
 * and D2H are queued), so neither the submission's host work nor the DMA
 * waits for packing.  {pack ms = until the last submission returned, call ms
 * = wait + the last digests}.  *chunks_out = submissions. */
#define MAX_CHUNKS 65536
/* host phases of the last chunked call (ms): offsets, waiting for the packing
 * workers, submits (overlapping the packing), final wait, final copy */
static double ph_off, ph_pack, ph_submit, ph_wait, ph_copy;
/* the longest single submit and the longest wait for the workers in one call:
 * a host that deschedules a worker shows up in the latter */
static double ph_max_submit, ph_max_pool;
/* the library's phases of the slowest submit seen (> 3 ms): where it blocked */
static double slow_submit[MIRSHA_PROF_PHASES];
static double slow_submit_ms;
static void submit_chunk(mirsha_multi* m, const uint8_t* arena, uint64_t total, const uint64_t* off,
                         const uint32_t* lens, uint32_t lo, uint32_t hi, uint8_t* dig_pinned, uint64_t* ticket) {
    if (m)
        CHECK(mirsha_submit_arena_multi(m, arena, total, off + lo, lens + lo, hi - lo, dig_pinned + 32ull * lo, ticket));
    else
        CHECK(mirsha_submit_batch(ctx, arena, total, off + lo, lens + lo, hi - lo, dig_pinned + 32ull * lo, ticket));
}

static void hash_batch_chunked(const Request* reqs, uint32_t n, uint8_t* arena, uint64_t* off, uint32_t* lens,
                               uint8_t* dig_pinned, uint8_t* dig, Pool* pool, uint64_t chunk_bytes, mirsha_multi* m,
                               double* pack_ms, double* call_ms, int* chunks_out) {
    static uint64_t ticket[MAX_CHUNKS], cat[MAX_CHUNKS];
    static uint32_t cfirst[MAX_CHUNKS + 1], cb0[MAX_CHUNKS], cb1[MAX_CHUNKS];
    static LenJob lj;
    const double t0 = now_ms();
    const uint64_t total = lengths_parallel(reqs, n, lens, pool, &lj);
    ph_off = now_ms() - t0;
    ph_pack = ph_submit = ph_max_submit = ph_max_pool = 0.0;
    /* Chunk boundaries (INTEGRATION.md planChunks): whole blocks [b0, b1)
     * until the chunk's bytes reach the budget -- a quarter, a half, then whole
     * budgets: the link starts early and stays busy while the workers pack the
     * next, larger chunk.  A block holding more than a whole budget (large
     * messages) is cut at request boundaries instead -- chunk k is then
     * requests [cfirst[k], cfirst[k+1]) of one block, starting at byte cat[k],
     * cb0[k] == cb1[k] -- so no submission outgrows one device arena
     * (MIRSHA_MAX_DEVICE_ARENA_BYTES). */
    int nk = 0;
    for (uint32_t b0 = 0; b0 < lj.nb;) {
        const uint64_t budget = nk == 0 ? chunk_bytes / 4 : nk == 1 ? chunk_bytes / 2 : chunk_bytes;
        const uint32_t r0 = b0 * lj.br, r1 = r0 + lj.br < n ? r0 + lj.br : n;
        if (lj.bpre[b0 + 1] - lj.bpre[b0] > chunk_bytes) {
            uint64_t at = lj.bpre[b0];
            for (uint32_t lo = r0; lo < r1;) {
                uint32_t hi = lo + 1;
                uint64_t s = lens[lo];
                while (hi < r1 && s + lens[hi] <= chunk_bytes) s += lens[hi++];
                if (nk == MAX_CHUNKS) exit(6);
                cfirst[nk] = lo;
                cb0[nk] = cb1[nk] = b0;
                cat[nk++] = at;
                at += s;
                lo = hi;
            }
            b0++;
            continue;
        }
        uint32_t b1 = b0 + 1;
        while (b1 < lj.nb && lj.bpre[b1] - lj.bpre[b0] < budget && lj.bpre[b1 + 1] - lj.bpre[b1] <= chunk_bytes) b1++;
        if (nk == MAX_CHUNKS) exit(6);
        cfirst[nk] = r0;
        cb0[nk] = b0;
        cb1[nk] = b1;
        cat[nk++] = lj.bpre[b0];
        b0 = b1;
    }
    cfirst[nk] = n;
    int copied = 0; /* chunks whose digests are in dig */
    ChunkJob job;
    for (int k = 0; k <= nk; k++) {
        /* workers: pack chunk k (if any) + the digests of chunks already back */
        const double tp = now_ms();
        const int part_block = k < nk && cb0[k] == cb1[k];
        job = (ChunkJob){reqs, arena, off, k < nk ? cfirst[k] : 0, k < nk ? cfirst[k + 1] : 0, dig_pinned, dig, 0, 0,
                         part_block ? NULL : lj.bpre, lens, n, lj.br, k < nk ? cb0[k] : 0, k < nk ? cb1[k] : 0};
        if (part_block) { /* a part of one oversized block: its few offsets here, the workers split its requests */
            uint64_t p = cat[k];
            for (uint32_t i = cfirst[k]; i < cfirst[k + 1]; i++) {
                off[i] = p;
                p += lens[i];
            }
        }
        int upto = copied;
        while (upto < k - 1) {
            int done = 0;
            if (m)
                CHECK(mirsha_poll_multi(m, ticket[upto], &done));
            else
                CHECK(mirsha_poll(ctx, ticket[upto], &done));
            if (!done) break;
            upto++;
        }
        if (upto > copied) {
            job.dlo = cfirst[copied];
            job.dhi = cfirst[upto];
            copied = upto;
        }
        if (k < nk || job.dhi > job.dlo) pool_start(pool, chunk_part, &job);
        /* caller: submit chunk k-1, packed in the previous round */
        const double ts = now_ms();
        if (k > 0) submit_chunk(m, arena, total, off, lens, cfirst[k - 1], cfirst[k], dig_pinned, &ticket[k - 1]);
        const double tw = now_ms();
        ph_submit += tw - ts;
        if (tw - ts > ph_max_submit) ph_max_submit = tw - ts;
        if (!m && k > 0 && tw - ts > 3.0 && tw - ts > slow_submit_ms) {
            slow_submit_ms = tw - ts;
            mirsha_ctx_host_profile(ctx, slow_submit, MIRSHA_PROF_PHASES);
        }
        if (k < nk || job.dhi > job.dlo) pool_wait(pool);
        const double te = now_ms();
        ph_pack += (ts - tp) + (te - tw);
        if (te - tw > ph_max_pool) ph_max_pool = te - tw;
    }
    const double t1 = now_ms();
    if (nk) {
        if (m)
            CHECK(mirsha_wait_multi(m, ticket[nk - 1]));
        else
            CHECK(mirsha_wait(ctx, ticket[nk - 1]));
        const double tw = now_ms();
        ph_wait = tw - t1;
        job = (ChunkJob){reqs, arena, off, 0, 0, dig_pinned, dig, cfirst[copied], n, NULL, NULL, 0, 0, 0, 0};
        pool_run(pool, chunk_part, &job);
        ph_copy = now_ms() - tw;
    }
    *pack_ms = t1 - t0;
    *call_ms = now_ms() - t1;
    *chunks_out = nk;
}

static int cmp_d(const void* a, const void* b) {
    const double x = *(const double*)a, y = *(const double*)b;
    return x < y ? -1 : x > y;
}

static double median(double* v, int k) {
    qsort(v, (size_t)k, sizeof(double), cmp_d);
    return v[k / 2];
}

static void hex4(const uint8_t* dig, char* out) {
    /* first 4 digests, comma-separated hex */
    char* o = out;
    for (int i = 0; i < 4; i++) {
        if (i) *o++ = ',';
        for (int k = 0; k < 32; k++) o += sprintf(o, "%02x", dig[32 * i + k]);
    }
}

typedef struct {
    double pack[64], call[64], tot[64];
} Leg;

static void leg_put(Leg* l, int r, double a, double b) {
    if (r < 0) return;
    l->pack[r] = a;
    l->call[r] = b;
    l->tot[r] = a + b;
}

static void leg_print(const char* name, Leg* l, int reps, uint32_t n, const char* extra) {
    const double t = median(l->tot, reps);
    printf("\"%s\": {\"pack_ms\": %.3f, \"call_ms\": %.3f, \"ms\": %.3f, \"digests_per_s\": %.1f%s}", name,
           median(l->pack, reps), median(l->call, reps), t, n / (t * 1e-3), extra);
}

enum { kWarm = 3 }; /* untimed calls per leg before the timed ones */

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)strtoul(argv[1], NULL, 10) : (1u << 20);
    const uint32_t data_len = argc > 2 ? (uint32_t)strtoul(argv[2], NULL, 10) : 256u;
    int threads = argc > 3 ? atoi(argv[3]) : 16;
    const int reps = argc > 4 ? atoi(argv[4]) : 5;
    const double chunk_mib = argc > 5 ? atof(argv[5]) : 16.0;
    g_nt = argc > 6 && strcmp(argv[6], "nt") == 0;
    /* optional large messages: request i with i % big_every == big_every - 1
     * carries big_len payload bytes (its block then outgrows a chunk budget) */
    const uint32_t big_every = argc > 7 ? (uint32_t)strtoul(argv[7], NULL, 10) : 0u;
    const uint32_t big_len = argc > 8 ? (uint32_t)strtoul(argv[8], NULL, 10) : 0u;
    if (threads < 1) threads = 1;
    if (threads > 64) threads = 64;
    if (n < 4 || reps < 1 || reps > 64 || chunk_mib <= 0) return 5;
    const uint64_t chunk_bytes = (uint64_t)(chunk_mib * 1048576.0);
    int ndev = 0;
    CHECK(mirsha_device_count(&ndev));
    if (ndev < 1) {
        fprintf(stderr, "no device\n");
        return 3;
    }
    CHECK(mirsha_ctx_create(0, &ctx));

    /* The requests: request i = client i % 16, reqNo i / 16, a data_len-byte
     * payload (config 2's generator, oracle_gen_requests), three heap slices. */
    Request* reqs = malloc(sizeof(Request) * n);
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t dl = big_every && i % big_every == big_every - 1 ? big_len : data_len;
        uint8_t* h0 = malloc(8);
        uint8_t* h1 = malloc(8);
        uint8_t* d = malloc(dl ? dl : 1);
        const uint64_t c = i % 16u, r = i / 16u;
        for (int b = 0; b < 8; b++) {
            h0[b] = (uint8_t)(c >> (8 * b));
            h1[b] = (uint8_t)(r >> (8 * b));
        }
        for (uint32_t j = 0; 8u * j < dl; j++) {
            const uint64_t v = splitmix64(splitmix64(0x6D69726266740002ull ^ i) + j);
            for (uint32_t b = 0; b < 8 && 8u * j + b < dl; b++) d[8u * j + b] = (uint8_t)(v >> (8 * b));
        }
        reqs[i] = (Request){{h0, h1, d}, {8, 8, dl}};
        total += 16u + dl;
    }
    void* ap = NULL;
    void* dp = NULL;
    CHECK(mirsha_host_alloc(ctx, total + 1, &ap));
    CHECK(mirsha_host_alloc(ctx, 32ull * n, &dp)); /* the binding's pinned digest buffer */
    uint8_t* arena = ap;
    uint8_t* dig_pinned = dp;
    uint64_t* off = malloc(8ull * n);
    uint32_t* lens = malloc(4ull * n);
    uint8_t* dig_s = malloc(32ull * n);
    uint8_t* dig_p = malloc(32ull * n);
    uint8_t* dig_o = malloc(32ull * n);
    uint8_t* dig_l = malloc(32ull * n);
    uint8_t* dig_m = malloc(32ull * n);
    Pool pool;
    pool_init(&pool, threads);

    Leg ser, par, one, lib, mul;
    char phases[512] = "";
    char calls[64 * 96 + 32] = ", \"calls\": [";
    int chunks = 0, mchunks = 0;
    for (int r = -kWarm; r < reps; r++) { /* r < 0: warm-up */
        double a, b;
        hash_batch_onecall(reqs, n, arena, off, lens, dig_s, NULL, &a, &b);
        leg_put(&ser, r, a, b);
        hash_batch_chunked(reqs, n, arena, off, lens, dig_pinned, dig_p, &pool, chunk_bytes, NULL, &a, &b, &chunks);
        leg_put(&par, r, a, b);
        if (r >= 0) {
            char one_call[96];
            snprintf(one_call, sizeof one_call, "%s[%.2f, %.2f, %.2f, %.2f]", r ? ", " : "", a + b, ph_max_pool,
                     ph_max_submit, ph_wait);
            strcat(calls, one_call);
        }
        if (r == reps - 1) {
            /* the library's phases of the last chunk's submission (validate, plan, queue) */
            double lp[MIRSHA_PROF_PHASES] = {0};
            mirsha_ctx_host_profile(ctx, lp, MIRSHA_PROF_PHASES);
            snprintf(phases, sizeof phases,
                     ", \"last_call_phases_ms\": {\"offsets\": %.3f, \"pack\": %.3f, \"submit\": %.3f, "
                     "\"wait\": %.3f, \"copy\": %.3f}, \"last_submit_ms\": {\"validate\": %.3f, "
                     "\"plan\": %.3f, \"queue\": %.3f, \"device\": %.3f}",
                     ph_off, ph_pack, ph_submit, ph_wait, ph_copy, lp[MIRSHA_PROF_VALIDATE], lp[MIRSHA_PROF_PLAN],
                     lp[MIRSHA_PROF_PACK], lp[MIRSHA_PROF_DEVICE]);
        }
        hash_batch_onecall(reqs, n, arena, off, lens, dig_o, &pool, &a, &b);
        leg_put(&one, r, a, b);
    }
    /* lib: slice pointer arrays in C memory, the library packs */
    const uint8_t** sp = malloc(sizeof(uint8_t*) * 3ull * n);
    uint64_t* sl = malloc(8ull * 3ull * n);
    uint32_t* sf = malloc(4ull * (n + 1));
    for (uint32_t i = 0; i < n; i++) {
        for (int s = 0; s < 3; s++) {
            sp[3ull * i + s] = reqs[i].ptr[s];
            sl[3ull * i + s] = reqs[i].len[s];
        }
        sf[i] = 3u * i;
    }
    sf[n] = 3u * n;
    for (int r = -kWarm; r < reps; r++) {
        const double t0 = now_ms();
        CHECK(mirsha_hash_slices(ctx, sp, sl, sf, n, dig_l));
        leg_put(&lib, r, 0.0, now_ms() - t0);
    }
    char lphases[256];
    {
        double lp[MIRSHA_PROF_PHASES] = {0};
        mirsha_ctx_host_profile(ctx, lp, MIRSHA_PROF_PHASES);
        snprintf(lphases, sizeof lphases,
                 ", \"last_call_phases_ms\": {\"validate\": %.3f, \"plan\": %.3f, \"pack\": %.3f, \"device\": %.3f, "
                 "\"scatter\": %.3f, \"total\": %.3f, \"chunks\": %.0f}",
                 lp[MIRSHA_PROF_VALIDATE], lp[MIRSHA_PROF_PLAN], lp[MIRSHA_PROF_PACK], lp[MIRSHA_PROF_DEVICE],
                 lp[MIRSHA_PROF_SCATTER], lp[MIRSHA_PROF_TOTAL], lp[MIRSHA_PROF_CHUNKS]);
    }
    /* multi: GPUHasherMulti over every device (device 0 twice on one GPU) */
    int devs[16], nd = ndev > 1 ? (ndev < 16 ? ndev : 16) : 2;
    for (int k = 0; k < nd; k++) devs[k] = ndev > 1 ? k : 0;
    mirsha_host_free(ap);
    mirsha_host_free(dp);
    ap = dp = NULL;
    CHECK(mirsha_multi_create(devs, nd, &multi));
    CHECK(mirsha_multi_host_alloc(multi, total + 1, &ap));
    CHECK(mirsha_multi_host_alloc(multi, 32ull * n, &dp));
    for (int r = -kWarm; r < reps; r++) {
        double a, b;
        hash_batch_chunked(reqs, n, ap, off, lens, dp, dig_m, &pool, chunk_bytes, multi, &a, &b, &mchunks);
        leg_put(&mul, r, a, b);
    }
    if (memcmp(dig_s, dig_p, 32ull * n) || memcmp(dig_s, dig_o, 32ull * n) || memcmp(dig_s, dig_l, 32ull * n) ||
        memcmp(dig_s, dig_m, 32ull * n)) {
        fprintf(stderr, "legs disagree\n");
        return 1;
    }
    char sample[4 * 65 + 8], extra[8192], mextra[96];
    hex4(dig_s, sample);
    strcat(calls, "], \"calls_note\": \"per call: ms, longest wait for the workers, longest submit, final wait\"");
    if (slow_submit_ms > 0) {
        char sl[256];
        snprintf(sl, sizeof sl,
                 ", \"slowest_submit_ms\": {\"total\": %.3f, \"validate\": %.3f, \"plan\": %.3f, \"queue\": %.3f}",
                 slow_submit_ms, slow_submit[MIRSHA_PROF_VALIDATE], slow_submit[MIRSHA_PROF_PLAN],
                 slow_submit[MIRSHA_PROF_PACK]);
        strcat(calls, sl);
    }
    snprintf(extra, sizeof extra, ", \"chunks\": %d, \"chunk_mib\": %.2f%s%s", chunks, chunk_mib, phases, calls);
    snprintf(mextra, sizeof mextra, ", \"chunks\": %d, \"devices\": %d", mchunks, nd);
    printf("{\"requests\": %u, \"request_bytes\": %u, \"bytes\": %llu, \"threads\": %d, \"reps\": %d, "
           "\"pack_stores\": \"%s\", ",
           n, 16u + data_len, (unsigned long long)total, threads, reps, g_nt ? "nt" : "plain");
    leg_print("serial", &ser, reps, n, "");
    printf(", ");
    leg_print("parallel", &par, reps, n, extra);
    printf(", ");
    leg_print("onecall", &one, reps, n, "");
    printf(", ");
    leg_print("lib", &lib, reps, n, lphases);
    printf(", ");
    leg_print("multi", &mul, reps, n, mextra);
    printf(", \"sample\": \"%s\"", sample);
    if (big_every && big_every <= n) { /* the first large request's digest */
        char bs[65];
        for (int k = 0; k < 32; k++) sprintf(bs + 2 * k, "%02x", dig_s[32ull * (big_every - 1) + k]);
        printf(", \"sample_big\": {\"index\": %u, \"payload_bytes\": %u, \"sha256\": \"%s\"}", big_every - 1, big_len, bs);
    }
    printf("}\n");
    pool_stop(&pool);
    mirsha_host_free(ap);
    mirsha_host_free(dp);
    mirsha_multi_destroy(multi);
    multi = NULL;
    mirsha_ctx_destroy(ctx);
    return 0;
}
