/*
 * cgo_path.c -- end-to-end cost of the Go binding's HashBatch
 *  at BASELINE config 2 size, from C (no Go toolchain here):
 * slices -> digests, with the binding's own packing included.
 *
 * Input: n client requests as the state machine hands them to the Processor
 * (state_machine.go:313-317: Data = [LE64(client), LE64(reqNo), payload]),
 * every slice its own heap allocation, as Go's [][]byte slices are.  Legs,
 * each the median of `reps` calls after one warm-up:
 *   serial    HashBatch as round 2 wrote it: one goroutine packs every slice
 *             into the mirsha_host_alloc arena, then mirsha_hash_batch;
 *   parallel  the same, the copy split over `threads` workers in contiguous
 *             request chunks (GOMAXPROCS goroutines), offsets computed first;
 *   lib       mirsha_hash_slices on C arrays of the slice pointers: the
 *             library's own 16-thread packing into its pinned ring,
 *             overlapped with the DMA (what a binding could use if the slices
 *             were C memory; Go's cgo rules forbid passing Go pointers stored
 *             in C memory, so the Go binding copies first).
 * Prints ONE JSON line; "sample" carries the first 4 digests of each leg for
 * tests/test_c_abi.py to compare with the oracle.  Exit 0 = ok.
 *
 * Usage: cgo_path [n] [data_len] [threads] [reps]
 */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mirsha.h"

static mirsha_ctx* ctx = NULL;

#define CHECK(call)                                                                                     \
    do {                                                                                                \
        int rc_ = (call);                                                                               \
        if (rc_ != MIRSHA_OK) {                                                                         \
            fprintf(stderr, "%s failed: %d: %s\n", #call, rc_, ctx ? mirsha_last_error(ctx) : "");     \
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

/* The binding's per-call buffers (Go: make([]uint64, n) etc.). */
typedef struct {
    const Request* reqs;
    uint8_t* arena;
    const uint64_t* off;
    uint32_t lo, hi;
} PackJob;

static void* pack_range(void* arg) {
    const PackJob* j = (const PackJob*)arg;
    for (uint32_t i = j->lo; i < j->hi; i++) {
        uint8_t* dst = j->arena + j->off[i];
        for (int s = 0; s < 3; s++) {
            memcpy(dst, j->reqs[i].ptr[s], j->reqs[i].len[s]);
            dst += j->reqs[i].len[s];
        }
    }
    return NULL;
}

/* HashBatch: offsets and lengths, the copy into the pinned arena (threads
 * workers), one mirsha_hash_batch.  Returns {pack ms, call ms}. */
static void hash_batch(const Request* reqs, uint32_t n, uint8_t* arena, uint64_t* off, uint32_t* lens, uint8_t* dig,
                       int threads, double* pack_ms, double* call_ms) {
    const double t0 = now_ms();
    uint64_t p = 0;
    for (uint32_t i = 0; i < n; i++) {
        off[i] = p;
        const uint64_t l = reqs[i].len[0] + reqs[i].len[1] + reqs[i].len[2];
        lens[i] = (uint32_t)l;
        p += l;
    }
    if (threads <= 1) {
        PackJob j = {reqs, arena, off, 0, n};
        pack_range(&j);
    } else {
        pthread_t th[64];
        PackJob jobs[64];
        const uint32_t step = (n + (uint32_t)threads - 1) / (uint32_t)threads;
        for (int t = 0; t < threads; t++) {
            const uint32_t lo = (uint32_t)t * step < n ? (uint32_t)t * step : n;
            const uint32_t hi = lo + step < n ? lo + step : n;
            jobs[t] = (PackJob){reqs, arena, off, lo, hi};
            if (pthread_create(&th[t], NULL, pack_range, &jobs[t]) != 0) exit(4);
        }
        for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
    }
    const double t1 = now_ms();
    CHECK(mirsha_hash_batch(ctx, arena, p, off, lens, n, dig));
    *pack_ms = t1 - t0;
    *call_ms = now_ms() - t1;
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

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)strtoul(argv[1], NULL, 10) : (1u << 20);
    const uint32_t data_len = argc > 2 ? (uint32_t)strtoul(argv[2], NULL, 10) : 256u;
    int threads = argc > 3 ? atoi(argv[3]) : 16;
    const int reps = argc > 4 ? atoi(argv[4]) : 5;
    if (threads < 1) threads = 1;
    if (threads > 64) threads = 64;
    if (n < 4 || reps < 1 || reps > 64) return 5;
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
        uint8_t* h0 = malloc(8);
        uint8_t* h1 = malloc(8);
        uint8_t* d = malloc(data_len ? data_len : 1);
        const uint64_t c = i % 16u, r = i / 16u;
        for (int b = 0; b < 8; b++) {
            h0[b] = (uint8_t)(c >> (8 * b));
            h1[b] = (uint8_t)(r >> (8 * b));
        }
        for (uint32_t j = 0; 8u * j < data_len; j++) {
            const uint64_t v = splitmix64(splitmix64(0x6D69726266740002ull ^ i) + j);
            for (uint32_t b = 0; b < 8 && 8u * j + b < data_len; b++) d[8u * j + b] = (uint8_t)(v >> (8 * b));
        }
        reqs[i] = (Request){{h0, h1, d}, {8, 8, data_len}};
        total += 16u + data_len;
    }
    void* ap = NULL;
    CHECK(mirsha_host_alloc(ctx, total + 1, &ap));
    uint8_t* arena = ap;
    uint64_t* off = malloc(8ull * n);
    uint32_t* lens = malloc(4ull * n);
    uint8_t* dig_s = malloc(32ull * n);
    uint8_t* dig_p = malloc(32ull * n);
    uint8_t* dig_l = malloc(32ull * n);

    double pk[64], cl[64], tot[64], pk2[64], cl2[64], tot2[64], lib[64];
    for (int r = -1; r < reps; r++) { /* r = -1: warm-up */
        double a, b;
        hash_batch(reqs, n, arena, off, lens, dig_s, 1, &a, &b);
        if (r >= 0) pk[r] = a, cl[r] = b, tot[r] = a + b;
        hash_batch(reqs, n, arena, off, lens, dig_p, threads, &a, &b);
        if (r >= 0) pk2[r] = a, cl2[r] = b, tot2[r] = a + b;
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
    for (int r = -1; r < reps; r++) {
        const double t0 = now_ms();
        CHECK(mirsha_hash_slices(ctx, sp, sl, sf, n, dig_l));
        if (r >= 0) lib[r] = now_ms() - t0;
    }
    if (memcmp(dig_s, dig_p, 32ull * n) || memcmp(dig_s, dig_l, 32ull * n)) {
        fprintf(stderr, "legs disagree\n");
        return 1;
    }
    const double m_tot = median(tot, reps), m_tot2 = median(tot2, reps), m_lib = median(lib, reps);
    char sample[4 * 65 + 8];
    hex4(dig_s, sample);
    printf("{\"requests\": %u, \"request_bytes\": %u, \"bytes\": %llu, \"threads\": %d, \"reps\": %d, "
           "\"serial\": {\"pack_ms\": %.3f, \"call_ms\": %.3f, \"ms\": %.3f, \"digests_per_s\": %.1f}, "
           "\"parallel\": {\"pack_ms\": %.3f, \"call_ms\": %.3f, \"ms\": %.3f, \"digests_per_s\": %.1f}, "
           "\"lib\": {\"ms\": %.3f, \"digests_per_s\": %.1f}, \"sample\": \"%s\"}\n",
           n, 16u + data_len, (unsigned long long)total, threads, reps, median(pk, reps), median(cl, reps), m_tot,
           n / (m_tot * 1e-3), median(pk2, reps), median(cl2, reps), m_tot2, n / (m_tot2 * 1e-3), m_lib,
           n / (m_lib * 1e-3), sample);
    mirsha_host_free(arena);
    mirsha_ctx_destroy(ctx);
    return 0;
}
