/*
 * cgo_sequence.c -- the C-ABI call sequence the Go binding in INTEGRATION.md
 * makes, compiled by gcc against include/mirsha.h and linked to libmirsha.so
 * (no Python, no torch in the process): what a cgo caller sees.
 *
 *   mirsha_ctx_create
 *   mirsha_host_alloc (once; the GPUHasher's pinned arena, grown on demand)
 *   per Ready() cycle: pack HashRequest.Data into the arena, mirsha_hash_batch
 *     (round 4's GPUHasher.HashBatch; processor.go:129-143)
 *   the chunked HashBatch: chunk k packed into the arena, mirsha_submit_batch
 *     with a pinned digest buffer (mirsha_host_alloc), mirsha_poll on earlier
 *     chunks, mirsha_wait on the last
 *   mirsha_submit_slices + mirsha_wait with the slice arrays in C memory
 *     (GPUHasher.SubmitBatch / PendingBatch.Wait; processor.go:447-470)
 *   one-request mirsha_hash_batch calls (gpuHash.Sum, the hash.Hash of
 *     processor.go:21)
 *   mirsha_host_free, mirsha_ctx_destroy
 *   GPUHasherMulti (several devices; here device 0 listed twice):
 *     mirsha_multi_create, mirsha_multi_host_alloc (portable pinned arena),
 *     mirsha_hash_arena_multi per cycle, the chunked HashBatch with
 *     mirsha_submit_arena_multi / mirsha_poll_multi / mirsha_wait_multi,
 *     mirsha_submit_slices_multi + mirsha_wait_multi, mirsha_host_free,
 *     mirsha_multi_destroy
 *
 * Requests are the testengine's (testengine/recorder.go:158-174): client c,
 * reqNo r, data = LE64(c) || "-" || LE64(r), hashed as state_machine.go:313-317
 * lays them out: LE64(c) || LE64(r) || data.  Digests are printed one per line
 * ("<tag> <index> <hex>") for tests/test_c_abi.py to compare with the golden
 * fixtures; built-in FIPS 180-4 vectors are checked here.  Exit 0 = ok.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mirsha.h"

#define CHECK(call)                                                                        \
    do {                                                                                   \
        int rc_ = (call);                                                                  \
        if (rc_ != MIRSHA_OK) {                                                            \
            fprintf(stderr, "%s failed: %d: %s\n", #call, rc_, ctx ? mirsha_last_error(ctx) : ""); \
            exit(2);                                                                       \
        }                                                                                  \
    } while (0)

static mirsha_ctx* ctx = NULL;
static uint8_t* arena = NULL;
static uint64_t arena_cap = 0;

static void le64(uint8_t* p, uint64_t v) {
    for (int i = 0; i < 8; i++) p[i] = (uint8_t)(v >> (8 * i));
}

static void print_hex(const char* tag, uint32_t i, const uint8_t* d) {
    printf("%s %u ", tag, i);
    for (int k = 0; k < 32; k++) printf("%02x", d[k]);
    printf("\n");
}

/* GPUHasher.arenaBytes: grow-only pinned arena (mirsha_host_alloc). */
static uint8_t* arena_bytes(uint64_t n) {
    if (n > arena_cap) {
        mirsha_host_free(arena);
        arena = NULL;
        arena_cap = 0;
        void* p = NULL;
        CHECK(mirsha_host_alloc(ctx, n + n / 2, &p));
        arena = (uint8_t*)p;
        arena_cap = n + n / 2;
    }
    return arena;
}

/* The testengine request i of a cycle: 3 slices, 33 bytes. */
static uint32_t pack_request(uint8_t* dst, uint64_t client, uint64_t req_no) {
    le64(dst, client);
    le64(dst + 8, req_no);
    le64(dst + 16, client);
    dst[24] = '-';
    le64(dst + 25, req_no);
    return 33;
}

static int hex_eq(const uint8_t* d, const char* hex) {
    char buf[65];
    for (int k = 0; k < 32; k++) sprintf(buf + 2 * k, "%02x", d[k]);
    return strcmp(buf, hex) == 0;
}

/* gpuHash.Sum over the bytes written so far: one request. */
static void gpu_sum(const uint8_t* msg, uint32_t len, uint8_t out[32]) {
    uint8_t* a = arena_bytes((uint64_t)len + 1);
    memcpy(a, msg, len);
    uint64_t off = 0;
    CHECK(mirsha_hash_batch(ctx, a, len, &off, &len, 1, out));
}

int main(void) {
    int ndev = 0;
    CHECK(mirsha_device_count(&ndev));
    if (ndev < 1) {
        fprintf(stderr, "no device\n");
        return 3;
    }
    CHECK(mirsha_ctx_create(0, &ctx));

    /* Two Ready() cycles of HashBatch: clients 0..3 x reqNo 0..199 = 800
     * requests, split 300 + 500 (the arena grows once). */
    const uint32_t n_total = 800;
    uint32_t done = 0;
    for (int cycle = 0; cycle < 2; cycle++) {
        const uint32_t n = cycle == 0 ? 300 : 500;
        uint8_t* a = arena_bytes(33ull * n + 1);
        uint64_t* off = malloc(8ull * n);
        uint32_t* len = malloc(4ull * n);
        uint8_t* dig = malloc(32ull * n);
        uint64_t p = 0;
        for (uint32_t k = 0; k < n; k++) {
            const uint32_t i = done + k;
            off[k] = p;
            len[k] = pack_request(a + p, i / 200, i % 200);
            p += len[k];
        }
        CHECK(mirsha_hash_batch(ctx, a, p, off, len, n, dig));
        for (uint32_t k = 0; k < n; k++) print_hex("req", done + k, dig + 32ull * k);
        free(off);
        free(len);
        free(dig);
        done += n;
    }

    /* The chunked HashBatch: the 800 requests packed chunk
     * by chunk (~3,300 bytes each: 8 chunks, more than the 4-slot ring) into
     * the arena, each chunk submitted as soon as it is packed; digests DMA'd
     * into a pinned buffer, polled per chunk, the last chunk waited for. */
    {
        uint8_t* a = arena_bytes(33ull * n_total + 1);
        void* dp = NULL;
        CHECK(mirsha_host_alloc(ctx, 32ull * n_total, &dp));
        uint8_t* dig = (uint8_t*)dp;
        uint64_t* off = malloc(8ull * n_total);
        uint32_t* len = malloc(4ull * n_total);
        uint64_t ticket[16];
        int nk = 0, polled = 0;
        for (uint32_t lo = 0; lo < n_total; lo += 100, nk++) {
            for (uint32_t i = lo; i < lo + 100; i++) {
                off[i] = 33ull * i;
                len[i] = pack_request(a + off[i], i / 200, i % 200);
            }
            CHECK(mirsha_submit_batch(ctx, a, 33ull * n_total, off + lo, len + lo, 100, dig + 32ull * lo, &ticket[nk]));
            int done = 0;
            CHECK(mirsha_poll(ctx, ticket[0], &done));
            polled += done;
        }
        CHECK(mirsha_wait(ctx, ticket[nk - 1]));
        for (uint32_t i = 0; i < n_total; i++) print_hex("chunk", i, dig + 32ull * i);
        free(off);
        free(len);
        mirsha_host_free(dp);
    }

    /* SubmitBatch / Wait: the same 800 requests as one slice each (C arrays,
     * freed after submit returns), dedup on; a second submission of the
     * first 20 in flight at the same time. */
    {
        uint8_t* a = arena_bytes(33ull * n_total + 1);
        const uint8_t** ptr = malloc(sizeof(uint8_t*) * n_total);
        uint64_t* slen = malloc(8ull * n_total);
        uint32_t* first = malloc(4ull * (n_total + 1));
        uint8_t* out1 = malloc(32ull * n_total);
        uint8_t* out2 = malloc(32ull * 20);
        for (uint32_t i = 0; i < n_total; i++) {
            ptr[i] = a + 33ull * i;
            slen[i] = pack_request(a + 33ull * i, i / 200, i % 200);
            first[i] = i;
        }
        first[n_total] = n_total;
        uint64_t t1 = 0, t2 = 0;
        CHECK(mirsha_submit_slices(ctx, ptr, slen, first, n_total, out1, MIRSHA_SUBMIT_DEDUP, &t1));
        CHECK(mirsha_submit_slices(ctx, ptr, slen, first, 20, out2, 0, &t2));
        free(ptr);
        free(slen);
        free(first);
        memset(a, 0, 33ull * n_total); /* the caller may reuse its bytes at once */
        CHECK(mirsha_wait(ctx, t2));   /* waits for t1 too: in-order completion */
        for (uint32_t i = 0; i < n_total; i++) print_hex("async", i, out1 + 32ull * i);
        if (memcmp(out1, out2, 32 * 20) != 0) {
            fprintf(stderr, "second submission differs\n");
            return 1;
        }
        free(out1);
        free(out2);
    }

    /* gpuHash.Sum: FIPS 180-4 example vectors and the reference's own
     * SHA-256("") (testengine/recorder_test.go:83). */
    {
        uint8_t d[32];
        gpu_sum((const uint8_t*)"", 0, d);
        if (!hex_eq(d, "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855")) return 1;
        gpu_sum((const uint8_t*)"abc", 3, d);
        if (!hex_eq(d, "ba7816bf8f01cfea414140de5dae2223b00361a396177a9cb410ff61f20015ad")) return 1;
        const char* two = "abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq";
        gpu_sum((const uint8_t*)two, (uint32_t)strlen(two), d);
        if (!hex_eq(d, "248d6a61d20638b8e5c026930c3e6039a33ce45964ff2167f6ecedd419db06c1")) return 1;
        uint8_t* mil = malloc(1000000);
        memset(mil, 'a', 1000000);
        gpu_sum(mil, 1000000, d);
        free(mil);
        if (!hex_eq(d, "cdc76e5c9914fb9281a1c7e284d73e67f1809a48a497200e046d39ccc7112cd0")) return 1;
        printf("fips ok\n");
    }

    mirsha_host_free(arena);
    mirsha_ctx_destroy(ctx);
    ctx = NULL;

    /* GPUHasherMulti: the 800 requests in one portable pinned arena, cut by
     * bytes over the devices (HashBatch), then as C slice arrays through the
     * asynchronous form (SubmitBatch / Wait). */
    {
        const int devs[2] = {0, ndev > 1 ? 1 : 0};
        mirsha_multi* m = NULL;
        int rc = mirsha_multi_create(devs, 2, &m);
        if (rc != MIRSHA_OK) {
            fprintf(stderr, "mirsha_multi_create failed: %d\n", rc);
            return 2;
        }
#define MCHECK(call)                                                                      \
    do {                                                                                  \
        int rc_ = (call);                                                                 \
        if (rc_ != MIRSHA_OK) {                                                           \
            fprintf(stderr, "%s failed: %d: %s\n", #call, rc_, mirsha_multi_last_error(m)); \
            exit(2);                                                                      \
        }                                                                                 \
    } while (0)
        void* pa = NULL;
        MCHECK(mirsha_multi_host_alloc(m, 33ull * n_total + 1, &pa));
        uint8_t* a = (uint8_t*)pa;
        uint64_t* off = malloc(8ull * n_total);
        uint32_t* len = malloc(4ull * n_total);
        uint8_t* dig = malloc(32ull * n_total);
        uint64_t p = 0;
        for (uint32_t i = 0; i < n_total; i++) {
            off[i] = p;
            len[i] = pack_request(a + p, i / 200, i % 200);
            p += len[i];
        }
        MCHECK(mirsha_hash_arena_multi(m, a, p, off, len, n_total, dig));
        for (uint32_t i = 0; i < n_total; i++) print_hex("multi", i, dig + 32ull * i);
        /* the chunked HashBatch over the devices: 4 chunks of 200 requests */
        {
            void* dp = NULL;
            MCHECK(mirsha_multi_host_alloc(m, 32ull * n_total, &dp));
            uint8_t* cd = (uint8_t*)dp;
            uint64_t ct[4];
            for (int k = 0; k < 4; k++) {
                MCHECK(mirsha_submit_arena_multi(m, a, p, off + 200 * k, len + 200 * k, 200, cd + 32ull * 200 * k, &ct[k]));
                int done = 0;
                MCHECK(mirsha_poll_multi(m, ct[0], &done));
            }
            MCHECK(mirsha_wait_multi(m, ct[3]));
            for (uint32_t i = 0; i < n_total; i++) print_hex("cmulti", i, cd + 32ull * i);
            mirsha_host_free(dp);
        }
        const uint8_t** ptr = malloc(sizeof(uint8_t*) * n_total);
        uint64_t* slen = malloc(8ull * n_total);
        uint32_t* first = malloc(4ull * (n_total + 1));
        for (uint32_t i = 0; i < n_total; i++) {
            ptr[i] = a + off[i];
            slen[i] = len[i];
            first[i] = i;
        }
        first[n_total] = n_total;
        uint64_t t = 0;
        memset(dig, 0, 32ull * n_total);
        MCHECK(mirsha_submit_slices_multi(m, ptr, slen, first, n_total, dig, 0, &t));
        free(ptr);
        free(slen);
        free(first);
        memset(a, 0, p); /* the caller may reuse its bytes at once */
        MCHECK(mirsha_wait_multi(m, t));
        for (uint32_t i = 0; i < n_total; i++) print_hex("amulti", i, dig + 32ull * i);
        free(off);
        free(len);
        free(dig);
        mirsha_host_free(pa);
        mirsha_multi_destroy(m);
    }
    printf("sequence ok\n");
    return 0;
}
