/*
 * evp_loop.c -- TEST INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg and
 * tests/).  BASELINE.md's CPU-baseline caveat: with no Go toolchain on the box,
 * time the reference hash loop through OpenSSL's EVP SHA-256 and label it
 * "OpenSSL stand-in for Go crypto/sha256".
 *
 * The loop is processor.go:133-143:
 *     for i, req := range actions.Hash {
 *         h := p.Hasher()                      // sha256.New
 *         for _, data := range req.Data { h.Write(data) }
 *         Digests[i] = h.Sum(nil)
 *     }
 * restated with EVP_DigestInit_ex2 per request (sha256.New), one
 * EVP_DigestUpdate per HashRequest.Data slice (h.Write) and EVP_DigestFinal_ex
 * (h.Sum).  A request of the synthetic streams is the three slices
 * state_machine.go:313-317 hands over -- LE64(ClientId), LE64(ReqNo), Data --
 * so a message of L >= 16 bytes is written as [0,8), [8,16), [16,L).  Batch
 * digests write one 32-byte RequestAck digest per entry (sequence.go:154-157).
 * One EVP_MD_CTX per thread is reused (Go allocates a fresh digest per
 * request; reusing is the faster, conservative choice for a baseline).  The
 * pool form pulls 64-request chunks from a shared counter and writes
 * Digests[i] in origin order (ProcessorWorkPool analogue, processor.go:312-361).
 */
#include <openssl/evp.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdlib.h>

static EVP_MD* g_md;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void fetch_md(void) { g_md = EVP_MD_fetch(NULL, "SHA256", NULL); }

static const EVP_MD* md(void) {
    pthread_once(&g_once, fetch_md);
    return g_md;
}

static int hash_one(EVP_MD_CTX* c, const uint8_t* m, uint32_t len, int split, uint8_t* out) {
    unsigned int dl = 0;
    if (!EVP_DigestInit_ex2(c, md(), NULL)) return -1;
    if (split && len >= 16) {
        if (!EVP_DigestUpdate(c, m, 8) || !EVP_DigestUpdate(c, m + 8, 8) || !EVP_DigestUpdate(c, m + 16, len - 16))
            return -1;
    } else if (!EVP_DigestUpdate(c, m, len)) {
        return -1;
    }
    return EVP_DigestFinal_ex(c, out, &dl) && dl == 32 ? 0 : -1;
}

typedef struct {
    const uint8_t* arena;
    const uint64_t* off;
    const uint32_t* len;
    uint32_t n;
    int split;
    uint8_t* out;
    _Atomic uint32_t next;
    _Atomic int err;
} Job;

static void* worker(void* arg) {
    Job* j = (Job*)arg;
    EVP_MD_CTX* c = EVP_MD_CTX_new();
    if (!c) {
        j->err = 1;
        return NULL;
    }
    for (;;) {
        const uint32_t a = atomic_fetch_add(&j->next, 64u);
        if (a >= j->n) break;
        const uint32_t b = a + 64u < j->n ? a + 64u : j->n;
        for (uint32_t i = a; i < b; i++)
            if (hash_one(c, j->arena + j->off[i], j->len[i], j->split, j->out + 32ull * i)) j->err = 1;
    }
    EVP_MD_CTX_free(c);
    return NULL;
}

/* Digests[i] of n requests (arena + off/len), `threads` workers (1 = the
 * serial Processor).  split: write each message as the reference's three
 * slices.  0 on success. */
int evp_hash_requests(const uint8_t* arena, const uint64_t* off, const uint32_t* len, uint32_t n, uint8_t* out,
                      int threads, int split) {
    if (!md()) return -1;
    Job j = {arena, off, len, n, split, out, 0, 0};
    if (threads <= 1 || n < 128) {
        worker(&j);
        return j.err ? -1 : 0;
    }
    pthread_t* tid = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
    if (!tid) return -1;
    for (int t = 0; t < threads; t++) pthread_create(&tid[t], NULL, worker, &j);
    for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    free(tid);
    return j.err ? -1 : 0;
}

/* Batch digests: list b = request digests idx[first[b] .. first[b+1]), one
 * 32-byte Write each; idx 0xFFFFFFFF = a null request, an empty Write
 * (client_tracker.go:840-847).  0 on success. */
int evp_batch_digests(const uint8_t* req_digests, const uint32_t* idx, const uint32_t* first, uint32_t n_batches,
                      uint8_t* out) {
    EVP_MD_CTX* c = EVP_MD_CTX_new();
    if (!c || !md()) {
        EVP_MD_CTX_free(c);
        return -1;
    }
    int rc = 0;
    for (uint32_t b = 0; b < n_batches && !rc; b++) {
        unsigned int dl = 0;
        if (!EVP_DigestInit_ex2(c, md(), NULL)) rc = -1;
        for (uint32_t k = first[b]; k < first[b + 1] && !rc; k++)
            if (idx[k] != 0xFFFFFFFFu && !EVP_DigestUpdate(c, req_digests + 32ull * idx[k], 32)) rc = -1;
        if (!rc && !(EVP_DigestFinal_ex(c, out + 32ull * b, &dl) && dl == 32)) rc = -1;
    }
    EVP_MD_CTX_free(c);
    return rc;
}

/* OpenSSL's version string, for the bench line. */
const char* evp_version(void) { return OpenSSL_version(OPENSSL_VERSION); }
