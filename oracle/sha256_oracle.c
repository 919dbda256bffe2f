/*
 * sha256_oracle.c — TEST INFRASTRUCTURE ONLY (see oracle.h header).
 *
 * CPU restatement of the reference's Actions.Hash path:
 *   - the Processor hash loop, processor.go:129-143 (fresh hasher per request,
 *     Write every Data slice, Sum(nil), Digests[i] in origin order);
 *   - the stdlib primitive it calls, crypto/sha256 (FIPS 180-4 §6.2), restated
 *     here from the standard, with an optional SHA-NI compression (the path Go's
 *     amd64 assembly takes on CPUs with SHA extensions) used only to make the
 *     CPU baseline a fair stand-in for the reference's speed;
 *   - the data layouts of the hash producers (proposer.go:16-20,
 *     state_machine.go:313-317, sequence.go:154-157, client_tracker.go:840-847).
 */
#include "oracle.h"

#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

static const uint32_t K256[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u,
    0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu,
    0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu,
    0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u,
    0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu,
    0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,
    0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u,
    0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u,
    0xc67178f2u};

static const uint32_t H0[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                               0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

#define ROTR(x, n) (((x) >> (n)) | ((x) << (32 - (n))))

/* FIPS 180-4 §6.2.2, one 64-byte block. */
static void compress_scalar(uint32_t h[8], const uint8_t* p, size_t nblocks) {
    while (nblocks--) {
        uint32_t w[64];
        for (int t = 0; t < 16; t++)
            w[t] = ((uint32_t)p[4 * t] << 24) | ((uint32_t)p[4 * t + 1] << 16) |
                   ((uint32_t)p[4 * t + 2] << 8) | (uint32_t)p[4 * t + 3];
        for (int t = 16; t < 64; t++) {
            uint32_t s0 = ROTR(w[t - 15], 7) ^ ROTR(w[t - 15], 18) ^ (w[t - 15] >> 3);
            uint32_t s1 = ROTR(w[t - 2], 17) ^ ROTR(w[t - 2], 19) ^ (w[t - 2] >> 10);
            w[t] = w[t - 16] + s0 + w[t - 7] + s1;
        }
        uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
        for (int t = 0; t < 64; t++) {
            uint32_t S1 = ROTR(e, 6) ^ ROTR(e, 11) ^ ROTR(e, 25);
            uint32_t ch = (e & f) ^ (~e & g);
            uint32_t t1 = hh + S1 + ch + K256[t] + w[t];
            uint32_t S0 = ROTR(a, 2) ^ ROTR(a, 13) ^ ROTR(a, 22);
            uint32_t maj = (a & b) ^ (a & c) ^ (b & c);
            uint32_t t2 = S0 + maj;
            hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
        }
        h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
        p += 64;
    }
}

#if defined(__x86_64__)
/* SHA-NI block function (the instruction class Go's crypto/sha256 amd64
 * assembly uses when the CPU reports SHA extensions). */
__attribute__((target("sha,sse4.1,ssse3"))) static void compress_shani(uint32_t h[8],
                                                                       const uint8_t* p,
                                                                       size_t nblocks) {
    const __m128i BSWAP = _mm_set_epi64x(0x0c0d0e0f08090a0bULL, 0x0405060700010203ULL);
    __m128i tmp = _mm_loadu_si128((const __m128i*)&h[0]);  /* DCBA */
    __m128i st1 = _mm_loadu_si128((const __m128i*)&h[4]);  /* HGFE */
    tmp = _mm_shuffle_epi32(tmp, 0xB1);                     /* CDAB */
    st1 = _mm_shuffle_epi32(st1, 0x1B);                     /* EFGH */
    __m128i st0 = _mm_alignr_epi8(tmp, st1, 8);             /* ABEF */
    st1 = _mm_blend_epi16(st1, tmp, 0xF0);                  /* CDGH */
    while (nblocks--) {
        const __m128i save0 = st0, save1 = st1;
        __m128i x[4];
        for (int i = 0; i < 4; i++)
            x[i] = _mm_shuffle_epi8(_mm_loadu_si128((const __m128i*)(p + 16 * i)), BSWAP);
#pragma GCC unroll 16
        for (int i = 0; i < 16; i++) {
            __m128i cur = x[i & 3];
            __m128i m = _mm_add_epi32(cur, _mm_loadu_si128((const __m128i*)&K256[4 * i]));
            st1 = _mm_sha256rnds2_epu32(st1, st0, m);
            m = _mm_shuffle_epi32(m, 0x0E);
            st0 = _mm_sha256rnds2_epu32(st0, st1, m);
            if (i < 12) {
                /* X[i+4] = msg2(msg1(X[i], X[i+1]) + alignr(X[i+3], X[i+2], 4), X[i+3]) */
                __m128i t = _mm_sha256msg1_epu32(cur, x[(i + 1) & 3]);
                t = _mm_add_epi32(t, _mm_alignr_epi8(x[(i + 3) & 3], x[(i + 2) & 3], 4));
                x[i & 3] = _mm_sha256msg2_epu32(t, x[(i + 3) & 3]);
            }
        }
        st0 = _mm_add_epi32(st0, save0);
        st1 = _mm_add_epi32(st1, save1);
        p += 64;
    }
    tmp = _mm_shuffle_epi32(st0, 0x1B);     /* FEBA */
    st1 = _mm_shuffle_epi32(st1, 0xB1);     /* DCHG */
    st0 = _mm_blend_epi16(tmp, st1, 0xF0);  /* DCBA */
    st1 = _mm_alignr_epi8(st1, tmp, 8);     /* HGFE */
    _mm_storeu_si128((__m128i*)&h[0], st0);
    _mm_storeu_si128((__m128i*)&h[4], st1);
}
#endif

static int g_force_impl = -1;

int oracle_sha256_has_shani(void) {
#if defined(__x86_64__)
    __builtin_cpu_init();
    return __builtin_cpu_supports("sha") ? 1 : 0;
#else
    return 0;
#endif
}

void oracle_sha256_force_impl(int impl) { g_force_impl = impl; }

static void compress(uint32_t h[8], const uint8_t* p, size_t nblocks) {
#if defined(__x86_64__)
    static int have = -1;
    if (have < 0) have = oracle_sha256_has_shani();
    int use = g_force_impl < 0 ? have : (g_force_impl == 1 && have);
    if (use) {
        compress_shani(h, p, nblocks);
        return;
    }
#endif
    compress_scalar(h, p, nblocks);
}

void oracle_sha256_reset(oracle_sha256* s) {
    memcpy(s->h, H0, sizeof(H0));
    s->total = 0;
    s->nbuf = 0;
}

void oracle_sha256_write(oracle_sha256* s, const uint8_t* p, size_t n) {
    s->total += n;
    if (s->nbuf) {
        size_t take = 64 - s->nbuf;
        if (take > n) take = n;
        memcpy(s->buf + s->nbuf, p, take);
        s->nbuf += (uint32_t)take;
        p += take;
        n -= take;
        if (s->nbuf == 64) {
            compress(s->h, s->buf, 1);
            s->nbuf = 0;
        }
    }
    if (n >= 64) {
        size_t nb = n / 64;
        compress(s->h, p, nb);
        p += nb * 64;
        n -= nb * 64;
    }
    if (n) {
        memcpy(s->buf, p, n);
        s->nbuf = (uint32_t)n;
    }
}

/* Sum(nil) does not modify the running state (Go's digest.Sum copies d). */
void oracle_sha256_sum(const oracle_sha256* s0, uint8_t out[32]) {
    oracle_sha256 s = *s0;
    uint64_t bits = s.total * 8;
    uint8_t pad[72];
    size_t padlen = (s.nbuf < 56) ? (56 - s.nbuf) : (120 - s.nbuf);
    memset(pad, 0, sizeof(pad));
    pad[0] = 0x80;
    for (int i = 0; i < 8; i++) pad[padlen + i] = (uint8_t)(bits >> (56 - 8 * i));
    oracle_sha256_write(&s, pad, padlen + 8);
    for (int i = 0; i < 8; i++) {
        out[4 * i] = (uint8_t)(s.h[i] >> 24);
        out[4 * i + 1] = (uint8_t)(s.h[i] >> 16);
        out[4 * i + 2] = (uint8_t)(s.h[i] >> 8);
        out[4 * i + 3] = (uint8_t)s.h[i];
    }
}

/* processor.go:133-143 */
void oracle_hash_requests(const uint8_t* arena, const uint64_t* off, const uint32_t* len,
                          uint32_t n, uint8_t* out) {
    oracle_sha256 h;
    for (uint32_t i = 0; i < n; i++) {
        oracle_sha256_reset(&h);                     /* h := p.Hasher()      :134 */
        oracle_sha256_write(&h, arena + off[i], len[i]); /* h.Write(data)    :136 */
        oracle_sha256_sum(&h, out + 32 * (size_t)i); /* Digest: h.Sum(nil)   :141 */
    }
}

void oracle_hash_slices(const uint8_t* const* slice_ptr, const uint64_t* slice_len,
                        const uint32_t* slice_first, uint32_t n, uint8_t* out) {
    oracle_sha256 h;
    for (uint32_t i = 0; i < n; i++) {
        oracle_sha256_reset(&h);
        for (uint32_t s = slice_first[i]; s < slice_first[i + 1]; s++)  /* range req.Data :135 */
            oracle_sha256_write(&h, slice_ptr[s], slice_len[s]);
        oracle_sha256_sum(&h, out + 32 * (size_t)i);
    }
}

typedef struct {
    const uint8_t* arena;
    const uint64_t* off;
    const uint32_t* len;
    uint8_t* out;
    uint32_t n;
    _Atomic uint32_t* next;  /* shared work counter: ProcessorWorkPool's channel hand-off */
} mt_job;

enum { kMtChunk = 256 };

static void* mt_worker(void* arg) {
    mt_job* j = (mt_job*)arg;
    oracle_sha256 h;
    for (;;) {
        const uint32_t b = atomic_fetch_add(j->next, kMtChunk);
        if (b >= j->n) break;
        const uint32_t e = b + kMtChunk < j->n ? b + kMtChunk : j->n;
        for (uint32_t i = b; i < e; i++) {
            oracle_sha256_reset(&h);  /* serviceHashPool reuses one hasher with Reset, :313,:325 */
            oracle_sha256_write(&h, j->arena + j->off[i], j->len[i]);
            oracle_sha256_sum(&h, j->out + 32 * (size_t)i);
        }
    }
    return NULL;
}

/* The ProcessorWorkPool analogue (processor.go:312-361): `threads` workers pull
 * requests from a shared counter (dynamic, like the reference's channel), each
 * writing digests at the request's own index (origin order kept). */
void oracle_hash_requests_mt(const uint8_t* arena, const uint64_t* off, const uint32_t* len,
                             uint32_t n, uint8_t* out, int threads) {
    if (threads <= 1 || n < 2) {
        oracle_hash_requests(arena, off, len, n, out);
        return;
    }
    if ((uint32_t)threads > n) threads = (int)n;
    _Atomic uint32_t next = 0;
    pthread_t* tid = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)threads);
    mt_job job = {arena, off, len, out, n, &next};
    for (int t = 0; t < threads; t++) pthread_create(&tid[t], NULL, mt_worker, &job);
    for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    free(tid);
}

/* sequence.go:154-157: data[i] = ack.Digest; null requests carry an empty
 * digest (client_tracker.go:840-847), i.e. a zero-length Write. */
void oracle_batch_digests(const uint8_t* req_digests, const uint32_t* idx,
                          const uint32_t* batch_first, uint32_t n_batches, uint8_t* out) {
    oracle_sha256 h;
    for (uint32_t b = 0; b < n_batches; b++) {
        oracle_sha256_reset(&h);
        for (uint32_t k = batch_first[b]; k < batch_first[b + 1]; k++) {
            if (idx[k] == ORACLE_NULL_REQUEST) continue; /* Write([]byte{}) */
            oracle_sha256_write(&h, req_digests + 32 * (size_t)idx[k], 32);
        }
        oracle_sha256_sum(&h, out + 32 * (size_t)b);
    }
}

void oracle_le64(uint64_t v, uint8_t out[8]) {
    for (int i = 0; i < 8; i++) out[i] = (uint8_t)(v >> (8 * i)); /* binary.LittleEndian.PutUint64 */
}

size_t oracle_request_message(uint64_t client_id, uint64_t req_no, const uint8_t* data,
                              size_t data_len, uint8_t* out) {
    oracle_le64(client_id, out);     /* uint64ToBytes(requestData.ClientId) :314 */
    oracle_le64(req_no, out + 8);    /* uint64ToBytes(requestData.ReqNo)    :315 */
    if (data_len) memcpy(out + 16, data, data_len); /* requestData.Data    :316 */
    return 16 + data_len;
}

uint64_t oracle_splitmix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

void oracle_gen_requests(uint64_t seed, uint64_t first, uint64_t count, uint32_t data_len,
                         uint8_t* arena) {
    const uint64_t stride = 16 + (uint64_t)data_len;
    for (uint64_t r = 0; r < count; r++) {
        uint64_t i = first + r;
        uint8_t* m = arena + r * stride;
        oracle_le64(i % 16, m);
        oracle_le64(i / 16, m + 8);
        uint64_t key = oracle_splitmix64(seed ^ i);
        for (uint32_t j = 0; j * 8 < data_len; j++) {
            uint64_t w = oracle_splitmix64(key + j);
            for (uint32_t b = 0; b < 8 && j * 8 + b < data_len; b++)
                m[16 + j * 8 + b] = (uint8_t)(w >> (8 * b));
        }
    }
}

uint32_t oracle_mixed_data_len(uint64_t seed, uint64_t i) {
    const uint64_t x = oracle_splitmix64(seed ^ i ^ ORACLE_LEN_TAG) >> 40;
    const uint64_t t = 10u * x;
    const uint64_t e = t >> 24, m = t & 0xFFFFFFu;
    return (uint32_t)((64ull << e) + (((64ull << e) * m) >> 24));
}

void oracle_mixed_lengths(uint64_t seed, uint64_t first, uint64_t n, uint32_t* len_out) {
    for (uint64_t r = 0; r < n; r++) len_out[r] = 16u + oracle_mixed_data_len(seed, first + r);
}

void oracle_gen_mixed(uint64_t seed, const uint64_t* ids, uint64_t n, uint8_t* arena, uint64_t* off_out,
                      uint32_t* len_out) {
    uint64_t p = 0;
    for (uint64_t k = 0; k < n; k++) {
        const uint64_t i = ids[k];
        const uint32_t dl = oracle_mixed_data_len(seed, i);
        uint8_t* m = arena + p;
        oracle_le64(i % 16, m);
        oracle_le64(i / 16, m + 8);
        const uint64_t key = oracle_splitmix64(seed ^ i);
        for (uint32_t j = 0; j * 8 < dl; j++) {
            const uint64_t w = oracle_splitmix64(key + j);
            for (uint32_t b = 0; b < 8 && j * 8 + b < dl; b++) m[16 + j * 8 + b] = (uint8_t)(w >> (8 * b));
        }
        off_out[k] = p;
        len_out[k] = 16u + dl;
        p += 16u + dl;
    }
}
