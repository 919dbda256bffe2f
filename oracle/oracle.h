/*
 * oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's Actions.Hash hot path (IBM MirBFT, Go).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may link,
 * load or call anything declared here, and only as the checker / the timed CPU
 * baseline.  The product path (mirbft_amd/, libmirsha.so) never touches it.
 *
 * Parity pinning: the reference is pure Go (no Go toolchain in this image), and
 * the arithmetic lives in Go's stdlib crypto/sha256 (Go 1.13/1.14, .travis.yml:5-6),
 * which implements FIPS 180-4 SHA-256.  This restatement is pinned by
 *   - FIPS 180-4 / NIST CAVP known-answer vectors (tests/golden/kat.json),
 *   - the reference's own only digest assertion, SHA-256("") after a
 *     checkpoint reset (testengine/recorder_test.go:83),
 *   - golden vectors produced by Python hashlib (OpenSSL 3.0.2, a second,
 *     independent FIPS 180-4 implementation) over byte layouts restated from
 *     the reference (tests/golden/make_golden.py).
 */
#ifndef MIRBFT_ORACLE_H
#define MIRBFT_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Streaming SHA-256 state: the hash.Hash returned by sha256.New()
 * (processor.go:21 `type Hasher func() hash.Hash`). */
typedef struct {
    uint32_t h[8];
    uint8_t buf[64];
    uint64_t total; /* bytes written */
    uint32_t nbuf;
} oracle_sha256;

void oracle_sha256_reset(oracle_sha256* s);                           /* h.Reset()  */
void oracle_sha256_write(oracle_sha256* s, const uint8_t* p, size_t n); /* h.Write(d) */
void oracle_sha256_sum(const oracle_sha256* s, uint8_t out[32]);     /* h.Sum(nil) */

/* 0 = portable scalar compression; 1 = x86 SHA-NI compression (what Go's
 * crypto/sha256 amd64 assembly uses when the CPU has SHA extensions). */
int oracle_sha256_has_shani(void);
void oracle_sha256_force_impl(int impl); /* -1 auto, 0 scalar, 1 shani */

/* processor.go:129-143 — for each request i: fresh hasher, Write its bytes,
 * Sum(nil) into out[32*i], origin order.  Request i = arena[off[i] .. off[i]+len[i]). */
void oracle_hash_requests(const uint8_t* arena, const uint64_t* off, const uint32_t* len,
                          uint32_t n, uint8_t* out);

/* Same loop over multi-slice requests (HashRequest.Data [][]byte, actions.go:157-164):
 * request i = concat of slices [slice_first[i], slice_first[i+1]). */
void oracle_hash_slices(const uint8_t* const* slice_ptr, const uint64_t* slice_len,
                        const uint32_t* slice_first, uint32_t n, uint8_t* out);

/* ProcessorWorkPool-style multi-threaded variant (processor.go:312-361) but
 * ORDER-PRESERVING (results written by index).  threads<=0 => 1. */
void oracle_hash_requests_mt(const uint8_t* arena, const uint64_t* off, const uint32_t* len,
                             uint32_t n, uint8_t* out, int threads);

/* sequence.go:154-157 (and batch_tracker.go:147-150, VerifyBatch): batch b's
 * digest = SHA-256(d[idx[k]] for k in [batch_first[b], batch_first[b+1])), each
 * d 32 bytes from req_digests; idx == 0xFFFFFFFF is a null request whose digest
 * is EMPTY (client_tracker.go:840-847) and contributes 0 bytes. */
#define ORACLE_NULL_REQUEST 0xFFFFFFFFu
void oracle_batch_digests(const uint8_t* req_digests, const uint32_t* idx,
                          const uint32_t* batch_first, uint32_t n_batches, uint8_t* out);

/* proposer.go:16-20 uint64ToBytes: 8-byte little endian. */
void oracle_le64(uint64_t v, uint8_t out[8]);

/* state_machine.go:313-317 / client_tracker.go:618-622: request message bytes
 * LE64(client) || LE64(reqNo) || data.  Returns bytes written (16 + data_len). */
size_t oracle_request_message(uint64_t client_id, uint64_t req_no, const uint8_t* data,
                              size_t data_len, uint8_t* out);

/* ---- synthetic workload generator — identical to the device
 * generator in mirbft_amd/csrc/mirsha_gen.hip ---- */
uint64_t oracle_splitmix64(uint64_t x);
/* Request i: ClientId = i % 16, ReqNo = i / 16, Data = data_len bytes where
 * 8-byte word j = splitmix64(splitmix64(seed ^ i) + j) (little-endian bytes).
 * Writes `count` messages of (16 + data_len) bytes starting at request `first`,
 * densely packed (message stride 16 + data_len). */
void oracle_gen_requests(uint64_t seed, uint64_t first, uint64_t count, uint32_t data_len,
                         uint8_t* arena);

/* BASELINE config 5 (mixed sizes): request i's data length is
 * log-uniform over the octaves of [64, 65536) and uniform inside an octave,
 * in integer arithmetic (bit-identical on host, device and numpy):
 *   x = splitmix64(seed ^ i ^ ORACLE_LEN_TAG) >> 40;  t = 10 x;
 *   e = t >> 24;  m = t & 0xFFFFFF;  data_len = (64 << e) + (((64 << e) * m) >> 24).
 * Message = LE64(i % 16) || LE64(i / 16) || data (bytes as oracle_gen_requests). */
#define ORACLE_LEN_TAG 0x4C454E4754480000ull
uint32_t oracle_mixed_data_len(uint64_t seed, uint64_t i);
/* Request lengths (16-byte header + data) of requests [first, first + n). */
void oracle_mixed_lengths(uint64_t seed, uint64_t first, uint64_t n, uint32_t* len_out);
/* Messages for the request ids[k] (any order), packed densely in that order:
 * off_out[k] / len_out[k] = offset / message length (16 + data_len) of ids[k]. */
void oracle_gen_mixed(uint64_t seed, const uint64_t* ids, uint64_t n, uint8_t* arena, uint64_t* off_out,
                      uint32_t* len_out);

#ifdef __cplusplus
}
#endif
#endif
