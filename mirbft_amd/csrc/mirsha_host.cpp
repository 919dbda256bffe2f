// mirsha_host.cpp — host-side packing and content-addressed dedup for the
// C-ABI (see mirsha_host.h).  Pure CPU code: no HIP calls, so the dedup plan
// is testable without a GPU (mirsha_dedup_plan, tests/test_host_dedup.py).
#include "mirsha_host.h"

#include <stdlib.h>
#include <string.h>
#include <emmintrin.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <map>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/mirsha.h"

namespace mirsha {
namespace host {

namespace {

int env_threads() {
    static const int v = [] {
        const char* e = getenv("MIRSHA_HOST_THREADS");
        return e ? atoi(e) : 0;
    }();
    return v;
}

bool weak_fp() {
    static const bool v = [] {
        // test-only (with MIRSHA_AB=1): every fingerprint equal
        const char* ab = getenv("MIRSHA_AB");
        const char* e = getenv("MIRSHA_DEDUP_WEAK_FP");
        return ab && ab[0] == '1' && e && e[0] == '1';
    }();
    return v;
}

inline uint64_t rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }

// Streaming word hash with a byte carry, so slicing does not matter: word k
// of the concatenated stream (8 bytes, little-endian) feeds lane k & 3, each
// lane one xor-multiply-rotate step (four independent chains, ~1.3 cycles per
// word).  Equal fingerprints are only candidates: dedup confirms every match
// byte for byte, so the hash needs spread, not collision resistance.
struct Fp {
    uint64_t h[4] = {0x6D69726274667030ull, 0x9E3779B97F4A7C15ull, 0xC2B2AE3D27D4EB4Full, 0x165667B19E3779F9ull};
    uint64_t carry = 0, total = 0;
    int nc = 0;
    uint64_t idx = 0;  // words consumed
    static constexpr uint64_t kM[4] = {0x94D049BB133111EBull, 0xBF58476D1CE4E5B9ull, 0xD6E8FEB86659FD93ull,
                                       0x9FB21C651E98DF25ull};
    inline void lane(int k, uint64_t w) { h[k] = rotl((h[k] ^ w) * kM[k], 23 + 8 * k); }
    inline void word(uint64_t w) { lane((int)(idx++ & 3u), w); }
    inline void words4(const uint8_t* p) {  // 4 words from a 4-aligned word index
        uint64_t a[4];
        memcpy(a, p, 32);
        lane(0, a[0]);
        lane(1, a[1]);
        lane(2, a[2]);
        lane(3, a[3]);
        idx += 4;
    }
    void bytes(const uint8_t* p, uint64_t n) {
        total += n;
        while (nc && n) {
            carry |= (uint64_t)*p++ << (8 * nc);
            n--;
            if (++nc == 8) { word(carry); carry = 0; nc = 0; }
        }
        while ((idx & 3u) && n >= 8) {  // realign so word k always feeds lane k & 3
            uint64_t a;
            memcpy(&a, p, 8);
            word(a);
            p += 8;
            n -= 8;
        }
        for (; n >= 32; p += 32, n -= 32) words4(p);
        while (n >= 8) {
            uint64_t a;
            memcpy(&a, p, 8);
            word(a);
            p += 8;
            n -= 8;
        }
        while (n) {
            carry |= (uint64_t)*p++ << (8 * nc);
            nc++;
            n--;
        }
    }
    uint64_t final() {
        if (nc) word(carry ^ ((uint64_t)nc << 56));
        uint64_t x = h[0] ^ rotl(h[1], 17) ^ rotl(h[2], 31) ^ rotl(h[3], 47) ^ total * 0xD6E8FEB86659FD93ull;
        x ^= x >> 32;
        x *= 0xD6E8FEB86659FD93ull;
        x ^= x >> 29;
        return x;
    }
};

}  // namespace

namespace {

// Persistent workers for parallel_for.  A staged host call runs a dozen
// parallel passes (validation, metadata, one pack per pinned chunk, digest
// copy-out); spawning and joining 16 std::threads per pass cost ~0.1-0.3 ms
// each, which was most of the validate / plan phases of a config-2 call.
// One job at a time (callers serialise on `submit_`); the calling thread takes
// parts too.  A parallel_for issued from inside a job runs inline.  The pool
// is created on first use and never destroyed (workers park on a condition
// variable until the process exits).
thread_local bool t_in_pool_job = false;
thread_local int t_pool_slot = 0, t_pool_threads = 0;  // use_pool

class Pool {
  public:
    explicit Pool(int workers) {
        for (int w = 0; w < workers; w++) std::thread([this] { loop(); }).detach();
    }
    void run(uint32_t n, int parts, const std::function<void(uint32_t, uint32_t)>& fn) {
        std::lock_guard<std::mutex> one(submit_);
        {
            std::lock_guard<std::mutex> g(m_);
            fn_ = &fn;
            n_ = n;
            parts_ = parts;
            step_ = (n + parts - 1) / parts;
            next_.store(0);
            left_ = parts;
            gen_++;
        }
        cv_.notify_all();
        work();
        std::unique_lock<std::mutex> g(m_);
        done_.wait(g, [this] { return left_ == 0; });
        fn_ = nullptr;
    }

  private:
    void work() {
        const bool was = t_in_pool_job;
        t_in_pool_job = true;
        for (;;) {
            const int p = next_.fetch_add(1);
            if (p >= parts_) break;
            const uint32_t lo = (uint32_t)std::min<uint64_t>((uint64_t)p * step_, n_);
            const uint32_t hi = (uint32_t)std::min<uint64_t>((uint64_t)(p + 1) * step_, n_);
            if (lo < hi) (*fn_)(lo, hi);
            std::lock_guard<std::mutex> g(m_);
            if (--left_ == 0) done_.notify_all();
        }
        t_in_pool_job = was;
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return gen_ != seen; });
                seen = gen_;
                if (!fn_) continue;
            }
            work();
        }
    }
    std::mutex submit_, m_;
    std::condition_variable cv_, done_;
    const std::function<void(uint32_t, uint32_t)>* fn_ = nullptr;
    uint32_t n_ = 0, step_ = 0;
    int parts_ = 0, left_ = 0;
    std::atomic<int> next_{0};
    uint64_t gen_ = 0;
};

Pool& pool() {
    static Pool* p = new Pool(max_threads() - 1);
    if (t_pool_slot <= 0) return *p;
    // Keyed by (slot, threads): a later mirsha_multi with a different share
    // of the host threads gets a pool of its own size.  Pools are
    // kept for the process (their workers park on a condition variable).
    static std::mutex mu;
    static std::map<std::pair<int, int>, Pool*> extra;
    std::lock_guard<std::mutex> g(mu);
    Pool*& q = extra[{t_pool_slot, t_pool_threads}];
    if (!q) q = new Pool(std::max(t_pool_threads, 1) - 1);
    return *q;
}

}  // namespace

int max_threads() {
    int t = env_threads();
    if (t <= 0) t = std::min(std::max((int)std::thread::hardware_concurrency(), 1), 16);
    return t;
}

void use_pool(int slot, int threads) {
    t_pool_slot = (slot > 0 && slot < kMaxPools) ? slot : 0;
    t_pool_threads = t_pool_slot ? std::max(threads, 1) : 0;
}

int threads_for(uint64_t bytes, uint32_t n) {
    if (n < 2 || bytes < (4ull << 20)) return 1;
    int t = t_pool_slot ? t_pool_threads : max_threads();
    const uint64_t by_bytes = bytes / (1ull << 20);  // >= 1 MiB per thread
    t = (int)std::min<uint64_t>((uint64_t)t, std::max<uint64_t>(1, by_bytes));
    return std::min<int>(t, (int)n);
}

void parallel_for(uint32_t n, int threads, const std::function<void(uint32_t, uint32_t)>& fn) {
    if (n == 0) return;
    threads = std::min<int>(threads, (int)n);
    if (threads <= 1 || t_in_pool_job) {
        fn(0, n);
        return;
    }
    pool().run(n, threads, fn);
}

uint64_t exclusive_scan(const uint32_t* len, uint32_t n, uint64_t* out) {
    // The caller's share of the host threads, as threads_for: a mirsha_multi
    // worker (pool slot set) gets its own slice of them.
    const int budget = t_pool_slot ? std::max(t_pool_threads, 1) : max_threads();
    const int T = n < (1u << 16) ? 1 : std::min<int>(budget, (int)(n >> 15));
    if (T <= 1) {
        uint64_t p = 0;
        for (uint32_t i = 0; i < n; i++) {
            out[i] = p;
            p += len[i];
        }
        return p;
    }
    const uint32_t step = (n + (uint32_t)T - 1) / (uint32_t)T;
    std::vector<uint64_t> part(T + 1, 0);
    parallel_for(n, T, [&](uint32_t a, uint32_t b) {
        uint64_t s = 0;
        for (uint32_t i = a; i < b; i++) s += len[i];
        part[a / step + 1] = s;
    });
    for (int k = 1; k <= T; k++) part[k] += part[k - 1];
    parallel_for(n, T, [&](uint32_t a, uint32_t b) {
        uint64_t p = part[a / step];
        for (uint32_t i = a; i < b; i++) {
            out[i] = p;
            p += len[i];
        }
    });
    return part[T];
}

uint64_t fingerprint(const uint8_t* const* ptr, const uint64_t* len, uint32_t s0, uint32_t s1) {
    if (weak_fp()) return 0;
    Fp f;
    for (uint32_t s = s0; s < s1; s++) {
        const uint64_t L = len[s];
        const uint8_t* p = ptr[s];
        if (f.nc == 0 && L == 8) {
            // Whole words at a word boundary of the stream (every slice of
            // epochChangeHashData: 8-byte LE64 fields and 32-byte digests,
            // stateless.go:311-340): no carry to thread through.
            uint64_t w;
            memcpy(&w, p, 8);
            f.total += 8;
            f.word(w);
        } else if (f.nc == 0 && L == 32 && (f.idx & 3u) == 0) {
            f.total += 32;
            f.words4(p);
        } else if (L) {
            f.bytes(p, L);
        }
    }
    return f.final();
}

namespace {
inline bool eq_bytes(const uint8_t* p, const uint8_t* q, uint64_t n) {
    if (p == q) return true;
    if (n == 8) {
        uint64_t x, y;
        memcpy(&x, p, 8);
        memcpy(&y, q, 8);
        return x == y;
    }
    if (n == 32) {
        uint64_t x[4], y[4];
        memcpy(x, p, 32);
        memcpy(y, q, 32);
        return ((x[0] ^ y[0]) | (x[1] ^ y[1]) | (x[2] ^ y[2]) | (x[3] ^ y[3])) == 0;
    }
    return memcmp(p, q, n) == 0;
}
}  // namespace

bool equal_concat(const uint8_t* const* ptr, const uint64_t* len, uint32_t a0, uint32_t a1, uint32_t b0,
                  uint32_t b1) {
    // Same slicing (the usual case: two copies of one message type): compare
    // slice by slice; any difference in the slice lengths falls through to
    // the general walk over the concatenations.
    if (a1 - a0 == b1 - b0) {
        uint32_t k = 0;
        for (; k < a1 - a0; k++) {
            const uint64_t L = len[a0 + k];
            if (L != len[b0 + k]) break;
            if (!eq_bytes(ptr[a0 + k], ptr[b0 + k], L)) return false;
        }
        if (k == a1 - a0) return true;
    }
    uint32_t sa = a0, sb = b0;
    uint64_t pa = 0, pb = 0;  // positions inside the current slices
    for (;;) {
        while (sa < a1 && pa == len[sa]) { sa++; pa = 0; }
        while (sb < b1 && pb == len[sb]) { sb++; pb = 0; }
        const bool ea = sa == a1, eb = sb == b1;
        if (ea || eb) return ea && eb;
        const uint64_t k = std::min(len[sa] - pa, len[sb] - pb);
        if (ptr[sa] + pa != ptr[sb] + pb && memcmp(ptr[sa] + pa, ptr[sb] + pb, k) != 0) return false;
        pa += k;
        pb += k;
    }
}

namespace {
inline uint64_t dedup_key(uint64_t fp, uint64_t len) { return fp ^ (len * 0x9E3779B97F4A7C15ull); }

// Test hook (with MIRSHA_AB=1): slices per segment, so that small test inputs
// run the multi-segment path.
uint64_t env_segment_slices() {
    static const uint64_t v = [] {
        const char* ab = getenv("MIRSHA_AB");
        const char* e = getenv("MIRSHA_DEDUP_SEGMENT_SLICES");
        return ab && ab[0] == '1' && e ? strtoull(e, nullptr, 10) : 0ull;
    }();
    return v;
}
}  // namespace

namespace {
// Key of a request's first min(64, L) bytes (slicing-independent): the
// speculation key of DedupScan::scan.  False if a slice with bytes has no
// address (the request is malformed; the fingerprint walk reports it).
bool prefix_key(const uint8_t* const* ptr, const uint64_t* len, uint32_t s0, uint32_t s1, uint64_t* key) {
    uint8_t buf[64];
    uint32_t got = 0;
    for (uint32_t s = s0; s < s1 && got < 64u; s++) {
        const uint64_t L = len[s];
        if (!L) continue;
        if (!ptr[s]) return false;
        const uint32_t k = (uint32_t)std::min<uint64_t>(L, 64u - got);
        memcpy(buf + got, ptr[s], k);
        got += k;
    }
    memset(buf + got, 0, 64u - got);
    Fp f;
    f.total = got;
    f.words4(buf);
    f.words4(buf + 32);
    *key = f.final();
    return true;
}

// equal_concat for a request `a` that is not validated yet: false (not equal)
// as soon as one of its slices with bytes has no address, and no byte of `a`
// past b's length is read.
bool equal_concat_checked(const uint8_t* const* ptr, const uint64_t* len, uint32_t a0, uint32_t a1, uint32_t b0,
                          uint32_t b1) {
    for (uint32_t s = a0; s < a1; s++)
        if (len[s] && !ptr[s]) return false;
    return equal_concat(ptr, len, a0, a1, b0, b1);
}
}  // namespace

DedupScan::DedupScan(const uint8_t* const* ptr, const uint64_t* len, const uint32_t* first, uint32_t n,
                     uint64_t max_len)
    : ptr_(ptr), len_(len), first_(first), n_(n), ns_(n ? first[n] : 0u), max_len_(max_len), req_len_(n, 0),
      fp_(n, 0), tent_(n, kUnset), err_(n, 0), ok_(n, 0) {
    head_.reserve((size_t)std::min<uint32_t>(n, 1u << 16) * 2);
}

std::vector<uint32_t> DedupScan::segments() const {
    // ~1/16 of the slice arrays per segment (config 4: 256 acks = 15.8 MB of
    // payload + 15.8 MB of slice arrays), at least 2^18 slices; a call below
    // 2^19 slices is one segment (the plain two-pass plan).
    uint64_t per = env_segment_slices();
    if (!per) per = ns_ < (1u << 19) ? ~0ull : std::max<uint64_t>(ns_ / 16u, 1u << 18);
    std::vector<uint32_t> b{0u};
    uint64_t next = per;
    for (uint32_t i = 1; i < n_; i++) {
        // first[] may be malformed here (scan reports it); cut only where it is monotone
        if (first_[i] >= next && first_[i] <= ns_ && first_[i] >= first_[b.back()]) {
            b.push_back(i);
            next = (uint64_t)first_[i] + per;
        }
    }
    b.push_back(n_);
    return b;
}

bool DedupScan::scan(uint32_t lo, uint32_t hi) {
    if (lo >= hi) return true;
    const bool weak = weak_fp();
    std::atomic<bool> bad{false};
    const uint64_t meta = 16ull * ((first_[hi] > first_[lo] && first_[hi] <= ns_) ? first_[hi] - first_[lo] : 0u);
    parallel_for(hi - lo, threads_for(meta, hi - lo), [&](uint32_t a, uint32_t b) {
        for (uint32_t i = lo + a; i < lo + b; i++) {
            err_[i] = 0;
            req_len_[i] = 0;
            fp_[i] = 0;
            if (first_[i + 1] < first_[i] || first_[i + 1] > ns_) { err_[i] = 1; bad = true; continue; }
            // Speculation: the head of an earlier segment with the same first
            // 64 bytes.  Equal bytes (one walk, compared slice by slice) make
            // the fingerprint walk unnecessary: equal contents have equal
            // lengths and fingerprints, and that head is the first request with
            // this content (heads are the first of their (fingerprint, length)
            // key).  A refuted guess costs the comparison up to the first
            // difference, then the request takes the fingerprint walk.
            if (!prefix_.empty()) {
                uint64_t pk;
                if (prefix_key(ptr_, len_, first_[i], first_[i + 1], &pk)) {
                    const auto it = prefix_.find(pk);
                    if (it != prefix_.end()) {
                        const uint32_t j = it->second;
                        if (equal_concat_checked(ptr_, len_, first_[i], first_[i + 1], first_[j], first_[j + 1])) {
                            req_len_[i] = req_len_[j];
                            fp_[i] = fp_[j];
                            tent_[i] = j;
                            ok_[i] = 1;
                            continue;
                        }
                    }
                }
            }
            Fp f;
            bool over = false;  // past max_len: no more bytes read (as slice_lengths, which reads none)
            for (uint32_t s = first_[i]; s < first_[i + 1]; s++) {
                const uint64_t L = len_[s];
                const uint8_t* p = ptr_[s];
                if (L && !p) { err_[i] = 2; break; }
                if (!over && f.total + L > max_len_) over = true;
                if (weak || over) { f.total += L; continue; }
                if (f.nc == 0 && L == 8) {  // as fingerprint(): whole words at a word boundary
                    uint64_t w;
                    memcpy(&w, p, 8);
                    f.total += 8;
                    f.word(w);
                } else if (f.nc == 0 && L == 32 && (f.idx & 3u) == 0) {
                    f.total += 32;
                    f.words4(p);
                } else if (L) {
                    f.bytes(p, L);
                }
            }
            if (!err_[i] && f.total > max_len_) err_[i] = 3;
            if (err_[i]) { bad = true; continue; }
            req_len_[i] = f.total;
            fp_[i] = weak ? 0 : f.final();
            // A head from an earlier segment (the table is read-only while
            // segments are scanned): confirm now, while this request's bytes
            // and slice arrays are still in this core's cache.
            const auto it = head_.find(dedup_key(fp_[i], f.total));
            if (it != head_.end()) {
                const uint32_t j = it->second;
                tent_[i] = j;
                ok_[i] = req_len_[j] == f.total &&
                         equal_concat(ptr_, len_, first_[i], first_[i + 1], first_[j], first_[j + 1]);
            }
        }
    });
    return !bad;
}

void DedupScan::assign(uint32_t lo, uint32_t hi, std::vector<uint32_t>& heads) {
    for (uint32_t i = lo; i < hi; i++) {
        if (tent_[i] != kUnset) continue;  // matched a head of an earlier segment in scan()
        const auto it = head_.emplace(dedup_key(fp_[i], req_len_[i]), i).first;
        tent_[i] = it->second;
        if (tent_[i] == i) {
            ok_[i] = 1;
            heads.push_back(i);
            uint64_t pk;
            if (prefix_key(ptr_, len_, first_[i], first_[i + 1], &pk)) prefix_.emplace(pk, i);
        } else {
            ok_[i] = kPending;
        }
    }
}

void DedupScan::confirm(uint32_t lo, uint32_t hi) {
    if (lo >= hi) return;
    uint64_t bytes = 0;
    uint32_t m = 0;
    for (uint32_t i = lo; i < hi; i++)
        if (ok_[i] == kPending) {
            bytes += req_len_[i];
            m++;
        }
    if (!m) return;
    parallel_for(hi - lo, threads_for(bytes, m), [&](uint32_t a, uint32_t b) {
        for (uint32_t i = lo + a; i < lo + b; i++) {
            if (ok_[i] != kPending) continue;
            const uint32_t j = tent_[i];
            ok_[i] = req_len_[i] == req_len_[j] &&
                     equal_concat(ptr_, len_, first_[i], first_[i + 1], first_[j], first_[j + 1]);
        }
    });
}

uint32_t DedupScan::resolve(uint32_t* rep, std::vector<uint32_t>* extra) {
    // Sequential: confirmed -> tentative rep; collided -> search the distinct
    // representatives already seen under this key (rare).
    std::unordered_map<uint64_t, std::vector<uint32_t>> reps;  // only keys that collided
    uint32_t distinct = 0;
    for (uint32_t i = 0; i < n_; i++) {
        const uint32_t j = tent_[i];
        if (j == i) {
            rep[i] = i;
            distinct++;
            continue;
        }
        if (ok_[i] == 1) {
            rep[i] = j;
            continue;
        }
        auto& cand = reps[dedup_key(fp_[i], req_len_[i])];
        uint32_t found = UINT32_MAX;
        for (uint32_t r : cand)
            if (req_len_[r] == req_len_[i] &&
                equal_concat(ptr_, len_, first_[i], first_[i + 1], first_[r], first_[r + 1])) {
                found = r;
                break;
            }
        if (found == UINT32_MAX) {
            cand.push_back(i);
            rep[i] = i;
            distinct++;
            if (extra) extra->push_back(i);
        } else {
            rep[i] = found;
        }
    }
    // rep[i] is the smallest equal index: equal requests share the key, so a
    // request equal to tent[i] (the key's first index) has rep tent[i]; the
    // first member of any other class under the key entered `reps` above.
    return distinct;
}

uint32_t dedup_plan(const uint8_t* const* ptr, const uint64_t* len, const uint32_t* first, uint32_t n,
                    uint32_t* rep, const uint8_t** err_out, std::vector<uint8_t>* err) {
    DedupScan d(ptr, len, first, n, ~0ull);
    const std::vector<uint32_t> seg = d.segments();
    std::vector<uint32_t> heads;
    for (size_t k = 0; k + 1 < seg.size(); k++) {
        if (!d.scan(seg[k], seg[k + 1])) {
            if (err) err->assign(d.err(), d.err() + n);
            if (err_out) *err_out = err ? err->data() : nullptr;
            return UINT32_MAX;
        }
        d.assign(seg[k], seg[k + 1], heads);
        d.confirm(seg[k], seg[k + 1]);
    }
    return d.resolve(rep, nullptr);
}

namespace {
// memcpy whose body bypasses the CPU caches (16-byte non-temporal stores):
// page-locked staging written this way DMAs at the link's 57.4 GB/s, written
// with plain stores at 52.4 (the lines are still dirty in CPU caches when the
// copy engine reads them; profiles/r05o).  Head and tail are plain stores.
// The caller fences (_mm_sfence) before the DMA may start.
void stream_copy(uint8_t* dst, const uint8_t* src, uint64_t n) {
    uint64_t h = (16 - ((uintptr_t)dst & 15)) & 15;
    if (h > n) h = n;
    if (h) memcpy(dst, src, h);
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
    if (n) memcpy(dst, src, n);
}

// Gathers small pieces into a cache-resident window and streams the window
// out whole; pieces of a window's size or more stream directly.
struct StreamWriter {
    static constexpr uint64_t kWin = 16384;
    alignas(64) uint8_t win[kWin];
    uint8_t* at = nullptr;  // destination of win[0]
    uint64_t fill = 0;
    void flush() {
        if (fill) stream_copy(at, win, fill);
        fill = 0;
    }
    void put(uint8_t* d, const uint8_t* s, uint64_t n) {
        if (!n) return;
        if (fill && (d != at + fill || fill + n > kWin)) flush();
        if (n >= kWin) {
            stream_copy(d, s, n);
            return;
        }
        if (!fill) at = d;
        memcpy(win + fill, s, n);
        fill += n;
    }
    void done() {
        flush();
        _mm_sfence();
    }
};
}  // namespace

void pack(const uint8_t* const* ptr, const uint64_t* len, const uint32_t* first, const uint32_t* which,
          uint32_t m, const uint64_t* dst_off, uint8_t* dst, int threads, bool stream) {
    parallel_for(m, threads, [&](uint32_t lo, uint32_t hi) {
        if (stream) {
            StreamWriter w;
            for (uint32_t k = lo; k < hi; k++) {
                const uint32_t i = which ? which[k] : k;
                uint8_t* d = dst + dst_off[k];
                for (uint32_t s = first[i]; s < first[i + 1]; s++) {
                    w.put(d, ptr[s], len[s]);
                    d += len[s];
                }
            }
            w.done();
            return;
        }
        for (uint32_t k = lo; k < hi; k++) {
            const uint32_t i = which ? which[k] : k;
            uint8_t* d = dst + dst_off[k];
            for (uint32_t s = first[i]; s < first[i + 1]; s++) {
                if (len[s]) memcpy(d, ptr[s], len[s]);
                d += len[s];
            }
        }
    });
}

namespace {
// Sequential body of pack_range over [a, b).
void pack_range_seq(const uint8_t* const* ptr, const uint64_t* len, const uint32_t* first, uint32_t n,
                    const uint64_t* poff, uint64_t a, uint64_t b, uint8_t* dst, StreamWriter* w) {
    if (a >= b) return;
    // last request starting at or before a (poff nondecreasing)
    uint32_t i = (uint32_t)(std::upper_bound(poff, poff + n, a) - poff);
    i = i ? i - 1 : 0;
    for (; i < n && poff[i] < b; i++) {
        uint64_t p = poff[i];
        for (uint32_t sl = first[i]; sl < first[i + 1] && p < b; sl++) {
            const uint64_t L = len[sl];
            const uint64_t lo = std::max(p, a), hi = std::min(p + L, b);
            if (lo < hi) {
                if (w)
                    w->put(dst + (lo - a), ptr[sl] + (lo - p), hi - lo);
                else
                    memcpy(dst + (lo - a), ptr[sl] + (lo - p), hi - lo);
            }
            p += L;
        }
    }
}
}  // namespace

void pack_range(const uint8_t* base, const uint8_t* const* ptr, const uint64_t* len, const uint32_t* first,
                uint32_t n, const uint64_t* poff, uint64_t a, uint64_t b, uint8_t* dst, int threads, bool stream) {
    if (a >= b) return;
    const uint64_t total = b - a;
    if (threads < 1) threads = 1;
    const uint64_t piece = (total + threads - 1) / threads;
    parallel_for((uint32_t)threads, threads, [&](uint32_t lo, uint32_t hi) {
        for (uint32_t t = lo; t < hi; t++) {
            const uint64_t x = a + std::min<uint64_t>(total, piece * t), y = a + std::min<uint64_t>(total, piece * (t + 1));
            if (x >= y) continue;
            if (!ptr && !stream) {
                memcpy(dst + (x - a), base + x, y - x);
            } else if (!ptr) {
                stream_copy(dst + (x - a), base + x, y - x);
                _mm_sfence();
            } else if (!stream) {
                pack_range_seq(ptr, len, first, n, poff, x, y, dst + (x - a), nullptr);
            } else {
                StreamWriter w;
                pack_range_seq(ptr, len, first, n, poff, x, y, dst + (x - a), &w);
                w.done();
            }
        }
    });
}

}  // namespace host
}  // namespace mirsha

extern "C" int mirsha_dedup_plan(const uint8_t* const* slice_ptr, const uint64_t* slice_len,
                                 const uint32_t* slice_first, uint32_t n, uint32_t* rep_out,
                                 uint32_t* n_unique_out) {
    if (n == 0) {
        if (n_unique_out) *n_unique_out = 0;
        return MIRSHA_OK;
    }
    if (!slice_first || !rep_out || slice_first[0] != 0) return MIRSHA_EINVAL;
    if (slice_first[n] && (!slice_ptr || !slice_len)) return MIRSHA_EINVAL;
    const uint32_t u = mirsha::host::dedup_plan(slice_ptr, slice_len, slice_first, n, rep_out, nullptr, nullptr);
    if (u == UINT32_MAX) return MIRSHA_EINVAL;  // slice_first not monotone / a NULL slice with bytes
    if (n_unique_out) *n_unique_out = u;
    return MIRSHA_OK;
}
