// host_unit.cpp -- CPU unit test of the library's host-side helpers
// (mirbft_amd/csrc/mirsha_host.cpp, compiled here with g++: no HIP, no GPU):
// the parallel exclusive scan behind slice-call offsets, slice packing into a
// staging arena (whole and by byte range, as the pinned ring fills chunk by
// chunk), parallel_for coverage, and per-(slot, threads) packing pools.
// Prints "host unit ok"; exit 1 with a message at the first mismatch.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "mirsha_host.h"

using namespace mirsha::host;

static int fails = 0;
#define EXPECT(cond, ...)                         \
    do {                                          \
        if (!(cond)) {                            \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);         \
            fprintf(stderr, "\n");                \
            fails++;                              \
        }                                         \
    } while (0)

static void test_scan(std::mt19937_64& rng) {
    for (uint32_t n : {0u, 1u, 7u, 65535u, 65536u, 1000003u, 1u << 21}) {
        std::vector<uint32_t> len(n);
        for (auto& x : len) x = (uint32_t)(rng() % 70000);
        std::vector<uint64_t> out(n, ~0ull);
        const uint64_t total = exclusive_scan(len.data(), n, out.data());
        uint64_t p = 0;
        bool ok = true;
        for (uint32_t i = 0; i < n; i++) {
            ok &= out[i] == p;
            p += len[i];
        }
        EXPECT(ok, "exclusive_scan offsets differ at n=%u", n);
        EXPECT(total == p, "exclusive_scan total %llu != %llu at n=%u", (unsigned long long)total,
               (unsigned long long)p, n);
    }
}

static void test_parallel_for() {
    for (uint32_t n : {1u, 2u, 17u, 1000u, 123457u})
        for (int t : {1, 2, 3, 8, 16}) {
            std::vector<int> hit(n, 0);
            parallel_for(n, t, [&](uint32_t a, uint32_t b) {
                for (uint32_t i = a; i < b; i++) hit[i]++;
            });
            bool ok = true;
            for (int h : hit) ok &= h == 1;
            EXPECT(ok, "parallel_for n=%u threads=%d did not cover every index once", n, t);
        }
}

// Requests of 0-3 slices (empty slices and empty requests included) over one
// random buffer; the packed arena is the concatenation in request order.
static void test_pack(std::mt19937_64& rng) {
    const uint32_t n = 5000;
    std::vector<uint8_t> buf(1 << 20);
    for (auto& b : buf) b = (uint8_t)rng();
    std::vector<const uint8_t*> ptr;
    std::vector<uint64_t> len;
    std::vector<uint32_t> first{0};
    std::vector<uint8_t> want;
    std::vector<uint64_t> poff(n), rlen(n);
    for (uint32_t i = 0; i < n; i++) {
        poff[i] = want.size();
        const int k = (int)(rng() % 4);
        for (int s = 0; s < k; s++) {
            const uint64_t l = (rng() % 5 == 0) ? 0 : (rng() % 60 == 0) ? rng() % 40000 : rng() % 700;
            const uint64_t o = rng() % (buf.size() - l);
            ptr.push_back(buf.data() + o);
            len.push_back(l);
            want.insert(want.end(), buf.begin() + (long)o, buf.begin() + (long)(o + l));
        }
        first.push_back((uint32_t)ptr.size());
        rlen[i] = want.size() - poff[i];
    }
    const uint64_t total = want.size();
    for (int t : {1, 4, 16})
        for (bool stream : {false, true}) {
            std::vector<uint8_t> got(total, 0xAA);
            pack(ptr.data(), len.data(), first.data(), nullptr, n, poff.data(), got.data(), t, stream);
            EXPECT(got == want, "pack with %d threads (stream %d)", t, (int)stream);
        }
    // a subset in another order, packed densely
    std::vector<uint32_t> which;
    for (uint32_t i = 0; i < n; i += 3) which.push_back(n - 1 - i);
    std::vector<uint64_t> woff(which.size());
    uint64_t p = 0;
    std::vector<uint8_t> wwant;
    for (size_t k = 0; k < which.size(); k++) {
        woff[k] = p;
        p += rlen[which[k]];
        wwant.insert(wwant.end(), want.begin() + (long)poff[which[k]], want.begin() + (long)(poff[which[k]] + rlen[which[k]]));
    }
    for (bool stream : {false, true}) {
        std::vector<uint8_t> wgot(p, 0);
        pack(ptr.data(), len.data(), first.data(), which.data(), (uint32_t)which.size(), woff.data(), wgot.data(), 8,
             stream);
        EXPECT(wgot == wwant, "pack of a reordered subset (stream %d)", (int)stream);
    }
    // destinations with gaps and out of order (the streaming writer flushes
    // its window at every discontinuity); bytes between them stay untouched
    {
        std::vector<uint64_t> goff(which.size());
        uint64_t q = 0;
        for (size_t k = which.size(); k-- > 0;) {  // later requests at lower addresses
            q += (k * 7) % 29;                       // a gap of 0..28 bytes
            goff[k] = q;
            q += rlen[which[k]];
        }
        std::vector<uint8_t> gwant(q, 0x77);
        for (size_t k = 0; k < which.size(); k++)
            std::copy(want.begin() + (long)poff[which[k]], want.begin() + (long)(poff[which[k]] + rlen[which[k]]),
                      gwant.begin() + (long)goff[k]);
        for (bool stream : {false, true}) {
            std::vector<uint8_t> ggot(q, 0x77);
            pack(ptr.data(), len.data(), first.data(), which.data(), (uint32_t)which.size(), goff.data(), ggot.data(),
                 5, stream);
            EXPECT(ggot == gwant, "pack to gapped, reversed destinations (stream %d)", (int)stream);
        }
    }
    // byte ranges [a, b) of the packed arena (the pinned ring's chunks), cut anywhere
    // (stream: non-temporal stores, destinations at every alignment)
    for (int rep = 0; rep < 100; rep++) {
        const bool stream = rep & 1;
        uint64_t a = rng() % (total + 1), b = rng() % (total + 1);
        if (a > b) std::swap(a, b);
        const uint64_t skew = rng() % 16;
        std::vector<uint8_t> buf_got(b - a + 1 + skew, 0x55);
        uint8_t* got = buf_got.data() + skew;
        pack_range(nullptr, ptr.data(), len.data(), first.data(), n, poff.data(), a, b, got, 1 + (int)(rng() % 16),
                   stream);
        EXPECT(std::equal(got, got + (b - a), want.begin() + (long)a), "pack_range [%llu, %llu) stream %d",
               (unsigned long long)a, (unsigned long long)b, (int)stream);
        EXPECT(got[b - a] == 0x55, "pack_range wrote past its end");
        std::vector<uint8_t> buf_flat(b - a + 1 + skew, 0x55);
        uint8_t* flat = buf_flat.data() + skew;
        pack_range(want.data(), nullptr, nullptr, nullptr, 0, nullptr, a, b, flat, 1 + (int)(rng() % 16), stream);
        EXPECT(std::equal(flat, flat + (b - a), want.begin() + (long)a), "pack_range from a contiguous base (stream %d)",
               (int)stream);
        EXPECT(flat[b - a] == 0x55, "pack_range (contiguous) wrote past its end");
    }
}

// A thread may select a pool slot with a thread count; a later selection of
// the same slot with a different count must get a pool of that size
// (threads_for is capped at the selected pool's size).
static void test_pools() {
    for (int threads : {2, 4, 3, 4}) {
        std::thread th([&] {
            use_pool(5, threads);
            EXPECT(threads_for(1ull << 40, 1u << 30) == threads, "threads_for with a %d-thread pool", threads);
            std::vector<int> hit(100000, 0);
            parallel_for(100000, threads, [&](uint32_t a, uint32_t b) {
                for (uint32_t i = a; i < b; i++) hit[i]++;
            });
            bool ok = true;
            for (int h : hit) ok &= h == 1;
            EXPECT(ok, "parallel_for on slot 5 with %d threads", threads);
        });
        th.join();
    }
}

int main() {
    std::mt19937_64 rng(20261018);
    test_scan(rng);
    test_parallel_for();
    test_pack(rng);
    test_pools();
    if (fails) {
        fprintf(stderr, "%d failure(s)\n", fails);
        return 1;
    }
    printf("host unit ok\n");
    return 0;
}
