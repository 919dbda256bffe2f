// processor.hpp — C++ host mirror of the reference's Processor hash path
// (Go package github.com/IBM/mirbft; no Go toolchain in this image, so the
// host side above the C-ABI is C++, with the reference's names and semantics).
//
//   reference                                   here
//   type Hasher func() hash.Hash  processor.go:21     mirbft::Hasher (factory of mirbft::Hash)
//   HashRequest{Data [][]byte; Origin}  actions.go:157-164   mirbft::HashRequest
//   HashResult{Digest; Request}         actions.go:224-230   mirbft::HashResult
//   ActionResults{Digests; ...}         actions.go:218-221   mirbft::ActionResults
//   (*Processor).Process hash loop      processor.go:129-143 mirbft::Processor::Process
//
// Processor::Process coalesces every HashRequest of one Ready() cycle into ONE
// batched device call (mirsha_hash_slices) and returns Digests[i] for
// actions.Hash[i] with the Request back-pointer, in origin order.  Failures
// throw std::runtime_error — the reference panics (processor.go:75,81,85,91).
// Options: dedup (hash each distinct request content once per cycle,
// mirsha_hash_slices_dedup) and the asynchronous Submit / Pending::Wait form
// (mirsha_submit_slices / mirsha_wait) for overlapping the cycle's hashing
// with its WAL writes and sends, as ProcessorWorkPool does (processor.go:447-470).
#pragma once
#include <array>
#include <cstdint>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

struct mirsha_ctx;

namespace mirbft {

struct Bytes {
    const uint8_t* data = nullptr;
    size_t size = 0;
};

// Origin is opaque to the hasher (actions.go:152-156): carried, never read.
struct HashRequest {
    std::vector<Bytes> Data;
    const void* Origin = nullptr;
};

struct HashResult {
    std::array<uint8_t, 32> Digest{};
    const HashRequest* Request = nullptr;
};

struct Actions {
    std::vector<const HashRequest*> Hash;  // actions.go:24
};

struct ActionResults {
    std::vector<HashResult> Digests;  // actions.go:219
};

// Streaming hash.Hash (Write/Sum/Reset) for single-message callers.
class Hash {
public:
    virtual ~Hash() = default;
    virtual void Write(const uint8_t* p, size_t n) = 0;
    virtual std::array<uint8_t, 32> Sum() const = 0;
    virtual void Reset() = 0;
};
using Hasher = std::function<std::unique_ptr<Hash>()>;

// One gfx950 engine (device context); the batched replacement for Hasher.
class GpuEngine {
public:
    explicit GpuEngine(int device = 0);
    ~GpuEngine();
    GpuEngine(const GpuEngine&) = delete;
    GpuEngine& operator=(const GpuEngine&) = delete;

    // Digests of reqs[i] (concat of its Data slices) at out[i], origin order.
    // dedup: identical requests are hashed once; *unique = distinct requests.
    void HashBatch(const std::vector<const HashRequest*>& reqs, std::vector<std::array<uint8_t, 32>>& out,
                   bool dedup = false, uint32_t* unique = nullptr);
    // Asynchronous form: packs reqs before returning; `out` (resized here) is
    // filled, in origin order, by Wait(ticket).
    uint64_t Submit(const std::vector<const HashRequest*>& reqs, std::vector<std::array<uint8_t, 32>>& out,
                    bool dedup = false);
    void Wait(uint64_t ticket);
    mirsha_ctx* ctx() { return ctx_; }

private:
    mirsha_ctx* ctx_ = nullptr;
};

// hash.Hash whose Sum runs on the GPU (buffers its writes).
std::unique_ptr<Hash> NewGpuSha256(GpuEngine& engine);

// One submitted cycle; Wait() returns its ActionResults (origin order).
// Owns the buffer the library writes the digests into (inside mirsha_wait, or
// when a later submission retires this one's ring slot), so it is move-only
// and its destructor waits for a cycle that was never collected.
class PendingResults {
public:
    PendingResults() = default;
    PendingResults(PendingResults&& o) noexcept { *this = std::move(o); }
    PendingResults& operator=(PendingResults&& o) noexcept;
    PendingResults(const PendingResults&) = delete;
    PendingResults& operator=(const PendingResults&) = delete;
    ~PendingResults();
    ActionResults Wait();

private:
    friend class Processor;
    GpuEngine* engine_ = nullptr;
    uint64_t ticket_ = 0;
    std::vector<const HashRequest*> reqs_;
    std::unique_ptr<std::vector<std::array<uint8_t, 32>>> digests_;
};

class Processor {
public:
    explicit Processor(GpuEngine& engine, bool dedup = false) : engine_(engine), dedup_(dedup) {}
    // processor.go:129-143, batched.
    ActionResults Process(const Actions& actions);
    // Asynchronous Process: queue the cycle's hashing and return at once.
    PendingResults Submit(const Actions& actions);

private:
    GpuEngine& engine_;
    bool dedup_;
};

}  // namespace mirbft

extern "C" {
// Small C entry for tests: hash n single-slice requests through
// mirbft::Processor (exercises the C++ mirror end to end).
int mirbft_host_process(int device, const uint8_t* const* data, const uint64_t* len, uint32_t n,
                        uint8_t* digests_out, char* err, uint32_t err_len);
// flags: bit 0 = dedup, bit 1 = asynchronous (Submit, then Wait), bit 2 =
// asynchronous with a dropped (never waited) cycle before four more.
int mirbft_host_process_ex(int device, const uint8_t* const* data, const uint64_t* len, uint32_t n,
                           uint8_t* digests_out, int flags, uint32_t* unique_out, char* err, uint32_t err_len);
}
