// processor.cpp — see processor.hpp.
#include "processor.hpp"

#include <cstring>

#include "../../include/mirsha.h"

namespace mirbft {

namespace {
[[noreturn]] void panic(mirsha_ctx* c, int rc, const char* what) {
    // The reference panics on processor failures (processor.go:75, :85, :91).
    throw std::runtime_error(std::string(what) + ": mirsha error " + std::to_string(rc) + ": " +
                             (c ? mirsha_last_error(c) : ""));
}
}  // namespace

GpuEngine::GpuEngine(int device) {
    int rc = mirsha_ctx_create(device, &ctx_);
    if (rc != MIRSHA_OK) panic(nullptr, rc, "could not create gfx950 hash engine");
}

GpuEngine::~GpuEngine() { mirsha_ctx_destroy(ctx_); }

void GpuEngine::HashBatch(const std::vector<const HashRequest*>& reqs,
                          std::vector<std::array<uint8_t, 32>>& out) {
    const uint32_t n = (uint32_t)reqs.size();
    out.resize(n);
    if (n == 0) return;
    std::vector<const uint8_t*> ptr;
    std::vector<uint64_t> len;
    std::vector<uint32_t> first(n + 1, 0);
    for (uint32_t i = 0; i < n; i++) {
        for (const Bytes& b : reqs[i]->Data) {  // for _, data := range req.Data (processor.go:135)
            ptr.push_back(b.data);
            len.push_back(b.size);
        }
        first[i + 1] = (uint32_t)ptr.size();
    }
    int rc = mirsha_hash_slices(ctx_, ptr.data(), len.data(), first.data(), n, out[0].data());
    if (rc != MIRSHA_OK) panic(ctx_, rc, "could not hash requests");
}

namespace {
class GpuSha256 final : public Hash {
public:
    explicit GpuSha256(GpuEngine& e) : e_(e) {}
    void Write(const uint8_t* p, size_t n) override { buf_.insert(buf_.end(), p, p + n); }
    std::array<uint8_t, 32> Sum() const override {
        HashRequest r;
        r.Data.push_back(Bytes{buf_.data(), buf_.size()});
        std::vector<std::array<uint8_t, 32>> out;
        e_.HashBatch({&r}, out);
        return out[0];
    }
    void Reset() override { buf_.clear(); }

private:
    GpuEngine& e_;
    std::vector<uint8_t> buf_;
};
}  // namespace

std::unique_ptr<Hash> NewGpuSha256(GpuEngine& engine) { return std::make_unique<GpuSha256>(engine); }

ActionResults Processor::Process(const Actions& actions) {
    ActionResults results;
    std::vector<std::array<uint8_t, 32>> digests;
    engine_.HashBatch(actions.Hash, digests);  // one device call per Ready() cycle
    results.Digests.resize(actions.Hash.size());
    for (size_t i = 0; i < actions.Hash.size(); i++) {  // Digests[i] for actions.Hash[i] (processor.go:139)
        results.Digests[i].Request = actions.Hash[i];
        results.Digests[i].Digest = digests[i];
    }
    return results;
}

}  // namespace mirbft

extern "C" int mirbft_host_process(int device, const uint8_t* const* data, const uint64_t* len, uint32_t n,
                                   uint8_t* digests_out, char* err, uint32_t err_len) {
    try {
        mirbft::GpuEngine engine(device);
        mirbft::Processor p(engine);
        std::vector<mirbft::HashRequest> reqs(n);
        mirbft::Actions a;
        for (uint32_t i = 0; i < n; i++) {
            reqs[i].Data.push_back(mirbft::Bytes{data[i], (size_t)len[i]});
            a.Hash.push_back(&reqs[i]);
        }
        mirbft::ActionResults r = p.Process(a);
        for (uint32_t i = 0; i < n; i++) {
            if (r.Digests[i].Request != &reqs[i]) throw std::runtime_error("origin order violated");
            memcpy(digests_out + 32ull * i, r.Digests[i].Digest.data(), 32);
        }
        return 0;
    } catch (const std::exception& e) {
        if (err && err_len) {
            strncpy(err, e.what(), err_len - 1);
            err[err_len - 1] = 0;
        }
        return -1;
    }
}
