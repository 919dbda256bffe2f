// processor.cpp — see processor.hpp.
#include "processor.hpp"

#include <algorithm>
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

namespace {
struct SliceLists {
    std::vector<const uint8_t*> ptr;
    std::vector<uint64_t> len;
    std::vector<uint32_t> first;
    explicit SliceLists(const std::vector<const HashRequest*>& reqs) : first(reqs.size() + 1, 0) {
        for (size_t i = 0; i < reqs.size(); i++) {
            for (const Bytes& b : reqs[i]->Data) {  // for _, data := range req.Data (processor.go:135)
                ptr.push_back(b.data);
                len.push_back(b.size);
            }
            first[i + 1] = (uint32_t)ptr.size();
        }
    }
};
}  // namespace

void GpuEngine::HashBatch(const std::vector<const HashRequest*>& reqs, std::vector<std::array<uint8_t, 32>>& out,
                          bool dedup, uint32_t* unique) {
    const uint32_t n = (uint32_t)reqs.size();
    out.resize(n);
    if (unique) *unique = n;
    if (n == 0) return;
    SliceLists sl(reqs);
    int rc = dedup ? mirsha_hash_slices_dedup(ctx_, sl.ptr.data(), sl.len.data(), sl.first.data(), n, out[0].data(),
                                              unique)
                   : mirsha_hash_slices(ctx_, sl.ptr.data(), sl.len.data(), sl.first.data(), n, out[0].data());
    if (rc != MIRSHA_OK) panic(ctx_, rc, "could not hash requests");
}

uint64_t GpuEngine::Submit(const std::vector<const HashRequest*>& reqs, std::vector<std::array<uint8_t, 32>>& out,
                           bool dedup) {
    const uint32_t n = (uint32_t)reqs.size();
    out.resize(std::max<uint32_t>(n, 1));
    SliceLists sl(reqs);
    uint64_t ticket = 0;
    int rc = mirsha_submit_slices(ctx_, sl.ptr.data(), sl.len.data(), sl.first.data(), n, out[0].data(),
                                  dedup ? MIRSHA_SUBMIT_DEDUP : 0, &ticket);
    if (rc != MIRSHA_OK) panic(ctx_, rc, "could not submit requests");
    out.resize(n);  // no reallocation: n <= capacity
    return ticket;
}

void GpuEngine::Wait(uint64_t ticket) {
    int rc = mirsha_wait(ctx_, ticket);
    if (rc != MIRSHA_OK) panic(ctx_, rc, "could not collect digests");
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

namespace {
ActionResults make_results(const std::vector<const HashRequest*>& reqs,
                           const std::vector<std::array<uint8_t, 32>>& digests) {
    ActionResults results;
    results.Digests.resize(reqs.size());
    for (size_t i = 0; i < reqs.size(); i++) {  // Digests[i] for actions.Hash[i] (processor.go:139)
        results.Digests[i].Request = reqs[i];
        results.Digests[i].Digest = digests[i];
    }
    return results;
}
}  // namespace

ActionResults Processor::Process(const Actions& actions) {
    std::vector<std::array<uint8_t, 32>> digests;
    engine_.HashBatch(actions.Hash, digests, dedup_);  // one device call per Ready() cycle
    return make_results(actions.Hash, digests);
}

PendingResults Processor::Submit(const Actions& actions) {
    PendingResults p;
    p.engine_ = &engine_;
    p.reqs_ = actions.Hash;
    p.digests_ = std::make_unique<std::vector<std::array<uint8_t, 32>>>();
    if (!p.reqs_.empty()) p.ticket_ = engine_.Submit(p.reqs_, *p.digests_, dedup_);
    return p;
}

PendingResults& PendingResults::operator=(PendingResults&& o) noexcept {
    if (this != &o) {
        if (ticket_) {  // overwriting an uncollected cycle: let it land first
            try { engine_->Wait(ticket_); } catch (...) {}
        }
        engine_ = o.engine_;
        ticket_ = o.ticket_;
        reqs_ = std::move(o.reqs_);
        digests_ = std::move(o.digests_);
        o.ticket_ = 0;
    }
    return *this;
}

PendingResults::~PendingResults() {
    if (ticket_) {
        try { engine_->Wait(ticket_); } catch (...) {}  // the buffer must outlive the library's write
    }
}

ActionResults PendingResults::Wait() {
    if (ticket_) {
        engine_->Wait(ticket_);
        ticket_ = 0;
    }
    return make_results(reqs_, *digests_);
}

}  // namespace mirbft

extern "C" int mirbft_host_process(int device, const uint8_t* const* data, const uint64_t* len, uint32_t n,
                                   uint8_t* digests_out, char* err, uint32_t err_len) {
    return mirbft_host_process_ex(device, data, len, n, digests_out, 0, nullptr, err, err_len);
}

extern "C" int mirbft_host_process_ex(int device, const uint8_t* const* data, const uint64_t* len, uint32_t n,
                                      uint8_t* digests_out, int flags, uint32_t* unique_out, char* err,
                                      uint32_t err_len) {
    try {
        mirbft::GpuEngine engine(device);
        mirbft::Processor p(engine, (flags & 1) != 0);
        std::vector<mirbft::HashRequest> reqs(n);
        mirbft::Actions a;
        for (uint32_t i = 0; i < n; i++) {
            reqs[i].Data.push_back(mirbft::Bytes{data[i], (size_t)len[i]});
            a.Hash.push_back(&reqs[i]);
        }
        mirbft::ActionResults r;
        if (flags & 4) {
            // A cycle dropped without Wait, then 4 more: the ring retires the
            // dropped one while later submissions are queued.
            { mirbft::PendingResults dropped = p.Submit(a); }
            std::vector<mirbft::PendingResults> more;
            for (int k = 0; k < 4; k++) more.push_back(p.Submit(a));
            for (auto& m : more) r = m.Wait();
        } else if (flags & 2) {
            mirbft::PendingResults pending = p.Submit(a);
            r = pending.Wait();
        } else {
            r = p.Process(a);
        }
        if (unique_out) {
            std::vector<std::array<uint8_t, 32>> tmp;
            *unique_out = n;
            if (flags & 1) engine.HashBatch(a.Hash, tmp, true, unique_out);
        }
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
