// mirsha_scan.hip — request offsets from request lengths on the device.
//
// A large synchronous call whose requests are packed back to back (every
// slice-list call, every gapless caller arena) has off[i] = len[0] + ... +
// len[i-1]: the pipelined host path then ships only the lengths and this
// exclusive scan (rocPRIM's decoupled look-back scan, one pass over 4 B per
// request) rebuilds the 8-byte offsets in HBM, instead of 8 MB more over PCIe
// per 2^20 requests.
#include <hip/hip_runtime.h>

#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

#include "mirsha_kernels.h"

namespace mirsha {

namespace {
struct Widen {
    __host__ __device__ uint64_t operator()(uint32_t x) const { return x; }
};
}  // namespace

hipError_t launch_offsets_scan(void* tmp, size_t& tmp_bytes, const uint32_t* len, uint64_t* off, uint32_t n,
                               hipStream_t s) {
    auto in = rocprim::make_transform_iterator(len, Widen());
    return rocprim::exclusive_scan(tmp, tmp_bytes, in, off, uint64_t(0), (size_t)n, rocprim::plus<uint64_t>(), s);
}

}  // namespace mirsha
