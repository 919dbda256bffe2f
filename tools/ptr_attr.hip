// ptr_attr.hip -- probe: what hipPointerGetAttributes reports for the
// library's page-locked allocations (mirsha_host_alloc, mirsha_multi_host_alloc)
// and an interior pointer of each: kernel_writable_host (mirsha_ctx.h)
// decides from `device` and `allocationFlags` whether a kernel may store
// digests there.
//   hipcc --offload-arch=gfx950 -O2 -I include -o tools/ptr_attr tools/ptr_attr.hip -L mirbft_amd/lib -lmirsha -Wl,-rpath,$PWD/mirbft_amd/lib
#include <hip/hip_runtime.h>

#include <cstdio>

#include "mirsha.h"

static void show(const char* what, const void* p) {
    hipPointerAttribute_t a;
    const hipError_t e = hipPointerGetAttributes(&a, p);
    printf("{\"what\": \"%s\", \"rc\": %d, \"type\": %d, \"device\": %d, \"flags\": %u, \"portable\": %d}\n", what, (int)e,
           (int)a.type, a.device, a.allocationFlags, (a.allocationFlags & hipHostMallocPortable) ? 1 : 0);
}

int main() {
    mirsha_ctx* c = nullptr;
    if (mirsha_ctx_create(0, &c) != MIRSHA_OK) return 2;
    void* h = nullptr;
    if (mirsha_host_alloc(c, 1 << 20, &h) != MIRSHA_OK) return 3;
    show("mirsha_host_alloc", h);
    show("mirsha_host_alloc+4096", (char*)h + 4096);
    int devs[2] = {0, 0};
    mirsha_multi* m = nullptr;
    if (mirsha_multi_create(devs, 2, &m) != MIRSHA_OK) return 4;
    void* mh = nullptr;
    if (mirsha_multi_host_alloc(m, 1 << 20, &mh) != MIRSHA_OK) return 5;
    show("mirsha_multi_host_alloc", mh);
    show("mirsha_multi_host_alloc+4096", (char*)mh + 4096);
    mirsha_host_free(h);
    mirsha_host_free(mh);
    mirsha_multi_destroy(m);
    mirsha_ctx_destroy(c);
    return 0;
}
