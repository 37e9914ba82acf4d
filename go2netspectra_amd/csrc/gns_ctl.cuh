// gns_ctl.cuh -- a batch's small control words in one launch each.
//
// Each engine batch zeroes a handful of device counters before its first kernel
// and, between dictionary resolve rounds, reads a few of them back to the host.
// As separate hipMemsetAsync / hipMemcpyAsync operations each costs its own
// runtime operation on the stream (about 5 us apiece here, in front of the
// batch and inside its one host round trip); one tiny kernel does all of them.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace gns {
namespace {

constexpr int kCtlMax = 16;

// word ranges to zero: p[i][0 .. n[i])
struct CtlZero {
    uint32_t *p[kCtlMax];
    uint32_t n[kCtlMax];
    int k = 0;
    void add(void *ptr, size_t bytes) { p[k] = static_cast<uint32_t *>(ptr); n[k] = (uint32_t)(bytes / 4); k++; }
};

__global__ __launch_bounds__(256) void k_ctl_zero(CtlZero z) {
    for (int i = 0; i < z.k; i++)
        for (uint32_t j = threadIdx.x; j < z.n[i]; j += 256) z.p[i][j] = 0u;
}

// words to read: dst[i] = *src[i] (dst: pinned host memory, written with vector stores)
struct CtlRead {
    const uint32_t *src[kCtlMax];
    uint32_t at[kCtlMax];  // destination word index
    int k = 0;
    void add(const void *ptr, size_t bytes, uint32_t word) {
        for (uint32_t w = 0; w < bytes / 4; w++) {
            src[k] = static_cast<const uint32_t *>(ptr) + w;
            at[k] = word + w;
            k++;
        }
    }
};

__global__ __launch_bounds__(64) void k_ctl_read(CtlRead r, uint32_t *dst) {
    const int i = (int)threadIdx.x;
    if (i < r.k) dst[r.at[i]] = *r.src[i];
}

inline hipError_t ctl_zero(const CtlZero &z, hipStream_t s) {
    hipLaunchKernelGGL(k_ctl_zero, dim3(1), dim3(256), 0, s, z);
    return hipGetLastError();
}

inline hipError_t ctl_read(const CtlRead &r, uint32_t *dst_pinned, hipStream_t s) {
    hipLaunchKernelGGL(k_ctl_read, dim3(1), dim3(64), 0, s, r, dst_pinned);
    return hipGetLastError();
}

}  // namespace
}  // namespace gns
