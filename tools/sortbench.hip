// Dev tool (not part of the library): rocPRIM radix sort of 100M (flow id, packet) pairs,
// the cost of a sort-based exact aggregator.  hipcc -O3 --offload-arch=gfx950 tools/sortbench.hip -o tools/sortbench.bin
#include <hip/hip_runtime.h>
#include <cstring>
#include <rocprim/rocprim.hpp>
#include <cstdio>
#include <cstdint>

__global__ void k_fill(uint32_t *k, uint64_t *v, uint32_t *v32, uint64_t n, uint32_t bits) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
        uint64_t x = i * 0x9E3779B97F4A7C15ull; x ^= x >> 29; x *= 0xBF58476D1CE4E5B9ull; x ^= x >> 32;
        // Zipf-ish: square a uniform to skew towards small ids
        const double u = (double)(x >> 11) * (1.0 / 9007199254740992.0);
        k[i] = (uint32_t)(u * u * (double)(1u << bits));
        v[i] = i << 32 | (64 + (x & 1023));
        v32[i] = (uint32_t)i;
    }
}

int main() {
    const uint64_t n = 100000000ull;
    const uint32_t bits = 22;
    uint32_t *k0, *k1, *v32a, *v32b; uint64_t *v0, *v1;
    hipMalloc(&k0, n * 4); hipMalloc(&k1, n * 4); hipMalloc(&v0, n * 8); hipMalloc(&v1, n * 8);
    hipMalloc(&v32a, n * 4); hipMalloc(&v32b, n * 4);
    hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, k0, v0, v32a, n, bits);
    size_t tb = 0, tb2 = 0;
    rocprim::radix_sort_pairs(nullptr, tb, k0, k1, v0, v1, n, 0, bits);
    rocprim::radix_sort_pairs(nullptr, tb2, k0, k1, v32a, v32b, n, 0, bits);
    if (tb2 > tb) tb = tb2;
    void *tmp; hipMalloc(&tmp, tb);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    for (int rep = 0; rep < 3; rep++) {
        float ms;
        hipEventRecord(a);
        rocprim::radix_sort_pairs(tmp, tb, k0, k1, v0, v1, n, 0, bits);
        hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
        printf("100M pairs u32 key (%u bits) + u64 value: %.3f ms\n", bits, ms);
        hipEventRecord(a);
        rocprim::radix_sort_pairs(tmp, tb, k0, k1, v32a, v32b, n, 0, bits);
        hipEventRecord(b); hipEventSynchronize(b); hipEventElapsedTime(&ms, a, b);
        printf("100M pairs u32 key (%u bits) + u32 value: %.3f ms\n", bits, ms);
        fflush(stdout);
    }
    return 0;
}
