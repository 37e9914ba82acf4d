// Probe (dev tool, not part of the library): do returning LDS atomic adds from
// the lanes of ONE wave instruction that hit the same address come back in
// lane order?  Counts pairs of lanes l1 < l2 with equal address whose returned
// old values are out of order, over many random address patterns.
// Build: hipcc -O3 --offload-arch=gfx950 tools/lds_order.hip -o lds_order
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ __launch_bounds__(256) void k(unsigned long long *viol, unsigned long long *pairs, int iters, int nad) {
    __shared__ uint32_t s[4][64];
    __shared__ uint32_t s_old[4][64], s_ad[4][64];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    uint32_t x = (blockIdx.x * 256 + threadIdx.x) * 0x9E3779B1u + 12345u;
    unsigned long long v = 0, pr = 0;
    for (int it = 0; it < iters; it++) {
        s[w][lane] = 0;
        x = x * 1664525u + 1013904223u;
        const uint32_t ad = (x >> 16) % (uint32_t)nad;
        const uint32_t add = 1u + ((x >> 8) & 7u);
        const uint32_t old = atomicAdd(&s[w][ad], add);
        s_old[w][lane] = old;
        s_ad[w][lane] = ad;
        for (uint32_t j = 0; j < lane; j++) {
            if (s_ad[w][j] == ad) {
                pr++;
                if (s_old[w][j] >= old) v++;
            }
        }
    }
    atomicAdd(viol, v);
    atomicAdd(pairs, pr);
}

int main() {
    unsigned long long *d;
    hipMalloc(&d, 16);
    const int nads[] = {1, 2, 4, 8, 32, 64};
    for (int nad : nads) {
        hipMemset(d, 0, 16);
        hipLaunchKernelGGL(k, dim3(4096), dim3(256), 0, 0, d, d + 1, 200, nad);
        unsigned long long h[2];
        hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
        printf("addresses %2d: same-address lane pairs %llu, out of lane order %llu\n", nad, h[1], h[0]);
    }
    return 0;
}
