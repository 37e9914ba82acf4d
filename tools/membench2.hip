// K1 floor study (dev tool, not part of the library): 100M 64-B records read
// per lane + 20 B/packet of writes, plus a dependent dictionary probe whose
// slot follows a Zipf(1.1) flow stream over 2^20 flows (like the bench), for
// record widths 64 / 32 / 16 B, with and without the 4-row MurmurHash3 chains
// over a 37-B key.  Build: hipcc -O3 --offload-arch=gfx950 tools/membench2.hip -o /tmp/membench2
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <vector>

constexpr uint64_t N = 100000000ull;
constexpr uint32_t NFLOWS = 1u << 20;

__device__ __forceinline__ uint32_t rotl(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ __forceinline__ uint32_t mm3_10(const uint32_t *k, uint32_t seed) {
    uint32_t h = seed;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        uint32_t x = k[i] * 0xcc9e2d51u;
        x = rotl(x, 15) * 0x1b873593u;
        h ^= x;
        h = rotl(h, 13) * 5u + 0xe6546b64u;
    }
    uint32_t x = (k[9] & 0xFFu) * 0xcc9e2d51u;
    x = rotl(x, 15) * 0x1b873593u;
    h ^= x;
    h ^= 37u;
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    return h;
}

// RW = record words read per probe (16, 8, 4); HASH = compute 4 row hashes of a 37-B key
template <int RW, int HASH>
__global__ __launch_bounds__(256) void k_probe(const uint4 *hdr, const uint32_t *sz, const uint32_t *slots,
                                               uint32_t *keyid, uint32_t *idx, const uint4 *tab, int probe) {
    for (uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x; p < N; p += (uint64_t)gridDim.x * 256) {
        uint4 v[4];
#pragma unroll
        for (int i = 0; i < 4; i++) v[i] = hdr[p * 4 + i];
        uint32_t h = sz[p];
#pragma unroll
        for (int i = 0; i < 4; i++) h ^= v[i].x + v[i].y * 3u + v[i].z * 5u + v[i].w * 7u;
        const uint32_t slot = slots[p];
        uint32_t kw[10] = {v[1].z, v[1].w, v[2].x, v[2].y, v[2].z, v[2].w, v[3].x, v[3].y, v[0].x, v[0].y};
        uint32_t acc = 0;
        if (probe) {
            uint4 r[RW / 4];
#pragma unroll
            for (int i = 0; i < RW / 4; i++) r[i] = tab[(uint64_t)slot * (RW / 4) + i];
#pragma unroll
            for (int i = 0; i < RW / 4; i++) acc ^= r[i].x ^ r[i].y ^ r[i].z ^ r[i].w;
        }
        keyid[p] = slot ^ acc;
#pragma unroll
        for (int rr = 0; rr < 4; rr++) {
            uint32_t b = acc + rr + h;
            if (HASH) b = mm3_10(kw, 0x1234567u * (rr + 1)) ^ acc;
            idx[rr * N + p] = b & 0xFFFFF;
        }
    }
}

int main() {
    // Zipf(1.1) ranks -> slots (host inverse CDF)
    std::vector<double> cdf(NFLOWS);
    double s = 0;
    for (uint32_t i = 0; i < NFLOWS; i++) { s += std::pow((double)(i + 1), -1.1); cdf[i] = s; }
    std::vector<uint32_t> hs(N);
    uint64_t x = 0x5EED0002ull;
    for (uint64_t p = 0; p < N; p++) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        const double u = (double)(x >> 11) * 0x1.0p-53 * s;
        uint32_t lo = 0, hi = NFLOWS - 1;
        while (lo < hi) { uint32_t m = (lo + hi) / 2; if (cdf[m] < u) lo = m + 1; else hi = m; }
        uint32_t r = lo * 0x9E3779B1u; r ^= r >> 15; r *= 0x2C1B3C6Du; r ^= r >> 12;
        hs[p] = r;
    }
    uint4 *hdr, *tab; uint32_t *sz, *keyid, *idx, *slots;
    hipMalloc(&hdr, N * 64); hipMalloc(&sz, N * 4); hipMalloc(&keyid, N * 4); hipMalloc(&idx, N * 16);
    hipMalloc(&slots, N * 4);
    hipMalloc(&tab, 256ull << 20);
    hipMemset(hdr, 1, N * 64); hipMemset(sz, 2, N * 4); hipMemset(tab, 3, 256ull << 20);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    const unsigned grid = (unsigned)(N / 256);
    struct V { const char *name; int rw, hash, probe; uint32_t slots_log2; };
    const V vs[] = {{"stream only", 16, 0, 0, 22},          {"probe 64B, 4M slots", 16, 0, 1, 22},
                    {"probe 64B, 2M slots", 16, 0, 1, 21},  {"probe 32B, 4M slots", 8, 0, 1, 22},
                    {"probe 16B, 4M slots", 4, 0, 1, 22},   {"probe 16B, 2M slots", 4, 0, 1, 21},
                    {"stream + hash", 16, 1, 0, 22},        {"probe 16B 4M + hash", 4, 1, 1, 22},
                    {"probe 64B 4M + hash", 16, 1, 1, 22}};
    for (const V &v : vs) {
        std::vector<uint32_t> sl(N);
        const uint32_t mask = (1u << v.slots_log2) - 1u;
        for (uint64_t p = 0; p < N; p++) sl[p] = hs[p] & mask;
        hipMemcpy(slots, sl.data(), N * 4, hipMemcpyHostToDevice);
        float best = 1e9f;
        for (int rep = 0; rep < 4; rep++) {
            hipEventRecord(a);
            if (v.rw == 16 && !v.hash) hipLaunchKernelGGL((k_probe<16, 0>), dim3(grid), dim3(256), 0, 0, hdr, sz, slots, keyid, idx, tab, v.probe);
            if (v.rw == 16 && v.hash) hipLaunchKernelGGL((k_probe<16, 1>), dim3(grid), dim3(256), 0, 0, hdr, sz, slots, keyid, idx, tab, v.probe);
            if (v.rw == 8) hipLaunchKernelGGL((k_probe<8, 0>), dim3(grid), dim3(256), 0, 0, hdr, sz, slots, keyid, idx, tab, v.probe);
            if (v.rw == 4 && !v.hash) hipLaunchKernelGGL((k_probe<4, 0>), dim3(grid), dim3(256), 0, 0, hdr, sz, slots, keyid, idx, tab, v.probe);
            if (v.rw == 4 && v.hash) hipLaunchKernelGGL((k_probe<4, 1>), dim3(grid), dim3(256), 0, 0, hdr, sz, slots, keyid, idx, tab, v.probe);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
        }
        printf("%-26s %.3f ms\n", v.name, best);
        fflush(stdout);
    }
    return 0;
}
