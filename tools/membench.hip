// Streaming micro-benchmark for the K1 access pattern (dev tool, not part of the
// library): 100M 64-byte records read per lane (4 x 16 B per lane, lanes 64 B
// apart) vs fully coalesced 1-KB instructions, with K1's 4 + 4*d bytes of
// per-packet writes.  Build: hipcc -O3 --offload-arch=gfx950 tools/membench.hip -o /tmp/membench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr uint64_t N = 100000000ull;

__global__ __launch_bounds__(256) void k_lane_records(const uint4 *hdr, const uint32_t *sz, uint32_t *out,
                                                      uint32_t *idx, int writes) {
    for (uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x; p < N; p += (uint64_t)gridDim.x * 256) {
        uint4 v[4];
#pragma unroll
        for (int i = 0; i < 4; i++) v[i] = hdr[p * 4 + i];
        uint32_t h = sz[p];
#pragma unroll
        for (int i = 0; i < 4; i++) h ^= v[i].x + v[i].y * 3u + v[i].z * 5u + v[i].w * 7u;
        out[p] = h;
        if (writes)
#pragma unroll
            for (int r = 0; r < 4; r++) idx[r * N + p] = h + r;
    }
}

__global__ __launch_bounds__(256) void k_coalesced(const uint4 *hdr, const uint32_t *sz, uint32_t *out,
                                                   uint32_t *idx, int writes) {
    // each wave reads its 64 records as 4 contiguous 1-KB instructions
    const uint32_t lane = threadIdx.x & 63u;
    for (uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x; p < N; p += (uint64_t)gridDim.x * 256) {
        const uint64_t w0 = p - lane;
        uint4 v[4];
#pragma unroll
        for (int i = 0; i < 4; i++) v[i] = hdr[w0 * 4 + (uint64_t)i * 64 + lane];
        uint32_t h = sz[p];
#pragma unroll
        for (int i = 0; i < 4; i++) h ^= v[i].x + v[i].y * 3u + v[i].z * 5u + v[i].w * 7u;
        out[p] = h;
        if (writes)
#pragma unroll
            for (int r = 0; r < 4; r++) idx[r * N + p] = h + r;
    }
}

// + a dependent random 64-B record read per packet (dictionary-probe-like) from a table of tabn records
__global__ __launch_bounds__(256) void k_lane_records_dict(const uint4 *hdr, const uint32_t *sz, uint32_t *out,
                                                           uint32_t *idx, const uint4 *tab, uint32_t tabmask,
                                                           int zipf) {
    for (uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x; p < N; p += (uint64_t)gridDim.x * 256) {
        uint4 v[4];
#pragma unroll
        for (int i = 0; i < 4; i++) v[i] = hdr[p * 4 + i];
        uint32_t h = sz[p];
#pragma unroll
        for (int i = 0; i < 4; i++) h ^= v[i].x + v[i].y * 3u + v[i].z * 5u + v[i].w * 7u;
        uint32_t x = (uint32_t)p * 0x9E3779B1u ^ h;
        x ^= x >> 15; x *= 0x2C1B3C6Du; x ^= x >> 12;
        // zipf-ish: a quarter of the packets hit a small hot set
        const uint32_t slot = (zipf && (x & 3u) != 0) ? (x >> 2) & 4095u : x & tabmask;
        uint4 r[4];
#pragma unroll
        for (int i = 0; i < 4; i++) r[i] = tab[(uint64_t)slot * 4 + i];
        h ^= r[0].x ^ r[1].y ^ r[2].z ^ r[3].w;
        out[p] = h;
#pragma unroll
        for (int rr = 0; rr < 4; rr++) idx[rr * N + p] = h + rr;
    }
}

int main() {
    uint4 *hdr; uint32_t *sz, *out, *idx;
    hipMalloc(&hdr, N * 64); hipMalloc(&sz, N * 4); hipMalloc(&out, N * 4); hipMalloc(&idx, N * 16);
    hipMemset(hdr, 1, N * 64); hipMemset(sz, 2, N * 4);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    const int grids[] = {2048, 8192, (int)(N / 256)};
    for (int g : grids)
        for (int kind = 0; kind < 2; kind++)
            for (int wr = 0; wr < 2; wr++) {
                float best = 1e9f;
                for (int rep = 0; rep < 5; rep++) {
                    hipEventRecord(a);
                    if (kind == 0) hipLaunchKernelGGL(k_lane_records, dim3(g), dim3(256), 0, 0, hdr, sz, out, idx, wr);
                    else hipLaunchKernelGGL(k_coalesced, dim3(g), dim3(256), 0, 0, hdr, sz, out, idx, wr);
                    hipEventRecord(b); hipEventSynchronize(b);
                    float ms; hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
                }
                const double bytes = N * (68.0 + 4.0 + (wr ? 16.0 : 0.0));
                printf("grid %7d %-10s writes %-3s %.3f ms  %.2f TB/s\n", g, kind ? "coalesced" : "per-lane",
                       wr ? "4+16" : "4", best, bytes / best / 1e9);
            }
    uint4 *tab;
    const uint64_t tabn = 1ull << 22;  // 4M records x 64 B = 256 MB, like the bench dictionary
    hipMalloc(&tab, tabn * 64);
    hipMemset(tab, 3, tabn * 64);
    for (int zipf = 0; zipf < 2; zipf++) {
        float best = 1e9f;
        for (int rep = 0; rep < 5; rep++) {
            hipEventRecord(a);
            hipLaunchKernelGGL(k_lane_records_dict, dim3((unsigned)(N / 256)), dim3(256), 0, 0, hdr, sz, out, idx, tab,
                               (uint32_t)(tabn - 1), zipf);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
        }
        printf("per-lane + 4+16 writes + random 64-B probe (%s): %.3f ms\n", zipf ? "3/4 in a 4K hot set" : "uniform over 256 MB", best);
    }
    return 0;
}
