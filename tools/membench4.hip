// K1 record-load shape study (dev tool, not part of the library): the K1 streams
// (100M 64-B records + 4-B sizes read, 20 B/packet written) with the record read
// (a) per lane (lane i loads record i with four 16-B loads: every wave-instruction
//     touches 64 records at a 64-B stride), as K1 does, or
// (b) coalesced (wave-instruction j loads bytes [1 KiB * j, 1 KiB * (j + 1)) of the
//     wave's 4 KiB) and transposed through LDS so that lane i again holds record i.
// Build: hipcc -O3 --offload-arch=gfx950 tools/membench4.hip -o /tmp/membench4
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

constexpr uint64_t N = 100000000ull;  // multiple of 64

__device__ __forceinline__ uint32_t mix(const uint4 (&v)[4], uint32_t s) {
    uint32_t h = s;
#pragma unroll
    for (int i = 0; i < 4; i++) h ^= v[i].x + v[i].y * 3u + v[i].z * 5u + v[i].w * 7u;
    return h;
}

template <int COAL, int ITEMS>
__global__ __launch_bounds__(256) void k_stream(const uint4 *hdr, const uint32_t *sz, uint32_t *keyid, uint32_t *idx) {
    __shared__ uint4 st[4][64 * 4];  // per wave: 64 records of 4 uint4
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    for (int it = 0; it < ITEMS; it++) {
        const uint64_t wbase = ((uint64_t)blockIdx.x * ITEMS + it) * 256 + wave * 64;  // first packet of the wave
        const uint64_t p = wbase + lane;
        uint4 v[4];
        if (COAL == 2) {
            // coalesced loads, then a 4x4 transpose inside each quad with DPP moves (no
            // LDS): lane 4m+i ends up with packet wbase + 16i + m
            uint4 c[4];
#pragma unroll
            for (int j = 0; j < 4; j++) c[j] = hdr[wbase * 4 + j * 64 + lane];
            uint32_t w[4][4];
#pragma unroll
            for (int j = 0; j < 4; j++) { w[j][0] = c[j].x; w[j][1] = c[j].y; w[j][2] = c[j].z; w[j][3] = c[j].w; }
            const uint32_t qi = lane & 3u;
            // stage 1: swap the off-diagonal 2x2 blocks (partner lane ^ 2, element ^ 2)
            uint32_t x[4][4];
#pragma unroll
            for (int j = 0; j < 4; j++)
#pragma unroll
                for (int d = 0; d < 4; d++) x[j][d] = __builtin_amdgcn_update_dpp(0, (int)w[j ^ 2][d], 0x4E, 0xF, 0xF, false);
#pragma unroll
            for (int j = 0; j < 4; j++)
#pragma unroll
                for (int d = 0; d < 4; d++) w[j][d] = (((qi >> 1) ^ (j >> 1)) & 1u) ? x[j][d] : w[j][d];
            // stage 2: transpose each 2x2 block (partner lane ^ 1, element ^ 1)
#pragma unroll
            for (int j = 0; j < 4; j++)
#pragma unroll
                for (int d = 0; d < 4; d++) x[j][d] = __builtin_amdgcn_update_dpp(0, (int)w[j ^ 1][d], 0xB1, 0xF, 0xF, false);
#pragma unroll
            for (int j = 0; j < 4; j++)
#pragma unroll
                for (int d = 0; d < 4; d++) w[j][d] = ((qi ^ (uint32_t)j) & 1u) ? x[j][d] : w[j][d];
#pragma unroll
            for (int j = 0; j < 4; j++) v[j] = make_uint4(w[j][0], w[j][1], w[j][2], w[j][3]);
        } else if (COAL) {
            uint4 c[4];
#pragma unroll
            for (int j = 0; j < 4; j++) c[j] = hdr[wbase * 4 + j * 64 + lane];
#pragma unroll
            for (int j = 0; j < 4; j++) st[wave][j * 64 + lane] = c[j];
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (int i = 0; i < 4; i++) v[i] = st[wave][lane * 4 + i];
            __builtin_amdgcn_wave_barrier();
        } else {
#pragma unroll
            for (int i = 0; i < 4; i++) v[i] = hdr[p * 4 + i];
        }
        const uint64_t q = COAL == 2 ? wbase + 16 * (lane & 3u) + (lane >> 2) : p;
        const uint32_t h = mix(v, sz[q]);
        keyid[q] = h;
#pragma unroll
        for (int rr = 0; rr < 4; rr++) idx[rr * N + q] = (h + rr) & 0xFFFFF;
    }
}

int main() {
    uint4 *hdr; uint32_t *sz, *keyid, *idx;
    hipMalloc(&hdr, N * 64); hipMalloc(&sz, N * 4); hipMalloc(&keyid, N * 4); hipMalloc(&idx, N * 16);
    hipMemset(hdr, 1, N * 64); hipMemset(sz, 2, N * 4);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    struct V { const char *name; int coal, items; };
    const V vs[] = {{"per-lane records, 1/thread", 0, 1}, {"coalesced+LDS, 1/thread", 1, 1},
                    {"per-lane records, 4/thread", 0, 4}, {"coalesced+LDS, 4/thread", 1, 4},
                    {"coalesced+DPP, 1/thread", 2, 1}, {"coalesced+DPP, 4/thread", 2, 4}};
    for (const V &v : vs) {
        float best = 1e9f;
        const unsigned grid = (unsigned)(N / 256 / v.items);
        for (int rep = 0; rep < 5; rep++) {
            hipEventRecord(a);
            if (v.coal == 1 && v.items == 1) hipLaunchKernelGGL((k_stream<1, 1>), dim3(grid), dim3(256), 0, 0, hdr, sz, keyid, idx);
            if (!v.coal && v.items == 1) hipLaunchKernelGGL((k_stream<0, 1>), dim3(grid), dim3(256), 0, 0, hdr, sz, keyid, idx);
            if (v.coal == 1 && v.items == 4) hipLaunchKernelGGL((k_stream<1, 4>), dim3(grid), dim3(256), 0, 0, hdr, sz, keyid, idx);
            if (!v.coal && v.items == 4) hipLaunchKernelGGL((k_stream<0, 4>), dim3(grid), dim3(256), 0, 0, hdr, sz, keyid, idx);
            if (v.coal == 2 && v.items == 1) hipLaunchKernelGGL((k_stream<2, 1>), dim3(grid), dim3(256), 0, 0, hdr, sz, keyid, idx);
            if (v.coal == 2 && v.items == 4) hipLaunchKernelGGL((k_stream<2, 4>), dim3(grid), dim3(256), 0, 0, hdr, sz, keyid, idx);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
        }
        printf("%-30s %.3f ms  (%.2f TB/s of 88 B/packet)\n", v.name, best, 88.0 * N / (best * 1e-3) / 1e12);
        fflush(stdout);
    }
    return 0;
}
