// LDS returning-add throughput on gfx950: cycles per wave-instruction for
// ds_add_rtn_u32 with 64 / 32 active lanes, random vs conflict-free addresses,
// against ds_read_b32 of the same addresses.  One 1024-thread block per CU.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

template <int MODE>
__global__ __launch_bounds__(1024) void k(uint32_t *out, int iters, uint64_t *cyc) {
    __shared__ uint32_t cnt[16][256];
    __shared__ uint32_t dummy[1024];
    const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    for (uint32_t i = tid; i < 16 * 256; i += 1024) (&cnt[0][0])[i] = 0;
    dummy[tid] = 0;
    __syncthreads();
    uint32_t x = (blockIdx.x * 1024 + tid) * 0x9E3779B1u + 1u, acc = 0;
    const uint64_t t0 = __builtin_readcyclecounter();
    for (int it = 0; it < iters; it++) {
        uint32_t r[8];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            x = x * 1664525u + 1013904223u;
            uint32_t b = (MODE & 1) ? lane * 4 + (j & 3) : (x >> 24);  // bit0: conflict-free addresses
            const bool valid = (MODE & 2) ? ((x >> 7) & 1) : true;       // bit1: ~half the lanes "hot"
            if (MODE & 4) r[j] = cnt[wave][b];                            // bit2: plain reads
            else {
                uint32_t *ad = valid ? &cnt[wave][b] : &dummy[tid];
                r[j] = atomicAdd(ad, valid ? 1u : 0u);
            }
        }
#pragma unroll
        for (int j = 0; j < 8; j++) acc += r[j];
    }
    const uint64_t t1 = __builtin_readcyclecounter();
    __syncthreads();
    out[blockIdx.x * 1024 + tid] = acc;
    if (tid == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    uint32_t *out; uint64_t *cyc;
    const int nb = 256, iters = 2000;
    hipMalloc(&out, nb * 1024 * 4); hipMalloc(&cyc, nb * 8);
    std::vector<uint64_t> h(nb);
    auto run = [&](auto kern, const char *name) {
        hipLaunchKernelGGL(kern, dim3(nb), dim3(1024), 0, 0, out, iters, cyc);
        hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
        hipEventRecord(a);
        hipLaunchKernelGGL(kern, dim3(nb), dim3(1024), 0, 0, out, iters, cyc);
        hipEventRecord(b); hipEventSynchronize(b);
        float ms; hipEventElapsedTime(&ms, a, b);
        hipMemcpy(h.data(), cyc, nb * 8, hipMemcpyDeviceToHost);
        double s = 0; for (auto v : h) s += v; s /= nb;
        // per CU: 16 waves x iters x 8 instructions
        printf("%-28s %.3f ms  %.2f cycles(ts) per wave-instr per CU\n", name, ms, s / (16.0 * iters * 8));
    };
    run(k<0>, "atomic rtn random 64 lanes");
    run(k<2>, "atomic rtn random, half dummy");
    run(k<1>, "atomic rtn conflict-free");
    run(k<4>, "read b32 random");
    run(k<5>, "read b32 conflict-free");
    return 0;
}
