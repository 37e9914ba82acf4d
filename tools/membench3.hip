// K3 write-pattern study (dev tool, not part of the library): 180M 8-byte
// entries scattered into 1024 bins in stream order, written as runs of R
// consecutive entries of one bin (R = 1 is K3's per-wave direct store pattern;
// larger R is what staging a block's updates by bin would give).  Each kernel
// also streams the 24 B/packet K3 reads (codes, ids, sizes) for 100M packets.
// Build: hipcc -O3 --offload-arch=gfx950 tools/membench3.hip -o tools/membench3.bin
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <vector>

constexpr uint64_t NPKT = 100000000ull;
constexpr uint64_t NENT = 180000000ull;
constexpr uint32_t NBINS = 1024;

// entry e (in stream order) goes to run (e / R); runs are dealt to bins round-robin by a hash,
// and each bin's runs are placed contiguously in the order they occur (stable partition)
__global__ __launch_bounds__(256) void k_write(uint64_t *out, const uint32_t *runpos, uint32_t R,
                                               const uint32_t *codes, const uint32_t *ids, const uint32_t *sizes,
                                               uint32_t *sink) {
    const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    uint32_t acc = 0;
    // the read stream: 24 B per packet (4 codes, id, size)
    for (uint64_t p = t; p < NPKT; p += (uint64_t)gridDim.x * 256) {
        acc += codes[p] + codes[NPKT + p] + codes[2 * NPKT + p] + codes[3 * NPKT + p] + ids[p] + sizes[p];
    }
    // the write stream: entry e -> runpos[e / R] + e % R
    for (uint64_t e = t; e < NENT; e += (uint64_t)gridDim.x * 256) {
        const uint32_t pos = runpos[e / R] + (uint32_t)(e % R);
        out[pos] = e ^ acc;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
    uint64_t *out; uint32_t *runpos, *codes, *ids, *sizes, *sink;
    hipMalloc(&out, NENT * 8); hipMalloc(&runpos, NENT * 4); hipMalloc(&codes, NPKT * 16);
    hipMalloc(&ids, NPKT * 4); hipMalloc(&sizes, NPKT * 4); hipMalloc(&sink, 4);
    hipMemset(codes, 1, NPKT * 16); hipMemset(ids, 2, NPKT * 4); hipMemset(sizes, 3, NPKT * 4);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    const uint32_t Rs[] = {1, 2, 4, 8, 16, 32, 64};
    for (uint32_t R : Rs) {
        const uint64_t nrun = (NENT + R - 1) / R;
        std::vector<uint32_t> bin(nrun), cnt(NBINS, 0), base(NBINS, 0), pos(nrun);
        for (uint64_t r = 0; r < nrun; r++) {
            uint32_t x = (uint32_t)r * 0x9E3779B1u; x ^= x >> 15; x *= 0x2C1B3C6Du; x ^= x >> 12;
            bin[r] = x % NBINS;
            cnt[bin[r]] += (uint32_t)((r + 1) * R <= NENT ? R : NENT - r * R);
        }
        uint32_t run = 0;
        for (uint32_t i = 0; i < NBINS; i++) { base[i] = run; run += cnt[i]; }
        for (uint64_t r = 0; r < nrun; r++) {
            pos[r] = base[bin[r]];
            base[bin[r]] += (uint32_t)((r + 1) * R <= NENT ? R : NENT - r * R);
        }
        hipMemcpy(runpos, pos.data(), nrun * 4, hipMemcpyHostToDevice);
        float best = 1e9f;
        for (int rep = 0; rep < 4; rep++) {
            hipEventRecord(a);
            hipLaunchKernelGGL(k_write, dim3(8192), dim3(256), 0, 0, out, runpos, R, codes, ids, sizes, sink);
            hipEventRecord(b); hipEventSynchronize(b);
            float ms; hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
        }
        printf("runs of %2u entries: %.3f ms\n", R, best);
        fflush(stdout);
    }
    return 0;
}
