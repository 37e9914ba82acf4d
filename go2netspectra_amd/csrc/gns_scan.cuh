// gns_scan.cuh -- exclusive scan of block-major histograms, shared by the
// Count-Min engine (K2, the (row, tile) bins) and the SuperSpread candidate
// partition (cell bins).  Internal linkage: each engine gets its own copy.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gns {
namespace {

// ---------------------------------------------------------------------------
// K2: exclusive scan of the per-block bin histograms (block-major), in place.
// ---------------------------------------------------------------------------
extern "C" __device__ unsigned __ockl_wfscan_add_u32(unsigned, bool);
// DPP inclusive scan over the whole wave (call with all 64 lanes active)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v) { return __ockl_wfscan_add_u32(v, true); }

// K2 over the block-major histogram hist[blk][bin] (K1 flushes one contiguous
// row per block, K3 loads one): offsets[blk][bin] = (updates of all bins
// before `bin`) + (updates of `bin` in blocks before `blk`), in place.  Blocks
// are taken in groups of kTGrp: group sums, a per-bin scan over the groups,
// a scan over the bins, then each group's run.  Threads of a wave hold
// consecutive bins, so every pass reads whole rows.
constexpr uint32_t kTGrp = 32;

static __global__ __launch_bounds__(256) void k_tscan_part(const uint32_t *hist, uint32_t nblk, uint32_t nbins,
                                                    uint32_t *part) {
    const uint32_t bin = blockIdx.x * 256 + threadIdx.x, g = blockIdx.y;
    if (bin >= nbins) return;
    const uint32_t b0 = g * kTGrp, b1 = min(nblk, b0 + kTGrp);
    uint32_t sum = 0;
#pragma unroll 8
    for (uint32_t b = b0; b < b1; b++) sum += hist[(uint64_t)b * nbins + bin];
    part[(uint64_t)g * nbins + bin] = sum;
}

static __global__ __launch_bounds__(256) void k_tscan_mid(uint32_t *part, uint32_t ngrp, uint32_t nbins, uint32_t *tot) {
    const uint32_t bin = blockIdx.x * 256 + threadIdx.x;
    if (bin >= nbins) return;
    uint32_t run = 0;
    for (uint32_t g0 = 0; g0 < ngrp; g0 += 16) {  // 16 loads in flight, then the scan
        uint32_t v[16];
#pragma unroll
        for (uint32_t j = 0; j < 16; j++) v[j] = g0 + j < ngrp ? part[(uint64_t)(g0 + j) * nbins + bin] : 0u;
#pragma unroll
        for (uint32_t j = 0; j < 16; j++) {
            if (g0 + j < ngrp) part[(uint64_t)(g0 + j) * nbins + bin] = run;
            run += v[j];
        }
    }
    tot[bin] = run;
}

// exclusive scan of the bin totals (nbins <= 8 * 1024), one 1024-thread block
static __global__ __launch_bounds__(1024) void k_tscan_bins(uint32_t *tot, uint32_t nbins, uint32_t *total) {
    __shared__ uint32_t s_w[16];
    constexpr uint32_t PER = 8;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    uint32_t v[PER], sum = 0;
#pragma unroll
    for (uint32_t i = 0; i < PER; i++) {
        const uint32_t b = tid * PER + i;
        v[i] = b < nbins ? tot[b] : 0u;
        sum += v[i];
    }
    const uint32_t inc = wave_incl_scan(sum);
    if (lane == 63) s_w[wave] = inc;
    __syncthreads();
    uint32_t base = 0, all = 0;
#pragma unroll
    for (uint32_t w = 0; w < 16; w++) {
        const uint32_t x = s_w[w];
        if (w < wave) base += x;
        all += x;
    }
    uint32_t run = base + inc - sum;
#pragma unroll
    for (uint32_t i = 0; i < PER; i++) {
        const uint32_t b = tid * PER + i;
        if (b < nbins) tot[b] = run;
        run += v[i];
    }
    if (tid == 0) *total = all;
}

static __global__ __launch_bounds__(256) void k_tscan_down(uint32_t *hist, uint32_t nblk, uint32_t nbins,
                                                    const uint32_t *part, const uint32_t *tot) {
    const uint32_t bin = blockIdx.x * 256 + threadIdx.x, g = blockIdx.y;
    if (bin >= nbins) return;
    const uint32_t b0 = g * kTGrp, b1 = min(nblk, b0 + kTGrp);
    uint32_t run = tot[bin] + part[(uint64_t)g * nbins + bin];
    for (uint32_t b = b0; b < b1; b++) {
        const uint64_t i = (uint64_t)b * nbins + bin;
        const uint32_t v = hist[i];
        hist[i] = run;
        run += v;
    }
}


}  // namespace
}  // namespace gns
