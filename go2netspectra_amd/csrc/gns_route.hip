// gns_route.hip -- device-side flow routing for the multi-GPU path (SURVEY.md
// §8e, BASELINE configs[3] "sharded by src-IP").
//
// A packet is owned by shard g = mm3(SrcIP slot, 0xA5A5A5A5) % G, so every flow
// of a source lands on one GPU and each GPU's sketch is exact for its
// sub-stream (the host restatement is go2netspectra_amd/dist.py shard_of).  The
// router turns one contiguous slice of the packet stream into G per-shard runs,
// STABLY (packet order kept inside each shard), laid out shard by shard:
//   R1 k_route_count   : parse each 64-byte record, owner shard -> one byte per
//                        packet, per-block shard histogram (ballot multisplit)
//   R2 k_route_scan    : exclusive offsets per (block, shard), shard-major
//   R3 k_route_scatter : per-wave stable ranks (ballot multisplit), copy the
//                        record + wire length to its shard's run
// An all-to-all (dist.route_exchange, RCCL) then sends run g to GPU g; received
// runs are concatenated in source-rank order, which, with rank r holding slice
// r of the stream, is exactly the stable filter stream[shard_of(src) == g].
//
// Records the parser drops or does not support carry no trustworthy SrcIP:
// they go to shard 0, whose engine counts them (dropped / unsupported) as the
// single-GPU engine would.
#include <algorithm>

#include "gns_common.hpp"

namespace gns {

constexpr uint32_t kRtChunk = 16384;  // packets per block
constexpr uint32_t kRtThreads = 256;
constexpr uint32_t kRtShardSeed = 0xA5A5A5A5u;
constexpr uint32_t kRtMaxShards = 64;

struct RouteArgs {
    const uint32_t *hdr;      // n * 16 words
    const uint32_t *wl;       // n
    uint64_t n;
    uint32_t G, gbits;        // shards, ceil(log2 G)
    uint8_t *shard;           // n
    uint32_t *hist;           // [nblk][G]: counts (R1), exclusive offsets (R2)
    uint32_t nblk;
    uint32_t *out_hdr;        // n * 16 words
    uint32_t *out_wl;
    uint32_t *totals;         // [G]
};

__device__ __forceinline__ uint32_t route_shard(const uint32_t (&w)[16], uint32_t wl, uint32_t G) {
    uint32_t tw[10];
    const int st = parse_record_fast(w, wl, true, tw);
    uint32_t kw[GNS_KWMAX];
#pragma unroll
    for (int i = 0; i < GNS_KWMAX; i++) kw[i] = i < 4 ? tw[i] : 0u;
    const uint32_t h = mm3_words(kw, 16, kRtShardSeed);
    return st == PARSE_OK ? h % G : 0u;
}

// lanes of the wave holding the same shard as this lane (ballot multisplit over
// the shard's bits); inactive lanes pass valid = false and match nothing
__device__ __forceinline__ uint64_t shard_peers(uint32_t s, bool valid, uint32_t gbits) {
    uint64_t m = __ballot(valid);
    for (uint32_t b = 0; b < gbits; b++) {
        const uint64_t ones = __ballot(valid && ((s >> b) & 1u));
        m &= ((s >> b) & 1u) ? ones : ~ones;
    }
    return valid ? m : 0ull;
}

__device__ __forceinline__ void load_rec(const uint32_t *hdr, uint64_t p, uint32_t (&w)[16]) {
    const uint4 *r = reinterpret_cast<const uint4 *>(hdr + p * 16);
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint4 v = r[i];
        w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
    }
}

__global__ __launch_bounds__(kRtThreads) void k_route_count(RouteArgs a) {
    __shared__ uint32_t s_hist[kRtMaxShards];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    for (uint32_t g = tid; g < a.G; g += kRtThreads) s_hist[g] = 0;
    __syncthreads();
    const uint64_t beg = (uint64_t)blockIdx.x * kRtChunk;
    const uint64_t end = min(a.n, beg + kRtChunk);
    for (uint64_t p0 = beg; p0 < end; p0 += kRtThreads) {  // block-uniform trip count
        const uint64_t p = p0 + tid;
        const bool valid = p < end;
        uint32_t s = 0;
        if (valid) {
            uint32_t w[16];
            load_rec(a.hdr, p, w);
            s = route_shard(w, a.wl[p], a.G);
            a.shard[p] = (uint8_t)s;
        }
        const uint64_t peers = shard_peers(s, valid, a.gbits);
        if (valid && (uint32_t)(__ffsll((long long)peers) - 1) == lane) atomicAdd(&s_hist[s], (uint32_t)__popcll(peers));
    }
    __syncthreads();
    for (uint32_t g = tid; g < a.G; g += kRtThreads) a.hist[(uint64_t)blockIdx.x * a.G + g] = s_hist[g];
}

// One workgroup: column scans of hist[nblk][G], shard-major offsets in place.
__global__ __launch_bounds__(1024) void k_route_scan(RouteArgs a) {
    __shared__ uint32_t s_part[1024];
    __shared__ uint32_t s_base;
    const uint32_t tid = threadIdx.x;
    if (tid == 0) s_base = 0;
    __syncthreads();
    for (uint32_t g = 0; g < a.G; g++) {
        for (uint32_t c0 = 0; c0 < a.nblk; c0 += 1024) {
            const uint32_t b = c0 + tid;
            const uint32_t v = b < a.nblk ? a.hist[(uint64_t)b * a.G + g] : 0u;
            s_part[tid] = v;
            __syncthreads();
            for (uint32_t o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan
                const uint32_t t = tid >= o ? s_part[tid - o] : 0u;
                __syncthreads();
                s_part[tid] += t;
                __syncthreads();
            }
            const uint32_t base = s_base;
            if (b < a.nblk) a.hist[(uint64_t)b * a.G + g] = base + s_part[tid] - v;
            __syncthreads();
            if (tid == 1023) s_base = base + s_part[1023];
            __syncthreads();
        }
        if (tid == 0) {
            const uint32_t start = g == 0 ? 0u : a.totals[a.G + g - 1];  // running end of shard g-1
            a.totals[g] = s_base - start;
            a.totals[a.G + g] = s_base;
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(kRtThreads) void k_route_scatter(RouteArgs a) {
    __shared__ uint32_t s_base[kRtMaxShards];
    __shared__ uint32_t s_wave[kRtThreads / 64][kRtMaxShards];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    for (uint32_t g = tid; g < a.G; g += kRtThreads) s_base[g] = a.hist[(uint64_t)blockIdx.x * a.G + g];
    const uint64_t beg = (uint64_t)blockIdx.x * kRtChunk;
    const uint64_t end = min(a.n, beg + kRtChunk);
    for (uint64_t p0 = beg; p0 < end; p0 += kRtThreads) {
        const uint64_t p = p0 + tid;
        const bool valid = p < end;
        uint32_t s = 0, w[16], len = 0;
        if (valid) {
            s = a.shard[p];
            load_rec(a.hdr, p, w);
            len = a.wl[p];
        }
        for (uint32_t g = tid; g < (kRtThreads / 64) * kRtMaxShards; g += kRtThreads) (&s_wave[0][0])[g] = 0;
        __syncthreads();
        const uint64_t peers = shard_peers(s, valid, a.gbits);
        const uint32_t rank = (uint32_t)__popcll(peers & ((1ull << lane) - 1ull));
        if (valid && rank == 0) s_wave[wave][s] = (uint32_t)__popcll(peers);
        __syncthreads();
        if (valid) {
            uint32_t pos = s_base[s] + rank;
            for (uint32_t v = 0; v < wave; v++) pos += s_wave[v][s];
            uint4 *o = reinterpret_cast<uint4 *>(a.out_hdr + (uint64_t)pos * 16);
#pragma unroll
            for (int i = 0; i < 4; i++) o[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
            a.out_wl[pos] = len;
        }
        __syncthreads();
        for (uint32_t g = tid; g < a.G; g += kRtThreads) {
            uint32_t t = 0;
            for (uint32_t v = 0; v < kRtThreads / 64; v++) t += s_wave[v][g];
            s_base[g] += t;
        }
        __syncthreads();
    }
}

__global__ void k_route_counts64(const uint32_t *totals, uint32_t G, int64_t *out) {
    for (uint32_t g = threadIdx.x; g < G; g += blockDim.x) out[g] = (int64_t)totals[g];
}

}  // namespace gns

using namespace gns;

struct gns_route {
    int device = 0;
    uint32_t G = 1, gbits = 0;
    hipStream_t stream = nullptr;
    uint8_t *shard = nullptr;
    uint64_t shard_n = 0;
    uint32_t *hist = nullptr;
    uint64_t hist_n = 0;
    uint32_t *totals = nullptr;  // [2G]: counts, running ends
    uint32_t *h_tot = nullptr;   // pinned [2G]
};

static void route_free(gns_route *r) {
    dfree(r->shard); dfree(r->hist); dfree(r->totals);
    if (r->h_tot) (void)hipHostFree(r->h_tot);
    if (r->stream) (void)hipStreamDestroy(r->stream);
}

extern "C" {

int gns_route_create(uint32_t nshards, int device, gns_route **out) {
    if (!out) { set_error("null argument"); return GNS_E_ARG; }
    *out = nullptr;
    if (nshards == 0 || nshards > kRtMaxShards) { set_error("nshards %u not in [1, %u]", nshards, kRtMaxShards); return GNS_E_ARG; }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        (void)hipGetLastError();
        set_error("no HIP device available");
        return GNS_E_NODEV;
    }
    if (device < 0 || device >= ndev) { set_error("device %d out of range", device); return GNS_E_ARG; }
    GNS_HIP(hipSetDevice(device));
    gns_route *r = new gns_route();
    r->device = device;
    r->G = nshards;
    while ((1u << r->gbits) < nshards) r->gbits++;
    int rc = GNS_OK;
    do {
        if (hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking) != hipSuccess) {
            set_error("hipStreamCreate failed"); rc = GNS_E_HIP; break;
        }
        if ((rc = dalloc_t(&r->totals, 2 * kRtMaxShards)) != GNS_OK) break;
        if (hipHostMalloc(reinterpret_cast<void **>(&r->h_tot), 2 * kRtMaxShards * 4, 0) != hipSuccess) {
            set_error("hipHostMalloc failed"); rc = GNS_E_OOM; break;
        }
    } while (0);
    if (rc) { route_free(r); delete r; return rc; }
    *out = r;
    return GNS_OK;
}

int gns_route_destroy(gns_route *r) {
    if (!r) return GNS_OK;
    (void)hipSetDevice(r->device);
    if (r->stream) (void)hipStreamSynchronize(r->stream);
    route_free(r);
    delete r;
    return GNS_OK;
}

static int route_launch(gns_route *r, const uint8_t *hdr, const uint32_t *wirelen, uint64_t n, uint8_t *out_hdr,
                        uint32_t *out_wirelen, hipStream_t st) {
    const uint32_t nblk = (uint32_t)((n + kRtChunk - 1) / kRtChunk);
    if (r->shard_n < n || r->hist_n < (uint64_t)nblk * r->G) {
        GNS_HIP(hipStreamSynchronize(st));  // an earlier partition may still read the scratch
        if (r->shard_n < n) {
            dfree(r->shard); r->shard = nullptr; r->shard_n = 0;
            GNS_TRY(dalloc_t(&r->shard, n));
            r->shard_n = n;
        }
        if (r->hist_n < (uint64_t)nblk * r->G) {
            dfree(r->hist); r->hist = nullptr; r->hist_n = 0;
            GNS_TRY(dalloc_t(&r->hist, (uint64_t)nblk * r->G));
            r->hist_n = (uint64_t)nblk * r->G;
        }
    }
    RouteArgs a{};
    a.hdr = reinterpret_cast<const uint32_t *>(hdr); a.wl = wirelen; a.n = n; a.G = r->G; a.gbits = r->gbits;
    a.shard = r->shard; a.hist = r->hist; a.nblk = nblk;
    a.out_hdr = reinterpret_cast<uint32_t *>(out_hdr); a.out_wl = out_wirelen; a.totals = r->totals;
    hipLaunchKernelGGL(k_route_count, dim3(nblk), dim3(kRtThreads), 0, st, a);
    hipLaunchKernelGGL(k_route_scan, dim3(1), dim3(1024), 0, st, a);
    hipLaunchKernelGGL(k_route_scatter, dim3(nblk), dim3(kRtThreads), 0, st, a);
    GNS_HIP(hipGetLastError());
    return GNS_OK;
}

int gns_route_partition(gns_route *r, const uint8_t *hdr, const uint32_t *wirelen, uint64_t n, uint8_t *out_hdr,
                        uint32_t *out_wirelen, uint64_t *counts) {
    if (!r || !counts || (n && (!hdr || !wirelen || !out_hdr || !out_wirelen))) {
        set_error("null argument"); return GNS_E_ARG;
    }
    if (n >= (1ull << 32)) { set_error("route batch of %llu packets (max 2^32 - 1)", (unsigned long long)n); return GNS_E_RANGE; }
    if (n == 0) { for (uint32_t g = 0; g < r->G; g++) counts[g] = 0; return GNS_OK; }
    (void)hipGetLastError();  // clear a stale error of an earlier runtime call on this thread
    GNS_HIP(hipSetDevice(r->device));
    GNS_TRY(route_launch(r, hdr, wirelen, n, out_hdr, out_wirelen, r->stream));
    GNS_HIP(hipMemcpyAsync(r->h_tot, r->totals, r->G * 4, hipMemcpyDeviceToHost, r->stream));
    GNS_HIP(hipStreamSynchronize(r->stream));
    for (uint32_t g = 0; g < r->G; g++) counts[g] = r->h_tot[g];
    return GNS_OK;
}

int gns_route_partition_async(gns_route *r, const uint8_t *hdr, const uint32_t *wirelen, uint64_t n,
                              uint8_t *out_hdr, uint32_t *out_wirelen, int64_t *counts_dev, void *stream) {
    if (!r || !counts_dev || (n && (!hdr || !wirelen || !out_hdr || !out_wirelen))) {
        set_error("null argument"); return GNS_E_ARG;
    }
    if (n >= (1ull << 32)) { set_error("route batch of %llu packets (max 2^32 - 1)", (unsigned long long)n); return GNS_E_RANGE; }
    (void)hipGetLastError();
    GNS_HIP(hipSetDevice(r->device));
    hipStream_t st = stream ? reinterpret_cast<hipStream_t>(stream) : r->stream;
    if (n == 0) {
        GNS_HIP(hipMemsetAsync(counts_dev, 0, r->G * 8, st));
        return GNS_OK;
    }
    GNS_TRY(route_launch(r, hdr, wirelen, n, out_hdr, out_wirelen, st));
    hipLaunchKernelGGL(k_route_counts64, dim3(1), dim3(64), 0, st, r->totals, r->G, counts_dev);
    GNS_HIP(hipGetLastError());
    return GNS_OK;
}

}  // extern "C"
