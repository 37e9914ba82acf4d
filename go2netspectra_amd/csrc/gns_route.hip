// gns_route.hip -- device-side flow routing for the multi-GPU path (SURVEY.md
// §8e, BASELINE configs[3] "sharded by src-IP").
//
// Every flow of every task must land on ONE shard, so that each GPU's sketch is
// exact for its sub-stream.  A router is built for an OWNER KEY: fields that
// every task's flow key contains (gns_route_owner_fields; task.go:265-300 builds
// a key from the configured fields).  Packets of one flow agree on those
// fields, so shard g = mm3(owner key, 0xA5A5A5A5) % G is a function of the flow.
//   - every task keys on SrcIP (the default tasks, configs/config.yaml:114,125):
//     the owner key is the SrcIP slot alone, and every flow of a source shares
//     a GPU (configs[3] "sharded by src-IP");
//   - otherwise the owner key is the fields the tasks share, in canonical field
//     order; for one task that is its whole flow key (e.g. ["DstIP"] or
//     ["DstPort","Protocol"], legal per config.go:59).
// IP slots enter the owner key canonicalised: an IPv4-mapped IPv6 slot
// (::ffff:a.b.c.d) hashes as the IPv4 slot a.b.c.d.  That keeps the owner a
// function of the EncodeFlow bytes (sketch tasks) AND of the To16 form the exact
// aggregator keys on (exact/task.go:330-366), which merges the two.
// The host restatement is go2netspectra_amd/dist.py (owner_fields, owner_of_*).
//
// The router turns one contiguous slice of the packet stream into G per-shard
// runs, STABLY (packet order kept inside each shard), laid out shard by shard:
//   R1 k_route_count   : parse each 64-byte record, owner shard -> one byte per
//                        packet, per-block shard histogram (ballot multisplit)
//   R2 k_route_scan    : exclusive offsets per (block, shard), shard-major
//   R3 k_route_scatter : per-wave stable ranks (ballot multisplit), copy the
//                        record + wire length to its shard's run
// An all-to-all (dist.route_exchange, RCCL) then sends run g to GPU g; received
// runs are concatenated in source-rank order, which, with rank r holding slice
// r of the stream, is exactly the stable filter stream[owner == g].
// Queries route the same way (k_route_keys: the owner of a task's flow key,
// dist.routed_query): a key goes to the shard whose sketch holds its flow.
//
// Records the parser drops or does not support carry no trustworthy tuple:
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
    KeyPlanN own;             // owner key over the canonical tuple bytes
};

// IPv4-mapped IPv6 slot (bytes 0..9 zero, 10..11 0xFF) -> the IPv4 slot (see above)
__device__ __forceinline__ void canon_slot(uint32_t (&tw)[10], int b) {
    if (tw[b] == 0u && tw[b + 1] == 0u && tw[b + 2] == 0xFFFF0000u) {
        tw[b] = tw[b + 3];
        tw[b + 3] = 0u;
        tw[b + 2] = 0u;
    }
}

// owner shard of a canonical tuple; SRC: the owner key is the SrcIP slot alone
template <bool SRC>
__device__ __forceinline__ uint32_t owner_of_tuple(uint32_t (&tw)[10], uint32_t K, const uint8_t *s_src, uint32_t G) {
    canon_slot(tw, 0);
    uint32_t kw[GNS_KWMAX];
    if constexpr (SRC) {
#pragma unroll
        for (int i = 0; i < GNS_KWMAX; i++) kw[i] = i < 4 ? tw[i] : 0u;
        return mm3_words(kw, 16, kRtShardSeed) % G;
    } else {
        canon_slot(tw, 4);
        make_key_m<PLAN_GENERIC, GNS_KWMAX>(K, s_src, tw, kw);
        return mm3_words(kw, K, kRtShardSeed) % G;
    }
}

template <bool SRC>
__device__ __forceinline__ uint32_t route_shard(const uint32_t (&w)[16], uint32_t wl, uint32_t K, const uint8_t *s_src,
                                                uint32_t G) {
    uint32_t tw[10];
    const int st = parse_record_fast(w, wl, true, tw);
    const uint32_t g = owner_of_tuple<SRC>(tw, K, s_src, G);
    return st == PARSE_OK ? g : 0u;
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

template <bool SRC>
__global__ __launch_bounds__(kRtThreads) void k_route_count(RouteArgs a) {
    __shared__ uint32_t s_hist[kRtMaxShards];
    __shared__ uint8_t s_src[80];
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    for (uint32_t g = tid; g < a.G; g += kRtThreads) s_hist[g] = 0;
    if constexpr (!SRC) stage_plan<PLAN_GENERIC>(a.own, s_src);
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
            s = route_shard<SRC>(w, a.wl[p], a.own.K, s_src, a.G);
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

// Owner shard of n flow keys of one task (keys[i*stride], K bytes laid out as
// the task's FlowFields): the key's fields are put back at their canonical tuple
// positions (inv[t] = key byte of tuple byte t, 255 = absent; the owner fields
// are all present, gns_route_owner_keys checks), then the tuple's owner as R1
// computes it for a packet of that flow.
struct RouteKeysArgs {
    const uint8_t *keys;
    uint32_t stride, K;
    uint64_t n;
    uint32_t G;
    uint32_t *owner;
    uint8_t inv[40];
    KeyPlanN own;
};

template <bool SRC>
__global__ __launch_bounds__(256) void k_route_keys(RouteKeysArgs a) {
    __shared__ uint8_t s_src[80];
    __shared__ uint8_t s_inv[40];
    if constexpr (!SRC) stage_plan<PLAN_GENERIC>(a.own, s_src);
    for (uint32_t j = threadIdx.x; j < 40; j += blockDim.x) s_inv[j] = a.inv[j];
    __syncthreads();
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t *k = a.keys + i * a.stride;
        uint32_t tw[10];
#pragma unroll
        for (int w = 0; w < 10; w++) {
            uint32_t v = 0;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const uint32_t j = s_inv[4 * w + b];
                if (j < a.K) v |= (uint32_t)k[j] << (8 * b);
            }
            tw[w] = v;
        }
        a.owner[i] = owner_of_tuple<SRC>(tw, a.own.K, s_src, a.G);
    }
}

}  // namespace gns

using namespace gns;

struct gns_route {
    int device = 0;
    uint32_t G = 1, gbits = 0;
    KeyPlanN own{};                // owner key (over canonical tuple bytes)
    bool src_only = true;          // owner key == the SrcIP slot
    gns_layout own_layout{};
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;     // recorded after every partition: the scratch is free once it fires
    uint8_t *kbuf = nullptr;       // staged host keys / owners (gns_route_owner_keys)
    uint64_t kbuf_n = 0;
    uint8_t *shard = nullptr;
    uint64_t shard_n = 0;
    uint32_t *hist = nullptr;
    uint64_t hist_n = 0;
    uint32_t *totals = nullptr;  // [2G]: counts, running ends
    uint32_t *h_tot = nullptr;   // pinned [2G]
};

static void route_free(gns_route *r) {
    dfree(r->shard); dfree(r->hist); dfree(r->totals); dfree(r->kbuf);
    if (r->h_tot) (void)hipHostFree(r->h_tot);
    if (r->done) (void)hipEventDestroy(r->done);
    if (r->stream) (void)hipStreamDestroy(r->stream);
}

static bool layout_has(const gns_layout &l, uint8_t f) {
    for (uint32_t i = 0; i < l.n_fields && i < 8; i++)
        if (l.fields[i] == f) return true;
    return false;
}

extern "C" {

int gns_route_owner_fields(const gns_layout *tasks, uint32_t n_tasks, gns_layout *owner) {
    if (!tasks || !owner || n_tasks == 0) { set_error("null argument or no tasks"); return GNS_E_ARG; }
    for (uint32_t t = 0; t < n_tasks; t++)
        if (tasks[t].n_fields > 8) { set_error("task %u: layout has %u fields (max 8)", t, tasks[t].n_fields); return GNS_E_ARG; }
    gns_layout o{};
    bool src = true;
    for (uint32_t t = 0; t < n_tasks; t++) src = src && layout_has(tasks[t], GNS_F_SRCIP);
    if (src) {
        o.n_fields = 1;
        o.fields[0] = GNS_F_SRCIP;
    } else {
        for (uint8_t f = GNS_F_SRCIP; f <= GNS_F_PROTO; f++) {
            bool all = true;
            for (uint32_t t = 0; t < n_tasks; t++) all = all && layout_has(tasks[t], f);
            if (all) o.fields[o.n_fields++] = f;
        }
    }
    if (o.n_fields == 0) {
        set_error("the tasks' flow keys share no field: no shard owns every flow of every task "
                  "(shard each task set on its own router)");
        return GNS_E_ARG;
    }
    *owner = o;
    return GNS_OK;
}

int gns_route_create_keyed(uint32_t nshards, const gns_layout *owner, int device, gns_route **out) {
    if (!out || !owner) { set_error("null argument"); return GNS_E_ARG; }
    *out = nullptr;
    if (nshards == 0 || nshards > kRtMaxShards) { set_error("nshards %u not in [1, %u]", nshards, kRtMaxShards); return GNS_E_ARG; }
    KeyPlanN own;
    GNS_TRY(make_plan(*owner, 0, &own));
    if (own.K == 0) { set_error("empty owner key (gns_route_owner_fields picks one)"); return GNS_E_ARG; }
    for (uint32_t i = 0; i < owner->n_fields; i++)
        for (uint32_t j = 0; j < i; j++)
            if (owner->fields[i] == owner->fields[j]) { set_error("owner key repeats a field"); return GNS_E_ARG; }
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
    r->own = own;
    r->own_layout = *owner;
    r->src_only = owner->n_fields == 1 && owner->fields[0] == GNS_F_SRCIP;
    while ((1u << r->gbits) < nshards) r->gbits++;
    int rc = GNS_OK;
    do {
        if (hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking) != hipSuccess) {
            set_error("hipStreamCreate failed"); rc = GNS_E_HIP; break;
        }
        if (hipEventCreateWithFlags(&r->done, hipEventDisableTiming) != hipSuccess) {
            set_error("hipEventCreate failed"); rc = GNS_E_HIP; break;
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

int gns_route_create(uint32_t nshards, int device, gns_route **out) {
    gns_layout src{};
    src.n_fields = 1;
    src.fields[0] = GNS_F_SRCIP;
    return gns_route_create_keyed(nshards, &src, device, out);
}

int gns_route_destroy(gns_route *r) {
    if (!r) return GNS_OK;
    (void)hipSetDevice(r->device);
    if (r->done) (void)hipEventSynchronize(r->done);
    if (r->stream) (void)hipStreamSynchronize(r->stream);
    route_free(r);
    delete r;
    return GNS_OK;
}

static int route_launch(gns_route *r, const uint8_t *hdr, const uint32_t *wirelen, uint64_t n, uint8_t *out_hdr,
                        uint32_t *out_wirelen, hipStream_t st) {
    const uint32_t nblk = (uint32_t)((n + kRtChunk - 1) / kRtChunk);
    // the scratch (shard bytes, histograms, totals) is shared by every partition of
    // the handle: order this one after the last, whichever stream that ran on
    GNS_HIP(hipStreamWaitEvent(st, r->done, 0));
    if (r->shard_n < n || r->hist_n < (uint64_t)nblk * r->G) {
        GNS_HIP(hipEventSynchronize(r->done));  // an earlier partition may still read the scratch
        GNS_HIP(hipStreamSynchronize(st));
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
    a.own = r->own;
    if (r->src_only)
        hipLaunchKernelGGL(k_route_count<true>, dim3(nblk), dim3(kRtThreads), 0, st, a);
    else
        hipLaunchKernelGGL(k_route_count<false>, dim3(nblk), dim3(kRtThreads), 0, st, a);
    hipLaunchKernelGGL(k_route_scan, dim3(1), dim3(1024), 0, st, a);
    hipLaunchKernelGGL(k_route_scatter, dim3(nblk), dim3(kRtThreads), 0, st, a);
    GNS_HIP(hipGetLastError());
    return GNS_OK;
}

// after the partition's last read of the scratch (and of totals, by the caller's copy)
static int route_done(gns_route *r, hipStream_t st) {
    GNS_HIP(hipEventRecord(r->done, st));
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
    GNS_TRY(route_done(r, r->stream));
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
    return route_done(r, st);
}

int gns_route_owner_layout(gns_route *r, gns_layout *owner) {
    if (!r || !owner) { set_error("null argument"); return GNS_E_ARG; }
    *owner = r->own_layout;
    return GNS_OK;
}

int gns_route_owner_keys(gns_route *r, const gns_layout *key_layout, const uint8_t *keys, uint32_t stride, uint64_t n,
                         uint32_t *owner, gns_mem where) {
    if (!r || !key_layout || !owner || (n && !keys)) { set_error("null argument"); return GNS_E_ARG; }
    KeyPlanN kp;
    GNS_TRY(make_plan(*key_layout, 0, &kp));
    for (uint32_t i = 0; i < r->own_layout.n_fields; i++)
        if (!layout_has(*key_layout, r->own_layout.fields[i])) {
            set_error("the key layout lacks owner field %u: its flows are not owned by one shard", r->own_layout.fields[i]);
            return GNS_E_ARG;
        }
    if (n == 0) return GNS_OK;  // nothing to route (any stride)
    if (stride < kp.K) { set_error("stride %u below the key's %u bytes", stride, kp.K); return GNS_E_ARG; }
    if (n >= (1ull << 32)) { set_error("%llu keys (max 2^32 - 1)", (unsigned long long)n); return GNS_E_RANGE; }
    RouteKeysArgs a{};
    for (int t = 0; t < 40; t++) a.inv[t] = 255;
    for (uint32_t j = 0; j < kp.K; j++) a.inv[kp.src[j]] = (uint8_t)j;  // make_plan: key byte j <- tuple byte src[j]
    a.stride = stride; a.K = kp.K; a.n = n; a.G = r->G; a.own = r->own;
    (void)hipGetLastError();
    GNS_HIP(hipSetDevice(r->device));
    hipStream_t st = r->stream;
    GNS_HIP(hipStreamWaitEvent(st, r->done, 0));
    if (where == GNS_MEM_HOST) {
        const uint64_t own_off = (n * stride + 15) & ~15ull;  // owners 16-byte aligned after odd-width keys
        const uint64_t need = own_off + n * 4;
        if (r->kbuf_n < need) {
            GNS_HIP(hipStreamSynchronize(st));
            dfree(r->kbuf); r->kbuf = nullptr; r->kbuf_n = 0;
            GNS_TRY(dalloc_t(&r->kbuf, need));
            r->kbuf_n = need;
        }
        GNS_HIP(hipMemcpyAsync(r->kbuf, keys, n * stride, hipMemcpyHostToDevice, st));
        a.keys = r->kbuf;
        a.owner = reinterpret_cast<uint32_t *>(r->kbuf + own_off);
    } else {
        a.keys = keys;
        a.owner = owner;
    }
    const uint32_t grid = (uint32_t)std::min<uint64_t>((n + 255) / 256, 4096);
    if (r->src_only)
        hipLaunchKernelGGL(k_route_keys<true>, dim3(grid), dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL(k_route_keys<false>, dim3(grid), dim3(256), 0, st, a);
    GNS_HIP(hipGetLastError());
    if (where == GNS_MEM_HOST) GNS_HIP(hipMemcpyAsync(owner, a.owner, n * 4, hipMemcpyDeviceToHost, st));
    GNS_HIP(hipStreamSynchronize(st));
    return GNS_OK;
}

}  // extern "C"
