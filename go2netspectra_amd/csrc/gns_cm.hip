// gns_cm.hip -- MI355X (gfx950) engine for Go2NetSpectra's fingerprinted
// "CountMin" (internal/engine/impl/sketch/statistic/count_min.go).
//
// Semantics: the device state after a sequence of inserts is bit-identical to
// count_min.go fed the same packets in the same order by ONE worker with the
// same row seeds.  Each bucket holds two independent
// (fingerprint, counter) pairs whose update rules are ORDER-DEPENDENT
// (count_min.go:99-155), so the engine never scatters with plain atomics.
//
// Pipeline per device batch:
//   K1 k_extract  : packet -> flow key (registers) -> flow id (exact dictionary)
//                   -> d row indices; per-block (row, tile) histograms.
//   K1b k_resolve : re-probe packets whose dictionary slot was claimed in the
//                   same launch (rare after the first batch).
//   K2 k_scan*    : exclusive scan of the histograms -> stable bin offsets.
//   K3 k_scatter  : stable partition of 8-byte bucket updates into (row, tile)
//                   bins (LDS-staged so every bin receives contiguous runs).
//   K4 k_apply    : persistent, one workgroup per CU taking bins from a work
//                   counter (largest first); the tile's bucket state lives in
//                   LDS; updates are applied chunk by chunk in stream order:
//                   order-free aggregate fast path where provably exact,
//                   sequential replay for the buckets where it is not.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <mutex>
#include <sys/resource.h>
#include <vector>

#include "gns_common.hpp"
#include "gns_ctl.cuh"
#include "gns_hh.hpp"
#include "gns_scan.cuh"
#include "gns_xcd.cuh"

namespace gns {

#ifndef GNS_TILE_BITS
#define GNS_TILE_BITS 12
#endif
#ifndef GNS_AP_THREADS
#define GNS_AP_THREADS 1024
#endif
#ifndef GNS_AP_ITEMS
#define GNS_AP_ITEMS 8
#endif
constexpr uint32_t kTileBitsMax = GNS_TILE_BITS;
constexpr uint32_t kTileMax = 1u << kTileBitsMax;   // buckets per LDS tile
constexpr uint32_t kMaxTilesPerRow = 1024;
// Update entry: lo = flow id (or kOvfFlag | overflow slot), hi = size << 16 | low,
// low = bucket within the (row, bin) range or the hot slot.  Sizes >= kSizeEsc
// take the overflow side table (and an exact replay); below it the per-chunk
// sums of K4 (kApChunk = 2^13 updates) stay under 2^32, so the packed
// own/foreign 32-bit halves of accS never carry.
constexpr uint32_t kEntShift = 16;
constexpr uint32_t kLowMask = (1u << kEntShift) - 1u;
constexpr uint32_t kSizeEsc = 0xFFFFu;
constexpr uint32_t kOvfFlag = 0x80000000u;
constexpr uint32_t kOvfCap = 1u << 20;             // initial overflow table (grows per batch as needed)
constexpr uint32_t kMaxBinsAll = 4096;               // d * bins per row (k_order, K3 LDS)
#ifndef GNS_EX_THREADS
#define GNS_EX_THREADS 256
#endif
constexpr int kExThreads = GNS_EX_THREADS;
constexpr size_t kExLdsSmall = 40 * 1024;             // K1 LDS above this: 1024-thread blocks
#ifndef GNS_CHUNK
#define GNS_CHUNK 16384
#endif
constexpr uint32_t kChunk = GNS_CHUNK;              // packets per K1/K3 block
// K1 packs a block's packet count (low 16 bits) and oversize count (high 16) in one word
static_assert(kChunk < 65536, "GNS_CHUNK must stay below 2^16 (K1's packed per-block counts)");
#ifndef GNS_SC_THREADS
#define GNS_SC_THREADS 512
#endif
constexpr int kScThreads = GNS_SC_THREADS;          // K3 block
constexpr int kScWaves = kScThreads / 64;
#ifndef GNS_SC_ITEMS
#define GNS_SC_ITEMS 8
#endif
constexpr int kScItems = GNS_SC_ITEMS;
constexpr uint32_t kScRound = kScThreads * kScItems; // 4096 updates staged in LDS per round
constexpr int kApThreads = GNS_AP_THREADS;
constexpr int kApWaves = kApThreads / 64;
constexpr int kApItems = GNS_AP_ITEMS;
constexpr uint32_t kApChunk = kApThreads * kApItems; // 8192 updates per K4 step
static_assert((uint64_t)kApChunk * (kSizeEsc - 1) < (1ull << 32), "K4 per-chunk size sums must fit 32 bits");
#ifndef GNS_HOT_BITS
#define GNS_HOT_BITS 7
#endif
constexpr uint32_t kHotBits = GNS_HOT_BITS;           // designated hot buckets per row = 2^kHotBits
constexpr uint32_t kHot = 1u << kHotBits;
#ifndef GNS_HOT_TAB_MUL
#define GNS_HOT_TAB_MUL 4
#endif
constexpr uint32_t kHotTab = kHot * GNS_HOT_TAB_MUL;  // lookup slots per row (load <= 1/GNS_HOT_TAB_MUL)
constexpr uint32_t kHotGroupBits = kHotBits + (GNS_HOT_TAB_MUL == 8 ? 1 : 0);  // 4-entry groups = kHotTab / 4
constexpr uint32_t kHotMinBits = 11;                // designate only buckets with C >= 1024
constexpr uint32_t kPendingId = 0xFFFFFFFEu;        // K1: flow not yet committed (equals no fingerprint)
constexpr uint32_t kStatsProf = 16;                 // engine stats words 16..31: profiling builds only

struct CmGeom {
    uint32_t w, d, wmask, pow2;
    uint32_t tile_bits, ntiles, nbins, nbits;  // nbits = ceil_log2(ntiles + kHot); ntiles = bins per row
    uint32_t bin_bits, sub_bits;               // bin = 2^sub_bits LDS tiles of 2^tile_bits buckets
    uint32_t nbins_all;                        // nbins + d*kHot (hot bins follow the tile bins)
    uint32_t blo, bspan;                       // bucket-range slice [blo, blo + bspan) applied by K4 (whole row: 0, w)
    uint32_t seeds[8];
};

// ---------------------------------------------------------------------------
// Designated hot buckets.  After every batch the buckets with the largest
// counters (a heavy flow's buckets) are designated for the next batch; their
// updates go to one bin per bucket, which the whole chip aggregates in
// parallel instead of one workgroup walking it.  Designation only moves work;
// exactness comes from the verify/fallback steps (k_hot_verify, k_hot_fallback).
// ---------------------------------------------------------------------------
// Per-row lookup table of the designated buckets, built once per batch by
// k_hot_table (deterministic: as if inserted in hot-slot order) and copied to LDS by K1:
// 128 groups of 4 entries (one 16-byte LDS read per lookup, no probing);
// entry = bucket << kHotBits | hot slot, empty = ~0.  A bucket whose group is full is
// simply not designated (designation only moves work).
static_assert(kHotTab / 4 == (1u << kHotGroupBits), "hot_group() yields kHotGroupBits bits");
__device__ __forceinline__ uint32_t hot_group(uint32_t b) { return (b * 0x9E3779B1u) >> (32 - kHotGroupBits); }

__device__ __forceinline__ int hot_lookup(const uint32_t *tabrow, uint32_t b) {
    const uint4 e = *reinterpret_cast<const uint4 *>(tabrow + hot_group(b) * 4);
    int h = -1;
    h = (e.w >> kHotBits) == b ? (int)(e.w & (kHot - 1u)) : h;
    h = (e.z >> kHotBits) == b ? (int)(e.z & (kHot - 1u)) : h;
    h = (e.y >> kHotBits) == b ? (int)(e.y & (kHot - 1u)) : h;
    h = (e.x >> kHotBits) == b ? (int)(e.x & (kHot - 1u)) : h;
    return h;
}

__device__ __forceinline__ uint32_t ceil_log2_dev(uint32_t x) { return x <= 1 ? 0u : 32u - __clz(x - 1u); }

__device__ __forceinline__ uint32_t row_index(const CmGeom &g, uint32_t h) {
    return g.pow2 ? (h & g.wmask) : (h % g.w);  // count_min.go:96 `% t.w`
}

// Per (hot slot, K1 block) summary of the block's updates to a designated
// bucket, relative to the batch-entry fingerprints (count_min.go:99-155):
// n updates, nfc / nfs of them foreign to the count / size owner, os / fs the
// owner / foreign size sums, smax the largest foreign size.  k_hot_decide
// turns them into the bucket's exact batch result without any per-update
// entry (hot updates are never scattered).
struct HotSum {
    uint32_t n, nfc, nfs, smax;
    unsigned long long os, fs;
};

// k_extract dynamic LDS: u64 os[S], fs[S] | u32 tab[d*kHotTab] | hist[nbins_all] |
// u32 hFc[S], hFs[S], nfc[S], nfs[S], smax[S]   (S = d*kHot hot slots)
__host__ __device__ inline size_t extract_lds_bytes(uint32_t nbins_all, uint32_t d) {
    return (size_t)d * kHot * 16 + ((size_t)nbins_all + d * kHotTab) * 4 + (size_t)d * kHot * 20;
}

// Counter words of stats[]: 0 inserted, 1 dropped, 2 unsupported, 3 dict-full, 4 ovf-full
struct ExtractArgs {
    InputDesc in;
    uint64_t n;
    KeyPlanN kp;
    CmGeom g;
    DictDev D;
    uint32_t epoch;
    uint32_t *keyid;
    uint32_t *idx;       // [d][n]
    uint64_t *pend;      // per-block regions of kChunk
    uint32_t *pend_cnt;  // [nblk]
    uint32_t *pend_total;
    uint32_t *hist;      // [nblk][nbins_all] (block-major)
    uint32_t nblk;
    const uint32_t *hot_ids;  // [d][kHot]
    const uint32_t *hot_tab;  // [d][kHotTab] lookup groups (k_hot_table)
    const uint32_t *Fc, *Fs;  // batch-entry fingerprints (hot slots' owners)
    HotSum *hsum;             // [d*kHot][nblk]
    unsigned long long *stats;
    // compact streams (CM kernels): per (block, K1 wave, row) the wave's
    // cold / hot row-updates in packet order, code = bucket (cold) or hot slot (hot)
    // << 12 | packet index within the wave's 4096-packet range; counts [blk][wave][row][2]
    uint32_t *cstr, *hstr, *scnt;
    uint32_t hoff;  // hstr - cstr (words)
};

// compact streams: a K1 wave owns kCsWave consecutive packets of its block
constexpr uint32_t kCsWaves = 4;                     // K1 waves per block (256 threads)
constexpr uint32_t kCsWave = kChunk / kCsWaves;      // packets per K1 wave = stream capacity
constexpr uint32_t kCsBits = 12;                     // packet index bits in a code
static_assert(kCsWave == (1u << kCsBits), "a code holds a 12-bit packet index");
constexpr uint32_t kCsNone = 0xFFFFFFFFu;

template <int KIND, int MODE>
__device__ __forceinline__ int packet_key(const InputDesc &in, uint32_t K, const uint8_t *s_src,
                                          uint64_t p, uint32_t (&kw)[GNS_KWMAX]) {
    if constexpr (KIND == IN_KEYS) {
        load_key_bytes<GNS_KWMAX>(in.keys + p * in.stride, K, (in.aligned & 1u) != 0, kw);
        return PARSE_OK;
    } else {
        uint32_t tw[10];
        const int st = load_tuple<KIND>(in, p, tw);
        if (st != PARSE_OK) return st;
        make_key_m<MODE, GNS_KWMAX>(K, s_src, tw, kw);
        return PARSE_OK;
    }
}

enum { CM_FOUND = 0, CM_PENDING = 1, CM_FULL = 2, CM_CLAIMED = 3 };

// Dictionary probe for the Count-Min engine: like dict_find_or_claim, but
// loads whole 64-byte records (r[] holds the found record, bucket cache
// included) and reports CM_CLAIMED when this lane inserted the key (the
// caller then writes the bucket words).  K is a compile-time constant in the
// specialized kernels.
template <int N>  // r: words 0..15 of the record (N >= 16)
__device__ __forceinline__ int cm_find_or_claim(const DictDev &D, const uint32_t (&kw)[GNS_KWMAX], uint32_t K,
                                                uint32_t slot, uint32_t epoch, uint32_t *out,
                                                uint32_t (&r)[N]) {
    static_assert(N >= 16, "record words 0..15");
    const uint32_t nkw = (K + 3) >> 2;
    for (int probe = 0; probe < GNS_DICT_MAX_PROBE; probe++) {
        const uint4 *q = reinterpret_cast<const uint4 *>(D.rec + (size_t)slot * D.RW);
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint4 v = (4u * i < D.RW) ? q[i] : make_uint4(0, 0, 0, 0);
            r[4 * i] = v.x; r[4 * i + 1] = v.y; r[4 * i + 2] = v.z; r[4 * i + 3] = v.w;
        }
        uint32_t tag = r[0];
        if (tag == 0) {
            uint32_t *tp = D.rec + (size_t)slot * D.RW;
            const uint32_t old = atomicCAS(tp, 0u, epoch);
            if (old == 0) {
#pragma unroll
                for (int i = 0; i < GNS_KWMAX; i++)
                    if ((uint32_t)i < nkw) tp[1 + i] = kw[i];
                *out = slot;
                return CM_CLAIMED;
            }
            tag = old;
            if (tag != epoch) {  // committed earlier: need its key words
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const uint4 v = (4u * i < D.RW) ? q[i] : make_uint4(0, 0, 0, 0);
                    r[4 * i] = v.x; r[4 * i + 1] = v.y; r[4 * i + 2] = v.z; r[4 * i + 3] = v.w;
                }
            }
        }
        if (tag == epoch) { *out = slot; return CM_PENDING; }
        bool eq = true;
#pragma unroll
        for (int i = 0; i < GNS_KWMAX; i++)
            if ((uint32_t)i < nkw) eq = eq && (r[1 + i] == kw[i]);
        if (eq) { *out = slot; return CM_FOUND; }
        slot = (slot + 1u) & D.mask;
    }
    return CM_FULL;
}

// Whole-wave sums through the device library's DPP reductions (row_shl /
// wave_shl / row_mirror, no LDS round trips).  Call with all 64 lanes active.
extern "C" __device__ unsigned long long __ockl_wfred_add_u64(unsigned long long);
extern "C" __device__ unsigned __ockl_wfred_add_u32(unsigned);
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) { return __ockl_wfred_add_u64(v); }

// K1 second half for one packet: resolve the first dictionary probe (r4,
// issued earlier by the caller), publish/hash the row buckets, bin codes,
// block histogram and designated-bucket summaries.
struct K1Lds {
    uint32_t *s_tab, *s_hist, *s_hFc, *s_hFs, *s_nfc, *s_nfs, *s_smax, *s_pend, *s_full, *s_claim;
    unsigned long long *s_os, *s_fs;
};

// Wave-uniform running lengths of the wave's compact streams (CM kernels), per row:
// cold count in the low 16 bits, hot count in the high 16 (each <= kCsWave).
template <int RMAX>
struct CsRun {
    uint32_t ch[RMAX];
    uint32_t sb;  // stream base of row 0 (uniform)
};

// record quads a K1 probe loads: words 0..15, and 16..19 (rows 4..7 of the bucket cache) for deep sketches
template <int RMAX>
constexpr int kProbeQuads = RMAX > 4 ? 5 : 4;

template <int RMAX, bool CM>
__device__ __forceinline__ void k1_consume(const ExtractArgs &a, const K1Lds &S, uint32_t K, uint32_t d, bool bw,
                                           uint64_t p, uint64_t beg, bool ok, const uint32_t (&kw)[GNS_KWMAX],
                                           uint32_t slot0, const uint4 (&r4)[kProbeQuads<RMAX>], uint32_t sz,
                                           uint32_t &n_ok, CsRun<RMAX> &cs) {
    constexpr int NQ = kProbeQuads<RMAX>;
    uint32_t *s_tab = S.s_tab, *s_hist = S.s_hist, *s_hFc = S.s_hFc, *s_hFs = S.s_hFs, *s_nfc = S.s_nfc;
    uint32_t *s_nfs = S.s_nfs, *s_smax = S.s_smax;
    unsigned long long *s_os = S.s_os, *s_fs = S.s_fs;
    uint32_t &s_pend = *S.s_pend, &s_full = *S.s_full;
    uint32_t kid = kPendingId;  // flow id when already committed (pending: foreign to every owner)
    uint32_t rec[4 * NQ];
    int res = CM_FULL;
    uint32_t out = 0;
    // first probe (the home slot, loaded by the caller): 0 hit, 1 claimed in this
    // launch, 2 empty, 3 another committed key (the key lies further along the chain)
    int first = 0;
    if (ok) {
#pragma unroll
        for (int i = 0; i < NQ; i++) {
            rec[4 * i] = r4[i].x; rec[4 * i + 1] = r4[i].y; rec[4 * i + 2] = r4[i].z; rec[4 * i + 3] = r4[i].w;
        }
        const uint32_t tag = rec[0];
        bool eq = tag != 0 && tag != a.epoch;
#pragma unroll
        for (int i = 0; i < GNS_KWMAX; i++)
            if ((uint32_t)i < ((K + 3) >> 2)) eq = eq && (rec[1 + i] == kw[i]);
        first = tag == a.epoch ? 1 : (eq ? 0 : (tag == 0 ? 2 : 3));
#ifdef GNS_K1_ABL_DICT
        (void)tag;
        first = 0;  // timing ablation: every packet "found" at its (in-range) probe slot
        rec[12] = rec[13] = rec[14] = rec[15] = 0;
#endif
        if (first == 0) { res = CM_FOUND; out = slot0; }
        else if (first == 1) { res = CM_PENDING; out = slot0; }
    }
    // row buckets: from the record's cache (rows 0..3 of a committed flow, 0..7 in a
    // 32-word record), else hashed
    uint32_t bk[RMAX];
#ifdef GNS_K1_ABL_DICT
    const bool cached = false;  // buckets hashed: the ablation's record holds no cache
#else
    const bool cached = bw && ok && first == 0;
#endif
    const uint32_t nc = (NQ > 4 && a.D.RW >= 32) ? 8u : 4u;  // cached rows
#pragma unroll
    for (uint32_t rr = 0; rr < RMAX; rr++) bk[rr] = (rr < nc && cached) ? rec[12 + rr] : 0u;
    if (__ballot(ok && !cached) || (RMAX > 4 && d > nc)) {
        uint32_t mk[GNS_KWMAX];
        mm3_premix<GNS_KWMAX>(kw, K, mk);
#pragma unroll
        for (uint32_t rr = 0; rr < RMAX; rr++) {
            if (rr >= d) break;
            if (ok && (!cached || rr >= nc)) bk[rr] = row_index(a.g, mm3_chain<GNS_KWMAX>(mk, K, a.g.seeds[rr]));
        }
    }
    // designated-bucket slots of the row buckets (LDS lookups, reused by the rows loop)
    int hs[RMAX];
    bool anyhot = false;
#pragma unroll
    for (uint32_t rr = 0; rr < RMAX; rr++) {
        hs[rr] = -1;
        if (rr >= d) break;
        if (ok) hs[rr] = hot_lookup(s_tab + rr * kHotTab, bk[rr]);
        anyhot = anyhot || hs[rr] >= 0;
    }
    if (ok && first >= 2) {
        // A flow whose home slot is empty is new: it is parked for k_resolve, which
        // claims it (and counts the claim against the dictionary cap; K1 stays at
        // 128 VGPRs without spills only without that code).  A committed flow
        // displaced from its home slot is parked too (k_resolve walks the rest of
        // the chain next launch; its bucket codes are already hashed) instead of
        // stalling the wave on a dependent probe.  The summaries treat a parked
        // packet as foreign to every owner, which is exact only for a flow that owns
        // no bucket (a new one does not): so a displaced packet that touches a
        // designated bucket walks the chain here (its rare claims count against the
        // dictionary cap like k_resolve's, so the 3/4-load bound holds).
        if (first == 2 || !anyhot) { res = CM_PENDING; out = first == 2 ? slot0 : ((slot0 + 1u) & a.D.mask); }
        else {
            res = cm_find_or_claim(a.D, kw, K, (slot0 + 1u) & a.D.mask, a.epoch, &out, rec);
            if (res == CM_CLAIMED) atomicAdd(S.s_claim, 1u);
        }
    }
    if (ok) {
        if (res == CM_FULL) {
            a.keyid[p] = GNS_ID_NONE;
            atomicAdd(&s_full, 1u);
            ok = false;
        } else if (res == CM_PENDING) {
            a.keyid[p] = GNS_ID_NONE;  // set by k_resolve
            const uint32_t q = atomicAdd(&s_pend, 1u);
            a.pend[beg + q] = (uint64_t)(p - beg) << 32 | out;
        } else {
            a.keyid[p] = out;
            kid = out;
        }
    }

    if (bw && res == CM_CLAIMED) {  // publish the bucket cache with the key (visible next launch)
        uint32_t *tp = a.D.rec + (size_t)out * a.D.RW;
#pragma unroll
        for (uint32_t rr = 0; rr < RMAX; rr++)
            if (rr < d && rr < nc) tp[12 + rr] = bk[rr];
    }
    if (!ok) sz = 0;
    // low 16 bits: packets inserted; high 16: of them with a size taking the
    // overflow side table (a block has <= kChunk packets, so neither carries)
    n_ok += (ok ? 1u : 0u) + (sz >= kSizeEsc ? 0x10000u : 0u);
#pragma unroll
    for (uint32_t rr = 0; rr < RMAX; rr++) {
        if (rr >= d) break;
        uint32_t binid = 0xFFFFFFFFu;
        int h = -1;
        if (ok) {
            const uint32_t b = bk[rr];
            h = hs[rr];
            // bin code for K3: bucket, or 1<<31 | hot slot for a designated bucket
            if constexpr (!CM) a.idx[(uint64_t)rr * a.n + p] = h >= 0 ? (0x80000000u | (uint32_t)h) : b;
            binid = h >= 0 ? a.g.nbins + rr * kHot + (uint32_t)h : rr * a.g.ntiles + (b >> a.g.bin_bits);
        }
        if constexpr (CM) {
            // compact streams: this wave's cold and hot row-rr updates, appended in packet
            // order (the wave's lanes hold consecutive packets), so K3 reads only the
            // updates it partitions and no per-packet code array exists
            // (the hot streams follow the cold ones in one buffer: hstr = cstr + a.hoff)
            const bool cold = ok && h < 0, hot = ok && h >= 0;
            const uint64_t mc = __ballot(cold), mh = __ballot(hot);
            const uint32_t run = cs.ch[rr];
            const uint32_t pc = __builtin_amdgcn_mbcnt_hi((uint32_t)(mc >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mc, 0u));
            const uint32_t ph = __builtin_amdgcn_mbcnt_hi((uint32_t)(mh >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mh, 0u));
            const uint32_t pos = cold ? (run & 0xFFFFu) + pc : a.hoff + (run >> 16) + ph;
            // packet index within the wave's range: the wave's range starts at a multiple of kCsWave
            const uint32_t code = (cold ? bk[rr] : (uint32_t)h) << kCsBits | ((uint32_t)p & (kCsWave - 1u));
            if (ok) a.cstr[cs.sb + rr * kCsWave + pos] = code;
            cs.ch[rr] = run + (uint32_t)__popcll(mc) + ((uint32_t)__popcll(mh) << 16);
        }
        // heavy bins: one LDS add for the wave's majority bin
        const uint32_t b0 = __builtin_amdgcn_readfirstlane(binid);
        const uint64_t mm = __ballot(binid == b0 && b0 != 0xFFFFFFFFu);
        const uint32_t cnt = __popcll(mm);
        const bool agg = cnt >= 4;  // wave-uniform
        const bool inmaj = agg && binid == b0;
        const bool leader = inmaj && (uint32_t)__ffsll((long long)mm) - 1 == (threadIdx.x & 63u);
        if (leader) atomicAdd(&s_hist[b0], cnt);
        if (binid != 0xFFFFFFFFu && !inmaj) atomicAdd(&s_hist[binid], 1u);
        // designated bucket: summary against the batch-entry owners
        uint64_t ownv = 0;
        if (h >= 0) {
            const uint32_t slot = rr * kHot + (uint32_t)h;
            if (kid != s_hFc[slot]) atomicAdd(&s_nfc[slot], 1u);
            if (kid != s_hFs[slot]) {
                atomicAdd(&s_nfs[slot], 1u);
                atomicAdd(&s_fs[slot], (unsigned long long)sz);
                atomicMax(&s_smax[slot], sz);
            } else {
                ownv = sz;
            }
        }
        if (agg && b0 >= a.g.nbins && b0 != 0xFFFFFFFFu) {  // wave-uniform: majority bin is hot
            const uint64_t tot = wave_sum64(inmaj ? ownv : 0ull);
            if (leader && tot) atomicAdd(&s_os[b0 - a.g.nbins], (unsigned long long)tot);
            if (!inmaj && ownv) atomicAdd(&s_os[binid - a.g.nbins], (unsigned long long)ownv);
        } else if (ownv) {
            atomicAdd(&s_os[binid - a.g.nbins], (unsigned long long)ownv);
        }
    }
}

// K1: parse/encode, dictionary, row buckets, block histogram, hot summaries.
// KB = key bytes when known at compile time (16 / 37), 0 = runtime a.kp.K.
// DD = depth when known at compile time (4: the rows loops unroll exactly), 0 = runtime
#ifndef GNS_EX_MINW
#define GNS_EX_MINW 4
#endif
// K1 at configs[4]'s geometry (d=8, 5-tuple key), A/B on one box (round 2-3 one-off scripts, retired):
//   two-stage pipeline, 1024 threads: 128 VGPRs + 66 spilled          5.42 ms / 100M
//   two-stage pipeline,  768 threads: 148 VGPRs, 12 waves per CU      4.47-4.50
//   plain loop,          768 threads:  92 VGPRs                        4.58-4.59
//   plain loop,          640 threads (two blocks per CU by LDS)        5.28-5.30
//   plain loop,         1024 threads:  93 VGPRs, 16 waves per CU      4.01-4.02
//   plain loop,          512 threads:  95 VGPRs, two blocks per CU    3.52        <- default
//     (round 3, same box, base 4.02-4.03; two independent
//     blocks per CU overlap one block's LDS set-up / flush and barriers with the
//     other's loop; the summaries' LDS atomics are what a lone block exposes:
//     timing ablations without them 4.06 -> 3.50, without the cold-bin histogram
//     adds 3.60.  Reducing each designated bucket's lanes
//     across the wave before one leader's atomics (tried in round 3) measured slower:
//     4.46 vs 4.02 here, 2.36 vs 2.22 at d=4; so did size sums as two 32-bit halves,
//     3.86 vs 3.55 here and 3.28 vs 2.37 at d=4.  The plain loop
//     at d=4 with five waves per SIMD (GNS_C2_PIPE=0 GNS_EX_MINW=5): 2.49 vs 2.37)
#ifndef GNS_K1_V4HASH
#define GNS_K1_V4HASH 1  // A/B: 0 hashes every wave's 5-tuple key generically
#endif
#ifndef GNS_C5_THREADS
#define GNS_C5_THREADS 512
#endif
constexpr int kC5Threads = GNS_C5_THREADS;
#ifndef GNS_C5_PIPE
#define GNS_C5_PIPE 0
#endif
constexpr bool kC5Pipe = GNS_C5_PIPE != 0;
#ifndef GNS_C2_PIPE
#define GNS_C2_PIPE 1
#endif
constexpr bool kC2Pipe = GNS_C2_PIPE != 0;  // the two-stage pipeline for d != 8 header records
// NT = threads per block: 256 (four blocks per CU) when the block's LDS fits four
// times in a CU, else 1024 (one block of 16 waves: wide or deep sketches, whose
// histogram and hot-slot tables take more than a quarter of the LDS).
// CM: compact streams instead of the per-packet code array (256-thread blocks only);
// then each wave takes a contiguous quarter of the block's packets, 64 at a time.
template <int KIND, int MODE, int KB, int DD, int NT, bool CM = false>
__global__ __launch_bounds__(NT, NT == 256 ? GNS_EX_MINW : (NT == 512 ? 2 : 1)) void k_extract(ExtractArgs a) {
    static_assert(!CM || NT == 256, "compact streams: four waves per block");
    constexpr bool WC = CM;  // (the classic outputs with this loop measured the same: 2.38 vs 2.35 ms)
    extern __shared__ __attribute__((aligned(16))) uint8_t xsm[];
    __shared__ uint32_t s_pend, s_drop, s_unsup, s_full, s_ok, s_claim;
    __shared__ uint8_t s_src[80];
#ifdef GNS_K1_XCD
    const uint32_t tid = threadIdx.x, blk = xcd_block(blockIdx.x, gridDim.x);  // A/B
#else
    const uint32_t tid = threadIdx.x, blk = blockIdx.x;
#endif
    const uint32_t NS = a.g.d * kHot;
    unsigned long long *s_os = reinterpret_cast<unsigned long long *>(xsm);
    unsigned long long *s_fs = s_os + NS;
    uint32_t *s_tab = reinterpret_cast<uint32_t *>(s_fs + NS);  // 16-byte aligned groups
    uint32_t *s_hist = s_tab + a.g.d * kHotTab;
    uint32_t *s_hFc = s_hist + a.g.nbins_all;
    uint32_t *s_hFs = s_hFc + NS, *s_nfc = s_hFs + NS, *s_nfs = s_nfc + NS, *s_smax = s_nfs + NS;
    stage_plan<MODE>(a.kp, s_src);
    const uint32_t K = KB ? (uint32_t)KB : a.kp.K;
    const uint32_t d = DD ? (uint32_t)DD : a.g.d;
    constexpr uint32_t RMAX = DD ? (uint32_t)DD : 8u;
    for (uint32_t i = tid; i < d * kHotTab; i += NT) s_tab[i] = a.hot_tab[i];
    for (uint32_t i = tid; i < a.g.nbins_all; i += NT) s_hist[i] = 0;
    for (uint32_t i = tid; i < NS; i += NT) {
        const uint32_t id = a.hot_ids[i];
        const uint64_t cell = (uint64_t)(i / kHot) * a.g.w + id;
        s_hFc[i] = id != GNS_ID_NONE ? a.Fc[cell] : GNS_ID_NONE;
        s_hFs[i] = id != GNS_ID_NONE ? a.Fs[cell] : GNS_ID_NONE;
        s_nfc[i] = 0; s_nfs[i] = 0; s_smax[i] = 0; s_os[i] = 0; s_fs[i] = 0;
    }
    if (tid == 0) { s_pend = 0; s_drop = 0; s_unsup = 0; s_full = 0; s_ok = 0; s_claim = 0; }
    __syncthreads();
    const uint64_t beg = (uint64_t)blk * kChunk;
    const uint64_t end = min(a.n, beg + kChunk);
    const bool bw = a.D.bw != 0;
    uint32_t n_ok = 0;
    const K1Lds S{s_tab, s_hist, s_hFc, s_hFs, s_nfc, s_nfs, s_smax, &s_pend, &s_full, &s_claim, s_os, s_fs};
    // lane's packets: classic p = beg + tid, beg + tid + NT, ...; CM: the wave's range
    // [wbeg, wend), p = wbeg + lane, + 64, ...  (wave-uniform trip counts either way)
    constexpr uint32_t STEP = WC ? 64u : (uint32_t)NT;
    const uint64_t wbeg = WC ? beg + (uint64_t)(tid >> 6) * (kChunk / (NT / 64)) : beg;
    const uint64_t wend = WC ? min(end, wbeg + kChunk / (NT / 64)) : end;
    const uint32_t loff = WC ? (tid & 63u) : tid;
    CsRun<RMAX> cs;
#pragma unroll
    for (uint32_t rr = 0; rr < RMAX; rr++) cs.ch[rr] = 0;
    cs.sb = (blk * kCsWaves + (tid >> 6)) * d * kCsWave;
    if constexpr (KIND == IN_HDR && (DD == 8 ? kC5Pipe : kC2Pipe)) {
        // Two-stage software pipeline over the block's packets: iteration k
        // parses packet k+1 and issues its dictionary probe (and the header
        // prefetch of packet k+2), then consumes packet k, whose probe was
        // issued one iteration earlier.  Probe and header latencies hide behind
        // a whole iteration of work instead of stalling it.
        uint4 hv[4];
        uint32_t hsz;
        auto load_hdr = [&](uint64_t q) {
            const uint64_t pc = min(q, end - 1);  // (end - 1 >= beg: a block has packets)
            const uint4 *r = reinterpret_cast<const uint4 *>(a.in.hdr + pc * 16);
#pragma unroll
            for (int i = 0; i < 4; i++) hv[i] = r[i];
            hsz = a.in.sizes[pc];
        };
        // stage B of packet q: parse the prefetched record, key, slot, issue the probe
        constexpr int NQ = kProbeQuads<RMAX>;
        auto stage_b = [&](uint64_t q, bool &okq, uint32_t (&kwq)[GNS_KWMAX], uint32_t &slotq, uint4 (&r4q)[NQ],
                           uint32_t &szq) {
            okq = q < wend;
            uint32_t cw[16];
#pragma unroll
            for (int i = 0; i < 4; i++) { cw[4 * i] = hv[i].x; cw[4 * i + 1] = hv[i].y; cw[4 * i + 2] = hv[i].z; cw[4 * i + 3] = hv[i].w; }
            szq = hsz;
            load_hdr(q + STEP);
            if (okq) {
                uint32_t tw[10];
                const int st = parse_record_fast(cw, szq, true, tw);
                if (st == PARSE_OK) make_key_m<MODE, GNS_KWMAX>(K, s_src, tw, kwq);
                else {
                    a.keyid[q] = GNS_ID_NONE;
                    atomicAdd(st == PARSE_DROP ? &s_drop : &s_unsup, 1u);
                    okq = false;
                }
            }
            uint32_t mk[GNS_KWMAX];
            // the 5-tuple key (PLAN_SLICE0, 37 bytes) of an IPv4 packet has six zero words
            // (the address slots' upper 12 bytes): when the whole wave is IPv4 they are
            // hashed as constants, which folds their mixing and chain steps (same slot)
            bool v4w = false;
            if constexpr (GNS_K1_V4HASH && MODE == PLAN_SLICE0 && KB == 37 && GNS_KWMAX >= 10) {
                const bool wide = okq && (kwq[1] | kwq[2] | kwq[3] | kwq[5] | kwq[6] | kwq[7]) != 0;
                v4w = __ballot(wide) == 0;  // wave-uniform
            }
            if (v4w) {
                uint32_t k4[GNS_KWMAX];
#pragma unroll
                for (int i = 0; i < GNS_KWMAX; i++) k4[i] = 0;
                k4[0] = kwq[0]; k4[4] = kwq[4]; k4[8] = kwq[8]; k4[9] = kwq[9];
                mm3_premix<GNS_KWMAX>(k4, K, mk);
                slotq = mm3_chain<GNS_KWMAX>(mk, K, a.D.seed) & a.D.mask;
            } else {
                mm3_premix<GNS_KWMAX>(kwq, K, mk);
                slotq = mm3_chain<GNS_KWMAX>(mk, K, a.D.seed) & a.D.mask;
            }
#ifdef GNS_K1_ABL_DICT
            // TIMING ABLATION ONLY (wrong counters; never a product build, tools/r06_k1abl.sh):
            // the probe reads one of the table's first 4096 records (256 KB, L2-resident), so
            // K1 keeps its streams, hashing, histogram and summaries but pays no dictionary miss
            slotq &= 4095u;
#endif
            if (okq) {
                const uint4 *rq = reinterpret_cast<const uint4 *>(a.D.rec + (size_t)slotq * a.D.RW);
#pragma unroll
                for (int i = 0; i < NQ; i++) r4q[i] = (4u * i < a.D.RW) ? rq[i] : make_uint4(0, 0, 0, 0);
            }
        };
        load_hdr(wbeg + loff);
        bool okc;
        uint32_t kwc[GNS_KWMAX], slotc, szc;
        uint4 r4c[NQ];
        stage_b(wbeg + loff, okc, kwc, slotc, r4c, szc);
        for (uint64_t p0 = wbeg; p0 < wend; p0 += STEP) {  // wave-uniform trip count
            bool okn = false;
            uint32_t kwn[GNS_KWMAX], slotn = 0, szn = 0;
            uint4 r4n[NQ];
            if (p0 + STEP < wend) stage_b(p0 + STEP + loff, okn, kwn, slotn, r4n, szn);
            k1_consume<RMAX, CM>(a, S, K, d, bw, p0 + loff, beg, okc, kwc, slotc, r4c, szc, n_ok, cs);
            okc = okn; slotc = slotn; szc = szn;
#pragma unroll
            for (int i = 0; i < GNS_KWMAX; i++) kwc[i] = kwn[i];
#pragma unroll
            for (int i = 0; i < NQ; i++) r4c[i] = r4n[i];
        }
    } else {
        for (uint64_t p0 = wbeg; p0 < wend; p0 += STEP) {  // wave-uniform trip count
            const uint64_t p = p0 + loff;
            bool ok = p < wend;
            uint32_t kw[GNS_KWMAX];
            if (ok) {
                const int st = packet_key<KIND, MODE>(a.in, K, s_src, p, kw);
                if (st != PARSE_OK) {
                    a.keyid[p] = GNS_ID_NONE;
                    atomicAdd(st == PARSE_DROP ? &s_drop : &s_unsup, 1u);
                    ok = false;
                }
            }
            uint32_t slot0;
            {
                uint32_t mk[GNS_KWMAX];
                mm3_premix<GNS_KWMAX>(kw, K, mk);
                slot0 = mm3_chain<GNS_KWMAX>(mk, K, a.D.seed) & a.D.mask;
            }
            uint4 r4[kProbeQuads<RMAX>];
            if (ok) {
                const uint4 *q = reinterpret_cast<const uint4 *>(a.D.rec + (size_t)slot0 * a.D.RW);
#pragma unroll
                for (int i = 0; i < kProbeQuads<RMAX>; i++) r4[i] = (4u * i < a.D.RW) ? q[i] : make_uint4(0, 0, 0, 0);
            }
            k1_consume<RMAX, CM>(a, S, K, d, bw, p, beg, ok, kw, slot0, r4, ok ? a.in.sizes[p] : 0u, n_ok, cs);
        }
    }
    if constexpr (CM) {  // the wave's stream lengths
        if ((tid & 63u) == 0) {
            uint32_t *sc = a.scnt + ((uint64_t)blk * kCsWaves + (tid >> 6)) * d * 2;
#pragma unroll
            for (uint32_t rr = 0; rr < RMAX; rr++)
                if (rr < d) { sc[rr * 2] = cs.ch[rr] & 0xFFFFu; sc[rr * 2 + 1] = cs.ch[rr] >> 16; }
        }
    }
    atomicAdd(&s_ok, n_ok);
    __syncthreads();
    for (uint32_t i = tid; i < a.g.nbins_all; i += NT) a.hist[(uint64_t)blk * a.g.nbins_all + i] = s_hist[i];
    for (uint32_t i = tid; i < NS; i += NT) {
        HotSum hs;
        hs.n = s_hist[a.g.nbins + i]; hs.nfc = s_nfc[i]; hs.nfs = s_nfs[i]; hs.smax = s_smax[i];
        hs.os = s_os[i]; hs.fs = s_fs[i];
        a.hsum[(uint64_t)i * a.nblk + blk] = hs;
    }
    if (tid == 0) {
        a.pend_cnt[blk] = s_pend;
        if (s_pend) atomicAdd(a.pend_total, s_pend);
        if (s_ok & 0xFFFFu) atomicAdd(&a.stats[0], (unsigned long long)(s_ok & 0xFFFFu));
        if (s_ok >> 16) atomicAdd(&a.stats[8], (unsigned long long)(s_ok >> 16));
        if (s_drop) atomicAdd(&a.stats[1], (unsigned long long)s_drop);
        if (s_unsup) atomicAdd(&a.stats[2], (unsigned long long)s_unsup);
        if (s_full) atomicAdd(&a.stats[3], (unsigned long long)s_full);
        dict_flush_claims(a.D, s_claim, &a.stats[3]);
    }
}

struct ResolveArgs {
    InputDesc in;
    uint64_t n;
    KeyPlanN kp;
    DictDev D;
    uint32_t epoch;
    uint32_t *keyid;
    const uint64_t *pend_in;
    const uint32_t *cnt_in;
    uint64_t *pend_out;
    uint32_t *cnt_out;
    uint32_t *total_out;
    uint32_t *total_in;  // zeroed by this round: the next round's total_out (read by the host before)
    unsigned long long *stats;
    CmGeom g;
};

// K1b: packets parked on a slot claimed in the previous launch.
template <int KIND, int MODE>
__global__ __launch_bounds__(kExThreads) void k_resolve(ResolveArgs a) {
    __shared__ uint32_t s_cnt, s_full, s_claim, s_abort;
    __shared__ uint8_t s_src[80];
    const uint32_t tid = threadIdx.x, blk = blockIdx.x;
    if (blk == 0 && tid == 0) *a.total_in = 0u;
    const uint32_t cnt = a.cnt_in[blk];
    if (cnt == 0) {  // block-uniform
        if (tid == 0) a.cnt_out[blk] = 0;
        return;
    }
    if (tid == 0) { s_cnt = 0; s_full = 0; s_claim = 0; s_abort = dict_aborted(a.D); }
    __syncthreads();
    if (s_abort) {
        if (tid == 0) a.cnt_out[blk] = 0;
        return;
    }
    stage_plan<MODE>(a.kp, s_src);
    const uint64_t beg = (uint64_t)blk * kChunk;
    for (uint32_t i = tid; i < cnt; i += kExThreads) {
        const uint64_t v = a.pend_in[beg + i];
        const uint64_t p = beg + (v >> 32);
        uint32_t kw[GNS_KWMAX];
        (void)packet_key<KIND, MODE>(a.in, a.kp.K, s_src, p, kw);
        uint32_t out, rec[16];
        const int r = cm_find_or_claim(a.D, kw, a.kp.K, (uint32_t)v, a.epoch, &out, rec);
        if (r == CM_FOUND || r == CM_CLAIMED) {
            a.keyid[p] = out;
            if (r == CM_CLAIMED) atomicAdd(&s_claim, 1u);
            if (r == CM_CLAIMED && a.D.bw) {  // bucket cache, as in k_extract
                uint32_t mk[GNS_KWMAX];
                mm3_premix<GNS_KWMAX>(kw, a.kp.K, mk);
                uint32_t *tp = a.D.rec + (size_t)out * a.D.RW;
                const uint32_t nc = a.D.RW >= 32 ? 8u : 4u;  // cached rows
                for (uint32_t rr = 0; rr < nc && rr < a.g.d; rr++)
                    tp[12 + rr] = row_index(a.g, mm3_chain<GNS_KWMAX>(mk, a.kp.K, a.g.seeds[rr]));
            }
        } else if (r == CM_PENDING) {
            const uint32_t q = atomicAdd(&s_cnt, 1u);
            a.pend_out[beg + q] = (v & 0xFFFFFFFF00000000ull) | out;
        } else {
            atomicAdd(&s_full, 1u);
        }
    }
    __syncthreads();
    if (tid == 0) {
        a.cnt_out[blk] = s_cnt;
        if (s_cnt) atomicAdd(a.total_out, s_cnt);
        if (s_full) atomicAdd(&a.stats[3], (unsigned long long)s_full);
        dict_flush_claims(a.D, s_claim, &a.stats[3]);
    }
}

// K2 (the block-major histogram scan) and wave_incl_scan: gns_scan.cuh

// ---------------------------------------------------------------------------
// K3: stable partition of row r's bucket updates into its tile bins.
// Entry (u64): lo = flow id (or kOvfFlag|ovf slot), hi = size<<12 | bucket&(tile-1)
// Per step (4096 packets, one row): stable rank of every update among the
// wave's updates to the same bin (returning LDS adds), per-bin prefix over the
// waves (= the global slot of each wave's run), then each update is stored
// straight to its slot.  Two barriers per step; the counters are
// double-buffered so the next step needs no barrier before counting.
// ---------------------------------------------------------------------------
struct ScatterArgs {
    uint64_t n;
    uint32_t xcd_map;  // K3s: consecutive K1 blocks to workgroups on one XCD (GNS_K3_XCD=0: off)
    CmGeom g;
    const uint32_t *keyid;
    const uint32_t *idx;
    const uint32_t *sizes;
    const uint32_t *offsets;  // scanned hist
    uint32_t nblk;
    uint64_t *entries;
    uint64_t *ovf;
    uint32_t *ovf_cnt;
    uint32_t ovf_cap;         // entries ovf holds (>= d * the batch's oversize packets)
    const uint32_t *hot_ids;
    unsigned long long *stats;
    // hot_mode 0: tile bins only (designated buckets are summarized by K1);
    // 1: only the hot slots flagged for the exact fallback (hflag2 & 3), and
    // only when *hany (the whole grid exits otherwise).
    uint32_t hot_mode;
    const uint32_t *hflag2;
    const uint32_t *hany;
    // compact streams (k_scatter_cs, k_hot_scatter_cs): K1's per-(block, wave, row) codes
    const uint32_t *cstr, *hstr, *scnt;
};

// LDS layout of k_scatter (dynamic): s_cnt[2][kScWaves][LB] (double-buffered), s_goff[d][LB],
// s_dummy[kScThreads] (rank adds of lanes without an update)
__host__ __device__ inline size_t scatter_lds_bytes(uint32_t LB, uint32_t d) {
    return (size_t)(2 * kScWaves + d) * LB * 4 + kScThreads * 4;
}

#ifdef GNS_K3_PROF
#define K3_MARK(i) do { if (threadIdx.x == 0) { const uint64_t tn_ = __builtin_amdgcn_s_memtime(); k3t[i] += tn_ - k3prev; k3prev = tn_; } } while (0)
#else
#define K3_MARK(i) do { } while (0)
#endif
// RANK 1: stable per-wave ranks from returning LDS adds; 0: ballot multisplit
// (used when the lane-order probe fails on this device).
template <int RANK>
__global__ __launch_bounds__(kScThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_scatter(ScatterArgs a) {
#ifdef GNS_K3_PROF
    uint64_t k3t[5] = {0, 0, 0, 0, 0}, k3prev = __builtin_amdgcn_s_memtime();
#endif
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t LB = a.g.ntiles + kHot;  // local bins of a row: tiles, then its hot buckets
    const uint32_t d = a.g.d;
    uint32_t *s_cnt2 = reinterpret_cast<uint32_t *>(smem);  // [2][kScWaves][LB]
    uint32_t *s_goff = s_cnt2 + 2 * kScWaves * LB;          // [d][LB]
    uint32_t *s_dummy = s_goff + d * LB;                    // [kScThreads]
    uint32_t par = 0;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t blk = blockIdx.x;
    const uint32_t tmask = (1u << a.g.bin_bits) - 1u;
    const uint64_t beg = (uint64_t)blk * kChunk;
    const uint64_t end = min(a.n, beg + kChunk);
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    if (a.hot_mode && *a.hany == 0) return;
    const uint32_t nbits = a.hot_mode ? a.g.nbits : ceil_log2_dev(a.g.ntiles);
    for (uint32_t i = tid; i < d * LB; i += kScThreads) {
        const uint32_t r = i / LB, t = i % LB;
        const uint64_t gb = t < a.g.ntiles ? (uint64_t)(r * a.g.ntiles + t)
                                           : (uint64_t)(a.g.nbins + r * kHot + (t - a.g.ntiles));
        s_goff[i] = a.offsets[(uint64_t)blk * a.g.nbins_all + gb];
    }
    for (uint32_t t = tid; t < 2 * kScWaves * LB; t += kScThreads) s_cnt2[t] = 0;
    // bin codes of the next two (round, row) steps are in flight while a step
    // runs (K3 is latency-bound: bytes in flight, not bandwidth)
    uint32_t bsn[kScItems];
#pragma unroll
    for (int i = 0; i < kScItems; i++) {
        const uint64_t p = beg + (uint64_t)wave * 64 * kScItems + (uint64_t)i * 64 + lane;
        bsn[i] = a.idx[p < end ? p : end - 1];
    }
    // and the step after it (two steps in flight)
    uint32_t bsn2[kScItems];
    {
        const uint32_t r1 = d > 1 ? 1u : 0u;
        const uint64_t rb1 = d > 1 ? beg : beg + kScRound;
        if (rb1 < end) {
#pragma unroll
            for (int i = 0; i < kScItems; i++) {
                const uint64_t p = rb1 + (uint64_t)wave * 64 * kScItems + (uint64_t)i * 64 + lane;
                bsn2[i] = a.idx[(uint64_t)r1 * a.n + (p < end ? p : end - 1)];
            }
        }
    }
    // flow ids and sizes once per round, loaded one round ahead (clamped loads)
    uint32_t idsn[kScItems], szsn[kScItems];
    auto load_ids = [&](uint64_t rb) {
#pragma unroll
        for (int i = 0; i < kScItems; i++) {
            const uint64_t p = rb + (uint64_t)wave * 64 * kScItems + (uint64_t)i * 64 + lane;
            const uint64_t pc = p < end ? p : end - 1;
            idsn[i] = p < end ? a.keyid[pc] : GNS_ID_NONE;
            szsn[i] = a.sizes[pc];
        }
    };
    load_ids(beg);
    for (uint64_t rb = beg; rb < end; rb += kScRound) {
        uint32_t ids[kScItems], szs[kScItems];
#pragma unroll
        for (int i = 0; i < kScItems; i++) { ids[i] = idsn[i]; szs[i] = szsn[i]; }
        if (rb + kScRound < end) load_ids(rb + kScRound);
        for (uint32_t r = 0; r < d; r++) {
            // no barrier needed here: this step's count buffer was cleared in the
            // previous step's phase 2, which a barrier closed
            uint32_t *s_cnt = s_cnt2 + par * kScWaves * LB;
            uint32_t *s_cnto = s_cnt2 + (par ^ 1u) * kScWaves * LB;
            par ^= 1u;
            if (r == 0 && rb == beg) __syncthreads();  // s_goff / buffers initialised
            uint32_t bs[kScItems];
#pragma unroll
            for (int i = 0; i < kScItems; i++) bs[i] = bsn[i];
            {
                // (nrb, nr) = the step after the next one
                const uint64_t rb1 = r + 1 < d ? rb : rb + kScRound;
                const uint32_t r1 = r + 1 < d ? r + 1 : 0u;
                const uint64_t nrb = r1 + 1 < d ? rb1 : rb1 + kScRound;
                const uint32_t nr = r1 + 1 < d ? r1 + 1 : 0u;
#pragma unroll
                for (int i = 0; i < kScItems; i++) bsn[i] = bsn2[i];
                if (nrb < end) {
#pragma unroll
                    for (int i = 0; i < kScItems; i++) {
                        const uint64_t p = nrb + (uint64_t)wave * 64 * kScItems + (uint64_t)i * 64 + lane;
                        bsn2[i] = a.idx[(uint64_t)nr * a.n + (p < end ? p : end - 1)];
                    }
                }
            }
            uint64_t ent[kScItems];
            uint32_t br[kScItems];  // bin << 16 | rank within (wave, bin); bin 0xFFFF = no update
            K3_MARK(0);
            // phase 1: stable per-wave ranks; wave w owns packets [rb + w*64*kScItems, ...), order (slot, lane)
#pragma unroll
            for (int i = 0; i < kScItems; i++) {
                bool valid = ids[i] != GNS_ID_NONE;
                {
                    const bool hot = (bs[i] >> 31) != 0;
                    if (a.hot_mode) valid = valid && hot && (a.hflag2[r * kHot + (bs[i] & 0x7FFFFFFFu)] & 3u) != 0;
                    else valid = valid && !hot;
                }
                uint32_t t = 0;
                uint64_t e = 0;
                if (valid) {
                    const uint32_t b = bs[i];
                    const bool hot = (b >> 31) != 0;
                    const uint32_t h = b & 0x7FFFFFFFu;
                    t = hot ? a.g.ntiles + h : (b >> a.g.bin_bits);
                    const uint32_t low = hot ? r * kHot + h : (b & tmask);
                    const uint32_t sz = szs[i];
                    uint32_t lo = ids[i], sf = sz;
                    if (sz >= kSizeEsc) {
                        const uint32_t q = atomicAdd(a.ovf_cnt, 1u);
                        if (q < a.ovf_cap) {
                            a.ovf[q] = (uint64_t)sz << 32 | ids[i];
                            lo = kOvfFlag | q;
                        } else {
                            atomicAdd(&a.stats[4], 1ull);
                            lo = kOvfFlag | (a.ovf_cap - 1);
                        }
                        sf = kSizeEsc;
                    }
                    e = (uint64_t)((sf << kEntShift) | low) << 32 | lo;
                }
                uint32_t rk = 0;
                if constexpr (RANK == 1) {
                    // returning LDS adds (issued after this loop, all items under one
                    // wait): same-address lanes of one instruction are served in lane
                    // order (verified at create by k_lds_order_probe)
                } else {
                    uint64_t peers = __ballot(valid);
                    for (uint32_t bit = 0; bit < nbits; bit++) {
                        const uint64_t m = __ballot(valid && ((t >> bit) & 1u));
                        peers &= ((t >> bit) & 1u) ? m : ~m;
                    }
                    const uint32_t before = __popcll(peers & lt_mask);
                    if (valid) {
                        rk = s_cnt[wave * LB + t] + before;
                        if (before == 0) s_cnt[wave * LB + t] += __popcll(peers);
                    }
                }
                ent[i] = e;
                br[i] = (valid ? t : 0xFFFFu) << 16 | rk;
            }
            if constexpr (RANK == 1) {
                // every lane adds (0 to its own dummy word without an update): no
                // divergence around the returning adds, one wait for all of them
                uint32_t rks[kScItems];
#pragma unroll
                for (int i = 0; i < kScItems; i++) {
                    const uint32_t t = br[i] >> 16;
                    uint32_t *ad = t != 0xFFFFu ? &s_cnt[wave * LB + t] : &s_dummy[tid];
                    rks[i] = atomicAdd(ad, t != 0xFFFFu ? 1u : 0u);
                }
#pragma unroll
                for (int i = 0; i < kScItems; i++) br[i] |= rks[i];
            }
            __syncthreads();
            K3_MARK(1);
            // phase 2: per bin, global base of each wave's run; clear the other buffer
            {
                uint32_t *goff = s_goff + r * LB;
                for (uint32_t t = tid; t < LB; t += kScThreads) {
                    uint32_t x[kScWaves];
#pragma unroll
                    for (uint32_t w = 0; w < (uint32_t)kScWaves; w++) x[w] = s_cnt[w * LB + t];
                    uint32_t c = goff[t];
#pragma unroll
                    for (uint32_t w = 0; w < (uint32_t)kScWaves; w++) { s_cnt[w * LB + t] = c; c += x[w]; }
                    goff[t] = c;
                }
                for (uint32_t t = tid; t < kScWaves * LB; t += kScThreads) s_cnto[t] = 0;
            }
            __syncthreads();
            K3_MARK(2);
#pragma unroll
            for (int i = 0; i < kScItems; i++) asm volatile("" ::"v"(bsn[i]));
            // phase 3: each update straight to its slot (runs per bin and wave are contiguous)
#pragma unroll
            for (int i = 0; i < kScItems; i++) {
                if ((br[i] >> 16) != 0xFFFFu) {
                    const uint32_t t = br[i] >> 16;
                    a.entries[s_cnt[wave * LB + t] + (br[i] & 0xFFFFu)] = ent[i];
                }
            }
            K3_MARK(4);
        }
    }
#ifdef GNS_K3_PROF
    if (threadIdx.x == 0 && !a.hot_mode) for (int i = 0; i < 5; i++) atomicAdd(&a.stats[kStatsProf + i], (unsigned long long)k3t[i]);
#endif
}

// ---------------------------------------------------------------------------
// K3s: the same stable partition, staged.  A 1024-thread block takes its K1
// block (16384 packets) in sub-passes of 8192 packets and, per row, ranks the
// cold updates like K3 (returning LDS adds per (wave, bin), waves owning
// contiguous packet ranges), lays them out bin by bin in LDS, and copies the
// bins out as contiguous runs (~15 updates per bin and sub-pass at the bench
// geometry).  Scattered 8-byte stores cost 2-3x the time of runs of >= 16
// (tools/membench3.hip); the output is identical to K3's.  Rows of at most
// 512 bins (the bench geometry has 256, configs[5] 512); wider rows use K3.
// ---------------------------------------------------------------------------
#ifndef GNS_ST_SUB
#define GNS_ST_SUB 8192
#endif
constexpr uint32_t kStSub = GNS_ST_SUB;               // packets per sub-pass
static_assert(kChunk % kStSub == 0, "whole sub-passes per K1 block");

// NT threads, rows of at most BINS bins: <1024, 256> (the bench geometry) and
// <1024, 512, kStSub, PK> (the wide/deep configs[4]/[5] geometry: 16 waves in one 136 KB
// block per CU; the former <512, 512>, 8 waves, stays behind GNS_K3_STAGED=u:
// K3s 3.08 -> 3.04 ms at configs[4], profiles/r05_ab_k3pack.txt).
// PK: the (wave, bin) counters as 16-bit halves, bins t and t + BINS/2 in one word (a wave
// counts at most SUB/kWaves updates of a bin per sub-pass), which is what lets 16 waves'
// counters fit
template <int NT, int BINS, int SUB = (int)kStSub, bool PK = false>
struct StLds {
    static constexpr int kWaves = NT / 64;
    static constexpr int kCw = PK ? BINS / 2 : BINS;  // counter words per wave
    uint64_t stage[SUB];
    uint16_t sbin[SUB];
    uint32_t cnt[2][kWaves][kCw];
    uint32_t lstart[BINS], gpos[BINS];
    uint32_t goff[8][BINS];
    uint32_t wsum[BINS / 64];
    uint32_t dummy[NT];  // rank adds of lanes without an update
};

template <int NT, int BINS, int SUB = (int)kStSub, bool PK = false>
__global__ __launch_bounds__(NT) void k_scatter_st(ScatterArgs a) {
    static_assert(!PK || (SUB / (NT / 64) < 65536 && BINS % 128 == 0), "16-bit counter halves");
    constexpr uint32_t kCw = StLds<NT, BINS, SUB, PK>::kCw;
    static_assert(kChunk % SUB == 0, "whole sub-passes per K1 block");
    constexpr int kStThreads = NT;
    constexpr int kStWaves = NT / 64;
    constexpr int kStItems = (uint32_t)SUB / NT;
    constexpr uint32_t kStBins = BINS;
    static_assert((uint32_t)SUB / kStWaves == kStItems * 64, "a wave owns kStItems x 64 consecutive packets of a sub-pass");
    static_assert(BINS <= NT && BINS % 64 == 0, "one thread per bin in the bin scan");
    __shared__ StLds<NT, BINS, SUB, PK> L;
#ifdef GNS_K3_PROF
    uint64_t k3t[5] = {0, 0, 0, 0, 0}, k3prev = __builtin_amdgcn_s_memtime();
#endif
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    uint32_t blk = blockIdx.x;
    const uint32_t d = a.g.d, nt = a.g.ntiles;
    // Workgroups are dealt round-robin over the 8 XCDs (MI355X_MICROARCH: observed, not promised),
    // so K1 block b and b + 1 -- whose runs of a bin are adjacent in `entries` and share the
    // partial lines at their boundary -- would be written through two different L2s.  Give each
    // XCD a contiguous range of K1 blocks instead: headline K3s 1.37 -> 1.25 ms, configs[4]
    // 3.42 -> 2.67 ms (profiles/r05_ab_k3xcd.txt).  Only the speed depends on the placement.
    if (a.xcd_map) blk = xcd_block(blk, gridDim.x);
    const uint32_t tmask = (1u << a.g.bin_bits) - 1u;
    const uint64_t beg = (uint64_t)blk * kChunk;
    const uint64_t end = min(a.n, beg + kChunk);
    for (uint32_t i = tid; i < d * kStBins; i += kStThreads) {
        const uint32_t r = i / kStBins, t = i % kStBins;
        L.goff[r][t] = t < nt ? a.offsets[(uint64_t)blk * a.g.nbins_all + r * nt + t] : 0u;
    }
    for (uint32_t i = tid; i < 2 * kStWaves * kCw; i += kStThreads) (&L.cnt[0][0][0])[i] = 0;
    // packet of item j in a sub-pass: wave-contiguous, (j, lane) order inside the wave
    auto pkt = [&](uint64_t sp, int j) { return sp + (uint64_t)wave * ((uint32_t)SUB / kStWaves) + (uint64_t)j * 64 + lane; };
    uint32_t ids[kStItems], szs[kStItems], cds[kStItems];
    uint32_t ncd[kStItems], nids[kStItems], nszs[kStItems];
    auto load_ids = [&](uint64_t sp, uint32_t (&di)[kStItems], uint32_t (&ds)[kStItems]) {
#pragma unroll
        for (int j = 0; j < kStItems; j++) {
            const uint64_t p = pkt(sp, j);
            const uint64_t pc = p < end ? p : end - 1;
            di[j] = p < end ? a.keyid[pc] : GNS_ID_NONE;
            ds[j] = a.sizes[pc];
        }
    };
    auto load_codes = [&](uint64_t sp, uint32_t r, uint32_t (&c)[kStItems]) {
#pragma unroll
        for (int j = 0; j < kStItems; j++) {
            const uint64_t p = pkt(sp, j);
            c[j] = a.idx[(uint64_t)r * a.n + (p < end ? p : end - 1)];
        }
    };
    load_ids(beg, ids, szs);
    load_codes(beg, 0, cds);
    uint32_t par = 0;
    __syncthreads();
    for (uint64_t sp = beg; sp < end; sp += (uint32_t)SUB) {
        for (uint32_t r = 0; r < d; r++) {
            uint32_t (&cnt)[kStWaves][kCw] = L.cnt[par];
            K3_MARK(4);  // loop
            // phase A: entries and stable ranks within (wave, bin)
            uint64_t ent[kStItems];
            uint32_t tb[kStItems];  // bin << 16 | rank, 0xFFFF bin = no update
#pragma unroll
            for (int j = 0; j < kStItems; j++) {
                const uint32_t b = cds[j];
                const bool valid = ids[j] != GNS_ID_NONE && (b >> 31) == 0;
                uint32_t t = 0xFFFFu, rk = 0;
                uint64_t e = 0;
                if (valid) {
                    t = b >> a.g.bin_bits;
                    const uint32_t low = b & tmask, sz = szs[j];
                    uint32_t lo = ids[j], sf = sz;
                    if (sz >= kSizeEsc) {
                        const uint32_t q = atomicAdd(a.ovf_cnt, 1u);
                        if (q < a.ovf_cap) {
                            a.ovf[q] = (uint64_t)sz << 32 | ids[j];
                            lo = kOvfFlag | q;
                        } else {
                            atomicAdd(&a.stats[4], 1ull);
                            lo = kOvfFlag | (a.ovf_cap - 1);
                        }
                        sf = kSizeEsc;
                    }
                    e = (uint64_t)((sf << kEntShift) | low) << 32 | lo;
                }
                ent[j] = e;
                tb[j] = t << 16 | rk;
            }
            // ranks: every lane adds (a lane without an update adds 0 to its own dummy
            // word), so the eight returning adds issue back to back under one wait;
            // same-address lanes are served in lane order
            {
                uint32_t rks[kStItems];
#pragma unroll
                for (int j = 0; j < kStItems; j++) {
                    const uint32_t t = tb[j] >> 16;
                    const uint32_t sh = PK && t != 0xFFFFu && t >= kCw ? 16u : 0u;
                    uint32_t *ad = t != 0xFFFFu ? &cnt[wave][PK ? t % kCw : t] : &L.dummy[tid];
                    rks[j] = atomicAdd(ad, t != 0xFFFFu ? 1u << sh : 0u);
                    if constexpr (PK) rks[j] = (rks[j] >> sh) & 0xFFFFu;
                }
#pragma unroll
                for (int j = 0; j < kStItems; j++) tb[j] |= rks[j];
            }
            // the next step's codes (and ids / sizes at a sub-pass boundary) load during C and D
            const uint32_t r1 = r + 1 < d ? r + 1 : 0u;
            const uint64_t sp1 = r + 1 < d ? sp : sp + (uint32_t)SUB;
            if (sp1 < end) {
                load_codes(sp1, r1, ncd);
                if (r1 == 0) load_ids(sp1, nids, nszs);
            }
            __syncthreads();
            K3_MARK(0);
            // phase C: per bin, prefix over the waves and the bin's total; scan of the totals
            uint32_t total = 0, incl = 0;
            if constexpr (PK) {  // both halves' prefix over the waves; the totals via lstart
                if (tid < kCw) {
                    uint32_t r0 = 0, r1 = 0;
#pragma unroll
                    for (int w = 0; w < kStWaves; w++) {
                        const uint32_t x = cnt[w][tid];
                        cnt[w][tid] = r0 | r1 << 16;
                        r0 += x & 0xFFFFu;
                        r1 += x >> 16;
                    }
                    L.lstart[tid] = r0;
                    L.lstart[tid + kCw] = r1;
                }
                __syncthreads();
                if (tid < kStBins) {
                    total = L.lstart[tid];
                    incl = wave_incl_scan(total);
                    if (lane == 63) L.wsum[wave] = incl;
                }
            } else if (tid < kStBins) {
                const uint32_t t = tid;
                uint32_t run = 0;
                if (t < nt) {
#pragma unroll
                    for (int w = 0; w < kStWaves; w++) {
                        const uint32_t x = cnt[w][t];
                        cnt[w][t] = run;
                        run += x;
                    }
                }
                total = run;
                incl = wave_incl_scan(total);
                if (lane == 63) L.wsum[wave] = incl;
            }
            __syncthreads();
            if (tid < kStBins) {
                uint32_t base = 0;
#pragma unroll
                for (uint32_t w = 0; w < kStBins / 64; w++) base += w < wave ? L.wsum[w] : 0u;
                const uint32_t t = tid;
                L.lstart[t] = base + incl - total;
                L.gpos[t] = L.goff[r][t];
                L.goff[r][t] += total;
            }
            __syncthreads();
            K3_MARK(1);
            // phase D: updates into the bin-ordered stage
#pragma unroll
            for (int j = 0; j < kStItems; j++) {
                const uint32_t t = tb[j] >> 16;
                if (t != 0xFFFFu) {
                    const uint32_t c = PK ? (cnt[wave][t % kCw] >> (t >= kCw ? 16u : 0u)) & 0xFFFFu : cnt[wave][t];
                    const uint32_t pos = L.lstart[t] + c + (tb[j] & 0xFFFFu);
                    L.stage[pos] = ent[j];
                    L.sbin[pos] = (uint16_t)t;
                }
            }
            __syncthreads();
            K3_MARK(2);
            // phase E: take the next step's inputs first (the wait for them lands here,
            // before this step's stores are issued, not after them), then the bins out
            // as contiguous runs; clear this step's counters
            if (sp1 < end) {
#pragma unroll
                for (int j = 0; j < kStItems; j++) cds[j] = ncd[j];
                if (r1 == 0) {
#pragma unroll
                    for (int j = 0; j < kStItems; j++) { ids[j] = nids[j]; szs[j] = nszs[j]; }
                }
            }
            uint32_t ntot = 0;
#pragma unroll
            for (uint32_t w = 0; w < kStBins / 64; w++) ntot += L.wsum[w];
            for (uint32_t i = tid; i < ntot; i += kStThreads) {
                const uint32_t t = L.sbin[i];
                a.entries[L.gpos[t] + (i - L.lstart[t])] = L.stage[i];
            }
            for (uint32_t i = tid; i < kStWaves * kCw; i += kStThreads) (&cnt[0][0])[i] = 0;
            par ^= 1u;
            K3_MARK(3);
        }
    }
#ifdef GNS_K3_PROF
    if (threadIdx.x == 0) for (int i = 0; i < 5; i++) atomicAdd(&a.stats[kStatsProf + i], (unsigned long long)k3t[i]);
#endif
}

// ---------------------------------------------------------------------------
// K3c: K3s over K1's compact cold streams.  Per (block, row) the stream is the
// four K1 waves' cold codes of that row in wave order = packet order, so only
// the updates that move are read (no per-packet codes, no lanes without an
// update): sub-passes of kStSub updates, the flow id and size of each gathered
// from the block's keyid / size words (the K1 block's 64 KB of each stays in
// L2 across its rows).  Ranks, stage and copy-out as K3s; the output is
// identical to K3s's.
// ---------------------------------------------------------------------------
template <int NT, int BINS>
__global__ __launch_bounds__(NT) void k_scatter_cs(ScatterArgs a) {
    constexpr int kStThreads = NT;
    constexpr int kStWaves = NT / 64;
    constexpr int kStItems = kStSub / NT;
    constexpr uint32_t kStBins = BINS;
    static_assert(kStSub / kStWaves == kStItems * 64, "a wave owns kStItems x 64 consecutive updates of a sub-pass");
    static_assert(BINS <= NT && BINS % 64 == 0, "one thread per bin in the bin scan");
    __shared__ StLds<NT, BINS> L;
    __shared__ uint32_t s_pre[8][kCsWaves + 1];  // per row: the K1 waves' stream starts, then the row total
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t blk = blockIdx.x, d = a.g.d, nt = a.g.ntiles;
    const uint32_t tmask = (1u << a.g.bin_bits) - 1u;
    const uint64_t beg = (uint64_t)blk * kChunk;
    for (uint32_t i = tid; i < d * kStBins; i += kStThreads) {
        const uint32_t r = i / kStBins, t = i % kStBins;
        L.goff[r][t] = t < nt ? a.offsets[(uint64_t)blk * a.g.nbins_all + r * nt + t] : 0u;
    }
    if (tid < d) {
        uint32_t run = 0;
        for (uint32_t w = 0; w < kCsWaves; w++) {
            s_pre[tid][w] = run;
            run += a.scnt[(((uint64_t)blk * kCsWaves + w) * d + tid) * 2];
        }
        s_pre[tid][kCsWaves] = run;
    }
    for (uint32_t i = tid; i < 2 * kStWaves * kStBins; i += kStThreads) (&L.cnt[0][0][0])[i] = 0;
    __syncthreads();
    // update j of a sub-pass at stream position x: wave-contiguous, (j, lane) order inside the wave
    auto spos = [&](uint32_t sp, int j) { return sp + wave * (kStSub / kStWaves) + (uint32_t)j * 64 + lane; };
    // codes of step (r, sp): bucket << 14 | packet offset in the block (the K1 wave's range
    // start + the code's index), kCsNone past the row's end
    auto load_codes = [&](uint32_t r, uint32_t sp, uint32_t (&c)[kStItems], uint32_t (&po)[kStItems]) {
        const uint32_t p1 = s_pre[r][1], p2 = s_pre[r][2], p3 = s_pre[r][3], tot = s_pre[r][4];
#pragma unroll
        for (int j = 0; j < kStItems; j++) {
            const uint32_t x = spos(sp, j);
            c[j] = kCsNone;
            po[j] = 0;
            if (x < tot) {
                const uint32_t w = (x >= p1 ? 1u : 0u) + (x >= p2 ? 1u : 0u) + (x >= p3 ? 1u : 0u);
                const uint32_t x0 = w == 0 ? 0u : (w == 1 ? p1 : (w == 2 ? p2 : p3));
                c[j] = a.cstr[(((uint64_t)blk * kCsWaves + w) * d + r) * kCsWave + (x - x0)];
                po[j] = w * kCsWave;
            }
        }
    };
    auto gather = [&](const uint32_t (&c)[kStItems], const uint32_t (&po)[kStItems], uint32_t (&di)[kStItems],
                      uint32_t (&ds)[kStItems]) {
#pragma unroll
        for (int j = 0; j < kStItems; j++) {
            const uint64_t pp = beg + po[j] + (c[j] & (kCsWave - 1u));
            di[j] = c[j] != kCsNone ? a.keyid[pp] : GNS_ID_NONE;
            ds[j] = c[j] != kCsNone ? a.sizes[pp] : 0u;
        }
    };
    // steps: rows in order, sub-passes of kStSub updates in each
    uint32_t r = 0, sp = 0;
    while (r < d && s_pre[r][kCsWaves] == 0) r++;
    uint32_t cds[kStItems], pos[kStItems], ids[kStItems], szs[kStItems];
    uint32_t ncd[kStItems], npo[kStItems];
    if (r < d) {
        load_codes(r, 0, cds, pos);
        gather(cds, pos, ids, szs);
    }
    uint32_t par = 0;
    while (r < d) {  // block-uniform
        // the next step
        uint32_t r1 = r, sp1 = sp + kStSub;
        if (sp1 >= s_pre[r1][kCsWaves]) {
            r1++;
            sp1 = 0;
            while (r1 < d && s_pre[r1][kCsWaves] == 0) r1++;
        }
        uint32_t (&cnt)[kStWaves][kStBins] = L.cnt[par];
        // phase A: entries and stable ranks within (wave, bin)
        uint64_t ent[kStItems];
        uint32_t tb[kStItems];  // bin << 16 | rank, 0xFFFF bin = no update
#pragma unroll
        for (int j = 0; j < kStItems; j++) {
            const bool valid = cds[j] != kCsNone && ids[j] != GNS_ID_NONE;
            uint32_t t = 0xFFFFu;
            uint64_t e = 0;
            if (valid) {
                const uint32_t b = cds[j] >> kCsBits;
                t = b >> a.g.bin_bits;
                const uint32_t low = b & tmask, sz = szs[j];
                uint32_t lo = ids[j], sf = sz;
                if (sz >= kSizeEsc) {
                    const uint32_t q = atomicAdd(a.ovf_cnt, 1u);
                    if (q < a.ovf_cap) {
                        a.ovf[q] = (uint64_t)sz << 32 | ids[j];
                        lo = kOvfFlag | q;
                    } else {
                        atomicAdd(&a.stats[4], 1ull);
                        lo = kOvfFlag | (a.ovf_cap - 1);
                    }
                    sf = kSizeEsc;
                }
                e = (uint64_t)((sf << kEntShift) | low) << 32 | lo;
            }
            ent[j] = e;
            tb[j] = t << 16;
        }
        {
            uint32_t rks[kStItems];
#pragma unroll
            for (int j = 0; j < kStItems; j++) {
                const uint32_t t = tb[j] >> 16;
                uint32_t *ad = t != 0xFFFFu ? &cnt[wave][t] : &L.dummy[tid];
                rks[j] = atomicAdd(ad, t != 0xFFFFu ? 1u : 0u);
            }
#pragma unroll
            for (int j = 0; j < kStItems; j++) tb[j] |= rks[j];
        }
        if (r1 < d) load_codes(r1, sp1, ncd, npo);
        __syncthreads();
        // phase C: per bin, prefix over the waves and the bin's total; scan of the totals
        uint32_t total = 0, incl = 0;
        if (tid < kStBins) {
            const uint32_t t = tid;
            uint32_t run = 0;
            if (t < nt) {
#pragma unroll
                for (int w = 0; w < kStWaves; w++) {
                    const uint32_t x = cnt[w][t];
                    cnt[w][t] = run;
                    run += x;
                }
            }
            total = run;
            incl = wave_incl_scan(total);
            if (lane == 63) L.wsum[wave] = incl;
        }
        __syncthreads();
        // the next step's flow ids and sizes (its codes have had phase C to arrive)
        uint32_t nids[kStItems], nszs[kStItems];
        if (r1 < d) gather(ncd, npo, nids, nszs);
        if (tid < kStBins) {
            uint32_t base = 0;
#pragma unroll
            for (uint32_t w = 0; w < kStBins / 64; w++) base += w < wave ? L.wsum[w] : 0u;
            const uint32_t t = tid;
            L.lstart[t] = base + incl - total;
            L.gpos[t] = L.goff[r][t];
            L.goff[r][t] += total;
        }
        __syncthreads();
        // phase D: updates into the bin-ordered stage
#pragma unroll
        for (int j = 0; j < kStItems; j++) {
            const uint32_t t = tb[j] >> 16;
            if (t != 0xFFFFu) {
                const uint32_t q = L.lstart[t] + cnt[wave][t] + (tb[j] & 0xFFFFu);
                L.stage[q] = ent[j];
                L.sbin[q] = (uint16_t)t;
            }
        }
        __syncthreads();
        // phase E: the bins out as contiguous runs; clear this step's counters
        uint32_t ntot = 0;
#pragma unroll
        for (uint32_t w = 0; w < kStBins / 64; w++) ntot += L.wsum[w];
        for (uint32_t i = tid; i < ntot; i += kStThreads) {
            const uint32_t t = L.sbin[i];
            a.entries[L.gpos[t] + (i - L.lstart[t])] = L.stage[i];
        }
        for (uint32_t i = tid; i < kStWaves * kStBins; i += kStThreads) (&cnt[0][0])[i] = 0;
        par ^= 1u;
        if (r1 < d) {
#pragma unroll
            for (int j = 0; j < kStItems; j++) { cds[j] = ncd[j]; pos[j] = npo[j]; ids[j] = nids[j]; szs[j] = nszs[j]; }
        }
        r = r1;
        sp = sp1;
    }
}

// The exact entry path for designated buckets over K1's compact hot streams
// (k_scatter's hot mode, for the slots k_hot_decide / k_hot_blockcheck flagged):
// one wave per K1 block walks each row's hot stream in order and writes the
// flagged slots' updates to their hot bins (ranks by ballot multisplit over the
// slot).  Rare (cold start, ownership changes); the whole grid exits when no
// slot is flagged.
__global__ __launch_bounds__(64) void k_hot_scatter_cs(ScatterArgs a) {
    __shared__ uint32_t s_base[8 * kHot];
    if (*a.hany == 0) return;
    const uint32_t lane = threadIdx.x, blk = blockIdx.x, d = a.g.d;
    const uint64_t beg = (uint64_t)blk * kChunk;
    const uint64_t lt = lane ? (~0ull >> (64u - lane)) : 0ull;
    for (uint32_t i = lane; i < d * kHot; i += 64) s_base[i] = a.offsets[(uint64_t)blk * a.g.nbins_all + a.g.nbins + i];
    __builtin_amdgcn_wave_barrier();
    for (uint32_t r = 0; r < d; r++) {
        for (uint32_t w = 0; w < kCsWaves; w++) {
            const uint64_t sb = (((uint64_t)blk * kCsWaves + w) * d + r) * kCsWave;
            const uint32_t n = a.scnt[(((uint64_t)blk * kCsWaves + w) * d + r) * 2 + 1];
            for (uint32_t x0 = 0; x0 < n; x0 += 64) {
                const uint32_t x = x0 + lane;
                uint32_t slot = 0, code = 0;
                bool valid = false;
                if (x < n) {
                    code = a.hstr[sb + x];
                    slot = r * kHot + (code >> kCsBits);
                    valid = (a.hflag2[slot] & 3u) != 0;
                }
                uint64_t peers = __ballot(valid);
#pragma unroll
                for (uint32_t bit = 0; bit < kHotBits + 3; bit++) {
                    const uint64_t m = __ballot(valid && ((slot >> bit) & 1u));
                    peers &= ((slot >> bit) & 1u) ? m : ~m;
                }
                if (valid) {
                    const uint64_t p = beg + w * kCsWave + (code & (kCsWave - 1u));
                    const uint32_t id = a.keyid[p], sz = a.sizes[p];
                    uint32_t lo = id, sf = sz;
                    if (sz >= kSizeEsc) {
                        const uint32_t q = atomicAdd(a.ovf_cnt, 1u);
                        if (q < a.ovf_cap) {
                            a.ovf[q] = (uint64_t)sz << 32 | id;
                            lo = kOvfFlag | q;
                        } else {
                            atomicAdd(&a.stats[4], 1ull);
                            lo = kOvfFlag | (a.ovf_cap - 1);
                        }
                        sf = kSizeEsc;
                    }
                    const uint32_t pos = s_base[slot] + (uint32_t)__popcll(peers & lt);
                    a.entries[pos] = (uint64_t)((sf << kEntShift) | slot) << 32 | lo;
                }
                __builtin_amdgcn_wave_barrier();
                if (valid && __popcll(peers & lt) == 0) s_base[slot] += (uint32_t)__popcll(peers);
                __builtin_amdgcn_wave_barrier();
            }
        }
    }
}

// Does a returning LDS add serve the same-address lanes of one wave
// instruction in lane order?  (K3's RANK 1 relies on it; measured on gfx950:
// tools/lds_order.hip, 0 of 1.3e10 same-address lane pairs out of order.)
__global__ __launch_bounds__(256) void k_lds_order_probe(uint32_t *viol, int iters) {
    __shared__ uint32_t s[4][64], s_old[4][64], s_ad[4][64];
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    uint32_t x = (blockIdx.x * 256 + threadIdx.x) * 0x9E3779B1u + 12345u, v = 0;
    for (int it = 0; it < iters; it++) {
        s[w][lane] = 0;
        x = x * 1664525u + 1013904223u;
        const uint32_t ad = (x >> 16) % (1u + (uint32_t)it % 16u);
        const uint32_t old = atomicAdd(&s[w][ad], 1u);
        s_old[w][lane] = old;
        s_ad[w][lane] = ad;
        for (uint32_t j = 0; j < lane; j++) v += (s_ad[w][j] == ad && s_old[w][j] >= old) ? 1u : 0u;
    }
    if (v) atomicAdd(viol, v);
}

// Order bins by size (largest first) so the heavy bins start first.
__global__ __launch_bounds__(1024) void k_order(const uint32_t *offsets, uint32_t nblk, uint32_t nbins,
                                                uint32_t nall, const uint32_t *total, uint32_t *order) {
    // K4 schedule: bins by decreasing size (1/8-octave classes; order within a
    // class is arbitrary: it only balances the launch, results do not depend on it)
    constexpr uint32_t NK = 33 * 8;
    __shared__ uint32_t s_cnt[NK];
    __shared__ uint16_t s_key[4096];
    for (uint32_t k = threadIdx.x; k < NK; k += 1024) s_cnt[k] = 0;
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nbins; b += 1024) {
        const uint32_t s0 = offsets[b];  // block 0's row: the start of every bin
        const uint32_t s1 = (b + 1 < nall) ? offsets[b + 1] : *total;
        const uint32_t sz = s1 - s0;
        const uint32_t lz = __clz(sz);
        const uint32_t key = sz == 0 ? 0u : (32u - lz) * 8u + ((sz << lz) >> 28 & 7u);
        s_key[b] = (uint16_t)key;
        atomicAdd(&s_cnt[key], 1u);
    }
    __syncthreads();
    if (threadIdx.x < 64) {  // descending exclusive scan of the class counts
        constexpr uint32_t PER = (NK + 63) / 64;
        const uint32_t lane = threadIdx.x;
        uint32_t x[PER], sum = 0;
#pragma unroll
        for (uint32_t q = 0; q < PER; q++) {
            const uint32_t k = lane * PER + q;  // k-th class from the top
            x[q] = k < NK ? s_cnt[NK - 1 - k] : 0u;
            sum += x[q];
        }
        uint32_t run = wave_incl_scan(sum) - sum;
#pragma unroll
        for (uint32_t q = 0; q < PER; q++) {
            const uint32_t k = lane * PER + q;
            if (k < NK) s_cnt[NK - 1 - k] = run;
            run += x[q];
        }
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nbins; b += 1024) order[atomicAdd(&s_cnt[s_key[b]], 1u)] = b;
}

// ---------------------------------------------------------------------------
// K4: apply one bin's updates to its LDS-resident tile, in stream order.
// ---------------------------------------------------------------------------
struct ApplyArgs {
    unsigned long long *stats;  // [5] replayed updates, [6] chunks, [7] chunks with a replay
    const uint64_t *entries;
    uint64_t *entries2;         // super-bin sub-partition scratch (sub_bits > 0)
    const uint16_t *rseg;       // [round][16] tile starts inside each k_subpart round, or null
    const uint32_t *offsets;
    uint32_t nblk, nbins;
    const uint32_t *total;
    const uint32_t *order;
    const uint64_t *ovf;
    CmGeom g;
    uint32_t *C, *Fc, *S, *Fs;
    uint32_t *work;             // persistent-schedule counter (zeroed before the launch)
};

// accN per bucket and chunk (32 bits): n [0,14) | n_foreign_count [14,28) | force (size
// escape) bit 28.  The size half needs no foreign-update count: a foreign update only
// replaces when S == 0 or its size exceeds S, so S > (foreign size sum) covers it and a
// bucket entering the chunk with S == 0 is replayed.
constexpr uint32_t kM14 = (1u << 14) - 1;
constexpr uint32_t kAccForce = 28;
static_assert(kApChunk < (1u << 14), "accN field widths");
static_assert(kScRound <= 65536, "K3 packs ranks in 16 bits");
#ifndef GNS_REPLAY_LEAD
#define GNS_REPLAY_LEAD 1  // 0: one LDS round per same-bucket lane (A/B)
#endif
#ifndef GNS_REP_CAP
#define GNS_REP_CAP 1536
#endif
constexpr uint32_t kRepCap = GNS_REP_CAP;

// ---------------------------------------------------------------------------
// Exact wave-parallel sequence for ONE bucket (count_min.go:99-155): 64
// updates per step; a prefix sum gives the counter before every update, the
// first update that would leave the linear regime (an "event": fingerprint
// take-over, counter wrap) is applied explicitly and the scan restarts after
// it.  Steps per 64 updates = events + 1.
// ---------------------------------------------------------------------------
extern "C" __device__ long __ockl_wfscan_add_i64(long, bool);
// DPP inclusive scan over the whole wave (call with all 64 lanes active)
__device__ __forceinline__ int64_t wave_incl_scan64(int64_t v) { return __ockl_wfscan_add_i64(v, true); }

// count half; F, C wave-uniform
__device__ __forceinline__ void count_seq64(bool valid, uint32_t k, uint32_t &F, uint32_t &C) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t start = 0;
    for (;;) {
        const bool act = valid && lane >= start;
        const bool own = k == F;
        const int64_t dlt = act ? (own ? 1 : -1) : 0;
        const int64_t P = wave_incl_scan64(dlt);
        const int64_t Cb = (int64_t)C + P - dlt;
        const bool ev = act && ((!own && Cb <= 1) || (own && Cb >= 0xFFFFFFFFll));
        const uint64_t m = __ballot(ev);
        if (!m) {
            C = (uint32_t)((int64_t)C + __shfl(P, 63, 64));
            return;
        }
        const uint32_t t = (uint32_t)__ffsll((long long)m) - 1;
        const int64_t cbt = __shfl(Cb, t, 64);
        const uint32_t kt = __shfl(k, t, 64);
        const bool ownt = kt == F;
        if (ownt) { C = 0; }                        // C+1 wraps to 0 (u32), F kept
        else if (cbt == 0) { C = 1; F = kt; }       // :214-218
        else { C = 0; F = kt; }                     // :226-231 reaches 0, F := flow
        start = t + 1;
        if (start >= 64) return;
    }
}

// size half; F, S wave-uniform
__device__ __forceinline__ void size_seq64(bool valid, uint32_t k, uint32_t s, uint32_t &F, uint32_t &S) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t start = 0;
    for (;;) {
        const bool act = valid && lane >= start;
        const bool own = k == F;
        const int64_t dlt = act ? (own ? (int64_t)s : -(int64_t)s) : 0;
        const int64_t W = wave_incl_scan64(dlt);
        const int64_t Sb = (int64_t)S + W - dlt;
        const bool ev = act && ((!own && (Sb == 0 || (int64_t)s > Sb)) || (own && Sb + (int64_t)s > 0xFFFFFFFFll));
        const uint64_t m = __ballot(ev);
        if (!m) {
            S = (uint32_t)((int64_t)S + __shfl(W, 63, 64));
            return;
        }
        const uint32_t t = (uint32_t)__ffsll((long long)m) - 1;
        const int64_t sbt = __shfl(Sb, t, 64);
        const uint32_t kt = __shfl(k, t, 64), st = __shfl(s, t, 64);
        if (kt == F) { S = (uint32_t)((uint64_t)sbt + st); }   // u32 wrap, F kept
        else { S = st; F = kt; }                               // :184-188 / :196-200
        start = t + 1;
        if (start >= 64) return;
    }
}

struct ApplyLds {
    // bucket state, halves paired: sCS = {C, S}, sF = {Fc, Fs} (classify reads both
    // fingerprints, decide both counters: one 8-byte LDS access each)
    uint2 sCS[kTileMax], sF[kTileMax];
    uint32_t accN[kTileMax];            // n | n_oth_c << 14 | force << 28; after decide: replay flags
    unsigned long long accS[kTileMax];  // sum_own | sum_oth<<32 ; replay owner words
    uint16_t s_list[kApChunk];
    uint64_t s_rep[kRepCap];            // the first kRepCap replay entries themselves (no global re-read)
    uint32_t s_wc[kApItems * kApWaves];
    uint32_t s_any, s_nlist;
#ifdef GNS_K4_PROF
    uint32_t s_pmax, s_psum;  // the chunk's largest and summed per-wave replay cycles (balance probe)
#endif
};

__device__ __forceinline__ void decode_entry(const uint64_t *ovf, uint64_t e, uint32_t &k, uint32_t &s) {
    const uint32_t lo = (uint32_t)e, hi = (uint32_t)(e >> 32);
    if (lo & kOvfFlag) {
        const uint64_t ov = ovf[lo & ~kOvfFlag];
        k = (uint32_t)ov; s = (uint32_t)(ov >> 32);
    } else {
        k = lo; s = hi >> kEntShift;
    }
}

// Replay of one 64-item group (count_min.go:99-155): pending lanes hold
// updates of this wave's buckets, in stream order by lane.  A bucket with >= 8
// updates in the group runs the wave-parallel sequence; the rest resolve
// same-bucket lanes lowest-lane-first.
__device__ __forceinline__ void replay_group(ApplyLds &L, bool pending, uint32_t b, uint32_t k, uint32_t s,
                                             uint32_t rf) {
    const uint32_t lane = threadIdx.x & 63u;
    // a bucket with many updates in this group (a contested bucket that
    // failed the linear check): wave-parallel sequence, 64 updates per step
    for (;;) {
        const uint64_t pm = __ballot(pending);
        if (!pm) break;
        const uint32_t lead = (uint32_t)__ffsll((long long)pm) - 1;
        const uint32_t b0 = __shfl(b, lead, 64);
        const bool mine = pending && b == b0;
        const uint64_t m0 = __ballot(mine);
        if (__popcll(m0) < 8) break;
        const uint32_t rf0 = __shfl(rf, lead, 64);
        if (rf0 & 2u) {
            uint32_t F = L.sF[b0].y, S = L.sCS[b0].y;
            size_seq64(mine, k, s, F, S);
            if (lane == lead) { L.sCS[b0].y = S; L.sF[b0].y = F; }
        }
        if (rf0 & 1u) {
            uint32_t F = L.sF[b0].x, C = L.sCS[b0].x;
            count_seq64(mine, k, F, C);
            if (lane == lead) { L.sCS[b0].x = C; L.sF[b0].x = F; }
        }
        if (mine) pending = false;
    }
#if GNS_REPLAY_LEAD
    // the rest: the lowest lane of each bucket's lanes (its leader) takes the bucket's
    // state into registers and applies its peers' updates in lane (= stream) order,
    // fetched with cross-lane reads, then writes the state back once
    unsigned long long *peer = L.accS;  // per bucket: the mask of this group's lanes on it
    if (pending) atomicOr(&peer[b], 1ull << lane);
    __builtin_amdgcn_wave_barrier();
    const uint64_t pm = pending ? (uint64_t)peer[b] : 0ull;
    const bool leader = pending && (uint32_t)__ffsll((long long)pm) - 1 == lane;
    uint2 cs = make_uint2(0, 0), f = make_uint2(0, 0);
    if (leader) { cs = L.sCS[b]; f = L.sF[b]; }
    uint64_t rem = leader ? pm : 0ull;
    while (__ballot(rem != 0)) {
        const uint32_t src = rem ? (uint32_t)__ffsll((long long)rem) - 1 : lane;
        const uint32_t kp = __shfl(k, src, 64), sp = __shfl(s, src, 64);
        if (rem) {
            if (rf & 2u) {  // size half, count_min.go:99-128
                uint32_t S = cs.y, F = f.y;
                if (S == 0) { S = sp; F = kp; }
                else if (F == kp) S = S + sp;
                else if (sp > S) { S = sp; F = kp; }
                else S = S - sp;
                cs.y = S; f.y = F;
            }
            if (rf & 1u) {  // count half, count_min.go:130-155
                uint32_t C = cs.x, F = f.x;
                if (C == 0) { C = 1; F = kp; }
                else if (F == kp) C = C + 1;
                else { C = C - 1; if (C == 0) F = kp; }
                cs.x = C; f.x = F;
            }
            rem &= rem - 1;
        }
    }
    if (leader) { L.sCS[b] = cs; L.sF[b] = f; peer[b] = 0; }
#else
    uint32_t *own = reinterpret_cast<uint32_t *>(L.accS);
    while (__ballot(pending)) {
        if (pending) atomicMax(&own[b], 64u - lane);
        const bool win = pending && own[b] == 64u - lane;
        if (win) {
            // (bucket b belongs to this wave and one lane wins it per round: the
            // whole pair is read and written back)
            uint2 cs = L.sCS[b], f = L.sF[b];
            if (rf & 2u) {  // size half, count_min.go:99-128
                uint32_t S = cs.y, F = f.y;
                if (S == 0) { S = s; F = k; }
                else if (F == k) S = S + s;
                else if (s > S) { S = s; F = k; }
                else S = S - s;
                cs.y = S; f.y = F;
            }
            if (rf & 1u) {  // count half, count_min.go:130-155
                uint32_t C = cs.x, F = f.x;
                if (C == 0) { C = 1; F = k; }
                else if (F == k) C = C + 1;
                else { C = C - 1; if (C == 0) F = k; }
                cs.x = C; f.x = F;
            }
            L.sCS[b] = cs; L.sF[b] = f;
            own[b] = 0;
            pending = false;
        }
    }
#endif
}

// A tile's bucket state in registers (kTileMax / kApThreads buckets per thread):
// the next tile is loaded while the current one is stored, so a workgroup's
// tile loads and stores overlap instead of alternating.
constexpr uint32_t kTilePer = kTileMax / kApThreads;
static_assert(kTileMax % kApThreads == 0, "tile = whole items per thread");
constexpr uint64_t kNoTile = ~0ull;
struct TilePre {
    uint32_t c[kTilePer], fc[kTilePer], s[kTilePer], fs[kTilePer];
    uint64_t cbase;
};

__device__ __forceinline__ void tile_fetch(const ApplyArgs &a, TilePre &pre, uint64_t cbase, uint32_t tn) {
    pre.cbase = cbase;
#pragma unroll
    for (uint32_t m = 0; m < kTilePer; m++) {
        // unconditional (clamped) loads: every register is written on every path, so
        // the old values die at the tile fill and no wait precedes the loads
        const uint32_t i = min(threadIdx.x + m * kApThreads, tn - 1u);
        pre.c[m] = a.C[cbase + i]; pre.fc[m] = a.Fc[cbase + i];
        pre.s[m] = a.S[cbase + i]; pre.fs[m] = a.Fs[cbase + i];
    }
}

__device__ __forceinline__ void tile_none(TilePre &pre) {
    pre.cbase = kNoTile;
#pragma unroll
    for (uint32_t m = 0; m < kTilePer; m++) { pre.c[m] = 0; pre.fc[m] = 0; pre.s[m] = 0; pre.fs[m] = 0; }
}

// Where K4 reads a tile's updates: one contiguous range of the entry array, or
// (super-bins) the tile's run in each k_subpart round, in round order.  at(q, h)
// returns logical update q; h is the caller's running segment hint.
struct EntFlat {
    const uint64_t *p;
    struct Cur {};
    __device__ __forceinline__ uint64_t at(uint32_t q, Cur &) const { return p[q]; }
    __device__ __forceinline__ uint64_t at_any(uint32_t q) const { return p[q]; }
};
struct SegLds;
struct EntSegs {
    const uint64_t *p;
    const SegLds *G;       // run r holds logical [spre[r], spre[r+1]) at p + sbase[r] (tables in LDS)
    uint32_t off, nseg;    // this tile's table: entries off .. off + nseg (spre has nseg + 1)
    // a wave's current run [lo, hi) at base (wave-uniform; the lanes of a wave ask for
    // consecutive q, and q only grows along apply_tile's loads)
    struct Cur { uint32_t r = 0, lo = 0, hi = 0, base = 0; };
    __device__ __forceinline__ uint64_t at(uint32_t q, Cur &c) const;
    __device__ __forceinline__ uint64_t at_any(uint32_t q) const;
};

// Updates [beg, end) (stream order; logical indices of src) of one LDS tile:
// buckets cbase .. cbase+tn-1.
// pre holds this tile's state if it was prefetched (pre.cbase == cbase); on
// return it holds the state of the tile at next_cbase (kNoTile: none), loaded
// after this tile's stores were issued.
template <class Src>
__device__ __forceinline__ void apply_tile(const ApplyArgs &a, ApplyLds &L, const Src &ent, uint32_t beg,
                                           uint32_t end, uint64_t cbase, uint32_t tn, uint32_t col0,
                                           TilePre &pre, uint64_t next_cbase, uint32_t next_tn) {
    uint32_t *accN = L.accN;
    unsigned long long *accS = L.accS;
    uint16_t *s_list = L.s_list;
    uint32_t *s_wc = L.s_wc;
    uint32_t &s_any = L.s_any, &s_nlist = L.s_nlist;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
#ifdef GNS_K4_PROF
    // phase cycles: 0 classify, 1 decide, 2 compact, 3 replay clear + loop top, 4 replay gather,
    // 5 tile load + store, 6 replay groups
    uint64_t pt[7] = {0, 0, 0, 0, 0, 0, 0}, tprev = __builtin_amdgcn_s_memtime();
#define K4_MARK(i) do { if (tid == 0) { const uint64_t tn_ = __builtin_amdgcn_s_memtime(); pt[i] += tn_ - tprev; tprev = tn_; } } while (0)
#else
#define K4_MARK(i) do { } while (0)
#endif
    if (pre.cbase != cbase) tile_fetch(a, pre, cbase, tn);
#pragma unroll
    for (uint32_t m = 0; m < kTilePer; m++) {
        const uint32_t i = tid + m * kApThreads;
        if (i < tn) {
            L.sCS[i] = make_uint2(pre.c[m], pre.s[m]); L.sF[i] = make_uint2(pre.fc[m], pre.fs[m]);
            accN[i] = 0; accS[i] = 0;
        }
    }
#ifdef GNS_K4_PROF
    __syncthreads();
    K4_MARK(5);
#endif
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    uint64_t e[kApItems], en[kApItems];
    typename Src::Cur hint{};
#pragma unroll
    for (int j = 0; j < kApItems; j++) {  // first chunk
        const uint32_t q = beg + j * kApThreads + tid;
        e[j] = q < end ? ent.at(q, hint) : 0ull;
    }
    // engine counters in registers (global atomics inside the loop would be
    // drained by the next chunk's load waits)
    uint32_t st_chunks = 0, st_rep = 0, st_crep = 0;
#ifdef GNS_K4_PROF
    uint64_t pmax_sum = 0, psum_sum = 0;
    if (tid == 0) { L.s_pmax = 0; L.s_psum = 0; }
#endif
    for (uint32_t cb = beg; cb < end; cb += kApChunk) {
        if (tid == 0) { s_any = 0; st_chunks++; }
        __syncthreads();
        K4_MARK(3);
        bool v[kApItems];
        // --- classify against the chunk-entry state, aggregate per bucket ---
#pragma unroll
        for (int j = 0; j < kApItems; j++) {
            const uint32_t q = cb + j * kApThreads + tid;
            const uint32_t lo = (uint32_t)e[j];
            const uint32_t hi = (uint32_t)(e[j] >> 32);
            const uint32_t b = hi & (kTileMax - 1u);
            // bucket-range slice (exact global mode): other handles own the rest of the row
            v[j] = q < end && (col0 + b) - a.g.blo < a.g.bspan;
            const bool ovf = (lo & kOvfFlag) != 0;
            uint32_t incN = 0;
            uint64_t incS = 0;
            if (v[j] && !ovf) {
                const uint32_t s = hi >> kEntShift;
                const uint2 f = L.sF[b];
                const bool oc = lo != f.x, os = lo != f.y;
                incN = 1u | (uint32_t)oc << 14;
                incS = os ? (uint64_t)s << 32 : (uint64_t)s;
            }
            // (designated buckets never reach K4, so a wave's updates rarely share a
            // bucket: plain per-lane LDS atomics beat a wave-majority pre-sum here)
            if (v[j] && !ovf) {
                atomicAdd(&accN[b], incN);
                atomicAdd(&accS[b], (unsigned long long)incS);
            }
            if (v[j] && ovf) {  // size >= 2^20-1: always replayed
                atomicAdd(&accN[b], 1u);
                atomicOr(&accN[b], 1u << kAccForce);
            }
        }
        // prefetch the next chunk while this one is decided / replayed
#pragma unroll
        for (int j = 0; j < kApItems; j++) {
            const uint32_t q = cb + kApChunk + j * kApThreads + tid;
            en[j] = q < end ? ent.at(q, hint) : 0ull;
        }
        __syncthreads();
        K4_MARK(0);
        // --- per bucket: exact aggregate update or mark for replay ---
        for (uint32_t i = tid; i < tn; i += kApThreads) {
            const uint32_t an = accN[i];
            if (!an) continue;
            const uint32_t n = an & kM14;
            const uint32_t noc = (an >> 14) & kM14;
            const bool force = ((an >> kAccForce) & 1u) != 0;
            const uint64_t as = accS[i];
            const uint32_t so = (uint32_t)as, sx = (uint32_t)(as >> 32);
            uint32_t rep = 0;
            if (!force) {
                // count half: C > n_oth keeps C >= 2 before every foreign packet
                // (count_min.go:145-151 never reaches 0) and no wrap.
                uint2 cs = L.sCS[i];
                const uint32_t C = cs.x;
                const uint32_t nown = n - noc;
                if (C > noc && (uint64_t)C + nown < (1ull << 32)) cs.x = C + nown - noc;
                else rep |= 1u;
                // size half: S > sum_oth keeps S > s (and S > 0) before every foreign
                // packet (:115-125 never replaces, :103-107 never sees S == 0) and no
                // wrap; own packets add (:109-114)
                const uint32_t S = cs.y;
                if (S > sx && (uint64_t)S + so < (1ull << 32)) cs.y = S + so - sx;
                else rep |= 2u;
                L.sCS[i] = cs;
            } else {
                rep = 3u;
            }
            accS[i] = 0;
            accN[i] = rep;
            if (rep) s_any = 1;
        }
        __syncthreads();
        K4_MARK(1);
        if (s_any) {
            // --- stable compaction of the updates that need replay ---
            bool need[kApItems];
            uint64_t bal[kApItems];
#pragma unroll
            for (int j = 0; j < kApItems; j++) {
                const uint32_t b = (uint32_t)(e[j] >> 32) & (kTileMax - 1u);
                need[j] = v[j] && accN[b] != 0;
                bal[j] = __ballot(need[j]);
                if (lane == 0) s_wc[j * kApWaves + wave] = __popcll(bal[j]);
            }
            __syncthreads();
            if (wave == 0) {  // exclusive scan of the kApItems*kApWaves wave counts, (item, wave) order
                constexpr uint32_t NC = kApItems * kApWaves;
                constexpr uint32_t PER = (NC + 63) / 64;
                uint32_t x[PER], sum = 0;
#pragma unroll
                for (uint32_t q = 0; q < PER; q++) {
                    x[q] = lane * PER + q < NC ? s_wc[lane * PER + q] : 0u;
                    sum += x[q];
                }
                const uint32_t inc = wave_incl_scan(sum);
                uint32_t run = inc - sum;
#pragma unroll
                for (uint32_t q = 0; q < PER; q++) {
                    if (lane * PER + q < NC) s_wc[lane * PER + q] = run;
                    run += x[q];
                }
                if (lane == 63) s_nlist = inc;
            }
            __syncthreads();
#pragma unroll
            for (int j = 0; j < kApItems; j++)
                if (need[j]) {
                    const uint32_t pos = s_wc[j * kApWaves + wave] + __popcll(bal[j] & lt_mask);
                    s_list[pos] = (uint16_t)(j * kApThreads + tid);
                    if (pos < kRepCap) L.s_rep[pos] = e[j];
                }
            __syncthreads();
            const uint32_t nlist = s_nlist;
            K4_MARK(2);
            st_rep += nlist;
            st_crep++;
            // --- sequential replay (count_min.go:99-155), in order.  Buckets are
            //     partitioned over the 16 waves (b % 16); each wave walks the
            //     list in order and applies its buckets' updates; lanes of one
            //     64-item group hitting distinct buckets run in parallel,
            //     same-bucket lanes in lane order (lowest lane wins a round).
            // Each wave first gathers the list positions of its own buckets (stream
            // order) into its slice of s_list, which is free once every replay entry
            // sits in s_rep, then replays only those: ~nlist/16 items instead of a
            // walk over the whole list.  A wave whose slice overflows walks the list.
            constexpr uint32_t kWl = kApChunk / kApWaves;
            uint32_t nmine = 0xFFFFFFFFu;
            if (nlist <= kRepCap) {
                uint16_t *wl = s_list + wave * kWl;
                uint32_t c = 0;
                for (uint32_t g0 = 0; g0 < nlist; g0 += 64) {
                    const uint32_t i = g0 + lane;
                    const bool mine = i < nlist && ((uint32_t)(L.s_rep[i] >> 32) & (kTileMax - 1u)) % kApWaves == wave;
                    const uint64_t m = __ballot(mine);
                    const uint32_t pos = c + __popcll(m & lt_mask);
                    if (mine && pos < kWl) wl[pos] = (uint16_t)i;
                    c += __popcll(m);
                }
                if (c <= kWl) nmine = c;
            }
            K4_MARK(4);
#ifdef GNS_K4_PROF
            const uint64_t t_rep0 = __builtin_amdgcn_s_memtime();
#endif
            if (nmine != 0xFFFFFFFFu) {
                const uint16_t *wl = s_list + wave * kWl;
                for (uint32_t g0 = 0; g0 < nmine; g0 += 64) {
                    const uint32_t j = g0 + lane;
                    bool pending = j < nmine;
                    uint32_t b = 0, k = 0, s = 0, rf = 0;
                    if (pending) {
                        const uint64_t ee = L.s_rep[wl[j]];
                        b = (uint32_t)(ee >> 32) & (kTileMax - 1u);
                        decode_entry(a.ovf, ee, k, s);
                        rf = (uint32_t)accN[b];
                    }
                    replay_group(L, pending, b, k, s, rf);
                }
                K4_MARK(6);
                __builtin_amdgcn_wave_barrier();
                for (uint32_t j = lane; j < nmine; j += 64) accN[(uint32_t)(L.s_rep[wl[j]] >> 32) & (kTileMax - 1u)] = 0;
            } else {
            for (uint32_t g0 = 0; g0 < nlist; g0 += 64) {
                const uint32_t i = g0 + lane;
                bool pending = false;
                uint32_t b = 0, k = 0, s = 0, rf = 0;
                if (i < nlist) {
                    const uint64_t ee = i < kRepCap ? L.s_rep[i] : ent.at_any(cb + s_list[i]);
                    b = (uint32_t)(ee >> 32) & (kTileMax - 1u);
                    pending = b % kApWaves == wave;
                    if (pending) {
                        decode_entry(a.ovf, ee, k, s);
                        rf = (uint32_t)accN[b];
                    }
                }
                replay_group(L, pending, b, k, s, rf);
            }
            // this wave's buckets are done: clear their replay flags
            __builtin_amdgcn_wave_barrier();
            for (uint32_t g0 = 0; g0 < nlist; g0 += 64) {
                const uint32_t i = g0 + lane;
                if (i < nlist) {
                    const uint64_t ee = i < kRepCap ? L.s_rep[i] : ent.at_any(cb + s_list[i]);
                    const uint32_t b = (uint32_t)(ee >> 32) & (kTileMax - 1u);
                    if (b % kApWaves == wave) accN[b] = 0;
                }
            }
            }
#ifdef GNS_K4_PROF
            {
                const uint32_t dt = (uint32_t)(__builtin_amdgcn_s_memtime() - t_rep0);
                if (lane == 0) { atomicMax(&L.s_pmax, dt); atomicAdd(&L.s_psum, dt); }
            }
#endif
        }
        __syncthreads();
#ifdef GNS_K4_PROF
        if (tid == 0) { pmax_sum += L.s_pmax; psum_sum += L.s_psum; L.s_pmax = 0; L.s_psum = 0; }
#endif
#pragma unroll
        for (int j = 0; j < kApItems; j++) e[j] = en[j];
    }
    // next tile's loads first, then this tile's stores: both are in flight together
    if (next_cbase != kNoTile) tile_fetch(a, pre, next_cbase, next_tn);
    else tile_none(pre);
    for (uint32_t i = tid; i < tn; i += kApThreads) {
        const uint2 cs = L.sCS[i], f = L.sF[i];
        a.C[cbase + i] = cs.x; a.Fc[cbase + i] = f.x;
        a.S[cbase + i] = cs.y; a.Fs[cbase + i] = f.y;
    }
#ifdef GNS_K4_PROF
    if (tid == 0) { atomicAdd(&a.stats[kStatsProf + 8], (unsigned long long)pmax_sum); atomicAdd(&a.stats[kStatsProf + 9], (unsigned long long)psum_sum); }
#endif
    if (tid == 0) {
        atomicAdd(&a.stats[5], (unsigned long long)st_rep);
        atomicAdd(&a.stats[6], (unsigned long long)st_chunks);
        if (st_crep) atomicAdd(&a.stats[7], (unsigned long long)st_crep);
    }
#ifdef GNS_K4_PROF
    __syncthreads();
    K4_MARK(5);
    if (tid == 0) for (int i = 0; i < 7; i++) atomicAdd(&a.stats[kStatsProf + i], (unsigned long long)pt[i]);
#endif
}

constexpr uint32_t kSubPairs = kApItems * kApWaves;  // (item, wave) groups of a k_subpart round, in stream order

// Super-bin sub-partition as a launch of its own, one workgroup per super-bin and
// two per CU (16 KB of LDS instead of K4's 156 KB), so that its barrier- and
// latency-bound rounds overlap across workgroups instead of running inside K4's
// one-workgroup-per-CU loop.  One pass: every round of kApChunk updates is
// grouped by tile in place of the round (stable inside each tile), and the
// round's tile starts go to rseg; K4 reads a tile as its run in each round, in
// round order, which is the tile's stream order.  (Round 4 counted every tile of
// the bin first and wrote each tile contiguously: a second read of every update.)
// Round r of bin b has index beg/kApChunk + r + b: unique
// and below total/kApChunk + nbins.
#ifndef GNS_SEG_ALL
#define GNS_SEG_ALL 416
#endif
constexpr uint32_t kSegAll = GNS_SEG_ALL;  // table entries (8 B each; K4's LDS is nearly full)
template <int NT>
__global__ __launch_bounds__(NT, NT == 512 ? 4 : 1) void k_subpart(ApplyArgs a, uint16_t *rseg) {
    constexpr int kW = NT / 64, kI = (int)kApChunk / NT;  // waves; updates per thread and round
    static_assert(kW * kI == (int)kSubPairs, "(item, wave) groups of a round");
    __shared__ uint32_t cnt[2][kSubPairs * 16];
    __shared__ uint32_t ttot[2][16];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t bin = blockIdx.x;  // block-uniform exit below
    const uint32_t sub_bits = a.g.sub_bits, nsub = 1u << sub_bits, tile_bits = a.g.tile_bits;
    const uint32_t beg = a.offsets[bin];
    const uint32_t end = (bin + 1 < a.g.nbins_all) ? a.offsets[bin + 1] : *a.total;
    if (beg >= end) return;
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    // a bin too big for K4's tables goes to the second K4 launch, which exits at once without one
    if (tid == 0 && (end - beg + kApChunk - 1) / kApChunk + 1 > kSegAll) atomicAdd(a.work + 2, 1u);
    if (tid < 32) (&ttot[0][0])[tid] = 0;
    uint64_t e[kI], en[kI];
#pragma unroll
    for (int j = 0; j < kI; j++) {
        const uint32_t q = beg + j * NT + tid;
        e[j] = q < end ? a.entries[q] : 0ull;
    }
    __syncthreads();
    uint32_t par = 0;
    for (uint32_t rb = beg; rb < end; rb += kApChunk) {
        uint32_t *cb = cnt[par], *tt = ttot[par];
        // the next round's updates load while this round is ranked and stored
#pragma unroll
        for (int j = 0; j < kI; j++) {
            const uint32_t q = rb + kApChunk + j * NT + tid;
            en[j] = q < end ? a.entries[q] : 0ull;
        }
        uint32_t sb[kI];  // tile | rank among the wave's earlier updates of the tile << 8
#pragma unroll
        for (int j = 0; j < kI; j++) {
            const uint32_t q = rb + j * NT + tid;
            const bool valid = q < end;
            const uint32_t sub = valid ? (((uint32_t)(e[j] >> 32) & kLowMask) >> tile_bits) : 0xFFu;
            uint64_t peers = __ballot(valid);
            for (uint32_t bit = 0; bit < sub_bits; bit++) {
                const uint64_t m = __ballot(valid && ((sub >> bit) & 1u));
                peers &= ((sub >> bit) & 1u) ? m : ~m;
            }
            const uint32_t before = __popcll(peers & lt_mask);
            sb[j] = sub | before << 8;
            // this wave's slots of group (j, wave): zeroed, then the first lane of
            // each tile's peers writes the count (one wave: LDS ops stay in order)
            if (lane < 16) cb[(j * kW + wave) * 16 + lane] = 0;
            if (valid && before == 0) {
                const uint32_t c = (uint32_t)__popcll(peers);
                cb[(j * kW + wave) * 16 + sub] = c;
                atomicAdd(&tt[sub], c);
            }
        }
        __syncthreads();
        if (wave < nsub) {  // (nsub <= kW) wave t: tile t's start in the round + exclusive scan of its group counts
            constexpr uint32_t GPL = kSubPairs / 64;  // groups per lane (1 or 2)
            static_assert(GPL * 64 == kSubPairs && GPL <= 2, "one or two groups per lane");
            const uint32_t t = wave;
            uint32_t b0 = 0;
            for (uint32_t u = 0; u < t; u++) b0 += tt[u];
            const uint32_t x0 = cb[(GPL * lane) * 16 + t], x1 = GPL == 2 ? cb[(GPL * lane + 1) * 16 + t] : 0u;
            const uint32_t inc = wave_incl_scan(x0 + x1);
            const uint32_t ex = b0 + inc - (x0 + x1);
            cb[(GPL * lane) * 16 + t] = ex;
            if (GPL == 2) cb[(GPL * lane + 1) * 16 + t] = ex + x0;
            if (lane == 0) rseg[((uint64_t)(rb / kApChunk) + bin) * 16 + t] = (uint16_t)b0;
        }
        // the next round's tile totals (last read in the previous round, before this round's first barrier)
        if (tid >= NT - 16) ttot[par ^ 1u][tid - (NT - 16)] = 0;
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kI; j++)
            if ((sb[j] & 0xFFu) != 0xFFu) a.entries2[rb + cb[(j * kW + wave) * 16 + (sb[j] & 0xFFu)] + (sb[j] >> 8)] = e[j];
#pragma unroll
        for (int j = 0; j < kI; j++) e[j] = en[j];
        par ^= 1u;
    }
}

// K4's view of a super-bin's tiles: each tile's run in every k_subpart round, in
// round order, with the runs' logical starts scanned.  All tiles' tables are built
// at the bin's start (wave t scans tile t: one barrier per bin) when they fit
// kSegAll entries (nsub * (rounds + 1): every C5 bin of typical size); otherwise
// one tile at a time in windows of rounds (a tile spread over several windows is
// stored and reloaded between them).
struct SegLds {
    uint32_t tot[16];             // the super-bin's updates per tile
    uint32_t sbase[kSegAll];      // physical start of a tile's run in a round
    uint32_t spre[kSegAll];       // logical start of each run, then the table's total
};

// The run of the wave's first lane comes from the cursor, advanced (wave-uniform
// reads, bisection) only when that lane has left it: about once per 16 wave loads
// at the bench geometry.  Lanes past the run's end step forward on their own.
__device__ __forceinline__ uint64_t EntSegs::at(uint32_t q, Cur &c) const {
    const uint32_t *spre = G->spre + off, *sbase = G->sbase + off;
    const uint32_t qf = __builtin_amdgcn_readfirstlane(q);
    if (qf >= c.hi) {  // wave-uniform
        uint32_t lo = c.r, hi = nseg;  // largest r with spre[r] <= qf (empty runs skipped)
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (spre[mid] <= qf) lo = mid; else hi = mid;
        }
        c.r = __builtin_amdgcn_readfirstlane(lo);
        c.lo = __builtin_amdgcn_readfirstlane(spre[c.r]);
        c.hi = __builtin_amdgcn_readfirstlane(spre[c.r + 1]);
        c.base = __builtin_amdgcn_readfirstlane(sbase[c.r]);
    }
    uint32_t idx = c.base + (q - c.lo);
    if (q >= c.hi) {
        uint32_t r2 = c.r + 1;
        while (spre[r2 + 1] <= q) r2++;  // spre[nseg] = the total > q
        idx = sbase[r2] + (q - spre[r2]);
    }
    return p[idx];
}

__device__ __forceinline__ uint64_t EntSegs::at_any(uint32_t q) const {
    const uint32_t *spre = G->spre + off, *sbase = G->sbase + off;
    uint32_t lo = 0, hi = nseg;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (spre[mid] <= q) lo = mid; else hi = mid;
    }
    return p[sbase[lo] + (q - spre[lo])];
}

// One wave: tile st's runs of rounds [w0, w0 + nr) into the table at off (nr + 1 entries).
__device__ __forceinline__ uint32_t seg_scan_wave(const ApplyArgs &a, SegLds &G, uint32_t beg, uint32_t end,
                                                  uint64_t ridx0, uint32_t nsub, uint32_t st, uint32_t w0,
                                                  uint32_t nr, uint32_t off) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t carry = 0;
    for (uint32_t i0 = 0; i0 < nr; i0 += 64) {
        const uint32_t i = i0 + lane;
        uint32_t len = 0;
        if (i < nr) {
            const uint32_t r = w0 + i;
            const uint32_t rb = beg + r * kApChunk, rl = min(kApChunk, end - rb);
            const uint16_t *rs = a.rseg + (ridx0 + r) * 16;
            const uint32_t s0 = rs[st], e0 = st + 1 < nsub ? rs[st + 1] : rl;
            G.sbase[off + i] = rb + s0;
            len = e0 - s0;
        }
        const uint32_t inc = wave_incl_scan(len);
        if (i < nr) G.spre[off + i] = carry + inc - len;
        carry += __shfl(inc, 63, 64);
    }
    if (lane == 0) G.spre[off + nr] = carry;
    return carry;
}

__device__ __forceinline__ void seg_totals(const ApplyArgs &a, SegLds &G, uint32_t beg, uint32_t end,
                                           uint64_t ridx0, uint32_t nsub) {
    const uint32_t tid = threadIdx.x;
    if (tid < 16) G.tot[tid] = 0;
    __syncthreads();
    const uint32_t R = (end - beg + kApChunk - 1) / kApChunk;
    for (uint32_t i = tid; i < R * nsub; i += kApThreads) {
        const uint32_t r = i / nsub, t = i % nsub;
        const uint32_t rl = min(kApChunk, end - (beg + r * kApChunk));
        const uint16_t *rs = a.rseg + (ridx0 + r) * 16;
        const uint32_t e = t + 1 < nsub ? rs[t + 1] : rl;
        if (e > rs[t]) atomicAdd(&G.tot[t], e - rs[t]);
    }
    __syncthreads();
}

// Persistent: each workgroup takes bins from the size-ordered schedule through
// a work counter, one bin ahead, so the next tile's state can be loaded while
// the current tile is stored.
struct ApplyTile {
    uint32_t bin;
    uint32_t beg, end;  // update range in the bin (super-bin: sub-partitioned later)
    uint32_t r, bbase;  // row, first bucket of the bin
    bool valid;
};

__device__ __forceinline__ ApplyTile apply_bin(const ApplyArgs &a, uint32_t k) {
    ApplyTile t{};
    t.valid = false;
    if (k >= a.g.nbins) return t;
    const uint32_t bin = a.order ? a.order[k] : k;
    t.bin = bin;
    t.beg = a.offsets[bin];
    t.end = (bin + 1 < a.g.nbins_all) ? a.offsets[bin + 1] : *a.total;
    t.r = bin / a.g.ntiles;
    t.bbase = (bin % a.g.ntiles) << a.g.bin_bits;
    t.valid = true;
    return t;
}

// MODE 0: rows of single tiles (bins = tiles); 1: super-bins read through k_subpart's
// rounds (3: the super-bins too big for MODE 1's tables, a second launch).  One
// variant per launch, so each inlines only its own tile loop (and stays within 128
// VGPRs).
template <int MODE>
__global__ __launch_bounds__(kApThreads) void k_apply(ApplyArgs a) {
    __shared__ ApplyLds L;
    __shared__ SegLds G;
    __shared__ uint32_t s_k;
    const CmGeom &g = a.g;
    const uint32_t tid = threadIdx.x;
    const uint32_t tw = 1u << g.tile_bits;
    TilePre pre;
    tile_none(pre);
    if constexpr (MODE == 3) {
        if (a.work[2] == 0) return;  // no bin needs windows (k_subpart counts them): the common case
    }
    unsigned int *work = a.work + (MODE == 3 ? 1 : 0);
    if (tid == 0) s_k = atomicAdd(work, 1u);
    __syncthreads();
    uint32_t k = s_k;
    __syncthreads();
    while (k < g.nbins) {
        if (tid == 0) s_k = atomicAdd(work, 1u);  // the bin after this one
        const ApplyTile cur = apply_bin(a, k);
        __syncthreads();
        const uint32_t kn = s_k;
        const ApplyTile nxt = apply_bin(a, kn);
        // first tile of the next bin (its state is prefetched; a super-bin's first
        // tile may turn out empty, which only wastes that prefetch)
        uint64_t nb_cbase = kNoTile;
        uint32_t nb_tn = 0;
        if (MODE != 3 && nxt.valid && nxt.beg < nxt.end && nxt.bbase < g.w) {
            nb_cbase = (uint64_t)nxt.r * g.w + nxt.bbase;
            nb_tn = min(tw, g.w - nxt.bbase);
        }
        if (cur.beg < cur.end) {
            if constexpr (MODE == 0) {
                apply_tile(a, L, EntFlat{a.entries}, cur.beg, cur.end, (uint64_t)cur.r * g.w + cur.bbase,
                           min(tw, g.w - cur.bbase), cur.bbase, pre, nb_cbase, nb_tn);
            } else {
                const uint32_t nsub = 1u << g.sub_bits;
                {  // MODE 1 / 3: rounds grouped by tile (k_subpart)
                    const uint64_t ridx0 = (uint64_t)(cur.beg / kApChunk) + cur.bin;
                    const uint32_t R = (cur.end - cur.beg + kApChunk - 1) / kApChunk;
                    // MODE 1: bins whose tables fit kSegAll, all tiles' at once or (bigger bins)
                    // one tile's at a time; MODE 3 (a second launch): the rest
                    const bool all = nsub * (R + 1) <= kSegAll;  // block-uniform
                    const bool fits = R + 1 <= kSegAll;
                    if ((MODE == 1) == fits) {
                        if (MODE == 1 && all) {
                            for (uint32_t t = tid >> 6; t < nsub; t += kApWaves) {  // wave t (mod waves): tile t
                                const uint32_t tot = seg_scan_wave(a, G, cur.beg, cur.end, ridx0, nsub, t, 0, R, t * (R + 1));
                                if ((tid & 63u) == 0) G.tot[t] = tot;
                            }
                            __syncthreads();
                        } else {
                            seg_totals(a, G, cur.beg, cur.end, ridx0, nsub);
                        }
                        for (uint32_t st = 0; st < nsub; st++) {
                            const uint32_t tbase = cur.bbase + (st << g.tile_bits);
                            if (tbase >= g.w || G.tot[st] == 0) continue;
                            uint64_t ncb = nb_cbase;
                            uint32_t ntn = nb_tn;
                            for (uint32_t s2 = st + 1; s2 < nsub; s2++) {
                                const uint32_t tb2 = cur.bbase + (s2 << g.tile_bits);
                                if (tb2 < g.w && G.tot[s2]) {
                                    ncb = (uint64_t)cur.r * g.w + tb2;
                                    ntn = min(tw, g.w - tb2);
                                    break;
                                }
                            }
                            const uint64_t cbase = (uint64_t)cur.r * g.w + tbase;
                            const uint32_t tn = min(tw, g.w - tbase);
                            if constexpr (MODE == 1) {
                                uint32_t off = st * (R + 1);
                                if (!all) {
                                    if (tid < 64) seg_scan_wave(a, G, cur.beg, cur.end, ridx0, nsub, st, 0, R, 0);
                                    __syncthreads();
                                    off = 0;
                                }
                                apply_tile(a, L, EntSegs{a.entries2, &G, off, R}, 0u, G.tot[st], cbase, tn, tbase, pre,
                                           ncb, ntn);
                                __syncthreads();
                            } else {
                                // windows of rounds; a tile spread over several is stored and
                                // reloaded between them (no prefetch of itself)
                                constexpr uint32_t kWin = kSegAll - 1;
                                for (uint32_t w0 = 0; w0 < R; w0 += kWin) {
                                    const uint32_t nr = min(kWin, R - w0);
                                    if (tid < 64) seg_scan_wave(a, G, cur.beg, cur.end, ridx0, nsub, st, w0, nr, 0);
                                    __syncthreads();
                                    const uint32_t n = G.spre[nr];
                                    const bool last = w0 + kWin >= R;
                                    if (n)
                                        apply_tile(a, L, EntSegs{a.entries2, &G, 0u, nr}, 0u, n, cbase, tn, tbase, pre,
                                                   last ? ncb : kNoTile, last ? ntn : 0u);
                                    __syncthreads();
                                }
                            }
                        }
                    }
                }
            }
        }
        __syncthreads();
        k = kn;
    }
}

// ---------------------------------------------------------------------------
// K4 over super-bins without the tile sweep (round 6; rows wider than the
// bins K3s can count, configs[4]: d=8 w=2^24, 512 super-bins of 8 tiles per
// row).  A 100M-packet batch gives a cold update to only ~6% of the 2^27
// buckets, so loading and storing every tile's 64 KB of state (2 GB per batch
// each way) and sub-partitioning every super-bin by tile first (k_subpart: a
// second read and write of all updates) cost more than the updates themselves.
// Here a workgroup takes a super-bin's updates in K3s's stream order and keeps
// only the buckets they touch, in an LDS hash table whose slots ARE the tile
// state slots of apply_tile: an update's bucket field is rewritten to its slot,
// so classify / decide / compaction / replay run unchanged.  A new bucket's
// state is gathered when its key is inserted; the table is written back (and
// cleared) when it fills and at the end of the bin.  A chunk whose buckets do
// not fit the table even after a write-back is taken in halves (a piece of 64
// updates always fits): buckets are independent, so writing state back between
// pieces of the stream changes nothing.
// ---------------------------------------------------------------------------
#ifdef GNS_SP_PROF  // profiling build: k_apply_sparse phase cycles of thread 0, each phase ending at a barrier
// 0 map probes, 1 gather + rewrite, 2 classify, 3 decide, 4 compact + replay, 5 flush, 6 loop top
#define SP_MARK(i) do { if (threadIdx.x == 0) { const uint64_t tn_ = __builtin_amdgcn_s_memtime(); sp_pt[i] += tn_ - sp_prev; sp_prev = tn_; } } while (0)
#define SP_PT , uint64_t (&sp_pt)[7], uint64_t &sp_prev
#define SP_PTA , sp_pt, sp_prev
#else
#define SP_MARK(i) do { } while (0)
#define SP_PT
#define SP_PTA
#endif
constexpr uint32_t kSpHashCap = kTileMax - kTileMax / 8;  // used slots before the table counts as full
constexpr uint32_t kSpProbe = 64;
constexpr uint32_t kSpNoSlot = 0xFFFFFFFFu;

struct alignas(16) SparseLds {
    uint32_t key[kTileMax];  // 0 empty, else bucket-in-bin + 1
    uint32_t used, ovf;
};

// Probe order of a bucket: its two home groups of 4 key positions (two hashes), then the groups
// after the second.  sp_map reads both home groups at once (two 16-byte LDS loads, one round
// trip), so a mapped bucket costs one read whatever the load, and an insert one compare-and-swap.
// A key sits at the first position of its order that was empty when it arrived (keys are never
// removed before a flush), so a lookup may stop at the first empty position.  A key at position
// p keeps its state in slot sp_perm(p): most keys sit in their group's first position, and
// without the permutation their slots would all be 0 mod 4, a quarter of the LDS banks, for every
// later access to the slot state.
constexpr uint32_t kSpGroups = kTileMax / 4u;
__device__ __forceinline__ void sp_groups(uint32_t b, uint32_t &g1, uint32_t &g2) {
    // b < 2^24 (a super-bin's bucket): 24-bit multiplies (full rate; a 32-bit one is quarter rate)
    // (HIP's __umul24 returns int: shift the unsigned bits)
    g1 = ((uint32_t)__umul24(b, 0x9E3779u) >> (32 - kTileBitsMax + 2)) & (kSpGroups - 1u);
    g2 = ((uint32_t)__umul24(b, 0x85EBCBu) >> (32 - kTileBitsMax + 2)) & (kSpGroups - 1u);
    if (g2 == g1) g2 = (g2 + 1u) & (kSpGroups - 1u);
}
__device__ __forceinline__ uint32_t sp_group(uint32_t g1, uint32_t g2, uint32_t k) {
    return k == 0u ? g1 : (g2 + k - 1u) & (kSpGroups - 1u);
}
// key position <-> state slot (an involution: bits 6..7 of p pick the XOR of its bits 0..1)
__device__ __forceinline__ uint32_t sp_perm(uint32_t p) { return p ^ ((p >> 6) & 3u); }

// slot of a bucket that is in the table (the replay fallback re-reads raw updates); every
// valid update of the piece was mapped, so a miss is an engine invariant broken: it raises
// stats[9], which the next flush reports as GNS_E_HIP
__device__ __forceinline__ uint32_t sp_find(const SparseLds &H, uint32_t b, unsigned long long *stats) {
    uint32_t g1, g2;
    sp_groups(b, g1, g2);
    const uint32_t key = b + 1;
    for (uint32_t k = 0; k <= kSpGroups; k++) {
        const uint32_t g = sp_group(g1, g2, k);
        for (uint32_t t = 0; t < 4u; t++)
            if (H.key[g * 4u + t] == key) return sp_perm(g * 4u + t);
    }
    atomicOr(&stats[9], 1ull);
    return 0;
}

// raw update -> the same update with its bucket field replaced by its slot
__device__ __forceinline__ uint64_t sp_rewrite(uint64_t e, uint32_t slot) {
    return (e & ~((uint64_t)(kTileMax - 1u) << 32)) | ((uint64_t)slot << 32);
}

// Write every used slot's state back to its bucket and clear the table.
__device__ __forceinline__ void sp_flush(const ApplyArgs &a, ApplyLds &L, SparseLds &H, uint64_t cbase SP_PT) {
    __syncthreads();
    SP_MARK(6);
    for (uint32_t i = threadIdx.x; i < kTileMax; i += kApThreads) {  // i: slot
        const uint32_t k = H.key[sp_perm(i)];
        if (k) {
            const uint64_t c = cbase + (k - 1u);
            const uint2 cs = L.sCS[i], f = L.sF[i];
            a.C[c] = cs.x; a.Fc[c] = f.x;
            a.S[c] = cs.y; a.Fs[c] = f.y;
            H.key[sp_perm(i)] = 0;
        }
    }
    if (threadIdx.x == 0) { H.used = 0; H.ovf = 0; }
    __syncthreads();
    SP_MARK(5);
}

// Map the updates of [lo, hi) (logical indices; the chunk's items e[j] at cb + j * threads + tid)
// to slots, gathering new buckets' state.  On success the in-range valid items are rewritten and
// their bits set in vm; on overflow nothing is rewritten and false is returned (block-uniform).
__device__ __forceinline__ bool sp_map(const ApplyArgs &a, ApplyLds &L, SparseLds &H, uint64_t (&e)[kApItems],
                                       uint32_t &vm, uint32_t cb, uint32_t lo, uint32_t hi, uint32_t end,
                                       uint64_t cbase, uint32_t col0, uint32_t bmask SP_PT) {
    const uint32_t tid = threadIdx.x;
    uint32_t sl[kApItems], nnew = 0;
#ifdef GNS_SP_PROF
    __syncthreads();
    SP_MARK(6);
#endif
#pragma unroll
    for (int j = 0; j < kApItems; j++) {
        sl[j] = kSpNoSlot;
        const uint32_t q = cb + j * kApThreads + tid;
        const uint32_t b = (uint32_t)(e[j] >> 32) & bmask;
        // bucket-range slice (exact global mode): other handles own the rest of the row
        if (q >= lo && q < hi && q < end && (col0 + b) - a.g.blo < a.g.bspan) {
            const uint32_t key = b + 1u;
            uint32_t g1, g2, k = 0;
            sp_groups(b, g1, g2);
            for (uint32_t p = 0; p < kSpProbe; p++) {
                const uint32_t ga = sp_group(g1, g2, k), gb = sp_group(g1, g2, k + 1u);
                const uint4 A = *reinterpret_cast<const uint4 *>(&H.key[ga * 4u]);
                const uint4 B = *reinterpret_cast<const uint4 *>(&H.key[gb * 4u]);
                // both reads in flight before either is used (one round trip, not two)
                asm volatile("" ::"v"(A.x), "v"(B.x));
                // the first position of the pair that holds the key or is empty
                uint32_t pos = 8u, val = 0u;
#define SP_AT(i_, v_) if ((v_) == key || (v_) == 0u) { pos = (i_); val = (v_); }
                SP_AT(7u, B.w) SP_AT(6u, B.z) SP_AT(5u, B.y) SP_AT(4u, B.x)
                SP_AT(3u, A.w) SP_AT(2u, A.z) SP_AT(1u, A.y) SP_AT(0u, A.x)
#undef SP_AT
                if (pos == 8u) { k += 2u; continue; }  // both full: the next two groups
                const uint32_t h = (pos < 4u ? ga : gb) * 4u + (pos & 3u);
                if (val == key) { sl[j] = sp_perm(h); break; }
                const uint32_t old = atomicCAS(&H.key[h], 0u, key);
                if (old == 0u) {  // new bucket: its state is gathered below
                    nnew++;
                    L.accN[sp_perm(h)] = 1u;
                    sl[j] = sp_perm(h);
                    break;
                }
                if (old == key) { sl[j] = sp_perm(h); break; }
                // taken by another key meanwhile: read the pair again
            }
            if (sl[j] == kSpNoSlot) H.ovf = 1u;
        }
    }
    // slots taken: one add per wave (the first chunk of a bin inserts most of its buckets)
    const uint32_t wnew = __ockl_wfred_add_u32(nnew);
    if ((tid & 63u) == 0 && wnew && atomicAdd(&H.used, wnew) + wnew > kSpHashCap) H.ovf = 1u;
    __syncthreads();
    SP_MARK(0);
    // Gather the new buckets' state, slot-major: a lane's loads for its four slots are all in
    // flight at once (gathering at the insert waited out one load latency per item and wave).
    // Runs whether or not the piece fits, so a flush writes back gathered state only.  accN is
    // zero between chunks (sp_chunk clears what it sets); the marks are cleared here.
    {
        constexpr uint32_t kPer = kTileMax / kApThreads;
        uint32_t cv[kPer], sv[kPer], fcv[kPer], fsv[kPer], gm = 0;
#pragma unroll
        for (uint32_t q = 0; q < kPer; q++) {
            const uint32_t i = q * kApThreads + tid;
            if (L.accN[i]) {
                gm |= 1u << q;
                const uint64_t c = cbase + (H.key[sp_perm(i)] - 1u);
                cv[q] = a.C[c]; sv[q] = a.S[c]; fcv[q] = a.Fc[c]; fsv[q] = a.Fs[c];
            }
        }
#pragma unroll
        for (uint32_t q = 0; q < kPer; q++)
            if ((gm >> q) & 1u) {
                const uint32_t i = q * kApThreads + tid;
                L.sCS[i] = make_uint2(cv[q], sv[q]);
                L.sF[i] = make_uint2(fcv[q], fsv[q]);
                L.accN[i] = 0u;
            }
    }
    __syncthreads();
    const bool ok = H.ovf == 0u;
    if (ok) {
#pragma unroll
        for (int j = 0; j < kApItems; j++)
            if (sl[j] != kSpNoSlot) { e[j] = sp_rewrite(e[j], sl[j]); vm |= 1u << j; }
    }
    __syncthreads();  // every lane has read ovf before a flush may clear it
    SP_MARK(1);
    return ok;
}

// classify / decide / compact / replay of the mapped items (vm) of one chunk: apply_tile's
// chunk body over slots (tn = every slot of the table; unused slots have accN == 0)
__device__ __forceinline__ void sp_chunk(const ApplyArgs &a, ApplyLds &L, const SparseLds &H,
                                         const uint64_t (&e)[kApItems], uint32_t vm, uint32_t cb, uint32_t bmask,
                                         uint32_t &st_chunks, uint32_t &st_rep, uint32_t &st_crep SP_PT) {
    uint32_t *accN = L.accN;
    unsigned long long *accS = L.accS;
    uint16_t *s_list = L.s_list;
    uint32_t *s_wc = L.s_wc;
    uint32_t &s_any = L.s_any, &s_nlist = L.s_nlist;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint64_t lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    if (tid == 0) { s_any = 0; st_chunks++; }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < kApItems; j++) {
        if (!((vm >> j) & 1u)) continue;
        const uint32_t lo = (uint32_t)e[j];
        const uint32_t hi = (uint32_t)(e[j] >> 32);
        const uint32_t b = hi & (kTileMax - 1u);
        if (lo & kOvfFlag) {  // size >= 2^20-1: always replayed
            atomicAdd(&accN[b], 1u);
            atomicOr(&accN[b], 1u << kAccForce);
        } else {
            const uint32_t s = hi >> kEntShift;
            const uint2 f = L.sF[b];
            const bool oc = lo != f.x, os = lo != f.y;
            atomicAdd(&accN[b], 1u | (uint32_t)oc << 14);
            atomicAdd(&accS[b], (unsigned long long)(os ? (uint64_t)s << 32 : (uint64_t)s));
        }
    }
    __syncthreads();
    SP_MARK(2);
    for (uint32_t i = tid; i < kTileMax; i += kApThreads) {
        const uint32_t an = accN[i];
        if (!an) continue;
        const uint32_t n = an & kM14;
        const uint32_t noc = (an >> 14) & kM14;
        const bool force = ((an >> kAccForce) & 1u) != 0;
        const uint64_t as = accS[i];
        const uint32_t so = (uint32_t)as, sx = (uint32_t)(as >> 32);
        uint32_t rep = 0;
        if (!force) {
            uint2 cs = L.sCS[i];
            const uint32_t C = cs.x;
            const uint32_t nown = n - noc;
            if (C > noc && (uint64_t)C + nown < (1ull << 32)) cs.x = C + nown - noc;
            else rep |= 1u;
            const uint32_t S = cs.y;
            if (S > sx && (uint64_t)S + so < (1ull << 32)) cs.y = S + so - sx;
            else rep |= 2u;
            L.sCS[i] = cs;
        } else {
            rep = 3u;
        }
        accS[i] = 0;
        accN[i] = rep;
        if (rep) s_any = 1;
    }
    __syncthreads();
    SP_MARK(3);
    if (s_any) {
        bool need[kApItems];
        uint64_t bal[kApItems];
#pragma unroll
        for (int j = 0; j < kApItems; j++) {
            const uint32_t b = (uint32_t)(e[j] >> 32) & (kTileMax - 1u);
            need[j] = ((vm >> j) & 1u) && accN[b] != 0;
            bal[j] = __ballot(need[j]);
            if (lane == 0) s_wc[j * kApWaves + wave] = __popcll(bal[j]);
        }
        __syncthreads();
        if (wave == 0) {
            constexpr uint32_t NC = kApItems * kApWaves;
            constexpr uint32_t PER = (NC + 63) / 64;
            uint32_t x[PER], sum = 0;
#pragma unroll
            for (uint32_t q = 0; q < PER; q++) {
                x[q] = lane * PER + q < NC ? s_wc[lane * PER + q] : 0u;
                sum += x[q];
            }
            const uint32_t inc = wave_incl_scan(sum);
            uint32_t run = inc - sum;
#pragma unroll
            for (uint32_t q = 0; q < PER; q++) {
                if (lane * PER + q < NC) s_wc[lane * PER + q] = run;
                run += x[q];
            }
            if (lane == 63) s_nlist = inc;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < kApItems; j++)
            if (need[j]) {
                const uint32_t pos = s_wc[j * kApWaves + wave] + __popcll(bal[j] & lt_mask);
                s_list[pos] = (uint16_t)(j * kApThreads + tid);
                if (pos < kRepCap) L.s_rep[pos] = e[j];
            }
        __syncthreads();
        const uint32_t nlist = s_nlist;
        st_rep += nlist;
        st_crep++;
        // the list's entries beyond kRepCap are re-read raw and mapped to their slots again
        auto rep_entry = [&](uint32_t i) -> uint64_t {
            if (i < kRepCap) return L.s_rep[i];
            const uint64_t raw = a.entries[cb + s_list[i]];
            return sp_rewrite(raw, sp_find(H, (uint32_t)(raw >> 32) & bmask, a.stats));
        };
        constexpr uint32_t kWl = kApChunk / kApWaves;
        uint32_t nmine = 0xFFFFFFFFu;
        if (nlist <= kRepCap) {
            uint16_t *wl = s_list + wave * kWl;
            uint32_t c = 0;
            for (uint32_t g0 = 0; g0 < nlist; g0 += 64) {
                const uint32_t i = g0 + lane;
                const bool mine = i < nlist && ((uint32_t)(L.s_rep[i] >> 32) & (kTileMax - 1u)) % kApWaves == wave;
                const uint64_t m = __ballot(mine);
                const uint32_t pos = c + __popcll(m & lt_mask);
                if (mine && pos < kWl) wl[pos] = (uint16_t)i;
                c += __popcll(m);
            }
            if (c <= kWl) nmine = c;
        }
        if (nmine != 0xFFFFFFFFu) {
            const uint16_t *wl = s_list + wave * kWl;
            for (uint32_t g0 = 0; g0 < nmine; g0 += 64) {
                const uint32_t j = g0 + lane;
                bool pending = j < nmine;
                uint32_t b = 0, k = 0, s = 0, rf = 0;
                if (pending) {
                    const uint64_t ee = L.s_rep[wl[j]];
                    b = (uint32_t)(ee >> 32) & (kTileMax - 1u);
                    decode_entry(a.ovf, ee, k, s);
                    rf = (uint32_t)accN[b];
                }
                replay_group(L, pending, b, k, s, rf);
            }
            __builtin_amdgcn_wave_barrier();
            for (uint32_t j = lane; j < nmine; j += 64) accN[(uint32_t)(L.s_rep[wl[j]] >> 32) & (kTileMax - 1u)] = 0;
        } else {
            for (uint32_t g0 = 0; g0 < nlist; g0 += 64) {
                const uint32_t i = g0 + lane;
                bool pending = false;
                uint32_t b = 0, k = 0, s = 0, rf = 0;
                if (i < nlist) {
                    const uint64_t ee = rep_entry(i);
                    b = (uint32_t)(ee >> 32) & (kTileMax - 1u);
                    pending = b % kApWaves == wave;
                    if (pending) {
                        decode_entry(a.ovf, ee, k, s);
                        rf = (uint32_t)accN[b];
                    }
                }
                replay_group(L, pending, b, k, s, rf);
            }
            __builtin_amdgcn_wave_barrier();
            for (uint32_t g0 = 0; g0 < nlist; g0 += 64) {
                const uint32_t i = g0 + lane;
                if (i < nlist) {
                    const uint32_t b = (uint32_t)(rep_entry(i) >> 32) & (kTileMax - 1u);
                    if (b % kApWaves == wave) accN[b] = 0;
                }
            }
        }
    }
    __syncthreads();
    SP_MARK(4);
}

__global__ __launch_bounds__(kApThreads) void k_apply_sparse(ApplyArgs a) {
    __shared__ ApplyLds L;
    __shared__ SparseLds H;
    __shared__ uint32_t s_k;
    const CmGeom &g = a.g;
    const uint32_t tid = threadIdx.x;
    const uint32_t bmask = (1u << g.bin_bits) - 1u;
    for (uint32_t i = tid; i < kTileMax; i += kApThreads) { H.key[i] = 0; L.accN[i] = 0; L.accS[i] = 0; }
    if (tid == 0) { H.used = 0; H.ovf = 0; s_k = atomicAdd(a.work, 1u); }
    __syncthreads();
    uint32_t k = s_k;
    __syncthreads();
    uint32_t st_chunks = 0, st_rep = 0, st_crep = 0;
#ifdef GNS_SP_PROF
    uint64_t sp_pt[7] = {0, 0, 0, 0, 0, 0, 0}, sp_prev = __builtin_amdgcn_s_memtime();
#endif
    while (k < g.nbins) {
        if (tid == 0) s_k = atomicAdd(a.work, 1u);  // the bin after this one
        const ApplyTile cur = apply_bin(a, k);
        const uint64_t cbase = (uint64_t)cur.r * g.w + cur.bbase;
        uint64_t e[kApItems], en[kApItems];
#pragma unroll
        for (int j = 0; j < kApItems; j++) {
            const uint32_t q = cur.beg + j * kApThreads + tid;
            e[j] = q < cur.end ? a.entries[q] : 0ull;
        }
        for (uint32_t cb = cur.beg; cb < cur.end; cb += kApChunk) {
#pragma unroll
            for (int j = 0; j < kApItems; j++) {  // the next chunk loads while this one is applied
                const uint32_t q = cb + kApChunk + j * kApThreads + tid;
                en[j] = q < cur.end ? a.entries[q] : 0ull;
            }
            const uint32_t hic = min(cb + kApChunk, cur.end);
            uint32_t lo = cb, span = kApChunk;
            while (lo < hic) {  // block-uniform
                const uint32_t hi = min(lo + span, hic);
                uint32_t vm = 0;
                bool ok = sp_map(a, L, H, e, vm, cb, lo, hi, cur.end, cbase, cur.bbase, bmask SP_PTA);
                if (!ok) {  // table full: write it back and map the piece into an empty one
                    sp_flush(a, L, H, cbase SP_PTA);
                    ok = sp_map(a, L, H, e, vm, cb, lo, hi, cur.end, cbase, cur.bbase, bmask SP_PTA);
                }
                if (!ok) {  // the piece alone has too many buckets: halve it
                    sp_flush(a, L, H, cbase SP_PTA);
                    span = max(span / 2, 64u);
                    continue;
                }
                sp_chunk(a, L, H, e, vm, cb, bmask, st_chunks, st_rep, st_crep SP_PTA);
                lo = hi;
            }
#pragma unroll
            for (int j = 0; j < kApItems; j++) e[j] = en[j];
        }
        sp_flush(a, L, H, cbase SP_PTA);
        k = s_k;
        __syncthreads();
    }
#ifdef GNS_SP_PROF
    if (tid == 0) for (int i = 0; i < 7; i++) atomicAdd(&a.stats[kStatsProf + i], (unsigned long long)sp_pt[i]);
#endif
    if (tid == 0) {
        atomicAdd(&a.stats[5], (unsigned long long)st_rep);
        atomicAdd(&a.stats[6], (unsigned long long)st_chunks);
        if (st_crep) atomicAdd(&a.stats[7], (unsigned long long)st_crep);
    }
}

constexpr uint32_t kHotSegs = 64;   // segments per hot bin (blocks working on one bucket)
constexpr uint32_t kChkCap = 4096;  // (slot, K1 block) exact size checks per batch

struct HotArgs {
    const uint64_t *entries;
    const uint32_t *offsets;
    uint32_t nblk;
    const uint32_t *total;
    const uint64_t *ovf;
    const uint32_t *hot_ids;
    CmGeom g;
    uint32_t *C, *Fc, *S, *Fs;
    long long *segtot;  // [d*kHot][kHotSegs][2]: count walk, size walk of each segment
    uint32_t *hflag;    // [d*kHot]: bit0/bit1 = count/size half saw an event (needs replay)
    // summary path (k_hot_decide / k_hot_blockcheck / k_hot_commit)
    const HotSum *hsum;     // [d*kHot][nblk]
    uint32_t *hflag2;       // [d*kHot]: bit0/bit1 = count/size half goes to the exact entry path
    uint32_t *hany;         // any hflag2 bit set in this batch
    uint32_t *hres;         // [d*kHot][2]: linear-regime C, S at batch end
    uint4 *chk;             // (slot, K1 block, walk lo, walk hi) blocks needing the exact size check
    uint32_t *nchk;
    uint32_t chk_cap;
    const uint32_t *keyid, *idx, *sizes;
    uint64_t n;
    const uint32_t *hstr, *scnt;  // compact hot streams (CM kernels), or null: per-packet codes in idx
};

__device__ __forceinline__ void hot_bin_range(const HotArgs &a, uint32_t hb, uint32_t &beg, uint32_t &end) {
    const uint32_t bin = a.g.nbins + hb;
    beg = a.offsets[bin];
    end = (bin + 1 < a.g.nbins_all) ? a.offsets[bin + 1] : *a.total;
}

__device__ __forceinline__ void hot_seg_range(uint32_t beg, uint32_t end, uint32_t sidx, uint32_t &sb,
                                              uint32_t &se) {
    const uint32_t len = end - beg;
    const uint32_t per = (((len + kHotSegs - 1) / kHotSegs) + 3u) & ~3u;
    sb = min(end, beg + sidx * per);
    se = min(end, sb + per);
}


// block (256) reduction of two int64
__device__ __forceinline__ void block_sum2(long long &x, long long &y, long long *sh /*8*/) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    x = (long long)wave_sum64((uint64_t)x);
    y = (long long)wave_sum64((uint64_t)y);
    if (lane == 0) { sh[wave] = x; sh[4 + wave] = y; }
    __syncthreads();
    x = sh[0] + sh[1] + sh[2] + sh[3];
    y = sh[4] + sh[5] + sh[6] + sh[7];
    __syncthreads();
}

// H1: walk totals of every segment of every hot bin (owner = batch-entry fingerprint)
__global__ __launch_bounds__(256) void k_hot_sum(HotArgs a) {
    __shared__ long long sh[8];
    if (*a.hany == 0) return;
    // grid-stride over (slot, segment): a small grid exits fast in the common case
    for (uint32_t wi = blockIdx.x; wi < a.g.d * kHot * kHotSegs; wi += gridDim.x) {
    const uint32_t hb = wi / kHotSegs, sidx = wi % kHotSegs;
    if ((a.hflag2[hb] & 3u) == 0) continue;
    const uint32_t id = a.hot_ids[hb];
    if (id == GNS_ID_NONE) continue;
    uint32_t beg, end, sb, se;
    hot_bin_range(a, hb, beg, end);
    hot_seg_range(beg, end, sidx, sb, se);
    const uint64_t cell = (uint64_t)(hb / kHot) * a.g.w + id;
    const uint32_t F_c = a.Fc[cell], F_s = a.Fs[cell];
    long long wc = 0, ws = 0;
    for (uint32_t q = sb + threadIdx.x; q < se; q += 256) {
        uint32_t k, s;
        decode_entry(a.ovf, a.entries[q], k, s);
        wc += (k == F_c) ? 1 : -1;
        ws += (k == F_s) ? (long long)s : -(long long)s;
    }
    block_sum2(wc, ws, sh);
    if (threadIdx.x == 0) {
        a.segtot[((size_t)hb * kHotSegs + sidx) * 2] = wc;
        a.segtot[((size_t)hb * kHotSegs + sidx) * 2 + 1] = ws;
    }
    }
}

// H2: exact check.  With no event the owner never changes and every counter
// follows u32 arithmetic on the running walk (count_min.go:109-113 owner adds
// wrap mod 2^32 exactly like the walk); an event is a foreign update that
// would find C <= 1 (:226-231 take-over) or S == 0 / s > S (:184-200).
__global__ __launch_bounds__(256) void k_hot_verify(HotArgs a) {
    __shared__ long long sh_w[2][4];
    const uint32_t tid = threadIdx.x;
    const uint32_t lane = tid & 63u, wave = tid >> 6;
    if (*a.hany == 0) return;
    for (uint32_t wi = blockIdx.x; wi < a.g.d * kHot * kHotSegs; wi += gridDim.x) {
    const uint32_t hb = wi / kHotSegs, sidx = wi % kHotSegs;
    if ((a.hflag2[hb] & 3u) == 0) continue;
    const uint32_t id = a.hot_ids[hb];
    if (id == GNS_ID_NONE) continue;
    uint32_t beg, end, sb, se;
    hot_bin_range(a, hb, beg, end);
    hot_seg_range(beg, end, sidx, sb, se);
    if (sb >= se) continue;
    const uint64_t cell = (uint64_t)(hb / kHot) * a.g.w + id;
    const uint32_t F_c = a.Fc[cell], F_s = a.Fs[cell];
    long long run_c = a.C[cell], run_s = a.S[cell];
    for (uint32_t j = 0; j < sidx; j++) {
        run_c += a.segtot[((size_t)hb * kHotSegs + j) * 2];
        run_s += a.segtot[((size_t)hb * kHotSegs + j) * 2 + 1];
    }
    uint32_t ev = 0;
    for (uint32_t q0 = sb; q0 < se; q0 += 1024) {  // 4 consecutive entries per thread
        uint32_t k[4], s[4];
        bool v[4];
        long long dc[4], ds[4], tc = 0, ts = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t q = q0 + tid * 4 + i;
            v[i] = q < se;
            k[i] = 0; s[i] = 0;
            if (v[i]) decode_entry(a.ovf, a.entries[q], k[i], s[i]);
            dc[i] = v[i] ? ((k[i] == F_c) ? 1 : -1) : 0;
            ds[i] = v[i] ? ((k[i] == F_s) ? (long long)s[i] : -(long long)s[i]) : 0;
            tc += dc[i]; ts += ds[i];
        }
        const long long ic = wave_incl_scan64(tc), is = wave_incl_scan64(ts);
        if (lane == 63) { sh_w[0][wave] = ic; sh_w[1][wave] = is; }
        __syncthreads();
        long long bc = 0, bs = 0, allc = 0, alls = 0;
#pragma unroll
        for (uint32_t w = 0; w < 4; w++) {
            if (w < wave) { bc += sh_w[0][w]; bs += sh_w[1][w]; }
            allc += sh_w[0][w]; alls += sh_w[1][w];
        }
        __syncthreads();
        long long pc = run_c + bc + ic - tc, ps = run_s + bs + is - ts;  // before my first entry
#pragma unroll
        for (int i = 0; i < 4; i++) {
            if (v[i]) {
                const uint32_t Cb = (uint32_t)pc, Sb = (uint32_t)ps;
                if (k[i] != F_c && Cb <= 1u) ev |= 1u;
                if (k[i] != F_s && (Sb == 0u || s[i] > Sb)) ev |= 2u;
            }
            pc += dc[i]; ps += ds[i];
        }
        run_c += allc; run_s += alls;
    }
    const uint32_t any = (uint32_t)(__ballot(ev & 1u) != 0) | ((uint32_t)(__ballot(ev & 2u) != 0) << 1);
    if (lane == 0 && any) atomicOr(&a.hflag[hb], any);
    }
}

// H3: apply the verified halves; flagged halves keep the batch-entry state
// for the in-order fallback.
__global__ __launch_bounds__(512) void k_hot_apply(HotArgs a) {
    const uint32_t hb = blockIdx.x * 512 + threadIdx.x;
    if (hb >= a.g.d * kHot) return;
    if (*a.hany == 0) return;
    const uint32_t f2 = a.hflag2[hb] & 3u;
    if (!f2) return;
    const uint32_t id = a.hot_ids[hb];
    if (id == GNS_ID_NONE) return;
    uint32_t beg, end;
    hot_bin_range(a, hb, beg, end);
    if (beg >= end) return;
    long long tc = 0, ts = 0;
    for (uint32_t j = 0; j < kHotSegs; j++) {
        tc += a.segtot[((size_t)hb * kHotSegs + j) * 2];
        ts += a.segtot[((size_t)hb * kHotSegs + j) * 2 + 1];
    }
    const uint64_t cell = (uint64_t)(hb / kHot) * a.g.w + id;
    const uint32_t f = a.hflag[hb];
    if ((f2 & 1u) && !(f & 1u)) a.C[cell] = (uint32_t)((long long)a.C[cell] + tc);
    if ((f2 & 2u) && !(f & 2u)) a.S[cell] = (uint32_t)((long long)a.S[cell] + ts);
}

// Exact in-order replay of one hot bin (cold start / ownership change).
__global__ __launch_bounds__(64) void k_hot_fallback(HotArgs a) {
    const uint32_t i = blockIdx.x, lane = threadIdx.x;
    if (*a.hany == 0) return;
    const uint32_t rep = a.hflag[i] & a.hflag2[i] & 3u;
    if (!rep) return;
    const uint32_t id = a.hot_ids[i];
    const uint64_t cell = (uint64_t)(i / kHot) * a.g.w + id;
    uint32_t beg, end;
    hot_bin_range(a, i, beg, end);
    uint32_t Fc = a.Fc[cell], C = a.C[cell], Fs = a.Fs[cell], S = a.S[cell];
    for (uint32_t cb = beg; cb < end; cb += 64) {
        const uint32_t q = cb + lane;
        const bool v = q < end;
        uint32_t k = 0, s = 0;
        if (v) decode_entry(a.ovf, a.entries[q], k, s);
        if (rep & 1u) count_seq64(v, k, Fc, C);
        if (rep & 2u) size_seq64(v, k, s, Fs, S);
    }
    if (lane == 0) {
        if (rep & 1u) { a.C[cell] = C; a.Fc[cell] = Fc; }
        if (rep & 2u) { a.S[cell] = S; a.Fs[cell] = Fs; }
    }
}

// ---------------------------------------------------------------------------
// Summary path for designated buckets.  K1 left one HotSum per (slot, K1
// block).  The count half is linear (owner fixed, C' = C + n_own - n_foreign)
// when C > n_foreign over the batch: every foreign update then finds C >= 2
// (count_min.go:145-150 never reaches 0) -- and no u32 wrap.  The size half
// is linear when every foreign update finds S >= max(s, 1) (:184-200 never
// replace), where S is the running walk W = S0 + sum(own) - sum(foreign) taken
// mod 2^32 (owner adds wrap exactly like the walk, :190-193).  Per K1 block j
// the walk stays in [W_j - fs_j, W_j + os_j]; if that interval lies inside one
// 2^32 period with low part >= max(smax_j, 1) the block is safe; otherwise
// k_hot_blockcheck replays the block's walk exactly.  Anything that fails goes
// to the exact entry path (K3 hot mode + k_hot_sum/verify/apply/fallback).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_hot_decide(HotArgs a) {
    __shared__ long long sh_w[4];
    __shared__ unsigned long long sh_r[3][4];
    __shared__ uint32_t s_fail;
    const uint32_t slot = blockIdx.x, tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t id = a.hot_ids[slot];
    if (id == GNS_ID_NONE) return;
    if (tid == 0) s_fail = 0;
    const uint64_t cell = (uint64_t)(slot / kHot) * a.g.w + id;
    const uint32_t C0 = a.C[cell], S0 = a.S[cell];
    const HotSum *hs = a.hsum + (uint64_t)slot * a.nblk;
    long long run = S0;
    unsigned long long N = 0, NFC = 0, NFS = 0;
    __syncthreads();
    for (uint32_t j0 = 0; j0 < a.nblk; j0 += 256) {
        const uint32_t j = j0 + tid;
        HotSum h{};
        if (j < a.nblk) h = hs[j];
        const long long dlt = (long long)h.os - (long long)h.fs;
        const long long inc = wave_incl_scan64(dlt);
        if (lane == 63) sh_w[wave] = inc;
        __syncthreads();
        long long base = 0, tot = 0;
#pragma unroll
        for (uint32_t w = 0; w < 4; w++) {
            if (w < wave) base += sh_w[w];
            tot += sh_w[w];
        }
        __syncthreads();
        const long long W = run + base + inc - dlt;  // walk before block j
        if (h.nfs) {
            const long long L = W - (long long)h.fs, U = W + (long long)h.os;
            const uint32_t m = h.smax > 1u ? h.smax : 1u;
            const bool safe = L >= 0 && (L >> 32) == (U >> 32) && (uint32_t)L >= m;
            if (!safe) {
                const uint32_t q = atomicAdd(a.nchk, 1u);
                if (q < a.chk_cap) a.chk[q] = make_uint4(slot, j, (uint32_t)W, (uint32_t)((unsigned long long)W >> 32));
                else s_fail = 1;
            }
        }
        run += tot;
        N += h.n; NFC += h.nfc; NFS += h.nfs;
    }
    N = wave_sum64(N); NFC = wave_sum64(NFC); NFS = wave_sum64(NFS);
    if (lane == 0) { sh_r[0][wave] = N; sh_r[1][wave] = NFC; sh_r[2][wave] = NFS; }
    __syncthreads();
    if (tid == 0) {
        N = sh_r[0][0] + sh_r[0][1] + sh_r[0][2] + sh_r[0][3];
        NFC = sh_r[1][0] + sh_r[1][1] + sh_r[1][2] + sh_r[1][3];
        NFS = sh_r[2][0] + sh_r[2][1] + sh_r[2][2] + sh_r[2][3];
        uint32_t f = 0;
        // count half
        if ((unsigned long long)C0 > NFC && (unsigned long long)C0 + (N - NFC) < (1ull << 32))
            a.hres[slot * 2] = (uint32_t)((unsigned long long)C0 + N - 2 * NFC);
        else
            f |= 1u;
        // size half: all-own is plain u32 addition; otherwise per-block checks
        if (NFS && (S0 == 0 || s_fail)) f |= 2u;
        a.hres[slot * 2 + 1] = (uint32_t)(unsigned long long)run;
        if (f) { atomicOr(&a.hflag2[slot], f); atomicOr(a.hany, 1u); }
    }
}

// Exact walk of one K1 block's updates to one designated bucket (size half).
__global__ __launch_bounds__(256) void k_hot_blockcheck(HotArgs a) {
    __shared__ long long sh_w[4];
    const uint32_t q = blockIdx.x, tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    if (q >= min(*a.nchk, a.chk_cap)) return;
    const uint4 c = a.chk[q];
    const uint32_t slot = c.x, blk = c.y;
    const uint32_t r = slot / kHot, code = 0x80000000u | (slot % kHot);
    const uint32_t Fs0 = a.Fs[(uint64_t)r * a.g.w + a.hot_ids[slot]];
    long long run = (long long)((unsigned long long)c.z | (unsigned long long)c.w << 32);
    const uint64_t beg = (uint64_t)blk * kChunk, end = min(a.n, beg + kChunk);
    const uint32_t *idxr = a.idx + (uint64_t)r * a.n;
    // compact streams: walk the block's row-r hot stream (its K1 waves in order = packet
    // order) instead of every packet's code
    uint32_t spre[kCsWaves + 1] = {0, 0, 0, 0, 0};
    if (a.hstr) {
        for (uint32_t w = 0; w < kCsWaves; w++)
            spre[w + 1] = spre[w] + a.scnt[(((uint64_t)blk * kCsWaves + w) * a.g.d + r) * 2 + 1];
    }
    const uint64_t lim = a.hstr ? (uint64_t)spre[kCsWaves] : end - beg;
    bool ev = false;
    for (uint64_t q0 = 0; q0 < lim; q0 += 1024) {  // 4 consecutive packets (stream entries) per thread
        long long dl[4], tl = 0;
        bool fo[4];
        uint32_t sv[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint64_t x = q0 + tid * 4 + i;
            uint64_t p = beg + x;
            bool hit = false;
            if (x < lim) {
                if (a.hstr) {
                    const uint32_t w = (x >= spre[1] ? 1u : 0u) + (x >= spre[2] ? 1u : 0u) + (x >= spre[3] ? 1u : 0u);
                    const uint32_t cc = a.hstr[(((uint64_t)blk * kCsWaves + w) * a.g.d + r) * kCsWave + (x - spre[w])];
                    p = beg + w * kCsWave + (cc & (kCsWave - 1u));
                    hit = (cc >> kCsBits) == slot % kHot;
                } else {
                    hit = idxr[p] == code;
                }
            }
            dl[i] = 0; fo[i] = false; sv[i] = 0;
            if (hit && a.keyid[p] != GNS_ID_NONE) {
                const uint32_t s = a.sizes[p];
                const bool own = a.keyid[p] == Fs0;
                dl[i] = own ? (long long)s : -(long long)s;
                fo[i] = !own;
                sv[i] = s;
            }
            tl += dl[i];
        }
        const long long inc = wave_incl_scan64(tl);
        if (lane == 63) sh_w[wave] = inc;
        __syncthreads();
        long long base = 0, tot = 0;
#pragma unroll
        for (uint32_t w = 0; w < 4; w++) {
            if (w < wave) base += sh_w[w];
            tot += sh_w[w];
        }
        __syncthreads();
        long long wb = run + base + inc - tl;
#pragma unroll
        for (int i = 0; i < 4; i++) {
            if (fo[i]) {
                const uint32_t Sb = (uint32_t)(unsigned long long)wb;
                if (wb < 0 || Sb == 0u || sv[i] > Sb) ev = true;
            }
            wb += dl[i];
        }
        run += tot;
    }
    if (__ballot(ev) && lane == 0) { atomicOr(&a.hflag2[slot], 2u); atomicOr(a.hany, 1u); }
}

// Commit the linear results of the halves that stay on the summary path.
__global__ __launch_bounds__(512) void k_hot_commit(HotArgs a) {
    const uint32_t slot = blockIdx.x * 512 + threadIdx.x;
    if (slot >= a.g.d * kHot) return;
    const uint32_t id = a.hot_ids[slot];
    if (id == GNS_ID_NONE) return;
    const uint64_t cell = (uint64_t)(slot / kHot) * a.g.w + id;
    const uint32_t f = a.hflag2[slot];
    if (!(f & 1u)) a.C[cell] = a.hres[slot * 2];
    if (!(f & 2u)) a.S[cell] = a.hres[slot * 2 + 1];
}

// Designation for the next batch: per row, the buckets whose counter bit
// length is in the top band holding at most kHot buckets (and >= 2^(kHotMinBits-1)).
// Designation key: bit length and the 3 bits below the leading one (a
// monotone 1/8-octave log scale), so the band picked by k_hot_pick holds
// close to kHot buckets.
constexpr uint32_t kHotKeys = 33 * 8;
__device__ __forceinline__ uint32_t hot_key(uint32_t v) {
    const uint32_t bits = v ? 32u - __clz(v) : 0u;
    return bits >= 4 ? bits * 8u + ((v >> (bits - 4u)) & 7u) : bits * 8u;
}

// Candidates of the next designation, collected by the histogram pass (round 6): every
// bucket whose key is within one octave below the previous batch's threshold.  When the
// new threshold is no more than an octave below the old one and the list did not
// overflow, the buckets k_hot_collect takes are all in the list, so it scans the list
// instead of the whole counter array (one pass over C per batch instead of two: 512 MB
// at configs[4]'s geometry).  Any designation is exact (the summary path proves each
// batch or falls back), so the choice only moves work.
constexpr uint32_t kHotCand = 4096;  // candidates kept per row

__global__ __launch_bounds__(256) void k_hot_hist(const uint32_t *C, CmGeom g, uint32_t *hh /*[d][kHotKeys]*/,
                                                  const uint32_t *thr_prev, uint32_t *hcand, uint32_t *hcn) {
    __shared__ uint32_t s[8 * kHotKeys];
    for (uint32_t i = threadIdx.x; i < g.d * kHotKeys; i += 256) s[i] = 0;
    __syncthreads();
    // row by row (no per-cell division), 16-byte loads when the row is whole words of 4
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint32_t r = 0; r < g.d; r++) {
        const uint32_t *Cr = C + (uint64_t)r * g.w;
        uint32_t *sr = s + r * kHotKeys;
        const uint32_t tp = thr_prev[r];  // 0xFFFFFFFF: no previous threshold (no candidates)
        const uint32_t ck = tp <= kHotKeys ? (tp >= 8u ? tp - 8u : 0u) : 0xFFFFFFFFu;
        uint32_t *cr = hcand + (uint64_t)r * kHotCand;
        auto cand = [&](uint32_t v, uint64_t c) {
            if (v >= (1u << (kHotMinBits - 1)) && hot_key(v) >= ck) {
                const uint32_t q = atomicAdd(&hcn[r], 1u);
                if (q < kHotCand) cr[q] = (uint32_t)c;
            }
        };
        if ((g.w & 3u) == 0) {
            // four 16-byte loads in flight per thread before their counts (the class adds
            // between single loads left the pass latency-bound with few blocks)
            const uint4 *C4 = reinterpret_cast<const uint4 *>(Cr);
            const uint64_t n4 = g.w / 4;
            for (uint64_t c0 = (uint64_t)blockIdx.x * 256 + threadIdx.x; c0 < n4; c0 += 4 * stride) {
                uint4 v[4];
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const uint64_t c = c0 + (uint64_t)u * stride;
                    v[u] = c < n4 ? C4[c] : make_uint4(0, 0, 0, 0);
                }
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    if (v[u].x >= (1u << (kHotMinBits - 1))) atomicAdd(&sr[hot_key(v[u].x)], 1u);
                    if (v[u].y >= (1u << (kHotMinBits - 1))) atomicAdd(&sr[hot_key(v[u].y)], 1u);
                    if (v[u].z >= (1u << (kHotMinBits - 1))) atomicAdd(&sr[hot_key(v[u].z)], 1u);
                    if (v[u].w >= (1u << (kHotMinBits - 1))) atomicAdd(&sr[hot_key(v[u].w)], 1u);
                    const uint64_t c = c0 + (uint64_t)u * stride;
                    if (c < n4) {
                        cand(v[u].x, 4 * c); cand(v[u].y, 4 * c + 1); cand(v[u].z, 4 * c + 2); cand(v[u].w, 4 * c + 3);
                    }
                }
            }
        } else {
            for (uint64_t c = (uint64_t)blockIdx.x * 256 + threadIdx.x; c < g.w; c += stride) {
                const uint32_t v = Cr[c];
                if (v >= (1u << (kHotMinBits - 1))) atomicAdd(&sr[hot_key(v)], 1u);
                cand(v, c);
            }
        }
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < g.d * kHotKeys; i += 256) if (s[i]) atomicAdd(&hh[i], s[i]);
}

__global__ void k_hot_pick(uint32_t *hh, CmGeom g, uint32_t *thr, uint32_t *hcnt, uint32_t *hot_ids,
                           const uint32_t *hcn, uint32_t *hfull) {
    __shared__ uint32_t s_hh[8 * kHotKeys];
    for (uint32_t i = threadIdx.x; i < g.d * kHot; i += blockDim.x) hot_ids[i] = GNS_ID_NONE;
    for (uint32_t i = threadIdx.x; i < g.d * kHotKeys; i += blockDim.x) { s_hh[i] = hh[i]; hh[i] = 0; }
    __syncthreads();
    const uint32_t r = threadIdx.x;
    if (r < g.d) {
        uint32_t cum = 0, t = kHotKeys;
        for (int k = (int)kHotKeys - 1; k >= (int)(kHotMinBits * 8); k--) {
            cum += s_hh[r * kHotKeys + k];
            if (cum > kHot) break;
            t = (uint32_t)k;
        }
        // the candidate list holds every bucket the collect takes iff it did not overflow and
        // the new threshold is at most one octave below the one the list was collected for
        const uint32_t tp = thr[r];
        hfull[r] = !(tp <= kHotKeys && t + 8u >= tp && hcn[r] <= kHotCand);
        thr[r] = t;
        hcnt[r] = 0;
    }
}

__global__ __launch_bounds__(256) void k_hot_collect(const uint32_t *C, CmGeom g, const uint32_t *thr,
                                                      uint32_t *hcnt, uint32_t *hot_ids, const uint32_t *hcand,
                                                      const uint32_t *hcn, const uint32_t *hfull) {
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint32_t r = 0; r < g.d; r++) {
        const uint32_t *Cr = C + (uint64_t)r * g.w;
        const uint32_t t = thr[r];
        auto take = [&](uint32_t v, uint64_t c) {
            if (v >= (1u << (kHotMinBits - 1)) && hot_key(v) >= t) {
                const uint32_t q = atomicAdd(&hcnt[r], 1u);
                if (q < kHot) hot_ids[r * kHot + q] = (uint32_t)c;
            }
        };
        if (!hfull[r]) {  // the histogram pass's candidate list holds them all (block-uniform)
            const uint32_t nc = hcn[r];
            for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < nc; i += (uint32_t)stride) {
                const uint32_t c = hcand[(uint64_t)r * kHotCand + i];
                take(Cr[c], c);
            }
            continue;
        }
        if ((g.w & 3u) == 0) {
            const uint4 *C4 = reinterpret_cast<const uint4 *>(Cr);
            for (uint64_t c = (uint64_t)blockIdx.x * 256 + threadIdx.x; c < g.w / 4; c += stride) {
                const uint4 v = C4[c];
                take(v.x, 4 * c); take(v.y, 4 * c + 1); take(v.z, 4 * c + 2); take(v.w, 4 * c + 3);
            }
        } else {
            for (uint64_t c = (uint64_t)blockIdx.x * 256 + threadIdx.x; c < g.w; c += stride) take(Cr[c], c);
        }
    }
}

// Lookup groups of the designated buckets (one thread per row, deterministic);
// a bucket whose group is full is dropped from the designation.
__global__ __launch_bounds__(1024) void k_hot_table(CmGeom g, uint32_t *hot_ids, uint32_t *hot_tab, uint32_t *hcn) {
    // entry h of a row takes slot j of its group, j = number of earlier valid
    // entries of the row in the same group (what inserting in h order gives);
    // j >= 4: the group is full and the bucket is not designated
    __shared__ uint32_t s_ids[8 * kHot];
    const uint32_t NS = g.d * kHot;
    for (uint32_t i = threadIdx.x; i < g.d * kHotTab; i += blockDim.x) hot_tab[i] = 0xFFFFFFFFu;
    if (threadIdx.x < g.d) hcn[threadIdx.x] = 0;  // the next histogram pass's candidate counts
    for (uint32_t i = threadIdx.x; i < NS; i += blockDim.x) s_ids[i] = hot_ids[i];
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < NS; i += blockDim.x) {
        const uint32_t r = i / kHot, h = i % kHot, b = s_ids[i];
        if (b == GNS_ID_NONE) continue;
        const uint32_t grp = hot_group(b);
        uint32_t j = 0;
        for (uint32_t h2 = 0; h2 < h; h2++) {
            const uint32_t b2 = s_ids[r * kHot + h2];
            j += (b2 != GNS_ID_NONE && hot_group(b2) == grp) ? 1u : 0u;
        }
        if (j < 4) hot_tab[r * kHotTab + grp * 4 + j] = b << kHotBits | h;
        else hot_ids[i] = GNS_ID_NONE;
    }
}

// ---------------------------------------------------------------------------
// Query (count_min.go:160-174), export, heavy-hitter candidates
// ---------------------------------------------------------------------------
struct QueryArgs {
    const uint8_t *keys;
    uint32_t stride, aligned;
    uint64_t n;
    uint32_t K;
    CmGeom g;
    DictDev D;
    const uint32_t *C, *Fc, *S, *Fs;
    uint64_t *out;
};

__global__ __launch_bounds__(256) void k_query(QueryArgs a) {
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= a.n) return;
    uint32_t kw[GNS_KWMAX];
    load_key_bytes<GNS_KWMAX>(a.keys + p * a.stride, a.K, a.aligned != 0, kw);
    const uint32_t id = dict_lookup(a.D, kw);
    uint32_t sz = 0, ct = 0;
    if (id != GNS_ID_NONE) {
        for (uint32_t rr = 0; rr < a.g.d; rr++) {
            const uint64_t c = (uint64_t)rr * a.g.w + row_index(a.g, mm3_n<GNS_KWMAX>(kw, a.K, a.g.seeds[rr]));
            if (a.Fs[c] == id) sz = max(sz, a.S[c]);
            if (a.Fc[c] == id) ct = max(ct, a.C[c]);
        }
    }
    a.out[p] = (uint64_t)ct << 32 | sz;
}

// flow ids -> key bytes (GNS_ID_NONE -> zero bytes, the reference's reset FP)
__global__ __launch_bounds__(256) void k_ids_to_bytes(const uint32_t *ids, uint64_t n, DictDev D,
                                                      uint8_t *out) {
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= n) return;
    const uint32_t id = ids[p];
    uint32_t r[12];
    if (id != GNS_ID_NONE) load_record(D, id, r);
    for (uint32_t j = 0; j < D.K; j++) {
        const uint32_t w = id != GNS_ID_NONE ? r[1 + (j >> 2)] : 0u;
        out[p * D.K + j] = (uint8_t)(w >> (8 * (j & 3)));
    }
}

// cells whose counter >= thr -> (value<<32 | id) candidate list
// kHhItems cells per lane; one global atomic per workgroup reserves the
// candidates' slots (a per-lane atomic on the one counter serialized every
// candidate: 0.59 ms per call at the bench geometry).  Order is irrelevant:
// the host dedupes and sorts.
constexpr uint32_t kHhItems = 8;
// Device-side heavy-hitter list (count_min.go:178-247 HeavyHitters), all
// hand-written (no library sort):
//   candidates   cells with value >= threshold (one global atomic per workgroup);
//   per-flow max every candidate atomicMax'es (epoch << 32 | value) into a dense
//                per-flow-id word, then the one candidate per flow that carries the
//                max and wins the flow's mark emits (id, max) -- the dedupe of
//                count_min.go:214-228's map, order-free, O(candidates);
//   order        a stable LSD radix sort of the unique entries (8-bit digits,
//                device-wide passes: block histograms, the K2 scan, stable
//                ballot-multisplit scatter) by the primary key (value desc, key
//                bytes 0..3); only when two entries tie on it (the same value and
//                the same first four key bytes) is the list re-sorted by the whole
//                key (bytes K-1..4 first, then the primary key).  A pass whose
//                digit is the same for every entry (IPv4 slots' zero padding) only
//                copies.  Canonical order: value desc, flow bytes asc.
// A candidate whose id is not a dictionary slot (a corrupt fingerprint word) is
// skipped and raises *bad: the host then fails the call with GNS_E_HIP instead of
// letting the per-flow words be indexed out of bounds.
__global__ __launch_bounds__(256) void k_hh_best(const uint64_t *cand, uint32_t n, unsigned long long *best,
                                                 uint32_t epoch, uint64_t slots, uint32_t *bad) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t c = cand[i];  // value << 32 | id
    if ((uint32_t)c >= slots) { atomicOr(bad, 1u); return; }
    atomicMax(&best[(uint32_t)c], (unsigned long long)epoch << 32 | (c >> 32));
}

__global__ __launch_bounds__(256) void k_hh_emit(const uint64_t *cand, uint32_t n, const unsigned long long *best,
                                                 uint32_t *mark, uint32_t epoch, uint64_t slots, uint32_t *uid,
                                                 uint32_t *uval, uint32_t *nu) {
    __shared__ uint32_t s_n, s_base;
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    bool out = false;
    uint32_t id = 0, v = 0;
    if (i < n) {
        const uint64_t c = cand[i];
        id = (uint32_t)c;
        v = (uint32_t)(c >> 32);
        out = id < slots && (uint32_t)best[id] == v && atomicExch(&mark[id], epoch) != epoch;  // one per flow
    }
    const uint32_t off = out ? atomicAdd(&s_n, 1u) : 0u;
    __syncthreads();
    if (threadIdx.x == 0) s_base = s_n ? atomicAdd(nu, s_n) : 0u;
    __syncthreads();
    if (out) {
        uid[s_base + off] = id;
        uval[s_base + off] = v;
    }
}

// A heavy-hitter list on the device: entry e has flow bytes ub[e*stride .. +K) and
// a value, uval[e] -- or, for packed rows [flow | u32 value] (uval null), the
// little-endian word at ub[e*stride + K].
struct HhSrc {
    const uint32_t *uval;
    const uint8_t *ub;
    uint32_t K, stride;
};
__device__ __forceinline__ uint32_t hh_val(const HhSrc &h, uint32_t e) {
    if (h.uval) return h.uval[e];
    const uint8_t *q = h.ub + (uint64_t)e * h.stride + h.K;
    return (uint32_t)q[0] | (uint32_t)q[1] << 8 | (uint32_t)q[2] << 16 | (uint32_t)q[3] << 24;
}
__device__ __forceinline__ uint32_t hh_byte(const HhSrc &h, uint32_t e, uint32_t b) {
    return b < h.K ? (uint32_t)h.ub[(uint64_t)e * h.stride + b] : 0u;
}

// One radix pass's digit of entry e: mode 0 = byte `b` of the value, inverted
// (descending); mode 1 = key byte b (0 beyond K).
struct RsDigit {
    uint32_t mode, b;
    HhSrc src;
};
__device__ __forceinline__ uint32_t rs_digit(const RsDigit &r, uint32_t e) {
    if (r.mode == 0) return 255u - ((hh_val(r.src, e) >> (8u * r.b)) & 255u);
    return hh_byte(r.src, e, r.b);
}

constexpr uint32_t kRsPer = 16;                 // entries per thread
constexpr uint32_t kRsBlock = 256 * kRsPer;     // entries per block of a pass

__global__ __launch_bounds__(256) void k_rs_hist(const uint32_t *perm, uint32_t n, RsDigit r, uint32_t *hist) {
    __shared__ uint32_t s_h[256];
    const uint32_t tid = threadIdx.x;
    s_h[tid] = 0;
    __syncthreads();
    const uint32_t beg = blockIdx.x * kRsBlock;
#pragma unroll 4
    for (uint32_t k = 0; k < kRsPer; k++) {
        const uint32_t j = beg + k * 256 + tid;
        if (j < n) atomicAdd(&s_h[rs_digit(r, perm[j])], 1u);
    }
    __syncthreads();
    hist[(uint64_t)blockIdx.x * 256 + tid] = s_h[tid];
}

// Stable scatter of one pass: entries of a block in (round, wave, lane) order =
// position order; per wave-instruction the lanes of one digit are found by
// eight ballots (no reliance on LDS-atomic lane order).  offs = the scanned
// block-major histogram (global start of every (block, digit) run); tot / total
// = the digit totals' exclusive scan: a digit holding every entry makes the pass
// a copy (the order cannot change).
__global__ __launch_bounds__(256) void k_rs_scatter(const uint32_t *perm, uint32_t n, RsDigit r, const uint32_t *offs,
                                                    const uint32_t *tot, const uint32_t *total, uint32_t *out) {
    __shared__ uint32_t s_base[256];
    __shared__ uint32_t s_wave[4][256];
    __shared__ uint32_t s_copy;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t beg = blockIdx.x * kRsBlock;
    if (tid == 0) {
        const uint32_t d0 = rs_digit(r, perm[0]);
        const uint32_t hi = d0 < 255u ? tot[d0 + 1] : *total;
        s_copy = hi - tot[d0] == n;
    }
    s_base[tid] = offs[(uint64_t)blockIdx.x * 256 + tid];
    __syncthreads();
    if (s_copy) {  // block-uniform
        for (uint32_t k = 0; k < kRsPer; k++) {
            const uint32_t j = beg + k * 256 + tid;
            if (j < n) out[j] = perm[j];
        }
        return;
    }
    const uint64_t lt = lane ? (~0ull >> (64u - lane)) : 0ull;
    for (uint32_t k = 0; k < kRsPer; k++) {
        if (beg + k * 256 >= n) break;  // block-uniform
        const uint32_t j = beg + k * 256 + tid;
        const bool valid = j < n;
        const uint32_t e = valid ? perm[j] : 0u;
        const uint32_t dg = valid ? rs_digit(r, e) : 0u;
        uint64_t peers = __ballot(valid);
#pragma unroll
        for (uint32_t bit = 0; bit < 8; bit++) {
            const uint64_t m = __ballot(valid && ((dg >> bit) & 1u));
            peers &= ((dg >> bit) & 1u) ? m : ~m;
        }
        s_wave[0][tid] = 0; s_wave[1][tid] = 0; s_wave[2][tid] = 0; s_wave[3][tid] = 0;
        __syncthreads();
        const uint32_t rank = (uint32_t)__popcll(peers & lt);
        if (valid && rank == 0) s_wave[wave][dg] = (uint32_t)__popcll(peers);
        __syncthreads();
        if (valid) {
            uint32_t pos = s_base[dg] + rank;
            for (uint32_t w = 0; w < wave; w++) pos += s_wave[w][dg];
            out[pos] = e;
        }
        __syncthreads();
        s_base[tid] += s_wave[0][tid] + s_wave[1][tid] + s_wave[2][tid] + s_wave[3][tid];
        __syncthreads();
    }
}

// Whether two neighbours of the primary order tie on (value, key bytes 0..3):
// only then does the list need the whole-key order.
__global__ __launch_bounds__(256) void k_hh_ties(const uint32_t *perm, uint32_t n, HhSrc h, uint32_t *flag) {
    const uint32_t j = blockIdx.x * 256 + threadIdx.x + 1;
    if (j >= n) return;
    const uint32_t a = perm[j - 1], b = perm[j];
    if (hh_val(h, a) != hh_val(h, b)) return;
    bool eq = true;
    for (uint32_t t = 0; t < 4 && t < h.K; t++) eq = eq && hh_byte(h, a, t) == hh_byte(h, b, t);
    if (eq) atomicOr(flag, 1u);
}

__global__ __launch_bounds__(256) void k_hh_iota(uint32_t *perm, uint32_t n) {
    const uint32_t j = blockIdx.x * 256 + threadIdx.x;
    if (j < n) perm[j] = j;
}

// ordered output: flow bytes and values in list order (one D2H each), or packed
// rows [flow | u32 value] (rows non-null: the multi-GPU exchange keeps them on the device)
__global__ __launch_bounds__(256) void k_hh_gather(const uint32_t *perm, HhSrc h, uint32_t n, uint8_t *ob,
                                                   uint32_t *ov, uint8_t *rows) {
    const uint32_t j = blockIdx.x * 256 + threadIdx.x;
    if (j >= n) return;
    const uint32_t u = perm[j], K = h.K;
    const uint32_t v = hh_val(h, u);
    if (rows) {
        uint8_t *o = rows + (uint64_t)j * (K + 4);
        for (uint32_t t = 0; t < K; t++) o[t] = hh_byte(h, u, t);
        o[K] = (uint8_t)v; o[K + 1] = (uint8_t)(v >> 8); o[K + 2] = (uint8_t)(v >> 16); o[K + 3] = (uint8_t)(v >> 24);
        return;
    }
    for (uint32_t t = 0; t < K; t++) ob[(uint64_t)j * K + t] = hh_byte(h, u, t);
    ov[j] = v;
}

__global__ __launch_bounds__(256) void k_hh_candidates(const uint32_t *val, const uint32_t *fp,
                                                       uint64_t cells, uint32_t thr,
                                                       uint64_t *cand, uint32_t *ncand, uint32_t cap) {
    __shared__ uint32_t s_n, s_base;
    if (threadIdx.x == 0) s_n = 0;
    __syncthreads();
    const uint64_t c0 = (uint64_t)blockIdx.x * 256 * kHhItems + threadIdx.x;
    uint64_t cv[kHhItems];
    uint32_t cnt = 0;
#pragma unroll
    for (uint32_t i = 0; i < kHhItems; i++) {
        const uint64_t c = c0 + (uint64_t)i * 256;
        cv[i] = 0;
        if (c < cells) {
            const uint32_t v = val[c];
            if (v > 0 && v >= thr) { cv[i] = (uint64_t)v << 32 | fp[c]; cnt++; }
        }
    }
    const uint32_t off = cnt ? atomicAdd(&s_n, cnt) : 0u;
    __syncthreads();
    if (threadIdx.x == 0) s_base = s_n ? atomicAdd(ncand, s_n) : 0u;
    __syncthreads();
    uint32_t q = s_base + off;
#pragma unroll
    for (uint32_t i = 0; i < kHhItems; i++)
        if (cv[i]) { if (q < cap) cand[q] = cv[i]; q++; }
}

__global__ void k_fill_u32(uint32_t *p, uint64_t n, uint32_t v) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
        p[i] = v;
}

}  // namespace gns

// ===========================================================================
// Host side
// ===========================================================================
using namespace gns;

// Grow-only device buffers of the read side (heavy hitters, queries, id -> key
// bytes): no allocation or free -- hipFree synchronizes the device -- once
// warm, so a snapshot view can query while the handle ingests.
struct CmScratch {
    uint64_t *cand = nullptr;
    uint32_t *ncand = nullptr;
    uint64_t cap = 0;               // candidates sc.cand holds
    uint32_t *ids = nullptr;
    uint64_t ids_n = 0;
    uint8_t *bytes = nullptr;
    uint64_t bytes_n = 0;
    uint8_t *qkeys = nullptr;
    uint64_t qkeys_n = 0;
    uint64_t *qout = nullptr;
    uint64_t qout_n = 0;
    // device heavy-hitter list: per-flow-id max / mark words (dense over the dictionary's
    // slots, epoch-tagged so they are never cleared), unique (id, value), order indices,
    // radix-pass histograms (block-major) and their scan
    unsigned long long *best = nullptr;
    uint32_t *mark = nullptr;
    uint64_t best_n = 0, mark_n = 0;
    uint32_t hh_epoch = 0;
    uint32_t *u32a = nullptr, *u32b = nullptr, *u32c = nullptr, *u32d = nullptr;
    uint64_t u32a_n = 0, u32b_n = 0, u32c_n = 0, u32d_n = 0;
    uint32_t *rsh = nullptr;    // [blocks][256] histograms, then [ngrp][256] group sums, [256] totals, total, tie flag
    uint64_t rsh_n = 0;
    uint8_t *obytes = nullptr;  // heavy hitters: ordered flow bytes
    uint64_t obytes_n = 0;
    uint8_t *hpin = nullptr;    // pinned host staging of the heavy-hitter rows (D2H into pageable
    uint64_t hpin_n = 0;        // caller memory went through the runtime's slow path)
    uint32_t *hsm = nullptr;    // pinned host words for the list's small read-backs (lengths, flags):
                                // a 4-byte D2H into a pageable stack word took 28-35 ms now and then
    void free_all() {
        dfree(obytes); obytes = nullptr; obytes_n = 0;
        if (hpin) (void)hipHostFree(hpin);
        hpin = nullptr; hpin_n = 0;
        if (hsm) (void)hipHostFree(hsm);
        hsm = nullptr;
        dfree(cand); dfree(ncand); dfree(ids); dfree(bytes); dfree(qkeys); dfree(qout);
        dfree(best); dfree(mark); dfree(u32a); dfree(u32b); dfree(u32c); dfree(u32d); dfree(rsh);
        cand = nullptr; ncand = nullptr; ids = nullptr; bytes = nullptr; qkeys = nullptr; qout = nullptr;
        best = nullptr; mark = nullptr; u32a = u32b = u32c = u32d = nullptr; rsh = nullptr;
        cap = 0; ids_n = bytes_n = qkeys_n = qout_n = 0;
        best_n = mark_n = u32a_n = u32b_n = u32c_n = u32d_n = rsh_n = 0; hh_epoch = 0;
    }
};

// Grows to twice the request: heavy-hitter lists grow window by window over a
// period, and every reallocation (hipFree synchronizes the device) cost more
// than the whole device-side list build.
template <typename T>
static int grow_buf(T **p, uint64_t &have, uint64_t need) {
    if (need <= have && *p) return GNS_OK;
    dfree(*p);
    *p = nullptr;
    have = 0;
    const uint64_t n = std::max<uint64_t>(2 * need, 1);
    GNS_TRY(dalloc(reinterpret_cast<void **>(p), n * sizeof(T)));
    have = n;
    return GNS_OK;
}

struct gns_cm {
    int device = 0;
    hipStream_t stream = nullptr;
    CmGeom g{};
    KeyPlanN kp{};
    uint32_t K = 0, st = 0, ct = 0;
    uint32_t *C = nullptr, *S = nullptr, *Fc = nullptr, *Fs = nullptr;
    CmScratch rd;                 // read-side buffers of the handle's own queries (grow-only)
    std::atomic<uint32_t> period{0};  // bumped by reset: snapshot views taken before it are stale
    std::mutex views_mu;              // guards `views` (view create/destroy vs reset / dictionary reclaim)
    std::vector<gns_cm_view *> views; // live snapshot views: reset and reclaim wait for their calls
    DictDev D{};
    uint64_t dict_slots = 0;
    uint64_t max_flows = 0;               // proactive reclaim once this many slots are claimed
    uint64_t claimed = 0;                 // D.ctl[0] as of the last batch
    bool full = false;                    // live flows + one 16K-packet batch exceed the dictionary (sticky)
    uint32_t *dctl = nullptr;             // D.ctl: [0] claimed slots, [1] abort flag
    DictScratch dsc;                      // rebuild scratch (grow-only)
    unsigned long long *stats_bak = nullptr;  // [3] counters before the running batch (undone on abort)
    uint64_t n_reclaim = 0, n_dropped = 0, last_live = 0, n_retry = 0, n_grow = 0;
    double reclaim_ms = 0.0;
    uint32_t epoch = 0;
    uint64_t bmax = 0;
    uint32_t nblk_max = 0;
    uint32_t *keyid = nullptr, *idx = nullptr;
    uint64_t *pend[2] = {nullptr, nullptr};
    uint32_t *pcnt[2] = {nullptr, nullptr};
    uint32_t *ptotal = nullptr;        // [2]
    uint32_t *hist = nullptr, *part = nullptr, *total = nullptr, *order = nullptr;
    uint64_t *entries = nullptr, *entries2 = nullptr;
    uint16_t *rseg = nullptr;          // [round][16] k_subpart round tile starts (sub_bits > 0)
    int subpart_nt = 0;                // GNS_SUBPART_NT (A/B)
    bool k4_sparse = true;             // super-bins through k_apply_sparse (GNS_K4_SPARSE=0: k_subpart + tiles)
    uint32_t *rec_sizes = nullptr;     // 16-byte compact records from device memory: a batch's sizes
    uint64_t *ovf = nullptr;
    uint32_t *ovf_cnt = nullptr;
    uint64_t ovf_cap = 0;                 // entries of ovf
    unsigned long long *stats = nullptr;  // [8] counters (gns_cm_counters), [8] oversize packets of the batch
    uint32_t *hot_ids = nullptr;          // [d][kHot] designated buckets for the next batch
    uint32_t *hot_tab = nullptr;          // [d][kHotTab] their lookup groups
    long long *segtot = nullptr;          // [d*kHot][kHotSegs][2]
    uint32_t *hflag = nullptr, *hhist = nullptr, *hthr = nullptr, *hcnt = nullptr;
    uint32_t *hcand = nullptr, *hcn = nullptr;  // designation candidates [d][kHotCand]; counts [8] + list-incomplete flags [8]
    HotSum *hsum = nullptr;               // [d*kHot][nblk_max]
    uint32_t *hflag2 = nullptr;           // [d*kHot + 2]: flags, then hany, nchk
    uint32_t *work = nullptr;             // K4 schedule counter
    uint32_t ncu = 256;                   // compute units (K4 persistent grid)
    uint32_t *hres = nullptr;             // [d*kHot][2]
    uint4 *chk = nullptr;                 // [kChkCap]
    bool warm = false;                    // a batch has run since create/reset
    bool lds_ordered = false;             // k_lds_order_probe passed: K3 ranks by LDS adds
    bool k3_half = false, k3_pack = false;
    uint32_t k3_xcd = 0;
    bool k3_staged = true;                // K3s (LDS-staged runs) where the geometry allows; GNS_K3_STAGED=0: K3
    // compact streams (K1 -> K3c): off by default (K3 -0.31 ms, K1 +0.51 ms
    // at the bench geometry); GNS_CMODE=1 turns them on where the geometry allows
    // (256-thread K1, K3s rows, buckets < 2^20)
    bool cmode = false;
    uint32_t *hstr = nullptr;             // [nblk][4][d][4096] hot codes (cold codes live in idx)
    uint32_t *scnt = nullptr;             // [nblk][4][d][2] stream lengths
    uint32_t *h_pin = nullptr;            // pinned host mirror of small counters
    // staging for host inputs: two device buffers; batch i+1's H2D copies run on
    // cstream while batch i computes on `stream` (events order the reuse)
    uint8_t *stage[2] = {nullptr, nullptr};
    size_t stage_bytes[2] = {0, 0};
    uint32_t *side_dev = nullptr;         // staged side records of a compact host insert
    uint64_t side_n = 0;
    hipStream_t cstream = nullptr;
    hipEvent_t ev_copied[2] = {nullptr, nullptr}, ev_used[2] = {nullptr, nullptr};
    StageTimer timer;
};

struct gns_cm_view {
    gns_cm *cm = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t ready = nullptr;
    uint32_t *C = nullptr, *S = nullptr, *Fc = nullptr, *Fs = nullptr;
    CmScratch rd;
    std::mutex mu;          // refresh vs queries: a refresh waits for the query in progress
    uint32_t period = ~0u;  // handle period of the snapshot (~0: never refreshed)
};

// Holds every registered view's mutex: no view call is running (each one
// synchronizes its stream before it returns), so the handle may rewrite what
// the views read (the flow dictionary) and bump the period they check.
struct ViewsQuiesced {
    std::unique_lock<std::mutex> reg;
    std::vector<std::unique_lock<std::mutex>> locks;
    explicit ViewsQuiesced(gns_cm *cm) : reg(cm->views_mu) {
        locks.reserve(cm->views.size());
        for (gns_cm_view *v : cm->views) locks.emplace_back(v->mu);
    }
};

namespace {

int stage_reserve(gns_cm *cm, int b, size_t bytes) {
    if (!cm->cstream) {
        GNS_HIP(hipStreamCreateWithFlags(&cm->cstream, hipStreamNonBlocking));
        for (int i = 0; i < 2; i++) {
            GNS_HIP(hipEventCreateWithFlags(&cm->ev_copied[i], hipEventDisableTiming));
            GNS_HIP(hipEventCreateWithFlags(&cm->ev_used[i], hipEventDisableTiming));
        }
    }
    if (cm->stage_bytes[b] >= bytes) return GNS_OK;
    GNS_HIP(hipEventSynchronize(cm->ev_used[b]));  // the batch that read it is done
    dfree(cm->stage[b]);
    cm->stage[b] = nullptr;
    cm->stage_bytes[b] = 0;
    GNS_TRY(dalloc(reinterpret_cast<void **>(&cm->stage[b]), bytes));
    cm->stage_bytes[b] = bytes;
    return GNS_OK;
}

int set_dev(gns_cm *cm) {
    (void)hipGetLastError();  // a stale error of an earlier runtime call on this thread (e.g. the
                              // host framework's) must not fail this call's launch checks
    GNS_HIP(hipSetDevice(cm->device));
    return GNS_OK;
}

int cm_free_all(gns_cm *cm) {
    dfree(cm->C); dfree(cm->S); dfree(cm->Fc); dfree(cm->Fs); cm->rd.free_all();
    dfree(cm->D.rec);
    dfree(cm->keyid); dfree(cm->idx); dfree(cm->scnt);  // hstr lives in idx
    dfree(cm->pend[0]); dfree(cm->pend[1]); dfree(cm->pcnt[0]); dfree(cm->pcnt[1]);
    dfree(cm->ptotal); dfree(cm->hist); dfree(cm->part); dfree(cm->total); dfree(cm->order);
    dfree(cm->entries); dfree(cm->entries2); dfree(cm->rseg); dfree(cm->rec_sizes); dfree(cm->ovf); dfree(cm->ovf_cnt); dfree(cm->stats);
    dfree(cm->stage[0]); dfree(cm->stage[1]); dfree(cm->side_dev);
    for (int i = 0; i < 2; i++) {
        if (cm->ev_copied[i]) (void)hipEventDestroy(cm->ev_copied[i]);
        if (cm->ev_used[i]) (void)hipEventDestroy(cm->ev_used[i]);
    }
    if (cm->cstream) (void)hipStreamDestroy(cm->cstream);
    dfree(cm->work);
    dfree(cm->hot_ids); dfree(cm->segtot); dfree(cm->hflag); dfree(cm->hhist); dfree(cm->hthr); dfree(cm->hcnt);
    dfree(cm->hcand); dfree(cm->hcn);
    dfree(cm->hsum); dfree(cm->hflag2); dfree(cm->hres); dfree(cm->chk); dfree(cm->hot_tab);
    dfree(cm->dctl); dfree(cm->stats_bak); cm->dsc.free_all();
    if (cm->h_pin) (void)hipHostFree(cm->h_pin);
    cm->timer.destroy();
    if (cm->stream) (void)hipStreamDestroy(cm->stream);
    return GNS_OK;
}

int cm_reset_state(gns_cm *cm) {
    const uint64_t cells = (uint64_t)cm->g.d * cm->g.w;
    GNS_HIP(hipMemsetAsync(cm->C, 0, cells * 4, cm->stream));
    GNS_HIP(hipMemsetAsync(cm->S, 0, cells * 4, cm->stream));
    GNS_HIP(hipMemsetAsync(cm->Fc, 0xFF, cells * 4, cm->stream));
    GNS_HIP(hipMemsetAsync(cm->Fs, 0xFF, cells * 4, cm->stream));
    GNS_HIP(hipMemsetAsync(cm->D.rec, 0, cm->dict_slots * cm->D.RW * 4, cm->stream));
    GNS_HIP(hipMemsetAsync(cm->hot_ids, 0xFF, (size_t)cm->g.d * kHot * 4, cm->stream));
    GNS_HIP(hipMemsetAsync(cm->hot_tab, 0xFF, (size_t)cm->g.d * kHotTab * 4, cm->stream));
    GNS_HIP(hipMemsetAsync(cm->hhist, 0, (size_t)cm->g.d * kHotKeys * 4, cm->stream));
    GNS_HIP(hipMemsetAsync(cm->hthr, 0xFF, 8 * 4, cm->stream));  // no previous threshold: no candidates
    GNS_HIP(hipMemsetAsync(cm->hcn, 0, 16 * 4, cm->stream));
    // the error words (3 dict-full, 4 ovf-full) belong to the period: a reset
    // empties the dictionary, so the next period starts without them
    GNS_HIP(hipMemsetAsync(cm->stats + 3, 0, 2 * sizeof(unsigned long long), cm->stream));
    GNS_HIP(hipMemsetAsync(cm->dctl, 0, 16, cm->stream));
    cm->claimed = 0;
    cm->full = false;
    cm->warm = false;
    return GNS_OK;
}

// Reclaim: rebuild the dictionary keeping the flows a bucket (or a snapshot
// view of the current period) still names (gns_dict.hip).  Views are quiesced
// and their snapshots remapped with the buckets, so a view answers exactly as
// before; a stale view (taken before a reset) names nothing: it answers
// GNS_E_ARG until refreshed, which overwrites its ids.  The table doubles
// while the live flows exceed a quarter of it, and to at least min_slots.
void cm_dict_limits(gns_cm *cm) {
    cm->D.cap = (uint32_t)(cm->dict_slots - cm->dict_slots / 4);  // claims beyond 3/4 load abort the batch
    cm->max_flows = std::max<uint64_t>(cm->max_flows, cm->dict_slots / 2);  // proactive reclaim at load 1/2
}

int cm_reclaim(gns_cm *cm, uint64_t min_slots = 0) {
    ViewsQuiesced q(cm);
    const uint64_t cells = (uint64_t)cm->g.d * cm->g.w;
    std::vector<DictIds> ids{{cm->Fc, cells}, {cm->Fs, cells}};
    const uint32_t period = cm->period.load();
    for (gns_cm_view *v : cm->views)
        if (v->period == period) { ids.push_back({v->Fc, cells}); ids.push_back({v->Fs, cells}); }
    const auto t0 = std::chrono::steady_clock::now();
    const uint64_t before = cm->claimed, slots0 = cm->dict_slots;
    uint64_t live = 0;
    GNS_TRY(dict_rebuild(cm->D, cm->dict_slots, ids.data(), (int)ids.size(), nullptr, ids.data(), (int)ids.size(),
                         std::min(kDictMaxSlots, std::max(cm->dict_slots, min_slots)), cm->stream, cm->dsc, &live,
                         nullptr, kDictMaxSlots));
    cm->reclaim_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    cm->n_reclaim++;
    if (cm->dict_slots != slots0) cm->n_grow++;
    cm_dict_limits(cm);
    cm->n_dropped += before > live ? before - live : 0;
    cm->claimed = live;
    cm->last_live = live;
    return GNS_OK;
}

// One device batch: n <= bmax packets, inputs already device-resident.
template <int KIND, int MODE>
int cm_run_batch(gns_cm *cm, const InputDesc &in, uint64_t n) {
    if (n == 0) return GNS_OK;
    hipStream_t s = cm->stream;
    const uint32_t nblk = (uint32_t)((n + kChunk - 1) / kChunk);
    const CmGeom &g = cm->g;
    ScopedStage total_stage(cm->timer, 5);
    // K1
    {  // one launch: resolve totals, this batch's abort flag, hot flags, oversize packets (K1)
        CtlZero z;
        z.add(cm->ptotal, 8);
        z.add(cm->dctl + 1, 4);
        z.add(cm->hflag2, ((size_t)g.d * kHot + 2) * 4);
        z.add(cm->stats + 8, 8);
        z.add(cm->ovf_cnt, 4);  // K3's oversize list (both K3 modes append)
        z.add(cm->work, 12);    // K4's work counters
        z.add(cm->hflag, (size_t)g.d * kHot * 4);
        GNS_HIP(ctl_zero(z, s));
    }
    if (++cm->epoch == 0) cm->epoch = 1;
    {
        ExtractArgs a{};
        a.in = in; a.n = n; a.kp = cm->kp; a.g = g; a.D = cm->D; a.epoch = cm->epoch;
        a.keyid = cm->keyid; a.idx = cm->idx; a.pend = cm->pend[0]; a.pend_cnt = cm->pcnt[0];
        a.pend_total = cm->ptotal; a.hist = cm->hist; a.nblk = nblk; a.hot_ids = cm->hot_ids;
        a.Fc = cm->Fc; a.Fs = cm->Fs; a.hsum = cm->hsum; a.hot_tab = cm->hot_tab;
        a.stats = cm->stats;
        a.cstr = cm->idx; a.hstr = cm->hstr; a.scnt = cm->scnt; a.hoff = (uint32_t)(cm->hstr - cm->idx);
        ScopedStage st(cm->timer, 0);
        const size_t lds = extract_lds_bytes(g.nbins_all, g.d);
        // 256-thread K1: with compact streams when the handle uses them
#define GNS_K1_256(KB_, DD_)                                                                                   \
    do {                                                                                                       \
        if (cm->cmode)                                                                                         \
            hipLaunchKernelGGL((k_extract<KIND, MODE, KB_, DD_, 256, true>), dim3(nblk), dim3(256), lds, s, a); \
        else                                                                                                   \
            hipLaunchKernelGGL((k_extract<KIND, MODE, KB_, DD_, 256>), dim3(nblk), dim3(kExThreads), lds, s, a); \
    } while (0)
        if constexpr (KIND == IN_REC16) {  // PCIe-bound host path: runtime key width and depth
            if (lds > kExLdsSmall)
                hipLaunchKernelGGL((k_extract<KIND, MODE, 0, 0, 1024>), dim3(nblk), dim3(1024), lds, s, a);
            else
                GNS_K1_256(0, 0);
        } else if (lds > kExLdsSmall) {  // deep / wide sketch: one large block per CU
            // configs[4] (d=8, 5-tuple): the plain loop, two 512-thread blocks per CU
            // (see kC5Threads)
            if (cm->K == 37 && g.d == 8)
                hipLaunchKernelGGL((k_extract<KIND, MODE, 37, 8, kC5Threads>), dim3(nblk), dim3(kC5Threads), lds, s, a);
            else if (cm->K == 37)
                hipLaunchKernelGGL((k_extract<KIND, MODE, 37, 0, 1024>), dim3(nblk), dim3(1024), lds, s, a);
            else if (cm->K == 16)
                hipLaunchKernelGGL((k_extract<KIND, MODE, 16, 0, 1024>), dim3(nblk), dim3(1024), lds, s, a);
            else
                hipLaunchKernelGGL((k_extract<KIND, MODE, 0, 0, 1024>), dim3(nblk), dim3(1024), lds, s, a);
        } else if (cm->K == 37 && g.d == 4)
            GNS_K1_256(37, 4);
        else if (cm->K == 37)
            GNS_K1_256(37, 0);
        else if (cm->K == 16 && g.d == 4)
            GNS_K1_256(16, 4);
        else if (cm->K == 16)
            GNS_K1_256(16, 0);
        else
            GNS_K1_256(0, 0);
#undef GNS_K1_256
        GNS_HIP(hipGetLastError());
    }
    // K1b: resolve parked packets until none remain.  The first two rounds are queued
    // behind K1 without a host round trip (K1 parks the flows displaced from their
    // home slot, so most batches have parked packets, and the second round nearly
    // always empties the list; a block with none exits at once), then the host reads
    // the remaining count once.
    int cur = 0;
    for (int round = 0;; round++) {
        if (round > 1) {
            CtlRead rd;  // one launch writes the words into the pinned mirror
            rd.add(cm->ptotal + cur, 4, 0);
            rd.add(cm->stats + 3, 8, 2);
            rd.add(cm->dctl, 4, 4);
            if (round == 2) rd.add(cm->stats + 8, 8, 6);
            GNS_HIP(ctl_read(rd, cm->h_pin, s));
            GNS_HIP(hipStreamSynchronize(s));
            cm->claimed = cm->h_pin[4];
            if (round == 2) {  // the overflow side table holds every oversize row-update of the batch
                const uint64_t big = (uint64_t)cm->h_pin[6] | (uint64_t)cm->h_pin[7] << 32;
                if (big * g.d > cm->ovf_cap) {
                    const uint64_t want = std::min<uint64_t>(std::max<uint64_t>(big * g.d + big * g.d / 4, kOvfCap), 1ull << 31);
                    dfree(cm->ovf);
                    cm->ovf = nullptr;
                    cm->ovf_cap = 0;
                    GNS_TRY(dalloc_t(&cm->ovf, want));
                    cm->ovf_cap = want;
                }
            }
            if (cm->h_pin[2] | cm->h_pin[3]) {
                set_error("flow dictionary full (%llu slots); raise max_flows",
                          (unsigned long long)cm->dict_slots);
                return GNS_E_FULL;
            }
            if (cm->h_pin[0] == 0) break;
        }
        if (round > 64) { set_error("dictionary resolve did not converge"); return GNS_E_FULL; }
        // ptotal[cur ^ 1] is zero: the batch's control zeroing (round 0) or the previous round
        if (++cm->epoch == 0) cm->epoch = 1;
        ResolveArgs a{};
        a.in = in; a.n = n; a.kp = cm->kp; a.D = cm->D; a.epoch = cm->epoch; a.keyid = cm->keyid;
        a.pend_in = cm->pend[cur]; a.cnt_in = cm->pcnt[cur];
        a.pend_out = cm->pend[cur ^ 1]; a.cnt_out = cm->pcnt[cur ^ 1]; a.total_out = cm->ptotal + (cur ^ 1);
        a.total_in = cm->ptotal + cur;
        a.stats = cm->stats; a.g = g;
        ScopedStage st(cm->timer, 1);
        hipLaunchKernelGGL((k_resolve<KIND, MODE>), dim3(nblk), dim3(kExThreads), 0, s, a);
        GNS_HIP(hipGetLastError());
        cur ^= 1;
    }
    // K2
    {
        ScopedStage st(cm->timer, 2);
        const uint32_t ngrp = (nblk + kTGrp - 1) / kTGrp;
        const dim3 g2((g.nbins_all + 255) / 256, ngrp);
        uint32_t *tot = cm->part + (size_t)ngrp * g.nbins_all;
        hipLaunchKernelGGL(k_tscan_part, g2, dim3(256), 0, s, cm->hist, nblk, g.nbins_all, cm->part);
        hipLaunchKernelGGL(k_tscan_mid, dim3((g.nbins_all + 255) / 256), dim3(256), 0, s, cm->part, ngrp, g.nbins_all, tot);
        hipLaunchKernelGGL(k_tscan_bins, dim3(1), dim3(1024), 0, s, tot, g.nbins_all, cm->total);
        hipLaunchKernelGGL(k_tscan_down, g2, dim3(256), 0, s, cm->hist, nblk, g.nbins_all, cm->part, tot);
        GNS_HIP(hipGetLastError());
    }
    // K3
    {
        ScatterArgs a{};
        a.n = n; a.g = g; a.keyid = cm->keyid; a.idx = cm->idx; a.sizes = in.sizes;
        a.xcd_map = cm->k3_xcd;
        a.offsets = cm->hist; a.nblk = nblk; a.entries = cm->entries; a.ovf = cm->ovf;
        a.ovf_cnt = cm->ovf_cnt; a.ovf_cap = (uint32_t)cm->ovf_cap; a.hot_ids = cm->hot_ids; a.stats = cm->stats;
        a.hot_mode = 0; a.hflag2 = cm->hflag2; a.hany = cm->hflag2 + g.d * kHot;
        a.cstr = cm->idx; a.hstr = cm->hstr; a.scnt = cm->scnt;
        ScopedStage st(cm->timer, 3);
        if (cm->cmode)
            hipLaunchKernelGGL((k_scatter_cs<1024, 256>), dim3(nblk), dim3(1024), 0, s, a);
        else if (cm->lds_ordered && cm->k3_staged && g.ntiles <= 256 && g.d <= 8 && cm->k3_half)
            hipLaunchKernelGGL((k_scatter_st<512, 256, 4096>), dim3(nblk), dim3(512), 0, s, a);
        else if (cm->lds_ordered && cm->k3_staged && g.ntiles <= 256 && g.d <= 8)
            hipLaunchKernelGGL((k_scatter_st<1024, 256>), dim3(nblk), dim3(1024), 0, s, a);
        else if (cm->lds_ordered && cm->k3_staged && g.ntiles <= 512 && g.d <= 8 && cm->k3_pack)
            hipLaunchKernelGGL((k_scatter_st<1024, 512, (int)kStSub, true>), dim3(nblk), dim3(1024), 0, s, a);
        else if (cm->lds_ordered && cm->k3_staged && g.ntiles <= 512 && g.d <= 8)
            hipLaunchKernelGGL((k_scatter_st<512, 512>), dim3(nblk), dim3(512), 0, s, a);
        else if (cm->lds_ordered)
            hipLaunchKernelGGL(k_scatter<1>, dim3(nblk), dim3(kScThreads), scatter_lds_bytes(g.ntiles + kHot, g.d), s, a);
        else
            hipLaunchKernelGGL(k_scatter<0>, dim3(nblk), dim3(kScThreads), scatter_lds_bytes(g.ntiles + kHot, g.d), s, a);
        GNS_HIP(hipGetLastError());
    }
    // K4
    {
        const bool ordered = g.nbins <= 4096;
        if (ordered)
            hipLaunchKernelGGL(k_order, dim3(1), dim3(1024), 0, s, cm->hist, nblk, g.nbins, g.nbins_all,
                               cm->total, cm->order);
        ApplyArgs a{};
        a.stats = cm->stats;
        a.entries = cm->entries; a.entries2 = cm->entries2; a.offsets = cm->hist; a.nblk = nblk; a.nbins = g.nbins;
        a.total = cm->total; a.order = ordered ? cm->order : nullptr; a.ovf = cm->ovf; a.g = g;
        a.C = cm->C; a.Fc = cm->Fc; a.S = cm->S; a.Fs = cm->Fs; a.work = cm->work;
        ScopedStage st(cm->timer, 4);
        if (g.sub_bits && cm->k4_sparse) {
            // super-bins in stream order, touched buckets only (k_apply_sparse): no
            // sub-partition pass and no tile sweep; GNS_K4_SPARSE=0 restores the tile path
            const dim3 apg(std::min(g.nbins, cm->ncu));
            hipLaunchKernelGGL(k_apply_sparse, apg, dim3(kApThreads), 0, s, a);
        } else if (g.sub_bits) {
            // 512-thread workgroups (16 updates per thread and round, two per CU) when a
            // wave per tile fits; GNS_SUBPART_NT=1024 for the A/B
            if ((1u << g.sub_bits) <= 8 && cm->subpart_nt != 1024)
                hipLaunchKernelGGL(k_subpart<512>, dim3(g.nbins), dim3(512), 0, s, a, cm->rseg);
            else
                hipLaunchKernelGGL(k_subpart<1024>, dim3(g.nbins), dim3(1024), 0, s, a, cm->rseg);
            GNS_HIP(hipGetLastError());
            a.rseg = cm->rseg;
        }
        // persistent: one workgroup per CU (the tile LDS fills a CU), bins from the schedule counter
        const dim3 apg(std::min(g.nbins, cm->ncu * (kApThreads <= 512 ? 2u : 1u)));  // workgroups the LDS fits per CU
        if (g.sub_bits && cm->k4_sparse) {
            // (launched above)
        } else if (!g.sub_bits) {
            hipLaunchKernelGGL(k_apply<0>, apg, dim3(kApThreads), 0, s, a);
        } else {
            hipLaunchKernelGGL(k_apply<1>, apg, dim3(kApThreads), 0, s, a);
            GNS_HIP(hipGetLastError());
            // super-bins too big for K4's LDS tables (none at the bench geometry): windows of rounds
            hipLaunchKernelGGL(k_apply<3>, apg, dim3(kApThreads), 0, s, a);
        }
        GNS_HIP(hipGetLastError());
    }
    // hot bins: chip-wide aggregate, exact decide, in-order fallback
    {
        HotArgs h{};
        h.entries = cm->entries; h.offsets = cm->hist; h.nblk = nblk; h.total = cm->total; h.ovf = cm->ovf;
        h.hot_ids = cm->hot_ids; h.g = g; h.C = cm->C; h.Fc = cm->Fc; h.S = cm->S; h.Fs = cm->Fs;
        h.segtot = cm->segtot; h.hflag = cm->hflag;
        h.hsum = cm->hsum; h.hflag2 = cm->hflag2; h.hany = cm->hflag2 + g.d * kHot; h.nchk = h.hany + 1;
        h.hres = cm->hres; h.chk = cm->chk; h.chk_cap = kChkCap;
        h.keyid = cm->keyid; h.idx = cm->idx; h.sizes = in.sizes; h.n = n;
        h.hstr = cm->cmode ? cm->hstr : nullptr; h.scnt = cm->scnt;
        ScopedStage st(cm->timer, 6);
        // summary path: decide, exact block checks, commit
        hipLaunchKernelGGL(k_hot_decide, dim3(g.d * kHot), dim3(256), 0, s, h);
        hipLaunchKernelGGL(k_hot_blockcheck, dim3(kChkCap), dim3(256), 0, s, h);
        hipLaunchKernelGGL(k_hot_commit, dim3((g.d * kHot + 511) / 512), dim3(512), 0, s, h);
        // exact entry path for flagged halves (device-side early exit when none)
        {
            ScatterArgs a{};
            a.n = n; a.g = g; a.keyid = cm->keyid; a.idx = cm->idx; a.sizes = in.sizes;
            a.offsets = cm->hist; a.nblk = nblk; a.entries = cm->entries; a.ovf = cm->ovf;
            a.ovf_cnt = cm->ovf_cnt; a.ovf_cap = (uint32_t)cm->ovf_cap; a.hot_ids = cm->hot_ids; a.stats = cm->stats;
            a.hot_mode = 1; a.hflag2 = cm->hflag2; a.hany = h.hany;
            a.cstr = cm->idx; a.hstr = cm->hstr; a.scnt = cm->scnt;
            if (cm->cmode)
                hipLaunchKernelGGL(k_hot_scatter_cs, dim3(nblk), dim3(64), 0, s, a);
            else if (cm->lds_ordered)
                hipLaunchKernelGGL(k_scatter<1>, dim3(nblk), dim3(kScThreads), scatter_lds_bytes(g.ntiles + kHot, g.d), s, a);
            else
                hipLaunchKernelGGL(k_scatter<0>, dim3(nblk), dim3(kScThreads), scatter_lds_bytes(g.ntiles + kHot, g.d), s, a);
        }
        hipLaunchKernelGGL(k_hot_sum, dim3(1024), dim3(256), 0, s, h);
        hipLaunchKernelGGL(k_hot_verify, dim3(1024), dim3(256), 0, s, h);
        hipLaunchKernelGGL(k_hot_apply, dim3((g.d * kHot + 511) / 512), dim3(512), 0, s, h);
        hipLaunchKernelGGL(k_hot_fallback, dim3(g.d * kHot), dim3(64), 0, s, h);
        GNS_HIP(hipGetLastError());
    }
    // designate the next batch's hot buckets from the counters
    {
        ScopedStage st(cm->timer, 7);
        const unsigned grid = (unsigned)std::min<uint64_t>(2048, ((uint64_t)g.w / 4 + 255) / 256 + 1);
        // few blocks for the histogram: its flush is one global atomic per (block, nonzero class)
        uint32_t *hcn = cm->hcn, *hfull = cm->hcn + 8;
        hipLaunchKernelGGL(k_hot_hist, dim3(std::min(grid, 512u)), dim3(256), 0, s, cm->C, g, cm->hhist, cm->hthr,
                           cm->hcand, hcn);
        hipLaunchKernelGGL(k_hot_pick, dim3(1), dim3(512), 0, s, cm->hhist, g, cm->hthr, cm->hcnt, cm->hot_ids, hcn,
                           hfull);
        hipLaunchKernelGGL(k_hot_collect, dim3(grid), dim3(256), 0, s, cm->C, g, cm->hthr, cm->hcnt, cm->hot_ids,
                           cm->hcand, hcn, hfull);
        hipLaunchKernelGGL(k_hot_table, dim3(1), dim3(1024), 0, s, g, cm->hot_ids, cm->hot_tab, hcn);
        GNS_HIP(hipGetLastError());
    }
    cm->warm = true;
    return GNS_OK;
}

InputDesc advance(const InputDesc &in, uint64_t off) {
    InputDesc d = in;
    if (d.hdr) d.hdr += off * 16;
    if (d.src16) d.src16 += off * 16;
    if (d.dst16) d.dst16 += off * 16;
    if (d.sport) d.sport += off;
    if (d.dport) d.dport += off;
    if (d.proto) d.proto += off;
    if (d.keys) d.keys += off * d.stride;
    if (d.rec16) d.rec16 += off * 4;
    if (d.sizes) d.sizes += off;
    return d;
}

template <int KIND>
int cm_batch(gns_cm *cm, const InputDesc &d, uint64_t m) {
    if constexpr (KIND == IN_KEYS) {
        return cm_run_batch<KIND, PLAN_SLICE0>(cm, d, m);
    } else {
        switch (plan_mode(cm->kp)) {
        case PLAN_SLICE0: return cm_run_batch<KIND, PLAN_SLICE0>(cm, d, m);
        case PLAN_SLICE4: return cm_run_batch<KIND, PLAN_SLICE4>(cm, d, m);
        default: return cm_run_batch<KIND, PLAN_GENERIC>(cm, d, m);
        }
    }
}

// One device batch (device-resident inputs) with dictionary recovery: a batch
// whose new flows overflow the dictionary is aborted before it changes the
// sketch, its counters are undone and its claims dropped with
// the dead flows (reclaim); it is re-run as is once, then in halves.  A piece
// of <= kChunk packets that does not fit a freshly rebuilt dictionary doubles
// the table instead, so the engine keeps counting whatever the stream brings,
// as the reference's fixed table of key bytes does (count_min.go:66-81,94-157):
// live ids are bounded by 2*d*w, the table by kDictMaxSlots.  fresh: the
// dictionary was rebuilt right before this batch.
template <int KIND>
int cm_batch_recover(gns_cm *cm, const InputDesc &d, uint64_t m, bool fresh) {
    if (m == 0) return GNS_OK;
    if (cm->full) {
        set_error("flow dictionary full (%llu slots, %llu live flows)",
                  (unsigned long long)cm->dict_slots, (unsigned long long)cm->last_live);
        return GNS_E_FULL;
    }
    if (cm->claimed >= cm->max_flows) {  // proactive: keep the load <= ~1/2
        GNS_TRY(cm_reclaim(cm));
        fresh = true;
    }
    for (;;) {
        GNS_HIP(hipMemcpyAsync(cm->stats_bak, cm->stats, 3 * sizeof(unsigned long long), hipMemcpyDeviceToDevice,
                               cm->stream));
        const int rc = cm_batch<KIND>(cm, d, m);
        if (rc != GNS_E_FULL) return rc;
        // not applied: undo its counters, drop its claims and the dead flows
        GNS_HIP(hipMemcpyAsync(cm->stats, cm->stats_bak, 3 * sizeof(unsigned long long), hipMemcpyDeviceToDevice,
                               cm->stream));
        GNS_HIP(hipMemsetAsync(cm->stats + 3, 0, sizeof(unsigned long long), cm->stream));
        cm->n_retry++;
        if (!fresh) {  // the flows that died since the last rebuild may be room enough
            GNS_TRY(cm_reclaim(cm));
            fresh = true;
            continue;
        }
        if (m > kChunk) {  // split: each half meets a fresh dictionary
            GNS_TRY(cm_reclaim(cm));
            break;
        }
        if (cm->dict_slots >= kDictMaxSlots) {  // cannot happen below 2*d*w + kChunk ~ 3/4 * 2^30 live flows
            GNS_TRY(cm_reclaim(cm));
            cm->full = true;
            const unsigned long long one = 1;
            GNS_HIP(hipMemcpy(cm->stats + 3, &one, sizeof(one), hipMemcpyHostToDevice));
            set_error("flow dictionary full: %llu live flows plus one %u-packet batch exceed %llu slots",
                      (unsigned long long)cm->last_live, kChunk, (unsigned long long)cm->dict_slots);
            return GNS_E_FULL;
        }
        GNS_TRY(cm_reclaim(cm, cm->dict_slots * 2));  // grow, then re-run the piece
    }
    const uint64_t h = ((m / 2 + kChunk - 1) / kChunk) * kChunk;
    GNS_TRY(cm_batch_recover<KIND>(cm, d, h, true));
    return cm_batch_recover<KIND>(cm, advance(d, h), m - h, false);
}

// 16-byte compact records: the wire lengths (word 3 bits 16..31) as the batch's size array
__global__ __launch_bounds__(256) void k_rec_sizes(const uint32_t *rec16, uint64_t n, uint32_t *sizes) {
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) sizes[i] = rec16[i * 4 + 3] >> 16;
}

// Host input: stage batch [off, off+m) into device buffer b on the copy stream,
// after the batch that last read b has finished; d points into the buffer.
int stage_host_batch(gns_cm *cm, int b, const InputDesc &in, uint64_t off, uint64_t m, InputDesc &d) {
    d = in;
    constexpr int NA = 8;
    const void *src[NA] = {in.hdr ? (const void *)(in.hdr + off * 16) : nullptr,
                           in.src16 ? (const void *)(in.src16 + off * 16) : nullptr,
                           in.dst16 ? (const void *)(in.dst16 + off * 16) : nullptr,
                           in.sport ? (const void *)(in.sport + off) : nullptr,
                           in.dport ? (const void *)(in.dport + off) : nullptr,
                           in.proto ? (const void *)(in.proto + off) : nullptr,
                           in.keys ? (const void *)(in.keys + off * in.stride) : nullptr,
                           in.rec16 ? (const void *)(in.rec16 + off * 4) : nullptr};
    const size_t bytes[NA] = {in.hdr ? m * 64 : 0, in.src16 ? m * 16 : 0, in.dst16 ? m * 16 : 0,
                              in.sport ? m * 2 : 0, in.dport ? m * 2 : 0, in.proto ? m : 0,
                              in.keys ? m * in.stride : 0, in.rec16 ? m * 16 : 0};
    size_t tot = (m * 4 + 15) & ~size_t(15);
    for (int i = 0; i < NA; i++) tot += (bytes[i] + 15) & ~size_t(15);
    GNS_TRY(stage_reserve(cm, b, tot));
    GNS_HIP(hipStreamWaitEvent(cm->cstream, cm->ev_used[b], 0));
    uint8_t *p = cm->stage[b];
    const void **dst[NA] = {(const void **)&d.hdr, (const void **)&d.src16, (const void **)&d.dst16,
                            (const void **)&d.sport, (const void **)&d.dport, (const void **)&d.proto,
                            (const void **)&d.keys, (const void **)&d.rec16};
    for (int i = 0; i < NA; i++) {
        if (!bytes[i]) continue;
        GNS_HIP(hipMemcpyAsync(p, src[i], bytes[i], hipMemcpyHostToDevice, cm->cstream));
        *dst[i] = p;
        p += (bytes[i] + 15) & ~size_t(15);
    }
    if (in.rec_len) {  // sizes from the staged records
        hipLaunchKernelGGL(k_rec_sizes, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, cm->cstream, d.rec16, m,
                           reinterpret_cast<uint32_t *>(p));
        GNS_HIP(hipGetLastError());
    } else {
        GNS_HIP(hipMemcpyAsync(p, in.sizes + off, m * 4, hipMemcpyHostToDevice, cm->cstream));
    }
    d.sizes = reinterpret_cast<const uint32_t *>(p);
    if (d.keys) d.aligned = (d.stride % 4 == 0 && d.stride >= ((cm->K + 3) & ~3u)) ? 1u : 0u;
    GNS_HIP(hipEventRecord(cm->ev_copied[b], cm->cstream));
    return GNS_OK;
}

template <int KIND>
int cm_insert(gns_cm *cm, InputDesc in, uint64_t n, gns_mem where) {
    GNS_TRY(set_dev(cm));
    // batch sizes: a cold handle's small first batch designates the heavy buckets early
    auto batch_len = [&](uint64_t off, bool warm) {
        const uint64_t m = std::min<uint64_t>(cm->bmax, n - off);
        return warm ? m : std::min<uint64_t>(m, std::max<uint64_t>(kChunk * 64, cm->bmax / 32));
    };
    if (where == GNS_MEM_DEVICE) {
        for (uint64_t off = 0, m = 0; off < n; off += m) {
            m = batch_len(off, cm->warm);
            InputDesc d = advance(in, off);
            if (in.rec_len) {  // 16-byte compact records: the batch's sizes unpacked on the stream
                if (!cm->rec_sizes) GNS_TRY(dalloc_t(&cm->rec_sizes, cm->bmax));
                hipLaunchKernelGGL(k_rec_sizes, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, cm->stream, d.rec16, m,
                                   cm->rec_sizes);
                GNS_HIP(hipGetLastError());
                d.sizes = cm->rec_sizes;
            }
            GNS_TRY(cm_batch_recover<KIND>(cm, d, m, false));
        }
        return GNS_OK;
    }
    // host input, double-buffered: the copies of batch i+1 are queued on the copy
    // stream before batch i runs (whose resolve rounds may wait on the host)
    if (n == 0) return GNS_OK;
    bool warm = cm->warm;
    uint64_t off = 0, m = batch_len(0, warm);
    InputDesc d;
    GNS_TRY(stage_host_batch(cm, 0, in, 0, m, d));
    for (int b = 0;; b ^= 1) {
        const uint64_t noff = off + m;
        const uint64_t nm = noff < n ? batch_len(noff, true) : 0;
        InputDesc nd;
        if (nm) GNS_TRY(stage_host_batch(cm, b ^ 1, in, noff, nm, nd));
        GNS_HIP(hipStreamWaitEvent(cm->stream, cm->ev_copied[b], 0));
        const int rc = cm_batch_recover<KIND>(cm, d, m, false);
        GNS_HIP(hipEventRecord(cm->ev_used[b], cm->stream));
        if (rc != GNS_OK) {
            (void)hipStreamSynchronize(cm->cstream);  // no copy may outlive the caller's arrays
            return rc;
        }
        if (!nm) break;
        off = noff; m = nm; d = nd;
    }
    // the caller may reuse its host arrays on return: every copy has been consumed
    // by a batch queued on the handle's stream; wait for the copies themselves
    GNS_HIP(hipStreamSynchronize(cm->cstream));
    return GNS_OK;
}

}  // namespace

extern "C" {

static int heavy_reserve(CmScratch &sc, uint64_t cells, uint64_t slots, uint32_t K, hipStream_t st);

int gns_cm_create(const gns_cm_params *p, gns_cm **out) {
    if (!p || !out) { set_error("null argument"); return GNS_E_ARG; }
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        (void)hipGetLastError();
        set_error("no HIP device available");
        return GNS_E_NODEV;
    }
    if (p->device < 0 || p->device >= ndev) { set_error("device %d out of range", p->device); return GNS_E_ARG; }
    gns_cm *cm = new gns_cm();
    cm->device = p->device;
    int rc = GNS_OK;
    do {
        if ((rc = set_dev(cm)) != GNS_OK) break;
        // count_min.go:48-59 defaults
        CmGeom &g = cm->g;
        g.w = p->width ? p->width : (1u << 20);
        g.d = p->depth ? p->depth : 3u;
        cm->st = p->size_threshold ? p->size_threshold : 512u * 1024u;
        cm->ct = p->count_threshold ? p->count_threshold : 512u;
        if (g.d > 8) { set_error("depth %u > 8 not supported", g.d); rc = GNS_E_ARG; break; }
        if ((rc = make_plan(p->flow, p->key_bytes, &cm->kp)) != GNS_OK) break;
        cm->K = cm->kp.K;
        if (g.w >= (1u << (32 - kHotBits))) {  // designated-bucket table entries hold bucket << kHotBits
            set_error("width %u >= 2^%u is not supported", g.w, 32 - kHotBits); rc = GNS_E_RANGE; break;
        }
        if (p->bucket_lo == 0 && p->bucket_hi == 0) {
            g.blo = 0; g.bspan = g.w;
        } else if (p->bucket_lo < p->bucket_hi && p->bucket_hi <= g.w) {
            g.blo = p->bucket_lo; g.bspan = p->bucket_hi - p->bucket_lo;
        } else {
            set_error("bucket range [%u, %u) is not inside [0, %u)", p->bucket_lo, p->bucket_hi, g.w);
            rc = GNS_E_ARG; break;
        }
        g.pow2 = (g.w & (g.w - 1)) == 0;
        g.wmask = g.pow2 ? g.w - 1 : 0;
        uint32_t tb = kTileBitsMax;
        while (tb > 8 && (uint64_t)g.d * ((g.w + (1u << tb) - 1) >> tb) < 1024) tb--;
        g.tile_bits = tb;
        // bins of 2^sub_bits tiles keep the per-row bin count (K1/K3 LDS, the
        // block histograms) and d * bins bounded for wide rows (C5: w = 2^24)
        uint32_t sb = 0;
        auto bins_at = [&](uint32_t bits) { return (uint32_t)(((uint64_t)g.w + (1ull << bits) - 1) >> bits); };
        while (bins_at(tb + sb) > kMaxTilesPerRow || (uint64_t)g.d * bins_at(tb + sb) > kMaxBinsAll) sb++;
        if (tb + sb > kEntShift || sb > 4) {
            set_error("width %u with depth %u is too wide (max %u buckets per row at this depth)", g.w, g.d,
                      (uint32_t)std::min<uint64_t>(0xFFFFFFFFull, (uint64_t)std::min(kMaxTilesPerRow, kMaxBinsAll / g.d) << kEntShift));
            rc = GNS_E_RANGE;
            break;
        }
        g.sub_bits = sb;
        g.bin_bits = tb + sb;
        g.ntiles = bins_at(g.bin_bits);
        g.nbins = g.d * g.ntiles;
        g.nbins_all = g.nbins + g.d * kHot;
        g.nbits = ceil_log2(g.ntiles + kHot);
        if (p->seeds) for (uint32_t i = 0; i < g.d; i++) g.seeds[i] = p->seeds[i];
        else default_seeds(g.seeds, g.d);
        if (hipStreamCreateWithFlags(&cm->stream, hipStreamNonBlocking) != hipSuccess) {
            set_error("hipStreamCreate failed"); rc = GNS_E_HIP; break;
        }
        cm->timer.stream = cm->stream;
        {
            int ncu = 0;
            if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, cm->device) == hipSuccess && ncu > 0)
                cm->ncu = (uint32_t)ncu;
        }
        const uint64_t cells = (uint64_t)g.d * g.w;
        if ((rc = dalloc_t(&cm->C, cells)) || (rc = dalloc_t(&cm->S, cells)) ||
            (rc = dalloc_t(&cm->Fc, cells)) || (rc = dalloc_t(&cm->Fs, cells)))
            break;
        // flow dictionary: power of two >= 2 * max_flows
        // (the initial capacity: the table grows with the live flows, see cm_reclaim)
        const uint64_t mf = p->max_flows ? p->max_flows : (4ull << 20);
        uint64_t slots = 1;
        while (slots < 2 * mf) slots <<= 1;
        if (slots > kDictMaxSlots) { set_error("max_flows too large"); rc = GNS_E_ARG; break; }
        cm->dict_slots = slots;
        cm->max_flows = mf;
        cm->D.mask = (uint32_t)(slots - 1);
        cm->D.K = cm->K;
        cm->D.RW = dict_record_words_cm(cm->K, g.d);
        cm->D.bw = cm->D.RW >= 16 && 1 + (cm->K + 3) / 4 <= 12 ? 1u : 0u;
        cm->D.seed = 0x2545F491u;
        if ((rc = dalloc_t(&cm->D.rec, slots * cm->D.RW)) != GNS_OK) break;
        if ((rc = dalloc_t(&cm->dctl, 4)) != GNS_OK || (rc = dalloc_t(&cm->stats_bak, 3)) != GNS_OK) break;
        cm->D.ctl = cm->dctl;
        cm_dict_limits(cm);
        // batch buffers
        cm->bmax = p->batch_packets ? p->batch_packets : (16ull << 20);
        cm->bmax = ((cm->bmax + kChunk - 1) / kChunk) * kChunk;
        if (cm->bmax > (1ull << 31)) { set_error("batch_packets too large"); rc = GNS_E_ARG; break; }
        // update positions are u32 and overflow-table slots 31-bit: d * batch <= 2^31
        const uint64_t bcap = (((1ull << 31) / g.d) / kChunk) * kChunk;
        if (cm->bmax > bcap) cm->bmax = bcap;
        cm->nblk_max = (uint32_t)(cm->bmax / kChunk);
        // K2 scratch: group sums [ngrp][nbins_all] + bin totals [nbins_all]
        const uint64_t nscan = ((uint64_t)(cm->nblk_max + kTGrp - 1) / kTGrp + 2) * g.nbins_all;
        if ((rc = dalloc_t(&cm->keyid, cm->bmax)) || (rc = dalloc_t(&cm->idx, cm->bmax * g.d)) ||
            (rc = dalloc_t(&cm->pend[0], cm->bmax)) || (rc = dalloc_t(&cm->pend[1], cm->bmax)) ||
            (rc = dalloc_t(&cm->pcnt[0], cm->nblk_max)) || (rc = dalloc_t(&cm->pcnt[1], cm->nblk_max)) ||
            (rc = dalloc_t(&cm->ptotal, 2)) || (rc = dalloc_t(&cm->hist, (uint64_t)g.nbins_all * cm->nblk_max)) ||
            (rc = dalloc_t(&cm->part, nscan)) || (rc = dalloc_t(&cm->total, 1)) ||
            (rc = dalloc_t(&cm->order, g.nbins)) || (rc = dalloc_t(&cm->entries, cm->bmax * g.d)) ||
            (g.sub_bits && (rc = dalloc_t(&cm->entries2, cm->bmax * g.d))) ||
            (g.sub_bits && (rc = dalloc_t(&cm->rseg, (cm->bmax * g.d / kApChunk + g.nbins + 2) * 16))) ||
            (rc = dalloc_t(&cm->ovf, kOvfCap)) || (rc = dalloc_t(&cm->ovf_cnt, 1)) ||
            (rc = dalloc_t(&cm->stats, kStatsProf + 16)) || (rc = dalloc_t(&cm->work, 4)) || (rc = dalloc_t(&cm->hot_ids, g.d * kHot)) ||
            (rc = dalloc_t(&cm->segtot, (size_t)g.d * kHot * kHotSegs * 2)) || (rc = dalloc_t(&cm->hflag, g.d * kHot)) ||
            (rc = dalloc_t(&cm->hhist, g.d * kHotKeys)) || (rc = dalloc_t(&cm->hthr, 8)) || (rc = dalloc_t(&cm->hcnt, 8)) ||
            (rc = dalloc_t(&cm->hcand, (size_t)g.d * kHotCand)) || (rc = dalloc_t(&cm->hcn, 16)) ||
            (rc = dalloc_t(&cm->hsum, (uint64_t)g.d * kHot * cm->nblk_max)) ||
            (rc = dalloc_t(&cm->hflag2, g.d * kHot + 2)) || (rc = dalloc_t(&cm->hres, g.d * kHot * 2)) ||
            (rc = dalloc_t(&cm->chk, kChkCap)) || (rc = dalloc_t(&cm->hot_tab, (size_t)g.d * kHotTab)))
            break;
        cm->ovf_cap = kOvfCap;
        if (hipHostMalloc(reinterpret_cast<void **>(&cm->h_pin), 64, 0) != hipSuccess) {
            set_error("hipHostMalloc failed"); rc = GNS_E_OOM; break;
        }
        if (hipMemsetAsync(cm->stats, 0, (kStatsProf + 16) * 8, cm->stream) != hipSuccess) { rc = GNS_E_HIP; break; }
        if ((rc = cm_reset_state(cm)) != GNS_OK) break;
        {   // lane-order probe for K3's ranking (GNS_K3_RANK=0 forces the ballot multisplit)
            const char *env = getenv("GNS_K3_RANK");
            uint32_t *viol = nullptr;
            if ((rc = dalloc_t(&viol, 1)) != GNS_OK) break;
            hipError_t e = hipMemsetAsync(viol, 0, 4, cm->stream);
            if (e == hipSuccess) {
                // every CU of every XCD several times over (4 blocks per CU, 64 rounds of random
                // same-address groups each): ~1 ms at create
                hipLaunchKernelGGL(k_lds_order_probe, dim3(4 * cm->ncu), dim3(256), 0, cm->stream, viol, 64);
                e = hipGetLastError();
            }
            uint32_t hv = 1;
            if (e == hipSuccess) e = hipMemcpyAsync(&hv, viol, 4, hipMemcpyDeviceToHost, cm->stream);
            if (e == hipSuccess) e = hipStreamSynchronize(cm->stream);
            dfree(viol);
            if (e != hipSuccess) { set_error("lds order probe: %s", hipGetErrorString(e)); rc = GNS_E_HIP; break; }
            cm->lds_ordered = hv == 0 && !(env && env[0] == '0');
            const char *es = getenv("GNS_K3_STAGED");
            cm->k3_staged = !(es && es[0] == '0');
            cm->k3_half = es && es[0] == 'h';
            const char *ex = getenv("GNS_K3_XCD");
            cm->k3_xcd = ex && ex[0] == '0' ? 0u : 1u;
            cm->k3_pack = !(es && es[0] == 'u');  // 512-bin rows: 1024-thread K3s, 16-bit counters (u: 512 threads)  // A/B: 512-thread K3s, 4096-packet sub-passes, two per CU
            const char *en = getenv("GNS_SUBPART_NT");
            cm->subpart_nt = en ? atoi(en) : 0;
            const char *esp = getenv("GNS_K4_SPARSE");  // super-bins: touched buckets only (0: tile path)
            cm->k4_sparse = !(esp && esp[0] == '0');
            const char *ec = getenv("GNS_CMODE");
            cm->cmode = ec && ec[0] == '1' && cm->lds_ordered && cm->k3_staged && g.ntiles <= 256 && g.d <= 8 &&
                        extract_lds_bytes(g.nbins_all, g.d) <= kExLdsSmall && g.w <= (1u << (32 - kCsBits));
            if (cm->cmode) {  // the hot streams after the cold ones (K1 addresses both from one base)
                dfree(cm->idx);
                cm->idx = nullptr;
                if ((rc = dalloc_t(&cm->idx, 2 * cm->bmax * g.d)) != GNS_OK) break;
                cm->hstr = cm->idx + cm->bmax * g.d;
                if ((rc = dalloc_t(&cm->scnt, (uint64_t)cm->nblk_max * kCsWaves * g.d * 2)) != GNS_OK) break;
            }
        }
        // the read side's heavy-hitter buffers (a window's first call allocates nothing)
        if ((rc = heavy_reserve(cm->rd, (uint64_t)cm->g.d * cm->g.w, cm->dict_slots, cm->K, cm->stream)) != GNS_OK) break;
        if (hipStreamSynchronize(cm->stream) != hipSuccess) { set_error("sync failed"); rc = GNS_E_HIP; break; }
    } while (0);
    if (rc != GNS_OK) {
        cm_free_all(cm);
        delete cm;
        return rc;
    }
    *out = cm;
    return GNS_OK;
}

int gns_cm_destroy(gns_cm *cm) {
    if (!cm) return GNS_OK;
    (void)hipSetDevice(cm->device);
    if (cm->stream) (void)hipStreamSynchronize(cm->stream);
    cm_free_all(cm);
    delete cm;
    return GNS_OK;
}

int gns_cm_insert_keys(gns_cm *cm, const uint8_t *keys, uint32_t stride, const uint32_t *sizes,
                       uint64_t n, gns_mem where) {
    if (!cm || (n && (!keys || !sizes))) { set_error("null argument"); return GNS_E_ARG; }
    if (stride < cm->K) { set_error("stride %u < key_bytes %u", stride, cm->K); return GNS_E_ARG; }
    InputDesc in{};
    in.keys = keys; in.stride = stride; in.sizes = sizes;
    in.aligned = (stride % 4 == 0 && (reinterpret_cast<uintptr_t>(keys) & 3) == 0 &&
                  stride >= ((cm->K + 3) & ~3u)) ? 1u : 0u;
    return cm_insert<IN_KEYS>(cm, in, n, where);
}

int gns_cm_insert_tuples(gns_cm *cm, const gns_tuples *t, uint64_t n, gns_mem where) {
    if (!cm || !t) { set_error("null argument"); return GNS_E_ARG; }
    if (n && (!t->src16 || !t->dst16 || !t->sport || !t->dport || !t->proto || !t->length)) {
        set_error("null tuple array"); return GNS_E_ARG;
    }
    InputDesc in{};
    in.src16 = t->src16; in.dst16 = t->dst16; in.sport = t->sport; in.dport = t->dport;
    in.proto = t->proto; in.sizes = t->length;
    return cm_insert<IN_TUPLE>(cm, in, n, where);
}

int gns_cm_insert_headers(gns_cm *cm, const uint8_t *hdr, const uint32_t *wirelen, uint64_t n,
                          gns_mem where) {
    if (!cm || (n && (!hdr || !wirelen))) { set_error("null argument"); return GNS_E_ARG; }
    InputDesc in{};
    in.hdr = reinterpret_cast<const uint32_t *>(hdr);
    in.sizes = wirelen;
    return cm_insert<IN_HDR>(cm, in, n, where);
}

int gns_cm_insert_compact(gns_cm *cm, const uint8_t *rec16, const uint32_t *wirelen, uint64_t n,
                          const uint8_t *side64, uint64_t n_side, gns_mem where) {
    if (!cm || (n && !rec16) || (n_side && !side64)) { set_error("null argument"); return GNS_E_ARG; }
    InputDesc in{};
    in.rec16 = reinterpret_cast<const uint32_t *>(rec16);
    in.sizes = wirelen;
    in.rec_len = wirelen ? 0u : 1u;  // no wirelen array: the 16-byte form
    in.side = reinterpret_cast<const uint32_t *>(side64);
    in.n_side = side64 ? n_side : 0;
    if (where == GNS_MEM_HOST && n_side) {
        // the side records of the whole call, staged once (escapes index them globally);
        // the batches of the previous call may still read the buffer
        GNS_TRY(set_dev(cm));
        GNS_HIP(hipStreamSynchronize(cm->stream));
        if (cm->side_n < n_side) {
            dfree(cm->side_dev);
            cm->side_dev = nullptr;
            cm->side_n = 0;
            GNS_TRY(dalloc_t(&cm->side_dev, n_side * 16));
            cm->side_n = n_side;
        }
        GNS_HIP(hipMemcpy(cm->side_dev, side64, n_side * 64, hipMemcpyHostToDevice));
        in.side = cm->side_dev;
    }
    return cm_insert<IN_REC16>(cm, in, n, where);
}

int gns_cm_flush(gns_cm *cm) {
    if (!cm) return GNS_E_ARG;
    GNS_TRY(set_dev(cm));
    {  // stats words 4..9 into the pinned mirror behind the stream's work: one round trip
        CtlRead rd;
        rd.add(cm->stats + 4, 48, 0);
        GNS_HIP(ctl_read(rd, cm->h_pin, cm->stream));
    }
    GNS_HIP(hipStreamSynchronize(cm->stream));
    cm->timer.collect();
    if (cm->h_pin[0] | cm->h_pin[1]) {
        set_error("overflow side table exhausted (internal error)");
        return GNS_E_RANGE;
    }
    if (cm->h_pin[10] | cm->h_pin[11]) {  // stats[9]: k_apply_sparse met an update it had not mapped
        set_error("sparse K4: an update's bucket was not in its table (internal error)");
        return GNS_E_HIP;
    }
    return GNS_OK;
}

}  // extern "C"

// Query (count_min.go:160-174) of n keys against state (C, Fc, S, Fs) on stream st:
// host keys / answers (staged through the grow-only scratch), or device keys /
// answers (dev: no copies; the call returns once the answers are written).
static int cm_query_impl(gns_cm *cm, hipStream_t st, CmScratch &sc, const uint32_t *C, const uint32_t *Fc,
                         const uint32_t *S, const uint32_t *Fs, const uint8_t *keys, uint32_t stride, uint64_t n,
                         uint64_t *out, bool dev = false) {
    if (!dev) {
        GNS_TRY(grow_buf(&sc.qkeys, sc.qkeys_n, n * stride));
        GNS_TRY(grow_buf(&sc.qout, sc.qout_n, n));
    }
    QueryArgs a{};
    a.keys = dev ? keys : sc.qkeys;
    a.stride = stride;
    a.aligned = (stride % 4 == 0 && stride >= ((cm->K + 3) & ~3u) && ((uintptr_t)a.keys & 3u) == 0);
    a.n = n; a.K = cm->K; a.g = cm->g; a.D = cm->D;
    a.C = C; a.Fc = Fc; a.S = S; a.Fs = Fs; a.out = dev ? out : sc.qout;
    hipError_t e = dev ? hipSuccess : hipMemcpyAsync(sc.qkeys, keys, n * stride, hipMemcpyHostToDevice, st);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_query, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a);
        e = hipGetLastError();
    }
    if (e == hipSuccess && !dev) e = hipMemcpyAsync(out, sc.qout, n * 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) { set_error("query: %s", hipGetErrorString(e)); return GNS_E_HIP; }
    return GNS_OK;
}

extern "C" {

int gns_cm_query(gns_cm *cm, const uint8_t *keys, uint32_t stride, uint64_t n, uint64_t *out) {
    if (!cm || (n && (!keys || !out))) { set_error("null argument"); return GNS_E_ARG; }
    if (n == 0) return GNS_OK;
    if (stride < cm->K) { set_error("stride < key_bytes"); return GNS_E_ARG; }
    GNS_TRY(set_dev(cm));
    return cm_query_impl(cm, cm->stream, cm->rd, cm->C, cm->Fc, cm->S, cm->Fs, keys, stride, n, out);
}

int gns_cm_query_device(gns_cm *cm, const uint8_t *keys, uint32_t stride, uint64_t n, uint64_t *out) {
    if (!cm || (n && (!keys || !out))) { set_error("null argument"); return GNS_E_ARG; }
    if (n == 0) return GNS_OK;
    if (stride < cm->K) { set_error("stride < key_bytes"); return GNS_E_ARG; }
    if (((uintptr_t)out & 7u) != 0) { set_error("answers not 8-byte aligned"); return GNS_E_ARG; }
    GNS_TRY(set_dev(cm));
    return cm_query_impl(cm, cm->stream, cm->rd, cm->C, cm->Fc, cm->S, cm->Fs, keys, stride, n, out, true);
}

// ids -> key bytes on stream `st`: through the grow-only scratch when small
// (heavy-hitter lists), a temporary buffer for whole-state exports.
static int cm_ids_to_host_bytes(gns_cm *cm, hipStream_t st, CmScratch &sc, const uint32_t *d_ids, uint64_t n,
                                uint8_t *host) {
    if (n == 0 || cm->K == 0) return GNS_OK;
    const uint64_t nb = n * cm->K;
    const bool tmp = nb > (64ull << 20);
    uint8_t *d = nullptr;
    if (tmp) GNS_TRY(dalloc(reinterpret_cast<void **>(&d), nb));
    else { GNS_TRY(grow_buf(&sc.bytes, sc.bytes_n, nb)); d = sc.bytes; }
    hipLaunchKernelGGL(k_ids_to_bytes, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, d_ids, n, cm->D, d);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipMemcpyAsync(host, d, nb, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (tmp) dfree(d);
    if (e != hipSuccess) { set_error("ids_to_bytes: %s", hipGetErrorString(e)); return GNS_E_HIP; }
    return GNS_OK;
}

int gns_cm_export_state(gns_cm *cm, uint32_t *C, uint32_t *S, uint8_t *FPc, uint8_t *FPs) {
    if (!cm) return GNS_E_ARG;
    GNS_TRY(set_dev(cm));
    GNS_HIP(hipStreamSynchronize(cm->stream));
    const uint64_t cells = (uint64_t)cm->g.d * cm->g.w;
    if (C) GNS_HIP(hipMemcpy(C, cm->C, cells * 4, hipMemcpyDeviceToHost));
    if (S) GNS_HIP(hipMemcpy(S, cm->S, cells * 4, hipMemcpyDeviceToHost));
    if (FPc) GNS_TRY(cm_ids_to_host_bytes(cm, cm->stream, cm->rd, cm->Fc, cells, FPc));
    if (FPs) GNS_TRY(cm_ids_to_host_bytes(cm, cm->stream, cm->rd, cm->Fs, cells, FPs));
    return GNS_OK;
}

// HeavyHitters (count_min.go:178-247): a flow's max over its buckets reaches the
// threshold iff one of its buckets does, so only cells >= threshold are
// candidates; dedupe by fingerprint keeping the max; sort value desc.
// the per-flow-id words cover every slot of the dictionary (zeroed when (re)allocated:
// the epochs of the calls start at 1); bump: a new call's epoch
static int heavy_flow_words(CmScratch &sc, uint64_t slots, hipStream_t st, bool bump) {
    if (sc.best_n < slots || !sc.best || sc.mark_n < slots || !sc.mark) {
        dfree(sc.best); dfree(sc.mark);
        sc.best = nullptr; sc.mark = nullptr; sc.best_n = sc.mark_n = 0;
        GNS_TRY(dalloc(reinterpret_cast<void **>(&sc.best), slots * 8));
        GNS_TRY(dalloc(reinterpret_cast<void **>(&sc.mark), slots * 4));
        sc.best_n = sc.mark_n = slots;
        GNS_HIP(hipMemsetAsync(sc.best, 0, slots * 8, st));
        GNS_HIP(hipMemsetAsync(sc.mark, 0, slots * 4, st));
        sc.hh_epoch = 0;
    }
    if (bump && ++sc.hh_epoch == 0) {  // wrapped: clear, restart at 1
        GNS_HIP(hipMemsetAsync(sc.best, 0, sc.best_n * 8, st));
        GNS_HIP(hipMemsetAsync(sc.mark, 0, sc.mark_n * 4, st));
        sc.hh_epoch = 1;
    }
    return GNS_OK;
}

// Read-side buffers of the heavy-hitter list sized up front (gns_cm_create /
// gns_cm_view_create), so a window's first call allocates nothing: candidates
// for min(cells, 4M) buckets, the per-flow words for the dictionary's slots,
// unique entries and their order for 1M flows.  Larger lists still grow them.
static int small_pin(CmScratch &sc) {
    if (!sc.hsm) GNS_HIP(hipHostMalloc(reinterpret_cast<void **>(&sc.hsm), 64, hipHostMallocDefault));
    return GNS_OK;
}

static int heavy_reserve(CmScratch &sc, uint64_t cells, uint64_t slots, uint32_t K, hipStream_t st) {
    GNS_TRY(heavy_flow_words(sc, slots, st, false));
    if (!sc.ncand) GNS_TRY(dalloc(reinterpret_cast<void **>(&sc.ncand), 16));
    if (!sc.cand) {
        const uint64_t want = std::min<uint64_t>(cells, 1ull << 22);
        GNS_TRY(dalloc(reinterpret_cast<void **>(&sc.cand), want * 8));
        sc.cap = want;
    }
    const uint64_t nu = std::min<uint64_t>(std::min(cells, slots), 1ull << 20);
    GNS_TRY(grow_buf(&sc.u32a, sc.u32a_n, nu / 2));
    GNS_TRY(grow_buf(&sc.u32b, sc.u32b_n, nu / 2 + 1));
    GNS_TRY(grow_buf(&sc.u32c, sc.u32c_n, nu));
    GNS_TRY(grow_buf(&sc.u32d, sc.u32d_n, nu / 2));
    GNS_TRY(grow_buf(&sc.bytes, sc.bytes_n, nu / 2 * std::max<uint32_t>(K, 1)));
    GNS_TRY(grow_buf(&sc.obytes, sc.obytes_n, nu / 2 * std::max<uint32_t>(K, 1)));
    if (!sc.hpin) {
        const uint64_t want = nu * (std::max<uint32_t>(K, 1) + 4);
        GNS_HIP(hipHostMalloc(reinterpret_cast<void **>(&sc.hpin), want, hipHostMallocDefault));
        sc.hpin_n = want;
    }
    // the order's pass histograms and the small pinned read-back words for nu entries too:
    // a window's first list then allocates nothing (an allocation inside one list call was
    // followed by an 18-36 ms dispatch stall of a LATER call, profiles/r06_hh_spikes.txt)
    const uint64_t nblk = (nu + kRsBlock - 1) / kRsBlock, ngrp = (nblk + kTGrp - 1) / kTGrp;
    GNS_TRY(grow_buf(&sc.rsh, sc.rsh_n, (nblk + ngrp + 1) * 256 + 4));
    return small_pin(sc);
}

// GNS_HH_TRACE=1: the heavy-hitter list's phases timed on stderr (each mark
// synchronizes the stream first; diagnostics only, never on by default).
struct HhTrace {
    bool on;
    hipStream_t st;
    std::chrono::steady_clock::time_point t;
    explicit HhTrace(hipStream_t s) : on(getenv("GNS_HH_TRACE") != nullptr), st(s), t(std::chrono::steady_clock::now()) {}
    void mark(const char *what, uint64_t n, bool sync = true) {
        if (!on) return;
        if (sync) (void)hipStreamSynchronize(st);
        const auto now = std::chrono::steady_clock::now();
        struct rusage ru;
        getrusage(RUSAGE_THREAD, &ru);
        fprintf(stderr, "[hh] %-12s n=%-9llu %8.3f ms  nivcsw=%ld nvcsw=%ld\n", what, (unsigned long long)n,
                std::chrono::duration<double, std::milli>(now - t).count(), ru.ru_nivcsw, ru.ru_nvcsw);
        t = now;
    }
};

// One stable LSD radix pass over perm (n entries) by digit r: in -> out.
static int rs_pass(CmScratch &sc, hipStream_t st, const uint32_t *in, uint32_t *out, uint32_t n, const RsDigit &r) {
    const uint32_t nblk = (n + kRsBlock - 1) / kRsBlock;
    const uint32_t ngrp = (nblk + kTGrp - 1) / kTGrp;
    uint32_t *hist = sc.rsh, *part = hist + (size_t)nblk * 256, *tot = part + (size_t)ngrp * 256, *total = tot + 256;
    hipLaunchKernelGGL(k_rs_hist, dim3(nblk), dim3(256), 0, st, in, n, r, hist);
    hipLaunchKernelGGL(k_tscan_part, dim3(1, ngrp), dim3(256), 0, st, hist, nblk, 256u, part);
    hipLaunchKernelGGL(k_tscan_mid, dim3(1), dim3(256), 0, st, part, ngrp, 256u, tot);
    hipLaunchKernelGGL(k_tscan_bins, dim3(1), dim3(1024), 0, st, tot, 256u, total);
    hipLaunchKernelGGL(k_tscan_down, dim3(1, ngrp), dim3(256), 0, st, hist, nblk, 256u, part, tot);
    hipLaunchKernelGGL(k_rs_scatter, dim3(nblk), dim3(256), 0, st, in, n, r, hist, tot, total, out);
    GNS_HIP(hipGetLastError());
    return GNS_OK;
}

// Canonical order of n entries of a device list (value desc, flow bytes asc) -> *perm_out
// (a device array of sc's): stable LSD radix passes by (value desc, key bytes 0..3), and by
// the whole key only when two neighbours tie on that.
static int hh_sort(CmScratch &sc, hipStream_t st, const HhSrc &src, uint32_t n, uint32_t **perm_out) {
    const unsigned g = (n + 255) / 256;
    const uint32_t K = src.K;
    GNS_TRY(grow_buf(&sc.u32c, sc.u32c_n, (uint64_t)n * 2));
    const uint32_t nblk = (n + kRsBlock - 1) / kRsBlock, ngrp = (nblk + kTGrp - 1) / kTGrp;
    GNS_TRY(grow_buf(&sc.rsh, sc.rsh_n, (uint64_t)(nblk + ngrp + 1) * 256 + 4));
    uint32_t *tie = sc.rsh + (size_t)(nblk + ngrp + 1) * 256 + 1;
    uint32_t *p[2] = {sc.u32c, sc.u32c + n};
    int cur = 0;
    // LSD: key bytes hi-1..0 (the last first), then the value (least significant byte first,
    // inverted: descending) -> (value desc, key bytes 0..hi-1 asc)
    auto sort_by = [&](uint32_t hi) -> int {
        hipLaunchKernelGGL(k_hh_iota, dim3(g), dim3(256), 0, st, p[0], n);
        cur = 0;
        RsDigit r{1, 0, src};
        for (int b = (int)hi - 1; b >= 0; b--) {
            r.b = (uint32_t)b;
            GNS_TRY(rs_pass(sc, st, p[cur], p[cur ^ 1], n, r));
            cur ^= 1;
        }
        r.mode = 0;
        for (uint32_t b = 0; b < 4; b++) {
            r.b = b;
            GNS_TRY(rs_pass(sc, st, p[cur], p[cur ^ 1], n, r));
            cur ^= 1;
        }
        return GNS_OK;
    };
    HhTrace tr(st);
    GNS_TRY(sort_by(std::min<uint32_t>(K, 4)));
    tr.mark("sort_primary", n);
    if (K > 4) {
        GNS_TRY(small_pin(sc));
        GNS_HIP(hipMemsetAsync(tie, 0, 4, st));
        hipLaunchKernelGGL(k_hh_ties, dim3(g), dim3(256), 0, st, p[cur], n, src, tie);
        GNS_HIP(hipMemcpyAsync(sc.hsm + 4, tie, 4, hipMemcpyDeviceToHost, st));
        GNS_HIP(hipStreamSynchronize(st));
        const uint32_t tflag = sc.hsm[4];
        tr.mark(tflag ? "ties:yes" : "ties:no", n);
        if (tflag) GNS_TRY(sort_by(K));  // the whole key: bytes K-1..0, then the value
        if (tflag) tr.mark("sort_full", n);
    }
    *perm_out = p[cur];
    return GNS_OK;
}

// rows_dev non-null: the ordered list as packed device rows [flow | u32 value] (capacity
// *n_io rows), no host copy; else flows / vals on the host.
// The list of one (value, fingerprint id) cell array of `cells` cells whose ids are
// slots of dictionary D: Count-Min's count and size lists, and SuperSpread's list
// (gns_ss.hip through gns::hh_heavy_list).
static int heavy_list(CmScratch &sc, hipStream_t st, const DictDev &Dd, uint64_t dict_slots, uint32_t K,
                      uint64_t cells, const uint32_t *val, const uint32_t *fp, uint32_t thr, uint8_t *flows,
                      uint32_t *vals, uint64_t *n_io, uint8_t *rows_dev = nullptr) {
    struct {
        uint64_t dict_slots;
        DictDev D;
    } cmv{dict_slots, Dd}, *cm = &cmv;
    HhTrace tr(st);
    GNS_TRY(heavy_reserve(sc, cells, cm->dict_slots, K, st));
    GNS_TRY(small_pin(sc));
    tr.mark("reserve", cells);
    // candidate buffer: grows to the number of cells at or above the threshold
    // (no cap: a low threshold can make every bucket a candidate, d*w < 2^32)
    uint32_t nc = 0;
    for (int pass = 0; pass < 2; pass++) {
        // [0] candidates, [1] unique, [2] bad-id flag: zeroed by a kernel on the list's stream
        tr.mark("pre_launch", 0, false);
        hipLaunchKernelGGL(k_fill_u32, dim3(1), dim3(64), 0, st, sc.ncand, (uint64_t)3, 0u);
        tr.mark("launched", 0, false);
        hipError_t e = hipGetLastError();
        if (e == hipSuccess) {
            hipLaunchKernelGGL(k_hh_candidates, dim3((unsigned)((cells + 256 * kHhItems - 1) / (256 * kHhItems))), dim3(256), 0,
                               st, val, fp, cells, thr, sc.cand, sc.ncand, (uint32_t)sc.cap);
            e = hipGetLastError();
        }
        tr.mark("cand_kernel", cells);
        if (e == hipSuccess) e = hipMemcpyAsync(sc.hsm, sc.ncand, 4, hipMemcpyDeviceToHost, st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) { set_error("heavy: %s", hipGetErrorString(e)); return GNS_E_HIP; }
        nc = sc.hsm[0];
        tr.mark("candidates", nc);
        if (nc <= sc.cap) break;
        // more candidates than the buffer holds: grow to the count and run again
        dfree(sc.cand);
        sc.cand = nullptr;
        sc.cap = 0;
        const uint64_t want = std::min<uint64_t>(cells, (uint64_t)nc + nc / 8);
        GNS_TRY(dalloc(reinterpret_cast<void **>(&sc.cand), want * 8));
        sc.cap = want;
    }
    const uint64_t *cand = sc.cand;
    // on the device: the max per flow over its buckets, one entry per flow
    uint32_t nu = 0;
    if (nc) {
        const unsigned g = (nc + 255) / 256;
        GNS_TRY(heavy_flow_words(sc, cm->dict_slots, st, true));
        GNS_TRY(grow_buf(&sc.u32a, sc.u32a_n, nc));
        GNS_TRY(grow_buf(&sc.u32b, sc.u32b_n, nc + 1));
        uint32_t *d_nu = sc.ncand + 1, *d_bad = sc.ncand + 2;
        const uint64_t slots = cm->dict_slots;
        hipLaunchKernelGGL(k_hh_best, dim3(g), dim3(256), 0, st, cand, nc, sc.best, sc.hh_epoch, slots, d_bad);
        hipLaunchKernelGGL(k_hh_emit, dim3(g), dim3(256), 0, st, cand, nc, sc.best, sc.mark, sc.hh_epoch, slots,
                           sc.u32a, sc.u32b, d_nu);
        GNS_HIP(hipGetLastError());
        GNS_HIP(hipMemcpyAsync(sc.hsm + 1, d_nu, 8, hipMemcpyDeviceToHost, st));
        GNS_HIP(hipStreamSynchronize(st));
        nu = sc.hsm[1];
        if (sc.hsm[2]) {
            set_error("heavy hitters: a bucket fingerprint names no dictionary slot (corrupt state)");
            return GNS_E_HIP;
        }
        tr.mark("dedupe", nu);
    }
    const uint64_t capn = *n_io;
    *n_io = nu;
    if (nu) {
        const unsigned g = (nu + 255) / 256;
        const uint32_t Kb = K ? K : 1;
        GNS_TRY(grow_buf(&sc.bytes, sc.bytes_n, (uint64_t)nu * Kb));
        GNS_TRY(grow_buf(&sc.obytes, sc.obytes_n, (uint64_t)nu * Kb));
        GNS_TRY(grow_buf(&sc.u32d, sc.u32d_n, (uint64_t)nu));
        tr.mark("grow", nu);
        if (K) hipLaunchKernelGGL(k_ids_to_bytes, dim3(g), dim3(256), 0, st, sc.u32a, (uint64_t)nu, cm->D, sc.bytes);
        tr.mark("ids_to_bytes", nu);
        const HhSrc src{sc.u32b, sc.bytes, K, K};
        uint32_t *perm = nullptr;
        GNS_TRY(hh_sort(sc, st, src, nu, &perm));
        tr.mark("sorted", nu);
        if (rows_dev) {
            if (nu <= capn) {
                hipLaunchKernelGGL(k_hh_gather, dim3(g), dim3(256), 0, st, perm, src, nu, nullptr, nullptr, rows_dev);
                GNS_HIP(hipGetLastError());
                GNS_HIP(hipStreamSynchronize(st));
            }
            return GNS_OK;
        }
        hipLaunchKernelGGL(k_hh_gather, dim3(g), dim3(256), 0, st, perm, src, nu, sc.obytes, sc.u32d, nullptr);
        GNS_HIP(hipGetLastError());
        const uint64_t m = std::min<uint64_t>(nu, capn);
        const uint64_t fb = (flows && K) ? m * K : 0, vb = vals ? m * 4 : 0;
        if (fb + vb > sc.hpin_n) {
            if (sc.hpin) (void)hipHostFree(sc.hpin);
            sc.hpin = nullptr; sc.hpin_n = 0;
            const uint64_t want = 2 * (fb + vb);
            GNS_HIP(hipHostMalloc(reinterpret_cast<void **>(&sc.hpin), want, hipHostMallocDefault));
            sc.hpin_n = want;
        }
        if (fb) GNS_HIP(hipMemcpyAsync(sc.hpin, sc.obytes, fb, hipMemcpyDeviceToHost, st));
        if (vb) GNS_HIP(hipMemcpyAsync(sc.hpin + fb, sc.u32d, vb, hipMemcpyDeviceToHost, st));
        GNS_HIP(hipStreamSynchronize(st));
        tr.mark("gather_d2h", m);
        if (fb) memcpy(flows, sc.hpin, fb);
        if (vb) memcpy(vals, sc.hpin + fb, vb);
        tr.mark("host_copy", m);
    }
    return GNS_OK;
}

static int cm_heavy_one(gns_cm *cm, hipStream_t st, CmScratch &sc, const uint32_t *val, const uint32_t *fp,
                        uint32_t thr, uint8_t *flows, uint32_t *vals, uint64_t *n_io, uint8_t *rows_dev = nullptr) {
    return heavy_list(sc, st, cm->D, cm->dict_slots, cm->K, (uint64_t)cm->g.d * cm->g.w, val, fp, thr, flows, vals,
                      n_io, rows_dev);
}

}  // extern "C"

namespace gns {
CmScratch *hh_scratch_new() { return new CmScratch(); }
void hh_scratch_free(CmScratch *sc) {
    if (!sc) return;
    sc->free_all();
    delete sc;
}
int hh_heavy_list(CmScratch *sc, hipStream_t st, const DictDev &D, uint64_t dict_slots, uint32_t K, uint64_t cells,
                  const uint32_t *val, const uint32_t *fp, uint32_t thr, uint8_t *flows, uint32_t *vals,
                  uint64_t *n_io) {
    return heavy_list(*sc, st, D, dict_slots, K, cells, val, fp, thr, flows, vals, n_io);
}
}  // namespace gns

extern "C" {

int gns_cm_heavy_hitters(gns_cm *cm, uint8_t *count_flows, uint32_t *counts, uint64_t *n_count,
                         uint8_t *size_flows, uint32_t *sizes, uint64_t *n_size) {
    if (!cm || !n_count || !n_size) { set_error("null argument"); return GNS_E_ARG; }
    GNS_TRY(set_dev(cm));
    GNS_HIP(hipStreamSynchronize(cm->stream));
    GNS_TRY(cm_heavy_one(cm, cm->stream, cm->rd, cm->C, cm->Fc, cm->ct, count_flows, counts, n_count));
    GNS_TRY(cm_heavy_one(cm, cm->stream, cm->rd, cm->S, cm->Fs, cm->st, size_flows, sizes, n_size));
    return GNS_OK;
}

int gns_cm_heavy_rows(gns_cm *cm, uint8_t *count_rows, uint64_t *n_count, uint8_t *size_rows, uint64_t *n_size) {
    if (!cm || !n_count || !n_size || (*n_count && !count_rows) || (*n_size && !size_rows)) {
        set_error("null argument"); return GNS_E_ARG;
    }
    GNS_TRY(set_dev(cm));
    GNS_HIP(hipStreamSynchronize(cm->stream));
    uint8_t dummy_c = 0, dummy_s = 0;  // a zero-capacity call only reports the lengths
    GNS_TRY(cm_heavy_one(cm, cm->stream, cm->rd, cm->C, cm->Fc, cm->ct, nullptr, nullptr, n_count,
                         count_rows ? count_rows : &dummy_c));
    GNS_TRY(cm_heavy_one(cm, cm->stream, cm->rd, cm->S, cm->Fs, cm->st, nullptr, nullptr, n_size,
                         size_rows ? size_rows : &dummy_s));
    return GNS_OK;
}

// per device, per host thread: the sort scratch of gns_hh_order_rows (grow-only; it lives as long
// as the thread -- freeing device memory from a thread-exit destructor could run after the HIP
// runtime's own teardown at process exit)
static thread_local std::vector<CmScratch *> t_hh_scratch;

int gns_hh_order_rows(const uint8_t *rows, uint32_t key_bytes, uint64_t n, uint8_t *out_rows, int device) {
    if ((n && (!rows || !out_rows)) || key_bytes > 37) { set_error("bad argument"); return GNS_E_ARG; }
    if (n >= (1ull << 31)) { set_error("%llu rows (max 2^31 - 1)", (unsigned long long)n); return GNS_E_RANGE; }
    if (n == 0) return GNS_OK;
    (void)hipGetLastError();
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
        (void)hipGetLastError(); set_error("device %d not available", device); return GNS_E_NODEV;
    }
    GNS_HIP(hipSetDevice(device));
    if ((int)t_hh_scratch.size() <= device) t_hh_scratch.resize(device + 1, nullptr);
    if (!t_hh_scratch[device]) t_hh_scratch[device] = new CmScratch();
    CmScratch &sc = *t_hh_scratch[device];
    hipStream_t st = nullptr;  // the legacy stream: ordered after the caller's device writes
    const HhSrc src{nullptr, rows, key_bytes, key_bytes + 4};
    uint32_t *perm = nullptr;
    GNS_TRY(hh_sort(sc, st, src, (uint32_t)n, &perm));
    hipLaunchKernelGGL(k_hh_gather, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, perm, src, (uint32_t)n,
                       nullptr, nullptr, out_rows);
    GNS_HIP(hipGetLastError());
    GNS_HIP(hipStreamSynchronize(st));
    return GNS_OK;
}

// ---------------------------------------------------------------------------
// Snapshot views: heavy hitters and queries concurrent with ingest
// (BASELINE configs[4]; the reference's snapshotter reads the live buckets
// while workers insert, manager.go:139-159 -- here the read side sees a
// consistent state taken at a point of the insert stream instead).
// ---------------------------------------------------------------------------
static void view_free(gns_cm_view *v) {
    dfree(v->C); dfree(v->S); dfree(v->Fc); dfree(v->Fs);
    v->rd.free_all();
    if (v->ready) (void)hipEventDestroy(v->ready);
    if (v->stream) (void)hipStreamDestroy(v->stream);
}

int gns_cm_view_create(gns_cm *cm, gns_cm_view **out) {
    if (!cm || !out) { set_error("null argument"); return GNS_E_ARG; }
    *out = nullptr;
    GNS_TRY(set_dev(cm));
    gns_cm_view *v = new gns_cm_view();
    v->cm = cm;
    const uint64_t cells = (uint64_t)cm->g.d * cm->g.w;
    int rc = GNS_OK;
    do {
        if ((rc = dalloc_t(&v->C, cells)) || (rc = dalloc_t(&v->S, cells)) || (rc = dalloc_t(&v->Fc, cells)) ||
            (rc = dalloc_t(&v->Fs, cells)))
            break;
        // high priority: the read side's small launches are dispatched ahead of the
        // ingest pipeline's queued workgroups (query latency under load)
        int lo_pri = 0, hi_pri = 0;
        (void)hipDeviceGetStreamPriorityRange(&lo_pri, &hi_pri);
        if (hipStreamCreateWithPriority(&v->stream, hipStreamNonBlocking, hi_pri) != hipSuccess ||
            hipEventCreateWithFlags(&v->ready, hipEventDisableTiming) != hipSuccess) {
            set_error("view stream/event"); rc = GNS_E_HIP; break;
        }
        if ((rc = heavy_reserve(v->rd, cells, cm->dict_slots, cm->K, v->stream)) != GNS_OK) break;
        if (hipStreamSynchronize(v->stream) != hipSuccess) { set_error("view sync"); rc = GNS_E_HIP; break; }
    } while (0);
    if (rc) { view_free(v); delete v; return rc; }
    {
        std::lock_guard<std::mutex> reg(cm->views_mu);
        cm->views.push_back(v);
    }
    *out = v;
    return GNS_OK;
}

int gns_cm_view_destroy(gns_cm_view *v) {
    if (!v) return GNS_OK;
    gns_cm *cm = v->cm;
    (void)hipSetDevice(cm->device);
    {
        std::lock_guard<std::mutex> reg(cm->views_mu);
        cm->views.erase(std::remove(cm->views.begin(), cm->views.end(), v), cm->views.end());
    }
    {   // wait for a view call in progress; the mutex is released before the delete
        std::lock_guard<std::mutex> lk(v->mu);
        if (v->stream) (void)hipStreamSynchronize(v->stream);
    }
    view_free(v);
    delete v;
    return GNS_OK;
}

int gns_cm_view_refresh(gns_cm_view *v) {
    if (!v) { set_error("null argument"); return GNS_E_ARG; }
    gns_cm *cm = v->cm;
    GNS_TRY(set_dev(cm));
    std::lock_guard<std::mutex> lk(v->mu);  // no view query is reading the snapshot
    const uint64_t bytes = (uint64_t)cm->g.d * cm->g.w * 4;
    // copies on the handle's stream: the snapshot is the state after every insert
    // issued so far and before any later one; the view's stream waits for it
    GNS_HIP(hipMemcpyAsync(v->C, cm->C, bytes, hipMemcpyDeviceToDevice, cm->stream));
    GNS_HIP(hipMemcpyAsync(v->S, cm->S, bytes, hipMemcpyDeviceToDevice, cm->stream));
    GNS_HIP(hipMemcpyAsync(v->Fc, cm->Fc, bytes, hipMemcpyDeviceToDevice, cm->stream));
    GNS_HIP(hipMemcpyAsync(v->Fs, cm->Fs, bytes, hipMemcpyDeviceToDevice, cm->stream));
    GNS_HIP(hipEventRecord(v->ready, cm->stream));
    GNS_HIP(hipStreamWaitEvent(v->stream, v->ready, 0));
    v->period = cm->period.load();
    return GNS_OK;
}

static int view_check(gns_cm_view *v) {
    if (v->period == ~0u) { set_error("view never refreshed"); return GNS_E_ARG; }
    if (v->period != v->cm->period.load()) { set_error("view is stale: the handle was reset; refresh it"); return GNS_E_ARG; }
    return GNS_OK;
}

int gns_cm_view_heavy_hitters(gns_cm_view *v, uint8_t *count_flows, uint32_t *counts, uint64_t *n_count,
                              uint8_t *size_flows, uint32_t *sizes, uint64_t *n_size) {
    if (!v || !n_count || !n_size) { set_error("null argument"); return GNS_E_ARG; }
    gns_cm *cm = v->cm;
    GNS_TRY(set_dev(cm));
    std::lock_guard<std::mutex> lk(v->mu);
    GNS_TRY(view_check(v));
    GNS_TRY(cm_heavy_one(cm, v->stream, v->rd, v->C, v->Fc, cm->ct, count_flows, counts, n_count));
    GNS_TRY(cm_heavy_one(cm, v->stream, v->rd, v->S, v->Fs, cm->st, size_flows, sizes, n_size));
    return GNS_OK;
}

int gns_cm_view_query(gns_cm_view *v, const uint8_t *keys, uint32_t stride, uint64_t n, uint64_t *out) {
    if (!v || (n && (!keys || !out))) { set_error("null argument"); return GNS_E_ARG; }
    if (n == 0) return GNS_OK;
    gns_cm *cm = v->cm;
    if (stride < cm->K) { set_error("stride < key_bytes"); return GNS_E_ARG; }
    GNS_TRY(set_dev(cm));
    std::lock_guard<std::mutex> lk(v->mu);
    GNS_TRY(view_check(v));
    return cm_query_impl(cm, v->stream, v->rd, v->C, v->Fc, v->S, v->Fs, keys, stride, n, out);
}

int gns_cm_reset(gns_cm *cm) {
    if (!cm) return GNS_E_ARG;
    GNS_TRY(set_dev(cm));
    // a view call that passed its period check still reads the dictionary: wait
    // for it before the dictionary is cleared (views answer GNS_E_ARG afterwards)
    ViewsQuiesced q(cm);
    cm->period.fetch_add(1);
    GNS_TRY(cm_reset_state(cm));
    GNS_HIP(hipStreamSynchronize(cm->stream));
    return GNS_OK;
}

int gns_cm_stats(gns_cm *cm, uint64_t stats[4]) {
    if (!cm || !stats) return GNS_E_ARG;
    GNS_TRY(set_dev(cm));
    GNS_HIP(hipStreamSynchronize(cm->stream));
    unsigned long long h[8];
    GNS_HIP(hipMemcpy(h, cm->stats, sizeof(h), hipMemcpyDeviceToHost));
    stats[0] = h[0]; stats[1] = h[1]; stats[2] = h[2];
    // distinct flows = occupied dictionary slots
    std::vector<uint32_t> tags;
    uint64_t occ = 0;
    const uint64_t chunk = 1 << 20;
    std::vector<uint32_t> buf;
    for (uint64_t s0 = 0; s0 < cm->dict_slots; s0 += chunk) {
        const uint64_t m = std::min(chunk, cm->dict_slots - s0);
        buf.resize(m * cm->D.RW);
        GNS_HIP(hipMemcpy(buf.data(), cm->D.rec + s0 * cm->D.RW, m * cm->D.RW * 4, hipMemcpyDeviceToHost));
        for (uint64_t i = 0; i < m; i++) occ += buf[i * cm->D.RW] != 0;
    }
    stats[3] = occ;
    return GNS_OK;
}

int gns_cm_counters(gns_cm *cm, uint64_t out[8]) {
    if (!cm || !out) return GNS_E_ARG;
    GNS_TRY(set_dev(cm));
    GNS_HIP(hipStreamSynchronize(cm->stream));
    unsigned long long h[kStatsProf + 16];
    GNS_HIP(hipMemcpy(h, cm->stats, sizeof(h), hipMemcpyDeviceToHost));
#if defined(GNS_SP_PROF)  // profiling build: k_apply_sparse phase cycles (SP_MARK order), chunks
    for (int i = 0; i < 7; i++) out[i] = h[kStatsProf + i];
    out[7] = h[6];
    return GNS_OK;
#endif
#ifdef GNS_K3_PROF  // profiling build: K3 phase cycles (loads, rank, scan, stage, write)
    for (int i = 0; i < 5; i++) out[i] = h[kStatsProf + i];
    for (int i = 5; i < 8; i++) out[i] = h[i];
    return GNS_OK;
#endif
#ifdef GNS_K4_PROF  // profiling build: K4 phase cycles (classify, decide, compact, replay, tile load,
                    // tile store, sub-partition), chunks
    // phases (classify, decide, compact, replay barrier + loop top, replay gather, tile load +
    // store, replay groups), then the slowest wave's and the summed per-wave replay cycles
    for (int i = 0; i < 4; i++) out[i] = h[kStatsProf + i];
    out[4] = h[kStatsProf + 9];
    out[5] = h[kStatsProf + 5];
    out[6] = h[kStatsProf + 8];
    out[7] = h[kStatsProf + 6];
#else
    for (int i = 0; i < 8; i++) out[i] = h[i];
#endif
    return GNS_OK;
}

int gns_cm_reclaim(gns_cm *cm) {
    if (!cm) return GNS_E_ARG;
    GNS_TRY(set_dev(cm));
    return cm_reclaim(cm);
}

int gns_cm_dict_stats(gns_cm *cm, uint64_t out[8]) {
    if (!cm || !out) return GNS_E_ARG;
    out[0] = cm->n_reclaim; out[1] = cm->n_dropped; out[2] = cm->last_live; out[3] = cm->claimed;
    out[4] = (uint64_t)(cm->reclaim_ms * 1000.0); out[5] = cm->n_retry;
    out[6] = cm->dict_slots; out[7] = cm->n_grow;
    return GNS_OK;
}

int gns_cm_set_timing(gns_cm *cm, int on) {
    if (!cm) return GNS_E_ARG;
    set_timing_arg(cm->timer, on);
    return GNS_OK;
}

int gns_cm_stage_times(gns_cm *cm, double ms[8], uint64_t launches[8], int reset) {
    if (!cm) return GNS_E_ARG;
    GNS_TRY(set_dev(cm));
    cm->timer.collect();
    for (int i = 0; i < 8; i++) {
        if (ms) ms[i] = cm->timer.ms[i];
        if (launches) launches[i] = cm->timer.launches[i];
    }
    if (reset) {
        for (int i = 0; i < 8; i++) { cm->timer.ms[i] = 0; cm->timer.launches[i] = 0; }
    }
    return GNS_OK;
}

void *gns_cm_stream(gns_cm *cm) { return cm ? (void *)cm->stream : nullptr; }

}  // extern "C"
