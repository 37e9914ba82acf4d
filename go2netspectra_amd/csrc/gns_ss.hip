// gns_ss.hip -- MI355X engine for Go2NetSpectra's SuperSpread
// (internal/engine/impl/sketch/statistic/super_spread.go).
//
// Semantics: the device state equals super_spread.go fed the same packets in
// the same order by ONE worker, with each GeneralHLL's seeds[0..1] derived from
// a master seed and rand.Float64() replaced by the declared counter-based
// generator ss_uniform(rng_seed, packet, row, draw).
//
// What is order-dependent, and how it is made parallel:
//   * HLL register updates (:90-103): a packet "encodes" iff its geometric
//     value lz exceeds the register's value at its time, i.e. the exclusive
//     prefix max of earlier updates to the same (cell, register).  Only
//     packets with lz > the batch-entry register can encode (registers only
//     grow): they are emitted as candidates, partitioned by cell bins and, per
//     bin, radix-sorted by (cell, register, packet) in LDS, where a segmented
//     max gives every candidate the register value it would see (k_sp_*).
//   * pbits (:105-109) and the sampled majority-vote counter (:200-233) are
//     sequential per cell: the successful encodes (at most maxValue per
//     register per batch, sparse) are sorted by (cell, packet) in the same LDS
//     pass and every cell is walked in stream order by one lane.
#include <cstdlib>
#include <cstring>

#include <algorithm>
#include <chrono>
#include <vector>

#include "gns_common.hpp"
#include "gns_ctl.cuh"
#include "gns_gomath.cuh"
#include "gns_hh.hpp"
#include "gns_scan.cuh"

namespace gns {

constexpr int kSsNW = 20;             // merged key words (flow ‖ elem <= 74 bytes)
constexpr uint32_t kSsPktBits = 27;   // packet index bits in the sort keys (batch <= 2^27)
constexpr int kSsThreads = 256;
constexpr uint32_t kSsChunk = 16384;
constexpr uint32_t kSsIdChunk = 1024;  // S3b encodes per workgroup (4 per lane: many short-lived waves)

struct SsGeom {
    uint32_t d, w, wmask, pow2, m, maxv, Kf, Km;
    uint32_t seeds[8];
    uint64_t hll_master, rng_seed;
    double base, b;
};

__device__ __forceinline__ uint32_t ss_row_index(const SsGeom &g, uint32_t h) {
    return g.pow2 ? (h & g.wmask) : (h % g.w);  // super_spread.go:193 `% ss.w`
}

struct SsExtractArgs {
    InputDesc in;
    uint64_t n;
    KeyPlanN kpf, kpm;
    SsGeom g;
    const uint8_t *regs;
    uint64_t *ckey;     // candidates: (cell*m + reg) << 27 | packet, block regions of chunk*d
    uint32_t *cval;     // lz
    uint32_t *cblk;     // [nblk]: candidates per block (in the block's own region)
    unsigned long long *stats;  // 0 inserted, 1 dropped, 2 unsupported, 3 dict full, 4 candidates, 5 encodes
};

// one wave-aggregated atomic for every lane that wants a slot (call convergently)
__device__ __forceinline__ uint32_t wave_alloc(uint32_t *ctr, bool want) {
    const uint64_t m = __ballot(want);
    if (m == 0) return 0;
    const uint32_t lane = __lane_id();
    const int leader = __ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if ((int)lane == leader) base = atomicAdd(ctr, (uint32_t)__popcll(m));
    base = __shfl(base, leader);
    return base + (uint32_t)__popcll(m & ((1ull << lane) - 1));
}

// flow key (kwf) and merged key flow‖elem (kwm) of packet p.  MF/MM: plan
// modes of the flow and merged layouts (SLICE0 for SrcIP / SrcIP‖DstIP).
template <int KIND, int MF, int MM, int KF = 0, int KM = 0>
__device__ __forceinline__ int ss_keys(const SsExtractArgs &a, const uint8_t *s_srcf, const uint8_t *s_srcm,
                                       uint64_t p, uint32_t (&kwf)[GNS_KWMAX], uint32_t (&kwm)[kSsNW]) {
    const uint32_t Kf = KF ? (uint32_t)KF : a.g.Kf, Km = KM ? (uint32_t)KM : a.g.Km;
    if constexpr (KIND == IN_KEYS) {
        const uint8_t *f = a.in.keys + p * a.in.stride;
        const uint8_t *e = a.in.keys2 + p * a.in.stride2;
        load_key_bytes<GNS_KWMAX>(f, a.g.Kf, false, kwf);
#pragma unroll
        for (int i = 0; i < kSsNW; i++) {
            uint32_t v = 0;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const uint32_t j = 4 * i + b;
                uint32_t byte = 0;
                if (j < a.g.Kf) byte = f[j];
                else if (j < a.g.Km) byte = e[j - a.g.Kf];
                v |= byte << (8 * b);
            }
            kwm[i] = v;
        }
        return PARSE_OK;
    } else {
        uint32_t tw[10];
        const int st = load_tuple<KIND>(a.in, p, tw);
        if (st != PARSE_OK) return st;
        make_key_m<MF, GNS_KWMAX>(Kf, s_srcf, tw, kwf);
        make_key_m<MM, kSsNW>(Km, s_srcm, tw, kwm);
        return PARSE_OK;
    }
}

// S1: keys, flow id, per-row HLL encode test against the batch-entry registers
// KF/KM: flow / merged key bytes when known at compile time (16/32 for the
// default task SrcIP / SrcIP|DstIP), 0 = runtime.
template <int KIND, int MF, int MM, int KF, int KM>
__global__ __launch_bounds__(kSsThreads) void k_ss_extract(SsExtractArgs a) {
    const uint32_t Kf = KF ? (uint32_t)KF : a.g.Kf, Km = KM ? (uint32_t)KM : a.g.Km;
    const uint32_t mmask = a.g.m - 1u;
    const bool mpow2 = (a.g.m & mmask) == 0;
    __shared__ uint8_t s_srcf[80], s_srcm[80];
    __shared__ uint32_t s_drop, s_unsup, s_ok, s_cc;
    const uint32_t tid = threadIdx.x, blk = blockIdx.x;
    for (uint32_t j = tid; j < 80; j += kSsThreads) { s_srcf[j] = a.kpf.src[j]; s_srcm[j] = a.kpm.src[j]; }
    if (tid == 0) { s_drop = 0; s_unsup = 0; s_ok = 0; s_cc = 0; }
    __syncthreads();
    const uint64_t beg = (uint64_t)blk * kSsChunk;
    const uint64_t end = min(a.n, beg + kSsChunk);
    uint64_t *rkey = a.ckey + beg * a.g.d;  // this block's candidate region (never overflows)
    uint32_t *rval = a.cval + beg * a.g.d;
    uint32_t n_ok = 0;
    for (uint64_t p = beg + tid; p < end; p += kSsThreads) {
        uint32_t kwf[GNS_KWMAX], kwm[kSsNW];
        const int st = ss_keys<KIND, MF, MM, KF, KM>(a, s_srcf, s_srcm, p, kwf, kwm);
        if (st != PARSE_OK) {
            atomicAdd(st == PARSE_DROP ? &s_drop : &s_unsup, 1u);
            continue;
        }
        uint32_t mkf[GNS_KWMAX], mkm[kSsNW];
        mm3_premix<GNS_KWMAX>(kwf, Kf, mkf);
        mm3_premix<kSsNW>(kwm, Km, mkm);
        n_ok++;
        for (uint32_t rr = 0; rr < a.g.d; rr++) {
            const uint32_t j = ss_row_index(a.g, mm3_chain<GNS_KWMAX>(mkf, Kf, a.g.seeds[rr]));
            const uint64_t cell = (uint64_t)rr * a.g.w + j;
            uint32_t s0, s1;
            ss_hll_seeds(a.g.hll_master, cell, s0, s1);
            const uint32_t h0 = mm3_chain<kSsNW>(mkm, Km, s0);  // geometricHash :66-70
            uint32_t lz = (h0 ? (uint32_t)__clz(h0) : 32u) + 1u;
            if (lz > a.g.maxv) lz = a.g.maxv;
            const uint32_t h1 = mm3_chain<kSsNW>(mkm, Km, s1);
            const uint32_t idx = mpow2 ? (h1 & mmask) : h1 % a.g.m;  // :87-88
            const uint64_t seg = cell * a.g.m + idx;
            const bool want = lz > a.regs[seg];  // can encode only if above the batch-entry register
            const uint32_t q = wave_alloc(&s_cc, want);
            if (want) {
                rkey[q] = seg << kSsPktBits | (p & ((1ull << kSsPktBits) - 1));
                rval[q] = lz;
            }
        }
    }
    atomicAdd(&s_ok, n_ok);
    __syncthreads();
    if (tid == 0) {
        a.cblk[blk] = s_cc;
        if (s_cc) atomicAdd(&a.stats[4], (unsigned long long)s_cc);
        if (s_ok) atomicAdd(&a.stats[0], (unsigned long long)s_ok);
        if (s_drop) atomicAdd(&a.stats[1], (unsigned long long)s_drop);
        if (s_unsup) atomicAdd(&a.stats[2], (unsigned long long)s_unsup);
    }
}

// S1 for header records with compile-time key widths and depth (the default
// task: SrcIP / SrcIP|DstIP, d=2): the same per-packet work as k_ss_extract,
// as a two-stage software pipeline.  Iteration k parses packet k+1, hashes
// its keys and issues its d batch-entry register reads (and prefetches the
// record of packet k+2), then emits the candidates of packet k, whose register
// reads were issued one iteration earlier.  Results are identical: candidates
// carry (segment, packet) and are radix-sorted afterwards, so their order in
// the block region does not matter.
#ifndef GNS_SS_MINW
#define GNS_SS_MINW 4
#endif
template <int MF, int MM, int KF, int KM, int DD>
__global__ __launch_bounds__(kSsThreads, GNS_SS_MINW) void k_ss_extract_hdr(SsExtractArgs a) {
    const uint32_t mmask = a.g.m - 1u;
    const bool mpow2 = (a.g.m & mmask) == 0;
    __shared__ uint8_t s_srcf[80], s_srcm[80];
    __shared__ uint32_t s_drop, s_unsup, s_ok, s_cc;
    const uint32_t tid = threadIdx.x, blk = blockIdx.x;
    for (uint32_t j = tid; j < 80; j += kSsThreads) { s_srcf[j] = a.kpf.src[j]; s_srcm[j] = a.kpm.src[j]; }
    if (tid == 0) { s_drop = 0; s_unsup = 0; s_ok = 0; s_cc = 0; }
    __syncthreads();
    const uint64_t beg = (uint64_t)blk * kSsChunk;
    const uint64_t end = min(a.n, beg + kSsChunk);
    uint64_t *rkey = a.ckey + beg * a.g.d;
    uint32_t *rval = a.cval + beg * a.g.d;
    uint32_t n_ok = 0;
    uint4 hv[4];
    uint32_t hsz;
    auto load_hdr = [&](uint64_t q) {
        const uint64_t pc = min(q, end - 1);
        const uint4 *r = reinterpret_cast<const uint4 *>(a.in.hdr + pc * 16);
#pragma unroll
        for (int i = 0; i < 4; i++) hv[i] = r[i];
        hsz = a.in.sizes[pc];
    };
    // stage B of packet q: parse, keys, row cells, register reads
    auto stage_b = [&](uint64_t q, bool &okq, uint64_t (&segq)[DD], uint32_t (&lzq)[DD], uint32_t (&regq)[DD]) {
        okq = q < end;
        uint32_t cw[16];
#pragma unroll
        for (int i = 0; i < 4; i++) { cw[4 * i] = hv[i].x; cw[4 * i + 1] = hv[i].y; cw[4 * i + 2] = hv[i].z; cw[4 * i + 3] = hv[i].w; }
        const uint32_t szq = hsz;
        load_hdr(q + kSsThreads);
        uint32_t kwf[GNS_KWMAX], kwm[kSsNW], tw[10];
#pragma unroll
        for (int i = 0; i < GNS_KWMAX; i++) kwf[i] = 0;
#pragma unroll
        for (int i = 0; i < kSsNW; i++) kwm[i] = 0;
#pragma unroll
        for (int i = 0; i < 10; i++) tw[i] = 0;
        if (okq) {
            const int st = parse_record_fast(cw, szq, true, tw);
            if (st == PARSE_OK) {
                make_key_m<MF, GNS_KWMAX>(KF, s_srcf, tw, kwf);
                make_key_m<MM, kSsNW>(KM, s_srcm, tw, kwm);
            } else {
                atomicAdd(st == PARSE_DROP ? &s_drop : &s_unsup, 1u);
                okq = false;
            }
        }
        auto rows = [&](const uint32_t (&mkf)[GNS_KWMAX], const uint32_t (&mkm)[kSsNW]) {
#pragma unroll
            for (int rr = 0; rr < DD; rr++) {
                const uint32_t j = ss_row_index(a.g, mm3_chain<GNS_KWMAX>(mkf, KF, a.g.seeds[rr]));
                const uint64_t cell = (uint64_t)rr * a.g.w + j;
                uint32_t s0, s1;
                ss_hll_seeds(a.g.hll_master, cell, s0, s1);
                const uint32_t h0 = mm3_chain<kSsNW>(mkm, KM, s0);  // geometricHash :66-70
                uint32_t lz = (h0 ? (uint32_t)__clz(h0) : 32u) + 1u;
                lzq[rr] = lz > a.g.maxv ? a.g.maxv : lz;
                const uint32_t h1 = mm3_chain<kSsNW>(mkm, KM, s1);
                const uint32_t idx = mpow2 ? (h1 & mmask) : h1 % a.g.m;  // :87-88
                segq[rr] = cell * a.g.m + idx;
                regq[rr] = okq ? (uint32_t)a.regs[segq[rr]] : 0xFFu;
            }
        };
        uint32_t mkf[GNS_KWMAX], mkm[kSsNW];
        // the default task's keys are the source / source and destination 16-byte
        // address slots (PLAN_SLICE0): when every lane of the wave holds IPv4
        // addresses, 12 of the 16 key words are zero, and with the zeros as
        // constants their mixing and chain steps fold away (same hash values)
        const bool wide = okq && (tw[1] | tw[2] | tw[3] | tw[5] | tw[6] | tw[7]) != 0;
        if (MF == PLAN_SLICE0 && MM == PLAN_SLICE0 && KF == 16 && KM == 32 && __ballot(wide) == 0) {  // wave-uniform
            uint32_t kf4[GNS_KWMAX], km4[kSsNW];
#pragma unroll
            for (int i = 0; i < GNS_KWMAX; i++) kf4[i] = 0;
#pragma unroll
            for (int i = 0; i < kSsNW; i++) km4[i] = 0;
            kf4[0] = kwf[0];
            km4[0] = kwm[0];
            km4[4] = kwm[4];
            mm3_premix<GNS_KWMAX>(kf4, KF, mkf);
            mm3_premix<kSsNW>(km4, KM, mkm);
            rows(mkf, mkm);
        } else {
            mm3_premix<GNS_KWMAX>(kwf, KF, mkf);
            mm3_premix<kSsNW>(kwm, KM, mkm);
            rows(mkf, mkm);
        }
    };
    load_hdr(beg + tid);
    bool okc;
    uint32_t lzc[DD], regc[DD];
    uint64_t segc[DD];
    stage_b(beg + tid, okc, segc, lzc, regc);
    for (uint64_t p0 = beg; p0 < end; p0 += kSsThreads) {  // wave-uniform trip count
        bool okn = false;
        uint32_t lzn[DD], regn[DD];
        uint64_t segn[DD];
        if (p0 + kSsThreads < end) stage_b(p0 + kSsThreads + tid, okn, segn, lzn, regn);
        const uint64_t p = p0 + tid;
        if (okc) n_ok++;
#pragma unroll
        for (int rr = 0; rr < DD; rr++) {
            const bool want = okc && lzc[rr] > regc[rr];  // can encode only if above the batch-entry register
            const uint32_t q = wave_alloc(&s_cc, want);
            if (want) {
                rkey[q] = segc[rr] << kSsPktBits | (p & ((1ull << kSsPktBits) - 1));
                rval[q] = lzc[rr];
            }
        }
        okc = okn;
#pragma unroll
        for (int rr = 0; rr < DD; rr++) { segc[rr] = segn[rr]; lzc[rr] = lzn[rr]; regc[rr] = regn[rr]; }
    }
    atomicAdd(&s_ok, n_ok);
    __syncthreads();
    if (tid == 0) {
        a.cblk[blk] = s_cc;
        if (s_cc) atomicAdd(&a.stats[4], (unsigned long long)s_cc);
        if (s_ok) atomicAdd(&a.stats[0], (unsigned long long)s_ok);
        if (s_drop) atomicAdd(&a.stats[1], (unsigned long long)s_drop);
        if (s_unsup) atomicAdd(&a.stats[2], (unsigned long long)s_unsup);
    }
}

// S3b: flow ids for the successful encodes only (the MV loop's owner test and
// the cell keys are the only consumers of flow identity, and only encodes
// reach them).  Encode q's packet index is in skey[q]; its flow key is
// re-derived from the input, looked up / claimed in the dictionary and the id
// stored in sval[q]'s high word.  FIRST: encodes [blk*kSsIdChunk, +kSsIdChunk), probing
// from the key's hash slot; otherwise the block's parked encodes
// ((q - beg) << 32 | slot to resume at), from the previous launch.
struct SsIdsArgs {
    InputDesc in;
    KeyPlanN kpf, kpm;
    SsGeom g;
    DictDev D;
    uint32_t epoch;
    const uint32_t *ns;  // encodes of the batch (device count)
    const uint64_t *skey;
    uint64_t *sval;
    const uint64_t *pend_in;
    const uint32_t *cnt_in;
    uint64_t *pend_out;
    uint32_t *cnt_out, *total_out;
    unsigned long long *stats;
};

// Grid-stride over chunks of kSsIdChunk encodes: chunk c = blockIdx.x + k * gridDim.x
// (its parked list at pend[c * kSsIdChunk ...], its count at cnt[c]).
template <int KIND, int MF, int MM, bool FIRST>
__global__ __launch_bounds__(kSsThreads) void k_ss_ids(SsIdsArgs r) {
    __shared__ uint8_t s_srcf[80], s_srcm[80];
    __shared__ uint32_t s_cnt, s_full, s_claim, s_abort;
    const uint32_t tid = threadIdx.x;
    for (uint32_t j = tid; j < 80; j += kSsThreads) { s_srcf[j] = r.kpf.src[j]; s_srcm[j] = r.kpm.src[j]; }
    if (tid == 0) { s_full = 0; s_claim = 0; s_abort = dict_aborted(r.D); }
    __syncthreads();
    const uint32_t ns = *r.ns;
    const uint32_t nch = (ns + kSsIdChunk - 1) / kSsIdChunk;
    SsExtractArgs a{};
    a.in = r.in; a.kpf = r.kpf; a.kpm = r.kpm; a.g = r.g;
    for (uint32_t ch = blockIdx.x; ch < nch; ch += gridDim.x) {  // block-uniform
        if (s_abort) {  // the batch overflowed the dictionary: it is re-run after a reclaim
            if (tid == 0) r.cnt_out[ch] = 0;
            continue;
        }
        if (tid == 0) s_cnt = 0;
        __syncthreads();
        const uint64_t beg = (uint64_t)ch * kSsIdChunk;
        const uint32_t cnt = FIRST ? (uint32_t)min<uint64_t>(kSsIdChunk, ns - beg) : r.cnt_in[ch];
        for (uint32_t i = tid; i < cnt; i += kSsThreads) {
            uint64_t q;
            uint32_t slot = 0;
            if (FIRST) q = beg + i;
            else { const uint64_t v = r.pend_in[beg + i]; q = beg + (v >> 32); slot = (uint32_t)v; }
            const uint64_t p = r.skey[q] & ((1ull << kSsPktBits) - 1);
            uint32_t kwf[GNS_KWMAX], kwm[kSsNW];
            (void)ss_keys<KIND, MF, MM>(a, s_srcf, s_srcm, p, kwf, kwm);  // parsed OK in S1
            if (FIRST) slot = mm3_n<GNS_KWMAX>(kwf, r.g.Kf, r.D.seed) & r.D.mask;
            uint32_t out;
            const int res = dict_find_or_claim(r.D, kwf, slot, r.epoch, &out);
            if (res == DICT_CLAIMED) atomicAdd(&s_claim, 1u);
            if (res == DICT_FOUND || res == DICT_CLAIMED) r.sval[q] = (uint64_t)out << 32 | (r.sval[q] & 0xFFFFFFFFull);
            else if (res == DICT_PENDING) r.pend_out[beg + atomicAdd(&s_cnt, 1u)] = (q - beg) << 32 | out;
            else atomicAdd(&s_full, 1u);
        }
        __syncthreads();
        if (tid == 0) {
            r.cnt_out[ch] = s_cnt;
            if (s_cnt) atomicAdd(r.total_out, s_cnt);
        }
    }
    __syncthreads();
    if (tid == 0) {
        if (s_full) atomicAdd(&r.stats[3], (unsigned long long)s_full);
        dict_flush_claims(r.D, s_claim, &r.stats[3]);
    }
}

// S5: every cell's encodes in stream order: register write, pbits (:105-109),
// sampling (:200-204), MV loop (:206-233).  Split in three so the long
// sequential walks (one lane per cell; a superspreader's cell holds thousands
// of encodes) carry only the state that is really sequential:
//   S5a (per cell)   pbits walk -> tempP of every encode (table lookups + 2 adds)
//   S5b (per encode) sampling from tempP: repeat count vv, or 0 (skip)
//   S5c (per cell)   MV loop over the sampled encodes (owner: one add)
// Same operations in the same order as the single walk, so bit-identical.
struct SsApplyArgs {
    const uint64_t *skey;
    const uint64_t *sval;  // flow id << 32 | reg | lz << 8 | old << 16
    const uint32_t *ns;    // encodes of the batch (device count)
    SsGeom g;
    uint64_t pkt_base;
    uint8_t *regs;
    double *pbits;
    uint32_t *values, *keys;
    double *tp;    // [n] pbits before each encode (S5a -> S5b); then log(1 - first MV draw) (S5b -> S5c)
    int64_t *rep;  // [n] MV repeat count, 0 = not sampled (S5b -> S5c)
    const uint32_t *heads;  // segment starts, [nh] count at heads[cells]
    const uint32_t *hlen;   // encodes per segment
    uint32_t cells;
};

#pragma clang fp contract(off)
__global__ __launch_bounds__(256) void k_ss_walk_pbits(SsApplyArgs a) {
    __shared__ double s_t[256];  // go_pow_int(base, k) / m for every register value k
    const double mD = (double)a.g.m;
    s_t[threadIdx.x] = go_pow_int(a.g.base, (double)threadIdx.x) / mD;
    __syncthreads();
    const uint32_t hi = blockIdx.x * 256 + threadIdx.x;
    if (hi >= a.heads[a.cells]) return;
    const uint32_t nenc = *a.ns;
    const uint32_t k0 = a.heads[hi];
    const uint64_t cell = a.skey[k0] >> kSsPktBits;
    double pb = a.pbits[cell];
    uint64_t vc = a.sval[k0];
    for (uint32_t k = k0;;) {
        const uint32_t kn = k + 1;
        const uint64_t kx = kn < nenc ? a.skey[kn] : ~0ull;
        const uint64_t vx = kn < nenc ? a.sval[kn] : 0ull;
        const uint32_t v = (uint32_t)vc;
        const uint32_t reg = v & 0xFFu, lz = (v >> 8) & 0xFFu, old = (v >> 16) & 0xFFu;
        a.regs[cell * a.g.m + reg] = (uint8_t)lz;
        a.tp[k] = pb;                                    // tempP (:105)
        pb = pb + (-s_t[old]);                           // :106
        if (lz < a.g.maxv) pb = pb + s_t[lz];            // :107-109
        if ((kx >> kSsPktBits) != cell) break;
        k = kn; vc = vx;
    }
    a.pbits[cell] = pb;
}

__global__ __launch_bounds__(256) void k_ss_sample(SsApplyArgs a) {
    const uint32_t nenc = *a.ns;
    for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < nenc; k += gridDim.x * 256) {
    const double tempP = a.tp[k];
    int64_t vv = 0;
    if (tempP != -1.0) {                                                  // :196
        const uint64_t key = a.skey[k];
        const uint32_t row = (uint32_t)((key >> kSsPktBits) / a.g.w);
        const double inv = 1.0 / tempP;
        const double cv = ceil(inv);
        const double pCU = inv / cv;                                      // :200
        const uint64_t pkt = a.pkt_base + (key & ((1ull << kSsPktBits) - 1));
        if (!(ss_uniform(a.g.rng_seed, pkt, row, 0) >= pCU)) {            // :201-204
            vv = (cv < 9223372036854775808.0) ? (int64_t)cv : INT64_MIN;  // :206, amd64 semantics
            // the MV loop's first draw does not depend on the cell state: its log here, in parallel
            a.tp[k] = gm_log(1.0 - ss_uniform(a.g.rng_seed, pkt, row, 1));
        }
    }
    a.rep[k] = vv;
    }
}

// S5c: the MV loop over a cell's sampled encodes (super_spread.go:206-233).
// Lane per cell, as S5a; a cell with a long chain (a superspreader's: thousands
// of encodes, few sampled) is walked by the whole wave afterwards, 64 encodes
// per coalesced load and only the sampled ones stepped through (ballot), the MV
// state wave-uniform and the encode's fields read with v_readlane -- a lane
// walking it would pay one dependent load round trip per encode.
constexpr uint32_t kSsLongChain = 48;

__device__ __forceinline__ uint32_t rl32(uint32_t v, int j) { return __builtin_amdgcn_readlane(v, j); }
__device__ __forceinline__ uint64_t rl64(uint64_t v, int j) {
    return (uint64_t)rl32((uint32_t)(v >> 32), j) << 32 | rl32((uint32_t)v, j);
}

// one sampled encode: vv repeats of the MV step for flow f (state in val/key)
struct MvState {
    uint32_t val, key, mval;
    double mppp, ml1m;
};
// b^-val and log1m(b^-val) for val < kSsMvTab, computed once per workgroup into LDS
// with the same functions: a foreign encode's decrements (val - 1 each) then read
// them instead of a pow and a log1m per decrement.
constexpr uint32_t kSsMvTab = 2048;
__device__ __forceinline__ void mv_encode(const SsApplyArgs &a, MvState &st, int64_t vv, uint32_t f, uint64_t pkt,
                                          uint32_t row, double lc, const double *tpp, const double *tl1m) {
    uint32_t draw = 1;
    while (vv > 0) {                                                    // :207-233
        if (st.val == 0 || st.key == f) {  // every remaining iteration increments (:211-220)
            if (st.val == 0) st.key = f;
            st.val = (uint32_t)((uint64_t)st.val + (uint64_t)vv);
            break;
        }
        // b^-val and log1m(b^-val) depend only on val: kept for the next foreign
        // encode while val does not change
        if (st.val != st.mval) {
            st.mval = st.val;
            if (st.val < kSsMvTab) {
                st.mppp = tpp[st.val];
                st.ml1m = tl1m[st.val];
            } else {
                st.mppp = go_pow_int(a.g.b, -(double)st.val);               // :222
                st.ml1m = (st.mppp > 0 && st.mppp < 1) ? gm_log1m(st.mppp) : 0.0;
            }
        }
        const double ppp = st.mppp;
        if (!(ppp > 0)) break;  // underflow: no later iteration can decrement
        if (ppp >= 1) {         // b <= 1: every iteration decrements
            const int64_t dec = (int64_t)st.val < vv ? (int64_t)st.val : vv;
            st.val -= (uint32_t)dec;
            vv -= dec;
            continue;
        }
        // declared generator: failed iterations before the next decrement
        // (:223-227) as one geometric waiting time; the first draw's log came from S5b
        const double lu = draw == 1 ? lc : gm_log(1.0 - ss_uniform(a.g.rng_seed, pkt, row, draw));
        draw++;
        const double q = lu / st.ml1m;
        if (!(q < (double)vv)) break;
        vv -= (int64_t)floor(q) + 1;
        st.val -= 1;
    }
}

__global__ __launch_bounds__(256) void k_ss_walk_mv(SsApplyArgs a) {
    __shared__ double s_pp[kSsMvTab], s_l1m[kSsMvTab];
    for (uint32_t v = threadIdx.x; v < kSsMvTab; v += 256) {
        const double p = go_pow_int(a.g.b, -(double)v);
        s_pp[v] = p;
        s_l1m[v] = (p > 0 && p < 1) ? gm_log1m(p) : 0.0;
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t hi = blockIdx.x * 256 + threadIdx.x;
    const uint32_t nh = a.heads[a.cells];
    const uint32_t nenc = *a.ns;
    const bool valid = hi < nh;
    const uint32_t len = valid ? a.hlen[hi] : 0u;
    if (valid && len <= kSsLongChain) {
        const uint32_t k0 = a.heads[hi];
        const uint64_t cell = a.skey[k0] >> kSsPktBits;
        const uint32_t row = (uint32_t)(cell / a.g.w);
        MvState st{a.values[cell], a.keys[cell], 0xFFFFFFFFu, 0.0, 0.0};
        uint64_t kc = a.skey[k0], vc = a.sval[k0];
        int64_t rc = a.rep[k0];
        double lc = a.tp[k0];
        for (uint32_t k = k0;;) {
            const uint32_t kn = k + 1;  // the next encode's inputs load while this one runs
            const uint64_t kx = kn < nenc ? a.skey[kn] : ~0ull;
            const uint64_t vx = kn < nenc ? a.sval[kn] : 0ull;
            const int64_t rx = kn < nenc ? a.rep[kn] : 0;
            const double lx = kn < nenc ? a.tp[kn] : 0.0;
            mv_encode(a, st, rc, (uint32_t)(vc >> 32), a.pkt_base + (kc & ((1ull << kSsPktBits) - 1)), row, lc, s_pp,
                      s_l1m);
            if ((kx >> kSsPktBits) != cell) break;
            k = kn; kc = kx; vc = vx; rc = rx; lc = lx;
        }
        a.values[cell] = st.val;
        a.keys[cell] = st.key;
    }
    // long chains of this wave's cells, one after another, by the whole wave
    uint64_t lm = __ballot(valid && len > kSsLongChain);
    while (lm) {  // wave-uniform
        const int jl = __ffsll((unsigned long long)lm) - 1;
        lm &= lm - 1;
        const uint32_t hj = rl32(hi, jl), nj = rl32(len, jl);
        const uint32_t k0 = a.heads[hj];
        const uint64_t cell = a.skey[k0] >> kSsPktBits;
        const uint32_t row = (uint32_t)(cell / a.g.w);
        MvState st{a.values[cell], a.keys[cell], 0xFFFFFFFFu, 0.0, 0.0};
        // windows of 64 encodes, three loads ahead of the one being stepped (a
        // superspreader's chain is thousands of encodes: the step is short, the load is not)
        struct Win { uint64_t k, v; int64_t r; double l; };
        auto ld = [&](uint32_t w0) {
            Win x{0ull, 0ull, 0, 0.0};
            if (w0 + lane < nj) {
                const uint32_t k = k0 + w0 + lane;
                x.k = a.skey[k]; x.r = a.rep[k]; x.v = a.sval[k]; x.l = a.tp[k];
            }
            return x;
        };
        Win n1 = ld(0), n2 = ld(64), n3 = ld(128), n4 = ld(192);
        for (uint32_t w0 = 0; w0 < nj; w0 += 64) {
            const Win cw = n1;
            n1 = n2; n2 = n3; n3 = n4; n4 = ld(w0 + 256);
            const bool in = w0 + lane < nj;
            const uint64_t kx = cw.k, vx = cw.v;
            const int64_t rx = cw.r;
            const double lx = cw.l;
            uint64_t sm = __ballot(in && rx > 0);
            if (sm && st.val != 0) {
                // Speculate over the window: the owner's encodes add vv (u32 wrap, :211-220)
                // and every other sampled encode leaves (val, key) alone -- its first draw
                // (the log from S5b) waits past all vv repeats (:223-227), or b^-val
                // underflows.  Each lane evaluates that test against the val it would see;
                // the first lane where it does not hold (a decrement, a takeover at val 0,
                // b <= 1) and everything after it run the sequential loop below, from the
                // exact state before that lane.  Same operations on the same values, so
                // bit-identical, and a chain's common case costs one step per window.
                const bool samp = in && rx > 0;
                const uint32_t f = (uint32_t)(vx >> 32);
                const bool own = samp && f == st.key;
                const uint32_t add = own ? (uint32_t)(uint64_t)rx : 0u;
                const uint32_t inc = wave_incl_scan(add);
                const uint32_t vb = st.val + (inc - add);  // val before this lane
                bool fail = false;
                if (samp && !own) {
                    if (vb == 0) {
                        fail = true;
                    } else {
                        const double ppp = vb < kSsMvTab ? s_pp[vb] : go_pow_int(a.g.b, -(double)vb);   // :222
                        if (ppp > 0) {
                            if (ppp >= 1) fail = true;
                            else if (lx / (vb < kSsMvTab ? s_l1m[vb] : gm_log1m(ppp)) < (double)rx) fail = true;
                        }
                    }
                }
                const uint64_t fm = __ballot(fail);
                if (!fm) {
                    st.val += __shfl(inc, 63);
                    sm = 0;
                } else {
                    const int F = __ffsll((unsigned long long)fm) - 1;
                    st.val = rl32(vb, F);
                    sm &= ~((1ull << F) - 1ull);  // lanes before F are settled
                }
            }
            while (sm) {
                const int j = __ffsll((unsigned long long)sm) - 1;
                sm &= sm - 1;
                const double lcj = __longlong_as_double((long long)rl64((uint64_t)__double_as_longlong(lx), j));
                mv_encode(a, st, (int64_t)rl64((uint64_t)rx, j), rl32((uint32_t)(vx >> 32), j),
                          a.pkt_base + (rl64(kx, j) & ((1ull << kSsPktBits) - 1)), row, lcj, s_pp, s_l1m);
            }
        }
        if (lane == 0) { a.values[cell] = st.val; a.keys[cell] = st.key; }
    }
}
#pragma clang fp contract(on)

// Query (super_spread.go:238-249)
struct SsQueryArgs {
    const uint8_t *flows;
    uint32_t stride;
    uint64_t n;
    SsGeom g;
    DictDev D;
    const uint32_t *values, *keys;
    uint64_t *out;
};

__global__ __launch_bounds__(256) void k_ss_query(SsQueryArgs a) {
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= a.n) return;
    uint32_t kw[GNS_KWMAX];
    load_key_bytes<GNS_KWMAX>(a.flows + p * a.stride, a.g.Kf, false, kw);
    const uint32_t id = dict_lookup(a.D, kw);
    uint32_t est = 0;
    if (id != GNS_ID_NONE) {
        for (uint32_t r = 0; r < a.g.d; r++) {
            const uint64_t c = (uint64_t)r * a.g.w + ss_row_index(a.g, mm3_n<GNS_KWMAX>(kw, a.g.Kf, a.g.seeds[r]));
            if (a.keys[c] == id && a.values[c] > est) est = a.values[c];
        }
    }
    a.out[p] = est > 1 ? est : 1;
}

__global__ __launch_bounds__(256) void k_ss_ids_to_bytes(const uint32_t *ids, uint64_t n, DictDev D,
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

// ---------------------------------------------------------------------------
// Candidate pipeline without a library sort or a host round trip (round 4):
//   P1 k_sp_hist     per S1 block region, histogram of its candidates over NB
//                    bins of consecutive cells (block-major, as Count-Min's K1)
//   P2 k_tscan_*     bin-major offsets (gns_scan.cuh)
//   P3 k_sp_scatter  candidates into their bins as packed words
//                    local seg << 35 | packet << 8 | lz, staged in LDS and copied
//                    out bin by bin (order inside a bin is free: the packet rides along)
//   P4 k_sp_bins     persistent, one 1024-thread workgroup per bin at a time:
//                    the bin (or each group of whole cells of a large bin, split
//                    by a cell histogram) is radix-sorted in LDS by (seg, packet);
//                    a segmented max gives every candidate the register value it
//                    would see (super_spread.go:90-103), so it encodes iff lz
//                    exceeds it; the encodes are sorted by (cell, packet) in LDS
//                    and written with one global atomic per group, plus the heads
//                    of the cells (S5's walks).  A cell with more candidates than
//                    fit LDS (a superspreader in a batch that starts from low
//                    registers) takes the order-free form of the same test: the
//                    earliest packet per (register, lz) by LDS atomicMin, suffix
//                    minima over lz, and a candidate encodes iff it is the earliest
//                    packet with an lz >= its own.
// Every launch is sized from host-known bounds; counts stay on the device.
// ---------------------------------------------------------------------------
constexpr uint32_t kSpCap = 8192;        // items a P4 workgroup holds in LDS
constexpr uint32_t kSpThreads = 512;     // 8 waves, 16 items per thread (1024 threads spilled at 128 VGPRs)
constexpr uint32_t kSpWaves = kSpThreads / 64;
constexpr uint32_t kSpPer = kSpCap / kSpThreads;   // 16 items per thread
constexpr uint32_t kSpSub = 4096;        // P3 candidates staged per sub-pass
constexpr uint32_t kSpMaxBins = 4096;
constexpr uint32_t kSpMaxCpb = 8192;     // cells per bin (P4's cell histogram)
constexpr uint32_t kSpV = 34;            // lz values (geometric values are <= 33)

struct SpGeom {
    uint32_t nb, cpb, cpb_bits, m, mbits;  // bins, cells per bin (power of two), m (mbits: log2 m if power of two, else 0xFF)
    uint32_t lbits;                        // bits of a local seg (cpb * m)
    uint32_t cells;
};

__device__ __forceinline__ uint64_t sp_cell(const SpGeom &s, uint64_t seg) {
    return s.mbits != 0xFFu ? seg >> s.mbits : seg / s.m;
}

// P1
__global__ __launch_bounds__(256) void k_sp_hist(const uint64_t *ckey, const uint32_t *cblk, uint32_t d, SpGeom s,
                                                 uint32_t *hist) {
    __shared__ uint32_t h[kSpMaxBins];
    const uint32_t blk = blockIdx.x, tid = threadIdx.x;
    for (uint32_t i = tid; i < s.nb; i += 256) h[i] = 0;
    __syncthreads();
    const uint32_t cnt = cblk[blk];
    const uint64_t *r = ckey + (uint64_t)blk * kSsChunk * d;
    for (uint32_t i = tid; i < cnt; i += 256) {
        const uint64_t cell = sp_cell(s, r[i] >> kSsPktBits);
        atomicAdd(&h[(uint32_t)(cell >> s.cpb_bits)], 1u);
    }
    __syncthreads();
    for (uint32_t i = tid; i < s.nb; i += 256) hist[(uint64_t)blk * s.nb + i] = h[i];
}

// P3: kSpSub-candidate sub-passes: count per bin, local starts, stage by bin, copy out runs
__global__ __launch_bounds__(256) void k_sp_scatter(const uint64_t *ckey, const uint32_t *cval, const uint32_t *cblk,
                                                    uint32_t d, SpGeom s, const uint32_t *offs, uint64_t *words) {
    __shared__ uint32_t gpos[kSpMaxBins], cnt[kSpMaxBins];
    __shared__ uint64_t stage[kSpSub];
    __shared__ uint16_t sbin[kSpSub];
    __shared__ uint32_t wsum[4];
    // (the XCD-contiguous order of gns_xcd.cuh measured neutral here: profiles/r05_ab_xcd_all.txt)
    const uint32_t blk = blockIdx.x, tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    for (uint32_t i = tid; i < s.nb; i += 256) { gpos[i] = offs[(uint64_t)blk * s.nb + i]; cnt[i] = 0; }
    __syncthreads();
    const uint32_t n = cblk[blk];
    const uint64_t base = (uint64_t)blk * kSsChunk * d;
    constexpr uint32_t kPer = kSpSub / 256;
    const uint32_t per = (s.nb + 255) / 256;  // bins per thread in the local scan
    for (uint32_t c0 = 0; c0 < n; c0 += kSpSub) {
        const uint32_t m = min(kSpSub, n - c0);
        uint64_t w[kPer];
        uint32_t b[kPer], rk[kPer];
#pragma unroll
        for (uint32_t j = 0; j < kPer; j++) {
            const uint32_t i = j * 256 + tid;
            b[j] = 0xFFFFFFFFu;
            if (i < m) {
                const uint64_t key = ckey[base + c0 + i];
                const uint64_t seg = key >> kSsPktBits;
                const uint64_t cell = sp_cell(s, seg);
                const uint32_t bin = (uint32_t)(cell >> s.cpb_bits);
                const uint64_t local = seg - ((uint64_t)bin << s.cpb_bits) * s.m;
                w[j] = local << 35 | (key & ((1ull << kSsPktBits) - 1)) << 8 | (cval[base + c0 + i] & 0xFFu);
                b[j] = bin;
                rk[j] = atomicAdd(&cnt[bin], 1u);
            }
        }
        __syncthreads();
        // exclusive scan of the bin counts (per bins per thread, then the waves)
        uint32_t sum = 0;
        for (uint32_t q = 0; q < per; q++) {
            const uint32_t i = tid * per + q;
            sum += i < s.nb ? cnt[i] : 0u;
        }
        const uint32_t inc = wave_incl_scan(sum);
        if (lane == 63) wsum[wave] = inc;
        __syncthreads();
        uint32_t run = inc - sum;
        for (uint32_t v = 0; v < wave; v++) run += wsum[v];
        for (uint32_t q = 0; q < per; q++) {
            const uint32_t i = tid * per + q;
            if (i < s.nb) { const uint32_t c = cnt[i]; cnt[i] = run; run += c; }
        }
        __syncthreads();
#pragma unroll
        for (uint32_t j = 0; j < kPer; j++)
            if (b[j] != 0xFFFFFFFFu) {
                const uint32_t pos = cnt[b[j]] + rk[j];
                stage[pos] = w[j];
                sbin[pos] = (uint16_t)b[j];
            }
        __syncthreads();
        for (uint32_t i = tid; i < m; i += 256) {
            const uint32_t bin = sbin[i];
            words[gpos[bin] + (i - cnt[bin])] = stage[i];
        }
        __syncthreads();
        // advance each bin's global cursor by its count (next starts - this start), clear
        for (uint32_t i = tid; i < s.nb; i += 256) {
            const uint32_t nx = i + 1 < s.nb ? cnt[i + 1] : m;
            gpos[i] += nx - cnt[i];
        }
        __syncthreads();
        for (uint32_t i = tid; i < s.nb; i += 256) cnt[i] = 0;
        __syncthreads();
    }
}

struct SpArgs {
    SpGeom s;
    const uint64_t *words;   // bin-major candidates (P3)
    uint64_t *words2;        // scratch of the same size (large bins, grouped by cells)
    const uint32_t *bstart;  // [nb] bin starts (the exclusive scan of the bin totals)
    const uint32_t *total;   // candidates in the batch
    const uint8_t *regs;     // batch-entry registers
    uint64_t *skey, *sval;   // encodes out: cell << 27 | packet, GNS_ID_NONE << 32 | reg | lz << 8 | old << 16
    uint32_t *scount;        // encodes written (device count)
    uint32_t *heads;         // [cells]: cell starts in skey, count at [cells]
    uint32_t *hlen;          // [cells]: encodes of the cell of heads[i]
    uint32_t *work;          // bin counter of the persistent grid
    const uint32_t *order;   // [nb] bins, largest first (k_sp_order)
    unsigned long long *err; // a cell with more encodes than LDS holds (cannot happen below 8192)
    uint32_t maxg;           // groups per window of a large bin (kSpMaxG; GNS_SS_SPG, tests only)
    uint32_t cap;            // encodes a cell may take in one batch: kSpCap (GNS_SS_TEST_SPCAP lowers it, tests only)
    unsigned long long *prof;  // GNS_SS_DEBUG: P4 phase cycles (sp_group), else null
};

constexpr uint32_t kSpMaxG = 512;       // cell groups of a large bin per window
constexpr uint32_t kSpHalf = kSpCap / 2;  // group slot width (candidates)
struct SpLds {
    uint64_t a[kSpCap], b[kSpCap];
    uint32_t cnt[256 * kSpWaves];  // radix counters, digit-major [digit][wave]
    uint32_t gtab[3 * kSpMaxG];    // groups of a window: start, count, first cell
    uint32_t gcur[kSpMaxG];
    uint32_t wsum[kSpWaves + 2];
    uint32_t bin, n_succ, gbase, hbase, ngrp, cend;
    uint32_t agg_seg[kSpWaves], agg_mx[kSpWaves], agg_fl[kSpWaves];
};

// f(i, x) for every x = src[i], i < n, with eight loads per thread in flight
// (a loop of one load per trip waits a full memory round trip per trip).  Words
// another wave of this workgroup wrote before a __syncthreads() are visible to
// plain loads (same CU, same L1).
template <typename F>
__device__ __forceinline__ void sp_for8(const uint64_t *src, uint32_t n, F f) {
    for (uint32_t i0 = 0; i0 < n; i0 += kSpThreads * 8) {  // block-uniform
        uint64_t x[8];
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) {
            const uint32_t i = i0 + j * kSpThreads + threadIdx.x;
            x[j] = i < n ? src[i] : 0ull;
        }
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) {
            const uint32_t i = i0 + j * kSpThreads + threadIdx.x;
            if (i < n) f(i, x[j]);
        }
    }
}

// Prefix over the kSpWaves per-wave values in ws[] (after a barrier): this wave's
// exclusive start and the total, from one LDS load and one DPP scan (a loop over
// the earlier waves waited one LDS round trip per wave, in every radix pass).
__device__ __forceinline__ uint32_t sp_wave_prefix(const uint32_t *ws, uint32_t *total = nullptr) {
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    const uint32_t x = lane < kSpWaves ? ws[lane] : 0u;
    const uint32_t inc = wave_incl_scan(x);
    if (total) *total = __shfl(inc, 63);
    return __shfl(inc - x, (int)wave);
}

// Exclusive scan of one value per thread over the workgroup; returns this
// thread's start.  Uses L.wsum; synchronises.
__device__ __forceinline__ uint32_t sp_block_excl(SpLds &L, uint32_t v, uint32_t *total = nullptr) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t inc = wave_incl_scan(v);
    __syncthreads();  // earlier readers of wsum are done
    if (lane == 63) L.wsum[wave] = inc;
    __syncthreads();
    const uint32_t run = inc - v + sp_wave_prefix(L.wsum, total);
    __syncthreads();
    return run;
}

// Stable LSD radix sort (8-bit digits) of n <= kSpCap items of L.a / L.b by bits
// [lo, hi); src is a or b; returns where the result is.  Item idx lives in lane
// idx % 64 of wave idx / 512 (slot (idx / 64) % 8): a wave owns 512 consecutive
// items, so returning LDS adds (same-address lanes served in lane order, the
// Count-Min K3 property, measured on gfx950: tools/lds_order.hip) give stable ranks.
__device__ __forceinline__ uint64_t *sp_sort(SpLds &L, uint64_t *src, uint32_t n, uint32_t lo, uint32_t hi) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    uint64_t *dst = src == L.a ? L.b : L.a;
    // items per lane for this n (block-uniform): a wave owns pt * 64 consecutive items,
    // so a small sort runs pt (not kSpPer) item slots per lane in every pass
    const uint32_t pt = (n + kSpThreads - 1) / kSpThreads;
    for (uint32_t sh = lo; sh < hi; sh += 8) {
        const uint32_t nd = min(8u, hi - sh), ndig = 1u << nd, dmask = ndig - 1u;
        for (uint32_t dg = lane; dg < ndig; dg += 64) L.cnt[dg * kSpWaves + wave] = 0;
        uint64_t x[kSpPer];
        uint32_t dg[kSpPer], rk[kSpPer];
#pragma unroll
        for (uint32_t j = 0; j < kSpPer; j++) {
            if (j >= pt) continue;  // block-uniform
            const uint32_t idx = wave * pt * 64 + j * 64 + lane;
            const bool v = idx < n;
            x[j] = v ? src[idx] : 0ull;
            dg[j] = (uint32_t)(x[j] >> sh) & dmask;
            rk[j] = atomicAdd(&L.cnt[dg[j] * kSpWaves + wave], v ? 1u : 0u);
        }
        __syncthreads();
        // exclusive scan over (digit, wave): ndig * 16 <= 4096 counters, 4 per thread
        const uint32_t nc = ndig * kSpWaves;
        uint32_t c[4], sum = 0;
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) {
            const uint32_t i = tid * 4 + q;
            c[q] = i < nc ? L.cnt[i] : 0u;
            sum += c[q];
        }
        const uint32_t inc = wave_incl_scan(sum);
        if (lane == 63) L.wsum[wave] = inc;
        __syncthreads();
        uint32_t run = inc - sum + sp_wave_prefix(L.wsum);
#pragma unroll
        for (uint32_t q = 0; q < 4; q++) {
            const uint32_t i = tid * 4 + q;
            if (i < nc) L.cnt[i] = run;
            run += c[q];
        }
        __syncthreads();
#pragma unroll
        for (uint32_t j = 0; j < kSpPer; j++) {
            if (j >= pt) continue;  // block-uniform
            const uint32_t idx = wave * pt * 64 + j * 64 + lane;
            if (idx < n) dst[L.cnt[dg[j] * kSpWaves + wave] + rk[j]] = x[j];
        }
        __syncthreads();
        uint64_t *t = src; src = dst; dst = t;
    }
    return src;
}

// Encodes of one group of whole cells (n <= kSpCap candidates in *src): sort by
// (local seg, packet), segmented running max of lz per register, encode test
// against the batch-entry register, encodes sorted by (cell, packet), written
// out with their cell heads.  bin0seg = first seg of the bin.
__device__ __noinline__ void sp_group(const SpArgs &a, SpLds &L, uint64_t *src, uint32_t n, uint64_t bin0seg, uint64_t bin0cell) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    uint64_t tprev = a.prof ? __builtin_amdgcn_s_memtime() : 0;
    auto mark = [&](int i) {  // diagnosis only (GNS_SS_DEBUG)
        if (a.prof && tid == 0) {
            const uint64_t t = __builtin_amdgcn_s_memtime();
            atomicAdd(&a.prof[i], (unsigned long long)(t - tprev));
            tprev = t;
        }
    };
    if (a.prof && tid == 0) atomicAdd(&a.prof[7], 1ull);
    uint64_t *srt = sp_sort(L, src, n, 8, 35 + a.s.lbits);
    mark(0);
    uint64_t *out = srt == L.a ? L.b : L.a;
    // thread-major: thread t holds sorted positions [pt * t, pt * t + pt)
    const uint32_t pt = (n + kSpThreads - 1) / kSpThreads;
    const uint32_t p0 = tid * pt;
    uint64_t x[kSpPer];
    uint32_t seg_last = 0xFFFFFFFFu, mx = 0, full = 1, have = 0;
#pragma unroll
    for (uint32_t j = 0; j < kSpPer; j++) {
        if (j >= pt) continue;  // block-uniform
        x[j] = p0 + j < n ? srt[p0 + j] : ~0ull;
        if (p0 + j < n) {
            const uint32_t sg = (uint32_t)(x[j] >> 35), lz = (uint32_t)x[j] & 0xFFu;
            if (have && sg != seg_last) { full = 0; mx = 0; }
            if (!have || sg != seg_last) mx = 0;
            mx = max(mx, lz);
            seg_last = sg;
            have = 1;
        }
    }
    // exclusive segmented max over the threads: aggregate (seg_last, mx, full, have);
    // combine(L, R) = !R.have ? L : (R.full && R.seg == L.seg ? (seg, max, L.full, 1) : R)
    uint32_t cs = seg_last, cm = mx, cf = full, ch = have;  // inclusive, built with shuffles
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t ls = __shfl_up(cs, o), lm = __shfl_up(cm, o), lf = __shfl_up(cf, o), lh = __shfl_up(ch, o);
        if (lane >= o && lh) {
            if (!ch) { cs = ls; cm = lm; cf = lf; ch = 1; }
            else if (cf && cs == ls) { cm = max(cm, lm); cf = lf; }
        }
    }
    if (lane == 63) { L.agg_seg[wave] = cs; L.agg_mx[wave] = cm; L.agg_fl[wave] = cf | (ch << 1); }
    __syncthreads();
    // carry into this thread = inclusive value of the previous lane, preceded by the earlier waves
    uint32_t ps = __shfl_up(cs, 1), pm = __shfl_up(cm, 1), pf = __shfl_up(cf, 1), ph = __shfl_up(ch, 1);
    if (lane == 0) ph = 0;
    // waves before this one (their last seg and its running max): the same segmented
    // scan over the wave aggregates, lane w holding wave w's, then lane wave - 1's value
    uint32_t ws, wm, wh;
    {
        uint32_t as = 0xFFFFFFFFu, am = 0, af = 1, ah = 0;
        if (lane < kSpWaves) { as = L.agg_seg[lane]; am = L.agg_mx[lane]; af = L.agg_fl[lane] & 1u; ah = L.agg_fl[lane] >> 1; }
        for (uint32_t o = 1; o < kSpWaves; o <<= 1) {
            const uint32_t ls = __shfl_up(as, o), lm = __shfl_up(am, o), lf = __shfl_up(af, o), lh = __shfl_up(ah, o);
            if (lane >= o && lh) {
                if (!ah) { as = ls; am = lm; af = lf; ah = 1; }
                else if (af && as == ls) { am = max(am, lm); af = lf; }
            }
        }
        const int src = wave > 0 ? (int)wave - 1 : 0;
        ws = __shfl(as, src); wm = __shfl(am, src); wh = wave > 0 ? __shfl(ah, src) : 0u;
    }
    uint32_t carry_seg = 0xFFFFFFFFu, carry_mx = 0;
    if (ph) {
        carry_seg = ps; carry_mx = pm;
        if (pf && wh && ws == ps) carry_mx = max(carry_mx, wm);
    } else if (wh) {
        carry_seg = ws; carry_mx = wm;
    }
    // encode test
    uint32_t succ = 0;
    uint64_t item[kSpPer];
    uint32_t rseg = carry_seg, rmx = carry_mx;
#pragma unroll
    for (uint32_t j = 0; j < kSpPer; j++) {
        item[j] = ~0ull;
        if (j >= pt) continue;  // block-uniform
        if (p0 + j < n) {
            const uint32_t sg = (uint32_t)(x[j] >> 35), lz = (uint32_t)x[j] & 0xFFu;
            const uint32_t pk = (uint32_t)(x[j] >> 8) & ((1u << kSsPktBits) - 1u);
            if (sg != rseg) { rseg = sg; rmx = 0; }
            const uint64_t seg = bin0seg + sg;
            const uint32_t old = max((uint32_t)a.regs[seg], rmx);
            if (lz > old) {
                const uint64_t cl = sp_cell(a.s, (uint64_t)sg);  // cell within the bin
                const uint32_t reg = (uint32_t)((uint64_t)sg - cl * a.s.m);
                item[j] = (cl << kSsPktBits | pk) << 24 | (uint64_t)(reg | lz << 8 | old << 16);
                succ++;
            }
            rmx = max(rmx, lz);
        }
    }
    // compact the encodes into `out` (order kept), then sort them by (cell, packet)
    const uint32_t inc = wave_incl_scan(succ);
    if (lane == 63) L.wsum[wave] = inc;
    __syncthreads();
    uint32_t ns = 0;
    uint32_t q = inc - succ + sp_wave_prefix(L.wsum, &ns);
#pragma unroll
    for (uint32_t j = 0; j < kSpPer; j++) {
        if (j >= pt) continue;  // block-uniform
        if (item[j] != ~0ull) out[q++] = item[j];
    }
    __syncthreads();
    if (ns == 0) return;
    uint32_t cbits = 0;
    while ((1u << cbits) < a.s.cpb) cbits++;
    mark(1);
    uint64_t *es = sp_sort(L, out, ns, 24, 24 + kSsPktBits + cbits);
    uint64_t *tbl = es == L.a ? L.b : L.a;  // [cpb] per cell: head index << 32 | start in es
    mark(2);
    // the group's heads (first encode of each cell): counted per thread, then one global
    // add for all their slots (an add per wave on the one counter every workgroup
    // shares was most of P4's time)
    auto is_head = [&](uint32_t i) {
        return i == 0 || (uint32_t)(es[i - 1] >> (24 + kSsPktBits)) != (uint32_t)(es[i] >> (24 + kSsPktBits));
    };
    uint32_t nhd = 0;
    for (uint32_t i = tid; i < ns; i += kSpThreads) nhd += is_head(i) ? 1u : 0u;
    uint32_t htot = 0;
    uint32_t hpos = sp_block_excl(L, nhd, &htot);
    if (tid == 0) {
        L.gbase = atomicAdd(a.scount, ns);
        L.hbase = atomicAdd(&a.heads[a.s.cells], htot);
    }
    __syncthreads();
    const uint32_t gb = L.gbase;
    hpos += L.hbase;
    for (uint32_t i = tid; i < ns; i += kSpThreads) {
        const uint64_t e = es[i];
        const uint64_t ck = e >> 24;
        const uint64_t cell = bin0cell + (ck >> kSsPktBits);
        a.skey[gb + i] = cell << kSsPktBits | (ck & ((1ull << kSsPktBits) - 1));
        a.sval[gb + i] = (uint64_t)GNS_ID_NONE << 32 | (e & 0xFFFFFFull);
        if (is_head(i)) {
            a.heads[hpos] = gb + i;
            tbl[(uint32_t)(ck >> kSsPktBits)] = (uint64_t)hpos << 32 | i;  // cell -> (head, start)
            hpos++;
        }
    }
    __syncthreads();
    mark(3);
    // chain lengths (S5c walks long chains with the whole wave): the last encode of each cell
    for (uint32_t i = tid; i < ns; i += kSpThreads) {
        const uint32_t c = (uint32_t)(es[i] >> (24 + kSsPktBits));
        if (i + 1 == ns || (uint32_t)(es[i + 1] >> (24 + kSsPktBits)) != c) {
            const uint64_t t = tbl[c];
            a.hlen[t >> 32] = i + 1 - (uint32_t)t;
        }
    }
    __syncthreads();
    mark(4);
}

// One cell with more candidates than LDS holds: the order-free form.  For every
// (register, lz) the earliest packet (LDS atomicMin), then suffix minima over lz:
// S[reg][v] = earliest packet with an lz >= v.  A candidate (reg, p, lz) encodes iff
// S[reg][lz] == p; the register value it sees is the largest v < lz with
// S[reg][v] < p, or the batch-entry register.
__device__ __noinline__ void sp_giant(const SpArgs &a, SpLds &L, const uint64_t *w2, uint32_t n, uint64_t bin0seg, uint64_t cellg,
                         uint32_t cl_in_bin) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u;
    const uint32_t m = a.s.m;
    uint32_t *S = reinterpret_cast<uint32_t *>(L.a);  // [m][kSpV] (m <= 256: 34 KB of the 64 KB)
    const uint64_t seg0 = (uint64_t)cl_in_bin * m;   // local seg of the cell's register 0
    for (uint32_t i = tid; i < m * kSpV; i += kSpThreads) S[i] = 0xFFFFFFFFu;
    if (tid == 0) L.n_succ = 0;
    __syncthreads();
    sp_for8(w2, n, [&](uint32_t, uint64_t x) {
        const uint32_t reg = (uint32_t)((x >> 35) - seg0), lz = min((uint32_t)x & 0xFFu, kSpV - 1);
        atomicMin(&S[reg * kSpV + lz], (uint32_t)(x >> 8) & ((1u << kSsPktBits) - 1u));
    });
    __syncthreads();
    for (uint32_t r = tid; r < m; r += kSpThreads) {
        uint32_t run = 0xFFFFFFFFu;
        for (int v = (int)kSpV - 1; v >= 0; v--) { run = min(run, S[r * kSpV + v]); S[r * kSpV + v] = run; }
    }
    __syncthreads();
    sp_for8(w2, n, [&](uint32_t, uint64_t x) {
        const uint32_t reg = (uint32_t)((x >> 35) - seg0), lz = (uint32_t)x & 0xFFu;
        const uint32_t pk = (uint32_t)(x >> 8) & ((1u << kSsPktBits) - 1u);
        if (S[reg * kSpV + lz] != pk) return;
        const uint32_t entry = a.regs[(cellg * m) + reg];
        uint32_t old = entry;
        for (int v = (int)lz - 1; v > (int)entry; v--)
            if (S[reg * kSpV + v] < pk) { old = (uint32_t)v; break; }
        const uint32_t q = atomicAdd(&L.n_succ, 1u);
        if (q < kSpCap) L.b[q] = (uint64_t)pk << 24 | (uint64_t)(reg | lz << 8 | old << 16);
    });
    __syncthreads();
    uint32_t ns = L.n_succ;
    if (ns > a.cap) {
        if (tid == 0) atomicAdd(a.err, 1ull);
        ns = min(ns, kSpCap);
    }
    if (ns == 0) return;
    uint64_t *es = sp_sort(L, L.b, ns, 24, 24 + kSsPktBits);
    if (tid == 0) {
        L.gbase = atomicAdd(a.scount, ns);
        const uint32_t h = atomicAdd(&a.heads[a.s.cells], 1u);
        a.heads[h] = L.gbase;
        a.hlen[h] = ns;
    }
    __syncthreads();
    const uint32_t gb = L.gbase;
    for (uint32_t i = tid; i < ns; i += kSpThreads) {
        const uint64_t e = es[i];
        a.skey[gb + i] = cellg << kSsPktBits | (e >> 24);
        a.sval[gb + i] = (uint64_t)GNS_ID_NONE << 32 | (e & 0xFFFFFFull);
    }
    __syncthreads();
    (void)lane;
}

// P4 schedule: bins by decreasing size (1/8-octave classes; the order inside a
// class is arbitrary), so a superspreader's bin starts first instead of setting
// the tail.  One workgroup, nb <= kSpMaxBins.
__global__ __launch_bounds__(1024) void k_sp_order(const uint32_t *bstart, const uint32_t *total, uint32_t nb,
                                                   uint32_t *order) {
    constexpr uint32_t NK = 33 * 8;
    __shared__ uint32_t s_cnt[NK];
    __shared__ uint16_t s_key[kSpMaxBins];
    for (uint32_t k = threadIdx.x; k < NK; k += 1024) s_cnt[k] = 0;
    __syncthreads();
    for (uint32_t b = threadIdx.x; b < nb; b += 1024) {
        const uint32_t sz = (b + 1 < nb ? bstart[b + 1] : *total) - bstart[b];
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
    for (uint32_t b = threadIdx.x; b < nb; b += 1024) order[atomicAdd(&s_cnt[s_key[b]], 1u)] = b;
}

// P4: persistent; bins from a work counter, largest first.
__global__ __launch_bounds__(kSpThreads) void k_sp_bins(SpArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t spsm[];
    SpLds &L = *reinterpret_cast<SpLds *>(spsm);
    const uint32_t tid = threadIdx.x;
    for (;;) {
        if (tid == 0) {
            const uint32_t k = atomicAdd(a.work, 1u);
            L.bin = k < a.s.nb ? a.order[k] : 0xFFFFFFFFu;
        }
        __syncthreads();
        const uint32_t bin = L.bin;
        __syncthreads();
        if (bin >= a.s.nb) return;
        const uint32_t b0 = a.bstart[bin];
        const uint32_t b1 = bin + 1 < a.s.nb ? a.bstart[bin + 1] : *a.total;
        const uint32_t n = b1 - b0;
        if (n == 0) continue;
        const uint64_t bin0cell = (uint64_t)bin << a.s.cpb_bits;
        const uint64_t bin0seg = bin0cell * a.s.m;
        if (n <= kSpCap) {
            sp_for8(a.words + b0, n, [&](uint32_t i, uint64_t x) { L.a[i] = x; });
            __syncthreads();
            sp_group(a, L, L.a, n, bin0seg, bin0cell);
            continue;
        }
        // a large bin: windows of cells.  Per window a cell histogram, its exclusive
        // scan P, and groups by position: the cells with P in [s * kSpHalf, (s + 1) *
        // kSpHalf) and at most kSpHalf candidates each form group 2s (< kSpCap
        // candidates), a cell with more forms group 2s + 1 alone (at most one such
        // cell starts per slot) and takes the order-free path.  The window's
        // candidates are grouped into words2, then the groups run one by one.
        uint32_t *ccnt = reinterpret_cast<uint32_t *>(L.b);  // [cpb] candidates per cell
        uint32_t *cgid = ccnt + kSpMaxCpb;                   // [cpb] group of the cell
        constexpr uint32_t kCpt = kSpMaxCpb / kSpThreads;                // cells per thread at most
        const uint32_t per = (a.s.cpb + kSpThreads - 1) / kSpThreads;
        for (uint32_t cw = 0; cw < a.s.cpb;) {
            for (uint32_t c = tid; c < a.s.cpb; c += kSpThreads) ccnt[c] = 0;
            for (uint32_t g = tid; g < a.maxg; g += kSpThreads) { L.gtab[3 * g + 1] = 0; L.gtab[3 * g + 2] = 0xFFFFFFFFu; }
            if (tid == 0) L.cend = a.s.cpb;
            __syncthreads();
            sp_for8(a.words + b0, n, [&](uint32_t, uint64_t x) {
                const uint32_t c = (uint32_t)sp_cell(a.s, x >> 35);
                if (c >= cw) atomicAdd(&ccnt[c], 1u);
            });
            __syncthreads();
            uint32_t k[kCpt], sum = 0;
#pragma unroll
            for (uint32_t q = 0; q < kCpt; q++) {
                const uint32_t c = tid * per + q;
                k[q] = (q < per && c < a.s.cpb) ? ccnt[c] : 0u;
                sum += k[q];
            }
            uint32_t run = sp_block_excl(L, sum);
#pragma unroll
            for (uint32_t q = 0; q < kCpt; q++) {
                const uint32_t c = tid * per + q;
                if (k[q]) {
                    const uint32_t slot = run / kSpHalf;
                    if (slot < a.maxg / 2) {
                        const uint32_t g = 2 * slot + (k[q] > kSpHalf ? 1u : 0u);
                        cgid[c] = g;
                        atomicAdd(&L.gtab[3 * g + 1], k[q]);
                        atomicMin(&L.gtab[3 * g + 2], c);
                    } else {
                        atomicMin(&L.cend, c);  // this cell opens the next window
                    }
                }
                run += k[q];
            }
            __syncthreads();
            // group starts: exclusive scan of the group counts (one per thread)
            const uint32_t gn_t = tid < a.maxg ? L.gtab[3 * tid + 1] : 0u;
            const uint32_t gs_t = sp_block_excl(L, gn_t);
            if (tid < a.maxg) { L.gtab[3 * tid] = gs_t; L.gcur[tid] = gs_t; }
            __syncthreads();
            const uint32_t ce = L.cend;
            sp_for8(a.words + b0, n, [&](uint32_t, uint64_t x) {
                const uint32_t c = (uint32_t)sp_cell(a.s, x >> 35);
                if (c >= cw && c < ce) a.words2[b0 + atomicAdd(&L.gcur[cgid[c]], 1u)] = x;
            });
            __syncthreads();
            for (uint32_t g = 0; g < a.maxg; g++) {
                const uint32_t gs = L.gtab[3 * g], gn = L.gtab[3 * g + 1], gf = L.gtab[3 * g + 2];
                if (gn == 0) continue;  // block-uniform
                __syncthreads();
                if (g & 1u) {
                    sp_giant(a, L, a.words2 + b0 + gs, gn, bin0seg, bin0cell + gf, gf);
                } else {
                    sp_for8(a.words2 + b0 + gs, gn, [&](uint32_t i, uint64_t x) { L.a[i] = x; });
                    __syncthreads();
                    sp_group(a, L, L.a, gn, bin0seg, bin0cell);
                }
            }
            __syncthreads();
            cw = ce;
        }
    }
}

}  // namespace gns

// ===========================================================================
// Host side
// ===========================================================================
using namespace gns;

struct gns_ss {
    int device = 0;
    hipStream_t stream = nullptr;
    SsGeom g{};
    KeyPlanN kpf{}, kpm{};
    uint32_t thr = 0;
    uint8_t *regs = nullptr;
    double *pbits = nullptr;
    uint32_t *values = nullptr, *keys = nullptr;
    DictDev D{};
    uint64_t dict_slots = 0;
    uint64_t max_flows = 0;  // dictionary capacity (gns_ss_params.max_flows)
    uint64_t claimed = 0;    // D.ctl[0] as of the last batch
    bool full = false;       // live flows + one batch piece exceed the dictionary (sticky)
    uint32_t *dctl = nullptr;
    DictScratch dsc;
    unsigned long long *stats_bak = nullptr;
    uint64_t n_reclaim = 0, n_dropped = 0, last_live = 0, n_retry = 0, n_grow = 0;
    double reclaim_ms = 0.0;
    uint32_t epoch = 0;
    uint64_t pkt = 0;     // records inserted since create (RNG packet index)
    bool s1_pipe = true;
    bool s1_nodict = false;  // pipelined S1 for header records (GNS_SS_PIPE=0: the plain loop)
    uint64_t n_encodes = 0, n_batches = 0;
    uint64_t bmax = 0;
    uint32_t nblk_max = 0;
    uint32_t *pcnt[2] = {nullptr, nullptr};
    uint32_t *ptotal = nullptr;
    uint64_t ccap = 0;
    // candidates (S1) -> ckey / cval; bin-major words (P3) -> ckey_s; P4 scratch
    // skey_s; encodes (P4) -> skey / sval.  After P4 the candidate buffers hold
    // S3b's parked lists, then S5's per-encode scratch.
    uint64_t *ckey = nullptr, *ckey_s = nullptr, *skey = nullptr, *skey_s = nullptr;
    uint32_t *cval = nullptr;
    uint64_t *sval = nullptr;
    uint32_t *counts = nullptr;  // [1] encodes, [2] P4 bin counter, [3] candidates (P2); [0] unused
    uint32_t *heads = nullptr;   // [cells + 1]: S5 segment starts (unordered), then their count
    uint32_t *hlen = nullptr;    // [cells]: encodes per segment
    uint32_t *cblk = nullptr;
    SpGeom sp{};
    uint32_t ncu = 0;
    uint32_t sp_maxg = 0;        // P4 groups per window of a large bin
    uint32_t sp_cap = kSpCap;    // encodes per cell and batch (GNS_SS_TEST_SPCAP, tests only)
    bool debug = false;          // GNS_SS_DEBUG
    unsigned long long *sprof = nullptr;  // [8] P4 phase ticks (debug)
    uint32_t *shist = nullptr;   // [nblk][nb] per-block bin histogram -> offsets
    uint32_t *spart = nullptr;   // [ngrp][nb] group partials, then [nb] bin starts
    uint32_t *sorder = nullptr;  // [nb] P4 schedule
    unsigned long long *stats = nullptr;
    uint32_t *h_pin = nullptr;
    uint8_t *stage = nullptr;
    size_t stage_bytes = 0;
    StageTimer timer;
    CmScratch *hh = nullptr;     // HeavyHitters' device list buffers (gns_hh.hpp), made on first use
};

namespace {

int ss_set_dev(gns_ss *ss) {
    (void)hipGetLastError();  // clear a stale error of an earlier runtime call on this thread
    GNS_HIP(hipSetDevice(ss->device));
    return GNS_OK;
}

void ss_free_all(gns_ss *ss) {
    dfree(ss->regs); dfree(ss->pbits); dfree(ss->values); dfree(ss->keys); dfree(ss->D.rec);
    dfree(ss->pcnt[0]); dfree(ss->pcnt[1]);
    dfree(ss->ptotal); dfree(ss->ckey); dfree(ss->ckey_s); dfree(ss->skey); dfree(ss->skey_s);
    dfree(ss->cval); dfree(ss->sval); dfree(ss->shist); dfree(ss->spart); dfree(ss->sorder);
    dfree(ss->counts); dfree(ss->heads); dfree(ss->hlen); dfree(ss->sprof); dfree(ss->cblk); dfree(ss->stats); dfree(ss->stage);
    dfree(ss->dctl); dfree(ss->stats_bak); ss->dsc.free_all();
    gns::hh_scratch_free(ss->hh);
    ss->hh = nullptr;
    if (ss->h_pin) (void)hipHostFree(ss->h_pin);
    ss->timer.destroy();
    if (ss->stream) (void)hipStreamDestroy(ss->stream);
}

int ss_reset_state(gns_ss *ss, bool init) {
    const uint64_t cells = (uint64_t)ss->g.d * ss->g.w;
    GNS_HIP(hipMemsetAsync(ss->regs, 0, cells * ss->g.m, ss->stream));
    GNS_HIP(hipMemsetAsync(ss->values, 0, cells * 4, ss->stream));
    GNS_HIP(hipMemsetAsync(ss->keys, 0xFF, cells * 4, ss->stream));
    GNS_HIP(hipMemsetAsync(ss->D.rec, 0, ss->dict_slots * ss->D.RW * 4, ss->stream));
    GNS_HIP(hipMemsetAsync(ss->stats + 3, 0, sizeof(unsigned long long), ss->stream));  // dict-full word
    GNS_HIP(hipMemsetAsync(ss->dctl, 0, 16, ss->stream));
    ss->claimed = 0;
    ss->full = false;
    if (init) {  // pbits starts at 1.0 (:44); Reset leaves it untouched (:297-311)
        std::vector<double> ones(cells, 1.0);
        GNS_HIP(hipMemcpyAsync(ss->pbits, ones.data(), cells * 8, hipMemcpyHostToDevice, ss->stream));
        GNS_HIP(hipStreamSynchronize(ss->stream));
    }
    return GNS_OK;
}

// S3b driver: flow ids of the encodes (sval high words; their count stays on
// the device), with the first-sight resolve rounds (a key claimed in this launch
// parks its other encodes until the claim is committed).  The candidate buffers
// are free after P4: ckey / ckey_s hold the parked lists.  Runs before any state
// is written, so an overflowing dictionary leaves the sketch unchanged.  The
// batch's one host round trip is here: after the second round, whether a third
// is needed (rarely) and whether the dictionary overflowed.
template <int KIND, int MF, int MM>
int ss_encode_ids(gns_ss *ss, const InputDesc &in) {
    hipStream_t s = ss->stream;
    const uint32_t grid = (uint32_t)std::min<uint64_t>((ss->ccap + kSsIdChunk - 1) / kSsIdChunk, 2048);
    uint64_t *pend[2] = {ss->ckey, ss->ckey_s};
    SsIdsArgs r{};
    r.in = in; r.kpf = ss->kpf; r.kpm = ss->kpm; r.g = ss->g; r.D = ss->D; r.ns = ss->counts + 1;
    r.skey = ss->skey; r.sval = ss->sval; r.stats = ss->stats;
    ScopedStage st(ss->timer, 1);
    GNS_HIP(hipMemsetAsync(ss->ptotal, 0, 8, s));
    int cur = 0;
    for (int round = 0;; round++) {
        if (++ss->epoch == 0) ss->epoch = 1;
        r.epoch = ss->epoch;
        r.pend_in = pend[cur]; r.cnt_in = ss->pcnt[cur];
        r.pend_out = pend[cur ^ 1]; r.cnt_out = ss->pcnt[cur ^ 1]; r.total_out = ss->ptotal + (cur ^ 1);
        if (round == 0) {
            r.pend_out = pend[0]; r.cnt_out = ss->pcnt[0]; r.total_out = ss->ptotal;
            hipLaunchKernelGGL((k_ss_ids<KIND, MF, MM, true>), dim3(grid), dim3(kSsThreads), 0, s, r);
        } else {
            hipLaunchKernelGGL((k_ss_ids<KIND, MF, MM, false>), dim3(grid), dim3(kSsThreads), 0, s, r);
            cur ^= 1;
        }
        GNS_HIP(hipGetLastError());
        // a fresh window parks the repeat encodes of every new flow: queue the
        // second round behind the first without a host round trip (an empty
        // parked list makes it a no-op; ptotal[1] was zeroed above)
        if (round == 0) continue;
        CtlRead rd;  // one launch writes the words into the pinned mirror
        rd.add(ss->ptotal + cur, 4, 0);
        rd.add(ss->stats + 3, 8, 2);
        rd.add(ss->dctl, 4, 4);
        if (round == 1) {
            rd.add(ss->counts + 1, 4, 5);
            rd.add(ss->stats + 6, 8, 6);
        }
        GNS_HIP(ctl_read(rd, ss->h_pin, s));
        GNS_HIP(hipStreamSynchronize(s));
        if (round == 1 && (ss->h_pin[6] | ss->h_pin[7])) {  // P4: a cell's encodes exceed kSpCap
            GNS_HIP(hipMemsetAsync(ss->stats + 6, 0, 8, s));
            set_error("a cell has more than %u encodes in one batch: use a smaller batch_packets", ss->sp_cap);
            return GNS_E_RANGE;
        }
        if (round == 1) ss->n_encodes += ss->h_pin[5];
        ss->claimed = ss->h_pin[4];
        if (ss->h_pin[2] | ss->h_pin[3]) {
            if (round == 1) ss->n_encodes -= ss->h_pin[5];  // the batch is re-run
            set_error("flow dictionary full (%llu slots)", (unsigned long long)ss->dict_slots);
            return GNS_E_FULL;
        }
        if (ss->h_pin[0] == 0) return GNS_OK;
        if (round > 64) { set_error("dictionary resolve did not converge"); return GNS_E_FULL; }
        GNS_HIP(hipMemsetAsync(ss->ptotal + (cur ^ 1), 0, 4, s));
    }
}

template <int KIND, int MF, int MM>
int ss_run_batch(gns_ss *ss, const InputDesc &in, uint64_t n) {
    if (n == 0) return GNS_OK;
    hipStream_t s = ss->stream;
    const uint32_t nblk = (uint32_t)((n + kSsChunk - 1) / kSsChunk);
    const uint32_t cells = ss->g.d * ss->g.w;
    const SpGeom &sg = ss->sp;
    ScopedStage total_stage(ss->timer, 5);
    {  // one launch: resolve totals, [1] encodes, [2] P4 bin counter, [3] candidates (P2), the
       // heads' end word, this batch's abort flag
        CtlZero z;
        z.add(ss->ptotal, 8);
        z.add(ss->counts, 16);
        z.add(ss->heads + cells, 4);
        z.add(ss->dctl + 1, 4);
        GNS_HIP(ctl_zero(z, s));
    }
    if (++ss->epoch == 0) ss->epoch = 1;
    SsExtractArgs x{};
    x.in = in; x.n = n; x.kpf = ss->kpf; x.kpm = ss->kpm;
    x.g = ss->g; x.regs = ss->regs;
    x.ckey = ss->ckey; x.cval = ss->cval; x.cblk = ss->cblk; x.stats = ss->stats;
    {
        ScopedStage st(ss->timer, 0);
        bool piped = false;
        if constexpr (KIND == IN_HDR && MF == PLAN_SLICE0 && MM == PLAN_SLICE0) {
            if (ss->s1_pipe && ss->g.Kf == 16 && ss->g.Km == 32 && ss->g.d == 2) {
                hipLaunchKernelGGL((k_ss_extract_hdr<MF, MM, 16, 32, 2>), dim3(nblk), dim3(kSsThreads), 0, s, x);
                piped = true;
            }
        }
        if (piped) {
        } else if (ss->g.Kf == 16 && ss->g.Km == 32)
            hipLaunchKernelGGL((k_ss_extract<KIND, MF, MM, 16, 32>), dim3(nblk), dim3(kSsThreads), 0, s, x);
        else
            hipLaunchKernelGGL((k_ss_extract<KIND, MF, MM, 0, 0>), dim3(nblk), dim3(kSsThreads), 0, s, x);
        GNS_HIP(hipGetLastError());
    }
    {   // P1-P4: candidates -> encodes sorted by (cell, packet), heads; no host round trip
        ScopedStage st(ss->timer, 2);
        const uint32_t ngrp = (nblk + kTGrp - 1) / kTGrp;
        const dim3 g2((sg.nb + 255) / 256, ngrp);
        uint32_t *tot = ss->spart + (size_t)ngrp * sg.nb;
        hipLaunchKernelGGL(k_sp_hist, dim3(nblk), dim3(256), 0, s, ss->ckey, ss->cblk, ss->g.d, sg, ss->shist);
        hipLaunchKernelGGL(k_tscan_part, g2, dim3(256), 0, s, ss->shist, nblk, sg.nb, ss->spart);
        hipLaunchKernelGGL(k_tscan_mid, dim3((sg.nb + 255) / 256), dim3(256), 0, s, ss->spart, ngrp, sg.nb, tot);
        hipLaunchKernelGGL(k_tscan_bins, dim3(1), dim3(1024), 0, s, tot, sg.nb, ss->counts + 3);
        hipLaunchKernelGGL(k_tscan_down, g2, dim3(256), 0, s, ss->shist, nblk, sg.nb, ss->spart, tot);
        if (ss->debug) {  // GNS_SS_DEBUG: the batch's bin sizes on stderr (synchronises; diagnosis only)
            std::vector<uint32_t> h(sg.nb + 1);
            GNS_HIP(hipMemcpyAsync(h.data(), tot, sg.nb * 4, hipMemcpyDeviceToHost, s));
            GNS_HIP(hipMemcpyAsync(h.data() + sg.nb, ss->counts + 3, 4, hipMemcpyDeviceToHost, s));
            GNS_HIP(hipStreamSynchronize(s));
            std::vector<uint32_t> sz(sg.nb);
            uint32_t big = 0;
            for (uint32_t b = 0; b < sg.nb; b++) { sz[b] = h[b + 1] - h[b]; big += sz[b] > kSpCap; }
            std::sort(sz.begin(), sz.end());
            fprintf(stderr, "gns_ss batch %llu: %u candidates, %u bins, %u above %u; largest %u %u %u, median %u\n",
                    (unsigned long long)ss->n_batches, h[sg.nb], sg.nb, big, kSpCap, sz[sg.nb - 1],
                    sg.nb > 1 ? sz[sg.nb - 2] : 0u, sg.nb > 2 ? sz[sg.nb - 3] : 0u, sz[sg.nb / 2]);
        }
        hipLaunchKernelGGL(k_sp_scatter, dim3(nblk), dim3(256), 0, s, ss->ckey, ss->cval, ss->cblk, ss->g.d, sg,
                           ss->shist, ss->ckey_s);
        SpArgs pa{};
        pa.s = sg; pa.words = ss->ckey_s; pa.words2 = ss->skey_s; pa.bstart = tot; pa.total = ss->counts + 3;
        pa.regs = ss->regs; pa.skey = ss->skey; pa.sval = ss->sval; pa.scount = ss->counts + 1;
        pa.heads = ss->heads; pa.hlen = ss->hlen; pa.work = ss->counts + 2; pa.err = ss->stats + 6;
        pa.maxg = ss->sp_maxg;
        pa.cap = ss->sp_cap;
        pa.prof = ss->debug ? ss->sprof : nullptr;
        if (ss->debug) GNS_HIP(hipMemsetAsync(ss->sprof, 0, 8 * 8, s));
        pa.order = ss->sorder;
        hipLaunchKernelGGL(k_sp_order, dim3(1), dim3(1024), 0, s, tot, ss->counts + 3, sg.nb, ss->sorder);
        hipLaunchKernelGGL(k_sp_bins, dim3(std::min(sg.nb, ss->ncu)), dim3(kSpThreads), sizeof(SpLds), s, pa);
        if (ss->debug) {
            unsigned long long h[8];
            GNS_HIP(hipMemcpyAsync(h, ss->sprof, sizeof h, hipMemcpyDeviceToHost, s));
            GNS_HIP(hipStreamSynchronize(s));
            const double g = h[7] ? (double)h[7] : 1.0;
            fprintf(stderr, "gns_ss P4: %llu groups; per group (memtime ticks) sort1 %.0f scan %.0f sort2 %.0f write %.0f tails %.0f\n",
                    h[7], h[0] / g, h[1] / g, h[2] / g, h[3] / g, h[4] / g);
            uint32_t nh = 0;
            GNS_HIP(hipMemcpy(&nh, ss->heads + cells, 4, hipMemcpyDeviceToHost));
            std::vector<uint32_t> hl(nh);
            if (nh) GNS_HIP(hipMemcpy(hl.data(), ss->hlen, nh * 4ull, hipMemcpyDeviceToHost));
            std::sort(hl.begin(), hl.end());
            uint64_t enc = 0, longc = 0, longe = 0;
            for (uint32_t v : hl) { enc += v; if (v > kSsLongChain) { longc++; longe += v; } }
            fprintf(stderr, "gns_ss chains: %u cells, %llu encodes, longest %u %u %u, median %u, %llu above %u holding %llu\n",
                    nh, (unsigned long long)enc, nh ? hl[nh - 1] : 0u, nh > 1 ? hl[nh - 2] : 0u, nh > 2 ? hl[nh - 3] : 0u,
                    nh ? hl[nh / 2] : 0u, (unsigned long long)longc, kSsLongChain, (unsigned long long)longe);
        }
        GNS_HIP(hipGetLastError());
    }
    GNS_TRY((ss_encode_ids<KIND, MF, MM>(ss, in)));
    {
        ScopedStage st(ss->timer, 3);
        // the candidate buffers are free now: pbits-before and repeat counts go there
        SsApplyArgs a{ss->skey, ss->sval, ss->counts + 1, ss->g, ss->pkt, ss->regs, ss->pbits, ss->values, ss->keys,
                      reinterpret_cast<double *>(ss->ckey), reinterpret_cast<int64_t *>(ss->skey_s), ss->heads,
                      ss->hlen, cells};
        const uint32_t hgrid = (cells + 255) / 256;  // one lane per touched cell at most
        const uint32_t egrid = (uint32_t)std::min<uint64_t>((ss->ccap + 255) / 256, 4096);
        hipLaunchKernelGGL(k_ss_walk_pbits, dim3(hgrid), dim3(256), 0, s, a);
        hipLaunchKernelGGL(k_ss_sample, dim3(egrid), dim3(256), 0, s, a);
        hipLaunchKernelGGL(k_ss_walk_mv, dim3(hgrid), dim3(256), 0, s, a);
        GNS_HIP(hipGetLastError());
    }
    ss->pkt += n;  // every record advances the RNG packet index
    ss->n_batches++;
    return GNS_OK;
}

// Reclaim (gns_dict.hip): only flows that own a cell (keys[]) can be named by a
// later comparison, query or heavy hitter; every other dictionary record is
// dropped.  The table doubles while the live flows exceed a quarter of it (live
// ids are at most d*w), and to at least min_slots.
void ss_dict_limits(gns_ss *ss) {
    ss->D.cap = (uint32_t)(ss->dict_slots - ss->dict_slots / 4);
    ss->max_flows = std::max<uint64_t>(ss->max_flows, ss->dict_slots / 2);
}

int ss_reclaim(gns_ss *ss, uint64_t min_slots = 0) {
    const uint64_t cells = (uint64_t)ss->g.d * ss->g.w;
    DictIds ids{ss->keys, cells};
    const auto t0 = std::chrono::steady_clock::now();
    const uint64_t before = ss->claimed, slots0 = ss->dict_slots;
    uint64_t live = 0;
    GNS_TRY(dict_rebuild(ss->D, ss->dict_slots, &ids, 1, nullptr, &ids, 1,
                         std::min(kDictMaxSlots, std::max(ss->dict_slots, min_slots)), ss->stream, ss->dsc, &live,
                         nullptr, kDictMaxSlots));
    ss->reclaim_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    ss->n_reclaim++;
    if (ss->dict_slots != slots0) ss->n_grow++;
    ss_dict_limits(ss);
    ss->n_dropped += before > live ? before - live : 0;
    ss->claimed = live;
    ss->last_live = live;
    return GNS_OK;
}

InputDesc ss_advance(const InputDesc &in, uint64_t off) {
    InputDesc d = in;
    if (d.hdr) d.hdr += off * 16;
    if (d.src16) d.src16 += off * 16;
    if (d.dst16) d.dst16 += off * 16;
    if (d.sport) d.sport += off;
    if (d.dport) d.dport += off;
    if (d.proto) d.proto += off;
    if (d.keys) d.keys += off * d.stride;
    if (d.keys2) d.keys2 += off * d.stride2;
    if (d.sizes) d.sizes += off;
    return d;
}

template <int KIND>
int ss_batch(gns_ss *ss, const InputDesc &d, uint64_t m) {
    if constexpr (KIND == IN_KEYS) {
        return ss_run_batch<KIND, PLAN_GENERIC, PLAN_GENERIC>(ss, d, m);
    } else if (plan_mode(ss->kpf) == PLAN_SLICE0 && plan_mode(ss->kpm) == PLAN_SLICE0) {
        return ss_run_batch<KIND, PLAN_SLICE0, PLAN_SLICE0>(ss, d, m);
    } else {
        return ss_run_batch<KIND, PLAN_GENERIC, PLAN_GENERIC>(ss, d, m);
    }
}

// A batch whose encodes overflow the dictionary is aborted in S3b, before any
// state write: undo its counters, reclaim, re-run it once, then in halves (the
// declared RNG is indexed by record, so the split does not change any draw); a
// piece of <= kSsChunk records that does not fit a fresh dictionary doubles the
// table instead, so every stream is counted (super_spread.go:182-235 has no
// failure mode).
template <int KIND>
int ss_batch_recover(gns_ss *ss, const InputDesc &d, uint64_t m, bool fresh) {
    if (m == 0) return GNS_OK;
    if (ss->full) {
        set_error("flow dictionary full (%llu slots, %llu live flows)", (unsigned long long)ss->dict_slots,
                  (unsigned long long)ss->last_live);
        return GNS_E_FULL;
    }
    if (ss->claimed >= ss->max_flows) {
        GNS_TRY(ss_reclaim(ss));
        fresh = true;
    }
    for (;;) {
        GNS_HIP(hipMemcpyAsync(ss->stats_bak, ss->stats, 3 * sizeof(unsigned long long), hipMemcpyDeviceToDevice,
                               ss->stream));
        const int rc = ss_batch<KIND>(ss, d, m);
        if (rc == GNS_E_RANGE && m > ss->sp_cap) {
            // P4: a cell got more than kSpCap encodes (S3b aborts before any state write).
            // Undo S1's counters and split: a cell takes at most one encode per record, so
            // pieces of <= kSpCap records always fit (the RNG is indexed by record, so the
            // split changes no draw)
            GNS_HIP(hipMemcpyAsync(ss->stats, ss->stats_bak, 3 * sizeof(unsigned long long), hipMemcpyDeviceToDevice,
                                   ss->stream));
            ss->n_retry++;
            const uint64_t h = m > 2ull * kSsChunk ? ((m / 2 + kSsChunk - 1) / kSsChunk) * kSsChunk : m / 2;
            GNS_TRY(ss_batch_recover<KIND>(ss, d, h, false));
            return ss_batch_recover<KIND>(ss, ss_advance(d, h), m - h, false);
        }
        if (rc != GNS_E_FULL) return rc;
        GNS_HIP(hipMemcpyAsync(ss->stats, ss->stats_bak, 3 * sizeof(unsigned long long), hipMemcpyDeviceToDevice,
                               ss->stream));
        GNS_HIP(hipMemsetAsync(ss->stats + 3, 0, sizeof(unsigned long long), ss->stream));
        ss->n_retry++;
        if (!fresh) {
            GNS_TRY(ss_reclaim(ss));
            fresh = true;
            continue;
        }
        if (m > kSsChunk) {
            GNS_TRY(ss_reclaim(ss));
            break;
        }
        if (ss->dict_slots >= kDictMaxSlots) {
            GNS_TRY(ss_reclaim(ss));
            ss->full = true;
            const unsigned long long one = 1;
            GNS_HIP(hipMemcpy(ss->stats + 3, &one, sizeof(one), hipMemcpyHostToDevice));
            set_error("flow dictionary full: %llu live flows plus one batch piece exceed %llu slots",
                      (unsigned long long)ss->last_live, (unsigned long long)ss->dict_slots);
            return GNS_E_FULL;
        }
        GNS_TRY(ss_reclaim(ss, ss->dict_slots * 2));
    }
    const uint64_t h = ((m / 2 + kSsChunk - 1) / kSsChunk) * kSsChunk;
    GNS_TRY(ss_batch_recover<KIND>(ss, d, h, true));
    return ss_batch_recover<KIND>(ss, ss_advance(d, h), m - h, false);
}

template <int KIND>
int ss_insert(gns_ss *ss, InputDesc in, uint64_t n, gns_mem where) {
    GNS_TRY(ss_set_dev(ss));
    for (uint64_t off = 0; off < n; off += ss->bmax) {
        const uint64_t m = std::min<uint64_t>(ss->bmax, n - off);
        InputDesc d = in;
        if (where == GNS_MEM_DEVICE) {
            d = ss_advance(in, off);
        } else {
            const void *src[8] = {in.hdr ? (const void *)(in.hdr + off * 16) : nullptr,
                                  in.src16 ? (const void *)(in.src16 + off * 16) : nullptr,
                                  in.dst16 ? (const void *)(in.dst16 + off * 16) : nullptr,
                                  in.sport ? (const void *)(in.sport + off) : nullptr,
                                  in.dport ? (const void *)(in.dport + off) : nullptr,
                                  in.proto ? (const void *)(in.proto + off) : nullptr,
                                  in.keys ? (const void *)(in.keys + off * in.stride) : nullptr,
                                  in.keys2 ? (const void *)(in.keys2 + off * in.stride2) : nullptr};
            const size_t bytes[8] = {in.hdr ? m * 64 : 0, in.src16 ? m * 16 : 0, in.dst16 ? m * 16 : 0,
                                     in.sport ? m * 2 : 0, in.dport ? m * 2 : 0, in.proto ? m : 0,
                                     in.keys ? m * in.stride : 0, in.keys2 ? m * in.stride2 : 0};
            size_t tot = 0;
            for (int i = 0; i < 8; i++) tot += (bytes[i] + 15) & ~size_t(15);
            tot += (m * 4 + 15) & ~size_t(15);
            if (ss->stage_bytes < tot) {
                dfree(ss->stage);
                ss->stage = nullptr;
                ss->stage_bytes = 0;
                GNS_TRY(dalloc(reinterpret_cast<void **>(&ss->stage), tot));
                ss->stage_bytes = tot;
            }
            uint8_t *p = ss->stage;
            const void **dst[8] = {(const void **)&d.hdr, (const void **)&d.src16, (const void **)&d.dst16,
                                   (const void **)&d.sport, (const void **)&d.dport, (const void **)&d.proto,
                                   (const void **)&d.keys, (const void **)&d.keys2};
            for (int i = 0; i < 8; i++) {
                if (!bytes[i]) continue;
                GNS_HIP(hipMemcpyAsync(p, src[i], bytes[i], hipMemcpyHostToDevice, ss->stream));
                *dst[i] = p;
                p += (bytes[i] + 15) & ~size_t(15);
            }
            if (in.sizes) {
                GNS_HIP(hipMemcpyAsync(p, in.sizes + off, m * 4, hipMemcpyHostToDevice, ss->stream));
                d.sizes = reinterpret_cast<const uint32_t *>(p);
            }
        }
        GNS_TRY(ss_batch_recover<KIND>(ss, d, m, false));
    }
    return GNS_OK;
}

}  // namespace

extern "C" {

int gns_ss_create(const gns_ss_params *p, gns_ss **out) {
    if (!p || !out) { set_error("null argument"); return GNS_E_ARG; }
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        (void)hipGetLastError();
        set_error("no HIP device available");
        return GNS_E_NODEV;
    }
    if (p->device < 0 || p->device >= ndev) { set_error("device %d out of range", p->device); return GNS_E_ARG; }
    gns_ss *ss = new gns_ss();
    ss->device = p->device;
    int rc = GNS_OK;
    do {
        if ((rc = ss_set_dev(ss)) != GNS_OK) break;
        SsGeom &g = ss->g;
        // super_spread.go:12-20,129-149 defaults
        g.w = p->width ? p->width : (1u << 20);
        g.d = p->depth ? p->depth : 3u;
        ss->thr = p->threshold ? p->threshold : 4096u;
        g.m = p->m ? p->m : 128u;
        const uint32_t size = p->size ? p->size : 5u;
        g.base = p->base != 0 ? p->base : 0.5;
        g.b = p->b != 0 ? p->b : 1.08;
        if (g.d > 8 || size > 8 || g.m > 256 || size == 0) {
            set_error("SuperSpread limits: depth <= 8, 1 <= size <= 8, m <= 256");
            rc = GNS_E_ARG;
            break;
        }
        g.maxv = (1u << size) - 1;
        if ((rc = make_plan(p->flow, p->flow_bytes, &ss->kpf)) != GNS_OK) break;
        KeyPlanN kpe;
        if ((rc = make_plan(p->elem, p->elem_bytes, &kpe)) != GNS_OK) break;
        g.Kf = ss->kpf.K;
        if (p->flow.n_fields || p->elem.n_fields) {
            if ((rc = make_plan2(p->flow, p->elem, &ss->kpm)) != GNS_OK) break;
        } else {
            ss->kpm.K = ss->kpf.K + kpe.K;
            ss->kpm.woff = -1;
        }
        g.Km = ss->kpf.K + kpe.K;
        if (g.Km > 74) { set_error("flow+elem key of %u bytes exceeds 74 (super_spread.go:20)", g.Km); rc = GNS_E_ARG; break; }
        g.pow2 = (g.w & (g.w - 1)) == 0;
        g.wmask = g.pow2 ? g.w - 1 : 0;
        if (p->seeds) for (uint32_t i = 0; i < g.d; i++) g.seeds[i] = p->seeds[i];
        else default_seeds(g.seeds, g.d);
        g.hll_master = p->hll_master;
        g.rng_seed = p->rng_seed;
        if ((uint64_t)g.d * g.w * g.m > (1ull << 36)) { set_error("d*w*m too large"); rc = GNS_E_ARG; break; }
        {   // P1-P4 bins: cpb (a power of two) consecutive cells, about 512 bins (P4's
            // fixed cost per bin outweighs fitting more bins in LDS whole: 512 / 1024 /
            // 2048 bins measured 0.54 / 0.70 / 1.01 ms per 100M; GNS_SS_BINS for A/B)
            SpGeom &sg = ss->sp;
            const uint64_t cells = (uint64_t)g.d * g.w;
            const char *benv = getenv("GNS_SS_BINS");
            const long tb = benv ? strtol(benv, nullptr, 10) : 512;
            const uint64_t target = (tb >= 64 && tb <= (long)kSpMaxBins) ? (uint64_t)tb : 512;
            sg.cpb = 1; sg.cpb_bits = 0;
            while ((uint64_t)sg.cpb * target < cells && sg.cpb < kSpMaxCpb) { sg.cpb <<= 1; sg.cpb_bits++; }
            const uint64_t nb = (cells + sg.cpb - 1) / sg.cpb;
            if (nb > kSpMaxBins) {
                set_error("SuperSpread: depth * width <= %u cells", kSpMaxBins * kSpMaxCpb);
                rc = GNS_E_ARG;
                break;
            }
            sg.nb = (uint32_t)nb;
            sg.m = g.m;
            sg.mbits = (g.m & (g.m - 1)) == 0 ? (uint32_t)__builtin_ctz(g.m) : 0xFFu;
            sg.lbits = 0;
            while ((1ull << sg.lbits) < (uint64_t)sg.cpb * g.m) sg.lbits++;
            sg.cells = (uint32_t)cells;
            int dev = 0, ncu = 0;
            if (hipGetDevice(&dev) != hipSuccess ||
                hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
                ncu = 256;
            ss->ncu = (uint32_t)ncu;
            ss->debug = getenv("GNS_SS_DEBUG") != nullptr;
            const char *env = getenv("GNS_SS_SPG");  // tests: small windows exercise the window loop
            const long v = env ? strtol(env, nullptr, 10) : 0;
            ss->sp_maxg = (v >= 2 && v <= (long)kSpMaxG) ? (uint32_t)(v & ~1L) : kSpMaxG;
            // tests: a lower per-cell encode cap makes the split-and-retry path of
            // ss_batch_recover reachable with ordinary streams (> 8192 encodes in one
            // cell needs m = 256 and registers climbing by 33 each)
            const char *ec = getenv("GNS_SS_TEST_SPCAP");
            const long c = ec ? strtol(ec, nullptr, 10) : 0;
            ss->sp_cap = (c >= 16 && c <= (long)kSpCap) ? (uint32_t)c : kSpCap;
        }
        if (hipStreamCreateWithFlags(&ss->stream, hipStreamNonBlocking) != hipSuccess) {
            set_error("hipStreamCreate failed"); rc = GNS_E_HIP; break;
        }
        ss->timer.stream = ss->stream;
        const uint64_t cells = (uint64_t)g.d * g.w;
        if ((rc = dalloc_t(&ss->regs, cells * g.m)) || (rc = dalloc_t(&ss->pbits, cells)) ||
            (rc = dalloc_t(&ss->values, cells)) || (rc = dalloc_t(&ss->keys, cells)) ||
            (rc = dalloc_t(&ss->heads, cells + 1)) || (rc = dalloc_t(&ss->hlen, cells)))
            break;
        uint64_t slots = 1;
        const uint64_t mf = p->max_flows ? p->max_flows : (4ull << 20);
        if (2 * mf > kDictMaxSlots) { set_error("max_flows > 2^29"); rc = GNS_E_ARG; break; }
        ss->max_flows = mf;
        while (slots < 2 * mf) slots <<= 1;
        ss->dict_slots = slots;
        ss->D.mask = (uint32_t)(slots - 1);
        ss->D.K = g.Kf;
        ss->D.RW = dict_record_words(g.Kf);
        ss->D.seed = 0x2545F491u;
        {
            const char *env = getenv("GNS_SS_PIPE");
            ss->s1_pipe = !(env && env[0] == '0');
        }
        if ((rc = dalloc_t(&ss->D.rec, slots * ss->D.RW)) != GNS_OK) break;
        if ((rc = dalloc_t(&ss->dctl, 4)) != GNS_OK || (rc = dalloc_t(&ss->stats_bak, 3)) != GNS_OK) break;
        ss->D.ctl = ss->dctl;
        ss_dict_limits(ss);
        ss->bmax = p->batch_packets ? p->batch_packets : (8ull << 20);
        ss->bmax = std::min<uint64_t>(((ss->bmax + kSsChunk - 1) / kSsChunk) * kSsChunk, 1ull << kSsPktBits);
        ss->nblk_max = (uint32_t)(ss->bmax / kSsChunk);
        ss->ccap = ss->bmax * g.d;
        const uint64_t nblk_enc = (ss->ccap + kSsIdChunk - 1) / kSsIdChunk;  // S3b blocks over encodes
        if ((rc = dalloc_t(&ss->pcnt[0], nblk_enc)) ||
            (rc = dalloc_t(&ss->pcnt[1], nblk_enc)) || (rc = dalloc_t(&ss->ptotal, 2)) ||
            (rc = dalloc_t(&ss->ckey, ss->ccap)) || (rc = dalloc_t(&ss->ckey_s, ss->ccap)) ||
            (rc = dalloc_t(&ss->skey, ss->ccap)) || (rc = dalloc_t(&ss->skey_s, ss->ccap)) ||
            (rc = dalloc_t(&ss->cval, ss->ccap)) || (rc = dalloc_t(&ss->sval, ss->ccap)) ||
            (rc = dalloc_t(&ss->counts, 4)) || (rc = dalloc_t(&ss->cblk, 2ull * ss->nblk_max)) ||
            (rc = dalloc_t(&ss->shist, (uint64_t)ss->nblk_max * ss->sp.nb)) ||
            (rc = dalloc_t(&ss->spart, ((uint64_t)(ss->nblk_max + kTGrp - 1) / kTGrp + 1) * ss->sp.nb)) ||
            (rc = dalloc_t(&ss->sorder, ss->sp.nb)) || (rc = dalloc_t(&ss->sprof, 8)) || (rc = dalloc_t(&ss->stats, 8)))
            break;
        if (hipHostMalloc(reinterpret_cast<void **>(&ss->h_pin), 64, 0) != hipSuccess) {
            set_error("hipHostMalloc failed"); rc = GNS_E_OOM; break;
        }
        if (hipMemsetAsync(ss->stats, 0, 64, ss->stream) != hipSuccess) { rc = GNS_E_HIP; break; }
        if ((rc = ss_reset_state(ss, true)) != GNS_OK) break;
    } while (0);
    if (rc != GNS_OK) {
        ss_free_all(ss);
        delete ss;
        return rc;
    }
    *out = ss;
    return GNS_OK;
}

int gns_ss_destroy(gns_ss *ss) {
    if (!ss) return GNS_OK;
    (void)hipSetDevice(ss->device);
    if (ss->stream) (void)hipStreamSynchronize(ss->stream);
    ss_free_all(ss);
    delete ss;
    return GNS_OK;
}

int gns_ss_insert_keys(gns_ss *ss, const uint8_t *flows, uint32_t fstride, const uint8_t *elems,
                       uint32_t estride, uint64_t n, gns_mem where) {
    if (!ss || (n && (!flows || (!elems && ss->g.Km > ss->g.Kf)))) { set_error("null argument"); return GNS_E_ARG; }
    if (fstride < ss->g.Kf || estride < ss->g.Km - ss->g.Kf) { set_error("stride smaller than key"); return GNS_E_ARG; }
    InputDesc in{};
    in.keys = flows; in.stride = fstride; in.keys2 = elems ? elems : flows; in.stride2 = estride;
    return ss_insert<IN_KEYS>(ss, in, n, where);
}

int gns_ss_insert_tuples(gns_ss *ss, const gns_tuples *t, uint64_t n, gns_mem where) {
    if (!ss || !t) { set_error("null argument"); return GNS_E_ARG; }
    if (n && (!t->src16 || !t->dst16 || !t->sport || !t->dport || !t->proto)) { set_error("null tuple array"); return GNS_E_ARG; }
    InputDesc in{};
    in.src16 = t->src16; in.dst16 = t->dst16; in.sport = t->sport; in.dport = t->dport; in.proto = t->proto;
    in.sizes = t->length;
    return ss_insert<IN_TUPLE>(ss, in, n, where);
}

int gns_ss_insert_headers(gns_ss *ss, const uint8_t *hdr, const uint32_t *wirelen, uint64_t n, gns_mem where) {
    if (!ss || (n && (!hdr || !wirelen))) { set_error("null argument"); return GNS_E_ARG; }
    InputDesc in{};
    in.hdr = reinterpret_cast<const uint32_t *>(hdr);
    in.sizes = wirelen;
    return ss_insert<IN_HDR>(ss, in, n, where);
}

int gns_ss_flush(gns_ss *ss) {
    if (!ss) return GNS_E_ARG;
    GNS_TRY(ss_set_dev(ss));
    GNS_HIP(hipStreamSynchronize(ss->stream));
    ss->timer.collect();
    return GNS_OK;
}

static int ss_query_impl(gns_ss *ss, const uint8_t *flows, uint32_t stride, uint64_t n, uint64_t *out, bool dev) {
    if (!ss || (n && (!flows || !out))) { set_error("null argument"); return GNS_E_ARG; }
    if (n == 0) return GNS_OK;
    if (stride < ss->g.Kf) { set_error("stride < flow_bytes"); return GNS_E_ARG; }
    if (dev && ((uintptr_t)out & 7u) != 0) { set_error("answers not 8-byte aligned"); return GNS_E_ARG; }
    GNS_TRY(ss_set_dev(ss));
    uint8_t *dk = nullptr;
    uint64_t *dout = nullptr;
    if (dev) {
        dk = const_cast<uint8_t *>(flows);
        dout = out;
    } else {
        GNS_TRY(dalloc(reinterpret_cast<void **>(&dk), n * stride));
        int rc = dalloc(reinterpret_cast<void **>(&dout), n * 8);
        if (rc) { dfree(dk); return rc; }
    }
    SsQueryArgs a{dk, stride, n, ss->g, ss->D, ss->values, ss->keys, dout};
    hipError_t e = dev ? hipSuccess : hipMemcpyAsync(dk, flows, n * stride, hipMemcpyHostToDevice, ss->stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_ss_query, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ss->stream, a);
        e = hipGetLastError();
    }
    if (e == hipSuccess && !dev) e = hipMemcpyAsync(out, dout, n * 8, hipMemcpyDeviceToHost, ss->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ss->stream);
    if (!dev) {
        dfree(dk);
        dfree(dout);
    }
    if (e != hipSuccess) { set_error("ss query: %s", hipGetErrorString(e)); return GNS_E_HIP; }
    return GNS_OK;
}

int gns_ss_query(gns_ss *ss, const uint8_t *flows, uint32_t stride, uint64_t n, uint64_t *out) {
    return ss_query_impl(ss, flows, stride, n, out, false);
}

int gns_ss_query_device(gns_ss *ss, const uint8_t *flows, uint32_t stride, uint64_t n, uint64_t *out) {
    return ss_query_impl(ss, flows, stride, n, out, true);
}

static int ss_ids_to_bytes(gns_ss *ss, const std::vector<uint32_t> &ids, std::vector<uint8_t> &bytes) {
    const uint32_t K = ss->g.Kf;
    bytes.assign(ids.size() * (K ? K : 1), 0);
    if (ids.empty() || K == 0) return GNS_OK;
    uint32_t *dids = nullptr;
    uint8_t *db = nullptr;
    GNS_TRY(dalloc(reinterpret_cast<void **>(&dids), ids.size() * 4));
    int rc = dalloc(reinterpret_cast<void **>(&db), ids.size() * K);
    if (rc) { dfree(dids); return rc; }
    hipError_t e = hipMemcpy(dids, ids.data(), ids.size() * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_ss_ids_to_bytes, dim3((unsigned)((ids.size() + 255) / 256)), dim3(256), 0,
                           ss->stream, dids, (uint64_t)ids.size(), ss->D, db);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(bytes.data(), db, ids.size() * K, hipMemcpyDeviceToHost, ss->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ss->stream);
    dfree(dids);
    dfree(db);
    if (e != hipSuccess) { set_error("ss ids_to_bytes: %s", hipGetErrorString(e)); return GNS_E_HIP; }
    return GNS_OK;
}

// HeavyHitters (super_spread.go:254-294) on the device.  The reference collects
// every flow holding a counter > 0, re-queries it (the max over the cells holding
// it) and keeps estimates >= threshold: a flow clears the threshold iff one of its
// cells does, so this is Count-Min's list computation over (values, keys) with
// the threshold (gns::hh_heavy_list: candidates >= thr, per-flow max, radix
// order).  Order: estimate desc, ties by flow bytes asc (Go's sort.Slice leaves
// them unordered).  Nothing but the list leaves the device.
int gns_ss_heavy_hitters(gns_ss *ss, uint8_t *flows, uint32_t *spreads, uint64_t *n_io) {
    if (!ss || !n_io) { set_error("null argument"); return GNS_E_ARG; }
    GNS_TRY(ss_set_dev(ss));
    GNS_HIP(hipStreamSynchronize(ss->stream));
    if (!ss->hh) ss->hh = gns::hh_scratch_new();
    const uint64_t cells = (uint64_t)ss->g.d * ss->g.w;
    return gns::hh_heavy_list(ss->hh, ss->stream, ss->D, ss->dict_slots, ss->g.Kf, cells, ss->values, ss->keys,
                              ss->thr, flows, spreads, n_io);
}

int gns_ss_reset(gns_ss *ss) {
    if (!ss) return GNS_E_ARG;
    GNS_TRY(ss_set_dev(ss));
    GNS_TRY(ss_reset_state(ss, false));
    GNS_HIP(hipStreamSynchronize(ss->stream));
    return GNS_OK;
}

int gns_ss_export_state(gns_ss *ss, uint32_t *values, uint8_t *keys, uint8_t *regs, double *pbits) {
    if (!ss) return GNS_E_ARG;
    GNS_TRY(ss_set_dev(ss));
    GNS_HIP(hipStreamSynchronize(ss->stream));
    const uint64_t cells = (uint64_t)ss->g.d * ss->g.w;
    if (values) GNS_HIP(hipMemcpy(values, ss->values, cells * 4, hipMemcpyDeviceToHost));
    if (regs) GNS_HIP(hipMemcpy(regs, ss->regs, cells * ss->g.m, hipMemcpyDeviceToHost));
    if (pbits) GNS_HIP(hipMemcpy(pbits, ss->pbits, cells * 8, hipMemcpyDeviceToHost));
    if (keys) {
        std::vector<uint32_t> ids(cells);
        GNS_HIP(hipMemcpy(ids.data(), ss->keys, cells * 4, hipMemcpyDeviceToHost));
        std::vector<uint8_t> kb;
        GNS_TRY(ss_ids_to_bytes(ss, ids, kb));
        if (ss->g.Kf) memcpy(keys, kb.data(), cells * ss->g.Kf);
    }
    return GNS_OK;
}

int gns_ss_stats(gns_ss *ss, uint64_t stats[4]) {
    if (!ss || !stats) return GNS_E_ARG;
    GNS_TRY(ss_set_dev(ss));
    GNS_HIP(hipStreamSynchronize(ss->stream));
    unsigned long long h[8];
    GNS_HIP(hipMemcpy(h, ss->stats, sizeof(h), hipMemcpyDeviceToHost));
    stats[0] = h[0]; stats[1] = h[1]; stats[2] = h[2]; stats[3] = ss->pkt;
    return GNS_OK;
}

int gns_ss_counters(gns_ss *ss, uint64_t out[8]) {
    if (!ss || !out) return GNS_E_ARG;
    GNS_TRY(ss_set_dev(ss));
    GNS_HIP(hipStreamSynchronize(ss->stream));
    unsigned long long h[8];
    GNS_HIP(hipMemcpy(h, ss->stats, sizeof(h), hipMemcpyDeviceToHost));
    out[0] = h[0]; out[1] = h[1]; out[2] = h[2]; out[3] = h[3]; out[4] = h[4];
    out[5] = ss->n_encodes; out[6] = ss->pkt; out[7] = ss->n_batches;
    return GNS_OK;
}

int gns_ss_reclaim(gns_ss *ss) {
    if (!ss) return GNS_E_ARG;
    GNS_TRY(ss_set_dev(ss));
    return ss_reclaim(ss);
}

int gns_ss_dict_stats(gns_ss *ss, uint64_t out[8]) {
    if (!ss || !out) return GNS_E_ARG;
    out[0] = ss->n_reclaim; out[1] = ss->n_dropped; out[2] = ss->last_live; out[3] = ss->claimed;
    out[4] = (uint64_t)(ss->reclaim_ms * 1000.0); out[5] = ss->n_retry;
    out[6] = ss->dict_slots; out[7] = ss->n_grow;
    return GNS_OK;
}

int gns_ss_set_timing(gns_ss *ss, int on) {
    if (!ss) return GNS_E_ARG;
    set_timing_arg(ss->timer, on);
    return GNS_OK;
}

int gns_ss_stage_times(gns_ss *ss, double ms[8], uint64_t launches[8], int reset) {
    if (!ss) return GNS_E_ARG;
    GNS_TRY(ss_set_dev(ss));
    ss->timer.collect();
    for (int i = 0; i < 8; i++) {
        if (ms) ms[i] = ss->timer.ms[i];
        if (launches) launches[i] = ss->timer.launches[i];
    }
    if (reset) for (int i = 0; i < 8; i++) { ss->timer.ms[i] = 0; ss->timer.launches[i] = 0; }
    return GNS_OK;
}

}  // extern "C"
