// gns_exact.hip -- MI355X engine for Go2NetSpectra's exact aggregator
// (internal/engine/impl/exact/task.go): per-flow PacketCount, ByteCount,
// StartTime (first packet) and EndTime (last packet, in stream order).
//
// Keys: the reference keys flows by the STRING strings.Join(fields, "-")
// with IPs printed by net.IP.String() (generateKeyAndFields, task.go:330-366).
// Two IPs print the same exactly when their 16-byte forms (To16) are equal:
// IPv4 (4-byte) and IPv4-mapped IPv6 both print as a dotted quad, every other
// IPv6 prints its 16 bytes.  The engine therefore keys flows by the key bytes
// of the sketch layout (task.go:265-300) with every IP field in To16 form, in
// the flow dictionary of gns_keys.cuh (full key bytes, exact compare).
//
// Nothing in task.go:124-149 depends on packet order except which packet is
// the flow's first and last: PacketCount / ByteCount are sums, StartTime is
// the timestamp of the packet with the smallest stream index, EndTime that of
// the largest.  So every path below produces per-flow (count, bytes, min
// index, max index) contributions, merged with add / min / max, and the
// timestamps are looked up once per batch from the merged indices.
//
//   X1  k_ex_extract   parse -> To16 tuple -> key -> flow id (dictionary);
//                      packets of the batch's designated heavy flows (the 512
//                      flows with the most packets so far) are aggregated in
//                      LDS per block (per-block partials), every other packet
//                      writes a 64-bit word (flow id | packet index | length)
//   X1b k_ex_resolve   re-probe packets parked on a same-launch claim
//   H   k_ex_hot_reduce  the partials of each designated flow -> flow state
//   P   k_ex_phist / k_ex_pscan_* / k_ex_pscatter / k_ex_pagg  X1 writes the
//                      words of the other flows (the tail: about 35% of a
//                      Zipf(1.1) stream) at the start of its block's region; they
//                      are partitioned into 512 bins of consecutive flow ids and
//                      each bin is aggregated in an LDS hash table by one
//                      workgroup, which merges each of its flows once
//   T   k_ex_times     StartTime / EndTime of the flows the batch touched
//   D   k_exh_*        designate the next batch's heavy flows
// A Zipf batch touches a flow in many places; per-block LDS aggregation of
// every flow left the tail flows to global atomics, three per packet; sorting
// every packet (rocPRIM radix sort of 100M words) made the sort the largest
// stage.  Designation sends the heavy flows through LDS; the tail needs no
// order at all (add / min / max), only locality by flow id.
#include <algorithm>
#include <chrono>
#include <cstring>
#include <vector>

#include "gns_common.hpp"
#include "gns_xcd.cuh"

namespace gns {

constexpr int kXThreads = 256;

constexpr uint32_t kXChunk = 16384;

// Designated heavy flows: kExHot per batch, looked up by flow id in a 4-way
// table of kExHotTab entries (id << 16 | hot slot; empty = ~0) that X1 keeps in LDS.
#ifndef GNS_EX_HOT_BITS
#define GNS_EX_HOT_BITS 9
#endif
constexpr uint32_t kExHotBits = GNS_EX_HOT_BITS;
constexpr uint32_t kExHot = 1u << kExHotBits;
constexpr uint32_t kExHotTab = 4 * kExHot;
constexpr uint32_t kExHotMinKey = 6 * 8;  // designate only flows with >= 64 packets
// One designated flow in one X1 block: bytes << 15 | packets (a block has at
// most 2^14 packets of < 2^32 bytes, so neither field carries into the other)
// and the largest packet index in the block.  No first-packet index: a flow is
// designated only with >= 64 packets counted, so its first packet is known.
constexpr uint32_t kHotCntBits = 15;
static_assert(kXChunk < (1u << kHotCntBits), "per-block packet count field");
struct ExHotPart {
    unsigned long long cb;
    uint32_t maxp, pad;
};
__device__ __forceinline__ uint32_t exh_group(uint32_t id) { return (id * 0x9E3779B1u) >> (32 - kExHotBits); }
__device__ __forceinline__ int exh_lookup(const unsigned long long *tab, uint32_t id) {
    const ulonglong2 *g = reinterpret_cast<const ulonglong2 *>(tab + exh_group(id) * 4);
    const ulonglong2 a = g[0], b = g[1];
    int h = -1;
    constexpr unsigned long long m = kExHot - 1u;
    h = (b.y >> 16) == id ? (int)(b.y & m) : h;
    h = (b.x >> 16) == id ? (int)(b.x & m) : h;
    h = (a.y >> 16) == id ? (int)(a.y & m) : h;
    h = (a.x >> 16) == id ? (int)(a.x & m) : h;
    return h;
}

struct ExIn {
    InputDesc in;
    const uint8_t *ipver;  // IN_TUPLE: 4 / 6 per packet (NULL -> 4)
    const int64_t *ts;
};

// IPv4 (4-byte net.IP, left-aligned in its slot) -> ::ffff:a.b.c.d, the form
// in which it compares equal to the same address arriving IPv4-mapped.
__device__ __forceinline__ void to16(uint32_t (&tw)[10], uint32_t sver, uint32_t dver) {
    if (sver == 4u) { tw[3] = tw[0]; tw[0] = 0u; tw[1] = 0u; tw[2] = 0xFFFF0000u; }
    if (dver == 4u) { tw[7] = tw[4]; tw[4] = 0u; tw[5] = 0u; tw[6] = 0xFFFF0000u; }
}

// canonical tuple words (load_tuple) -> exact key with To16 IP fields
template <int KIND, int MODE>
__device__ __forceinline__ int ex_key_tw(const ExIn &x, uint32_t K, const uint8_t *s_src, uint64_t p,
                                         uint32_t (&tw)[10], uint32_t (&kw)[GNS_KWMAX]) {
    uint32_t sv, dv;
    if constexpr (KIND == IN_HDR) { sv = tw[9] >> 24; dv = (tw[9] >> 16) & 0xFFu; }
    else { sv = dv = x.ipver ? x.ipver[p] : 4u; }
    // a net.IP of neither 4 nor 16 bytes prints as "?<hex>" / "<nil>" (net/ip.go):
    // outside the canonical form, counted as unsupported
    if (sv == 0u || dv == 0u) return PARSE_UNSUPPORTED;
    to16(tw, sv, dv);
    tw[9] &= 0xFFu;
    make_key_m<MODE, GNS_KWMAX>(K, s_src, tw, kw);
    return PARSE_OK;
}

template <int KIND, int MODE>
__device__ __forceinline__ int ex_key(const ExIn &x, uint32_t K, const uint8_t *s_src, uint64_t p,
                                      uint32_t (&kw)[GNS_KWMAX]) {
    uint32_t tw[10];
    const int st = load_tuple<KIND>(x.in, p, tw);
    if (st != PARSE_OK) return st;
    return ex_key_tw<KIND, MODE>(x, K, s_src, p, tw, kw);
}

struct ExArgs {
    ExIn x;
    uint64_t n;
    KeyPlanN kp;
    DictDev D;
    uint32_t epoch;
    uint64_t *sk;        // X2 sort words: flow id | packet index | wire length (SortWord)
    uint32_t none_key;   // flow field of a packet without a flow id (sorts last)
    uint32_t hot_key;    // flow field of a designated flow's packet (none_key + 1: not sorted)
    uint32_t sb, ib;     // SortWord field widths: wire length, packet index
    const unsigned long long *hot_tab;  // [kExHotTab] designated flows
    ExHotPart *hpart;    // [kExHot][nblk] per-block partials
    uint32_t *ccnt;      // [nblk] words X1 wrote at the start of its block's region
    uint32_t nblk;
    uint64_t *pend;
    uint32_t *pend_cnt, *pend_total;
    unsigned long long *stats;  // 0 inserted, 1 dropped, 2 unsupported, 3 dict full
};

// X2 sorts one 64-bit word per packet: flow id in the top bits (the radix sort's
// key range), then the packet index within the batch (ib bits), then the wire
// length (sb bits; a length >= 2^sb - 1 is stored as the escape 2^sb - 1 and
// read back from the batch's length array by X3).  A keys-only sort of 8 bytes
// per packet instead of 4-byte keys with 8-byte values.
__device__ __forceinline__ uint64_t sort_word(uint32_t flow, uint64_t idx, uint32_t size, uint32_t sb,
                                              uint32_t ib) {
    const uint32_t esc = (1u << sb) - 1u;
    return (uint64_t)flow << (ib + sb) | idx << sb | (size < esc ? size : esc);
}

// Home-slot record of a key (issued early; consumed by ex_consume).
__device__ __forceinline__ void ex_probe_issue(const DictDev &D, uint32_t slot, uint4 (&r4)[4]) {
    const uint4 *q = reinterpret_cast<const uint4 *>(D.rec + (size_t)slot * D.RW);
#pragma unroll
    for (int i = 0; i < 4; i++) r4[i] = (4u * i < D.RW) ? q[i] : make_uint4(0, 0, 0, 0);
}

// X1 second half for one packet: resolve the home-slot probe.  A hit gives the
// flow id; a flow displaced from its home slot by another committed key is parked
// (k_ex_resolve walks the rest of the chain in the next launch) instead of
// stalling the wave on dependent probes; an empty home slot is claimed here.
struct ExHotLds {
    const unsigned long long *tab;
    unsigned long long *cb;
    uint32_t *maxp;
};

constexpr uint64_t kNoWord = ~0ull;
// Word of a packet of an undesignated flow, written densely at the start of the
// block's region (ballot + one LDS add per wave); returns its position in the
// region (parked packets record it for k_ex_resolve), or ~0u for no word.
__device__ __forceinline__ uint32_t ex_emit(const ExArgs &a, uint64_t beg, uint64_t w, uint32_t *s_ncold) {
    const bool has = w != kNoWord;
    const uint64_t m = __ballot(has);
    if (!m) return ~0u;
    const uint32_t lane = __lane_id();
    const uint32_t leader = (uint32_t)__ffsll((long long)m) - 1u;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(s_ncold, (uint32_t)__popcll(m));
    base = __shfl(base, (int)leader);
    const uint32_t q = base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    if (has) a.sk[beg + q] = w;
    return has ? q : ~0u;
}

// X1 second half for one packet; returns the packet's word (kNoWord: none) and
// whether it is parked (*park: the dictionary slot to resume from).
__device__ __forceinline__ uint64_t ex_consume(const ExArgs &a, uint64_t p, uint64_t beg, bool ok,
                                               const uint32_t (&kw)[GNS_KWMAX], uint32_t K, uint32_t slot0,
                                               const uint4 (&r4)[4], uint32_t sz, uint32_t *s_full,
                                               uint32_t *s_claim, uint32_t &n_ok, const ExHotLds &H,
                                               uint32_t &park) {
    park = ~0u;
    if (!ok) return kNoWord;
    uint32_t rec[16];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        rec[4 * i] = r4[i].x; rec[4 * i + 1] = r4[i].y; rec[4 * i + 2] = r4[i].z; rec[4 * i + 3] = r4[i].w;
    }
    const uint32_t tag = rec[0];
    bool eq = tag != 0 && tag != a.epoch;
#pragma unroll
    for (int i = 0; i < GNS_KWMAX; i++)
        if ((uint32_t)i < ((K + 3) >> 2)) eq = eq && (rec[1 + i] == kw[i]);
    uint32_t out = slot0;
    int r = DICT_FOUND;
    if (eq) {  // a designated flow: aggregated in LDS, no word to sort
        const int h = exh_lookup(H.tab, out);
        if (h >= 0) {
            const uint32_t lp = (uint32_t)(p - beg);
            atomicAdd(&H.cb[h], (unsigned long long)sz << kHotCntBits | 1ull);
            atomicMax(&H.maxp[h], lp);
            n_ok++;
            return kNoWord;
        }
    } else {
        if (tag == a.epoch) r = DICT_PENDING;                                    // claimed in this launch
        else if (tag != 0) { r = DICT_PENDING; out = (slot0 + 1u) & a.D.mask; }  // displaced
        else r = dict_find_or_claim(a.D, kw, slot0, a.epoch, &out);              // empty: claim
    }
    if (r == DICT_CLAIMED) {
        atomicAdd(s_claim, 1u);
        r = DICT_FOUND;
    }
    if (r == DICT_FULL) {
        atomicAdd(s_full, 1u);
        return kNoWord;
    }
    n_ok++;
    // a parked packet's word keeps none_key until k_ex_resolve fills in its flow id
    if (r != DICT_FOUND) park = out;
    return sort_word(r == DICT_FOUND ? out : a.none_key, p, sz, a.sb, a.ib);
}

// pend entry: packet (14 bits) | word position (14 bits) in the block | slot to resume from
static_assert(kXChunk <= (1u << 14), "pend entries hold 14-bit block offsets");
__device__ __forceinline__ uint64_t pend_entry(uint32_t lp, uint32_t q, uint32_t slot) {
    return (uint64_t)lp << 50 | (uint64_t)q << 36 | slot;
}
__device__ __forceinline__ void ex_emit_park(const ExArgs &a, uint64_t beg, uint64_t p, uint64_t w, uint32_t park,
                                             uint32_t *s_ncold, uint32_t *s_pend) {
    const uint32_t q = ex_emit(a, beg, w, s_ncold);
    if (park != ~0u) a.pend[beg + atomicAdd(s_pend, 1u)] = pend_entry((uint32_t)(p - beg), q, park);
}

template <int KIND, int MODE>
__global__ __launch_bounds__(kXThreads) void k_ex_extract(ExArgs a) {
    __shared__ uint8_t s_src[80];
    __shared__ uint32_t s_pend, s_drop, s_unsup, s_full, s_ok, s_claim, s_abort, s_ncold;
    __shared__ __attribute__((aligned(16))) unsigned long long s_htab[kExHotTab];
    __shared__ unsigned long long s_hcb[kExHot];
    __shared__ uint32_t s_hmax[kExHot];
    const uint32_t tid = threadIdx.x, blk = blockIdx.x;
    if (tid == 0) { s_pend = 0; s_drop = 0; s_unsup = 0; s_full = 0; s_ok = 0; s_claim = 0; s_ncold = 0; s_abort = dict_aborted(a.D); }
    for (uint32_t i = tid; i < kExHotTab; i += kXThreads) s_htab[i] = a.hot_tab[i];
    for (uint32_t i = tid; i < kExHot; i += kXThreads) { s_hcb[i] = 0; s_hmax[i] = 0; }
    const ExHotLds H{s_htab, s_hcb, s_hmax};
    __syncthreads();
    if (s_abort) {  // the batch overflowed the dictionary: re-run after the table grows
        if (tid == 0) a.pend_cnt[blk] = 0;
        return;
    }
    stage_plan<MODE>(a.kp, s_src);
    const uint32_t K = a.kp.K;
    const uint64_t beg = (uint64_t)blk * kXChunk;
    const uint64_t end = min(a.n, beg + kXChunk);
    uint32_t n_ok = 0;
    if constexpr (KIND == IN_HDR) {
        // Two-stage software pipeline (as Count-Min's K1): iteration k parses packet
        // k+1 and issues its home-slot probe (and the record prefetch of packet k+2),
        // then consumes packet k, whose probe was issued one iteration earlier.
        uint4 hv[4];
        uint32_t hsz;
        auto load_hdr = [&](uint64_t q) {
            const uint64_t pc = min(q, end - 1);
            const uint4 *r = reinterpret_cast<const uint4 *>(a.x.in.hdr + pc * 16);
#pragma unroll
            for (int i = 0; i < 4; i++) hv[i] = r[i];
            hsz = a.x.in.sizes[pc];
        };
        auto stage_b = [&](uint64_t q, bool &okq, uint32_t (&kwq)[GNS_KWMAX], uint32_t &slotq, uint4 (&r4q)[4],
                           uint32_t &szq) {
            okq = q < end;
            uint32_t cw[16];
#pragma unroll
            for (int i = 0; i < 4; i++) { cw[4 * i] = hv[i].x; cw[4 * i + 1] = hv[i].y; cw[4 * i + 2] = hv[i].z; cw[4 * i + 3] = hv[i].w; }
            szq = hsz;
            load_hdr(q + kXThreads);
#pragma unroll
            for (int i = 0; i < GNS_KWMAX; i++) kwq[i] = 0;
            if (okq) {
                uint32_t tw[10];
                int st = parse_record_fast(cw, szq, true, tw);
                if (st == PARSE_OK) st = ex_key_tw<KIND, MODE>(a.x, K, s_src, q, tw, kwq);
                if (st != PARSE_OK) {
                    atomicAdd(st == PARSE_DROP ? &s_drop : &s_unsup, 1u);
                    okq = false;
                }
            }
            slotq = mm3_n<GNS_KWMAX>(kwq, K, a.D.seed) & a.D.mask;
            if (okq) ex_probe_issue(a.D, slotq, r4q);
        };
        load_hdr(beg + tid);
        bool okc;
        uint32_t kwc[GNS_KWMAX], slotc, szc;
        uint4 r4c[4];
        stage_b(beg + tid, okc, kwc, slotc, r4c, szc);
        for (uint64_t p0 = beg; p0 < end; p0 += kXThreads) {  // wave-uniform trip count
            bool okn = false;
            uint32_t kwn[GNS_KWMAX], slotn = 0, szn = 0;
            uint4 r4n[4];
            if (p0 + kXThreads < end) stage_b(p0 + kXThreads + tid, okn, kwn, slotn, r4n, szn);
            uint32_t park;
            const uint64_t w = ex_consume(a, p0 + tid, beg, okc, kwc, K, slotc, r4c, szc, &s_full, &s_claim, n_ok, H, park);
            ex_emit_park(a, beg, p0 + tid, w, park, &s_ncold, &s_pend);
            okc = okn; slotc = slotn; szc = szn;
#pragma unroll
            for (int i = 0; i < GNS_KWMAX; i++) kwc[i] = kwn[i];
#pragma unroll
            for (int i = 0; i < 4; i++) r4c[i] = r4n[i];
        }
    } else {
        for (uint64_t p0 = beg; p0 < end; p0 += kXThreads) {  // wave-uniform trip count
            const uint64_t p = p0 + tid;
            bool ok = p < end;
            uint32_t kw[GNS_KWMAX];
            const uint32_t sz = ok ? a.x.in.sizes[p] : 0u;
            if (ok) {
                const int st = ex_key<KIND, MODE>(a.x, K, s_src, p, kw);
                if (st != PARSE_OK) {
                    atomicAdd(st == PARSE_DROP ? &s_drop : &s_unsup, 1u);
                    ok = false;
                }
            }
            uint4 r4[4];
            uint32_t slot0 = 0;
            if (ok) {
                slot0 = mm3_n<GNS_KWMAX>(kw, K, a.D.seed) & a.D.mask;
                ex_probe_issue(a.D, slot0, r4);
            }
            uint32_t park;
            const uint64_t w = ex_consume(a, p, beg, ok, kw, K, slot0, r4, sz, &s_full, &s_claim, n_ok, H, park);
            ex_emit_park(a, beg, p, w, park, &s_ncold, &s_pend);
        }
    }
    atomicAdd(&s_ok, n_ok);
    __syncthreads();
    for (uint32_t i = tid; i < kExHot; i += kXThreads) {
        ExHotPart hp;
        hp.cb = s_hcb[i]; hp.maxp = s_hmax[i]; hp.pad = 0;
        a.hpart[(uint64_t)i * a.nblk + blk] = hp;
    }
    if (tid == 0) {
        a.pend_cnt[blk] = s_pend;
        a.ccnt[blk] = s_ncold;
        if (s_pend) atomicAdd(a.pend_total, s_pend);
        if (s_ok) atomicAdd(&a.stats[0], (unsigned long long)s_ok);
        if (s_drop) atomicAdd(&a.stats[1], (unsigned long long)s_drop);
        if (s_unsup) atomicAdd(&a.stats[2], (unsigned long long)s_unsup);
        if (s_full) atomicAdd(&a.stats[3], (unsigned long long)s_full);
        dict_flush_claims(a.D, s_claim, &a.stats[3]);
    }
}

struct ExResolveArgs {
    ExArgs x;
    const uint64_t *pend_in;
    const uint32_t *cnt_in;
    uint64_t *pend_out;
    uint32_t *cnt_out, *total_out;
};

template <int KIND, int MODE>
__global__ __launch_bounds__(kXThreads) void k_ex_resolve(ExResolveArgs r) {
    __shared__ uint8_t s_src[80];
    __shared__ uint32_t s_cnt, s_full, s_claim, s_abort;
    __shared__ __attribute__((aligned(16))) unsigned long long s_htab[kExHotTab];
    __shared__ unsigned long long s_hcb[kExHot];
    __shared__ uint32_t s_hmax[kExHot];
    const ExArgs &a = r.x;
    const uint32_t tid = threadIdx.x, blk = blockIdx.x;
    const uint32_t cnt = r.cnt_in[blk];
    if (cnt == 0) {  // block-uniform
        if (tid == 0) r.cnt_out[blk] = 0;
        return;
    }
    if (tid == 0) { s_cnt = 0; s_full = 0; s_claim = 0; s_abort = dict_aborted(a.D); }
    for (uint32_t j = tid; j < kExHotTab; j += kXThreads) s_htab[j] = a.hot_tab[j];
    for (uint32_t j = tid; j < kExHot; j += kXThreads) { s_hcb[j] = 0; s_hmax[j] = 0; }
    __syncthreads();
    if (s_abort) {
        if (tid == 0) r.cnt_out[blk] = 0;
        return;
    }
    stage_plan<MODE>(a.kp, s_src);
    const uint64_t beg = (uint64_t)blk * kXChunk;
    for (uint32_t i = tid; i < cnt; i += kXThreads) {
        const uint64_t v = r.pend_in[beg + i];
        const uint64_t p = beg + (v >> 50);
        uint32_t kw[GNS_KWMAX];
        (void)ex_key<KIND, MODE>(a.x, a.kp.K, s_src, p, kw);
        uint32_t out;
        const int res = dict_find_or_claim(a.D, kw, (uint32_t)(v & 0xFFFFFFFFFull), a.epoch, &out);
        if (res == DICT_CLAIMED) atomicAdd(&s_claim, 1u);
        if (res == DICT_FOUND || res == DICT_CLAIMED) {  // X1 wrote the word with none_key: fill in the flow field
            // a designated flow displaced from its home slot: into the block's partials
            // (its word is marked hot_key and skipped by P), as X1 does at the home slot
            const int h = res == DICT_FOUND ? exh_lookup(s_htab, out) : -1;
            if (h >= 0) {
                atomicAdd(&s_hcb[h], (unsigned long long)a.x.in.sizes[p] << kHotCntBits | 1ull);
                atomicMax(&s_hmax[h], (uint32_t)(p - beg));
                out = a.hot_key;
            }
            const uint32_t sh = a.ib + a.sb;
            const uint64_t wq = beg + ((v >> 36) & 0x3FFFu);
            a.sk[wq] = (a.sk[wq] & ((1ull << sh) - 1ull)) | (uint64_t)out << sh;
        }
        else if (res == DICT_PENDING) r.pend_out[beg + atomicAdd(&s_cnt, 1u)] = (v & ~0xFFFFFFFFFull) | out;
        else atomicAdd(&s_full, 1u);
    }
    __syncthreads();
    for (uint32_t j = tid; j < kExHot; j += kXThreads)
        if (s_hcb[j]) {  // X1 wrote this block's partials before this launch
            ExHotPart *hp = a.hpart + (uint64_t)j * a.nblk + blk;
            atomicAdd(&hp->cb, s_hcb[j]);
            atomicMax(&hp->maxp, s_hmax[j]);
        }
    if (tid == 0) {
        r.cnt_out[blk] = s_cnt;
        if (s_cnt) atomicAdd(r.total_out, s_cnt);
        if (s_full) atomicAdd(&a.stats[3], (unsigned long long)s_full);
        dict_flush_claims(a.D, s_claim, &a.stats[3]);
    }
}

// per-flow state, one array per field: first = stream index of the first packet (~0: none
// yet), last = stream index of the last packet + 1 (0: none), start / end = StartTime /
// EndTime in ns.  (One 64-byte record per flow measured slower: a run's two counter
// atomics then hit one line.)
struct FlowState {
    unsigned long long *pkts, *bytes, *first, *last;
    long long *start, *end;
};

extern "C" __device__ unsigned long long __ockl_wfred_add_u64(unsigned long long);
extern "C" __device__ unsigned __ockl_wfred_min_u32(unsigned);
extern "C" __device__ unsigned __ockl_wfred_max_u32(unsigned);
extern "C" __device__ unsigned __ockl_wfred_add_u32(unsigned);
extern "C" __device__ unsigned __ockl_wfscan_add_u32(unsigned, bool);

// H: the per-block partials of each designated flow -> its flow state (one
// workgroup per hot slot; the only writer of these flows until P4, which merges
// the flow's packets that were parked in X1).  first stays: a designated flow
// had packets before this batch.
template <bool LIST>
__global__ __launch_bounds__(256) void k_ex_hot_reduce(const ExHotPart *hpart, uint32_t nblk, const uint32_t *hot_ids,
                                                       uint64_t pkt_base, FlowState f, uint32_t *touch, uint32_t *tcnt) {
    __shared__ unsigned long long s_by[4];
    __shared__ uint32_t s_c[4], s_mx[4];
    const uint32_t slot = blockIdx.x, tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t id = hot_ids[slot];
    if (id == GNS_ID_NONE) return;  // block-uniform
    uint32_t c = 0, mx = 0;
    unsigned long long by = 0;
    for (uint32_t b = tid; b < nblk; b += 256) {
        const ExHotPart hp = hpart[(uint64_t)slot * nblk + b];
        if (hp.cb) {
            c += (uint32_t)(hp.cb & ((1u << kHotCntBits) - 1u));
            by += hp.cb >> kHotCntBits;
            mx = max(mx, b * kXChunk + hp.maxp);
        }
    }
    c = __ockl_wfred_add_u32(c);
    by = __ockl_wfred_add_u64(by);
    mx = __ockl_wfred_max_u32(mx);
    if (lane == 0) { s_c[wave] = c; s_by[wave] = by; s_mx[wave] = mx; }
    __syncthreads();
    if (tid == 0) {
        for (int w = 1; w < 4; w++) { c += s_c[w]; by += s_by[w]; mx = max(mx, s_mx[w]); }
        if (c) {
            f.pkts[id] += c;
            f.bytes[id] += by;
            f.last[id] = max(f.last[id], pkt_base + mx + 1);
            // H lists the designated flows it updated; P lists a flow only on its first merge
            // of the batch (last <= pkt_base), and H has already moved `last` past pkt_base
            // here, so parked packets of a designated flow never add a second entry
            if constexpr (LIST) touch[atomicAdd(tcnt, 1u)] = id;
        }
    }
}

// P: the tail words go to kPBins bins of consecutive flow ids (order-free: no
// stable partition is needed, the merge is add / min / max), then one
// workgroup per bin aggregates its words in an LDS hash table and merges each
// flow once.  Every flow id lies in exactly one bin, so the merge needs no
// global atomics.
//   P1 k_ex_phist     per X1 region: bin histogram  -> ph[blk][bin]
//   P2 k_ex_pscan_*   exclusive offsets of every (region, bin) in bin-major order
//   P3 k_ex_pscatter  per region, sub-passes of kPSub words staged bin by bin in
//                     LDS and copied out as runs
//   P4 k_ex_pagg      per bin: LDS hash (flow id -> count, bytes, min / max
//                     index), flushed into the flow state
constexpr uint32_t kPBinBits = 9;
constexpr uint32_t kPBins = 1u << kPBinBits;
constexpr uint32_t kPGroup = 64;  // regions per P2 group

__global__ __launch_bounds__(256) void k_ex_phist(const uint64_t *in, const uint32_t *ccnt, uint32_t ks,
                                                  uint32_t pshift, uint32_t none_key, uint32_t *ph) {
    __shared__ uint32_t h[kPBins];
    const uint32_t blk = blockIdx.x, n = ccnt[blk];
    for (uint32_t i = threadIdx.x; i < kPBins; i += 256) h[i] = 0;
    __syncthreads();
    const uint64_t *w = in + (uint64_t)blk * kXChunk;
    for (uint32_t i = threadIdx.x; i < n; i += 256) {
        const uint32_t id = (uint32_t)(w[i] >> ks);
        if (id < none_key) atomicAdd(&h[id >> pshift], 1u);  // (a resolved designated flow's word is skipped)
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < kPBins; i += 256) ph[(uint64_t)blk * kPBins + i] = h[i];
}
// per group of kPGroup regions: bin sums
__global__ __launch_bounds__(kPBins) void k_ex_pscan_a(const uint32_t *ph, uint32_t nblk, uint32_t *gs) {
    const uint32_t g = blockIdx.x, b = threadIdx.x;
    const uint32_t r1 = min(nblk, (g + 1) * kPGroup);
    uint32_t sum = 0;
    for (uint32_t r = g * kPGroup; r < r1; r++) sum += ph[(uint64_t)r * kPBins + b];
    gs[(uint64_t)g * kPBins + b] = sum;
}
// one workgroup: per bin, exclusive offsets of the groups; bin starts (pb[kPBins] = total)
__global__ __launch_bounds__(kPBins) void k_ex_pscan_b(uint32_t *gs, uint32_t ng, uint32_t *pb) {
    __shared__ uint32_t s_w[kPBins / 64];
    const uint32_t b = threadIdx.x, lane = b & 63u, wave = b >> 6;
    uint32_t run = 0;
    for (uint32_t g0 = 0; g0 < ng; g0 += 8) {  // 8 independent loads in flight, then the prefix
        uint32_t x[8];
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) x[j] = g0 + j < ng ? gs[(uint64_t)(g0 + j) * kPBins + b] : 0u;
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) {
            if (g0 + j < ng) gs[(uint64_t)(g0 + j) * kPBins + b] = run;
            run += x[j];
        }
    }
    const uint32_t inc = __ockl_wfscan_add_u32(run, true);
    if (lane == 63) s_w[wave] = inc;
    __syncthreads();
    uint32_t base = 0;
    for (uint32_t w = 0; w < wave; w++) base += s_w[w];
    const uint32_t start = base + inc - run;
    pb[b] = start;
    if (b == kPBins - 1) pb[kPBins] = base + inc;
    for (uint32_t g0 = 0; g0 < ng; g0 += 8) {
        uint32_t x[8];
#pragma unroll
        for (uint32_t j = 0; j < 8; j++) x[j] = g0 + j < ng ? gs[(uint64_t)(g0 + j) * kPBins + b] : 0u;
#pragma unroll
        for (uint32_t j = 0; j < 8; j++)
            if (g0 + j < ng) gs[(uint64_t)(g0 + j) * kPBins + b] = x[j] + start;
    }
}
// per group: the regions' offsets, in place over the histogram
__global__ __launch_bounds__(kPBins) void k_ex_pscan_c(uint32_t *ph, uint32_t nblk, const uint32_t *gs) {
    const uint32_t g = blockIdx.x, b = threadIdx.x;
    const uint32_t r1 = min(nblk, (g + 1) * kPGroup);
    uint32_t run = gs[(uint64_t)g * kPBins + b];
    for (uint32_t r = g * kPGroup; r < r1; r++) {
        const uint32_t x = ph[(uint64_t)r * kPBins + b];
        ph[(uint64_t)r * kPBins + b] = run;
        run += x;
    }
}

constexpr uint32_t kPSub = 4096;  // words per P3 sub-pass
constexpr uint32_t kPItems = kPSub / kPBins;
__global__ __launch_bounds__(kPBins) void k_ex_pscatter(const uint64_t *in, const uint32_t *ccnt, const uint32_t *po,
                                                        uint32_t ks, uint32_t pshift, uint32_t none_key, uint64_t *out) {
    __shared__ uint64_t stage[kPSub];
    __shared__ uint16_t sbin[kPSub];
    __shared__ uint32_t cnt[kPBins], lstart[kPBins], goff[kPBins], dummy[kPBins], s_w[kPBins / 64];
    const uint32_t blk = xcd_block(blockIdx.x, gridDim.x);  // adjacent regions on one XCD (gns_xcd.cuh)
    const uint32_t n = ccnt[blk], tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    if (n == 0) return;  // block-uniform
    const uint64_t *src = in + (uint64_t)blk * kXChunk;
    goff[tid] = po[(uint64_t)blk * kPBins + tid];
    cnt[tid] = 0;
    __syncthreads();
    for (uint32_t sp = 0; sp < n; sp += kPSub) {
        uint64_t w[kPItems];
        uint32_t bn[kPItems], rk[kPItems];
#pragma unroll
        for (uint32_t j = 0; j < kPItems; j++) {
            const uint32_t i = sp + j * kPBins + tid;
            w[j] = i < n ? src[i] : 0ull;
            const uint32_t id = (uint32_t)(w[j] >> ks);
            bn[j] = i < n && id < none_key ? id >> pshift : 0xFFFFu;
        }
        // ranks (any order): every lane adds, a lane without a word adds 0 to its own word
#pragma unroll
        for (uint32_t j = 0; j < kPItems; j++) {
            uint32_t *ad = bn[j] != 0xFFFFu ? &cnt[bn[j]] : &dummy[tid];
            rk[j] = atomicAdd(ad, bn[j] != 0xFFFFu ? 1u : 0u);
        }
        __syncthreads();
        const uint32_t c = cnt[tid];
        const uint32_t inc = __ockl_wfscan_add_u32(c, true);
        if (lane == 63) s_w[wave] = inc;
        __syncthreads();
        uint32_t base = 0;
        for (uint32_t v = 0; v < wave; v++) base += s_w[v];
        lstart[tid] = base + inc - c;
        __syncthreads();
#pragma unroll
        for (uint32_t j = 0; j < kPItems; j++)
            if (bn[j] != 0xFFFFu) {
                const uint32_t pos = lstart[bn[j]] + rk[j];
                stage[pos] = w[j];
                sbin[pos] = (uint16_t)bn[j];
            }
        __syncthreads();
        uint32_t m = 0;  // words staged in this sub-pass (designated flows' words are not)
        for (uint32_t v = 0; v < kPBins / 64; v++) m += s_w[v];
        for (uint32_t i = tid; i < m; i += kPBins) {
            const uint32_t bb = sbin[i];
            out[goff[bb] + (i - lstart[bb])] = stage[i];
        }
        __syncthreads();
        goff[tid] += c;
        cnt[tid] = 0;
        __syncthreads();
    }
}

// P4: one workgroup per bin, two per CU.  Words in chunks of kAggChunk; before a
// chunk the table is flushed if it could overflow (a bin with more distinct flows
// than the table merges in several rounds; each flow's partial results add up).
// A flow holding >= 6 of a wave's words (a heavy tail flow) has them folded into
// one update (up to GNS_AGG_FOLD such flows per wave and chunk).
constexpr uint32_t kAggThreads = 1024;
constexpr uint32_t kAggChunk = kAggThreads;
#ifndef GNS_AGG_DEPTH
#define GNS_AGG_DEPTH 1
#endif
constexpr uint32_t kAggDepth = GNS_AGG_DEPTH;  // chunks of words in flight
#ifndef GNS_AGG_CAP
#define GNS_AGG_CAP 3072
#endif
#ifndef GNS_AGG_FOLD
#define GNS_AGG_FOLD 4
#endif
constexpr uint64_t kExListSlots = 1ull << 23;  // T/D read the touched list above this many slots
constexpr uint32_t kAggCap = GNS_AGG_CAP;  // 24 B per entry: 72 KB
constexpr int kAggMinBlocks = kAggCap * 24 <= 78 * 1024 ? 2 : 1;
static_assert(kAggCap > kAggChunk, "a chunk fits an empty table");
// Touched-flow list (T and D read it instead of scanning the table): a flow is
// appended when its first merge of the batch lands (its last index is then still
// from an earlier batch), so each flow appears once.  One global add per flush
// for the whole workgroup's appends (the counter is shared by every workgroup).

template <bool LIST>
__device__ __forceinline__ void pagg_flush(uint32_t *key, uint32_t *cn, uint32_t *mn, uint32_t *mx,
                                           unsigned long long *by, uint64_t pkt_base, FlowState f, uint32_t *touch,
                                           uint32_t *tcnt) {
    // every entry's four state words are loaded before any is merged (all in flight together)
    constexpr uint32_t kPer = (kAggCap + kAggThreads - 1) / kAggThreads;
    uint32_t id[kPer];
    unsigned long long pk[kPer], bt[kPer], ls[kPer], fs[kPer];
#pragma unroll
    for (uint32_t j = 0; j < kPer; j++) {
        const uint32_t e = threadIdx.x + j * kAggThreads;
        id[j] = e < kAggCap ? key[e] : GNS_ID_NONE;
        if (id[j] != GNS_ID_NONE) { pk[j] = f.pkts[id[j]]; bt[j] = f.bytes[id[j]]; ls[j] = f.last[id[j]]; fs[j] = f.first[id[j]]; }
    }
    if constexpr (LIST) {  // the touched-flow list (large tables only: the scan variant compiles without it)
        __shared__ uint32_t s_tw[kAggThreads / 64], s_tbase;
        const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
        uint32_t c = 0;
#pragma unroll
        for (uint32_t j = 0; j < kPer; j++) c += (id[j] != GNS_ID_NONE && ls[j] <= pkt_base) ? 1u : 0u;
        const uint32_t inc = __ockl_wfscan_add_u32(c, true);
        if (lane == 63) s_tw[wave] = inc;
        __syncthreads();
        const uint32_t x = lane < kAggThreads / 64 ? s_tw[lane] : 0u;
        const uint32_t winc = __ockl_wfscan_add_u32(x, true);
        const uint32_t tot = __shfl(winc, 63);  // (all lanes active)
        if (threadIdx.x == 0) s_tbase = atomicAdd(tcnt, tot);
        __syncthreads();
        uint32_t pos = s_tbase + __shfl(winc - x, (int)wave) + inc - c;
#pragma unroll
        for (uint32_t j = 0; j < kPer; j++)
            if (id[j] != GNS_ID_NONE && ls[j] <= pkt_base) touch[pos++] = id[j];
    }
#pragma unroll
    for (uint32_t j = 0; j < kPer; j++) {
        const uint32_t e = threadIdx.x + j * kAggThreads;
        if (id[j] == GNS_ID_NONE) continue;
        f.pkts[id[j]] = pk[j] + cn[e];
        f.bytes[id[j]] = bt[j] + by[e];
        f.last[id[j]] = max(ls[j], pkt_base + mx[e] + 1);
        if (fs[j] >= pkt_base) f.first[id[j]] = min(fs[j], pkt_base + mn[e]);  // no packet before this batch
        key[e] = GNS_ID_NONE; cn[e] = 0; mn[e] = ~0u; mx[e] = 0; by[e] = 0;
    }
}
// Table slot of a flow: buckets of 4 keys read with one 16-byte LDS load; keys
// fill a bucket's slots in order and spill to the next bucket only when it is
// full, so a bucket with an empty slot and no match ends the search (a linear
// probe of single keys measured long dependent chains at 2/3 load).
constexpr uint32_t kAggBuckets = kAggCap / 4;
static_assert(kAggCap % 4 == 0, "whole buckets");
__device__ __forceinline__ uint32_t pagg_slot(uint32_t *key, uint32_t id, uint32_t *s_n) {
    uint32_t b = (uint32_t)(((uint64_t)(id * 0x9E3779B1u) * kAggBuckets) >> 32);
    for (;;) {
        const uint4 k4 = reinterpret_cast<const uint4 *>(key)[b];
        if (k4.x == id) return 4 * b;
        if (k4.y == id) return 4 * b + 1;
        if (k4.z == id) return 4 * b + 2;
        if (k4.w == id) return 4 * b + 3;
        const uint32_t e = k4.x == GNS_ID_NONE ? 0u : k4.y == GNS_ID_NONE ? 1u : k4.z == GNS_ID_NONE ? 2u
                         : k4.w == GNS_ID_NONE ? 3u : 4u;
        if (e == 4u) {  // full: the key, if present, is further along
            b = b + 1 == kAggBuckets ? 0u : b + 1;
            continue;
        }
        const uint32_t old = atomicCAS(&key[4 * b + e], GNS_ID_NONE, id);
        if (old == GNS_ID_NONE) { atomicAdd(s_n, 1u); return 4 * b + e; }
        if (old == id) return 4 * b + e;
        // another flow took that slot: read the bucket again
    }
}
template <bool LIST>
__global__ __launch_bounds__(kAggThreads, kAggMinBlocks) void k_ex_pagg(const uint64_t *in, const uint32_t *pb, uint32_t sb,
                                                            uint32_t ib, const uint32_t *sizes, uint64_t pkt_base,
                                                            FlowState f, uint32_t *touch, uint32_t *tcnt) {
    __shared__ __attribute__((aligned(16))) uint32_t key[kAggCap];
    __shared__ uint32_t cn[kAggCap], mn[kAggCap], mx[kAggCap];
    __shared__ unsigned long long by[kAggCap];
    __shared__ uint32_t s_n;
    const uint32_t bin = blockIdx.x, tid = threadIdx.x, lane = tid & 63u;
    const uint32_t beg = pb[bin], end = pb[bin + 1];
    if (beg == end) return;  // block-uniform
    for (uint32_t e = tid; e < kAggCap; e += kAggThreads) { key[e] = GNS_ID_NONE; cn[e] = 0; mn[e] = ~0u; mx[e] = 0; by[e] = 0; }
    if (tid == 0) s_n = 0;
    const uint32_t ks = sb + ib, esc = (1u << sb) - 1u;
    const uint64_t imask = (1ull << ib) - 1ull;
    // the words of the next kAggDepth chunks are in flight (P4 is latency-bound on them)
    uint64_t wq[kAggDepth];
#pragma unroll
    for (uint32_t j = 0; j < kAggDepth; j++) {
        const uint32_t i = beg + j * kAggChunk + tid;
        wq[j] = i < end ? in[i] : ~0ull;
    }
    __syncthreads();
    for (uint32_t c0 = beg; c0 < end; c0 += kAggChunk) {  // block-uniform trip count
        if (s_n > kAggCap - kAggChunk) {  // block-uniform (read after the barrier)
            pagg_flush<LIST>(key, cn, mn, mx, by, pkt_base, f, touch, tcnt);
            __syncthreads();
            if (tid == 0) s_n = 0;
            __syncthreads();
        }
        const uint64_t w = wq[0];
#pragma unroll
        for (uint32_t j = 0; j + 1 < kAggDepth; j++) wq[j] = wq[j + 1];
        {
            const uint32_t i = c0 + kAggDepth * kAggChunk + tid;
            wq[kAggDepth - 1] = i < end ? in[i] : ~0ull;
        }
        bool v = w != ~0ull;
        const uint32_t id = v ? (uint32_t)(w >> ks) : GNS_ID_NONE;
        const uint32_t idx = (uint32_t)((w >> sb) & imask);
        uint32_t sz = (uint32_t)w & esc;
        if (v && sz == esc) sz = sizes[idx];  // lengths too large for the word's field (rare)
        // heavy flows holding many of the wave's words: one folded update each
        // (same-address LDS atomics serialize lane by lane)
#pragma unroll 1
        for (int fold = 0; fold < GNS_AGG_FOLD; fold++) {
            const uint64_t vm = __ballot(v);
            if (!vm) break;  // wave-uniform
            const uint32_t id0 = __shfl(id, (int)(__ffsll((long long)vm) - 1));
            const bool in_m = v && id == id0;
            const uint64_t m = __ballot(in_m);
            if (__popcll(m) < 6) break;  // wave-uniform
            const unsigned long long tb = __ockl_wfred_add_u64(in_m ? (unsigned long long)sz : 0ull);
            const uint32_t tmn = __ockl_wfred_min_u32(in_m ? idx : ~0u);
            const uint32_t tmx = __ockl_wfred_max_u32(in_m ? idx : 0u);
            if (lane == (uint32_t)__ffsll((long long)m) - 1u) {
                const uint32_t h = pagg_slot(key, id0, &s_n);
                atomicAdd(&cn[h], (uint32_t)__popcll(m));
                atomicAdd(&by[h], tb);
                atomicMin(&mn[h], tmn);
                atomicMax(&mx[h], tmx);
            }
            v = v && !in_m;
        }
        if (v) {
            const uint32_t h = pagg_slot(key, id, &s_n);
            atomicAdd(&cn[h], 1u);
            atomicAdd(&by[h], (unsigned long long)sz);
            atomicMin(&mn[h], idx);
            atomicMax(&mx[h], idx);
        }
        __syncthreads();
    }
    pagg_flush<LIST>(key, cn, mn, mx, by, pkt_base, f, touch, tcnt);
}

// T: StartTime / EndTime from the merged stream indices of the flows this batch
// touched (task.go:137,141-142).
__global__ __launch_bounds__(256) void k_ex_times(FlowState f, uint64_t slots, uint64_t pkt_base, uint64_t n,
                                                  const int64_t *ts) {
    const uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= slots) return;
    const unsigned long long l = f.last[s], fs = f.first[s];
    if (l > pkt_base && l <= pkt_base + n) f.end[s] = ts[l - 1 - pkt_base];
    if (fs >= pkt_base && fs < pkt_base + n) f.start[s] = ts[fs - pkt_base];
}

// D: designate the next batch's heavy flows: the flows in the largest 1/8-octave
// bands of the packet count that together hold at most kExHot flows.
__device__ __forceinline__ uint32_t exh_key(unsigned long long p) {
    if (p < 8) return 0;
    const uint32_t lz = 63u - (uint32_t)__clzll((long long)p);
    return lz * 8u + (uint32_t)((p >> (lz - 3)) & 7u);
}
__global__ __launch_bounds__(256) void k_exh_hist(const unsigned long long *pkts, uint64_t slots, uint32_t *hist) {
    __shared__ uint32_t h[512];
    for (uint32_t i = threadIdx.x; i < 512; i += 256) h[i] = 0;
    __syncthreads();
    for (uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x; s < slots; s += (uint64_t)gridDim.x * 256) {
        const uint32_t k = exh_key(pkts[s]);
        if (k >= kExHotMinKey) atomicAdd(&h[k], 1u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < 512; i += 256)
        if (h[i]) atomicAdd(&hist[i], h[i]);
}
// threshold = the smallest key whose suffix count (flows with a key >= it) is <= kExHot
__global__ __launch_bounds__(512) void k_exh_pick(const uint32_t *hist, uint32_t *thr) {
    __shared__ uint32_t s_w[8];
    __shared__ uint32_t s_t;
    const uint32_t k = threadIdx.x, lane = k & 63u, wave = k >> 6;
    if (k == 0) s_t = 512;
    // suffix sums: scan over the reversed keys
    const uint32_t r = 511u - k;  // thread k holds key r
    const uint32_t v = r >= kExHotMinKey ? hist[r] : 0u;
    const uint32_t inc = __ockl_wfscan_add_u32(v, true);
    if (lane == 63) s_w[wave] = inc;
    __syncthreads();
    uint32_t base = 0;
    for (uint32_t w = 0; w < wave; w++) base += s_w[w];
    const uint32_t suffix = base + inc;  // flows with a key >= r
    if (r >= kExHotMinKey && suffix <= kExHot) atomicMin(&s_t, r);
    __syncthreads();
    if (k == 0) *thr = s_t;
}
__global__ __launch_bounds__(256) void k_exh_collect(const unsigned long long *pkts, uint64_t slots,
                                                     const uint32_t *thr, uint32_t *cnt, uint32_t *hot_ids) {
    const uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= slots) return;
    const uint32_t k = exh_key(pkts[s]);
    if (k >= *thr && k >= kExHotMinKey) {
        const uint32_t q = atomicAdd(cnt, 1u);
        if (q < kExHot) hot_ids[q] = (uint32_t)s;
    }
}
// T and D over the batch's touched-flow list instead of every slot: tables above
// kExListSlots (a table that grew with the period), where a scan would cost more
// than the batch.  The list's random gathers cost more than the scan below that.
__global__ __launch_bounds__(256) void k_ex_times_list(FlowState f, const uint32_t *touch, const uint32_t *tcnt,
                                                  uint64_t slots, uint64_t pkt_base, uint64_t n, const int64_t *ts) {
    const uint64_t nt = *tcnt;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < nt; i += (uint64_t)gridDim.x * 256) {
        const uint32_t s = touch[i];
        const unsigned long long l = f.last[s], fs = f.first[s];
        if (l > pkt_base && l <= pkt_base + n) f.end[s] = ts[l - 1 - pkt_base];
        if (fs >= pkt_base && fs < pkt_base + n) f.start[s] = ts[fs - pkt_base];
    }
}

__global__ __launch_bounds__(256) void k_exh_hist_list(const unsigned long long *pkts, const uint32_t *touch,
                                                  const uint32_t *tcnt, uint64_t slots, uint32_t *hist) {
    __shared__ uint32_t h[512];
    for (uint32_t i = threadIdx.x; i < 512; i += 256) h[i] = 0;
    __syncthreads();
    const uint64_t nt = *tcnt;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < nt; i += (uint64_t)gridDim.x * 256) {
        const uint32_t k = exh_key(pkts[touch[i]]);
        if (k >= kExHotMinKey) atomicAdd(&h[k], 1u);
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < 512; i += 256)
        if (h[i]) atomicAdd(&hist[i], h[i]);
}
__global__ __launch_bounds__(256) void k_exh_collect_list(const unsigned long long *pkts, const uint32_t *touch,
                                                     const uint32_t *tcnt, uint64_t slots, const uint32_t *thr,
                                                     uint32_t *cnt, uint32_t *hot_ids) {
    const uint64_t nt = *tcnt;
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < nt; i += (uint64_t)gridDim.x * 256) {
        const uint32_t s = touch[i];
        const uint32_t k = exh_key(pkts[s]);
        if (k >= *thr && k >= kExHotMinKey) {
            const uint32_t q = atomicAdd(cnt, 1u);
            if (q < kExHot) hot_ids[q] = s;
        }
    }
}
// the lookup table, heaviest flows first (64 at a time): a flow whose 4-entry group
// is full is simply not designated, and that should be one of the lightest
// (a heavy flow left in the tail would serialise its P4 bin)
__global__ __launch_bounds__(kExHot) void k_exh_table(uint32_t *hot_ids, const unsigned long long *pkts,
                                                      unsigned long long *hot_tab) {
    __shared__ unsigned long long t[kExHotTab];
    __shared__ unsigned long long s_p[kExHot];
    __shared__ uint32_t s_ord[kExHot];
    const uint32_t i = threadIdx.x;
    for (uint32_t j = i; j < kExHotTab; j += kExHot) t[j] = ~0ull;
    const uint32_t id = hot_ids[i];
    const unsigned long long p = id != GNS_ID_NONE ? pkts[id] : 0ull;
    s_p[i] = p;
    __syncthreads();
    uint32_t rank = 0;
    for (uint32_t j = 0; j < kExHot; j++) {
        const unsigned long long q = s_p[j];
        rank += (q > p || (q == p && j < i)) ? 1u : 0u;
    }
    s_ord[rank] = i;
    __syncthreads();
    for (uint32_t r0 = 0; r0 < kExHot; r0 += 64) {
        if (i < 64) {
            const uint32_t h = s_ord[r0 + i];
            const uint32_t hid = hot_ids[h];
            if (hid != GNS_ID_NONE) {
                const uint32_t g = exh_group(hid) * 4;
                bool in = false;
                for (uint32_t e = 0; e < 4 && !in; e++)
                    in = atomicCAS(&t[g + e], ~0ull, (unsigned long long)hid << 16 | h) == ~0ull;
                if (!in) hot_ids[h] = GNS_ID_NONE;
            }
        }
        __syncthreads();
    }
    for (uint32_t j = i; j < kExHotTab; j += kExHot) hot_tab[j] = t[j];
}

__global__ __launch_bounds__(256) void k_ex_query(const uint8_t *flows, uint32_t stride, uint64_t n, uint32_t K,
                                                  DictDev D, FlowState f, uint64_t *out) {
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= n) return;
    uint32_t kw[GNS_KWMAX];
    load_key_bytes<GNS_KWMAX>(flows + p * stride, K, false, kw);
    const uint32_t id = dict_lookup(D, kw);
    out[p] = id == GNS_ID_NONE ? 0ull : (uint64_t)(f.pkts[id] << 32 | f.bytes[id]);  // task.go:323
}

// occupied dictionary slots -> ids (snapshot)
__global__ __launch_bounds__(256) void k_ex_list(DictDev D, uint64_t slots, const unsigned long long *pkts,
                                                 uint32_t *ids, uint32_t *count) {
    const uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const bool occ = s < slots && D.rec[s * D.RW] != 0u && pkts[s] != 0ull;
    const uint64_t m = __ballot(occ);
    if (m == 0) return;
    const uint32_t lane = __lane_id();
    const int leader = __ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if ((int)lane == leader) base = atomicAdd(count, (uint32_t)__popcll(m));
    base = __shfl(base, leader);
    if (occ) ids[base + __popcll(m & ((1ull << lane) - 1))] = (uint32_t)s;
}

__global__ __launch_bounds__(256) void k_ex_gather(const uint32_t *ids, uint64_t n, DictDev D, FlowState f,
                                                   uint8_t *keys, long long *start, long long *end,
                                                   unsigned long long *pkts, unsigned long long *bytes) {
    const uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= n) return;
    const uint32_t id = ids[p];
    uint32_t r[12];
    load_record(D, id, r);
    for (uint32_t j = 0; j < D.K; j++) keys[p * D.K + j] = (uint8_t)(r[1 + (j >> 2)] >> (8 * (j & 3)));
    start[p] = f.start[id]; end[p] = f.end[id]; pkts[p] = f.pkts[id]; bytes[p] = f.bytes[id];
}

// table growth: per-flow state follows its record to the new slot (gns_dict.hip remap)
__global__ __launch_bounds__(256) void k_ex_permute(FlowState o, uint64_t slots, const uint32_t *remap, FlowState f) {
    const uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= slots) return;
    const uint32_t t = remap[s];
    if (t >= kDictMarked) return;  // dropped (GNS_ID_NONE) or never reinserted
    f.pkts[t] = o.pkts[s]; f.bytes[t] = o.bytes[s]; f.first[t] = o.first[s]; f.last[t] = o.last[s];
    f.start[t] = o.start[s]; f.end[t] = o.end[s];
}

__global__ __launch_bounds__(256) void k_ex_init(FlowState f, uint64_t slots) {
    const uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= slots) return;
    f.pkts[s] = 0; f.bytes[s] = 0; f.first[s] = ~0ull; f.last[s] = 0; f.start[s] = 0; f.end[s] = 0;
}

}  // namespace gns

using namespace gns;

struct gns_ex {
    int device = 0;
    bool force_list = false;  // GNS_EX_LIST=1: T/D over the touched list at any table size (tests)
    hipStream_t stream = nullptr;
    KeyPlanN kp{};
    uint32_t K = 0;
    DictDev D{};
    uint64_t slots = 0;
    uint64_t claimed = 0;                    // D.ctl[0] as of the last batch
    uint32_t *dctl = nullptr;
    DictScratch dsc;
    unsigned long long *stats_bak = nullptr;
    uint64_t n_grow = 0, n_retry = 0;
    double grow_ms = 0.0;
    FlowState f{};
    uint32_t epoch = 0;
    uint64_t pkt = 0, batches = 0;
    uint64_t bmax = 0;
    uint32_t nblk_max = 0;
    uint64_t *sk[2] = {nullptr, nullptr};    // X1 block regions of tail words; the same partitioned by bin
    uint32_t *hot_ids = nullptr;             // [kExHot] designated flows (GNS_ID_NONE: unused slot)
    unsigned long long *hot_tab = nullptr;   // [kExHotTab] their lookup table
    ExHotPart *hpart = nullptr;              // [kExHot][nblk_max]
    uint32_t *hctl = nullptr;                // [0..511] count histogram, [512] threshold, [513] count, [514] tail words, [515] touched
    uint32_t *touch = nullptr;               // [bmax + kExHot] flows the batch touched (T, D)
    uint32_t *ccnt = nullptr;                // [nblk_max] X1 region word counts
    bool warm = false;                       // flows designated (a batch ran since create / reset / growth)
    uint32_t *ph = nullptr, *pgs = nullptr, *pb = nullptr;  // P histograms / offsets, group sums, bin starts
    uint32_t key_bits = 0;                   // flow field bits: flow ids < slots, invalid = slots
    uint32_t sb = 0, ib = 0;                 // sort word: wire length bits, packet index bits
    uint64_t *pend[2] = {nullptr, nullptr};
    uint32_t *pcnt[2] = {nullptr, nullptr};
    uint32_t *ptotal = nullptr;
    unsigned long long *stats = nullptr;
    uint32_t *h_pin = nullptr;
    uint8_t *stage = nullptr;
    size_t stage_bytes = 0;
    StageTimer timer;
};

namespace {

int ex_set_dev(gns_ex *ex) {
    (void)hipGetLastError();  // clear a stale error of an earlier runtime call on this thread
    GNS_HIP(hipSetDevice(ex->device));
    return GNS_OK;
}

void ex_free_all(gns_ex *ex) {
    dfree(ex->D.rec); dfree(ex->f.pkts); dfree(ex->f.bytes); dfree(ex->f.first); dfree(ex->f.last);
    dfree(ex->f.start); dfree(ex->f.end); dfree(ex->pend[0]); dfree(ex->pend[1]);
    dfree(ex->pcnt[0]); dfree(ex->pcnt[1]); dfree(ex->ptotal); dfree(ex->stats); dfree(ex->stage);
    dfree(ex->sk[0]); dfree(ex->sk[1]); dfree(ex->ph); dfree(ex->pgs); dfree(ex->pb);
    dfree(ex->hot_ids); dfree(ex->touch); dfree(ex->hot_tab); dfree(ex->hpart); dfree(ex->hctl); dfree(ex->ccnt);
    dfree(ex->dctl); dfree(ex->stats_bak); ex->dsc.free_all();
    if (ex->h_pin) (void)hipHostFree(ex->h_pin);
    ex->timer.destroy();
    if (ex->stream) (void)hipStreamDestroy(ex->stream);
}

// no designated flows (after create / reset, and after a table growth renumbers the flows)
int ex_hot_clear(gns_ex *ex) {
    ex->warm = false;
    GNS_HIP(hipMemsetAsync(ex->hot_ids, 0xFF, kExHot * 4, ex->stream));
    GNS_HIP(hipMemsetAsync(ex->hot_tab, 0xFF, kExHotTab * 8, ex->stream));
    return GNS_OK;
}

int ex_clear(gns_ex *ex) {
    GNS_HIP(hipMemsetAsync(ex->D.rec, 0, ex->slots * ex->D.RW * 4, ex->stream));
    GNS_HIP(hipMemsetAsync(ex->dctl, 0, 16, ex->stream));
    ex->claimed = 0;
    GNS_HIP(hipMemsetAsync(ex->stats + 3, 0, sizeof(unsigned long long), ex->stream));  // dict-full word
    GNS_TRY(ex_hot_clear(ex));
    hipLaunchKernelGGL(k_ex_init, dim3((unsigned)((ex->slots + 255) / 256)), dim3(256), 0, ex->stream, ex->f,
                       ex->slots);
    GNS_HIP(hipGetLastError());
    return GNS_OK;
}

template <int KIND, int MODE>
int ex_run_batch(gns_ex *ex, const ExIn &xin, uint64_t n) {
    if (n == 0) return GNS_OK;
    hipStream_t s = ex->stream;
    const uint32_t nblk = (uint32_t)((n + kXChunk - 1) / kXChunk);
    ScopedStage total_stage(ex->timer, 5);
    GNS_HIP(hipMemsetAsync(ex->ptotal, 0, 8, s));
    GNS_HIP(hipMemsetAsync(ex->dctl + 1, 0, 4, s));  // abort flag of this batch
    if (++ex->epoch == 0) ex->epoch = 1;
    ExArgs x{};
    x.x = xin; x.n = n; x.kp = ex->kp; x.D = ex->D; x.epoch = ex->epoch;
    x.sk = ex->sk[0]; x.none_key = (uint32_t)ex->slots; x.hot_key = x.none_key + 1; x.sb = ex->sb; x.ib = ex->ib;
    x.hot_tab = ex->hot_tab; x.hpart = ex->hpart; x.ccnt = ex->ccnt; x.nblk = nblk;
    x.pend = ex->pend[0]; x.pend_cnt = ex->pcnt[0]; x.pend_total = ex->ptotal; x.stats = ex->stats;
    {
        ScopedStage st(ex->timer, 0);
        hipLaunchKernelGGL((k_ex_extract<KIND, MODE>), dim3(nblk), dim3(kXThreads), 0, s, x);
        GNS_HIP(hipGetLastError());
    }
    // resolve rounds; the first is queued behind X1 without a host round trip (X1
    // parks the flows displaced from their home slot; a block with none exits at once)
    int cur = 0;
    for (int round = 0;; round++) {
        if (round > 0) {
            GNS_HIP(hipMemcpyAsync(ex->h_pin, ex->ptotal + cur, 4, hipMemcpyDeviceToHost, s));
            GNS_HIP(hipMemcpyAsync(ex->h_pin + 2, ex->stats + 3, 8, hipMemcpyDeviceToHost, s));
            GNS_HIP(hipMemcpyAsync(ex->h_pin + 4, ex->dctl, 4, hipMemcpyDeviceToHost, s));
            GNS_HIP(hipStreamSynchronize(s));
            ex->claimed = ex->h_pin[4];
            if (ex->h_pin[2] | ex->h_pin[3]) { set_error("flow dictionary full; raise max_flows"); return GNS_E_FULL; }
            if (ex->h_pin[0] == 0) break;
        }
        if (round > 64) { set_error("dictionary resolve did not converge"); return GNS_E_FULL; }
        GNS_HIP(hipMemsetAsync(ex->ptotal + (cur ^ 1), 0, 4, s));
        if (++ex->epoch == 0) ex->epoch = 1;
        ExResolveArgs r{};
        r.x = x; r.x.epoch = ex->epoch;
        r.pend_in = ex->pend[cur]; r.cnt_in = ex->pcnt[cur];
        r.pend_out = ex->pend[cur ^ 1]; r.cnt_out = ex->pcnt[cur ^ 1]; r.total_out = ex->ptotal + (cur ^ 1);
        ScopedStage st(ex->timer, 1);
        hipLaunchKernelGGL((k_ex_resolve<KIND, MODE>), dim3(nblk), dim3(kXThreads), 0, s, r);
        GNS_HIP(hipGetLastError());
        cur ^= 1;
    }
    // T and D over the batch's touched-flow list once the table is large (a table that
    // grew with the period would make a full scan cost more than the batch); below
    // that, a sequential scan of every slot is cheaper than the list's random gathers
    uint32_t *touch = (ex->slots > kExListSlots || ex->force_list) ? ex->touch : nullptr;
    const uint32_t ks = ex->sb + ex->ib;
    // flow ids < slots = 2^(key_bits - 1): bin = id >> pshift
    const uint32_t pshift = ex->key_bits - 1 > kPBinBits ? ex->key_bits - 1 - kPBinBits : 0u;
    const uint32_t ng = (nblk + kPGroup - 1) / kPGroup;
    {
        ScopedStage st(ex->timer, 4);
        GNS_HIP(hipMemsetAsync(ex->hctl + 515, 0, 4, s));  // touched flows of this batch
        if (touch)
            hipLaunchKernelGGL(k_ex_hot_reduce<true>, dim3(kExHot), dim3(256), 0, s, ex->hpart, nblk, ex->hot_ids, ex->pkt,
                               ex->f, touch, ex->hctl + 515);
        else
            hipLaunchKernelGGL(k_ex_hot_reduce<false>, dim3(kExHot), dim3(256), 0, s, ex->hpart, nblk, ex->hot_ids, ex->pkt,
                               ex->f, touch, ex->hctl + 515);
        GNS_HIP(hipGetLastError());
    }
    {
        ScopedStage st(ex->timer, 2);
        const uint32_t none_key = (uint32_t)ex->slots;
        hipLaunchKernelGGL(k_ex_phist, dim3(nblk), dim3(256), 0, s, ex->sk[0], ex->ccnt, ks, pshift, none_key, ex->ph);
        hipLaunchKernelGGL(k_ex_pscan_a, dim3(ng), dim3(kPBins), 0, s, ex->ph, nblk, ex->pgs);
        hipLaunchKernelGGL(k_ex_pscan_b, dim3(1), dim3(kPBins), 0, s, ex->pgs, ng, ex->pb);
        hipLaunchKernelGGL(k_ex_pscan_c, dim3(ng), dim3(kPBins), 0, s, ex->ph, nblk, ex->pgs);
        hipLaunchKernelGGL(k_ex_pscatter, dim3(nblk), dim3(kPBins), 0, s, ex->sk[0], ex->ccnt, ex->ph, ks, pshift,
                           none_key, ex->sk[1]);
        GNS_HIP(hipGetLastError());
    }
    {
        ScopedStage st(ex->timer, 3);
        if (touch)
            hipLaunchKernelGGL(k_ex_pagg<true>, dim3(kPBins), dim3(kAggThreads), 0, s, ex->sk[1], ex->pb, ex->sb, ex->ib,
                           xin.in.sizes, ex->pkt, ex->f, touch, ex->hctl + 515);
        else
            hipLaunchKernelGGL(k_ex_pagg<false>, dim3(kPBins), dim3(kAggThreads), 0, s, ex->sk[1], ex->pb, ex->sb, ex->ib,
                           xin.in.sizes, ex->pkt, ex->f, touch, ex->hctl + 515);
        GNS_HIP(hipGetLastError());
    }
    {   // timestamps of the touched flows; the next batch's designated flows
        ScopedStage st(ex->timer, 4);
        if (touch) {
            const unsigned sg = (unsigned)std::min<uint64_t>((n + kExHot + 255) / 256, 4096);
            hipLaunchKernelGGL(k_ex_times_list, dim3(sg), dim3(256), 0, s, ex->f, touch, ex->hctl + 515, ex->slots, ex->pkt,
                               n, xin.ts);
            GNS_HIP(hipMemsetAsync(ex->hctl, 0, 514 * 4, s));
            GNS_HIP(hipMemsetAsync(ex->hot_ids, 0xFF, kExHot * 4, s));
            hipLaunchKernelGGL(k_exh_hist_list, dim3(std::min(sg, 2048u)), dim3(256), 0, s, ex->f.pkts, touch,
                               ex->hctl + 515, ex->slots, ex->hctl);
            hipLaunchKernelGGL(k_exh_pick, dim3(1), dim3(512), 0, s, ex->hctl, ex->hctl + 512);
            hipLaunchKernelGGL(k_exh_collect_list, dim3(sg), dim3(256), 0, s, ex->f.pkts, touch, ex->hctl + 515,
                               ex->slots, ex->hctl + 512, ex->hctl + 513, ex->hot_ids);
        } else {
            const unsigned sg = (unsigned)((ex->slots + 255) / 256);
            hipLaunchKernelGGL(k_ex_times, dim3(sg), dim3(256), 0, s, ex->f, ex->slots, ex->pkt, n, xin.ts);
            GNS_HIP(hipMemsetAsync(ex->hctl, 0, 514 * 4, s));
            GNS_HIP(hipMemsetAsync(ex->hot_ids, 0xFF, kExHot * 4, s));
            hipLaunchKernelGGL(k_exh_hist, dim3(std::min<unsigned>(sg, 2048)), dim3(256), 0, s, ex->f.pkts, ex->slots,
                               ex->hctl);
            hipLaunchKernelGGL(k_exh_pick, dim3(1), dim3(512), 0, s, ex->hctl, ex->hctl + 512);
            hipLaunchKernelGGL(k_exh_collect, dim3(sg), dim3(256), 0, s, ex->f.pkts, ex->slots, ex->hctl + 512,
                               ex->hctl + 513, ex->hot_ids);
        }
        hipLaunchKernelGGL(k_exh_table, dim3(1), dim3(kExHot), 0, s, ex->hot_ids, ex->f.pkts, ex->hot_tab);
        GNS_HIP(hipGetLastError());
    }
    ex->pkt += n;
    ex->batches++;
    ex->warm = true;
    return GNS_OK;
}

// Sort-word fields for the current table: flow ids < slots (invalid packets =
// slots), packet index, wire length (>= 12 bits; a longer length is read back by X3).
int ex_geometry(gns_ex *ex) {
    uint32_t kb = 1;
    while ((1ull << kb) <= ex->slots) kb++;
    ex->key_bits = kb;
    if (64 - kb - ceil_log2(ex->bmax) < 12) ex->bmax = 1ull << (52 - kb);
    ex->nblk_max = (uint32_t)(ex->bmax / kXChunk);
    ex->ib = std::max<uint32_t>(1, ceil_log2(ex->bmax));
    ex->sb = std::min<uint32_t>(31, 64 - kb - ex->ib);
    return GNS_OK;
}

// The exact aggregator keeps every flow of the period (exact/task.go:135-148
// grows a Go map): when the dictionary fills, the table doubles.  Flows with
// packets are reinserted (gns_dict.hip) and their state follows them; the
// claims of an aborted batch (flows without packets yet) are dropped.
int ex_grow(gns_ex *ex) {
    const uint64_t old_slots = ex->slots, new_slots = old_slots * 2;
    if (new_slots > (1ull << 30)) {
        set_error("exact flow dictionary cannot grow beyond 2^30 slots (%llu flows)", (unsigned long long)ex->claimed);
        return GNS_E_FULL;
    }
    const auto t0 = std::chrono::steady_clock::now();
    FlowState nf{};
    int rc = GNS_OK;
    if ((rc = dalloc_t(&nf.pkts, new_slots)) || (rc = dalloc_t(&nf.bytes, new_slots)) ||
        (rc = dalloc_t(&nf.first, new_slots)) || (rc = dalloc_t(&nf.last, new_slots)) ||
        (rc = dalloc_t(&nf.start, new_slots)) || (rc = dalloc_t(&nf.end, new_slots))) {
        dfree(nf.pkts); dfree(nf.bytes); dfree(nf.first); dfree(nf.last); dfree(nf.start); dfree(nf.end);
        return rc;
    }
    uint64_t slots = ex->slots, live = 0;
    rc = dict_rebuild(ex->D, slots, nullptr, 0, ex->f.pkts, nullptr, 0, new_slots, ex->stream, ex->dsc, &live, nullptr);
    if (rc != GNS_OK) {
        dfree(nf.pkts); dfree(nf.bytes); dfree(nf.first); dfree(nf.last); dfree(nf.start); dfree(nf.end);
        return rc;
    }
    hipLaunchKernelGGL(k_ex_init, dim3((unsigned)((new_slots + 255) / 256)), dim3(256), 0, ex->stream, nf, new_slots);
    hipLaunchKernelGGL(k_ex_permute, dim3((unsigned)((old_slots + 255) / 256)), dim3(256), 0, ex->stream, ex->f,
                       old_slots, ex->dsc.remap, nf);
    GNS_HIP(hipGetLastError());
    GNS_HIP(hipStreamSynchronize(ex->stream));
    dfree(ex->f.pkts); dfree(ex->f.bytes); dfree(ex->f.first); dfree(ex->f.last); dfree(ex->f.start); dfree(ex->f.end);
    ex->f = nf;
    ex->slots = new_slots;
    ex->D.cap = (uint32_t)(new_slots - new_slots / 4);
    ex->claimed = live;
    GNS_TRY(ex_geometry(ex));
    GNS_TRY(ex_hot_clear(ex));  // designated ids name old slots
    ex->n_grow++;
    ex->grow_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return GNS_OK;
}

template <int KIND>
int ex_dispatch(gns_ex *ex, const ExIn &x, uint64_t n) {
    switch (plan_mode(ex->kp)) {
    case PLAN_SLICE0: return ex_run_batch<KIND, PLAN_SLICE0>(ex, x, n);
    case PLAN_SLICE4: return ex_run_batch<KIND, PLAN_SLICE4>(ex, x, n);
    default: return ex_run_batch<KIND, PLAN_GENERIC>(ex, x, n);
    }
}

// One device batch with table growth: a batch that overflows the dictionary is
// aborted before X3 touches the flow state, its counters are undone, the table
// doubles and the batch runs again.
ExIn ex_advance(const ExIn &x0, uint64_t off) {
    ExIn x = x0;
    InputDesc &d = x.in;
    if (d.hdr) d.hdr += off * 16;
    if (d.src16) d.src16 += off * 16;
    if (d.dst16) d.dst16 += off * 16;
    if (d.sport) d.sport += off;
    if (d.dport) d.dport += off;
    if (d.proto) d.proto += off;
    if (d.sizes) d.sizes += off;
    if (x.ipver) x.ipver += off;
    x.ts += off;
    return x;
}

template <int KIND>
int ex_batch_recover(gns_ex *ex, const ExIn &x, uint64_t m) {
    if (ex->claimed >= ex->slots / 2) GNS_TRY(ex_grow(ex));  // keep the load <= ~1/2
    if (m > ex->bmax) {  // a grown table leaves fewer sort-word bits for the packet index
        for (uint64_t off = 0; off < m; off += ex->bmax)
            GNS_TRY(ex_batch_recover<KIND>(ex, ex_advance(x, off), std::min<uint64_t>(ex->bmax, m - off)));
        return GNS_OK;
    }
    for (;;) {
        GNS_HIP(hipMemcpyAsync(ex->stats_bak, ex->stats, 3 * sizeof(unsigned long long), hipMemcpyDeviceToDevice, ex->stream));
        const int rc = ex_dispatch<KIND>(ex, x, m);
        if (rc != GNS_E_FULL) return rc;
        GNS_HIP(hipMemcpyAsync(ex->stats, ex->stats_bak, 3 * sizeof(unsigned long long), hipMemcpyDeviceToDevice, ex->stream));
        GNS_HIP(hipMemsetAsync(ex->stats + 3, 0, sizeof(unsigned long long), ex->stream));
        ex->n_retry++;
        const int g = ex_grow(ex);
        if (g != GNS_OK) {
            const unsigned long long one = 1;
            (void)hipMemcpy(ex->stats + 3, &one, sizeof(one), hipMemcpyHostToDevice);
            return g;
        }
        if (m > ex->bmax) return ex_batch_recover<KIND>(ex, x, m);
    }
}

template <int KIND>
int ex_insert(gns_ex *ex, const ExIn &x0, uint64_t n, gns_mem where) {
    GNS_TRY(ex_set_dev(ex));
    for (uint64_t off = 0, m = 0; off < n; off += m) {
        // a batch without designated flows sends every packet through P (the heavy
        // flows serialise in P4's LDS atomics): keep it short, so that designation
        // starts early (as Count-Min's cold start)
        const uint64_t cap = ex->warm ? ex->bmax : std::min<uint64_t>(ex->bmax, std::max<uint64_t>(1ull << 20, ex->bmax / 32));
        m = std::min<uint64_t>(cap, n - off);
        ExIn x = x0;
        InputDesc &d = x.in;
        const InputDesc &in = x0.in;
        if (where == GNS_MEM_DEVICE) {
            x = ex_advance(x0, off);
        } else {
            const void *src[9] = {in.hdr ? (const void *)(in.hdr + off * 16) : nullptr,
                                  in.src16 ? (const void *)(in.src16 + off * 16) : nullptr,
                                  in.dst16 ? (const void *)(in.dst16 + off * 16) : nullptr,
                                  in.sport ? (const void *)(in.sport + off) : nullptr,
                                  in.dport ? (const void *)(in.dport + off) : nullptr,
                                  in.proto ? (const void *)(in.proto + off) : nullptr,
                                  in.sizes ? (const void *)(in.sizes + off) : nullptr,
                                  x0.ipver ? (const void *)(x0.ipver + off) : nullptr,
                                  (const void *)(x0.ts + off)};
            const size_t bytes[9] = {in.hdr ? m * 64 : 0, in.src16 ? m * 16 : 0, in.dst16 ? m * 16 : 0,
                                     in.sport ? m * 2 : 0, in.dport ? m * 2 : 0, in.proto ? m : 0,
                                     in.sizes ? m * 4 : 0, x0.ipver ? m : 0, m * 8};
            size_t tot = 0;
            for (int i = 0; i < 9; i++) tot += (bytes[i] + 15) & ~size_t(15);
            if (ex->stage_bytes < tot) {
                dfree(ex->stage);
                ex->stage = nullptr;
                ex->stage_bytes = 0;
                GNS_TRY(dalloc(reinterpret_cast<void **>(&ex->stage), tot));
                ex->stage_bytes = tot;
            }
            uint8_t *p = ex->stage;
            const void **dst[9] = {(const void **)&d.hdr, (const void **)&d.src16, (const void **)&d.dst16,
                                   (const void **)&d.sport, (const void **)&d.dport, (const void **)&d.proto,
                                   (const void **)&d.sizes, (const void **)&x.ipver, (const void **)&x.ts};
            for (int i = 0; i < 9; i++) {
                if (!bytes[i]) continue;
                GNS_HIP(hipMemcpyAsync(p, src[i], bytes[i], hipMemcpyHostToDevice, ex->stream));
                *dst[i] = p;
                p += (bytes[i] + 15) & ~size_t(15);
            }
        }
        GNS_TRY(ex_batch_recover<KIND>(ex, x, m));
    }
    return GNS_OK;
}

}  // namespace

extern "C" {

int gns_ex_create(const gns_ex_params *p, gns_ex **out) {
    if (!p || !out) { set_error("null argument"); return GNS_E_ARG; }
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        (void)hipGetLastError();
        set_error("no HIP device available");
        return GNS_E_NODEV;
    }
    if (p->device < 0 || p->device >= ndev) { set_error("device %d out of range", p->device); return GNS_E_ARG; }
    gns_ex *ex = new gns_ex();
    ex->device = p->device;
    int rc = GNS_OK;
    do {
        if ((rc = ex_set_dev(ex)) != GNS_OK) break;
        if (p->key.n_fields == 0) { set_error("exact task needs key_fields"); rc = GNS_E_ARG; break; }
        for (uint32_t i = 0; i < p->key.n_fields; i++)
            if (p->key.fields[i] < GNS_F_SRCIP || p->key.fields[i] > GNS_F_PROTO) {
                set_error("unknown key field id %u (task.go:363 rejects it)", p->key.fields[i]);
                rc = GNS_E_ARG;
            }
        if (rc) break;
        if ((rc = make_plan(p->key, 0, &ex->kp)) != GNS_OK) break;
        ex->K = ex->kp.K;
        if (hipStreamCreateWithFlags(&ex->stream, hipStreamNonBlocking) != hipSuccess) {
            set_error("hipStreamCreate failed"); rc = GNS_E_HIP; break;
        }
        ex->timer.stream = ex->stream;
        const uint64_t mf = p->max_flows ? p->max_flows : (4ull << 20);
        uint64_t slots = 1;
        while (slots < 2 * mf) slots <<= 1;
        if (slots > (1ull << 30)) { set_error("max_flows too large"); rc = GNS_E_ARG; break; }
        ex->slots = slots;
        ex->D.mask = (uint32_t)(slots - 1);
        ex->D.K = ex->K;
        ex->D.RW = dict_record_words(ex->K);
        ex->D.seed = 0x5BD1E995u;
        {
            const char *env = getenv("GNS_EX_LIST");
            ex->force_list = env && env[0] == '1';
        }
        ex->bmax = p->batch_packets ? p->batch_packets : (16ull << 20);
        ex->bmax = std::min<uint64_t>(((ex->bmax + kXChunk - 1) / kXChunk) * kXChunk, 1ull << 31);
        {   // sort word fields (ex_geometry, before the batch buffers are sized)
            uint32_t kb = 1;
            while ((1ull << kb) <= slots) kb++;
            if (64 - kb - ceil_log2(ex->bmax) < 12) ex->bmax = 1ull << (52 - kb);
        }
        ex->nblk_max = (uint32_t)(ex->bmax / kXChunk);
        if ((rc = dalloc_t(&ex->D.rec, slots * ex->D.RW)) || (rc = dalloc_t(&ex->f.pkts, slots)) ||
            (rc = dalloc_t(&ex->f.bytes, slots)) || (rc = dalloc_t(&ex->f.first, slots)) ||
            (rc = dalloc_t(&ex->f.last, slots)) || (rc = dalloc_t(&ex->f.start, slots)) ||
            (rc = dalloc_t(&ex->f.end, slots)) ||
            (rc = dalloc_t(&ex->pend[0], ex->bmax)) || (rc = dalloc_t(&ex->pend[1], ex->bmax)) ||
            (rc = dalloc_t(&ex->pcnt[0], ex->nblk_max)) || (rc = dalloc_t(&ex->pcnt[1], ex->nblk_max)) ||
            (rc = dalloc_t(&ex->ptotal, 2)) || (rc = dalloc_t(&ex->stats, 8)) ||
            (rc = dalloc_t(&ex->sk[0], ex->bmax)) || (rc = dalloc_t(&ex->sk[1], ex->bmax)) ||
            (rc = dalloc_t(&ex->hot_ids, kExHot)) || (rc = dalloc_t(&ex->touch, ex->bmax + kExHot)) || (rc = dalloc_t(&ex->hot_tab, kExHotTab)) ||
            (rc = dalloc_t(&ex->hpart, (uint64_t)kExHot * ex->nblk_max)) || (rc = dalloc_t(&ex->hctl, 516)) ||
            (rc = dalloc_t(&ex->ccnt, ex->nblk_max)) || (rc = dalloc_t(&ex->ph, (uint64_t)ex->nblk_max * kPBins)) ||
            (rc = dalloc_t(&ex->pgs, (uint64_t)(ex->nblk_max / kPGroup + 1) * kPBins)) ||
            (rc = dalloc_t(&ex->pb, kPBins + 1)))
            break;
        if ((rc = ex_geometry(ex)) != GNS_OK) break;
        if ((rc = dalloc_t(&ex->dctl, 4)) != GNS_OK || (rc = dalloc_t(&ex->stats_bak, 3)) != GNS_OK) break;
        ex->D.ctl = ex->dctl;
        ex->D.cap = (uint32_t)(slots - slots / 4);
        if (hipHostMalloc(reinterpret_cast<void **>(&ex->h_pin), 64, 0) != hipSuccess) {
            set_error("hipHostMalloc failed"); rc = GNS_E_OOM; break;
        }
        if (hipMemsetAsync(ex->stats, 0, 64, ex->stream) != hipSuccess) { rc = GNS_E_HIP; break; }
        if ((rc = ex_clear(ex)) != GNS_OK) break;
        if (hipStreamSynchronize(ex->stream) != hipSuccess) { rc = GNS_E_HIP; break; }
    } while (0);
    if (rc != GNS_OK) {
        ex_free_all(ex);
        delete ex;
        return rc;
    }
    *out = ex;
    return GNS_OK;
}

int gns_ex_destroy(gns_ex *ex) {
    if (!ex) return GNS_OK;
    (void)hipSetDevice(ex->device);
    if (ex->stream) (void)hipStreamSynchronize(ex->stream);
    ex_free_all(ex);
    delete ex;
    return GNS_OK;
}

int gns_ex_insert_tuples(gns_ex *ex, const gns_tuples *t, const uint8_t *ipver, const int64_t *ts_ns,
                         uint64_t n, gns_mem where) {
    if (!ex || !t) { set_error("null argument"); return GNS_E_ARG; }
    if (n && (!t->src16 || !t->dst16 || !t->sport || !t->dport || !t->proto || !t->length || !ts_ns)) {
        set_error("null tuple array"); return GNS_E_ARG;
    }
    ExIn x{};
    x.in.src16 = t->src16; x.in.dst16 = t->dst16; x.in.sport = t->sport; x.in.dport = t->dport;
    x.in.proto = t->proto; x.in.sizes = t->length;
    x.ipver = ipver; x.ts = ts_ns;
    return ex_insert<IN_TUPLE>(ex, x, n, where);
}

int gns_ex_insert_headers(gns_ex *ex, const uint8_t *hdr, const uint32_t *wirelen, const int64_t *ts_ns,
                          uint64_t n, gns_mem where) {
    if (!ex || (n && (!hdr || !wirelen || !ts_ns))) { set_error("null argument"); return GNS_E_ARG; }
    ExIn x{};
    x.in.hdr = reinterpret_cast<const uint32_t *>(hdr);
    x.in.sizes = wirelen;
    x.ts = ts_ns;
    return ex_insert<IN_HDR>(ex, x, n, where);
}

int gns_ex_flush(gns_ex *ex) {
    if (!ex) return GNS_E_ARG;
    GNS_TRY(ex_set_dev(ex));
    GNS_HIP(hipStreamSynchronize(ex->stream));
    ex->timer.collect();
    return GNS_OK;
}

static int ex_query_impl(gns_ex *ex, const uint8_t *flows, uint32_t stride, uint64_t n, uint64_t *out, bool dev) {
    if (!ex || (n && (!flows || !out))) { set_error("null argument"); return GNS_E_ARG; }
    if (n == 0) return GNS_OK;
    if (stride < ex->K) { set_error("stride < key bytes"); return GNS_E_ARG; }
    if (dev && ((uintptr_t)out & 7u) != 0) { set_error("answers not 8-byte aligned"); return GNS_E_ARG; }
    GNS_TRY(ex_set_dev(ex));
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
    hipError_t e = dev ? hipSuccess : hipMemcpyAsync(dk, flows, n * stride, hipMemcpyHostToDevice, ex->stream);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_ex_query, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ex->stream, dk, stride, n,
                           ex->K, ex->D, ex->f, dout);
        e = hipGetLastError();
    }
    if (e == hipSuccess && !dev) e = hipMemcpyAsync(out, dout, n * 8, hipMemcpyDeviceToHost, ex->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ex->stream);
    if (!dev) {
        dfree(dk);
        dfree(dout);
    }
    if (e != hipSuccess) { set_error("exact query: %s", hipGetErrorString(e)); return GNS_E_HIP; }
    return GNS_OK;
}

int gns_ex_query(gns_ex *ex, const uint8_t *flows, uint32_t stride, uint64_t n, uint64_t *out) {
    return ex_query_impl(ex, flows, stride, n, out, false);
}

int gns_ex_query_device(gns_ex *ex, const uint8_t *flows, uint32_t stride, uint64_t n, uint64_t *out) {
    return ex_query_impl(ex, flows, stride, n, out, true);
}

int gns_ex_snapshot(gns_ex *ex, uint8_t *keys, int64_t *start_ns, int64_t *end_ns, uint64_t *pkts,
                    uint64_t *bytes, uint64_t *n_io) {
    if (!ex || !n_io) { set_error("null argument"); return GNS_E_ARG; }
    GNS_TRY(ex_set_dev(ex));
    hipStream_t s = ex->stream;
    uint32_t *ids = nullptr, *cnt = nullptr;
    GNS_TRY(dalloc(reinterpret_cast<void **>(&cnt), 16));
    int rc = dalloc(reinterpret_cast<void **>(&ids), ex->slots * 4);
    if (rc) { dfree(cnt); return rc; }
    uint32_t nf = 0;
    hipError_t e = hipMemsetAsync(cnt, 0, 4, s);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(k_ex_list, dim3((unsigned)((ex->slots + 255) / 256)), dim3(256), 0, s, ex->D, ex->slots,
                           ex->f.pkts, ids, cnt);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(&nf, cnt, 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    const uint64_t cap = *n_io;
    *n_io = nf;
    const uint64_t m = std::min<uint64_t>(cap, nf);
    if (e == hipSuccess && m > 0 && (keys || start_ns || end_ns || pkts || bytes)) {
        // slot order (deterministic)
        std::vector<uint32_t> h(nf);
        e = hipMemcpy(h.data(), ids, (size_t)nf * 4, hipMemcpyDeviceToHost);
        std::sort(h.begin(), h.end());
        if (e == hipSuccess) e = hipMemcpy(ids, h.data(), (size_t)m * 4, hipMemcpyHostToDevice);
        uint8_t *dk = nullptr;
        long long *ds = nullptr, *de = nullptr;
        unsigned long long *dp = nullptr, *db = nullptr;
        const size_t kb = (size_t)m * std::max<uint32_t>(ex->K, 1);
        if (e == hipSuccess && (dalloc(reinterpret_cast<void **>(&dk), kb) || dalloc_t(&ds, m) || dalloc_t(&de, m) ||
                                dalloc_t(&dp, m) || dalloc_t(&db, m)))
            e = hipErrorOutOfMemory;
        if (e == hipSuccess) {
            hipLaunchKernelGGL(k_ex_gather, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, ids, m, ex->D, ex->f,
                               dk, ds, de, dp, db);
            e = hipGetLastError();
        }
        if (e == hipSuccess && keys) e = hipMemcpyAsync(keys, dk, (size_t)m * ex->K, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess && start_ns) e = hipMemcpyAsync(start_ns, ds, m * 8, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess && end_ns) e = hipMemcpyAsync(end_ns, de, m * 8, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess && pkts) e = hipMemcpyAsync(pkts, dp, m * 8, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess && bytes) e = hipMemcpyAsync(bytes, db, m * 8, hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        dfree(dk); dfree(ds); dfree(de); dfree(dp); dfree(db);
    }
    dfree(ids);
    dfree(cnt);
    if (e != hipSuccess) { set_error("exact snapshot: %s", hipGetErrorString(e)); return GNS_E_HIP; }
    return GNS_OK;
}

int gns_ex_reset(gns_ex *ex) {
    if (!ex) return GNS_E_ARG;
    GNS_TRY(ex_set_dev(ex));
    GNS_TRY(ex_clear(ex));
    GNS_HIP(hipStreamSynchronize(ex->stream));
    return GNS_OK;
}

int gns_ex_counters(gns_ex *ex, uint64_t out[8]) {
    if (!ex || !out) return GNS_E_ARG;
    GNS_TRY(ex_set_dev(ex));
    GNS_HIP(hipStreamSynchronize(ex->stream));
    unsigned long long h[8];
    GNS_HIP(hipMemcpy(h, ex->stats, sizeof(h), hipMemcpyDeviceToHost));
    uint64_t nf = 0;
    GNS_TRY(gns_ex_snapshot(ex, nullptr, nullptr, nullptr, nullptr, nullptr, &nf));
    out[0] = h[0]; out[1] = h[1]; out[2] = h[2]; out[3] = h[3];
    out[4] = nf; out[5] = ex->pkt; out[6] = ex->batches; out[7] = 0;
    return GNS_OK;
}

int gns_ex_dict_stats(gns_ex *ex, uint64_t out[8]) {
    if (!ex || !out) return GNS_E_ARG;
    out[0] = ex->n_grow; out[1] = 0; out[2] = ex->slots; out[3] = ex->claimed;
    out[4] = (uint64_t)(ex->grow_ms * 1000.0); out[5] = ex->n_retry;
    out[6] = ex->slots; out[7] = ex->n_grow;
    return GNS_OK;
}

int gns_ex_set_timing(gns_ex *ex, int on) {
    if (!ex) return GNS_E_ARG;
    set_timing_arg(ex->timer, on);
    return GNS_OK;
}

int gns_ex_stage_times(gns_ex *ex, double ms[8], uint64_t launches[8], int reset) {
    if (!ex) return GNS_E_ARG;
    GNS_TRY(ex_set_dev(ex));
    ex->timer.collect();
    for (int i = 0; i < 8; i++) {
        if (ms) ms[i] = ex->timer.ms[i];
        if (launches) launches[i] = ex->timer.launches[i];
    }
    if (reset) for (int i = 0; i < 8; i++) { ex->timer.ms[i] = 0; ex->timer.launches[i] = 0; }
    return GNS_OK;
}

}  // extern "C"
