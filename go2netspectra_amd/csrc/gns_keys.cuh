// gns_keys.cuh -- per-packet key derivation from the three input kinds, and the
// exact device flow dictionary (key bytes -> dense flow id).
//
// Flow ids make the bucket fingerprints 4-byte integers: two keys compare equal
// iff their ids are equal, because the dictionary stores full key bytes and
// compares them byte-exactly on every probe.  The dictionary is an
// open-addressing table with linear probing.  Slots are claimed with a device
// atomicCAS that writes the claim epoch; a slot claimed in the *current* launch
// is never read (its key bytes are not yet visible), the packet is parked in a
// pending list and re-probed by the next launch (kernel boundaries publish the
// key bytes).  Records: word 0 = tag (0 empty, else claim epoch), words
// 1..nkw = key words, padded to RW (multiple of 4) words.
#pragma once
#include "gns_device.cuh"

namespace gns {

enum InputKind { IN_HDR = 0, IN_TUPLE = 1, IN_KEYS = 2, IN_REC16 = 3 };

// Compact host record (IN_REC16): 16 bytes + the wire length,
// for the PCIe-bound host-inclusive path.  Words = canonical tuple words
// {tw[0], tw[4], tw[8], tw[9]}: IPv4 source / destination (left-aligned
// slots), ports, protocol | IP versions << 16.  Tuple byte 37 (bits 8..15 of
// word 3) is zero in every tuple and carries the record class instead:
//   kRecTuple  the IPv4 tuple above;
//   kRecDrop   no IP layer (parser.go:48-49: not counted);
//   kRecSide   anything else (IPv6, unsupported shapes): word 0 indexes a
//              64-byte record in the side array, parsed as gns_*_insert_headers would.
// The 16-byte form (InputDesc.rec_len) carries the wire length in bits 16..31 of
// word 3 instead of the IP versions, which a tuple record then implies (IPv4 both
// ways; any other tuple escapes to the side array): 16 B per packet over the bus.
enum { kRecTuple = 0, kRecDrop = 1, kRecSide = 2 };

struct InputDesc {
    const uint32_t *hdr;      // IN_HDR: n*16 words
    const uint8_t *src16;     // IN_TUPLE
    const uint8_t *dst16;
    const uint16_t *sport;
    const uint16_t *dport;
    const uint8_t *proto;
    const uint8_t *keys;      // IN_KEYS: flow keys, n*stride bytes
    const uint8_t *keys2;     // IN_KEYS: element keys (SuperSpread)
    const uint32_t *sizes;    // per-packet size (wirelen / length / sizes)
    const uint32_t *rec16;    // IN_REC16: n*4 words
    const uint32_t *side;     // IN_REC16: 64-byte records named by kRecSide escapes
    uint64_t n_side;          // IN_REC16: records in side (an escape at or past it is unsupported)
    uint32_t rec_len;         // IN_REC16: wire lengths in the records (sizes then unpacked from them)
    uint32_t stride, stride2;
    uint32_t aligned;         // bit0: keys word-loadable, bit1: keys2 word-loadable
};

template <int NW>
__device__ __forceinline__ uint32_t mm3_n(const uint32_t (&kw)[NW], uint32_t K, uint32_t seed) {
    const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
    uint32_t h = seed;
    const uint32_t nb = K >> 2;
#pragma unroll
    for (int i = 0; i < NW; i++) {
        uint32_t k = kw[i];
        if ((uint32_t)i < nb) {
            k *= c1; k = rotl32(k, 15); k *= c2;
            h ^= k; h = rotl32(h, 13); h = h * 5u + 0xe6546b64u;
        } else if ((uint32_t)i == nb && (K & 3u)) {
            k *= c1; k = rotl32(k, 15); k *= c2;
            h ^= k;
        }
    }
    h ^= K;
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    return h;
}

// MurmurHash3 split: the per-block key mixing k*c1, rotl 15, *c2 does not depend
// on the seed, so a key hashed under several seeds (d rows + the dictionary)
// is mixed once (mm3_premix) and each seed only runs the cheap h-chain.
template <int NW>
__device__ __forceinline__ void mm3_premix(const uint32_t (&kw)[NW], uint32_t K, uint32_t (&mk)[NW]) {
    const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
#pragma unroll
    for (int i = 0; i < NW; i++) {
        uint32_t k = kw[i];
        k *= c1; k = rotl32(k, 15); k *= c2;
        mk[i] = (4u * i < K) ? k : 0u;
    }
}

template <int NW>
__device__ __forceinline__ uint32_t mm3_chain(const uint32_t (&mk)[NW], uint32_t K, uint32_t seed) {
    uint32_t h = seed;
    const uint32_t nb = K >> 2;
#pragma unroll
    for (int i = 0; i < NW; i++) {
        if ((uint32_t)i < nb) {
            h ^= mk[i]; h = rotl32(h, 13); h = h * 5u + 0xe6546b64u;
        } else if ((uint32_t)i == nb && (K & 3u)) {
            h ^= mk[i];
        }
    }
    h ^= K;
    h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
    return h;
}

// Load K key bytes at p into little-endian words (bytes >= K zero).
template <int NW>
__device__ __forceinline__ void load_key_bytes(const uint8_t *p, uint32_t K, bool word_ok,
                                               uint32_t (&kw)[NW]) {
    if (word_ok) {
        const uint32_t *q = reinterpret_cast<const uint32_t *>(p);
#pragma unroll
        for (int i = 0; i < NW; i++) kw[i] = (4u * i < K) ? (q[i] & tail_mask(K, i)) : 0u;
    } else {
#pragma unroll
        for (int i = 0; i < NW; i++) {
            uint32_t v = 0;
#pragma unroll
            for (int b = 0; b < 4; b++)
                if ((uint32_t)(4 * i + b) < K) v |= (uint32_t)p[4 * i + b] << (8 * b);
            kw[i] = v;
        }
    }
}

// Canonical tuple words for packet p from a header record or a PacketInfo.
// Returns PARSE_*.
template <int KIND>
__device__ __forceinline__ int load_tuple(const InputDesc &in, uint64_t p, uint32_t (&tw)[10]) {
    if constexpr (KIND == IN_HDR) {
        uint32_t w[16];
        const uint4 *r = reinterpret_cast<const uint4 *>(in.hdr + p * 16);
#pragma unroll
        for (int i = 0; i < 4; i++) {
            uint4 v = r[i];
            w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
        }
        return parse_record_fast(w, in.sizes[p], true, tw);
    } else if constexpr (KIND == IN_REC16) {
        const uint4 r = *reinterpret_cast<const uint4 *>(in.rec16 + p * 4);
        const uint32_t cls = (r.w >> 8) & 0xFFu;
        tw[0] = r.x; tw[1] = 0; tw[2] = 0; tw[3] = 0;
        tw[4] = r.y; tw[5] = 0; tw[6] = 0; tw[7] = 0;
        tw[8] = r.z; tw[9] = in.rec_len ? ((r.w & 0xFFu) | 0x04040000u) : r.w;
        if (cls == kRecTuple) return PARSE_OK;
        if (cls == kRecDrop) return PARSE_DROP;
        int st = PARSE_UNSUPPORTED;
        if (cls == kRecSide && (uint64_t)r.x < in.n_side) {  // a short or missing side array: unsupported, never read
            uint32_t w[16];
            const uint4 *q = reinterpret_cast<const uint4 *>(in.side + (uint64_t)r.x * 16);
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const uint4 v = q[i];
                w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
            }
            st = parse_record(w, in.sizes[p], tw);
        }
        return st;
    } else {
        const uint4 s = *reinterpret_cast<const uint4 *>(in.src16 + p * 16);
        const uint4 d = *reinterpret_cast<const uint4 *>(in.dst16 + p * 16);
        tw[0] = s.x; tw[1] = s.y; tw[2] = s.z; tw[3] = s.w;
        tw[4] = d.x; tw[5] = d.y; tw[6] = d.z; tw[7] = d.w;
        set_ports(tw, in.sport[p], in.dport[p], in.proto[p]);
        return PARSE_OK;
    }
}

// Generic byte-selection key builder over a plan with up to NW*4 bytes.
struct KeyPlanN {
    uint32_t K;
    int32_t woff;        // >= 0: key == tuple bytes [4*woff, 4*woff+K)
    uint8_t src[80];     // tuple byte index per key byte
};

enum PlanMode { PLAN_SLICE0 = 0, PLAN_SLICE4 = 1, PLAN_GENERIC = 2 };

__host__ __device__ inline int plan_mode(const KeyPlanN &kp) {
    return kp.woff == 0 ? PLAN_SLICE0 : (kp.woff == 4 ? PLAN_SLICE4 : PLAN_GENERIC);
}

// Key words from tuple words.  MODE is a template parameter so the slice
// layouts compile to plain word moves; the generic layout reads its byte
// source table from LDS (s_src, staged once per block by stage_plan()).
template <int MODE, int NW>
__device__ __forceinline__ void make_key_m(uint32_t K, const uint8_t *s_src, const uint32_t (&tw)[10],
                                           uint32_t (&kw)[NW]) {
    if constexpr (MODE == PLAN_SLICE0) {
#pragma unroll
        for (int i = 0; i < NW; i++) kw[i] = (i < 10 ? tw[i < 10 ? i : 0] : 0u) & tail_mask(K, i);
    } else if constexpr (MODE == PLAN_SLICE4) {
#pragma unroll
        for (int i = 0; i < NW; i++) kw[i] = (i + 4 < 10 ? tw[i + 4 < 10 ? i + 4 : 0] : 0u) & tail_mask(K, i);
    } else {
#pragma unroll
        for (int i = 0; i < NW; i++) {
            uint32_t v = 0;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const int j = 4 * i + b;
                if ((uint32_t)j < K) v |= tuple_byte(tw, s_src[j]) << (8 * b);
            }
            kw[i] = v;
        }
    }
}

template <int MODE>
__device__ __forceinline__ void stage_plan(const KeyPlanN &kp, uint8_t *s_src) {
    if constexpr (MODE == PLAN_GENERIC) {
        for (uint32_t j = threadIdx.x; j < 80; j += blockDim.x) s_src[j] = kp.src[j];
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------
// Flow dictionary
// ---------------------------------------------------------------------------
struct DictDev {
    uint32_t *rec;     // slots * RW words
    uint32_t mask;     // slots - 1
    uint32_t RW;       // record words: 4, 8 or 16 (a record never straddles a 64-byte line)
    uint32_t seed;     // slot hash seed
    uint32_t K;        // key bytes
    uint32_t bw;       // Count-Min: words 12..15 cache the flow's row 0..3 buckets
    uint32_t *ctl;     // [0] slots claimed since the last rebuild / reset, [1] abort flag of the batch
    uint32_t cap;      // claims beyond this abort the batch (the host reclaims and retries it)
};

// rebuild mark (gns_dict.hip); ids are slots below it
constexpr uint32_t kDictMarked = 0xFFFFFFFEu;

enum { DICT_FOUND = 0, DICT_PENDING = 1, DICT_FULL = 2, DICT_ABSENT = 3, DICT_CLAIMED = 4 };

// Claim accounting, one global atomic per block: the block's claims are added
// to ctl[0]; crossing the cap raises the batch's abort flag and the caller's
// dictionary-full word (the host then reclaims dead flows / grows the table and
// re-runs the batch, which was not applied).
__device__ __forceinline__ void dict_flush_claims(const DictDev &D, uint32_t n, unsigned long long *full_word) {
    if (n == 0 || D.ctl == nullptr) return;
    const uint32_t old = atomicAdd(&D.ctl[0], n);
    if ((uint64_t)old + n > D.cap) {
        atomicExch(&D.ctl[1], 1u);
        atomicAdd(full_word, 1ull);
    }
}

// the batch was aborted (read by one thread, then shared: block-uniform exits)
__device__ __forceinline__ bool dict_aborted(const DictDev &D) {
    return D.ctl != nullptr && __hip_atomic_load(&D.ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
}
#define GNS_DICT_MAX_PROBE 4096

__device__ __forceinline__ void load_record(const DictDev &D, uint32_t slot, uint32_t (&r)[12]) {
    const uint4 *q = reinterpret_cast<const uint4 *>(D.rec + (size_t)slot * D.RW);
#pragma unroll
    for (int i = 0; i < 3; i++) {
        uint4 v = (4u * i < D.RW) ? q[i] : make_uint4(0, 0, 0, 0);
        r[4 * i] = v.x; r[4 * i + 1] = v.y; r[4 * i + 2] = v.z; r[4 * i + 3] = v.w;
    }
}

// Find the id of kw, claiming an empty slot for it if absent.
// DICT_FOUND / DICT_CLAIMED (this lane inserted the key): *out = id.
// DICT_PENDING: *out = slot to resume at next launch.
__device__ __forceinline__ int dict_find_or_claim(const DictDev &D, const uint32_t (&kw)[GNS_KWMAX],
                                                  uint32_t slot, uint32_t epoch, uint32_t *out) {
    const uint32_t nkw = (D.K + 3) >> 2;
    for (int probe = 0; probe < GNS_DICT_MAX_PROBE; probe++) {
        uint32_t r[12];
        load_record(D, slot, r);
        uint32_t tag = r[0];
        if (tag == 0) {
            uint32_t *tp = D.rec + (size_t)slot * D.RW;
            const uint32_t old = atomicCAS(tp, 0u, epoch);
            if (old == 0) {
#pragma unroll
                for (int i = 0; i < GNS_KWMAX; i++)
                    if ((uint32_t)i < nkw) tp[1 + i] = kw[i];
                *out = slot;
                return DICT_CLAIMED;
            }
            tag = old;
            if (tag != epoch) load_record(D, slot, r);  // committed earlier: need its key words
        }
        if (tag == epoch) { *out = slot; return DICT_PENDING; }
        bool eq = true;
#pragma unroll
        for (int i = 0; i < GNS_KWMAX; i++)
            if ((uint32_t)i < nkw) eq = eq && (r[1 + i] == kw[i]);
        if (eq) { *out = slot; return DICT_FOUND; }
        slot = (slot + 1u) & D.mask;
    }
    return DICT_FULL;
}

// Read-only lookup (after all inserts of the period are committed).
__device__ __forceinline__ uint32_t dict_lookup(const DictDev &D, const uint32_t (&kw)[GNS_KWMAX]) {
    const uint32_t nkw = (D.K + 3) >> 2;
    uint32_t slot = mm3_n<GNS_KWMAX>(kw, D.K, D.seed) & D.mask;
    for (int probe = 0; probe < GNS_DICT_MAX_PROBE; probe++) {
        uint32_t r[12];
        load_record(D, slot, r);
        if (r[0] == 0) return GNS_ID_NONE;
        bool eq = true;
#pragma unroll
        for (int i = 0; i < GNS_KWMAX; i++)
            if ((uint32_t)i < nkw) eq = eq && (r[1 + i] == kw[i]);
        if (eq) return slot;
        slot = (slot + 1u) & D.mask;
    }
    return GNS_ID_NONE;
}

}  // namespace gns
