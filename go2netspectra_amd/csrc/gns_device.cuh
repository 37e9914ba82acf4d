// gns_device.cuh -- gfx950 device helpers for the sketch hot path.
//
//   * MurmurHash3_x86_32 over a key held in registers as little-endian u32 words
//     (reference: internal/engine/impl/sketch/statistic/hash.go:13-53).
//   * 64-byte header record -> canonical 5-tuple words
//     (reference: internal/protocol/parser.go:23-67 over gopacket layers; the
//     record contract is DESIGN.md "Header records").
//   * flow-key assembly from the 5-tuple (reference: task.go:265-300).
//
// Canonical tuple words tw[10] (37 meaningful bytes, little-endian words):
//   bytes  0..15  SrcIP slot  (IPv4 left-aligned, 12 zero bytes; task.go:281-286)
//   bytes 16..31  DstIP slot
//   bytes 32..33  SrcPort big-endian, 34..35 DstPort big-endian
//   byte  36      Protocol
// Every flow-key layout is a byte selection from this 37-byte string.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define GNS_KWMAX 10        // ceil(37 / 4): longest key the reference allows (task.go:74)
#define GNS_ID_NONE 0xFFFFFFFFu

namespace gns {

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

// hash.go:13-53; key bytes k[0..K) packed little-endian in kw[], bytes >= K zero.
__device__ __forceinline__ uint32_t mm3_words(const uint32_t (&kw)[GNS_KWMAX], uint32_t K,
                                              uint32_t seed) {
    const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
    uint32_t h = seed;
    const uint32_t nb = K >> 2;
#pragma unroll
    for (int i = 0; i < GNS_KWMAX; i++) {
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

// ---------------------------------------------------------------------------
// byte access into a 64-byte record held as 16 little-endian words
// ---------------------------------------------------------------------------
template <int B>
__device__ __forceinline__ uint32_t rec_byte(const uint32_t (&w)[16]) {
    static_assert(B >= 0 && B < 64, "record byte out of range");
    return (w[B / 4] >> (8 * (B % 4))) & 0xFFu;
}
template <int B>
__device__ __forceinline__ uint32_t rec_be16(const uint32_t (&w)[16]) {
    return (rec_byte<B>(w) << 8) | rec_byte<B + 1>(w);
}
template <int B>
__device__ __forceinline__ uint32_t rec_u32(const uint32_t (&w)[16]) {  // bytes B..B+3, LE
    static_assert(B >= 0 && B + 3 < 64, "record word out of range");
    if constexpr (B % 4 == 0) return w[B / 4];
    else return __builtin_amdgcn_alignbyte(w[B / 4 + 1], w[B / 4], B % 4);  // v_alignbyte_b32 funnel shift
}

enum { PARSE_OK = 0, PARSE_DROP = 1, PARSE_UNSUPPORTED = 2 };

__device__ __forceinline__ bool udp_tunnel_port(uint32_t p) {
    return p == 4789u || p == 6081u || p == 2152u;
}

// (byte 36 = proto; bytes 37..39 = 0: callers add the IP version bytes after it)
__device__ __forceinline__ void set_ports(uint32_t (&tw)[10], uint32_t sport, uint32_t dport,
                                          uint32_t proto) {
    // bytes 32..35 = sport BE, dport BE; byte 36 = proto
    tw[8] = (sport >> 8) | ((sport & 0xFFu) << 8) | ((dport >> 8) << 16) | ((dport & 0xFFu) << 24);
    tw[9] = proto;
}

// L3/L4 decode of a record whose VLAN tags were shifted out: the ethertype is
// at bytes 12-13 and the L3 header at byte 14.  nv = number of removed tags
// (the original L2 header length is 14 + 4*nv); lim = record bytes still
// present (64 - 4*nv).  Offsets are compile-time constants: no dynamic
// indexing into the record registers.  Writes the IP version bytes (38, 39).
//
// gopacket v1.1.19 keeps a layer whose decode fails with the fields it set
// before the failing check (decodeIPv4 / decodeIPv6 / decodeTCP / decodeUDP
// call p.AddLayer before returning the error), and parser.go:38-61 reads them:
//   IPv4 data < 20 bytes       -> IPv4 layer with nil IPs: counted, zero IPs, proto 0
//   IPv4 Length < 20, IHL < 5, IHL*4 > Length -> IPs + protocol, ports 0
//   IPv6 data < 40 bytes       -> nil IPs, NextHeader 0
//   IPv6 Length 0 (no HBH)     -> IPs + NextHeader, ports 0
//   TCP < 20 bytes / UDP < 8   -> the layer with ports 0; a TCP data offset < 5 or
//                                 beyond the data errs after the ports are read
// Encapsulations and IPv6 extension chains whose inner layers gopacket decodes
// further are UNSUPPORTED here: the host packer decodes such frames and hands
// them over as pre-parsed 0x88B5 records.
__device__ __forceinline__ int parse_l3(const uint32_t (&w)[16], uint32_t type, uint32_t wirelen,
                                        uint32_t nv, uint32_t (&tw)[10]) {
    constexpr int OFF = 14;
    const uint32_t l2hdr = 14u + 4u * nv;
    const uint32_t lim = 64u - 4u * nv;
    const uint32_t l2len = wirelen > l2hdr ? wirelen - l2hdr : 0u;
    if (type == 0x0800u) {  // gopacket IPv4.DecodeFromBytes
        if (l2len < 20) return PARSE_OK;  // nil IPs (version bytes 0), protocol 0, no ports
        const uint32_t ihl = rec_byte<OFF>(w) & 15u;
        uint32_t tot = rec_be16<OFF + 2>(w);
        if (tot == 0) tot = l2len;  // TSO
        const uint32_t proto = rec_byte<OFF + 9>(w);
        tw[0] = rec_u32<OFF + 12>(w);  // parser.go:40-41: 4-byte IPv4, left-aligned slot
        tw[4] = rec_u32<OFF + 16>(w);
        tw[9] = proto | 4u << 24 | 4u << 16;
        if (tot < 20 || ihl < 5 || ihl * 4 > tot) return PARSE_OK;  // decode error: no further layers
        if (ihl > 5) return PARSE_UNSUPPORTED;                      // options: the host packer
        const uint32_t frag = rec_be16<OFF + 6>(w);
        if (frag & 0x3FFFu) return PARSE_OK;  // MF or offset: LayerTypeFragment, ports 0
        const uint32_t avail = (tot < l2len ? tot : l2len) - 20u;
        if (avail == 0) return PARSE_OK;      // empty payload: no next layer
        if (proto == 6u) {
            if (avail >= 20) {
                set_ports(tw, rec_be16<OFF + 20>(w), rec_be16<OFF + 22>(w), proto);
                tw[9] |= 4u << 24 | 4u << 16;
            }
            return PARSE_OK;
        }
        if (proto == 17u) {
            if (avail < 8) return PARSE_OK;
            const uint32_t sp = rec_be16<OFF + 20>(w), dp = rec_be16<OFF + 22>(w);
            if (udp_tunnel_port(sp) || udp_tunnel_port(dp)) return PARSE_UNSUPPORTED;
            set_ports(tw, sp, dp, proto);
            tw[9] |= 4u << 24 | 4u << 16;
            return PARSE_OK;
        }
        switch (proto) {  // inner layers gopacket decodes (HBH, IP-in-IP, routing, GRE, AH, dest opts, MPLS)
        case 0: case 4: case 41: case 43: case 47: case 51: case 60: case 137:
            return PARSE_UNSUPPORTED;
        default:
            return PARSE_OK;  // ICMP, IPv6 fragment header, ESP, ...: ports 0
        }
    }
    if (type == 0x86DDu) {  // gopacket IPv6.DecodeFromBytes
        if (l2len < 40) return PARSE_OK;  // nil IPs, NextHeader 0
        const uint32_t plen = rec_be16<OFF + 4>(w);
        const uint32_t nh = rec_byte<OFF + 6>(w);
        tw[0] = rec_u32<OFF + 8>(w);  tw[1] = rec_u32<OFF + 12>(w);
        tw[2] = rec_u32<OFF + 16>(w); tw[3] = rec_u32<OFF + 20>(w);
        tw[4] = rec_u32<OFF + 24>(w); tw[5] = rec_u32<OFF + 28>(w);
        tw[6] = rec_u32<OFF + 32>(w); tw[7] = rec_u32<OFF + 36>(w);
        tw[9] = nh | 6u << 24 | 6u << 16;  // parser.go:47: first NextHeader
        if (nh == 0) return PARSE_UNSUPPORTED;  // hop-by-hop (jumbogram rules): the host packer
        if (plen == 0) return PARSE_OK;         // "IPv6 length 0, but next header is ..."
        const uint32_t cap = l2len - 40u;
        const uint32_t avail = plen < cap ? plen : cap;
        if (avail == 0) return PARSE_OK;
        switch (nh) {
        case 4: case 41: case 43: case 47: case 51: case 60: case 137:
            return PARSE_UNSUPPORTED;
        default: break;
        }
        if (nh == 6u || nh == 17u) {
            if (avail < (nh == 6u ? 20u : 8u)) return PARSE_OK;
            if (OFF + 40 + 4 > lim) return PARSE_UNSUPPORTED;  // ports beyond the record
            const uint32_t sp = rec_be16<OFF + 40>(w), dp = rec_be16<OFF + 42>(w);
            if (nh == 17u && (udp_tunnel_port(sp) || udp_tunnel_port(dp))) return PARSE_UNSUPPORTED;
            set_ports(tw, sp, dp, nh);
            tw[9] |= 6u << 24 | 6u << 16;
            return PARSE_OK;
        }
        return PARSE_OK;
    }
    switch (type) {  // parser.go:48-49 "not an IP packet"
    case 0x0806: case 0x8035: case 0x88CC: case 0x8808: case 0x888E: case 0x88F7: case 0x8863:
        return PARSE_DROP;
    default:
        return PARSE_UNSUPPORTED;
    }
}

// 64-byte record -> canonical tuple words (bytes 0..36 = src16, dst16, sport,
// dport BE, proto; byte 39 / 38 = IP version of the source / destination:
// 4 or 6, 0 for a net.IP of another length).  Returns PARSE_*.
__device__ __forceinline__ int parse_record(const uint32_t (&w)[16], uint32_t wirelen,
                                            uint32_t (&tw)[10]) {
#pragma unroll
    for (int i = 0; i < 10; i++) tw[i] = 0;
    const uint32_t t0 = rec_be16<12>(w);
    if (t0 == 0x88B5u) {  // pre-parsed record (host packer escape)
        if (rec_byte<14>(w) != 1u) return PARSE_UNSUPPORTED;
        tw[0] = w[4]; tw[1] = w[5]; tw[2] = w[6];  tw[3] = w[7];
        tw[4] = w[8]; tw[5] = w[9]; tw[6] = w[10]; tw[7] = w[11];
        set_ports(tw, rec_be16<48>(w), rec_be16<50>(w), rec_byte<52>(w));
        // IP versions: byte 39 = source, byte 38 = destination (record byte 53; 0 -> same
        // as the source).  Bytes 37..39 lie outside every key plan.
        const uint32_t sv = rec_byte<15>(w), dv0 = rec_byte<53>(w);
        tw[9] |= sv << 24 | (dv0 ? dv0 : sv) << 16;
        return PARSE_OK;
    }
    // gopacket Dot1Q: up to two tags (4 bytes = one word each) before the ethertype
    uint32_t nv = 0, type = t0;
    if (t0 == 0x8100u || t0 == 0x88A8u) {
        const uint32_t t1 = rec_be16<16>(w);
        nv = 1; type = t1;
        if (t1 == 0x8100u || t1 == 0x88A8u) {
            const uint32_t t2 = rec_be16<20>(w);
            nv = 2; type = t2;
            if (t2 == 0x8100u || t2 == 0x88A8u) return PARSE_UNSUPPORTED;
        }
    }
    // shift the tags out: bytes 12.. move down by 4*nv (whole words from word 3 on)
    uint32_t ws[16];
#pragma unroll
    for (int i = 0; i < 16; i++) {
        const uint32_t a1 = (i >= 3 && i + 1 < 16) ? w[i + 1 < 16 ? i + 1 : 15] : w[i];
        const uint32_t a2 = (i >= 3 && i + 2 < 16) ? w[i + 2 < 16 ? i + 2 : 15] : w[i];
        ws[i] = nv == 0 ? w[i] : (nv == 1 ? a1 : a2);
    }
    return parse_l3(ws, type, wirelen, nv, tw);
}

// Branch-free fast path for the dominant record shape: untagged Ethernet II,
// IPv4 with IHL 5, not a fragment, TCP (>= 20 bytes) or UDP (no tunnel port).
// Returns true and fills tw exactly as parse_record would; false means "use
// parse_record" (tw is then garbage).  The host packer copies exactly the
// frames of this shape verbatim (gns_frame.cpp fast_shape).
__device__ __forceinline__ bool parse_fast_ipv4(const uint32_t (&w)[16], uint32_t wirelen, uint32_t (&tw)[10]) {
    constexpr int OFF = 14;
    const uint32_t type = rec_be16<12>(w);
    const uint32_t ihl = rec_byte<OFF>(w) & 15u;
    const uint32_t l2len = wirelen > 14u ? wirelen - 14u : 0u;
    uint32_t tot = rec_be16<OFF + 2>(w);
    tot = tot == 0 ? l2len : tot;
    const uint32_t proto = rec_byte<OFF + 9>(w);
    const uint32_t frag = rec_be16<OFF + 6>(w);
    const uint32_t avail = (tot < l2len ? tot : l2len) - 20u;  // wraps when < 20: rejected below
    const uint32_t sp = rec_be16<OFF + 20>(w), dp = rec_be16<OFF + 22>(w);
    const bool tcp = proto == 6u && avail >= 20u;
    const bool udp = proto == 17u && avail >= 8u && !udp_tunnel_port(sp) && !udp_tunnel_port(dp);
    const bool ok = type == 0x0800u && ihl == 5u && (frag & 0x3FFFu) == 0 && tot >= 20u && l2len >= 20u &&
                    (tcp || udp);
    tw[0] = rec_u32<OFF + 12>(w); tw[1] = 0; tw[2] = 0; tw[3] = 0;
    tw[4] = rec_u32<OFF + 16>(w); tw[5] = 0; tw[6] = 0; tw[7] = 0;
    set_ports(tw, sp, dp, proto);
    tw[9] |= 4u << 24 | 4u << 16;
    return ok;
}

// parse_record with the fast path first; the general decoder runs only when
// some active lane of the wave needs it.
__device__ __forceinline__ int parse_record_fast(const uint32_t (&w)[16], uint32_t wirelen, bool valid,
                                                 uint32_t (&tw)[10]) {
    const bool fast = parse_fast_ipv4(w, wirelen, tw);
    int st = PARSE_OK;
    if (__ballot(valid && !fast)) {
        if (valid && !fast) st = parse_record(w, wirelen, tw);
    }
    return st;
}

// byte idx (0..36) of the canonical tuple; 255 (or >= 40) -> 0
__device__ __forceinline__ uint32_t tuple_byte(const uint32_t (&tw)[10], uint32_t idx) {
    uint32_t w = 0;
#pragma unroll
    for (int i = 0; i < 10; i++) w = ((idx >> 2) == (uint32_t)i) ? tw[i] : w;
    return idx < 40u ? (w >> ((idx & 3u) * 8u)) & 0xFFu : 0u;
}

// mask of the bytes of word i that are < K
__device__ __forceinline__ uint32_t tail_mask(uint32_t K, int i) {
    const int rem = (int)K - 4 * i;
    return rem >= 4 ? 0xFFFFFFFFu : (rem <= 0 ? 0u : ((1u << (8 * rem)) - 1u));
}

}  // namespace gns
