// gns_frame.cpp -- host decode of whole captured frames into 64-byte records.
//
// The device parses 64-byte records: Ethernet II, up to two 802.1Q/802.1ad
// tags, IPv4 (IHL 5) / IPv6 without extension headers, TCP/UDP (gns_device.cuh
// parse_record).  Go2NetSpectra decodes every captured frame with gopacket
// (pkg/pcap/reader.go:35-49) and parser.go:23-67 then takes
//   - the FIRST IPv4 layer anywhere in the frame, else the first IPv6 layer
//     (SrcIP, DstIP, Protocol / first NextHeader);
//   - the ports of the FIRST TCP layer, else of the first UDP layer, else 0;
//   - no IP layer at all: "not an IP packet", the packet is not counted.
// So for a tunnelled or option-carrying frame the tuple can come from layers
// far beyond the first 64 bytes.  The packer (gns_pcap.cpp) copies a frame
// verbatim when it has the device's fast-path shape (fast_shape below, the
// host twin of parse_fast_ipv4) and otherwise decodes it here, on the whole
// captured frame, and writes a pre-parsed 0x88B5 record (or a record the
// device drops, for a frame without an IP layer).
//
// decode_frame restates the gopacket v1.1.19 decoders the reference's frames
// reach (layers/ethernet.go, dot1q.go, llc.go, ip4.go, ip6.go, ip6 extension
// headers, ipsec.go (AH), gre.go, vxlan.go, geneve.go, gtp.go, mpls.go,
// pppoe.go, ppp.go, tcp.go, udp.go), with gopacket's own rules for failures:
//   - decodeIPv4 / decodeIPv6 / decodeTCP / decodeUDP add the layer before
//     they return a DecodeFromBytes error (fields set before the failing check
//     are kept), and decoding stops there;
//   - decoders that go through decodingLayerDecoder (Dot1Q, LLC, VXLAN, GRE,
//     ...) add nothing on error; slicing past the data panics, which gopacket
//     recovers as a decode failure: that layer is not added either;
//   - PacketBuilder.NextDecoder does nothing on an empty payload.
// Parity with executed gopacket is unpinned (the reference's pcap fixtures are
// not in the repository); tests/golden/frame_vectors.json holds the
// hand-derived cases and oracle/pyref.py an independent restatement.
#include <cstring>

#include "gns_common.hpp"

namespace {

inline uint16_t be16(const uint8_t *p) { return (uint16_t)(p[0] << 8 | p[1]); }
inline uint32_t be32(const uint8_t *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

enum Layer {
    L_STOP, L_ETH, L_DOT1Q, L_LLC, L_SNAP, L_IPV4, L_IPV6, L_HBH, L_V6ROUTE, L_V6DEST, L_V6FRAG, L_AH, L_TCP,
    L_UDP, L_GRE, L_VXLAN, L_GENEVE, L_GTPU, L_MPLS, L_PPPOE, L_PPP, L_ETHERIP
};

Layer ethertype_layer(uint16_t t) {  // EthernetType decoders (enums.go) on the way to an IP layer
    switch (t) {
    case 0x0800: return L_IPV4;
    case 0x86DD: return L_IPV6;
    case 0x8100: case 0x88A8: return L_DOT1Q;
    case 0x8847: case 0x8848: return L_MPLS;
    case 0x8863: case 0x8864: return L_PPPOE;
    case 0x880B: return L_PPP;
    case 0x6558: return L_ETH;  // transparent Ethernet bridging (GRE, Geneve)
    default: return L_STOP;     // ARP, LLDP, EAPOL, unknown types: no IP layer follows
    }
}

Layer ipproto_layer(uint8_t p) {  // IPProtocol decoders
    switch (p) {
    case 0: return L_HBH;
    case 4: return L_IPV4;
    case 6: return L_TCP;
    case 17: return L_UDP;
    case 41: return L_IPV6;
    case 43: return L_V6ROUTE;
    case 44: return L_V6FRAG;
    case 47: return L_GRE;
    case 51: return L_AH;
    case 60: return L_V6DEST;
    case 97: return L_ETHERIP;
    case 137: return L_MPLS;
    default: return L_STOP;  // ICMP, ESP, SCTP, UDPLite, ...: no IP / TCP / UDP layer follows
    }
}

// UDP.NextLayerType: the destination port's registered layer, else the
// source port's.  Registered ports of gopacket v1.1.19 (ports.go); only
// VXLAN, Geneve and GTP-U lead to further IP layers.
Layer udp_port_layer(uint16_t p, bool *registered) {
    switch (p) {
    case 4789: *registered = true; return L_VXLAN;
    case 6081: *registered = true; return L_GENEVE;
    case 2152: *registered = true; return L_GTPU;
    case 53: case 123: case 67: case 68: case 546: case 547: case 5060: case 6343: case 3784: case 623: case 1812:
        *registered = true;
        return L_STOP;
    default:
        *registered = false;
        return L_STOP;
    }
}

enum Tlv { TLV_OK, TLV_PANIC, TLV_BAD };

// IPv6 TLV options of a hop-by-hop / destination header of `actual` bytes.
// An option running past the header slices past the data: a recovered panic
// (the layer is not added).  getIPv6HopByHopJumboLength reads the FIRST
// jumbogram option: data length 4 and a value > 65535, else an error.
Tlv tlv_options(const uint8_t *d, uint32_t actual, bool *jumbo) {
    bool seen = false, bad = false;
    for (uint32_t o = 2; o < actual;) {
        if (d[o] == 0) { o += 1; continue; }  // Pad1
        if (o + 2 > actual) return TLV_PANIC;
        const uint32_t olen = d[o + 1], tot = olen + 2;
        if (o + tot > actual) return TLV_PANIC;
        if (d[o] == 0xC2 && !seen) {
            seen = true;
            if (olen != 4 || be32(d + o + 2) <= 65535u) bad = true;
        }
        o += tot;
    }
    *jumbo = seen && !bad;
    return bad ? TLV_BAD : TLV_OK;
}

}  // namespace

namespace gns {

struct FrameTuple {
    bool ip = false;  // an IPv4 or IPv6 layer exists
    uint8_t src[16] = {}, dst[16] = {};
    uint8_t ver = 0;  // net.IP length class of SrcIP/DstIP: 4, 6, 0 = nil
    uint8_t proto = 0;
    uint16_t sport = 0, dport = 0;
};

// [pos, end) is the data handed to the next decoder: the payload of the layer
// added last (packet.go NextDecoder), never longer than the enclosing one.
void decode_frame(const uint8_t *d, uint32_t caplen, FrameTuple *out) {
    *out = FrameTuple{};
    bool v4 = false, v6 = false, tcp = false, udp = false, v4nil = false, v6nil = false;
    uint8_t v4s[4] = {}, v4d[4] = {}, v4p = 0, v6s[16] = {}, v6d[16] = {}, v6p = 0;
    uint16_t tsp = 0, tdp = 0, usp = 0, udp_ = 0;
    uint32_t pos = 0, end = caplen;
    auto first_v6 = [&](const uint8_t *p) {
        if (v6) return;
        v6 = true;
        memcpy(v6s, p + 8, 16);
        memcpy(v6d, p + 24, 16);
        v6p = p[6];
    };
    // every decoder that names a next layer consumed >= 1 byte except a Geneve
    // header whose uint8 offset wrapped: bound the walk all the same
    Layer lt = L_ETH;
    for (uint32_t step = 0; lt != L_STOP && step < (1u << 20); step++) {
        if (pos >= end) break;  // NextDecoder on an empty payload does nothing
        const uint8_t *p = d + pos;
        const uint32_t n = end - pos;
        Layer next = L_STOP;
        switch (lt) {
        case L_ETH: {  // decodeEthernet: error before AddLayer
            if (n < 14) break;
            const uint16_t t = be16(p + 12);
            pos += 14;
            if (t < 0x0600) {  // 802.3 length: LLC, payload cut to Length
                if (end - pos > t) end = pos + t;
                next = L_LLC;
            } else {
                next = ethertype_layer(t);
            }
            break;
        }
        case L_DOT1Q:
            if (n < 4) break;
            next = ethertype_layer(be16(p + 2));
            pos += 4;
            break;
        case L_LLC: {
            if (n < 3) break;
            const uint8_t dsap = p[0] & 0xFE, ssap = p[1] & 0xFE, ctl = p[2];
            uint32_t h = 3;
            if ((ctl & 1) == 0 || (ctl & 3) == 1) {
                if (n < 4) break;
                h = 4;
            }
            pos += h;
            if (dsap == 0xAA && ssap == 0xAA) next = L_SNAP;
            break;
        }
        case L_SNAP:
            if (n < 5) break;  // data[5:] past the data: recovered panic
            next = ethertype_layer(be16(p + 3));
            pos += 5;
            break;
        case L_IPV4: {  // decodeIPv4: AddLayer before the error check
            if (n < 20) {
                if (!v4) { v4 = true; v4nil = true; }
                break;
            }
            const uint32_t ihl = p[0] & 15u;
            uint32_t tot = be16(p + 2);
            if (tot == 0) tot = (uint16_t)n;  // TSO: uint16(len(data))
            if (!v4) {
                v4 = true;
                memcpy(v4s, p + 12, 4);
                memcpy(v4d, p + 16, 4);
                v4p = p[9];
            }
            if (tot < 20 || ihl < 5 || ihl * 4 > tot) break;
            if (n > tot) end = pos + tot;
            else if (n < tot && ihl * 4 > n) break;  // "Not all IP header bytes available"
            bool bad = false;
            for (uint32_t o = 20; o < ihl * 4;) {  // options
                const uint8_t ot = p[o];
                if (ot == 0) break;  // end of options: the rest is padding
                if (ot == 1) { o++; continue; }
                if (ihl * 4 - o < 2) { bad = true; break; }
                const uint32_t ol = p[o + 1];
                if (ihl * 4 - o < ol || ol <= 2) { bad = true; break; }
                o += ol;
            }
            if (bad) break;
            const uint16_t ff = be16(p + 6);
            pos += ihl * 4;
            if ((ff & 0x2000) || (ff & 0x1FFF)) break;  // LayerTypeFragment
            next = ipproto_layer(p[9]);
            break;
        }
        case L_IPV6: {  // decodeIPv6: AddLayer (and HopByHop) before the error check
            if (n < 40) {
                if (!v6) { v6 = true; v6nil = true; }
                break;
            }
            const uint32_t plen = be16(p + 4);
            if (p[6] == 0) {  // hop-by-hop decoded as part of the IPv6 layer
                const uint8_t *h = p + 40;
                const uint32_t hn = n - 40;
                if (hn < 2 || hn < (uint32_t)h[1] * 8 + 8) { first_v6(p); break; }  // extension base error
                const uint32_t actual = (uint32_t)h[1] * 8 + 8;
                bool jumbo = false;
                const Tlv tv = tlv_options(h, actual, &jumbo);
                if (tv == TLV_PANIC) break;  // no IPv6 layer
                first_v6(p);
                if (tv == TLV_BAD || jumbo != (plen == 0)) break;
                // NextDecoder reads the payload of the HopByHop layer (added last):
                // the bytes after it, not cut to the IPv6 length
                pos += 40 + actual;
                next = ipproto_layer(h[0]);
                break;
            }
            first_v6(p);
            if (plen == 0) break;  // "IPv6 length 0, but next header is ..."
            if (n - 40 > plen) end = pos + 40 + plen;
            pos += 40;
            next = ipproto_layer(p[6]);
            break;
        }
        case L_HBH: case L_V6DEST: {
            if (n < 2 || n < (uint32_t)p[1] * 8 + 8) break;
            const uint32_t actual = (uint32_t)p[1] * 8 + 8;
            bool jumbo = false;
            if (tlv_options(p, actual, &jumbo) == TLV_PANIC) break;
            next = ipproto_layer(p[0]);
            pos += actual;
            break;
        }
        case L_V6ROUTE: {  // only source routing (type 0) decodes; other types err
            if (n < 2 || n < (uint32_t)p[1] * 8 + 8) break;
            const uint32_t actual = (uint32_t)p[1] * 8 + 8;
            if (p[2] != 0 || (actual - 8) % 16 != 0) break;
            next = ipproto_layer(p[0]);
            pos += actual;
            break;
        }
        case L_V6FRAG:  // then gopacket.DecodeFragment: no further layers
            break;
        case L_AH: {
            if (n < 12) break;
            const uint32_t actual = ((uint32_t)p[1] + 2) * 4;
            if (n < actual || actual < 12) break;  // truncated / data[12:8] panic
            next = ipproto_layer(p[0]);
            pos += actual;
            break;
        }
        case L_ETHERIP:
            if (n < 2) break;
            pos += 2;
            next = L_ETH;
            break;
        case L_TCP:  // decodeTCP: ports read once the 20-byte header is there
            if (!tcp) {
                tcp = true;
                if (n >= 20) { tsp = be16(p); tdp = be16(p + 2); }
            }
            break;  // application payload: no IP layers follow
        case L_UDP: {
            if (!udp) {
                udp = true;
                if (n >= 8) { usp = be16(p); udp_ = be16(p + 2); }
            }
            if (n < 8) break;
            const uint32_t ulen = be16(p + 4);
            if (ulen >= 1 && ulen < 8) break;  // "UDP packet too small"
            if (ulen >= 8 && n > ulen) end = pos + ulen;
            bool reg = false;
            next = udp_port_layer(be16(p + 2), &reg);
            if (!reg) next = udp_port_layer(be16(p), &reg);
            pos += 8;
            break;
        }
        case L_GRE: {
            if (n < 4) break;
            const uint8_t f0 = p[0], f1 = p[1];
            uint32_t o = 4;
            const bool cs = f0 & 0x80, rt = f0 & 0x40, key = f0 & 0x20, seq = f0 & 0x10, ack = f1 & 0x80;
            if (cs || rt) o += 4;
            if (key) o += 4;
            if (seq) o += 4;
            bool bad = o > n;
            if (!bad && rt) {
                for (;;) {  // source route entries up to the null entry
                    if (o + 4 > n) { bad = true; break; }
                    const uint16_t af = be16(p + o);
                    const uint8_t sl = p[o + 3];
                    if (o + 4 + sl > n) { bad = true; break; }
                    o += 4 + sl;
                    if (af == 0 && sl == 0) break;
                }
            }
            if (!bad && ack) { o += 4; bad = o > n; }
            if (bad) break;
            next = ethertype_layer(be16(p + 2));
            pos += o;
            break;
        }
        case L_VXLAN:
            if (n < 8) break;
            next = L_ETH;
            pos += 8;
            break;
        case L_GENEVE: {  // offsets are uint8 in geneve.go
            if (n < 7) break;
            const uint8_t olen = (uint8_t)((p[0] & 0x3Fu) * 4);
            if (n < (uint8_t)(8 + olen)) break;
            uint8_t off = 8;
            int32_t left = olen;
            bool bad = false;
            while (left > 0) {
                if (off > n) { bad = true; break; }  // data[offset:]: panic
                const uint32_t dn = n - off;
                if (dn < 4) { bad = true; break; }  // "option too short" / data[3]
                const uint8_t L = (uint8_t)((p[off + 3] & 0xFu) * 4 + 4);
                if (dn < L) { bad = true; break; }
                left -= L;
                off = (uint8_t)(off + L);
            }
            if (bad || off > n) break;
            next = ethertype_layer(be16(p + 2));
            pos += off;
            break;
        }
        case L_GTPU: {  // lengths are uint16 in gtp.go
            if (n < 8) break;
            const uint16_t n16 = (uint16_t)n;
            if (n16 < (uint16_t)(8 + be16(p + 2))) break;
            uint32_t c = 8;
            if (p[0] & 0x07) {  // sequence number, N-PDU or extension flag
                c = 12;
                if (n < 12) break;
                if (p[0] & 0x04) {
                    bool bad = false;
                    for (bool more = true; more;) {
                        if (c >= n) { bad = true; break; }  // data[cIndex]: panic
                        const uint32_t len4 = p[c];
                        if (len4 == 0) { bad = true; break; }
                        const uint16_t l = (uint16_t)(c + len4 * 4);
                        if (n16 < l) { bad = true; break; }
                        if (l < c + 4) { bad = true; break; }  // wrapped (frames over 64 KiB): a panic
                        c = l;
                        more = p[c - 1] != 0;
                    }
                    if (bad) break;
                }
            }
            if (c > n) break;
            pos += c;
            if (pos >= end) break;
            const uint8_t vn = d[pos] >> 4;
            next = vn == 4 ? L_IPV4 : (vn == 6 ? L_IPV6 : L_PPP);
            break;
        }
        case L_MPLS: {
            if (n < 4) break;
            const bool bottom = p[2] & 0x01;
            pos += 4;
            if (!bottom) { next = L_MPLS; break; }
            if (pos >= end) break;
            const uint8_t b = d[pos];  // ProtocolGuessingDecoder
            if (b >= 0x45 && b <= 0x4F) next = L_IPV4;
            else if ((b >> 4) == 6) next = L_IPV6;
            break;
        }
        case L_PPPOE: {
            if (n < 6) break;
            // data[6:6+Length] is bounded by the slice's capacity -- the end of the
            // captured frame (gopacket copies each frame into a buffer of its
            // length) -- not by the enclosing layer, and the sum is a uint16
            const uint32_t len = be16(p + 4);
            if (6 + len > caplen - pos || 6 + len > 0xFFFFu) break;
            end = pos + 6 + len;
            pos += 6;
            if (p[1] == 0x00) next = L_PPP;  // session data
            break;
        }
        case L_PPP: {
            uint32_t o = 0;
            if (p[0] == 0xFF) {
                if (n < 2) break;
                if (p[1] == 0x03) o = 2;
            }
            if (o >= n) break;
            uint16_t type;
            if ((p[o] & 1) == 0) {
                if (o + 1 >= n) break;
                if ((p[o + 1] & 1) == 0) break;  // "PPP has invalid type"
                type = be16(p + o);
                o += 2;
            } else {
                type = p[o];
                o += 1;
            }
            pos += o;
            if (type == 0x0021) next = L_IPV4;
            else if (type == 0x0057) next = L_IPV6;
            else if (type == 0x0281 || type == 0x0283) next = L_MPLS;
            break;
        }
        default:
            break;
        }
        lt = next;
    }
    if (v4) {
        out->ip = true;
        out->ver = v4nil ? 0 : 4;
        if (!v4nil) { memcpy(out->src, v4s, 4); memcpy(out->dst, v4d, 4); }
        out->proto = v4p;
    } else if (v6) {
        out->ip = true;
        out->ver = v6nil ? 0 : 6;
        if (!v6nil) { memcpy(out->src, v6s, 16); memcpy(out->dst, v6d, 16); }
        out->proto = v6p;
    }
    if (tcp) { out->sport = tsp; out->dport = tdp; }
    else if (udp) { out->sport = usp; out->dport = udp_; }
}

namespace {

bool tunnel_port(uint16_t x) { return x == 4789 || x == 6081 || x == 2152; }

// IPv4 (IHL 5, not a fragment) carrying TCP with >= 20 or UDP with >= 8 bytes
// and no tunnel port, judged on `len` bytes after the Ethernet header (a zero
// IPv4 length is uint16(len) in gopacket, len on the device)
bool fast_ipv4(const uint8_t *d, uint32_t len, bool gopacket) {
    if (len < 20) return false;
    const uint8_t *ip = d + 14;
    uint32_t tot = be16(ip + 2);
    if (tot == 0) tot = gopacket ? (uint16_t)len : len;
    if ((ip[0] & 15u) != 5 || (be16(ip + 6) & 0x3FFF) || tot < 20) return false;
    const uint32_t avail = (tot < len ? tot : len) - 20;
    if (ip[9] == 6) return avail >= 20;
    if (ip[9] == 17) return avail >= 8 && !tunnel_port(be16(ip + 20)) && !tunnel_port(be16(ip + 22));
    return false;
}

}  // namespace

// A frame is copied verbatim when the device's fast path (parse_fast_ipv4,
// which sizes the frame by its wire length) takes it AND gopacket, which sizes
// it by the captured length, reaches the same IPv4 + TCP/UDP layers: then both
// read the tuple from the same bytes (< 38, all captured).
bool fast_shape(const uint8_t *d, uint32_t caplen, uint32_t wirelen) {
    if (caplen < 42 || be16(d + 12) != 0x0800) return false;
    return fast_ipv4(d, wirelen > 14 ? wirelen - 14 : 0, false) && fast_ipv4(d, caplen - 14, true);
}

// 0x88B5 pre-parsed record (the contract of gns_device.cuh parse_record), or a
// record the device drops (ARP ethertype) for a frame without an IP layer.
void write_record(const FrameTuple &t, uint8_t *r) {
    memset(r, 0, 64);
    if (!t.ip) {
        r[12] = 0x08; r[13] = 0x06;
        return;
    }
    r[12] = 0x88; r[13] = 0xB5;
    r[14] = 1;
    r[15] = t.ver;
    memcpy(r + 16, t.src, 16);
    memcpy(r + 32, t.dst, 16);
    r[48] = t.sport >> 8; r[49] = t.sport & 0xFF;
    r[50] = t.dport >> 8; r[51] = t.dport & 0xFF;
    r[52] = t.proto;
    r[53] = t.ver;
}

// verbatim (0), escaped (1), dropped (2)
int frame_record(const uint8_t *frame, uint32_t caplen, uint32_t wirelen, uint8_t *rec) {
    if (fast_shape(frame, caplen, wirelen)) {
        const uint32_t c = caplen < 64 ? caplen : 64;
        memcpy(rec, frame, c);
        if (c < 64) memset(rec + c, 0, 64 - c);
        return 0;
    }
    FrameTuple t;
    decode_frame(frame, caplen, &t);
    write_record(t, rec);
    return t.ip ? 1 : 2;
}

}  // namespace gns

extern "C" int gns_frame_record(const uint8_t *frame, uint32_t caplen, uint32_t wirelen, uint8_t *rec64) {
    if (!frame || !rec64) { gns::set_error("null argument"); return GNS_E_ARG; }
    return gns::frame_record(frame, caplen, wirelen, rec64);
}

// Compact host record (IN_REC16, gns_keys.cuh) of a record frame_record wrote
// (code = its return value): the IPv4 tuple exactly as the device parser reads
// it from that record -- a verbatim frame has the fast-path shape, so the tuple
// sits at fixed offsets (parse_fast_ipv4); a 0x88B5 record carries it as
// fields (parse_record) -- or the drop class, or kRecSide when the tuple does
// not fit (IPv6 addresses): the caller then appends the 64-byte record to the
// side array and stores its index in word 0.
namespace gns {
int compact_record(int code, const uint8_t *rec, uint8_t *out16) {
    memset(out16, 0, 16);
    if (code == 0) {
        memcpy(out16, rec + 26, 4);      // IPv4 source (left-aligned slot)
        memcpy(out16 + 4, rec + 30, 4);  // destination
        memcpy(out16 + 8, rec + 34, 4);  // ports, big-endian bytes
        out16[12] = rec[23];
        out16[14] = 4;
        out16[15] = 4;
        return gns::kRecTuple;
    }
    if (code == 2) {
        out16[13] = gns::kRecDrop;
        return gns::kRecDrop;
    }
    bool narrow = rec[14] == 1;
    for (int i = 4; i < 16 && narrow; i++) narrow = rec[16 + i] == 0 && rec[32 + i] == 0;
    if (!narrow) {
        out16[13] = gns::kRecSide;
        return gns::kRecSide;
    }
    memcpy(out16, rec + 16, 4);
    memcpy(out16 + 4, rec + 32, 4);
    memcpy(out16 + 8, rec + 48, 4);
    out16[12] = rec[52];
    out16[15] = rec[15];
    out16[14] = rec[53] ? rec[53] : rec[15];
    return gns::kRecTuple;
}

int compact_record16(int code, const uint8_t *rec, uint32_t orig, uint8_t *out16) {
    if (orig > 0xFFFFu) return -1;
    int cls = compact_record(code, rec, out16);
    if (cls == gns::kRecTuple && (out16[14] != 4 || out16[15] != 4)) {  // only IPv4 tuples stay compact
        memset(out16, 0, 16);
        out16[13] = gns::kRecSide;
        cls = gns::kRecSide;
    }
    out16[14] = (uint8_t)(orig & 0xFFu);  // word 3 bits 16..31: the wire length
    out16[15] = (uint8_t)(orig >> 8);
    return cls;
}
}  // namespace gns
