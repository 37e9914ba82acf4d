"""Whole-frame decode as gopacket v1.1.19 + parser.go do it (TEST INFRASTRUCTURE).

Independent restatement (shares no code with go2netspectra_amd/csrc/gns_frame.cpp)
of the decode chain the reference runs on every captured frame:

  pkg/pcap/reader.go:35-49        gopacket.NewPacketSource(handle, LinkTypeEthernet)
  internal/protocol/parser.go:37-61  first IPv4 layer else first IPv6 layer
                                  (SrcIP, DstIP, Protocol / NextHeader); ports of the
                                  first TCP layer else the first UDP layer; no IP
                                  layer -> "not an IP packet" (not counted)

gopacket is a go.mod dependency (github.com/google/gopacket v1.1.19) absent from
/root/reference; its decoders are restated from the published v1.1.19 sources
(layers/ethernet.go, dot1q.go, llc.go, ip4.go, ip6.go, ipsec.go, gre.go,
vxlan.go, geneve.go, gtp.go, mpls.go, pppoe.go, ppp.go, etherip.go, tcp.go,
udp.go, ports.go, enums.go; packet.go NextDecoder / decodingLayerDecoder).
Failure rules that decide what parser.go sees:
  * decodeIPv4 / decodeIPv6 / decodeTCP / decodeUDP add the layer, then return
    the DecodeFromBytes error: fields set before the failing check stay;
  * decoders built on decodingLayerDecoder add nothing on error;
  * a slice or index past the data panics; gopacket recovers it as a decode
    failure of that layer, which is then not added;
  * NextDecoder feeds the payload of the layer added LAST and does nothing when
    that payload is empty.
Parity with executed gopacket is UNPINNED (no reference pcap fixtures exist in
the repository); tests/golden/frame_vectors.json pins both restatements to
hand-derived frames.

Only tests/ may import this module.
"""
from __future__ import annotations

import struct


class _Panic(Exception):
    """A Go slice / index out of range inside a decoder."""


def _b(data: bytes, i: int) -> int:
    if i >= len(data):
        raise _Panic
    return data[i]


def _u16(data: bytes, i: int) -> int:
    if i + 2 > len(data):
        raise _Panic
    return struct.unpack_from(">H", data, i)[0]


def _u32(data: bytes, i: int) -> int:
    if i + 4 > len(data):
        raise _Panic
    return struct.unpack_from(">I", data, i)[0]


def _tail(data: bytes, i: int) -> bytes:  # data[i:]
    if i > len(data):
        raise _Panic
    return data[i:]


class Packet:
    def __init__(self):
        self.layers = []  # (name, dict)

    def add(self, name, **f):
        self.layers.append((name, f))

    def first(self, name):
        for n, f in self.layers:
            if n == name:
                return f
        return None


# ---- EthernetType / IPProtocol / UDPPort -> decoder (enums.go, ports.go) ----

def _ethertype(t):
    return {0x0800: dec_ipv4, 0x86DD: dec_ipv6, 0x8100: dec_dot1q, 0x88A8: dec_dot1q, 0x8847: dec_mpls,
            0x8848: dec_mpls, 0x8863: dec_pppoe, 0x8864: dec_pppoe, 0x880B: dec_ppp, 0x6558: dec_ethernet}.get(t)


def _ipproto(p):
    return {0: dec_hopbyhop, 4: dec_ipv4, 6: dec_tcp, 17: dec_udp, 41: dec_ipv6, 43: dec_v6routing,
            44: dec_v6fragment, 47: dec_gre, 51: dec_ah, 60: dec_v6destination, 97: dec_etherip,
            137: dec_mpls}.get(p)


_UDP_PORTS = {53: None, 123: None, 67: None, 68: None, 546: None, 547: None, 5060: None, 6343: None,
              3784: None, 623: None, 1812: None}


def _udp_port(p):
    """(registered, decoder)"""
    if p == 4789:
        return True, dec_vxlan
    if p == 6081:
        return True, dec_geneve
    if p == 2152:
        return True, dec_gtpu
    return p in _UDP_PORTS, None


# ---- decoders: dec(data, pk, cap) -> (a, b, next decoder) or None ----
# The payload handed on is data[a:b] (b may exceed len(data) up to cap, the
# bytes to the end of the frame: Go slices are bounded by capacity, and
# gopacket copies each captured frame into a buffer of exactly its length).

def dec_ethernet(data, pk, cap):
    if len(data) < 14:
        return None
    et = _u16(data, 12)
    pk.add("Ethernet")
    if et < 0x0600:  # 802.3 length field: LLC, payload cut to it
        return 14, min(len(data), 14 + et), dec_llc
    return 14, len(data), _ethertype(et)


def dec_dot1q(data, pk, cap):
    if len(data) < 4:
        return None
    pk.add("Dot1Q")
    return 4, len(data), _ethertype(_u16(data, 2))


def dec_llc(data, pk, cap):
    if len(data) < 3:
        return None
    dsap, ssap, ctl = data[0] & 0xFE, data[1] & 0xFE, data[2]
    h = 3
    if ctl & 1 == 0 or ctl & 3 == 1:
        if len(data) < 4:
            return None
        h = 4
    pk.add("LLC")
    return h, len(data), (dec_snap if dsap == 0xAA and ssap == 0xAA else None)


def dec_snap(data, pk, cap):
    t = _u16(data, 3)
    _tail(data, 5)
    pk.add("SNAP")
    return 5, len(data), _ethertype(t)


def dec_ipv4(data, pk, cap):
    if len(data) < 20:
        pk.add("IPv4", src=None, dst=None, proto=0)
        return None
    ihl = data[0] & 0x0F
    length = _u16(data, 2)
    flags_frag = _u16(data, 6)
    proto = data[9]
    pk.add("IPv4", src=bytes(data[12:16]), dst=bytes(data[16:20]), proto=proto)
    if length == 0:
        length = len(data) & 0xFFFF
    if length < 20 or ihl < 5 or ihl * 4 > length:
        return None
    if len(data) > length:
        data = data[:length]
    elif len(data) < length and ihl * 4 > len(data):
        return None
    opts = data[20:ihl * 4]
    while opts:
        t = opts[0]
        if t == 0:
            break
        if t == 1:
            opts = opts[1:]
            continue
        if len(opts) < 2:
            return None
        ol = opts[1]
        if len(opts) < ol or ol <= 2:
            return None
        opts = opts[ol:]
    if flags_frag & 0x2000 or flags_frag & 0x1FFF:
        return None  # LayerTypeFragment
    return ihl * 4, len(data), _ipproto(proto)


def _ext_base(data):
    """decodeIPv6ExtensionBase: (next header, actual length) or None on error"""
    if len(data) < 2:
        return None
    actual = data[1] * 8 + 8
    if len(data) < actual:
        return None
    return data[0], actual


def _tlv_opts(contents):
    """decodeIPv6HeaderTLVOption over contents[2:] -> [(type, data)]; panics past the data"""
    out = []
    d = contents[2:]
    while d:
        t = d[0]
        if t == 0:
            out.append((0, b""))
            d = d[1:]
            continue
        ol = _b(d, 1)
        out.append((t, d[2:ol + 2]))
        d = _tail(d, ol + 2)
    return out


def dec_ipv6(data, pk, cap):
    if len(data) < 40:
        pk.add("IPv6", src=None, dst=None, proto=0)
        return None
    length = _u16(data, 4)
    nh = data[6]
    fields = dict(src=bytes(data[8:24]), dst=bytes(data[24:40]), proto=nh)
    if nh == 0:  # hop-by-hop decoded with the IPv6 header
        base = _ext_base(data[40:])
        if base is None:
            pk.add("IPv6", **fields)
            return None
        hnext, actual = base
        opts = _tlv_opts(data[40:40 + actual])  # a panic here: no IPv6 layer
        pk.add("IPv6", **fields)
        pk.add("IPv6HopByHop")
        jumbo = next((od for t, od in opts if t == 0xC2), None)
        if jumbo is not None and (len(jumbo) != 4 or struct.unpack(">I", jumbo)[0] <= 65535):
            return None
        if (jumbo is not None) != (length == 0):
            return None
        # the layer added last is the HopByHop: its payload follows it, uncut
        return 40 + actual, len(data), _ipproto(hnext)
    pk.add("IPv6", **fields)
    if length == 0:
        return None
    return 40, min(len(data), 40 + length), _ipproto(nh)


def dec_hopbyhop(data, pk, cap):
    base = _ext_base(data)
    if base is None:
        return None
    nh, actual = base
    _tlv_opts(data[:actual])
    pk.add("IPv6HopByHop")
    return actual, len(data), _ipproto(nh)


dec_v6destination = dec_hopbyhop


def dec_v6routing(data, pk, cap):
    base = _ext_base(data)
    if base is None:
        return None
    nh, actual = base
    if data[2] != 0 or (actual - 8) % 16:  # only type 0 decodes
        return None
    pk.add("IPv6Routing")
    return actual, len(data), _ipproto(nh)


def dec_v6fragment(data, pk, cap):
    return None  # gopacket.DecodeFragment follows


def dec_ah(data, pk, cap):
    if len(data) < 12:
        return None
    actual = (data[1] + 2) * 4
    if len(data) < actual or actual < 12:
        return None
    pk.add("IPSecAH")
    return actual, len(data), _ipproto(data[0])


def dec_etherip(data, pk, cap):
    _tail(data, 2)
    pk.add("EtherIP")
    return 2, len(data), dec_ethernet


def dec_tcp(data, pk, cap):
    if len(data) < 20:
        pk.add("TCP", sport=0, dport=0)
    else:
        pk.add("TCP", sport=_u16(data, 0), dport=_u16(data, 2))
    return None


def dec_udp(data, pk, cap):
    if len(data) < 8:
        pk.add("UDP", sport=0, dport=0)
        return None
    sp, dp, ln = _u16(data, 0), _u16(data, 2), _u16(data, 4)
    pk.add("UDP", sport=sp, dport=dp)
    if 0 < ln < 8:
        return None
    reg, nxt = _udp_port(dp)
    if not reg:
        reg, nxt = _udp_port(sp)
    return 8, (min(ln, len(data)) if ln else len(data)), nxt


def dec_gre(data, pk, cap):
    f0, f1 = _b(data, 0), _b(data, 1)
    proto = _u16(data, 2)
    off = 4
    if f0 & 0xC0:
        off += 4
    if f0 & 0x20:
        off += 4
    if f0 & 0x10:
        off += 4
    if f0 & 0x40:
        while True:
            af, sl = _u16(data, off), _b(data, off + 3)
            off += 4 + sl
            if af == 0 and sl == 0:
                break
    if f1 & 0x80:
        off += 4
    _tail(data, off)
    pk.add("GRE")
    return off, len(data), _ethertype(proto)


def dec_vxlan(data, pk, cap):
    if len(data) < 8:
        return None
    pk.add("VXLAN")
    return 8, len(data), dec_ethernet


def dec_geneve(data, pk, cap):
    if len(data) < 7:
        return None
    olen = (data[0] & 0x3F) * 4
    if len(data) < (8 + olen) & 0xFF:  # uint8 offsets in geneve.go
        return None
    off, left = 8, olen
    while left > 0:
        d = _tail(data, off)
        if len(d) < 3:
            return None
        ln = ((_b(d, 3) & 0xF) * 4 + 4) & 0xFF
        if len(d) < ln:
            return None
        left -= ln
        off = (off + ln) & 0xFF
    _tail(data, off)
    pk.add("Geneve")
    return off, len(data), _ethertype(_u16(data, 2))


def dec_gtpu(data, pk, cap):
    n = len(data)
    if n < 8:
        return None
    if n & 0xFFFF < (8 + _u16(data, 2)) & 0xFFFF:  # uint16 lengths in gtp.go
        return None
    c = 8
    if data[0] & 0x07:  # sequence number, N-PDU or extension header flag
        c = 12
        if n < 12:
            return None
        if data[0] & 0x04:
            more = True
            while more:
                ln4 = _b(data, c)
                if ln4 == 0:
                    return None
                li = (c + ln4 * 4) & 0xFFFF
                if n & 0xFFFF < li:
                    return None
                if li < c + 4:  # wrapped (frames over 64 KiB): treated as a panic
                    raise _Panic
                c = li
                more = data[c - 1] != 0
    _tail(data, c)
    pk.add("GTPv1U")
    if c == n:
        return None
    v = data[c] >> 4
    return c, n, (dec_ipv4 if v == 4 else dec_ipv6 if v == 6 else dec_ppp)


def dec_mpls(data, pk, cap):
    _tail(data, 4)
    bottom = data[2] & 1
    pk.add("MPLS")
    return 4, len(data), (dec_mpls_payload if bottom else dec_mpls)


def dec_mpls_payload(data, pk, cap):  # ProtocolGuessingDecoder
    b = data[0]
    if 0x45 <= b <= 0x4F:
        return dec_ipv4(data, pk, cap)
    if b >> 4 == 6:
        return dec_ipv6(data, pk, cap)
    return None


def dec_pppoe(data, pk, cap):
    code = _b(data, 1)
    ln = _u16(data, 4)
    if 6 + ln > min(cap, 0xFFFF):  # data[6:6+Length]: bounded by capacity, uint16 sum
        raise _Panic
    pk.add("PPPoE")
    return 6, 6 + ln, (dec_ppp if code == 0 else None)


def dec_ppp(data, pk, cap):
    off = 0
    if _b(data, 0) == 0xFF and _b(data, 1) == 0x03:
        off = 2
    if _b(data, off) & 1 == 0:
        if _b(data, off + 1) & 1 == 0:
            return None  # "PPP has invalid type"
        t = _u16(data, off)
        off += 2
    else:
        t = data[off]
        off += 1
    pk.add("PPP")
    return off, len(data), {0x0021: dec_ipv4, 0x0057: dec_ipv6, 0x0281: dec_mpls, 0x0283: dec_mpls}.get(t)


def decode(frame: bytes) -> Packet:
    frame = bytes(frame)
    pk = Packet()
    start, end, dec = 0, len(frame), dec_ethernet
    while dec is not None and start < end:  # NextDecoder: nothing on an empty payload
        try:
            r = dec(frame[start:end], pk, len(frame) - start)
        except _Panic:
            break
        if r is None:
            break
        a, b, dec = r
        start, end = start + a, start + b
    return pk


def frame_tuple(frame: bytes):
    """parser.go:37-61 over decode(frame): None for "not an IP packet", else
    (src16, dst16, sport, dport, proto, ip_version) with ip_version 4 / 6 / 0 (nil)."""
    pk = decode(frame)
    ip = pk.first("IPv4")
    ver = 4
    if ip is None:
        ip, ver = pk.first("IPv6"), 6
    if ip is None:
        return None
    if ip["src"] is None:
        src = dst = bytes(16)
        ver = 0
    else:
        src = ip["src"] + bytes(16 - len(ip["src"]))
        dst = ip["dst"] + bytes(16 - len(ip["dst"]))
    l4 = pk.first("TCP") or pk.first("UDP")
    sp, dp = (l4["sport"], l4["dport"]) if l4 else (0, 0)
    return src, dst, sp, dp, ip["proto"], ver


def _fast_ipv4(frame: bytes, n: int, wrap16: bool) -> bool:
    if n < 20:
        return False
    ip = frame[14:]
    tot = struct.unpack_from(">H", ip, 2)[0] or ((n & 0xFFFF) if wrap16 else n)
    if ip[0] & 15 != 5 or struct.unpack_from(">H", ip, 6)[0] & 0x3FFF or tot < 20:
        return False
    avail = min(tot, n) - 20
    sp, dp = struct.unpack_from(">HH", ip, 20)
    if ip[9] == 6:
        return avail >= 20
    if ip[9] == 17:
        return avail >= 8 and sp not in (4789, 6081, 2152) and dp not in (4789, 6081, 2152)
    return False


def fast_shape(frame: bytes, wirelen: int) -> bool:
    """The frames gns_pack_pcap copies verbatim (the device fast path takes them)."""
    if len(frame) < 42 or frame[12:14] != b"\x08\x00":
        return False
    return _fast_ipv4(frame, max(wirelen - 14, 0), False) and _fast_ipv4(frame, len(frame) - 14, True)


def frame_record(frame: bytes, wirelen: int) -> bytes:
    """The 64-byte record gns_pack_pcap writes for a captured frame."""
    if fast_shape(frame, wirelen):
        return bytes(frame[:64]) + bytes(max(0, 64 - len(frame)))
    t = frame_tuple(frame)
    r = bytearray(64)
    if t is None:
        r[12:14] = b"\x08\x06"
        return bytes(r)
    src, dst, sp, dp, proto, ver = t
    r[12:16] = bytes([0x88, 0xB5, 1, ver])
    r[16:32], r[32:48] = src, dst
    r[48:53] = struct.pack(">HHB", sp, dp, proto)
    r[53] = ver
    return bytes(r)
