#!/usr/bin/env python3
"""Generate tests/golden/frame_vectors.json: whole captured frames and the
5-tuple the reference derives from each (gopacket v1.1.19 decode, reader.go:35-49,
then parser.go:37-61: first IPv4 layer else first IPv6 layer; ports of the
first TCP layer else the first UDP layer; no IP layer -> not counted).

The frames are built below; every expected tuple is WRITTEN OUT BY HAND from
reading the gopacket decoders (the "why" is in each case's note), not computed
by either restatement, so the fixture pins gns_frame.cpp (product) and
oracle/pyframe.py (checker) independently.  Parity with executed gopacket is
unpinned: no capture fixtures for these encapsulations exist in the reference.

Fields: frame (hex, the captured bytes), wirelen, then expect = null (no IP
layer) or {src, dst (hex, 4 or 16 bytes or "" for nil), sport, dport, proto,
ver}, and verbatim = whether gns_pack_pcap copies the frame as is.

Run from the repo root: python tests/golden/make_frame_vectors.py
"""
import json
import os
import struct

HERE = os.path.dirname(os.path.abspath(__file__))

MAC = bytes.fromhex("0066778899aa001122334455")
A4, B4 = bytes([10, 0, 0, 1]), bytes([10, 0, 0, 2])
C4, D4 = bytes([192, 168, 1, 1]), bytes([192, 168, 1, 2])
A6 = bytes.fromhex("20010db8000000000000000000000001")
B6 = bytes.fromhex("20010db8000000000000000000000002")
C6 = bytes.fromhex("fe800000000000000000000000000009")
D6 = bytes.fromhex("fe80000000000000000000000000000a")


def eth(etype, payload):
    return MAC + struct.pack(">H", etype) + payload


def vlan(etype, payload, tpid_next=None):
    return struct.pack(">HH", 5, etype) + payload


def ipv4(src, dst, proto, payload, opts=b"", frag=0, tot=None):
    ihl = 5 + len(opts) // 4
    total = 4 * ihl + len(payload) if tot is None else tot
    h = struct.pack(">BBHHHBBH", 0x40 | ihl, 0, total, 1, frag, 64, proto, 0) + src + dst + opts
    return h + payload


def ipv6(src, dst, nh, payload, plen=None):
    ln = len(payload) if plen is None else plen
    return struct.pack(">IHBB", 0x60000000, ln, nh, 64) + src + dst + payload


def tcp(sp, dp, data=b""):
    return struct.pack(">HHIIBBHHH", sp, dp, 1, 0, 0x50, 0x18, 512, 0, 0) + data


def udp(sp, dp, payload=b"", ln=None):
    return struct.pack(">HHHH", sp, dp, 8 + len(payload) if ln is None else ln, 0) + payload


def ext(nh, body):  # IPv6 extension header of 8*(1+k) bytes
    b = bytes([nh, (len(body) + 2) // 8 - 1]) + body
    assert len(b) % 8 == 0
    return b


def pad(b, n=60):  # Ethernet minimum frame (without FCS)
    return b + bytes(max(0, n - len(b)))


def tup(src, dst, sport, dport, proto, ver):
    return {"src": src.hex(), "dst": dst.hex(), "sport": sport, "dport": dport, "proto": proto, "ver": ver}


V = []


def case(name, frame, expect, verbatim=False, wirelen=None, note=""):
    V.append({"name": name, "frame": frame.hex(), "wirelen": len(frame) if wirelen is None else wirelen,
              "expect": expect, "verbatim": verbatim, "note": note})


inner_tcp4 = ipv4(C4, D4, 6, tcp(1111, 2222, b"x" * 8))
inner_udp4 = ipv4(C4, D4, 17, udp(3333, 4444, b"y" * 8))
inner_tcp6 = ipv6(C6, D6, 6, tcp(5555, 6666))

case("ipv4_tcp_plain", pad(eth(0x0800, ipv4(A4, B4, 6, tcp(40000, 443, b"z" * 20)))),
     tup(A4, B4, 40000, 443, 6, 4), verbatim=True, note="device fast-path shape")
case("ipv4_udp_plain", pad(eth(0x0800, ipv4(A4, B4, 17, udp(5000, 53, b"q" * 12)))),
     tup(A4, B4, 5000, 53, 17, 4), verbatim=True)
case("ipv4_icmp", pad(eth(0x0800, ipv4(A4, B4, 1, b"\x08\x00" + bytes(30)))), tup(A4, B4, 0, 0, 1, 4),
     note="ICMPv4 payload: no TCP/UDP layer, ports 0")
case("ipv4_options_tcp", pad(eth(0x0800, ipv4(A4, B4, 6, tcp(1234, 80), opts=b"\x01\x01\x01\x00"))),
     tup(A4, B4, 1234, 80, 6, 4), note="NOP NOP NOP EOL: options decode, TCP follows the 24-byte header")
case("ipv4_options_rr_tcp", pad(eth(0x0800, ipv4(A4, B4, 6, tcp(1234, 81), opts=b"\x07\x07\x04" + bytes(4) + b"\x00"))),
     tup(A4, B4, 1234, 81, 6, 4), note="record-route option length 7 then EOL")
case("ipv4_bad_option", pad(eth(0x0800, ipv4(A4, B4, 6, tcp(1234, 82), opts=b"\x44\x02\x00\x00"))),
     tup(A4, B4, 0, 0, 6, 4), note="option length 2 <= 2: decode error after the IPs; layer kept, no TCP")
case("ipv4_fragment_mf", pad(eth(0x0800, ipv4(A4, B4, 6, tcp(1, 2), frag=0x2000))), tup(A4, B4, 0, 0, 6, 4),
     note="MF set: LayerTypeFragment, no TCP layer")
case("ipv4_tso_len0", pad(eth(0x0800, ipv4(A4, B4, 6, tcp(7, 8, b"p" * 20), tot=0))), tup(A4, B4, 7, 8, 6, 4),
     verbatim=True, note="total length 0: TSO, length = data length")
case("ipv4_short_header", eth(0x0800, bytes([0x45]) + bytes(9)), tup(b"", b"", 0, 0, 0, 0),
     note="IPv4 data < 20 bytes: layer added with nil IPs and protocol 0")
case("ipv4_in_ipv4", pad(eth(0x0800, ipv4(A4, B4, 4, inner_tcp4))), tup(A4, B4, 1111, 2222, 4, 4),
     note="first IPv4 = outer; ports of the inner TCP")
case("ipv6_in_ipv4", eth(0x0800, ipv4(A4, B4, 41, inner_tcp6)), tup(A4, B4, 5555, 6666, 41, 4),
     note="6in4: first IPv4 = outer")
case("vlan3_ipv4_udp", pad(eth(0x8100, vlan(0x8100, vlan(0x88A8, vlan(0x0800, inner_udp4))))),
     tup(C4, D4, 3333, 4444, 17, 4), note="three tags: Dot1Q decodes any depth")
case("qinq_ipv6_tcp", eth(0x88A8, vlan(0x8100, vlan(0x86DD, ipv6(A6, B6, 6, tcp(443, 50000))))),
     tup(A6, B6, 443, 50000, 6, 6), note="IPv6 ports at bytes 62..65, past the 64-byte record")
case("ipv6_tcp_plain", eth(0x86DD, ipv6(A6, B6, 6, tcp(22, 60000))), tup(A6, B6, 22, 60000, 6, 6))
hbh_pad = ext(6, b"\x01\x04" + bytes(4))
case("ipv6_hbh_tcp", eth(0x86DD, ipv6(A6, B6, 0, hbh_pad + tcp(1000, 2000))), tup(A6, B6, 1000, 2000, 0, 6),
     note="hop-by-hop with PadN; Protocol = first NextHeader (0)")
hbh_jumbo = ext(6, b"\xc2\x04" + struct.pack(">I", 70000))
case("ipv6_hbh_jumbo", eth(0x86DD, ipv6(A6, B6, 0, hbh_jumbo + tcp(1001, 2001), plen=0)),
     tup(A6, B6, 1001, 2001, 0, 6), note="jumbogram option (70000 > 65535) with payload length 0")
case("ipv6_hbh_len0_nojumbo", eth(0x86DD, ipv6(A6, B6, 0, hbh_pad + tcp(1002, 2002), plen=0)),
     tup(A6, B6, 0, 0, 0, 6), note="length 0 without jumbogram: error after the IPs, no TCP")
case("ipv6_hbh_small_jumbo", eth(0x86DD, ipv6(A6, B6, 0, ext(6, b"\xc2\x04" + struct.pack(">I", 1000)) +
                                              tcp(1003, 2003), plen=0)),
     tup(A6, B6, 0, 0, 0, 6), note="jumbo length <= 65535: error, layer kept")
case("ipv6_hbh_truncated", eth(0x86DD, ipv6(A6, B6, 0, bytes([6, 1, 1, 0]), plen=4)), tup(A6, B6, 0, 0, 0, 6),
     note="extension base error (16-byte header, 4 bytes): IPv6 layer kept")
case("ipv6_hbh_option_overrun", eth(0x86DD, ipv6(A6, B6, 0, bytes([6, 0, 0x05, 0x09, 0, 0, 0, 0]) + tcp(1, 2))),
     None, note="TLV option runs past the header: panic inside DecodeFromBytes, no IPv6 layer -> not IP")
rt0 = ext(17, bytes([0, 1]) + bytes(4) + C6)
case("ipv6_routing0_udp", eth(0x86DD, ipv6(A6, B6, 43, rt0 + udp(7000, 8000, b"u" * 4))),
     tup(A6, B6, 7000, 8000, 43, 6), note="type-0 routing header, one address")
rt4 = ext(6, bytes([4, 1]) + bytes(4) + C6)
case("ipv6_routing4_tcp", eth(0x86DD, ipv6(A6, B6, 43, rt4 + tcp(1, 2))), tup(A6, B6, 0, 0, 43, 6),
     note="routing type 4 (SRH): 'Unknown IPv6 routing header type', no TCP")
case("ipv6_dest_frag_tcp", eth(0x86DD, ipv6(A6, B6, 60, ext(44, b"\x01\x04" + bytes(4)) +
                                             bytes([6, 0, 0, 0, 0, 0, 0, 1]) + tcp(3, 4))),
     tup(A6, B6, 0, 0, 60, 6), note="destination options then fragment header: DecodeFragment, no TCP")
ah = bytes([6, 4, 0, 0]) + struct.pack(">II", 0x100, 1) + bytes(12)
case("ipv6_ah_tcp", eth(0x86DD, ipv6(A6, B6, 51, ah + tcp(9000, 9001))), tup(A6, B6, 9000, 9001, 51, 6),
     note="AH length (4+2)*4 = 24")
case("ipv6_short_header", eth(0x86DD, bytes([0x60]) + bytes(20)), tup(b"", b"", 0, 0, 0, 0),
     note="IPv6 data < 40: nil IPs, NextHeader 0")
case("gre_ipv4", pad(eth(0x0800, ipv4(A4, B4, 47, b"\x00\x00\x08\x00" + inner_tcp4))),
     tup(A4, B4, 1111, 2222, 47, 4), note="GRE -> inner IPv4/TCP; IPs of the outer IPv4")
case("gre_key_seq_ipv6", eth(0x0800, ipv4(A4, B4, 47, b"\x30\x00\x86\xdd" + bytes(8) +
                                           ipv6(C6, D6, 17, udp(1200, 1300, b"v" * 4)))),
     tup(A4, B4, 1200, 1300, 47, 4), note="key and sequence present")
case("gre_teb_ethernet", eth(0x0800, ipv4(A4, B4, 47, b"\x00\x00\x65\x58" + eth(0x0800, inner_tcp4))),
     tup(A4, B4, 1111, 2222, 47, 4), note="transparent Ethernet bridging")
case("gre_routing", eth(0x0800, ipv4(A4, B4, 47, b"\x40\x00\x08\x00" + bytes(4) + b"\x08\x00\x00\x04" +
                                      bytes(4) + bytes(4) + inner_tcp4)),
     tup(A4, B4, 1111, 2222, 47, 4), note="routing present: checksum/offset, one SRE of 4 bytes, null SRE")
vx = b"\x08\x00\x00\x00\x00\x00\x2a\x00"
case("vxlan_tcp", eth(0x0800, ipv4(A4, B4, 17, udp(49152, 4789, vx + eth(0x0800, inner_tcp4)))),
     tup(A4, B4, 1111, 2222, 17, 4), note="first TCP is the inner one")
case("vxlan_udp", eth(0x0800, ipv4(A4, B4, 17, udp(49152, 4789, vx + eth(0x0800, inner_udp4)))),
     tup(A4, B4, 49152, 4789, 17, 4), note="first UDP is the outer one")
case("vxlan_sport_dns_dport", eth(0x0800, ipv4(A4, B4, 17, udp(4789, 53, vx + eth(0x0800, inner_tcp4)))),
     tup(A4, B4, 4789, 53, 17, 4), note="destination port 53 is registered (DNS): VXLAN not tried")
gen = bytes([0x02, 0x00, 0x65, 0x58, 0, 0, 1, 0]) + b"\x01\x02\x03\x01" + bytes(4)
case("geneve_tcp", eth(0x0800, ipv4(A4, B4, 17, udp(50000, 6081, gen + eth(0x0800, inner_tcp4)))),
     tup(A4, B4, 1111, 2222, 17, 4), note="Geneve with one 8-byte option")
case("gtpu_tcp", eth(0x0800, ipv4(A4, B4, 17, udp(2152, 2152, b"\x30\xff" + struct.pack(">HI", len(inner_tcp4), 7) +
                                                    inner_tcp4))),
     tup(A4, B4, 1111, 2222, 17, 4), note="GTP-U without optional fields")
gtp_ext = b"\x34\xff" + struct.pack(">HI", 8 + len(inner_tcp6), 7) + b"\x00\x01\x00\x85" + b"\x01\x05\x00\x00"
case("gtpu_ext_ipv6", eth(0x0800, ipv4(A4, B4, 17, udp(2152, 2152, gtp_ext + inner_tcp6))),
     tup(A4, B4, 5555, 6666, 17, 4), note="extension flag: one 4-byte PDU session container, next type 0")
mpls = struct.pack(">I", (100 << 12) | 64) + struct.pack(">I", (200 << 12) | 0x100 | 64)
case("mpls2_ipv4", pad(eth(0x8847, mpls + inner_tcp4)), tup(C4, D4, 1111, 2222, 6, 4),
     note="two labels, bottom of stack guessed IPv4 (0x45)")
case("mpls_ipv6", eth(0x8847, struct.pack(">I", (300 << 12) | 0x100 | 64) + ipv6(A6, B6, 17, udp(53, 5353, b"d" * 4))),
     tup(A6, B6, 53, 5353, 17, 6), note="guessed IPv6 (0x6X)")
case("pppoe_ipv4", pad(eth(0x8864, bytes([0x11, 0x00, 0x00, 0x01]) + struct.pack(">H", 2 + len(inner_tcp4)) +
                           b"\x00\x21" + inner_tcp4)),
     tup(C4, D4, 1111, 2222, 6, 4), note="PPPoE session, PPP protocol 0x0021")
case("pppoe_ppp_compressed_ipv6", eth(0x8864, bytes([0x11, 0x00, 0x00, 0x01]) + struct.pack(">H", 1 + len(inner_tcp6)) +
                                      b"\x57" + inner_tcp6),
     tup(C6, D6, 5555, 6666, 6, 6), note="one-byte PPP protocol field (0x57)")
case("pppoe_discovery", pad(eth(0x8863, bytes([0x11, 0x09, 0, 0, 0, 4]) + b"\x01\x01\x00\x00")), None,
     note="PADI: no PPP payload, no IP layer")
case("llc_snap_ipv4", pad(eth(8 + len(inner_tcp4), b"\xaa\xaa\x03\x00\x00\x00\x08\x00" + inner_tcp4)),
     tup(C4, D4, 1111, 2222, 6, 4), note="802.3 length, LLC/SNAP with EtherType 0x0800")
case("etherip", eth(0x0800, ipv4(A4, B4, 97, b"\x30\x00" + eth(0x0800, inner_tcp4))),
     tup(A4, B4, 1111, 2222, 97, 4), note="EtherIP (97): 2-byte header, then Ethernet")
case("arp", pad(eth(0x0806, bytes.fromhex("0001080006040001") + MAC[6:] + A4 + bytes(6) + B4)), None,
     note="not an IP packet")
case("runt", MAC[:10], None, note="shorter than an Ethernet header")
full = pad(eth(0x0800, ipv4(A4, B4, 6, tcp(30000, 80, b"w" * 946))))
case("snapped_tcp", full[:40], tup(A4, B4, 0, 0, 6, 4), wirelen=len(full),
     note="caplen 40 of 1000: TCP data is 6 bytes < 20, ports 0 (the wire length would say otherwise)")
case("snapped_tcp_54", full[:54], tup(A4, B4, 30000, 80, 6, 4), wirelen=len(full), verbatim=True,
     note="snapped but the TCP header is captured: fast path")


if __name__ == "__main__":
    with open(os.path.join(HERE, "frame_vectors.json"), "w") as f:
        json.dump({"source": "tests/golden/make_frame_vectors.py (hand-derived, gopacket v1.1.19 + parser.go)",
                   "vectors": V}, f, indent=1)
        f.write("\n")
    print(len(V), "frame vectors")
