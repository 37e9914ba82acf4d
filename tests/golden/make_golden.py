#!/usr/bin/env python3
"""Generate the committed golden fixtures in tests/golden/.

  mm3_kat.json      public MurmurHash3_x86_32 known answers (SMHasher
                    verification value and published vectors) -- the external
                    pin of hash.go:13-53.
  cm_traces.json    hand-derived single-bucket traces of count_min.go:99-155
                    (w=1, d=1: every update hits the same bucket, so the
                    expected states follow from reading the Go code; they are
                    written out literally below, not computed).
  parse_vectors.json 64-byte frame records with the 5-tuple parser.go:23-67 +
                    gopacket would produce (written out literally).
  cm_stream.npz     4096-packet stream, w=256 d=3 K=16: full exported state and
                    heavy-hitter lists from the C oracle, cross-checked against
                    the independent pure-Python restatement (oracle/pyref.py)
                    before being written.
  ss_stream.npz     SuperSpread stream fixture (C oracle == Python restatement).

Run from the repo root: python tests/golden/make_golden.py
"""
import json
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle import oracle as orc  # noqa: E402
from oracle import pyref  # noqa: E402

MM3_KAT = [
    {"data": "", "seed": 0, "hash": 0x00000000},
    {"data": "", "seed": 1, "hash": 0x514E28B7},
    {"data": "", "seed": 0xFFFFFFFF, "hash": 0x81F16F39},
    {"data": "00000000", "seed": 0, "hash": 0x2362F9DE},
    {"data": "61616161", "seed": 0x9747B28C, "hash": 0x5A97808A},
    {"data": "48656c6c6f2c20776f726c6421", "seed": 0x9747B28C, "hash": 0x24884CBA},
    {"data": "54686520717569636b2062726f776e20666f78206a756d7073206f76657220746865206c617a7920646f67",
     "seed": 0x9747B28C, "hash": 0x2FA826CD},
]
SMHASHER_VERIFICATION = 0xB0F57EE3

# Hand-derived traces.  Keys are 4-byte strings; size in bytes.  After every
# update the expected bucket state (C, FPc, S, FPs) is listed, following
# count_min.go:99-155 line by line.
A, B, Cc = "aaaa", "bbbb", "cccc"
CM_TRACES = [
    {"name": "takeover_on_empty_then_majority",
     "updates": [[A, 100], [A, 50], [B, 30], [B, 200], [A, 10]],
     # 1: C==0 -> (a,1); S==0 -> (a,100)
     # 2: own -> C=2; own -> S=150
     # 3: b foreign: C=1 (F stays a); 30<=150 -> S=120 (F a)
     # 4: b foreign: C=0 -> F=b; 200>120 -> (b,200)
     # 5: a: C==0 -> (a,1); a foreign vs b: 10<=200 -> S=190 (F b)
     "states": [[1, A, 100, A], [2, A, 150, A], [1, A, 120, A], [0, B, 200, B], [1, A, 190, B]]},
    {"name": "size_subtract_to_zero_keeps_fp",
     "updates": [[A, 40], [B, 40], [Cc, 0], [B, 5]],
     # 1: (a,1) (a,40)
     # 2: b: C: 1-1=0 -> F=b; S: 40 not > 40 -> S=0, F stays a
     # 3: c: C==0 -> (c,1); S==0 -> (c,0)
     # 4: b: C: c!=b -> 0 -> F=b; S==0 -> (b,5)
     "states": [[1, A, 40, A], [0, B, 0, A], [1, Cc, 0, Cc], [0, B, 5, B]]},
    {"name": "size_wraps_u32",
     "updates": [[A, 0xFFFFFFF0], [A, 0x20], [B, 0x8], [B, 0x9]],
     # 1: (a,1) (a,0xFFFFFFF0)
     # 2: own: C=2; S=(0xFFFFFFF0+0x20) mod 2^32 = 0x10
     # 3: b: C=1; 8 <= 0x10 -> S=8 (F a)
     # 4: b: C=0 -> F=b; 9 > 8 -> (b,9)
     "states": [[1, A, 0xFFFFFFF0, A], [2, A, 0x10, A], [1, A, 0x8, A], [0, B, 0x9, B]]},
    {"name": "zero_size_on_empty_sets_fp",
     "updates": [[A, 0], [B, 0], [B, 0]],
     # 1: C (a,1); S==0 -> (a,0)
     # 2: b: C 1-1=0 -> F=b; S==0 -> (b,0)
     # 3: b: C==0 -> (b,1); S==0 -> (b,0)
     "states": [[1, A, 0, A], [0, B, 0, B], [1, B, 0, B]]},
]


def frame(*, src, dst, sport, dport, proto, v6=False, vlans=0, frag=0, ihl=5, ethertype=None, doff=5,
          total=None, wirelen=200):
    b = bytearray(64)
    b[0:12] = bytes.fromhex("006677889aaa001122334455")
    off = 12
    for _ in range(vlans):
        b[off:off + 4] = b"\x81\x00\x00\x07"
        off += 4
    et = ethertype if ethertype is not None else (0x86DD if v6 else 0x0800)
    b[off:off + 2] = struct.pack(">H", et)
    ip = off + 2
    if et == 0x0800:
        b[ip] = 0x40 | ihl
        tot = (wirelen - ip) if total is None else total
        b[ip + 2:ip + 4] = struct.pack(">H", tot)
        b[ip + 6:ip + 8] = struct.pack(">H", frag)
        b[ip + 9] = proto
        b[ip + 12:ip + 16] = bytes(src)
        b[ip + 16:ip + 20] = bytes(dst)
        l4 = ip + 4 * ihl
    elif et == 0x86DD:
        b[ip] = 0x60
        b[ip + 4:ip + 6] = struct.pack(">H", (wirelen - ip - 40) if total is None else total)
        b[ip + 6] = proto
        b[ip + 8:ip + 24] = bytes(src)
        b[ip + 24:ip + 40] = bytes(dst)
        l4 = ip + 40
    else:
        return bytes(b)
    for j, v in enumerate(struct.pack(">HH", sport, dport)):
        if l4 + j < 64:
            b[l4 + j] = v
    if proto == 6 and l4 + 12 < 64:
        b[l4 + 12] = doff << 4
    return bytes(b)


def slot(ip):
    return bytes(ip) + bytes(16 - len(ip))


V4S, V4D = bytes([10, 0, 0, 1]), bytes([192, 168, 7, 9])
V6S = bytes.fromhex("20010db8000000000000000000000001")
V6D = bytes.fromhex("20010db80000000000000000000000ff")
OK, DROP, UNSUP = 0, 1, 2
PARSE = [
    ("ipv4_tcp", frame(src=V4S, dst=V4D, sport=12345, dport=443, proto=6), 200, OK, V4S, V4D, 12345, 443, 6),
    ("ipv4_udp", frame(src=V4S, dst=V4D, sport=5353, dport=53, proto=17), 120, OK, V4S, V4D, 5353, 53, 17),
    ("ipv4_icmp_ports_zero", frame(src=V4S, dst=V4D, sport=0x0800, dport=0, proto=1), 98, OK, V4S, V4D, 0, 0, 1),
    ("vlan_ipv4_tcp", frame(src=V4S, dst=V4D, sport=1, dport=2, proto=6, vlans=1), 200, OK, V4S, V4D, 1, 2, 6),
    ("qinq_ipv4_udp", frame(src=V4S, dst=V4D, sport=7, dport=8, proto=17, vlans=2), 200, OK, V4S, V4D, 7, 8, 17),
    ("ipv4_fragment_ports_zero", frame(src=V4S, dst=V4D, sport=1, dport=2, proto=6, frag=0x2000), 200, OK,
     V4S, V4D, 0, 0, 6),
    # decodeTCP adds the layer with the ports it read before the data-offset check fails
    ("ipv4_tcp_bad_doff_ports_read", frame(src=V4S, dst=V4D, sport=1, dport=2, proto=6, doff=3), 200, OK,
     V4S, V4D, 1, 2, 6),
    ("ipv4_tcp_truncated_ports_zero", frame(src=V4S, dst=V4D, sport=1, dport=2, proto=6, total=30), 200, OK,
     V4S, V4D, 0, 0, 6),
    ("ipv6_tcp", frame(src=V6S, dst=V6D, sport=40000, dport=80, proto=6, v6=True), 200, OK, V6S, V6D, 40000, 80, 6),
    ("vlan_ipv6_udp", frame(src=V6S, dst=V6D, sport=9, dport=10, proto=17, v6=True, vlans=1), 200, OK,
     V6S, V6D, 9, 10, 17),
    ("qinq_ipv6_tcp_ports_outside_record", frame(src=V6S, dst=V6D, sport=9, dport=10, proto=6, v6=True, vlans=2),
     200, UNSUP, None, None, 0, 0, 0),
    ("ipv6_hop_by_hop_unsupported", frame(src=V6S, dst=V6D, sport=9, dport=10, proto=0, v6=True), 200, UNSUP,
     None, None, 0, 0, 0),
    ("ipv4_options_unsupported", frame(src=V4S, dst=V4D, sport=1, dport=2, proto=6, ihl=6), 200, UNSUP,
     None, None, 0, 0, 0),
    # decodeIPv4 adds the layer before returning "Invalid (too small) IP header length":
    # parser.go reads its IPs and protocol; no transport layer follows
    # (frame() writes the "ports" at IHL*4 = 16 bytes into the header: over DstIP)
    ("ipv4_bad_ihl_layer_kept", frame(src=V4S, dst=V4D, sport=1, dport=2, proto=6, ihl=4), 200, OK,
     V4S, bytes([0, 1, 0, 2]), 0, 0, 6),
    ("ipv4_total_below_20_layer_kept", frame(src=V4S, dst=V4D, sport=1, dport=2, proto=6, total=12), 200, OK,
     V4S, V4D, 0, 0, 6),
    # fewer than 20 bytes after Ethernet: "Invalid ip4 header" before any field is set (nil IPs)
    ("ipv4_short_data_nil_ips", frame(src=V4S, dst=V4D, sport=1, dport=2, proto=6), 30, OK,
     bytes(4), bytes(4), 0, 0, 0),
    ("ipv6_short_data_nil_ips", frame(src=V6S, dst=V6D, sport=1, dport=2, proto=6, v6=True), 40, OK,
     bytes(4), bytes(4), 0, 0, 0),
    ("ipv6_length_zero_layer_kept", frame(src=V6S, dst=V6D, sport=1, dport=2, proto=6, v6=True, total=0), 200, OK,
     V6S, V6D, 0, 0, 6),
    ("ipv6_fragment_header_ports_zero", frame(src=V6S, dst=V6D, sport=1, dport=2, proto=44, v6=True), 200, OK,
     V6S, V6D, 0, 0, 44),
    ("ipv6_no_decoder_ports_zero", frame(src=V6S, dst=V6D, sport=1, dport=2, proto=135, v6=True), 200, OK,
     V6S, V6D, 0, 0, 135),
    ("ipv4_gre_unsupported", frame(src=V4S, dst=V4D, sport=0, dport=0, proto=47), 200, UNSUP, None, None, 0, 0, 0),
    ("ipv4_proto0_hop_by_hop_unsupported", frame(src=V4S, dst=V4D, sport=0, dport=0, proto=0), 200, UNSUP,
     None, None, 0, 0, 0),
    ("vxlan_unsupported", frame(src=V4S, dst=V4D, sport=999, dport=4789, proto=17), 200, UNSUP, None, None, 0, 0, 0),
    ("ipip_unsupported", frame(src=V4S, dst=V4D, sport=0, dport=0, proto=4), 200, UNSUP, None, None, 0, 0, 0),
    ("arp_dropped", frame(src=V4S, dst=V4D, sport=0, dport=0, proto=0, ethertype=0x0806), 60, DROP,
     None, None, 0, 0, 0),
    ("mpls_unsupported", frame(src=V4S, dst=V4D, sport=0, dport=0, proto=0, ethertype=0x8847), 60, UNSUP,
     None, None, 0, 0, 0),
]


def preparsed():
    b = bytearray(64)
    b[12:14] = b"\x88\xb5"
    b[14] = 1
    b[15] = 4
    b[16:32] = slot(V4S)
    b[32:48] = slot(V4D)
    b[48:52] = struct.pack(">HH", 4444, 5555)
    b[52] = 6
    return bytes(b)


def main():
    # --- MM3 ---
    for kat in MM3_KAT:
        d = bytes.fromhex(kat["data"])
        assert orc.mm3(d, kat["seed"]) == kat["hash"] == pyref.mm3(d, kat["seed"]), kat
    json.dump({"vectors": [{**k, "hash": f"0x{k['hash']:08X}"} for k in MM3_KAT],
               "smhasher_verification": f"0x{SMHASHER_VERIFICATION:08X}",
               "source": "public MurmurHash3_x86_32 test vectors (SMHasher; aappleby/smhasher)"},
              open(os.path.join(HERE, "mm3_kat.json"), "w"), indent=1)
    # --- hand traces (checked against both restatements) ---
    for tr in CM_TRACES:
        c = orc.CountMin(1, 1, 1, 1, 4, np.array([7], np.uint32))
        p = pyref.CountMinSeq(1, 1, 1, 1, 4, [7])
        for (k, s), st in zip(tr["updates"], tr["states"]):
            kb = k.encode()
            c.insert_keys(np.frombuffer(kb, np.uint8).reshape(1, 4), np.array([s], np.uint32))
            p.insert(kb, s)
            C, S, Fc, Fs = c.export()
            got = [int(C[0]), bytes(Fc[0]).decode(), int(S[0]), bytes(Fs[0]).decode()]
            assert got == st, (tr["name"], got, st)
            assert [p.C[0], p.Fc[0].decode(), p.S[0], p.Fs[0].decode()] == st
    json.dump({"bucket": "w=1 d=1 key_bytes=4 (every update hits the same bucket)",
               "state_fields": ["C", "FPc", "S", "FPs"], "traces": CM_TRACES},
              open(os.path.join(HERE, "cm_traces.json"), "w"), indent=1)
    # --- parse vectors ---
    vecs = []
    for name, rec, wl, st, s, d, sp, dp, pr in PARSE + [("preparsed_escape", preparsed(), 300, OK, V4S, V4D,
                                                          4444, 5555, 6)]:
        got = orc.parse_hdr64(rec, wl)
        exp = (st, slot(s) if s else None, slot(d) if d else None, sp, dp, pr)
        if st == OK:
            assert got == exp, (name, got, exp)
        else:
            assert got[0] == st, (name, got)
        vecs.append({"name": name, "record": rec.hex(), "wirelen": wl, "status": st,
                     "src16": slot(s).hex() if s else None, "dst16": slot(d).hex() if d else None,
                     "sport": sp, "dport": dp, "proto": pr})
    json.dump({"status": {"0": "ok", "1": "dropped (not IP, parser.go:48-49)", "2": "outside fast-parse subset"},
               "vectors": vecs}, open(os.path.join(HERE, "parse_vectors.json"), "w"), indent=1)
    # --- stream fixture ---
    from helpers import sizes_u32, zipf_keys
    rng = np.random.default_rng(20260424)
    keys, _, _ = zipf_keys(rng, 4096, 300, 16)
    sizes = sizes_u32(rng, 4096)
    sizes[::97] = 0
    seeds = np.array([0x9747B28C, 0x12345678, 0xDEADBEEF], np.uint32)
    c = orc.CountMin(256, 3, 3000, 20, 16, seeds)
    c.insert_keys(keys, sizes)
    p = pyref.CountMinSeq(256, 3, 3000, 20, 16, seeds.tolist())
    for k, s in zip(keys, sizes):
        p.insert(bytes(k), int(s))
    C, S, Fc, Fs = c.export()
    assert C.tolist() == p.C and S.tolist() == p.S
    assert [bytes(x) for x in Fc] == p.Fc and [bytes(x) for x in Fs] == p.Fs
    hc, hs = c.heavy("count"), c.heavy("size")
    assert hc == p.heavy("count") and hs == p.heavy("size")
    np.savez_compressed(os.path.join(HERE, "cm_stream.npz"), keys=keys, sizes=sizes, seeds=seeds, C=C, S=S,
                        FPc=Fc, FPs=Fs, hh_count_flows=np.array([f for f, _ in hc], dtype="S16"),
                        hh_count=np.array([v for _, v in hc], np.uint32),
                        hh_size_flows=np.array([f for f, _ in hs], dtype="S16"),
                        hh_size=np.array([v for _, v in hs], np.uint32),
                        params=np.array([256, 3, 3000, 20, 16], np.uint32))
    # --- SuperSpread fixture ---
    rng = np.random.default_rng(7)
    flows = rng.integers(0, 256, (40, 16), dtype=np.uint8)
    fl = flows[rng.integers(0, 40, 3000) % np.maximum(1, rng.integers(1, 40, 3000))]
    el = rng.integers(0, 256, (3000, 16), dtype=np.uint8)
    sseeds = np.array([0x1111, 0x2222], np.uint32)
    ss = orc.SuperSpread(64, 2, 20, 32, 5, 0.5, 1.08, 16, 16, sseeds, 0xABCDEF, 0x13579)
    ss.insert(fl, el)
    ps = pyref.SuperSpreadSeq(64, 2, 20, 32, 5, 0.5, 1.08, 16, 16, sseeds.tolist(), 0xABCDEF, 0x13579)
    for f, e in zip(fl, el):
        ps.insert(bytes(f), bytes(e))
    values, skeys, regs, pbits = ss.export()
    assert values.tolist() == ps.values and [bytes(k) for k in skeys] == ps.keys
    assert regs.tolist() == ps.regs and pbits.tolist() == ps.pbits
    sh = ss.heavy()
    assert sh == ps.heavy()
    np.savez_compressed(os.path.join(HERE, "ss_stream.npz"), flows=fl, elems=el, seeds=sseeds, values=values,
                        keys=skeys, regs=regs, pbits=pbits, hh_flows=np.array([f for f, _ in sh], dtype="S16"),
                        hh=np.array([v for _, v in sh], np.uint32),
                        params=np.array([64, 2, 20, 32, 5, 16, 16], np.uint32),
                        fparams=np.array([0.5, 1.08]), seeds64=np.array([0xABCDEF, 0x13579], np.uint64))
    print("golden fixtures written")


if __name__ == "__main__":
    main()
