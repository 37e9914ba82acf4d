"""Test-side generators: key streams, packet tuples and 64-byte frame records."""
from __future__ import annotations

import struct

import numpy as np


def assert_same_flows(got: dict, want: dict, what: str = "flows") -> None:
    """Dict-of-flows equality that names the first mismatches (a plain `==` inside a
    test makes pytest diff two large dicts, which can take minutes)."""
    if got == want:
        return
    missing = [k for k in want if k not in got]
    extra = [k for k in got if k not in want]
    diff = [k for k in want if k in got and got[k] != want[k]]
    msg = [f"{what}: {len(got)} got vs {len(want)} expected; {len(missing)} missing, {len(extra)} extra, "
           f"{len(diff)} differ"]
    for k in diff[:3]:
        msg.append(f"  {k!r}: got {got[k]!r} want {want[k]!r}")
    for k in missing[:3]:
        msg.append(f"  missing {k!r}: want {want[k]!r}")
    for k in extra[:3]:
        msg.append(f"  extra {k!r}: got {got[k]!r}")
    raise AssertionError("\n".join(msg))


def assert_same_list(got: list, want: list, what: str = "list") -> None:
    """List equality that reports the first differing position instead of a difflib dump."""
    if got == want:
        return
    for i, (a, b) in enumerate(zip(got, want)):
        if a != b:
            raise AssertionError(f"{what}: first difference at {i} of {len(got)}/{len(want)}: got {a!r} want {b!r}")
    raise AssertionError(f"{what}: lengths differ: got {len(got)} want {len(want)}")


def zipf_index(rng, n: int, nflows: int, s: float = 1.1) -> np.ndarray:
    p = np.arange(1, nflows + 1, dtype=np.float64) ** -s
    cdf = np.cumsum(p)
    cdf /= cdf[-1]
    return np.minimum(np.searchsorted(cdf, rng.random(n), side="right"), nflows - 1)


def zipf_keys(rng, n: int, nflows: int, K: int, s: float = 1.1):
    flows = rng.integers(0, 256, (nflows, max(K, 1)), dtype=np.uint8)[:, :K]
    idx = zipf_index(rng, n, nflows, s)
    return np.ascontiguousarray(flows[idx]), flows, idx


def sizes_u32(rng, n: int, big_frac: float = 0.0) -> np.ndarray:
    s = rng.integers(0, 1600, n, dtype=np.uint64)
    if big_frac > 0:
        big = rng.random(n) < big_frac
        s[big] = rng.integers(1 << 20, 1 << 32, int(big.sum()), dtype=np.uint64)
    return s.astype(np.uint32)


def random_tuples(rng, n: int, nflows: int, v6_frac: float = 0.0, s: float = 1.1):
    """Zipf packets over nflows random 5-tuples; returns SoA dict."""
    src = np.zeros((nflows, 16), np.uint8)
    dst = np.zeros((nflows, 16), np.uint8)
    v6 = rng.random(nflows) < v6_frac
    src[:, :4] = rng.integers(0, 256, (nflows, 4))
    dst[:, :4] = rng.integers(0, 256, (nflows, 4))
    src[v6] = rng.integers(0, 256, (int(v6.sum()), 16))
    dst[v6] = rng.integers(0, 256, (int(v6.sum()), 16))
    sport = rng.integers(0, 65536, nflows).astype(np.uint16)
    dport = rng.integers(0, 65536, nflows).astype(np.uint16)
    proto = np.where(rng.random(nflows) < 0.8, 6, 17).astype(np.uint8)
    idx = zipf_index(rng, n, nflows, s)
    length = rng.integers(64, 1519, n).astype(np.uint32)
    return dict(src16=src[idx], dst16=dst[idx], sport=sport[idx], dport=dport[idx], proto=proto[idx],
                length=length, v6=v6[idx])


def frame64(src16, dst16, sport, dport, proto, wirelen, v6=False, vlans=0, frag=0, doff=5, tot=None):
    """First 64 bytes of an Ethernet frame carrying the tuple."""
    b = bytearray(64)
    b[0:6] = b"\x00\x66\x77\x88\x99\xaa"
    b[6:12] = b"\x00\x11\x22\x33\x44\x55"
    off = 12
    for _ in range(vlans):
        b[off:off + 4] = b"\x81\x00\x00\x05"
        off += 4
    l2 = off + 2
    if not v6:
        b[off:off + 2] = b"\x08\x00"
        ip = l2
        total = (wirelen - l2) if tot is None else tot
        b[ip] = 0x45
        b[ip + 2:ip + 4] = struct.pack(">H", max(0, min(total, 0xFFFF)))
        b[ip + 6:ip + 8] = struct.pack(">H", frag)
        b[ip + 8] = 64
        b[ip + 9] = proto
        b[ip + 12:ip + 16] = bytes(src16[:4])
        b[ip + 16:ip + 20] = bytes(dst16[:4])
        l4 = ip + 20
    else:
        b[off:off + 2] = b"\x86\xdd"
        ip = l2
        b[ip] = 0x60
        plen = (wirelen - l2 - 40) if tot is None else tot
        b[ip + 4:ip + 6] = struct.pack(">H", max(0, min(plen, 0xFFFF)))
        b[ip + 6] = proto
        b[ip + 7] = 64
        b[ip + 8:ip + 24] = bytes(src16)
        b[ip + 24:ip + 40] = bytes(dst16)
        l4 = ip + 40
    for j, v in enumerate(struct.pack(">HH", int(sport), int(dport))):
        if l4 + j < 64:
            b[l4 + j] = v
    if proto == 6 and l4 + 12 < 64:
        b[l4 + 12] = (doff & 15) << 4
    return bytes(b)


def frames_from_tuples(t, rng=None, vlan_frac=0.0):
    n = len(t["length"])
    hdr = np.zeros((n, 64), np.uint8)
    for i in range(n):
        vl = 1 if (rng is not None and rng.random() < vlan_frac) else 0
        hdr[i] = np.frombuffer(frame64(t["src16"][i], t["dst16"][i], t["sport"][i], t["dport"][i],
                                       t["proto"][i], int(t["length"][i]), v6=bool(t["v6"][i]), vlans=vl),
                               np.uint8)
    return hdr


# ---------------------------------------------------------------------------
# Thrift PacketInfo messages (traffic.thrift) for the live-path tests: a third,
# pure-Python restatement of the decode (generated readers + lib/go Skip) and a
# generator of valid, reordered, padded and broken messages.
# ---------------------------------------------------------------------------
def py_thrift_decode(msg: bytes):
    """-> None if rejected, else (ts, src bytes, dst bytes, sport, dport, proto, length)."""
    class Bad(Exception):
        pass

    pos = [0]

    def take(k):
        if k < 0 or len(msg) - pos[0] < k:
            raise Bad()
        b = msg[pos[0]:pos[0] + k]
        pos[0] += k
        return b

    def i8():
        return take(1)[0]

    def i16():
        return struct.unpack(">H", take(2))[0]

    def i32():
        return struct.unpack(">i", take(4))[0]

    def i64():
        return struct.unpack(">q", take(8))[0]

    def binary():
        n = i32()
        if n < 0:
            raise Bad()
        return take(n)

    def skip(t, depth):
        if depth <= 0:
            raise Bad()
        if t in (2, 3):
            take(1)
        elif t == 6:
            take(2)
        elif t == 8:
            take(4)
        elif t in (4, 10):
            take(8)
        elif t == 16:
            take(16)
        elif t == 11:
            binary()
        elif t == 12:
            while True:
                ft = i8()
                if ft == 0:
                    return
                i16()
                skip(ft, depth - 1)
        elif t == 13:
            kt, vt, n = i8(), i8(), i32()
            if n < 0:
                raise Bad()
            for _ in range(n):
                skip(kt, depth - 1)
                skip(vt, depth - 1)
        elif t in (14, 15):
            et, n = i8(), i32()
            if n < 0:
                raise Bad()
            for _ in range(n):
                skip(et, depth - 1)
        else:
            raise Bad()

    def five_tuple():
        got, v = set(), {}
        while True:
            t = i8()
            if t == 0:
                break
            fid = i16()
            if fid in (1, 2) and t == 11:
                v[fid] = binary()
            elif fid in (3, 4, 5) and t == 8:
                v[fid] = i32()
            else:
                skip(t, 64)
                continue
            got.add(fid)
        if got != {1, 2, 3, 4, 5}:
            raise Bad()
        return v

    try:
        top, ft = {}, None
        while True:
            t = i8()
            if t == 0:
                break
            fid = i16()
            if fid in (1, 3) and t == 10:
                top[fid] = i64()
            elif fid == 2 and t == 12:
                ft = five_tuple()
                top[2] = True
            else:
                skip(t, 64)
        if set(top) != {1, 2, 3}:
            return None
        return (top[1], ft[1], ft[2], ft[3] & 0xFFFF, ft[4] & 0xFFFF, ft[5] & 0xFF, top[3])
    except Bad:
        return None


def _junk_value(rng, depth=0):
    """(wire type, encoded value) of a random skippable value."""
    t = int(rng.choice([2, 3, 4, 6, 8, 10, 11, 12, 13, 14, 15, 16]))
    if depth > 3 and t in (12, 13, 14, 15):
        t = 8
    if t in (2, 3):
        return t, bytes([int(rng.integers(0, 256))])
    if t == 6:
        return t, struct.pack(">h", int(rng.integers(-30000, 30000)))
    if t == 8:
        return t, struct.pack(">i", int(rng.integers(-2**31, 2**31)))
    if t in (4, 10):
        return t, bytes(rng.integers(0, 256, 8, dtype=np.uint8))
    if t == 16:
        return t, bytes(rng.integers(0, 256, 16, dtype=np.uint8))
    if t == 11:
        b = bytes(rng.integers(0, 256, int(rng.integers(0, 12)), dtype=np.uint8))
        return t, struct.pack(">i", len(b)) + b
    if t == 12:
        body = b""
        for _ in range(int(rng.integers(0, 3))):
            ft, fv = _junk_value(rng, depth + 1)
            body += bytes([ft]) + struct.pack(">h", int(rng.integers(1, 100))) + fv
        return t, body + b"\x00"
    if t == 13:
        n = int(rng.integers(0, 3))
        kt, _ = _junk_value(rng, depth + 1)
        vt, _ = _junk_value(rng, depth + 1)
        body = b""
        for _ in range(n):
            body += _junk_of(rng, kt, depth + 1) + _junk_of(rng, vt, depth + 1)
        return t, bytes([kt, vt]) + struct.pack(">i", n) + body
    n = int(rng.integers(0, 3))
    et, _ = _junk_value(rng, depth + 1)
    return t, bytes([et]) + struct.pack(">i", n) + b"".join(_junk_of(rng, et, depth + 1) for _ in range(n))


def _junk_of(rng, t, depth):
    for _ in range(100):
        tt, v = _junk_value(rng, depth)
        if tt == t:
            return v
    return {2: b"\x01", 3: b"\x01", 6: b"\x00\x01", 8: b"\x00" * 4, 4: b"\x00" * 8, 10: b"\x00" * 8,
            16: b"\x00" * 16, 11: b"\x00" * 4, 12: b"\x00", 13: b"\x08\x08\x00\x00\x00\x00",
            14: b"\x08\x00\x00\x00\x00", 15: b"\x08\x00\x00\x00\x00"}[t]


def thrift_messages(rng, n, nflows=500, bad_frac=0.1, v6_frac=0.3):
    """Valid PacketInfo messages (canonical, reordered, padded with unknown
    fields, duplicated fields, odd IP lengths) and broken ones (truncated,
    missing fields, wrong types, negative sizes, junk)."""
    from go2netspectra_amd.thrift import marshal_packet_info
    flows = []
    for _ in range(nflows):
        v6 = rng.random() < v6_frac
        ln = 16 if v6 else 4
        if rng.random() < 0.02:
            ln = int(rng.integers(0, 20))
        s = bytes(rng.integers(0, 256, ln, dtype=np.uint8))
        d = bytes(rng.integers(0, 256, 16 if v6 else 4, dtype=np.uint8))
        flows.append((s, d, int(rng.integers(-70000, 70000)), int(rng.integers(0, 65536)), int(rng.integers(0, 300))))
    msgs = []
    for i in range(n):
        s, d, sp, dp, pr = flows[int(zipf_index(rng, 1, nflows)[0])]
        ts = int(rng.integers(-2**62, 2**62))
        ln = int(rng.integers(0, 2**33)) if rng.random() < 0.05 else int(rng.integers(40, 1600))
        m = marshal_packet_info(ts, s, d, sp, dp, pr, ln)
        u = rng.random()
        if u < 0.15:  # reorder top-level fields and add unknown ones
            f1 = b"\x0a\x00\x01" + struct.pack(">q", ts)
            f3 = b"\x0a\x00\x03" + struct.pack(">q", ln)
            f2 = m[11:-(11 + 1)]
            parts = [f1, f2, f3]
            rng.shuffle(parts)
            jt, jv = _junk_value(rng)
            parts.insert(int(rng.integers(0, 4)), bytes([jt]) + struct.pack(">h", int(rng.integers(4, 50))) + jv)
            m = b"".join(parts) + b"\x00"
        elif u < 0.2:  # known id with the wrong type (skipped), then the real field
            jt, jv = _junk_value(rng)
            if jt != 10:
                m = bytes([jt]) + b"\x00\x01" + jv + m
        elif u < 0.23:  # trailing bytes after STOP are ignored
            m = m + bytes(rng.integers(0, 256, 5, dtype=np.uint8))
        if rng.random() < bad_frac:
            kind = int(rng.integers(0, 5))
            if kind == 0:
                m = m[: int(rng.integers(0, len(m)))]
            elif kind == 1:
                m = m[3 + 8:]  # drop the timestamp field
            elif kind == 2:
                m = b"\x0b\x00\x09" + struct.pack(">i", -1) + m  # negative binary size
            elif kind == 3:
                m = b"\x11\x00\x07" + m  # unknown wire type 17
            else:
                m = bytes(rng.integers(0, 256, int(rng.integers(1, 80)), dtype=np.uint8))
        msgs.append(m)
    return msgs


def pcapgen_records(rng, n: int):
    """scripts/pcapgen/main.go:17-97-shaped traffic as 64-byte records, vectorized:
    Ethernet / IPv4 (IHL 5) / TCP SYN with uniform random addresses and ports, so
    practically every packet is a new flow; frames of 104-1503 bytes (wire length)."""
    hdr = np.zeros((n, 64), np.uint8)
    hdr[:, 0:6] = np.frombuffer(b"\x00\x66\x77\x88\x99\xaa", np.uint8)
    hdr[:, 6:12] = np.frombuffer(b"\x00\x11\x22\x33\x44\x55", np.uint8)
    hdr[:, 12] = 0x08
    wl = rng.integers(104, 1504, n).astype(np.uint32)
    tot = wl - 14
    hdr[:, 14] = 0x45
    hdr[:, 16] = (tot >> 8).astype(np.uint8)
    hdr[:, 17] = (tot & 0xFF).astype(np.uint8)
    hdr[:, 22] = 64
    hdr[:, 23] = 6
    hdr[:, 26:38] = rng.integers(0, 256, (n, 12), dtype=np.uint8)  # src, dst, sport, dport
    hdr[:, 46] = 0x50  # data offset 5
    hdr[:, 47] = 0x02  # SYN
    return hdr, wl
