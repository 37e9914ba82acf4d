"""Test-side generators: key streams, packet tuples and 64-byte frame records."""
from __future__ import annotations

import struct

import numpy as np


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
