"""Pure-Python restatement of the reference sketch path (TEST INFRASTRUCTURE).

Independent of gns_oracle.c (written separately, shares no code) so that the
two restatements cross-check each other on small cases.  Citations are
/root/reference paths:

  hash.go:13-53            mm3()
  task.go:265-300,327-338  encode_key(), FIELD_SIZE
  count_min.go:47-265      CountMinSeq
  super_spread.go:24-311   SuperSpreadSeq (declared RNG, see gns_oracle.h)

Only tests/ (and bench.py's cpu_baseline leg via oracle.py) may import this.
"""
from __future__ import annotations

import math
import struct

M32 = 0xFFFFFFFF
M64 = 0xFFFFFFFFFFFFFFFF


def _rotl(x: int, r: int) -> int:
    return ((x << r) | (x >> (32 - r))) & M32


def mm3(data: bytes, seed: int) -> int:
    """MurmurHash3_x86_32, hash.go:13-53."""
    c1, c2 = 0xCC9E2D51, 0x1B873593
    h = seed & M32
    n = len(data) // 4
    for i in range(n):
        k = int.from_bytes(data[4 * i:4 * i + 4], "little")
        k = (k * c1) & M32
        k = _rotl(k, 15)
        k = (k * c2) & M32
        h ^= k
        h = _rotl(h, 13)
        h = (h * 5 + 0xE6546B64) & M32
    tail = data[4 * n:]
    k = 0
    if len(tail) == 3:
        k ^= tail[2] << 16
    if len(tail) >= 2:
        k ^= tail[1] << 8
    if len(tail) >= 1:
        k ^= tail[0]
        k = (k * c1) & M32
        k = _rotl(k, 15)
        k = (k * c2) & M32
        h ^= k
    h ^= len(data) & M32
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & M32
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & M32
    h ^= h >> 16
    return h


FIELD_SIZE = {"SrcIP": 16, "DstIP": 16, "SrcPort": 2, "DstPort": 2, "Protocol": 1}


def ip_slot(ip: bytes) -> bytes:
    """copy(buf[off:], ip) into a zeroed 16-byte slot (task.go:281-286)."""
    return bytes(ip[:16]) + bytes(16 - min(len(ip), 16))


def encode_key(fields, src: bytes, dst: bytes, sport: int, dport: int, proto: int) -> bytes:
    """EncodeFlow over the configured fields (task.go:265-300)."""
    out = b""
    for f in fields:
        if f == "SrcIP":
            out += ip_slot(src)
        elif f == "DstIP":
            out += ip_slot(dst)
        elif f == "SrcPort":
            out += struct.pack(">H", sport & 0xFFFF)
        elif f == "DstPort":
            out += struct.pack(">H", dport & 0xFFFF)
        elif f == "Protocol":
            out += bytes([proto & 0xFF])
    return out


class CountMinSeq:
    """count_min.go with injected seeds, one worker, stream order."""

    def __init__(self, width, depth, st, ct, key_bytes, seeds):
        self.w = width or (1 << 20)
        self.d = depth or 3
        self.st = st or 512 * 1024
        self.ct = ct or 512
        self.K = key_bytes
        self.seeds = list(seeds)[: self.d]
        n = self.d * self.w
        self.C = [0] * n
        self.S = [0] * n
        self.Fc = [bytes(self.K)] * n
        self.Fs = [bytes(self.K)] * n

    def insert(self, key: bytes, size: int) -> None:
        for i in range(self.d):
            c = i * self.w + mm3(key, self.seeds[i]) % self.w
            S = self.S[c]
            if S == 0:
                self.S[c], self.Fs[c] = size & M32, key
            elif self.Fs[c] == key:
                self.S[c] = (S + size) & M32
            elif size > S:
                self.S[c], self.Fs[c] = size & M32, key
            else:
                self.S[c] = S - size
            C = self.C[c]
            if C == 0:
                self.C[c], self.Fc[c] = 1, key
            elif self.Fc[c] == key:
                self.C[c] = (C + 1) & M32
            else:
                self.C[c] = C - 1
                if C - 1 == 0:
                    self.Fc[c] = key

    def query(self, key: bytes) -> int:
        sz = ct = 0
        for i in range(self.d):
            c = i * self.w + mm3(key, self.seeds[i]) % self.w
            if self.Fs[c] == key:
                sz = max(sz, self.S[c])
            if self.Fc[c] == key:
                ct = max(ct, self.C[c])
        return (ct << 32) | sz

    def heavy(self, which: str):
        vals, fps, thr = (self.C, self.Fc, self.ct) if which == "count" else (self.S, self.Fs, self.st)
        best = {}
        for v, f in zip(vals, fps):
            if v > 0:
                best[f] = max(best.get(f, 0), v)
        out = [(f, v) for f, v in best.items() if v >= thr]
        out.sort(key=lambda fv: (-fv[1], fv[0]))
        return out


def mix64(z: int) -> int:
    z &= M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def ss_uniform(rng_seed: int, pkt: int, row: int, draw: int) -> float:
    x = mix64(rng_seed + pkt * 0x9E3779B97F4A7C15)
    x = mix64(x ^ ((row << 32) | draw) ^ 0xD1B54A32D192ED03)
    return float(x >> 11) * 2.0 ** -53


def hll_seeds(master: int, cell: int):
    x = mix64(master + cell * 0x9E3779B97F4A7C15)
    return x & M32, x >> 32


def go_pow_int(x: float, y: float) -> float:
    """Go math.Pow for integer y, x > 0 (pow.go: Frexp, square-and-multiply, Ldexp)."""
    if y == 0 or x == 1:
        return 1.0
    if y == 1:
        return x
    yi = abs(y)
    a1, ae = 1.0, 0
    x1, xe = math.frexp(x)
    i = int(yi)
    while i != 0:
        if xe < -(1 << 12) or (1 << 12) < xe:
            ae += xe
            break
        if i & 1:
            a1 *= x1
            ae += xe
        x1 *= x1
        xe <<= 1
        if x1 < 0.5:
            x1 += x1
            xe -= 1
        i >>= 1
    if y < 0:
        a1 = 1 / a1
        ae = -ae
    try:
        return math.ldexp(a1, ae)  # single rounding, like Go's Ldexp (also for subnormals)
    except OverflowError:
        return math.inf


def det_log(x: float) -> float:
    """Deterministic log on (0, 1] (fdlibm reduction + polynomial, as Go's math.Log)."""
    Ln2Hi, Ln2Lo = 6.93147180369123816490e-01, 1.90821492927058770002e-10
    L1, L2, L3 = 6.666666666666735130e-01, 3.999999999940941908e-01, 2.857142874366239149e-01
    L4, L5, L6 = 2.222219843214978396e-01, 1.818357216161805012e-01, 1.531383769920937332e-01
    L7 = 1.479819860511658591e-01
    f1, ki = math.frexp(x)
    if f1 < 0.70710678118654752440:
        f1 *= 2
        ki -= 1
    f = f1 - 1
    k = float(ki)
    s = f / (2 + f)
    s2 = s * s
    s4 = s2 * s2
    t1 = s2 * (L1 + s4 * (L3 + s4 * (L5 + s4 * L7)))
    t2 = s4 * (L2 + s4 * (L4 + s4 * L6))
    R = t1 + t2
    hfsq = 0.5 * f * f
    return k * Ln2Hi - ((hfsq - (s * (hfsq + R) + k * Ln2Lo)) - f)


def det_log1m(p: float) -> float:
    if p < 1e-4:
        t = p * p
        r = p + t * 0.5
        r = r + t * p * (1.0 / 3.0)
        return -r
    return det_log(1.0 - p)


class SuperSpreadSeq:
    """super_spread.go with injected HLL seeds and the declared generator."""

    def __init__(self, width, depth, threshold, m, size, base, b, kf, ke, seeds, hll_master, rng_seed):
        self.w = width or (1 << 20)
        self.d = depth or 3
        self.thr = threshold or 4096
        self.m = m or 128
        self.size = size or 5
        self.base = base or 0.5
        self.b = b or 1.08
        self.maxv = (1 << self.size) - 1
        self.kf, self.ke = kf, ke
        self.seeds = list(seeds)[: self.d]
        self.hm, self.rs = hll_master, rng_seed
        n = self.d * self.w
        self.regs = [[0] * self.m for _ in range(n)]
        self.pbits = [1.0] * n
        self.values = [0] * n
        self.keys = [bytes(kf)] * n
        self.pkt = 0

    def _encode(self, cell, merged):
        s0, s1 = hll_seeds(self.hm, cell)
        h = mm3(merged, s0)
        lz = (32 - h.bit_length()) + 1
        lz = min(lz, self.maxv)
        idx = mm3(merged, s1) % self.m
        old = self.regs[cell][idx]
        if lz <= old:
            return -1.0
        self.regs[cell][idx] = lz
        res = self.pbits[cell]
        self.pbits[cell] = self.pbits[cell] + (-go_pow_int(self.base, float(old)) / float(self.m))
        if lz < self.maxv:
            self.pbits[cell] = self.pbits[cell] + go_pow_int(self.base, float(lz)) / float(self.m)
        return res

    def insert(self, flow: bytes, elem: bytes) -> None:
        merged = flow + elem
        pkt = self.pkt
        self.pkt += 1
        for i in range(self.d):
            cell = i * self.w + mm3(flow, self.seeds[i]) % self.w
            p = self._encode(cell, merged)
            if p == -1.0:
                continue
            inv = 1.0 / p if p != 0 else math.inf
            cv = math.ceil(inv) if math.isfinite(inv) else math.inf
            pcu = inv / cv if math.isfinite(inv) else math.nan
            if ss_uniform(self.rs, pkt, i, 0) >= pcu:
                continue
            vv = int(cv) if cv < 2.0 ** 63 else -(1 << 63)
            self._mv(cell, flow, vv, pkt, i)

    def _mv(self, cell, flow, vv, pkt, row):
        """super_spread.go:207-233; foreign decrements as geometric waiting times."""
        draw = 1
        while vv > 0:
            if self.values[cell] == 0 or self.keys[cell] == flow:
                if self.values[cell] == 0:
                    self.keys[cell] = flow
                self.values[cell] = (self.values[cell] + vv) & M32
                return
            ppp = go_pow_int(self.b, -float(self.values[cell]))
            if not ppp > 0:
                return
            if ppp >= 1:
                k = min(self.values[cell], vv)
                self.values[cell] -= k
                vv -= k
                continue
            u = ss_uniform(self.rs, pkt, row, draw)
            draw += 1
            q = det_log(1.0 - u) / det_log1m(ppp)
            if not q < float(vv):
                return
            vv -= int(math.floor(q)) + 1
            self.values[cell] -= 1

    def estimate(self, flow: bytes) -> int:
        est = 0
        for i in range(self.d):
            cell = i * self.w + mm3(flow, self.seeds[i]) % self.w
            if self.keys[cell] == flow:
                est = max(est, self.values[cell])
        return est

    def query(self, flow: bytes) -> int:
        return max(1, self.estimate(flow))

    def heavy(self):
        flows = {self.keys[c] for c in range(len(self.values)) if self.values[c] > 0}
        out = [(f, self.estimate(f)) for f in flows]
        out = [(f, v) for f, v in out if v >= self.thr]
        out.sort(key=lambda fv: (-fv[1], fv[0]))
        return out
