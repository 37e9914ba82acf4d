"""ctypes binding of the C oracle (TEST INFRASTRUCTURE / CPU BASELINE ONLY).

Loads oracle/libgns_oracle.so (built by `make -C oracle` or __graft_entry__.build()).
Product code in go2netspectra_amd/ must never import this module.
"""
from __future__ import annotations

import ctypes as ct
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libgns_oracle.so")
_lib = None

FIELD_IDS = {"SrcIP": 1, "DstIP": 2, "SrcPort": 3, "DstPort": 4, "Protocol": 5}

u8p = ct.POINTER(ct.c_uint8)
u32p = ct.POINTER(ct.c_uint32)


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        build()
    L = ct.CDLL(_LIB_PATH)
    L.or_mm3.restype = ct.c_uint32
    L.or_mm3.argtypes = [ct.c_void_p, ct.c_uint32, ct.c_uint32]
    L.or_parse_hdr64_len.restype = ct.c_int
    L.or_parse_hdr64_len.argtypes = [ct.c_void_p, ct.c_uint32, ct.c_void_p]
    L.or_encode_key.restype = ct.c_uint32
    L.or_encode_key.argtypes = [ct.c_void_p, ct.c_uint32, ct.c_void_p, ct.c_void_p]
    L.or_cm_new.restype = ct.c_void_p
    L.or_cm_new.argtypes = [ct.c_uint32] * 5 + [ct.c_void_p]
    L.or_cm_free.argtypes = [ct.c_void_p]
    L.or_cm_params.argtypes = [ct.c_void_p] + [ct.c_void_p] * 4
    L.or_cm_insert.argtypes = [ct.c_void_p, ct.c_void_p, ct.c_uint32]
    L.or_cm_insert_batch.argtypes = [ct.c_void_p, ct.c_void_p, ct.c_uint32, ct.c_void_p, ct.c_uint64]
    L.or_cm_insert_hdr64.restype = ct.c_uint64
    L.or_cm_insert_hdr64.argtypes = [ct.c_void_p, ct.c_void_p, ct.c_void_p, ct.c_uint64, ct.c_void_p,
                                     ct.c_uint32]
    L.or_cm_insert_hdr64_pool.restype = ct.c_uint64
    L.or_cm_insert_hdr64_pool.argtypes = [ct.c_void_p, ct.c_void_p, ct.c_void_p, ct.c_uint64,
                                          ct.c_void_p, ct.c_uint32, ct.c_int]
    L.or_cm_query.restype = ct.c_uint64
    L.or_cm_query.argtypes = [ct.c_void_p, ct.c_void_p]
    L.or_cm_export.argtypes = [ct.c_void_p] + [ct.c_void_p] * 4
    L.or_cm_import.argtypes = [ct.c_void_p] + [ct.c_void_p] * 4
    L.or_cm_heavy.restype = ct.c_uint32
    L.or_cm_heavy.argtypes = [ct.c_void_p, ct.c_int, ct.c_void_p, ct.c_void_p, ct.c_uint32]
    L.or_cm_reset.argtypes = [ct.c_void_p]
    L.or_ss_new.restype = ct.c_void_p
    L.or_ss_new.argtypes = [ct.c_uint32] * 5 + [ct.c_double, ct.c_double, ct.c_uint32, ct.c_uint32,
                                                ct.c_void_p, ct.c_uint64, ct.c_uint64]
    L.or_ss_free.argtypes = [ct.c_void_p]
    L.or_ss_insert.argtypes = [ct.c_void_p, ct.c_void_p, ct.c_void_p]
    L.or_ss_insert_batch.argtypes = [ct.c_void_p, ct.c_void_p, ct.c_uint32, ct.c_void_p, ct.c_uint32,
                                     ct.c_uint64]
    L.or_ss_insert_hdr64.restype = ct.c_uint64
    L.or_ss_insert_hdr64.argtypes = [ct.c_void_p, ct.c_void_p, ct.c_void_p, ct.c_uint64, ct.c_void_p, ct.c_uint32,
                                     ct.c_void_p, ct.c_uint32]
    L.or_ss_query.restype = ct.c_uint64
    L.or_ss_query.argtypes = [ct.c_void_p, ct.c_void_p]
    L.or_ss_heavy.restype = ct.c_uint32
    L.or_ss_heavy.argtypes = [ct.c_void_p, ct.c_void_p, ct.c_void_p, ct.c_uint32]
    L.or_ss_export.argtypes = [ct.c_void_p] + [ct.c_void_p] * 4
    L.or_ss_reset.argtypes = [ct.c_void_p]
    L.or_ss_packets.restype = ct.c_uint64
    L.or_ss_packets.argtypes = [ct.c_void_p]
    L.or_mix64.restype = ct.c_uint64
    L.or_mix64.argtypes = [ct.c_uint64]
    L.or_det_log.restype = ct.c_double
    L.or_det_log.argtypes = [ct.c_double]
    L.or_det_log1m.restype = ct.c_double
    L.or_det_log1m.argtypes = [ct.c_double]
    L.or_ex_new.restype = ct.c_void_p
    L.or_ex_new.argtypes = [ct.c_void_p, ct.c_uint32]
    L.or_ex_free.argtypes = [ct.c_void_p]
    L.or_ex_reset.argtypes = [ct.c_void_p]
    L.or_ex_insert_tuples.argtypes = [ct.c_void_p] + [ct.c_void_p] * 8 + [ct.c_uint64]
    L.or_ex_insert_hdr64.restype = ct.c_uint64
    L.or_ex_insert_hdr64.argtypes = [ct.c_void_p, ct.c_void_p, ct.c_void_p, ct.c_void_p, ct.c_uint64]
    L.or_ex_query.restype = ct.c_uint64
    L.or_ex_query.argtypes = [ct.c_void_p, ct.c_void_p]
    L.or_ex_count.restype = ct.c_uint64
    L.or_ex_count.argtypes = [ct.c_void_p]
    L.or_ex_export.restype = ct.c_uint64
    L.or_ex_export.argtypes = [ct.c_void_p, ct.c_void_p, ct.c_uint64] + [ct.c_void_p] * 4
    L.or_thrift_decode.restype = ct.c_uint64
    L.or_thrift_decode.argtypes = [ct.c_void_p] * 2 + [ct.c_uint64] + [ct.c_void_p] * 10
    L.or_ss_uniform.restype = ct.c_double
    L.or_ss_uniform.argtypes = [ct.c_uint64, ct.c_uint64, ct.c_uint32, ct.c_uint32]
    L.or_go_pow.restype = ct.c_double
    L.or_go_pow.argtypes = [ct.c_double, ct.c_double]
    _lib = L
    return L


def _p(a: np.ndarray):
    return a.ctypes.data_as(ct.c_void_p)


def mm3(data: bytes, seed: int) -> int:
    buf = (ct.c_uint8 * max(1, len(data))).from_buffer_copy(data or b"\0")
    return lib().or_mm3(buf, len(data), seed & 0xFFFFFFFF)


class TupleRec(ct.Structure):
    _fields_ = [("src", ct.c_uint8 * 16), ("dst", ct.c_uint8 * 16), ("sport", ct.c_uint16),
                ("dport", ct.c_uint16), ("proto", ct.c_uint8), ("ipver", ct.c_uint8), ("dst_ipver", ct.c_uint8)]


def parse_hdr64(rec: bytes, wirelen: int):
    """-> (status, src16, dst16, sport, dport, proto)"""
    assert len(rec) == 64
    buf = (ct.c_uint8 * 64).from_buffer_copy(rec)
    t = TupleRec()
    st = lib().or_parse_hdr64_len(buf, wirelen & 0xFFFFFFFF, ct.byref(t))
    return st, bytes(t.src), bytes(t.dst), t.sport, t.dport, t.proto


def field_ids(fields) -> np.ndarray:
    return np.array([FIELD_IDS.get(f, 0) for f in fields] or [0], dtype=np.uint8)


class CountMin:
    """Sequential oracle CountMin (count_min.go) over injected seeds."""

    def __init__(self, width, depth, st, ct_, key_bytes, seeds):
        self.L = lib()
        seeds = np.ascontiguousarray(seeds, dtype=np.uint32)
        self.h = self.L.or_cm_new(width, depth, st, ct_, key_bytes, _p(seeds))
        w, d, s, c = (ct.c_uint32(), ct.c_uint32(), ct.c_uint32(), ct.c_uint32())
        self.L.or_cm_params(self.h, ct.byref(w), ct.byref(d), ct.byref(s), ct.byref(c))
        self.w, self.d, self.st, self.ct, self.K = w.value, d.value, s.value, c.value, key_bytes

    def __del__(self):
        if getattr(self, "h", None):
            self.L.or_cm_free(self.h)
            self.h = None

    def insert_keys(self, keys: np.ndarray, sizes: np.ndarray):
        keys = np.ascontiguousarray(keys, dtype=np.uint8)
        sizes = np.ascontiguousarray(sizes, dtype=np.uint32)
        n = sizes.shape[0]
        stride = keys.shape[1] if keys.ndim == 2 else self.K
        self.L.or_cm_insert_batch(self.h, _p(keys), stride, _p(sizes), n)

    def insert_hdr64(self, hdr: np.ndarray, wirelen: np.ndarray, fields) -> int:
        hdr = np.ascontiguousarray(hdr, dtype=np.uint8)
        wirelen = np.ascontiguousarray(wirelen, dtype=np.uint32)
        f = field_ids(fields)
        return self.L.or_cm_insert_hdr64(self.h, _p(hdr), _p(wirelen), wirelen.shape[0], _p(f), len(fields))

    def insert_hdr64_pool(self, hdr, wirelen, fields, nthreads: int) -> int:
        hdr = np.ascontiguousarray(hdr, dtype=np.uint8)
        wirelen = np.ascontiguousarray(wirelen, dtype=np.uint32)
        f = field_ids(fields)
        return self.L.or_cm_insert_hdr64_pool(self.h, _p(hdr), _p(wirelen), wirelen.shape[0], _p(f),
                                              len(fields), nthreads)

    def query(self, key: bytes) -> int:
        buf = (ct.c_uint8 * max(1, len(key))).from_buffer_copy(key or b"\0")
        return self.L.or_cm_query(self.h, buf)

    def export(self):
        n = self.d * self.w
        C = np.empty(n, np.uint32)
        S = np.empty(n, np.uint32)
        Fc = np.empty((n, max(self.K, 1)), np.uint8)
        Fs = np.empty((n, max(self.K, 1)), np.uint8)
        self.L.or_cm_export(self.h, _p(C), _p(S), _p(Fc), _p(Fs))
        return C, S, Fc[:, : self.K], Fs[:, : self.K]

    def heavy_arrays(self, which: str):
        """(flows [n, K] u8, values [n] u32) in the canonical order, without per-entry objects"""
        w = 0 if which == "count" else 1
        n = self.L.or_cm_heavy(self.h, w, None, None, 0)
        flows = np.empty((max(n, 1), max(self.K, 1)), np.uint8)
        vals = np.empty(max(n, 1), np.uint32)
        self.L.or_cm_heavy(self.h, w, _p(flows), _p(vals), n)
        return flows[:n, : self.K], vals[:n]

    def heavy(self, which: str):
        w = 0 if which == "count" else 1
        n = self.L.or_cm_heavy(self.h, w, None, None, 0)
        flows = np.empty((max(n, 1), max(self.K, 1)), np.uint8)
        vals = np.empty(max(n, 1), np.uint32)
        self.L.or_cm_heavy(self.h, w, _p(flows), _p(vals), n)
        return [(bytes(flows[i, : self.K]), int(vals[i])) for i in range(n)]

    def reset(self):
        self.L.or_cm_reset(self.h)


class SuperSpread:
    def __init__(self, width, depth, threshold, m, size, base, b, kf, ke, seeds, hll_master, rng_seed):
        self.L = lib()
        seeds = np.ascontiguousarray(seeds, dtype=np.uint32)
        self.h = self.L.or_ss_new(width, depth, threshold, m, size, base, b, kf, ke, _p(seeds),
                                  hll_master, rng_seed)
        if not self.h:
            raise ValueError("bad SuperSpread parameters")
        self.w = width or (1 << 20)
        self.d = depth or 3
        self.m = m or 128
        self.kf, self.ke = kf, ke

    def __del__(self):
        if getattr(self, "h", None):
            self.L.or_ss_free(self.h)
            self.h = None

    def insert(self, flows: np.ndarray, elems: np.ndarray):
        flows = np.ascontiguousarray(flows, dtype=np.uint8)
        elems = np.ascontiguousarray(elems, dtype=np.uint8)
        n = flows.shape[0]
        self.L.or_ss_insert_batch(self.h, _p(flows), self.kf, _p(elems), self.ke, n)

    def insert_hdr64(self, hdr, wirelen, flow_fields, elem_fields) -> int:
        hdr = np.ascontiguousarray(hdr, dtype=np.uint8)
        wirelen = np.ascontiguousarray(wirelen, dtype=np.uint32)
        ff = np.array([FIELD_IDS[f] for f in flow_fields] or [0], np.uint8)
        ef = np.array([FIELD_IDS[f] for f in elem_fields] or [0], np.uint8)
        return self.L.or_ss_insert_hdr64(self.h, _p(hdr), _p(wirelen), len(wirelen), _p(ff), len(flow_fields),
                                         _p(ef), len(elem_fields))

    def packets(self) -> int:
        return self.L.or_ss_packets(self.h)

    def query(self, flow: bytes) -> int:
        buf = (ct.c_uint8 * max(1, len(flow))).from_buffer_copy(flow or b"\0")
        return self.L.or_ss_query(self.h, buf)

    def heavy(self):
        n = self.L.or_ss_heavy(self.h, None, None, 0)
        flows = np.empty((max(n, 1), max(self.kf, 1)), np.uint8)
        vals = np.empty(max(n, 1), np.uint32)
        self.L.or_ss_heavy(self.h, _p(flows), _p(vals), n)
        return [(bytes(flows[i, : self.kf]), int(vals[i])) for i in range(n)]

    def export(self):
        n = self.d * self.w
        values = np.empty(n, np.uint32)
        keys = np.empty((n, max(self.kf, 1)), np.uint8)
        regs = np.empty((n, self.m), np.uint8)
        pbits = np.empty(n, np.float64)
        self.L.or_ss_export(self.h, _p(values), _p(keys), _p(regs), _p(pbits))
        return values, keys[:, : self.kf], regs, pbits

    def reset(self):
        self.L.or_ss_reset(self.h)


class Exact:
    """Sequential exact aggregator (exact/task.go) with Go-formatted string keys."""

    def __init__(self, fields):
        self.L = lib()
        f = field_ids(fields)
        self.fields = list(fields)
        self.h = self.L.or_ex_new(_p(f), len(fields))

    def __del__(self):
        if getattr(self, "h", None):
            self.L.or_ex_free(self.h)
            self.h = None

    def insert_tuples(self, src16, dst16, sport, dport, proto, ipver, length, ts):
        arrs = [np.ascontiguousarray(src16, np.uint8), np.ascontiguousarray(dst16, np.uint8),
                np.ascontiguousarray(sport, np.uint16), np.ascontiguousarray(dport, np.uint16),
                np.ascontiguousarray(proto, np.uint8), np.ascontiguousarray(ipver, np.uint8),
                np.ascontiguousarray(length, np.uint32), np.ascontiguousarray(ts, np.int64)]
        self.L.or_ex_insert_tuples(self.h, *[_p(a) for a in arrs], len(arrs[-1]))

    def insert_hdr64(self, hdr, wirelen, ts) -> int:
        hdr = np.ascontiguousarray(hdr, np.uint8)
        wirelen = np.ascontiguousarray(wirelen, np.uint32)
        ts = np.ascontiguousarray(ts, np.int64)
        return self.L.or_ex_insert_hdr64(self.h, _p(hdr), _p(wirelen), _p(ts), len(wirelen))

    def query(self, flow: bytes) -> int:
        buf = (ct.c_uint8 * max(1, len(flow))).from_buffer_copy(flow or b"\0")
        return self.L.or_ex_query(self.h, buf)

    def reset(self):
        self.L.or_ex_reset(self.h)

    def export(self):
        """{key string: (start_ns, end_ns, packets, bytes)}"""
        n = self.L.or_ex_count(self.h)
        cap = max(1, n) * 128
        keys = ct.create_string_buffer(cap)
        st, en = np.zeros(max(n, 1), np.int64), np.zeros(max(n, 1), np.int64)
        pk, by = np.zeros(max(n, 1), np.uint64), np.zeros(max(n, 1), np.uint64)
        self.L.or_ex_export(self.h, keys, cap, _p(st), _p(en), _p(pk), _p(by))
        names = keys.value.decode().split("\n")[:n]
        return {k: (int(st[i]), int(en[i]), int(pk[i]), int(by[i])) for i, k in enumerate(names)}


def thrift_decode(buf: bytes, offsets: np.ndarray) -> dict:
    """Sequential restatement of UnmarshalPacketInfo over a message batch."""
    L = lib()
    n = len(offsets) - 1
    b = np.frombuffer(bytes(buf) or b"\0", np.uint8)
    offsets = np.ascontiguousarray(offsets, np.uint64)
    out = dict(ok=np.zeros(n, np.uint8), src16=np.zeros((n, 16), np.uint8), dst16=np.zeros((n, 16), np.uint8),
               sport=np.zeros(n, np.uint16), dport=np.zeros(n, np.uint16), proto=np.zeros(n, np.uint8),
               sver=np.zeros(n, np.uint8), dver=np.zeros(n, np.uint8), length=np.zeros(n, np.int64),
               ts=np.zeros(n, np.int64))
    keys = ["ok", "src16", "dst16", "sport", "dport", "proto", "sver", "dver", "length", "ts"]
    L.or_thrift_decode(_p(b), _p(offsets), n, *[_p(out[k]) for k in keys])
    return out
