"""statistic.Sketch mirror backed by the MI355X engine.

Reference: internal/engine/impl/sketch/statistic/sketch.go:5-28
    type Sketch interface {
        Insert(flow, elem []byte, size uint32)
        Query(flow []byte) uint64
        HeavyHitters() HeavyRecord
        Reset()
    }

CountMin (count_min.go) and SuperSpread (super_spread.go) keep those four
methods (Go names kept as aliases) and add the batched entry points the GPU
needs: insert_keys / insert_tuples / insert_headers take whole packet batches,
host (numpy) or device-resident (torch tensors on the handle's GPU).
"""
from __future__ import annotations

import ctypes as ct
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import check


# --- sketch.go:13-28 -------------------------------------------------------
@dataclass
class HeavySize:
    Flow: bytes
    Size: int


@dataclass
class HeavyCount:
    Flow: bytes
    Count: int


@dataclass
class HeavyRecord:
    """HeavyRecord{Size, Count}.  Size is None for SuperSpread (writers use
    `Size is not None` to tell Count-Min from SuperSpread, writer_text.go:45-93)."""
    Size: Optional[List[HeavySize]] = field(default_factory=list)
    Count: List[HeavyCount] = field(default_factory=list)


def _is_device(x) -> bool:
    return hasattr(x, "data_ptr") and getattr(x, "is_cuda", False)


def _ptr(x) -> int:
    if _is_device(x):
        if not x.is_contiguous():
            raise ValueError("device tensors must be contiguous")
        return x.data_ptr()
    return x.ctypes.data


def _host(x, dtype) -> np.ndarray:
    return np.ascontiguousarray(x, dtype=dtype)


def _where(*arrays) -> int:
    dev = [_is_device(a) for a in arrays if a is not None]
    if dev and all(dev):
        _lib.device_ready(*arrays)
        return _lib.MEM_DEVICE
    if any(dev):
        raise ValueError("mix of host and device arrays in one call")
    return _lib.MEM_HOST


def _seeds_arg(seeds, depth):
    if seeds is None:
        return None, None
    arr = np.ascontiguousarray(seeds, dtype=np.uint32)
    if depth and arr.shape[0] < depth:
        raise ValueError(f"need {depth} seeds, got {arr.shape[0]}")
    return arr, arr.ctypes.data


def _cm_heavy_arrays(fn, h, key_bytes, hint=None):
    """gns_cm_heavy_hitters / gns_cm_view_heavy_hitters into buffers of the capacity
    `hint` ([count, size], updated in place); a list longer than its buffer is
    fetched again with the full length the first call reported."""
    K = max(key_bytes, 1)
    hint = hint if hint is not None else [0, 0]
    while True:
        cc, cs = max(hint[0], 1), max(hint[1], 1)
        cf = np.empty((cc, K), np.uint8)  # rows [0, n) are written by the call
        cv = np.empty(cc, np.uint32)
        sf = np.empty((cs, K), np.uint8)
        sv = np.empty(cs, np.uint32)
        nc, ns = ct.c_uint64(cc), ct.c_uint64(cs)
        check(fn(h, cf.ctypes.data, cv.ctypes.data, ct.byref(nc), sf.ctypes.data, sv.ctypes.data, ct.byref(ns)))
        if nc.value <= cc and ns.value <= cs:
            # next call: room for some growth, so a window usually needs one call
            hint[0], hint[1] = 2 * nc.value + 64, 2 * ns.value + 64
            return cf[:nc.value], cv[:nc.value], sf[:ns.value], sv[:ns.value]
        hint[0], hint[1] = max(hint[0], nc.value), max(hint[1], ns.value)


def _cm_heavy_record(arrays, key_bytes) -> "HeavyRecord":
    cf, cv, sf, sv = arrays
    kb = key_bytes
    return HeavyRecord(Size=[HeavySize(bytes(sf[i, :kb]), int(sv[i])) for i in range(len(sv))],
                       Count=[HeavyCount(bytes(cf[i, :kb]), int(cv[i])) for i in range(len(cv))])


class CountMinView:
    """Snapshot of a CountMin taken at a point of its insert stream (refresh()),
    queried from any thread while the handle keeps inserting: the read side of
    BASELINE configs[4] ("queries concurrent with ingest").  The reference's
    snapshotter reads live buckets under concurrent inserts (manager.go:139-159);
    a view answers exactly what the handle would have answered at the refresh."""

    def __init__(self, cm: "CountMin"):
        self._L = cm._L
        self._cm = cm
        self.key_bytes = cm.key_bytes
        self._hh_hint = [0, 0]
        h = ct.c_void_p()
        check(self._L.gns_cm_view_create(cm._h, ct.byref(h)))
        self._h = h

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.gns_cm_view_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def refresh(self) -> None:
        """Ingest side: snapshot the state after every insert issued so far (asynchronous)."""
        check(self._L.gns_cm_view_refresh(self._h))

    def heavy_hitters_arrays(self):
        return _cm_heavy_arrays(self._L.gns_cm_view_heavy_hitters, self._h, self.key_bytes, self._hh_hint)

    def heavy_hitters(self) -> "HeavyRecord":
        return _cm_heavy_record(self.heavy_hitters_arrays(), self.key_bytes)

    def query_many(self, keys) -> np.ndarray:
        keys = _host(keys, np.uint8)
        n = keys.shape[0]
        out = np.zeros(n, dtype=np.uint64)
        if n:
            keys = keys.reshape(n, -1)
            check(self._L.gns_cm_view_query(self._h, keys.ctypes.data, keys.shape[1], n, out.ctypes.data))
        return out


class CountMin:
    """Fingerprinted majority-vote "CountMin" of count_min.go on one GPU.

    Defaults mirror NewCountMin (count_min.go:48-59).  Row seeds are injected
    (the reference draws them from math/rand/v2, count_min.go:61-64)."""

    def __init__(self, width: int = 0, depth: int = 0, size_threshold: int = 0,
                 count_threshold: int = 0, flow_fields: Optional[Sequence[str]] = None,
                 key_bytes: Optional[int] = None, seeds=None, max_flows: int = 0,
                 batch_packets: int = 0, device: int = 0, bucket_range=None):
        """bucket_range=(lo, hi): apply only the updates whose row bucket is in
        [lo, hi) (SURVEY §8e exact global mode; dist.bucket_slice / dist.assemble_slices)."""
        self._L = _lib.load()
        self.flow_fields = list(flow_fields or [])
        kb = key_bytes if key_bytes is not None else _lib.layout_bytes(self.flow_fields)
        p = _lib.CmParams()
        p.width, p.depth = width, depth
        p.size_threshold, p.count_threshold = size_threshold, count_threshold
        p.flow = _lib.Layout.of(self.flow_fields)
        p.key_bytes = kb
        self._seeds, p.seeds = _seeds_arg(seeds, depth or 3)
        p.max_flows, p.batch_packets, p.device = max_flows, batch_packets, device
        if bucket_range is not None:
            p.bucket_lo, p.bucket_hi = int(bucket_range[0]), int(bucket_range[1])
        h = ct.c_void_p()
        check(self._L.gns_cm_create(ct.byref(p), ct.byref(h)))
        self._h = h
        self.bucket_range = tuple(bucket_range) if bucket_range is not None else None
        self.width = width or (1 << 20)
        self.depth = depth or 3
        self.size_threshold = size_threshold or 512 * 1024
        self.count_threshold = count_threshold or 512
        self.key_bytes = kb
        self.device = device
        self._hh_hint = [0, 0]

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.gns_cm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- batched inserts (stream order = call order, then array order) ---
    def insert_keys(self, keys, sizes) -> None:
        """Sketch.Insert for a batch: keys[n, stride] uint8 (first key_bytes used)."""
        where = _where(keys, sizes)
        if where == _lib.MEM_HOST:
            sizes = _host(sizes, np.uint32)
            keys = (_host(keys, np.uint8).reshape(len(sizes), -1) if len(sizes)
                    else np.zeros((0, max(self.key_bytes, 1)), np.uint8))  # empty batch
        n = int(sizes.shape[0])
        stride = int(keys.shape[1]) if n else max(self.key_bytes, 1)
        check(self._L.gns_cm_insert_keys(self._h, _ptr(keys), stride, _ptr(sizes), n, where))

    def insert_tuples(self, batch) -> None:
        """Task.ProcessPacket for a PacketBatch (packets.PacketBatch)."""
        t, keep, where = batch.c_struct()
        check(self._L.gns_cm_insert_tuples(self._h, ct.byref(t), len(batch), where))
        del keep

    def insert_headers(self, hdr, wirelen) -> None:
        """64-byte header records [n, 64] uint8 + wire lengths [n] uint32."""
        where = _where(hdr, wirelen)
        if where == _lib.MEM_HOST:
            hdr = _host(hdr, np.uint8)
            wirelen = _host(wirelen, np.uint32)
        n = int(wirelen.shape[0])
        check(self._L.gns_cm_insert_headers(self._h, _ptr(hdr), _ptr(wirelen), n, where))

    def insert_compact(self, rec16, wirelen, side=None) -> None:
        """Compact 16-byte records [n, 16] + wire lengths [n] (+ the 64-byte side
        records their escapes name, [n_side, 64]): the same stream as the 64-byte
        records they were made from (packets.compact_headers / read_pcap_compact).
        wirelen None: the 16-byte form, whose records carry the wire lengths
        (packets.compact_headers(..., rec_len=True) / read_pcap_compact(..., rec_len=True))."""
        where = _where(*[a for a in (rec16, wirelen, side) if a is not None])
        if where == _lib.MEM_HOST:
            rec16 = _host(rec16, np.uint8)
            wirelen = _host(wirelen, np.uint32) if wirelen is not None else None
            side = _host(side, np.uint8) if side is not None else None
        n = int(rec16.shape[0])
        if wirelen is not None and int(wirelen.shape[0]) != n:
            raise ValueError("rec16 and wirelen lengths differ")
        ns = int(side.shape[0]) if side is not None else 0
        check(self._L.gns_cm_insert_compact(self._h, _ptr(rec16), _ptr(wirelen) if wirelen is not None else None, n,
                                            _ptr(side) if ns else None, ns, where))

    def flush(self) -> None:
        check(self._L.gns_cm_flush(self._h))

    # --- statistic.Sketch ---
    def insert(self, flow: bytes, elem: bytes = b"", size: int = 0) -> None:
        """Insert(flow, elem, size); elem is unused by CountMin (count_min.go:94)."""
        k = np.frombuffer(bytes(flow), dtype=np.uint8).reshape(1, -1)
        self.insert_keys(k, np.array([size], dtype=np.uint32))

    def query_many(self, keys) -> np.ndarray:
        """Query for n keys [n, K] -> count<<32 | size each.  Host keys give a numpy
        uint64 array; a device tensor gives a device int64 tensor (the uint64 bits),
        answered without leaving the GPU (gns_cm_query_device)."""
        if _lib.is_device(keys):
            return _lib.query_device(self._L.gns_cm_query_device, self._h, keys)
        keys = _host(keys, np.uint8)
        n = keys.shape[0]
        out = np.zeros(n, dtype=np.uint64)
        if n:
            keys = keys.reshape(n, -1)
            check(self._L.gns_cm_query(self._h, keys.ctypes.data, keys.shape[1], n, out.ctypes.data))
        return out

    def query(self, flow: bytes) -> int:
        """Query(flow) = count<<32 | size (count_min.go:160-174)."""
        if len(flow) != self.key_bytes:
            return 0  # bytes.Equal against FS-byte fingerprints never matches
        return int(self.query_many(np.frombuffer(bytes(flow), np.uint8).reshape(1, -1))[0])

    def heavy_hitters_arrays(self):
        """HeavyHitters as arrays (count flows [n,K], counts, size flows, sizes): the
        snapshot handed to a writer without building per-flow Python objects."""
        return _cm_heavy_arrays(self._L.gns_cm_heavy_hitters, self._h, self.key_bytes, self._hh_hint)

    def heavy_hitters(self) -> HeavyRecord:
        return _cm_heavy_record(self.heavy_hitters_arrays(), self.key_bytes)

    def heavy_hitters_rows_device(self):
        """HeavyHitters as two DEVICE tensors of packed rows [flow | u32 value] (count list,
        size list; uint8 [n, key_bytes + 4]) in canonical order: the multi-GPU window exchange
        all-gathers them and merges on the device (dist.allgather_heavy_rows)."""
        import torch
        dev = torch.device("cuda", self.device)
        W = self.key_bytes + 4
        nc, ns = ct.c_uint64(0), ct.c_uint64(0)
        check(self._L.gns_cm_heavy_rows(self._h, None, ct.byref(nc), None, ct.byref(ns)))
        while True:
            cr = torch.empty((max(nc.value, 1), W), dtype=torch.uint8, device=dev)
            sr = torch.empty((max(ns.value, 1), W), dtype=torch.uint8, device=dev)
            c2, s2 = ct.c_uint64(cr.shape[0]), ct.c_uint64(sr.shape[0])
            check(self._L.gns_cm_heavy_rows(self._h, cr.data_ptr(), ct.byref(c2), sr.data_ptr(), ct.byref(s2)))
            if c2.value <= cr.shape[0] and s2.value <= sr.shape[0]:
                return cr[: c2.value], sr[: s2.value]
            nc, ns = c2, s2  # the lists changed between the calls (cannot on one handle; kept for safety)

    def view(self) -> "CountMinView":
        """A snapshot view whose heavy hitters / queries run concurrently with
        this handle's inserts (gns_cm_view_*); refresh() it at window boundaries."""
        return CountMinView(self)

    def reset(self) -> None:
        check(self._L.gns_cm_reset(self._h))

    # Go-style names (statistic.Sketch)
    Insert = insert
    Query = query
    HeavyHitters = heavy_hitters
    Reset = reset

    # --- parity / observability ---
    def export_counters(self, C=None, S=None):
        """Counter rows only (C, S as u32 [d*w]) to host memory: the per-window D2H."""
        n = self.depth * self.width
        C = np.empty(n, np.uint32) if C is None else C
        S = np.empty(n, np.uint32) if S is None else S
        check(self._L.gns_cm_export_state(self._h, C.ctypes.data, S.ctypes.data, None, None))
        return C, S

    def export_state(self):
        n = self.depth * self.width
        K = max(self.key_bytes, 1)
        C = np.empty(n, np.uint32)
        S = np.empty(n, np.uint32)
        Fc = np.empty((n, K), np.uint8)
        Fs = np.empty((n, K), np.uint8)
        check(self._L.gns_cm_export_state(self._h, C.ctypes.data, S.ctypes.data, Fc.ctypes.data,
                                          Fs.ctypes.data))
        return C, S, Fc[:, : self.key_bytes], Fs[:, : self.key_bytes]

    def stats(self) -> dict:
        s = (ct.c_uint64 * 4)()
        check(self._L.gns_cm_stats(self._h, s))
        return {"inserted": s[0], "dropped": s[1], "unsupported": s[2], "flows": s[3]}

    def counters(self) -> dict:
        c = (ct.c_uint64 * 8)()
        check(self._L.gns_cm_counters(self._h, c))
        names = ["inserted", "dropped", "unsupported", "dict_full", "ovf_full", "replayed", "chunks",
                 "chunks_replay"]
        return dict(zip(names, list(c)))

    def dict_stats(self) -> dict:
        """Flow-dictionary reclaim counters (gns_cm_dict_stats)."""
        return _lib.dict_stats(self._L.gns_cm_dict_stats, self._h)

    def reclaim(self) -> None:
        """Drop the flows no bucket names from the dictionary now (gns_cm_reclaim)."""
        check(self._L.gns_cm_reclaim(self._h))

    def set_timing(self, on: bool = True, stages=None) -> None:
        """Per-stage HIP-event timing; ``stages`` (names of STAGES) limits it to those stages
        (each timed stage puts two events into every batch)."""
        check(self._L.gns_cm_set_timing(self._h, _lib.timing_arg(on, stages, self.STAGES)))

    STAGES = ["extract", "resolve", "scan", "scatter", "apply", "insert", "hot", "designate"]

    def stage_times(self, reset: bool = False) -> dict:
        ms = (ct.c_double * 8)()
        ln = (ct.c_uint64 * 8)()
        check(self._L.gns_cm_stage_times(self._h, ms, ln, 1 if reset else 0))
        return {name: (ms[i], ln[i]) for i, name in enumerate(self.STAGES)}

    def stream(self) -> int:
        return int(self._L.gns_cm_stream(self._h) or 0)


class SuperSpread:
    """SuperSpread of super_spread.go on one GPU (declared RNG, injected HLL seeds)."""

    def __init__(self, width: int = 0, depth: int = 0, threshold: int = 0, m: int = 0, size: int = 0,
                 base: float = 0.0, b: float = 0.0, flow_fields: Optional[Sequence[str]] = None,
                 elem_fields: Optional[Sequence[str]] = None, flow_bytes: Optional[int] = None,
                 elem_bytes: Optional[int] = None, seeds=None, hll_master: int = 0x1234ABCD5678EF01,
                 rng_seed: int = 0x0DDBA11CAFEF00D5, batch_packets: int = 0, device: int = 0,
                 max_flows: int = 0):
        self._L = _lib.load()
        self.flow_fields = list(flow_fields or [])
        self.elem_fields = list(elem_fields or [])
        fb = flow_bytes if flow_bytes is not None else _lib.layout_bytes(self.flow_fields)
        eb = elem_bytes if elem_bytes is not None else _lib.layout_bytes(self.elem_fields)
        p = _lib.SsParams()
        p.width, p.depth, p.threshold, p.m, p.size = width, depth, threshold, m, size
        p.base, p.b = base, b
        p.flow, p.elem = _lib.Layout.of(self.flow_fields), _lib.Layout.of(self.elem_fields)
        p.flow_bytes, p.elem_bytes = fb, eb
        self._seeds, p.seeds = _seeds_arg(seeds, depth or 3)
        p.hll_master, p.rng_seed, p.batch_packets, p.device = hll_master, rng_seed, batch_packets, device
        p.max_flows = max_flows
        h = ct.c_void_p()
        check(self._L.gns_ss_create(ct.byref(p), ct.byref(h)))
        self._h = h
        self.width, self.depth = width or (1 << 20), depth or 3
        self.threshold, self.m = threshold or 4096, m or 128
        self.flow_bytes, self.elem_bytes = fb, eb
        self.device = device

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.gns_ss_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def insert_keys(self, flows, elems) -> None:
        where = _where(flows, elems)
        if where == _lib.MEM_HOST:
            if len(flows) == 0:  # empty batch (numpy cannot infer -1 of a size-0 reshape)
                flows = np.zeros((0, max(self.flow_bytes, 1)), np.uint8)
                elems = np.zeros((0, max(self.elem_bytes, 1)), np.uint8)
            else:
                flows = _host(flows, np.uint8).reshape(len(flows), -1)
                elems = _host(elems, np.uint8).reshape(len(elems), -1)
        n = int(flows.shape[0])
        fs = int(flows.shape[1]) if n else max(self.flow_bytes, 1)
        es = int(elems.shape[1]) if n else max(self.elem_bytes, 1)
        check(self._L.gns_ss_insert_keys(self._h, _ptr(flows), fs, _ptr(elems), es, n, where))

    def insert_tuples(self, batch) -> None:
        t, keep, where = batch.c_struct()
        check(self._L.gns_ss_insert_tuples(self._h, ct.byref(t), len(batch), where))
        del keep

    def insert_headers(self, hdr, wirelen) -> None:
        where = _where(hdr, wirelen)
        if where == _lib.MEM_HOST:
            hdr = _host(hdr, np.uint8)
            wirelen = _host(wirelen, np.uint32)
        check(self._L.gns_ss_insert_headers(self._h, _ptr(hdr), _ptr(wirelen), int(wirelen.shape[0]), where))

    def flush(self) -> None:
        check(self._L.gns_ss_flush(self._h))

    def insert(self, flow: bytes, elem: bytes, size: int = 0) -> None:
        self.insert_keys(np.frombuffer(bytes(flow), np.uint8).reshape(1, -1),
                         np.frombuffer(bytes(elem), np.uint8).reshape(1, -1))

    def query_many(self, flows) -> np.ndarray:
        """max(1, estimate) for n flows; a device tensor in -> a device int64 tensor out."""
        if _lib.is_device(flows):
            return _lib.query_device(self._L.gns_ss_query_device, self._h, flows)
        flows = _host(flows, np.uint8)
        n = flows.shape[0]
        out = np.zeros(n, dtype=np.uint64)
        if n:
            flows = flows.reshape(n, -1)
            check(self._L.gns_ss_query(self._h, flows.ctypes.data, flows.shape[1], n, out.ctypes.data))
        return out

    def query(self, flow: bytes) -> int:
        """max(1, spread estimate), super_spread.go:238-249."""
        if len(flow) != self.flow_bytes:
            return 1
        return int(self.query_many(np.frombuffer(bytes(flow), np.uint8).reshape(1, -1))[0])

    def heavy_hitters_arrays(self):
        """HeavyHitters as arrays (flows [n, flow_bytes], spreads): one device call into
        buffers sized from the previous list (a longer list is fetched again)."""
        K = max(self.flow_bytes, 1)
        hint = getattr(self, "_hh_cap", 0)
        while True:
            cap = max(hint, 1)
            f = np.empty((cap, K), np.uint8)
            v = np.empty(cap, np.uint32)
            n = ct.c_uint64(cap)
            check(self._L.gns_ss_heavy_hitters(self._h, f.ctypes.data, v.ctypes.data, ct.byref(n)))
            if n.value <= cap:
                self._hh_cap = 2 * n.value + 64
                return f[: n.value, : self.flow_bytes], v[: n.value]
            hint = n.value

    def heavy_hitters(self) -> HeavyRecord:
        """HeavyHitters (super_spread.go:254-294): Count = (flow, spread estimate), Size = None."""
        f, v = self.heavy_hitters_arrays()
        return HeavyRecord(Size=None, Count=[HeavyCount(bytes(f[i]), int(v[i])) for i in range(len(v))])

    def reset(self) -> None:
        check(self._L.gns_ss_reset(self._h))

    Insert = insert
    Query = query
    HeavyHitters = heavy_hitters
    Reset = reset

    def export_state(self):
        n = self.depth * self.width
        values = np.empty(n, np.uint32)
        keys = np.empty((n, max(self.flow_bytes, 1)), np.uint8)
        regs = np.empty((n, self.m), np.uint8)
        pbits = np.empty(n, np.float64)
        check(self._L.gns_ss_export_state(self._h, values.ctypes.data, keys.ctypes.data, regs.ctypes.data,
                                          pbits.ctypes.data))
        return values, keys[:, : self.flow_bytes], regs, pbits

    def stats(self) -> dict:
        s = (ct.c_uint64 * 4)()
        check(self._L.gns_ss_stats(self._h, s))
        return {"inserted": s[0], "dropped": s[1], "unsupported": s[2], "packets": s[3]}

    def counters(self) -> dict:
        s = (ct.c_uint64 * 8)()
        check(self._L.gns_ss_counters(self._h, s))
        names = ["inserted", "dropped", "unsupported", "dict_full", "candidates", "encodes", "records", "batches"]
        return {k: int(s[i]) for i, k in enumerate(names)}

    def dict_stats(self) -> dict:
        """Flow-dictionary reclaim counters (gns_ss_dict_stats)."""
        return _lib.dict_stats(self._L.gns_ss_dict_stats, self._h)

    def reclaim(self) -> None:
        check(self._L.gns_ss_reclaim(self._h))

    def set_timing(self, on: bool = True, stages=None) -> None:
        check(self._L.gns_ss_set_timing(self._h, _lib.timing_arg(on, stages, self.STAGES)))

    STAGES = ["extract", "resolve", "encode", "apply", "unused", "total"]

    def stage_times(self, reset: bool = False) -> dict:
        ms = (ct.c_double * 8)()
        ln = (ct.c_uint64 * 8)()
        check(self._L.gns_ss_stage_times(self._h, ms, ln, 1 if reset else 0))
        return {name: (ms[i], ln[i]) for i, name in enumerate(self.STAGES)}
