"""Exact aggregator on the GPU: the model.Task of internal/engine/impl/exact.

Reference: exact/task.go -- New (:83-103), ProcessPacket (:124-149), Snapshot
(:153-191), Reset (:194-210), AlerterMsg (:213-282), Query (:298-326),
generateKeyAndFields (:330-366); exact/statistic/flow.go (Flow, Shard,
SnapshotData).  The device engine (csrc/gns_exact.hip, C ABI gns_ex_*) keys
flows by canonical bytes (IP fields in 16-byte To16 form); the Go key string
and the Fields map are rebuilt here from those bytes for snapshots.
"""
from __future__ import annotations

import ctypes as ct
import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import check
from .packets import HeaderBatch, PacketBatch
from .task import _check, go_ip_string

DEFAULT_SHARDS = 256  # exact/task.go:72


@dataclass
class Flow:  # exact/statistic/flow.go:9-16
    Key: str
    Fields: Dict[str, object]
    StartTime: int  # ns since epoch (time.Time UnixNano)
    EndTime: int
    ByteCount: int
    PacketCount: int


@dataclass
class Shard:
    Flows: Dict[str, Flow] = field(default_factory=dict)


@dataclass
class SnapshotData:
    TaskName: str
    Shards: List[Shard]


def _ptr(a):
    return a.data_ptr() if hasattr(a, "data_ptr") else a.ctypes.data


def _is_dev(a) -> bool:
    return hasattr(a, "data_ptr") and getattr(a, "is_cuda", False)


class ExactAggregator:
    """One exact task's device state (gns_ex handle)."""

    def __init__(self, key_fields: Sequence[str], max_flows: int = 0, batch_packets: int = 0, device: int = 0):
        self._L = _lib.load()
        self.key_fields = list(key_fields)
        self.key_bytes = sum(_lib.FIELD_SIZE.get(f, 0) for f in self.key_fields)
        p = _lib.ExParams()
        p.key = _lib.Layout.of(self.key_fields)
        p.max_flows, p.batch_packets, p.device = max_flows, batch_packets, device
        h = ct.c_void_p()
        check(self._L.gns_ex_create(ct.byref(p), ct.byref(h)))
        self._h = h

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.gns_ex_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def insert_tuples(self, batch: PacketBatch) -> None:
        n = len(batch)
        t, keep, where = batch.c_struct()
        ipver, ts = batch.ipver, batch.ts
        if ts is None:
            raise ValueError("exact aggregation needs per-packet timestamps (PacketBatch.ts)")
        if where == _lib.MEM_HOST:
            ts = np.ascontiguousarray(ts, np.int64)
            ipver = None if ipver is None else np.ascontiguousarray(ipver, np.uint8)
        elif not _is_dev(ts) or (ipver is not None and not _is_dev(ipver)):
            raise ValueError("mix of host and device arrays")
        check(self._L.gns_ex_insert_tuples(self._h, ct.byref(t), None if ipver is None else _ptr(ipver), _ptr(ts),
                                           n, where))
        del keep

    def insert_headers(self, hdr, wirelen, ts) -> None:
        dev = [_is_dev(a) for a in (hdr, wirelen, ts)]
        if all(dev):
            _lib.device_ready(hdr, wirelen, ts)
            where = _lib.MEM_DEVICE
        elif any(dev):
            raise ValueError("mix of host and device arrays")
        else:
            where = _lib.MEM_HOST
            hdr = np.ascontiguousarray(hdr, np.uint8)
            wirelen = np.ascontiguousarray(wirelen, np.uint32)
            ts = np.ascontiguousarray(ts, np.int64)
        check(self._L.gns_ex_insert_headers(self._h, _ptr(hdr), _ptr(wirelen), _ptr(ts), int(wirelen.shape[0]),
                                            where))

    def flush(self) -> None:
        check(self._L.gns_ex_flush(self._h))

    def query_many(self, flows) -> np.ndarray:
        """PacketCount<<32 | ByteCount for n flows; a device tensor in -> a device int64 tensor out."""
        if _lib.is_device(flows):
            return _lib.query_device(self._L.gns_ex_query_device, self._h, flows)
        flows = np.ascontiguousarray(flows, np.uint8)
        n = flows.shape[0]
        out = np.zeros(n, np.uint64)
        if n:
            flows = flows.reshape(n, -1)
            check(self._L.gns_ex_query(self._h, flows.ctypes.data, flows.shape[1], n, out.ctypes.data))
        return out

    def snapshot_arrays(self):
        """(keys [n,K] canonical bytes, start, end, packets, bytes), dictionary slot order."""
        n = ct.c_uint64(0)
        check(self._L.gns_ex_snapshot(self._h, None, None, None, None, None, ct.byref(n)))
        m = n.value
        K = max(self.key_bytes, 1)
        keys = np.zeros((max(m, 1), K), np.uint8)
        st, en = np.zeros(max(m, 1), np.int64), np.zeros(max(m, 1), np.int64)
        pk, by = np.zeros(max(m, 1), np.uint64), np.zeros(max(m, 1), np.uint64)
        n2 = ct.c_uint64(m)
        check(self._L.gns_ex_snapshot(self._h, keys.ctypes.data, st.ctypes.data, en.ctypes.data, pk.ctypes.data,
                                      by.ctypes.data, ct.byref(n2)))
        m = min(m, n2.value)
        return keys[:m, : self.key_bytes], st[:m], en[:m], pk[:m], by[:m]

    def reset(self) -> None:
        check(self._L.gns_ex_reset(self._h))

    def counters(self) -> dict:
        s = (ct.c_uint64 * 8)()
        check(self._L.gns_ex_counters(self._h, s))
        names = ["inserted", "dropped", "unsupported", "dict_full", "flows", "records", "batches", "_"]
        return {k: int(s[i]) for i, k in enumerate(names) if k != "_"}

    def dict_stats(self) -> dict:
        """Table growth counters (gns_ex_dict_stats): growths, -, slots, claimed, us, re-run batches."""
        d = _lib.dict_stats(self._L.gns_ex_dict_stats, self._h)
        return {"growths": d["reclaims"], "slots": d["live"], "claimed": d["claimed"], "grow_us": d["reclaim_us"],
                "retried_batches": d["retried_batches"]}

    def set_timing(self, on: bool = True, stages=None) -> None:
        check(self._L.gns_ex_set_timing(self._h, _lib.timing_arg(on, stages, self.STAGES)))

    STAGES = ["extract", "resolve", "partition", "aggregate", "hot", "total"]

    def stage_times(self, reset: bool = False) -> dict:
        ms = (ct.c_double * 8)()
        ln = (ct.c_uint64 * 8)()
        check(self._L.gns_ex_stage_times(self._h, ms, ln, 1 if reset else 0))
        return {name: (ms[i], ln[i]) for i, name in enumerate(self.STAGES)}


def key_string(key: bytes, fields: Sequence[str]):
    """Go key string and Fields map from canonical key bytes (task.go:330-366)."""
    parts, vals, off = [], {}, 0
    for f in fields:
        if f in ("SrcIP", "DstIP"):
            v = go_ip_string(key[off:off + 16])
            off += 16
        elif f in ("SrcPort", "DstPort"):
            v = struct.unpack(">H", key[off:off + 2])[0]
            off += 2
        elif f == "Protocol":
            v = key[off]
            off += 1
        else:
            raise ValueError(f"unknown key field: {f}")
        parts.append(str(v))
        vals[f] = v
    return "-".join(parts), vals


class ExactTask:
    """model.Task of the exact aggregator (exact/task.go)."""

    def __init__(self, name: str, key_fields: Sequence[str], num_shards: int = 0, device: int = 0,
                 max_flows: int = 0, batch_packets: int = 0):
        if num_shards == 0 or num_shards >= 32768:  # task.go:85-87
            num_shards = DEFAULT_SHARDS
        self.name_ = name
        self.key_fields = list(key_fields)
        self.shard_count = num_shards
        self.agg = ExactAggregator(self.key_fields, max_flows=max_flows, batch_packets=batch_packets, device=device)

    def name(self) -> str:
        return self.name_

    def fields(self):  # task.go:111-114: exact tasks serialize no field list
        return None

    def decode_flow_func(self):
        return lambda flow, fields: ""

    def process_packets(self, batch) -> None:
        if isinstance(batch, HeaderBatch):
            ts = batch.ts if batch.ts is not None else np.zeros(len(batch), np.int64)
            self.agg.insert_headers(batch.hdr, batch.wirelen, ts)
        else:
            self.agg.insert_tuples(batch)

    def process_packet(self, info) -> None:
        """ProcessPacket(*PacketInfo); info = (src, dst, sport, dport, proto, length[, ts_ns])."""
        self.process_packets(PacketBatch.from_packets([info]))

    def query(self, flow: bytes) -> int:
        """Query (task.go:298-326): PacketCount<<32 | ByteCount, IP fields read as 16-byte IPs."""
        if len(flow) != self.agg.key_bytes:
            return 0
        return int(self.agg.query_many(np.frombuffer(bytes(flow), np.uint8).reshape(1, -1))[0])

    def flows(self) -> List[Flow]:
        keys, st, en, pk, by = self.agg.snapshot_arrays()
        out = []
        for i in range(len(pk)):
            k, vals = key_string(bytes(keys[i]), self.key_fields)
            out.append(Flow(k, vals, int(st[i]), int(en[i]), int(by[i]), int(pk[i])))
        return out

    def snapshot(self) -> SnapshotData:
        """Snapshot (task.go:153-191).  The reference spreads flows over shards by a
        randomly seeded maphash; here by a fixed hash of the key string."""
        import zlib
        shards = [Shard() for _ in range(self.shard_count)]
        for f in self.flows():
            shards[zlib.crc32(f.Key.encode()) % self.shard_count].Flows[f.Key] = f
        return SnapshotData(self.name_, shards)

    def reset(self) -> None:
        self.agg.reset()

    def flush(self) -> None:
        self.agg.flush()

    def alerter_msg(self, rules) -> str:
        """AlerterMsg (task.go:213-282): total_packets / total_bytes / total_flows."""
        keys, st, en, pk, by = self.agg.snapshot_arrays()
        totals = {"total_packets": (float(int(pk.sum())), "packets"), "total_bytes": (float(int(by.sum())), "bytes"),
                  "total_flows": (float(len(pk)), "flows")}
        msgs = []
        for rule in rules:
            if rule.get("task_name") != self.name_:
                continue
            metric = rule.get("metric")
            if metric not in totals:
                continue
            value, unit = totals[metric]
            op, thr = rule.get("operator", ">"), float(rule.get("threshold", 0))
            if _check(value, thr, op):
                msgs.append(f"<h3>Alert: {rule.get('name', '')}</h3><ul><li><b>Task:</b> <code>{rule.get('task_name')}</code></li>"
                            f"<li><b>Metric:</b> <code>{metric}</code></li><li><b>Condition:</b> <code>{op} {thr:.2f}</code></li>"
                            f"<li><b>Observed Value:</b> <code>{value:.0f} {unit}</code></li></ul>")
        return "<br><hr><br>".join(msgs)

    Name = name
    Fields = fields
    DecodeFlowFunc = decode_flow_func
    ProcessPacket = process_packet
    Query = query
    Snapshot = snapshot
    Reset = reset
    AlerterMsg = alerter_msg


def NewExact(name: str, key_fields: Sequence[str], num_shards: int = 0, **kw) -> ExactTask:  # exact/task.go:83
    return ExactTask(name, key_fields, num_shards, **kw)
