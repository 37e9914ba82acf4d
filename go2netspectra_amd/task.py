"""sketch.Task mirror: the aggregator plugin the Manager drives.

Reference: internal/engine/impl/sketch/task.go (New :106-138, ProcessPacket
:156-169, Query :172, Snapshot :177, Reset :182, AlerterMsg :187-243, EncodeFlow
:279-300, DecodeFlow :303-325, fieldByteSize :327-338) behind model.Task
(internal/model/task.go:6-15).

GPU-first differences, by design:
  * process_packets(batch) is the hot entry point: one call per packet batch
    instead of one per packet from N worker goroutines.  process_packet(info)
    is kept for API parity and forwards a batch of one.
  * Row seeds (and SuperSpread's HLL seeds / RNG key) are injected so results
    are reproducible; the reference draws them from unseedable global RNGs.
"""
from __future__ import annotations

import ipaddress
import logging
import struct
from typing import List, Optional, Sequence

import numpy as np

from .config import SketchTaskDef
from .packets import HeaderBatch, PacketBatch
from .sketch import CountMin, HeavyRecord, SuperSpread

log = logging.getLogger("go2netspectra_amd")

FIELD_SIZE = {"SrcIP": 16, "DstIP": 16, "SrcPort": 2, "DstPort": 2, "Protocol": 1}


def field_byte_size(f: str) -> int:  # task.go:327-338
    return FIELD_SIZE.get(f, 0)


def go_ip_string(b: bytes) -> str:
    """net.IP(b).String() for a 16-byte slot (Go prints IPv4-mapped as dotted quad)."""
    b = bytes(b)
    if len(b) == 16 and b[:10] == bytes(10) and b[10:12] == b"\xff\xff":
        return str(ipaddress.IPv4Address(b[12:]))
    if len(b) == 4:
        return str(ipaddress.IPv4Address(b))
    return ipaddress.IPv6Address(b).compressed


def decode_flow(flow: bytes, fields: Sequence[str]) -> str:
    """DecodeFlow (task.go:303-325)."""
    parts, off = [], 0
    for f in fields:
        if f in ("SrcIP", "DstIP"):
            parts.append(go_ip_string(flow[off:off + 16]))
            off += 16
        elif f in ("SrcPort", "DstPort"):
            parts.append(str(struct.unpack(">H", flow[off:off + 2])[0]))
            off += 2
        elif f == "Protocol":
            parts.append(str(flow[off]))
            off += 1
    return " ".join(parts)


def _check(value: float, threshold: float, op: str) -> bool:  # task.go:246-262
    if op == ">":
        return value > threshold
    if op == "<":
        return value < threshold
    if op == "=":
        return value == threshold
    if op == ">=":
        return value >= threshold
    if op == "<=":
        return value <= threshold
    log.warning("unknown operator '%s' in alerter rule", op)
    return False


class SketchTask:
    """model.Task implementation for skt_type 0 (CountMin) and 1 (SuperSpread)."""

    def __init__(self, cfg: SketchTaskDef, device: int = 0, seeds=None, max_flows: int = 0,
                 batch_packets: int = 0, hll_master: Optional[int] = None,
                 rng_seed: Optional[int] = None):
        self.name_ = cfg.Name
        self.flow_fields = list(cfg.FlowFields)
        self.element_fields = list(cfg.ElementFields)
        self.flow_size = sum(field_byte_size(f) for f in self.flow_fields)
        self.elem_size = sum(field_byte_size(f) for f in self.element_fields)
        if cfg.SketchType == 0:
            self.sketch = CountMin(cfg.Width, cfg.Depth, cfg.SizeThreshold, cfg.CountThreshold,
                                   flow_fields=self.flow_fields, seeds=seeds, max_flows=max_flows,
                                   batch_packets=batch_packets, device=device)
        elif cfg.SketchType == 1:
            kw = {}
            if hll_master is not None:
                kw["hll_master"] = hll_master
            if rng_seed is not None:
                kw["rng_seed"] = rng_seed
            self.sketch = SuperSpread(cfg.Width, cfg.Depth, cfg.CountThreshold, cfg.M, cfg.Size, cfg.Base,
                                      cfg.B, flow_fields=self.flow_fields, elem_fields=self.element_fields,
                                      seeds=seeds, batch_packets=batch_packets, device=device, **kw)
        else:  # task.go:126-127 log.Fatalf
            raise ValueError(f"Unknown sketch type: {cfg.SketchType} for task {cfg.Name}")

    # --- model.Task ---
    def name(self) -> str:
        return self.name_

    def fields(self) -> List[str]:
        return self.flow_fields

    def decode_flow(self, flow: bytes, fields: Sequence[str]) -> str:
        return decode_flow(flow, fields)

    def decode_flow_func(self):
        return self.decode_flow

    def process_packets(self, batch) -> None:
        """Batched ProcessPacket: PacketBatch or HeaderBatch (or device equivalents)."""
        if isinstance(batch, HeaderBatch):
            self.sketch.insert_headers(batch.hdr, batch.wirelen)
        else:
            self.sketch.insert_tuples(batch)

    def process_packet(self, info) -> None:
        """ProcessPacket(*PacketInfo); info = (src, dst, sport, dport, proto, length)."""
        self.process_packets(PacketBatch.from_packets([info]))

    def query(self, flow: bytes) -> int:
        return self.sketch.query(flow)

    def snapshot(self) -> HeavyRecord:
        return self.sketch.heavy_hitters()

    def reset(self) -> None:
        self.sketch.reset()

    def flush(self) -> None:
        self.sketch.flush()

    def alerter_msg(self, rules) -> str:
        """AlerterMsg (task.go:187-243); rules: dicts with task_name/metric/operator/threshold/name."""
        snap = self.snapshot()
        msgs = []
        for rule in rules:
            if rule.get("task_name") != self.name_:
                continue
            metric, op, thr = rule.get("metric"), rule.get("operator", ">"), float(rule.get("threshold", 0))
            hitters = []
            if metric == "heavy_hitter_count":
                for h in snap.Count:
                    if _check(float(h.Count), thr, op):
                        hitters.append(f"<tr><td><code>{decode_flow(h.Flow, self.flow_fields)}</code></td><td>{h.Count}</td></tr>")
            elif metric == "heavy_hitter_size":
                for h in snap.Size or []:
                    if _check(float(h.Size), thr, op):
                        hitters.append(f"<tr><td><code>{decode_flow(h.Flow, self.flow_fields)}</code></td><td>{h.Size} bytes</td></tr>")
            elif metric == "super_spreader_spread" and snap.Size is None:
                for h in snap.Count:
                    if _check(float(h.Count), thr, op):
                        hitters.append(f"<tr><td><code>{decode_flow(h.Flow, self.flow_fields)}</code></td><td>{h.Count}</td></tr>")
            if hitters:
                table = ("<table border=\"1\" cellpadding=\"5\" cellspacing=\"0\">"
                         "<tr><th>Flow/Source</th><th>Value</th></tr>" + "".join(hitters) + "</table>")
                msgs.append(f"<h3>Alert: {rule.get('name', '')}</h3><ul><li><b>Task:</b> <code>{rule.get('task_name')}</code></li>"
                            f"<li><b>Metric:</b> <code>{metric}</code></li><li><b>Condition:</b> <code>{op} {thr:.2f}</code></li>"
                            f"</ul><p><b>Triggering Items:</b></p>{table}")
        return "<br><hr><br>".join(msgs)

    # Go-style names
    Name = name
    Fields = fields
    DecodeFlow = decode_flow
    DecodeFlowFunc = decode_flow_func
    ProcessPacket = process_packet
    Query = query
    Snapshot = snapshot
    Reset = reset
    AlerterMsg = alerter_msg


def New(cfg: SketchTaskDef, **kw) -> SketchTask:  # task.go:106
    return SketchTask(cfg, **kw)
