"""Thrift live path: PacketInfo messages (api/thrift/v1/traffic.thrift) as sent
over NATS by the probe (internal/probe/publisher.go:66) and decoded by the
engine (internal/engine/streamaggregator/stream_aggregator.go:84-90).

* marshal_packet_info -- MarshalPacketInfo (packetcodec.go:54-73): Thrift
  binary protocol, fields in id order, the IPs' net.IP bytes as given.
* decode_messages -- UnmarshalPacketInfo for a whole batch on the GPU
  (gns_thrift_decode): messages back to back + offsets -> device-resident
  HeaderBatch of pre-parsed records that every engine's insert_headers takes.
  Rejected messages become records the parser drops (the reference logs and
  drops them).
"""
from __future__ import annotations

import ctypes as ct
import ipaddress
import struct
from typing import Iterable, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import check
from .packets import HeaderBatch


def _ip_bytes(ip) -> bytes:
    if isinstance(ip, str):
        return ipaddress.ip_address(ip).packed
    if isinstance(ip, (ipaddress.IPv4Address, ipaddress.IPv6Address)):
        return ip.packed
    return bytes(ip)


def marshal_packet_info(ts_ns: int, src, dst, sport: int, dport: int, proto: int, length: int) -> bytes:
    """TBinaryProtocol encoding of PacketInfo{ts, FiveTuple{src, dst, ports, proto}, length}."""
    s, d = _ip_bytes(src), _ip_bytes(dst)
    ft = (b"\x0b\x00\x01" + struct.pack(">i", len(s)) + s +
          b"\x0b\x00\x02" + struct.pack(">i", len(d)) + d +
          b"\x08\x00\x03" + struct.pack(">i", sport) +
          b"\x08\x00\x04" + struct.pack(">i", dport) +
          b"\x08\x00\x05" + struct.pack(">i", proto) + b"\x00")
    return (b"\x0a\x00\x01" + struct.pack(">q", ts_ns) + b"\x0c\x00\x02" + ft +
            b"\x0a\x00\x03" + struct.pack(">q", length) + b"\x00")


def pack_messages(msgs: Iterable[bytes]) -> Tuple[bytes, np.ndarray]:
    """NATS payloads back to back + offsets[n+1] (the batch the engine decodes)."""
    msgs = [bytes(m) for m in msgs]
    offs = np.zeros(len(msgs) + 1, np.uint64)
    if msgs:
        offs[1:] = np.cumsum([len(m) for m in msgs])
    return b"".join(msgs), offs


def decode_messages(buf, offsets, device: int = 0):
    """-> (HeaderBatch with device tensors hdr [n,64] / wirelen [n] / ts [n], rejected count)."""
    import torch
    L = _lib.load()
    offsets = np.ascontiguousarray(offsets, np.uint64)
    n = len(offsets) - 1
    dev = torch.device("cuda", device)
    hdr = torch.empty((max(n, 1), 64), dtype=torch.uint8, device=dev)
    wl = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    ts = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    bad = ct.c_uint64(0)
    if isinstance(buf, (bytes, bytearray, memoryview)):
        b = np.frombuffer(bytes(buf) or b"\0", np.uint8)
        bp, nb = b.ctypes.data, len(buf)
    else:
        b = np.ascontiguousarray(buf, np.uint8)
        bp, nb = b.ctypes.data, b.nbytes
    check(L.gns_thrift_decode(bp, nb, offsets.ctypes.data, n, hdr.data_ptr(), wl.data_ptr(), ts.data_ptr(),
                              ct.byref(bad), _lib.MEM_HOST, device))
    return HeaderBatch(hdr[:n], wl[:n], ts[:n]), int(bad.value)


def unmarshal_batch(msgs: Sequence[bytes], device: int = 0):
    return decode_messages(*pack_messages(msgs), device=device)
