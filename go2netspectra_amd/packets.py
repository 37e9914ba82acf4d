"""Packet batches: the inputs of the sketch hot path.

* PacketBatch -- model.PacketInfo (internal/model/packet.go:9-22) as SoA arrays,
  the batched form of Task.ProcessPacket's argument.  IP addresses are stored
  as the 16-byte slots EncodeFlow writes (task.go:281-286): IPv4 left-aligned
  with 12 zero bytes, IPv6 as-is.
* HeaderBatch -- 64-byte frame records + wire lengths, what the fused-parse
  entry point consumes; read_pcap() builds one from a pcap file
  (pkg/pcap/reader.go:35-49).
* SyntheticTraffic -- the benchmark's Zipf 5-tuple stream,
  generated on the GPU.
"""
from __future__ import annotations

import ctypes as ct
import ipaddress
import os
import struct
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _lib
from ._lib import check


def ip_slot(ip) -> bytes:
    """16-byte EncodeFlow slot of an address (bytes of len 4/16, str or ipaddress)."""
    if isinstance(ip, str):
        ip = ipaddress.ip_address(ip).packed
    elif isinstance(ip, (ipaddress.IPv4Address, ipaddress.IPv6Address)):
        ip = ip.packed
    ip = bytes(ip)[:16]
    return ip + bytes(16 - len(ip))


def ip_version(ip) -> int:
    """4 for a 4-byte net.IP (IPv4 layer), 6 for a 16-byte one."""
    if isinstance(ip, str):
        return ipaddress.ip_address(ip).version
    if isinstance(ip, (ipaddress.IPv4Address, ipaddress.IPv6Address)):
        return ip.version
    return 4 if len(bytes(ip)) == 4 else 6


@dataclass
class PacketBatch:
    src16: "np.ndarray"   # [n,16] uint8
    dst16: "np.ndarray"   # [n,16] uint8
    sport: "np.ndarray"   # [n] uint16
    dport: "np.ndarray"   # [n] uint16
    proto: "np.ndarray"   # [n] uint8
    length: "np.ndarray"  # [n] uint32 (uint32(PacketInfo.Length), task.go:168)
    ipver: Optional["np.ndarray"] = None  # [n] uint8 4/6: len(net.IP) 4 or 16 (exact keys)
    ts: Optional["np.ndarray"] = None     # [n] int64 PacketInfo.Timestamp.UnixNano()

    def __len__(self) -> int:
        return int(self.length.shape[0])

    @classmethod
    def from_packets(cls, packets) -> "PacketBatch":
        """packets: iterable of (src, dst, sport, dport, proto, length[, ts_ns]).  The IP
        version of each packet is that of its source address (net.IP length 4 or 16)."""
        rows = list(packets)
        n = len(rows)
        b = cls(np.zeros((n, 16), np.uint8), np.zeros((n, 16), np.uint8), np.zeros(n, np.uint16),
                np.zeros(n, np.uint16), np.zeros(n, np.uint8), np.zeros(n, np.uint32),
                np.zeros(n, np.uint8), np.zeros(n, np.int64))
        for i, row in enumerate(rows):
            s, d, sp, dp, pr, ln = row[:6]
            b.src16[i] = np.frombuffer(ip_slot(s), np.uint8)
            b.dst16[i] = np.frombuffer(ip_slot(d), np.uint8)
            b.sport[i], b.dport[i], b.proto[i], b.length[i] = sp, dp, pr, ln & 0xFFFFFFFF
            b.ipver[i] = ip_version(s)
            b.ts[i] = row[6] if len(row) > 6 else i
        return b

    def to(self, device):
        """Copy to a torch device (device-resident batches skip the H2D stage)."""
        import torch
        f = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(device)
        return PacketBatch(f(self.src16), f(self.dst16), f(self.sport.view(np.int16)),
                           f(self.dport.view(np.int16)), f(self.proto), f(self.length.view(np.int32)),
                           None if self.ipver is None else f(self.ipver),
                           None if self.ts is None else f(self.ts))

    def c_struct(self):
        arrs = [self.src16, self.dst16, self.sport, self.dport, self.proto, self.length]
        dev = [hasattr(a, "data_ptr") and getattr(a, "is_cuda", False) for a in arrs]
        if all(dev):
            _lib.device_ready(*arrs, self.ipver, self.ts)
            t = _lib.Tuples(*[a.data_ptr() for a in arrs])
            return t, arrs, _lib.MEM_DEVICE
        if any(dev):
            raise ValueError("mix of host and device arrays")
        keep = [np.ascontiguousarray(a) for a in arrs]
        t = _lib.Tuples(*[a.ctypes.data for a in keep])
        return t, keep, _lib.MEM_HOST

    def keys(self, fields) -> np.ndarray:
        """EncodeFlow over the configured fields for every packet -> [n, K] uint8."""
        parts = []
        for f in fields:
            if f == "SrcIP":
                parts.append(np.asarray(self.src16, np.uint8))
            elif f == "DstIP":
                parts.append(np.asarray(self.dst16, np.uint8))
            elif f == "SrcPort":
                parts.append(np.asarray(self.sport, ">u2").view(np.uint8).reshape(-1, 2))
            elif f == "DstPort":
                parts.append(np.asarray(self.dport, ">u2").view(np.uint8).reshape(-1, 2))
            elif f == "Protocol":
                parts.append(np.asarray(self.proto, np.uint8).reshape(-1, 1))
        if not parts:
            return np.zeros((len(self), 0), np.uint8)
        return np.ascontiguousarray(np.concatenate(parts, axis=1))


@dataclass
class HeaderBatch:
    hdr: "np.ndarray"      # [n,64] uint8
    wirelen: "np.ndarray"  # [n] uint32
    ts: Optional["np.ndarray"] = None  # [n] int64 capture timestamps (ns)

    def __len__(self) -> int:
        return int(self.wirelen.shape[0])


def read_pcap(path: str, limit: Optional[int] = None) -> HeaderBatch:
    """pcap or pcapng -> 64-byte records (C++ packer, one pass, no per-packet objects)."""
    L = _lib.load()
    total = ct.c_uint64(0)
    # one pass when the capacity guess holds (records of >= 76 bytes: a 16-byte record
    # header and a 60-byte minimum Ethernet frame); otherwise a second pass at the exact
    # count the first one reported.  The packer writes every byte of a record, so the
    # buffers need no clearing (untouched capacity costs no memory).
    cap = limit if limit is not None else max(1, (os.path.getsize(path) - 24) // 76 + 1)
    while True:
        hdr = np.empty((cap, 64), np.uint8)
        wl = np.empty(cap, np.uint32)
        ts = np.empty(cap, np.int64)
        r = L.gns_pack_pcap_ts(os.fsencode(path), hdr.ctypes.data, wl.ctypes.data, ts.ctypes.data, cap,
                               ct.byref(total))
        if r < 0:
            check(int(r))
        if limit is not None or total.value <= cap:
            return HeaderBatch(hdr[:r], wl[:r], ts[:r])
        cap = total.value


def read_pcap_compact(path: str, limit: Optional[int] = None, rec_len: bool = False):
    """pcap or pcapng -> compact records (rec16 [n, 16], wirelen [n], side [n_side, 64]);
    see include/gns_sketch.h gns_cm_insert_compact.  rec_len: the 16-byte form, the wire
    lengths inside the records (wirelen is then None; GNS_E_RANGE above 65535)."""
    L = _lib.load()
    total, nside = ct.c_uint64(0), ct.c_uint64(0)
    cap = limit if limit is not None else max(1, (os.path.getsize(path) - 24) // 76 + 1)
    side_cap = max(1024, cap // 64)
    while True:
        rec = np.empty((cap, 16), np.uint8)
        wl = None if rec_len else np.empty(cap, np.uint32)
        side = np.empty((side_cap, 64), np.uint8)
        if rec_len:
            r = L.gns_pack_pcap_compact16(os.fsencode(path), rec.ctypes.data, cap, side.ctypes.data, side_cap,
                                          ct.byref(nside), ct.byref(total))
        else:
            r = L.gns_pack_pcap_compact(os.fsencode(path), rec.ctypes.data, wl.ctypes.data, cap, side.ctypes.data,
                                        side_cap, ct.byref(nside), ct.byref(total))
        if r == _lib.GNS_E_RANGE and nside.value > side_cap:
            side_cap = nside.value
            continue
        if r < 0:
            check(int(r))
        if limit is not None or total.value <= cap:
            return rec[:r], (None if wl is None else wl[:r]), side[:nside.value]
        cap = total.value


def compact_headers(hdr, wirelen, rec_len: bool = False):
    """Device-resident 64-byte records (torch uint8 [n, 64] + wire lengths) -> compact
    records on the same device: (rec16 [n, 16] uint8, side [n_side, 64] uint8).
    rec_len: the 16-byte form (wire lengths inside the records)."""
    import torch
    L = _lib.load()
    n = int(wirelen.shape[0])
    _lib.device_ready(hdr, wirelen)
    rec = torch.empty((n, 16), dtype=torch.uint8, device=hdr.device)
    cap = max(1024, n // 256)
    while True:
        side = torch.empty((cap, 64), dtype=torch.uint8, device=hdr.device)
        ns = ct.c_uint64(0)
        fn = L.gns_compact_headers16 if rec_len else L.gns_compact_headers
        r = fn(hdr.data_ptr(), wirelen.data_ptr(), n, rec.data_ptr(), side.data_ptr(), cap, ct.byref(ns),
               hdr.device.index or 0)
        if r == _lib.GNS_E_RANGE and ns.value > cap:
            cap = ns.value
            continue
        check(r)
        return rec, side[:ns.value]


def write_pcap(path: str, frames, wirelens=None, snaplen: int = 65536, ts_ns=None) -> None:
    """Classic little-endian microsecond pcap writer (tests / tools)."""
    import struct
    with open(path, "wb") as f:
        f.write(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, snaplen, 1))
        for i, fr in enumerate(frames):
            fr = bytes(fr)
            wl = len(fr) if wirelens is None else int(wirelens[i])
            sec, usec = (i, 0) if ts_ns is None else divmod(int(ts_ns[i]) // 1000, 1_000_000)
            f.write(struct.pack("<IIII", sec, usec, len(fr), wl))
            f.write(fr)


def write_pcapgen(path: str, n: int, seed: int = 0x5EED0C1, t0_us: int = 1_700_000_000_000_000) -> None:
    """A capture in the format of the reference's generator (scripts/pcapgen/main.go:17-97),
    the input of BASELINE configs[0] (pcap-analyzer, Count-Min d=4 w=65536):
      - classic pcap, pcapgo.NewWriter: microsecond magic, v2.4, snaplen 65536, Ethernet;
      - per packet: Ethernet 00:11:22:33:44:55 -> 00:66:77:88:99:aa, IPv4 (IHL 5, TTL 64,
        protocol TCP, random 4-byte source and destination), TCP SYN with random ports in
        [1024, 65535), random seq/ack, window 14600, then 50..1449 random payload bytes
        (main.go:43-47: rand.Intn(1400) + 50), i.e. frames of 104..1503 bytes;
      - lengths fixed (FixLengths); the IPv4 header checksum is computed, the TCP checksum
        is left 0 (gopacket does not verify checksums when decoding, parser.go never
        reads them);
      - timestamps: t0 + i microseconds (main.go:80 uses time.Now()).
    Written with numpy in one pass (a 1M-packet capture is ~0.8 GB)."""
    rng = np.random.default_rng(seed)
    plen = rng.integers(50, 1450, n).astype(np.int64)
    flen = 54 + plen
    rec = 16 + flen
    offs = 24 + np.concatenate([[0], np.cumsum(rec)[:-1]]).astype(np.int64)
    total = 24 + int(rec.sum())
    buf = np.frombuffer(bytearray(rng.bytes(total)), np.uint8).copy()  # payload bytes random
    buf[:24] = np.frombuffer(struct.pack("<IHHiIII", 0xA1B2C3D4, 2, 4, 0, 0, 65536, 1), np.uint8)
    h = np.zeros((n, 70), np.uint8)
    ts = t0_us + np.arange(n, dtype=np.int64)
    h[:, 0:4] = (ts // 1_000_000).astype("<u4").view(np.uint8).reshape(n, 4)
    h[:, 4:8] = (ts % 1_000_000).astype("<u4").view(np.uint8).reshape(n, 4)
    h[:, 8:12] = flen.astype("<u4").view(np.uint8).reshape(n, 4)
    h[:, 12:16] = h[:, 8:12]
    e = 16
    h[:, e:e + 6] = [0x00, 0x66, 0x77, 0x88, 0x99, 0xAA]
    h[:, e + 6:e + 12] = [0x00, 0x11, 0x22, 0x33, 0x44, 0x55]
    h[:, e + 12:e + 14] = [0x08, 0x00]
    ip = e + 14
    h[:, ip] = 0x45
    h[:, ip + 2:ip + 4] = (flen - 14).astype(">u2").view(np.uint8).reshape(n, 2)
    h[:, ip + 8] = 64
    h[:, ip + 9] = 6
    h[:, ip + 12:ip + 20] = rng.integers(0, 256, (n, 8), dtype=np.uint8)
    words = h[:, ip:ip + 20].astype(np.uint32).reshape(n, 10, 2)
    csum = (words[:, :, 0] << 8 | words[:, :, 1]).sum(axis=1)
    csum = (csum & 0xFFFF) + (csum >> 16)
    csum = (csum & 0xFFFF) + (csum >> 16)
    h[:, ip + 10:ip + 12] = (~csum & 0xFFFF).astype(">u2").view(np.uint8).reshape(n, 2)
    tcp = ip + 20
    ports = rng.integers(1024, 65535, (n, 2)).astype(">u2")
    h[:, tcp:tcp + 4] = ports.view(np.uint8).reshape(n, 4)
    h[:, tcp + 4:tcp + 12] = rng.integers(0, 256, (n, 8), dtype=np.uint8)
    h[:, tcp + 12] = 5 << 4
    h[:, tcp + 13] = 0x02  # SYN
    h[:, tcp + 14:tcp + 16] = [14600 >> 8, 14600 & 0xFF]
    h[:, tcp + 16:tcp + 20] = 0
    idx = offs[:, None] + np.arange(70)[None, :]
    buf[idx] = h
    with open(path, "wb") as f:
        f.write(buf.tobytes())


def write_pcapng(path: str, frames, wirelens=None, ts_units=None, tsresol=None, tsoffset=None,
                  big_endian: bool = False, iface_of=None, n_ifaces: int = 1, snaplen: int = 0,
                  simple: bool = False, sections=None, extra_blocks: bool = False) -> None:
    """pcapng writer (tests / tools): one Section Header, n_ifaces Ethernet Interface
    Description blocks (if_tsresol / if_tsoffset options when given), then one Enhanced
    Packet block per frame (ts_units[i] in the interface's timestamp units; interface
    iface_of[i]), or Simple Packet blocks when `simple`.  `sections`: indices of frames
    before which a new section (with its own interface blocks) starts.  `extra_blocks`
    interleaves blocks a reader must skip (name resolution, statistics, custom)."""
    import struct
    e = ">" if big_endian else "<"

    def block(btype, body):
        body = body + bytes(-len(body) % 4)
        n = 12 + len(body)
        return struct.pack(e + "II", btype, n) + body + struct.pack(e + "I", n)

    def opt(code, val):
        return struct.pack(e + "HH", code, len(val)) + val + bytes(-len(val) % 4)

    def section():
        out = block(0x0A0D0D0A, struct.pack(e + "IHHq", 0x1A2B3C4D, 1, 0, -1))
        for _ in range(n_ifaces):
            opts = b""
            if tsresol is not None:
                opts += opt(9, bytes([tsresol]))
            if tsoffset is not None:
                opts += opt(14, struct.pack(e + "q", tsoffset))
            if opts:
                opts += opt(0, b"")
            out += block(1, struct.pack(e + "HHI", 1, 0, snaplen) + opts)
        return out

    starts = set(sections or ())
    with open(path, "wb") as f:
        f.write(section())
        for i, fr in enumerate(frames):
            if i in starts:
                f.write(section())
            fr = bytes(fr)
            wl = len(fr) if wirelens is None else int(wirelens[i])
            if extra_blocks and i % 7 == 3:
                f.write(block(4, opt(1, b"\x0a\x00\x00\x01host\x00") + opt(0, b"")))  # name resolution
                f.write(block(5, struct.pack(e + "III", 0, 0, 0)))                     # interface statistics
                f.write(block(0x00000BAD, struct.pack(e + "I", 32473) + b"custom"))    # custom block
            if simple:
                f.write(block(3, struct.pack(e + "I", wl) + fr))
            else:
                t = i if ts_units is None else int(ts_units[i])
                ifc = 0 if iface_of is None else int(iface_of[i])
                f.write(block(6, struct.pack(e + "IIIII", ifc, (t >> 32) & 0xFFFFFFFF, t & 0xFFFFFFFF, len(fr), wl)
                              + fr))


class SyntheticTraffic:
    """Zipf 5-tuple header stream generated on the GPU (gns_synth_*).

    shard g of nshards (multi-GPU) is the STABLE FILTER of the
    global stream: exactly the packets whose owner (dist.shard_of of the SrcIP
    slot) is g, in stream order -- what the routing step (dist.route_exchange)
    delivers to GPU g.  It is produced by generating the global stream in chunks
    and keeping shard g's run of the device partition (gns_route_partition);
    fill() continues where the previous call stopped."""

    _CHUNK = 1 << 24

    def __init__(self, flows: int = 1 << 20, zipf_s: float = 1.1, shard: int = 0, nshards: int = 1,
                 device: int = 0, tuple_seed: int = 0x5EED0001, rank_seed: int = 0x5EED0002,
                 len_seed: int = 0x5EED0003, fanout: int = 0):
        """fanout > 0: every packet's DstIP is drawn Zipf(zipf_s) over `fanout`
        destinations (per-source fan-out, the SuperSpread C3 stream)."""
        self._L = _lib.load()
        if not 0 <= shard < max(nshards, 1):
            raise ValueError(f"shard {shard} not in [0, {nshards})")
        p = _lib.SynthParams(flows, zipf_s, tuple_seed, rank_seed, len_seed, 0, 1, device, fanout)
        h = ct.c_void_p()
        check(self._L.gns_synth_create(ct.byref(p), ct.byref(h)))
        self._h = h
        self.device = device
        self.shard, self.nshards = shard, max(nshards, 1)
        nf = ct.c_uint32(0)
        check(self._L.gns_synth_flows(self._h, ct.byref(nf)))
        self.flows = nf.value
        self._router = None
        self._cursor = (0, 0, None)  # (shard packets delivered, global packets consumed, carried run)

    def _fill_global(self, hdr, wirelen, first: int) -> None:
        n = int(wirelen.shape[0])
        check(self._L.gns_synth_fill(self._h, hdr.data_ptr(), wirelen.data_ptr(), first, n))

    def fill(self, hdr, wirelen, first: int = 0) -> None:
        """Fill device tensors hdr[n,64] (uint8) and wirelen[n] (int32/uint32 view)
        with packets first..first+n-1 of this shard's stream."""
        if self.nshards == 1:
            return self._fill_global(hdr, wirelen, first)
        import torch
        from .dist import Router
        if self._router is None:
            self._router = Router(self.nshards, self.device)
        done, gpos, carry = self._cursor
        if first != done:  # not a continuation: restart and skip to `first`
            done, gpos, carry = 0, 0, None
        n = int(wirelen.shape[0])
        skip, got = first - done, 0
        dev = torch.device("cuda", self.device)
        while got < n:
            if carry is None or carry[1].shape[0] == 0:
                m = self._CHUNK
                gh = torch.empty((m, 64), dtype=torch.uint8, device=dev)
                gw = torch.empty((m,), dtype=torch.int32, device=dev)
                self._fill_global(gh, gw, gpos)
                gpos += m
                oh, ow, counts = self._router.partition(gh, gw)
                lo = int(counts[: self.shard].sum())
                c = int(counts[self.shard])
                carry = (oh[lo:lo + c].clone(), ow[lo:lo + c].clone())
                continue
            ch, cw = carry
            if skip:
                t = min(skip, cw.shape[0])
                skip -= t
                carry = (ch[t:], cw[t:])
                continue
            t = min(n - got, cw.shape[0])
            hdr[got:got + t].copy_(ch[:t])
            wirelen[got:got + t].copy_(cw[:t].view(wirelen.dtype))
            got += t
            carry = (ch[t:], cw[t:])
        self._cursor = (first + n, gpos, carry)
        torch.cuda.current_stream(dev).synchronize()  # like gns_synth_fill: complete on return

    def generate(self, n: int, first: int = 0):
        import torch
        dev = torch.device("cuda", self.device)
        hdr = torch.empty((n, 64), dtype=torch.uint8, device=dev)
        wl = torch.empty((n,), dtype=torch.int32, device=dev)
        self.fill(hdr, wl, first)
        return hdr, wl

    def close(self) -> None:
        if getattr(self, "_router", None) is not None:
            self._router.close()
            self._router = None
        if getattr(self, "_h", None):
            self._L.gns_synth_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
