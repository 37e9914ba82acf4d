"""CPU: the C ABI library loads and exports every declared symbol; host-side
mirror of the reference plugin surface (config keys, factory, DecodeFlow,
key encoding, pcap packer, shard routing); the product fails loudly without
a GPU."""
import os
import re
import subprocess

import numpy as np
import pytest

import go2netspectra_amd as g
from go2netspectra_amd import _lib
from go2netspectra_amd.dist import shard_of
from oracle import pyref

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "gns_sketch.h")).read()
    return sorted(set(re.findall(r"\b(gns_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_declared_symbol():
    lib = _lib.LIB_PATH
    assert os.path.exists(lib), "build the library first (__graft_entry__.build())"
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (gns_[a-z0-9_]+)", out))
    missing = [s for s in header_symbols() if s not in exported]
    assert not missing, missing
    assert set(_lib.EXPORTED) <= exported
    L = g.load()  # binds every signature
    assert L.gns_version().startswith(b"gns-sketch")


def test_no_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(g.GnsError) as e:
        g.CountMin(256, 2, key_bytes=16)
    assert "NODEV" in str(e.value)


def test_config_yaml_keys():
    cfg = g.parse_config("""
aggregator:
  types: ["sketch"]
  period: "60s"
  num_workers: 16
  sketch:
    tasks:
      - name: "cm_src_left"
        skt_type: 0
        flow_fields: ["SrcIP"]
        element_fields: ["DstIP", "SrcPort", "DstPort", "Protocol"]
        width: ${GNS_TEST_WIDTH}
        depth: 2
        size_thereshold: 4096000
        count_thereshold: 4096
      - name: "ss_src_dst"
        skt_type: 1
        flow_fields: ["SrcIP"]
        element_fields: ["DstIP"]
        width: 32768
        depth: 2
        count_thereshold: 1
        m : 128
        size: 5
        b: 1.08
        base: 0.5
""".replace("${GNS_TEST_WIDTH}", "32768"))
    t0, t1 = cfg.Aggregator.Sketch.Tasks
    assert (t0.Name, t0.SketchType, t0.Width, t0.Depth, t0.SizeThreshold, t0.CountThreshold) == \
        ("cm_src_left", 0, 32768, 2, 4096000, 4096)
    assert (t1.SketchType, t1.M, t1.Size, t1.B, t1.Base, t1.CountThreshold) == (1, 128, 5, 1.08, 0.5, 1)
    assert cfg.Aggregator.Types == ["sketch"] and cfg.Aggregator.NumWorkers == 16


def test_config_env_expansion(monkeypatch):
    monkeypatch.setenv("GNS_W", "4096")
    cfg = g.parse_config("aggregator:\n  types: [sketch]\n  sketch:\n    tasks:\n      - name: x\n        width: ${GNS_W}\n")
    assert cfg.Aggregator.Sketch.Tasks[0].Width == 4096


def test_factory_registry():
    with pytest.raises(RuntimeError):  # task_factory.go:25-27 panics on duplicates
        g.register_aggregator("sketch", lambda cfg: None)
    cfg = g.parse_config("aggregator:\n  types: [nosuch]\n")
    with pytest.raises(KeyError):
        g.create(cfg)


def test_decode_flow_matches_go_formatting():
    from go2netspectra_amd.packets import ip_slot
    # an IPv4 key is 4 bytes + 12 zero bytes: Go's net.IP(16 bytes).String() prints it as IPv6
    flow = ip_slot(bytes([192, 0, 2, 1])) + bytes([0x30, 0x39, 0x01, 0xbb, 6])
    assert g.decode_flow(flow, ["SrcIP", "SrcPort", "DstPort", "Protocol"]) == "c000:201:: 12345 443 6"
    mapped = bytes(10) + b"\xff\xff" + bytes([10, 1, 2, 3])
    assert g.decode_flow(mapped, ["DstIP"]) == "10.1.2.3"
    v6 = bytes.fromhex("20010db8000000000000000000000001")
    assert g.decode_flow(v6, ["SrcIP"]) == "2001:db8::1"


def test_packet_batch_keys_match_reference_encoding():
    rng = np.random.default_rng(0)
    from helpers import random_tuples
    t = random_tuples(rng, 200, 50, v6_frac=0.3)
    b = g.PacketBatch(t["src16"], t["dst16"], t["sport"], t["dport"], t["proto"], t["length"])
    for fields in (["SrcIP"], ["SrcIP", "DstIP", "SrcPort", "DstPort", "Protocol"], ["DstPort", "SrcIP"]):
        keys = b.keys(fields)
        for i in range(0, 200, 17):
            want = pyref.encode_key(fields, bytes(t["src16"][i]), bytes(t["dst16"][i]), int(t["sport"][i]),
                                    int(t["dport"][i]), int(t["proto"][i]))
            assert bytes(keys[i]) == want


def test_pcap_packer_roundtrip(tmp_path):
    from helpers import frame64
    rng = np.random.default_rng(2)
    frames, wl = [], []
    for i in range(300):
        ln = int(rng.integers(60, 1500))
        full = frame64(rng.integers(0, 256, 16, dtype=np.uint8), rng.integers(0, 256, 16, dtype=np.uint8),
                       int(rng.integers(0, 65536)), int(rng.integers(0, 65536)), 6, ln) + bytes(max(0, ln - 64))
        cap = full[: int(rng.integers(40, len(full) + 1))]  # snaplen truncation
        frames.append(cap)
        wl.append(ln)
    path = str(tmp_path / "t.pcap")
    g.write_pcap(path, frames, wl)
    _check_records(g.read_pcap(path), frames, wl)


def _random_frames(rng, n):
    from helpers import frame64
    frames, wl = [], []
    for i in range(n):
        ln = int(rng.integers(60, 1500))
        full = frame64(rng.integers(0, 256, 16, dtype=np.uint8), rng.integers(0, 256, 16, dtype=np.uint8),
                       int(rng.integers(0, 65536)), int(rng.integers(0, 65536)), 6, ln) + bytes(max(0, ln - 64))
        frames.append(full[: int(rng.integers(1, len(full) + 1))])  # snaplen truncation, down to 1 byte
        wl.append(ln)
    return frames, wl


def _check_records(hb, frames, wl):
    """fast-shape frames verbatim (first 64 bytes, zero padded), all others as the
    host decode's 0x88B5 / drop records (gns_frame.cpp; oracle/pyframe.py restates it)"""
    from oracle import pyframe
    assert len(hb) == len(frames)
    for i, fr in enumerate(frames):
        assert bytes(hb.hdr[i]) == pyframe.frame_record(fr, wl[i])
        assert hb.wirelen[i] == wl[i]


@pytest.mark.parametrize("big_endian", [False, True])
@pytest.mark.parametrize("tsresol,tsoffset", [(None, None), (9, None), (3, 7), (0x94, -3), (12, 1_700_000_000)])
def test_pcapng_enhanced_packets(tmp_path, big_endian, tsresol, tsoffset):
    """pcapng as libpcap reads it (gopacket pcap.OpenOffline, reader.go:21): records and wire
    lengths as in classic pcap; timestamps in the interface's if_tsresol units (10^-r, or
    2^-r with the top bit set; default microseconds) plus if_tsoffset seconds, scaled to ns."""
    rng = np.random.default_rng(5)
    frames, wl = _random_frames(rng, 200)
    units = (10 ** 6 if tsresol is None else (2 ** (tsresol & 0x7F) if tsresol & 0x80 else 10 ** tsresol))
    ts_units = rng.integers(0, 2 ** 62, len(frames), dtype=np.uint64)
    ts_units[:3] = [0, units - 1, units]
    path = str(tmp_path / "t.pcapng")
    g.write_pcapng(path, frames, wl, ts_units=ts_units, tsresol=tsresol, tsoffset=tsoffset, big_endian=big_endian,
                   extra_blocks=True)
    hb = g.read_pcap(path)
    _check_records(hb, frames, wl)
    off = tsoffset or 0
    want = [((int(t) // units + off) * 10 ** 9 + (int(t) % units) * 10 ** 9 // units) for t in ts_units]
    want = np.array([(w + 2 ** 63) % 2 ** 64 - 2 ** 63 for w in want], np.int64)  # the engine's int64 ns
    assert np.array_equal(hb.ts, want)


def test_pcapng_interfaces_sections_and_simple_packets(tmp_path):
    rng = np.random.default_rng(6)
    frames, wl = _random_frames(rng, 120)
    p1 = str(tmp_path / "multi.pcapng")  # three interfaces, a second section half way
    g.write_pcapng(p1, frames, wl, iface_of=rng.integers(0, 3, len(frames)), n_ifaces=3, sections=[60])
    _check_records(g.read_pcap(p1), frames, wl)
    p2 = str(tmp_path / "simple.pcapng")  # Simple Packet blocks: captured = min(wire length, snaplen)
    full = [fr + bytes(w - len(fr)) for fr, w in zip(frames, wl)]
    g.write_pcapng(p2, [f[:48] for f in full], wl, simple=True, snaplen=48)
    hb = g.read_pcap(p2)
    _check_records(hb, [f[:48] for f in full], wl)
    assert not hb.ts.any()
    assert len(g.read_pcap(p2, limit=10)) == 10


def test_pcapng_rejects_what_libpcap_rejects(tmp_path):
    import struct
    from go2netspectra_amd._lib import GnsError
    rng = np.random.default_rng(7)
    frames, wl = _random_frames(rng, 10)
    p = str(tmp_path / "badif.pcapng")  # a packet on an interface with no description block
    g.write_pcapng(p, frames, wl, iface_of=[0] * 9 + [1])
    with pytest.raises(GnsError, match="interface 1"):
        g.read_pcap(p)
    p = str(tmp_path / "raw.pcapng")  # non-Ethernet link type (101 = raw IP)
    g.write_pcapng(p, frames, wl)
    data = bytearray(open(p, "rb").read())
    shb_len = struct.unpack_from("<I", data, 4)[0]
    struct.pack_into("<H", data, shb_len + 8, 101)
    open(p, "wb").write(bytes(data))
    with pytest.raises(GnsError, match="linktype 101"):
        g.read_pcap(p)
    p = str(tmp_path / "trunc.pcapng")  # a truncated last block ends the capture
    g.write_pcapng(p, frames, wl)
    data = open(p, "rb").read()
    open(p, "wb").write(data[:-10])
    _check_records(g.read_pcap(p), frames[:9], wl[:9])


def test_shard_of_is_mm3_of_src_slot(oracle):
    rng = np.random.default_rng(4)
    src = rng.integers(0, 256, (500, 16), dtype=np.uint8)
    sh = shard_of(src, 8)
    for i in range(0, 500, 7):
        assert sh[i] == oracle.mm3(bytes(src[i]), 0xA5A5A5A5) % 8


def test_merge_heavy_arrays_canonical_order():
    """The array-form union (bench per-window exchange) orders like merge_heavy: value
    desc, then full key bytes asc, also for ties beyond the first four key bytes."""
    from go2netspectra_amd.dist import merge_heavy, merge_heavy_arrays
    rng = np.random.default_rng(3)
    for K in (2, 4, 16, 37):
        n = 4000
        f = rng.integers(0, 256, (n, K), dtype=np.uint8)
        f[:, : min(K, 4)] = rng.integers(0, 2, (n, min(K, 4)))  # long runs tied on the first bytes
        f = np.unique(f, axis=0)
        v = rng.integers(0, 4, len(f)).astype(np.uint32)
        perm = rng.permutation(len(f))
        gf, gv = merge_heavy_arrays(f[perm], v[perm])
        want = merge_heavy([[(bytes(f[i]), int(v[i])) for i in range(len(f))]])
        assert [(bytes(a), int(b)) for a, b in zip(gf, gv)] == want
    e = merge_heavy_arrays(np.zeros((0, 8), np.uint8), np.zeros(0, np.uint32))
    assert len(e[0]) == 0 and len(e[1]) == 0


def test_pcapgen_capture_format(tmp_path):
    """configs[0]'s input, scripts/pcapgen/main.go:17-97: TCP SYN over IPv4, frames of
    104..1503 bytes, ports in [1024, 65535), read back by the packer; every record is in
    the device parser's fast subset and parses to the written tuple."""
    import struct
    import go2netspectra_amd as g
    from oracle import oracle as orc
    path = str(tmp_path / "pg.pcap")
    g.write_pcapgen(path, 20_000, seed=3)
    raw = open(path, "rb").read()
    assert struct.unpack("<IHHiIII", raw[:24]) == (0xA1B2C3D4, 2, 4, 0, 0, 65536, 1)
    hb = g.read_pcap(path)
    assert len(hb) == 20_000
    assert hb.wirelen.min() >= 104 and hb.wirelen.max() <= 1503
    h = hb.hdr
    assert (h[:, 12] == 8).all() and (h[:, 13] == 0).all() and (h[:, 14] == 0x45).all() and (h[:, 23] == 6).all()
    assert (h[:, 47] == 0x02).all()  # SYN
    sport = h[:, 34].astype(int) << 8 | h[:, 35]
    assert sport.min() >= 1024 and sport.max() < 65535
    assert (hb.ts[1:] - hb.ts[:-1] == 1000).all()  # microsecond steps, ns timestamps
    for i in range(0, 20_000, 997):
        st, s16, d16, sp, dp, pr = orc.parse_hdr64(bytes(h[i]), int(hb.wirelen[i]))
        assert st == 0 and s16[:4] == bytes(h[i, 26:30]) and sp == sport[i] and pr == 6


def test_compact_packer_equals_the_parsed_records(tmp_path):
    """gns_pack_pcap_compact: every compact record is the tuple the device parser reads
    from the 64-byte record gns_pack_pcap writes for the same frame (the C oracle's
    parse of that record), the drop class for frames without an IP layer, or an
    escape naming that exact 64-byte record in the side array."""
    from oracle import oracle as orc
    from test_configs_gpu import _encap_flows
    rng = np.random.default_rng(5)
    flows = _encap_flows(rng, 800)
    frames, wl = _random_frames(rng, 400)  # plain IPv4/TCP, truncated captures included
    frames += [f for f, _ in flows]
    wl += [w for _, w in flows]
    frames += frames[:50]
    wl += wl[:50]
    path = str(tmp_path / "c.pcap")
    g.write_pcap(path, frames, wl)
    hb = g.read_pcap(path)
    rec, cwl, side = g.read_pcap_compact(path)
    assert len(rec) == len(hb) == len(frames) and np.array_equal(cwl, hb.wirelen)
    seen = {0: 0, 1: 0, 2: 0}
    for j in range(len(rec)):
        cls = int(rec[j, 13])
        seen[cls] += 1
        st, src, dst, sp, dp, pr = orc.parse_hdr64(bytes(hb.hdr[j]), int(cwl[j]))
        if cls == 0:
            assert st == 0, j
            assert src[4:] == bytes(12) and dst[4:] == bytes(12)
            assert bytes(rec[j, 0:4]) == src[:4] and bytes(rec[j, 4:8]) == dst[:4]
            assert bytes(rec[j, 8:12]) == bytes([sp >> 8, sp & 255, dp >> 8, dp & 255]) and rec[j, 12] == pr
        elif cls == 1:
            assert st == 1, j  # PARSE_DROP
        else:
            assert cls == 2
            k = int(rec[j, 0:4].view("<u4")[0])
            assert bytes(side[k]) == bytes(hb.hdr[j])
    assert seen[0] > 0 and seen[1] > 0 and seen[2] > 0, seen


def test_compact16_packer_carries_wire_lengths(tmp_path):
    """gns_pack_pcap_compact16: the 20-byte form's records with the wire length in word 3
    bits 16..31; a class-0 record is an IPv4 tuple both ways (the 20-byte form's other
    narrow tuples, e.g. host-decoded IPv6 with zero upper slot bytes, escape to the side
    array here), every escape names its exact 64-byte record, and a frame whose wire
    length exceeds 65535 makes the call fail (the 20-byte form then holds it)."""
    from test_configs_gpu import _encap_flows
    rng = np.random.default_rng(6)
    flows = _encap_flows(rng, 600)
    frames, wl = _random_frames(rng, 300)
    frames += [f for f, _ in flows]
    wl += [w for _, w in flows]
    path = str(tmp_path / "c16.pcap")
    g.write_pcap(path, frames, wl)
    hb = g.read_pcap(path)
    rec, cwl, side = g.read_pcap_compact(path)
    rec16, none16, side16 = g.read_pcap_compact(path, rec_len=True)
    assert none16 is None and len(rec16) == len(rec)
    w3 = np.ascontiguousarray(rec16[:, 12:16]).view("<u4").reshape(-1)
    assert np.array_equal(w3 >> 16, cwl)
    for j in range(len(rec)):
        c20, c16 = int(rec[j, 13]), int(rec16[j, 13])
        v4 = c20 == 0 and rec[j, 14] == 4 and rec[j, 15] == 4
        if v4 or c20 == 1:
            assert c16 == c20 and bytes(rec16[j, :13]) == bytes(rec[j, :13]), j
        else:
            assert c16 == 2, j
            k = int(rec16[j, 0:4].view("<u4")[0])
            assert bytes(side16[k]) == bytes(hb.hdr[j])
    big = str(tmp_path / "big.pcap")
    g.write_pcap(big, frames[:10], [70_000] + wl[1:10], snaplen=262144)
    with pytest.raises(g.GnsError):
        g.read_pcap_compact(big, rec_len=True)
    r2, w2, _ = g.read_pcap_compact(big)
    assert w2[0] == 70_000


@pytest.mark.parametrize("cut", [0, 37, 9])
def test_parallel_record_walk_equals_sequential(tmp_path, monkeypatch, cut):
    """Classic captures are walked in pieces on several threads (gns_pcap.cpp classic());
    the records, their order, the wire lengths and the timestamps equal the single-thread
    walk's, also with a truncated trailer (cut bytes off the end: inside a record's data or
    inside its header), and over several windows of the file -- the pieces are used only when
    every walk lands on its successor's start."""
    path = str(tmp_path / "walk.pcap")
    g.write_pcapgen(path, 6000, seed=11)
    if cut:
        with open(path, "r+b") as f:
            f.truncate(os.path.getsize(path) - cut)
    monkeypatch.setenv("GNS_PACK_PAR_MIN", "0")
    out = {}
    for t, win in ((1, None), (3, None), (8, None), (8, 1 << 20), (3, 300_000)):
        monkeypatch.setenv("GNS_PACK_THREADS", str(t))
        if win:  # several windows, each cut into pieces
            monkeypatch.setenv("GNS_PACK_WINDOW", str(win))
        hb = g.read_pcap(path)
        rec, wl, side = g.read_pcap_compact(path)
        rec16, _, side16 = g.read_pcap_compact(path, rec_len=True)
        ts = hb.ts if hb.ts is not None else np.zeros(0)
        lim = g.read_pcap(path, limit=2500)  # a cap inside a piece
        rl, wll, sl = g.read_pcap_compact(path, limit=2500)
        out[t, win] = (hb.hdr.copy(), hb.wirelen.copy(), ts.copy(), rec, wl, side, rec16, side16,
                       lim.hdr.copy(), lim.wirelen.copy(), rl, wll, sl)
    ref = out[1, None]
    assert len(ref[0]) == 6000 - (1 if cut else 0) and len(ref[8]) == 2500
    for key, got in out.items():
        for a, b in zip(ref, got):
            assert np.array_equal(a, b), key


def test_timing_arg_encodes_stage_masks():
    """gns_*_set_timing's argument (include/gns_sketch.h GNS_TIMING_MASK)."""
    from go2netspectra_amd import _lib
    names = ["extract", "resolve", "scan", "scatter", "apply", "insert", "hot", "designate"]
    assert _lib.timing_arg(False, None, names) == 0
    assert _lib.timing_arg(True, None, names) == 1
    assert _lib.timing_arg(True, ["extract"], names) == _lib.GNS_TIMING_MASK | 1
    assert _lib.timing_arg(True, ["extract", "scatter", "apply", "insert"], names) == 0x139
    with pytest.raises(ValueError):
        _lib.timing_arg(True, ["nope"], names)
