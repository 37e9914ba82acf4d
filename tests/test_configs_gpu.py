"""BASELINE configs checked against the oracle on the GPU, at the kernels and
launch shapes the benchmarks time (verdict r2 #1):
  configs[4]: 5-tuple header records at d=8 w=2^24 through insert_headers (the
              1024-thread K1 instantiation k_extract<IN_HDR, ., 37, 0, 1024>),
              and the hybrid bench's concurrent exact + Count-Min ingest on two
              host threads / two streams (bench.py bench_hybrid).
"""
import threading

import numpy as np
import pytest

from helpers import assert_same_flows, assert_same_list

pytestmark = pytest.mark.gpu

FIVE = ["SrcIP", "DstIP", "SrcPort", "DstPort", "Protocol"]


def _same_state(cm, orc):
    C, S, Fc, Fs = cm.export_state()
    oC, oS, oFc, oFs = orc.export()
    for name, a, b in (("C", C, oC), ("S", S, oS), ("FPc", Fc, oFc), ("FPs", Fs, oFs)):
        if not np.array_equal(a, b):
            bad = np.flatnonzero(a != b) if a.ndim == 1 else np.flatnonzero((a != b).any(axis=1))
            raise AssertionError(f"{name} differs in {len(bad)} cells, first {bad[:5]}")


def test_c5_geometry_header_records(gpu, oracle):
    """configs[4] geometry (d=8, w=2^24) on device-resident 5-tuple header records,
    2M Zipf packets in two calls: full state, queries and both heavy-hitter lists."""
    import torch
    from go2netspectra_amd import CountMin, SyntheticTraffic
    n = 2_000_000
    hdr, wl = SyntheticTraffic().generate(n)
    seeds = np.random.default_rng(55).integers(0, 2**32, 8, dtype=np.uint64).astype(np.uint32)
    cm = CountMin(1 << 24, 8, 1 << 18, 200, flow_fields=FIVE, seeds=seeds, max_flows=1 << 21)
    cm.insert_headers(hdr[: n // 2], wl[: n // 2])
    cm.insert_headers(hdr[n // 2:], wl[n // 2:])
    cm.flush()
    torch.cuda.synchronize()
    orc = oracle.CountMin(1 << 24, 8, 1 << 18, 200, 37, seeds)
    h, w = hdr.cpu().numpy(), wl.cpu().numpy().view(np.uint32)
    assert orc.insert_hdr64(h, w, FIVE) == n
    _same_state(cm, orc)
    hh = cm.heavy_hitters()
    assert_same_list([(x.Flow, x.Count) for x in hh.Count], orc.heavy("count"))
    assert_same_list([(x.Flow, x.Size) for x in hh.Size], orc.heavy("size"))
    keys = np.zeros((4096, 37), np.uint8)
    keys[:, 0:4], keys[:, 16:20], keys[:, 32:36], keys[:, 36] = h[:4096, 26:30], h[:4096, 30:34], h[:4096, 34:38], h[:4096, 23]
    assert np.array_equal(cm.query_many(keys), np.array([orc.query(bytes(k)) for k in keys], np.uint64))
    del orc


def test_hybrid_concurrent_exact_and_countmin(gpu, oracle):
    """bench_hybrid's ingest: per window the exact aggregator runs on its own host
    thread / stream while the Count-Min handle ingests the same records from the
    main thread; a snapshot view answers heavy hitters after each window.  Both
    engines must equal their sequential oracles."""
    import torch
    from go2netspectra_amd import CountMin, ExactTask, HeaderBatch, SyntheticTraffic
    n, windows = 600_000, 3
    syn = SyntheticTraffic()
    seeds = np.random.default_rng(66).integers(0, 2**32, 8, dtype=np.uint64).astype(np.uint32)
    ex = ExactTask("per_five_tuple", FIVE, 128, max_flows=1 << 21, batch_packets=n)
    cm = CountMin(1 << 22, 8, 1 << 18, 200, flow_fields=FIVE, seeds=seeds, max_flows=1 << 21, batch_packets=n)
    view = cm.view()
    o_cm = oracle.CountMin(1 << 22, 8, 1 << 18, 200, 37, seeds)
    o_ex = oracle.Exact(FIVE)
    for k in range(windows):
        hdr, wl = syn.generate(n, first=k * n)
        ts = torch.arange(n, dtype=torch.int64, device="cuda") * 100 + k * n * 100 + 1_700_000_000_000_000_000
        errs = []

        def ex_step():
            try:
                ex.process_packets(HeaderBatch(hdr, wl, ts))
                ex.flush()
            except Exception as e:  # pragma: no cover - reported below
                errs.append(e)

        te = threading.Thread(target=ex_step)
        te.start()
        cm.insert_headers(hdr, wl)
        te.join()
        assert not errs, errs
        view.refresh()
        h, w = hdr.cpu().numpy(), wl.cpu().numpy().view(np.uint32)
        o_cm.insert_hdr64(h, w, FIVE)
        o_ex.insert_hdr64(h, w, ts.cpu().numpy())
        hh = view.heavy_hitters()
        assert_same_list([(x.Flow, x.Count) for x in hh.Count], o_cm.heavy("count"))
        assert_same_list([(x.Flow, x.Size) for x in hh.Size], o_cm.heavy("size"))
    cm.flush()
    _same_state(cm, o_cm)
    got = {f.Key: (f.StartTime, f.EndTime, f.PacketCount, f.ByteCount) for f in ex.flows()}
    assert_same_flows(got, o_ex.export())
    view.close()


def test_c1_pcapgen_capture(gpu, oracle, tmp_path):
    """configs[0]: a 1M-packet capture in the reference generator's format
    (scripts/pcapgen/main.go: TCP SYN, uniform IPs / ports, 104..1503-byte frames),
    read by the host packer (pkg/pcap/reader.go:35-49) and inserted from host
    memory into Count-Min d=4 w=65536 (cmd/pcap-analyzer): full state and both
    heavy-hitter lists equal the oracle fed the same records."""
    from go2netspectra_amd import CountMin, read_pcap, write_pcapgen
    path = str(tmp_path / "c1.pcap")
    write_pcapgen(path, 1_000_000)
    hb = read_pcap(path)
    assert len(hb) == 1_000_000
    seeds = np.random.default_rng(1).integers(0, 2**32, 4, dtype=np.uint64).astype(np.uint32)
    cm = CountMin(65536, 4, 1000, 2, flow_fields=FIVE, seeds=seeds, max_flows=1 << 21)
    cm.insert_headers(hb.hdr, hb.wirelen)
    cm.flush()
    assert cm.stats()["inserted"] == 1_000_000
    orc = oracle.CountMin(65536, 4, 1000, 2, 37, seeds)
    assert orc.insert_hdr64(hb.hdr, hb.wirelen, FIVE) == 1_000_000
    _same_state(cm, orc)
    hh = cm.heavy_hitters()
    assert_same_list([(x.Flow, x.Count) for x in hh.Count], orc.heavy("count"))
    assert_same_list([(x.Flow, x.Size) for x in hh.Size], orc.heavy("size"))
    n_size = len(hh.Size)
    assert n_size > 0  # unique flows: count fingerprints never reach 2, sizes do reach 1000


def _encap_flows(rng, n_flows):
    """(frame, wirelen) per flow over the encapsulations gns_frame.cpp decodes on
    the host (builders of tests/golden/make_frame_vectors.py), random addresses
    and ports; a few flows are ARP (no IP layer)."""
    import importlib.util
    import os
    import struct
    spec = importlib.util.spec_from_file_location(
        "mfv", os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "make_frame_vectors.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    out = []
    for i in range(n_flows):
        a4, b4, c4, d4 = (bytes(rng.integers(0, 256, 4, dtype=np.uint8)) for _ in range(4))
        a6, b6 = (bytes(rng.integers(0, 256, 16, dtype=np.uint8)) for _ in range(2))
        sp, dp = (int(x) for x in rng.integers(1024, 65535, 2))
        l4 = m.tcp(sp, dp, b"t" * 20) if rng.random() < 0.6 else m.udp(sp, dp, b"u" * 12)
        pr = 6 if len(l4) == 40 else 17
        shape = i % 16
        if shape == 0:
            f = m.eth(0x0800, m.ipv4(a4, b4, pr, l4))
        elif shape == 1:
            f = m.eth(0x0800, m.ipv4(a4, b4, pr, l4, opts=b"\x01\x01\x01\x00"))
        elif shape == 2:
            f = m.eth(0x8100, m.vlan(0x8100, m.vlan(0x8100, m.vlan(0x0800, m.ipv4(a4, b4, pr, l4)))))
        elif shape == 3:
            f = m.eth(0x86DD, m.ipv6(a6, b6, 0, m.ext(pr, b"\x01\x04" + bytes(4)) + l4))
        elif shape == 4:
            f = m.eth(0x86DD, m.ipv6(a6, b6, 60, m.ext(pr, b"\x01\x04" + bytes(4)) + l4))
        elif shape == 5:
            f = m.eth(0x0800, m.ipv4(a4, b4, 47, b"\x00\x00\x08\x00" + m.ipv4(c4, d4, pr, l4)))
        elif shape == 6:
            f = m.eth(0x0800, m.ipv4(a4, b4, 17, m.udp(sp, 4789, m.vx + m.eth(0x0800, m.ipv4(c4, d4, pr, l4)))))
        elif shape == 7:
            f = m.eth(0x0800, m.ipv4(a4, b4, 17, m.udp(sp, 6081, m.gen + m.eth(0x0800, m.ipv4(c4, d4, pr, l4)))))
        elif shape == 8:
            inner = m.ipv4(c4, d4, pr, l4)
            f = m.eth(0x0800, m.ipv4(a4, b4, 17, m.udp(2152, 2152, b"\x30\xff" + struct.pack(">HI", len(inner), 7) + inner)))
        elif shape == 9:
            f = m.eth(0x8847, m.mpls + m.ipv4(c4, d4, pr, l4))
        elif shape == 10:
            inner = m.ipv6(a6, b6, pr, l4)
            f = m.eth(0x8864, bytes([0x11, 0, 0, 1]) + struct.pack(">H", 2 + len(inner)) + b"\x00\x57" + inner)
        elif shape == 11:
            f = m.eth(0x0800, m.ipv4(a4, b4, 41, m.ipv6(a6, b6, pr, l4)))
        elif shape == 12:
            f = m.eth(0x86DD, m.ipv6(a6, b6, 51, bytes([pr, 4, 0, 0]) + bytes(20) + l4))
        elif shape == 13:
            inner = m.ipv4(c4, d4, pr, l4)
            f = m.eth(len(inner) + 8, b"\xaa\xaa\x03\x00\x00\x00\x08\x00" + inner)
        elif shape == 14:
            f = m.pad(m.eth(0x0806, bytes(28)))
        else:
            f = m.eth(0x86DD, m.ipv6(a6, b6, pr, l4))
        f = m.pad(f)
        out.append((f, len(f) + int(rng.integers(0, 200))))
    return out


def test_encapsulated_capture_decoded_on_host(gpu, oracle, tmp_path):
    """Verdict r2 #4: a capture of tunnelled / optioned / extension-header frames
    (IPv4 options, 3 VLAN tags, IPv6 hop-by-hop / destination / AH chains,
    GRE, VXLAN, Geneve, GTP-U, MPLS, PPPoE, 6in4, LLC/SNAP, ARP): the packer
    decodes every frame outside the device fast path into a 0x88B5 record
    (gns_frame.cpp, == oracle/pyframe.py), the device reports unsupported == 0,
    and Count-Min state + heavy hitters equal the oracle fed the same records."""
    from go2netspectra_amd import CountMin, read_pcap, write_pcap
    from oracle import pyframe
    rng = np.random.default_rng(77)
    flows = _encap_flows(rng, 4000)
    n = 400_000
    pick = np.minimum(rng.zipf(1.3, n) - 1, len(flows) - 1)
    path = str(tmp_path / "encap.pcap")
    write_pcap(path, [flows[i][0] for i in pick], [flows[i][1] for i in pick])
    hb = read_pcap(path)
    assert len(hb) == n
    for i in np.unique(pick)[:4000:7]:
        j = int(np.flatnonzero(pick == i)[0])
        assert bytes(hb.hdr[j]) == pyframe.frame_record(*flows[i])
    n_arp = int(sum(1 for i in pick if i % 16 == 14))
    seeds = np.random.default_rng(8).integers(0, 2**32, 4, dtype=np.uint64).astype(np.uint32)
    cm = CountMin(65536, 4, 20000, 50, flow_fields=FIVE, seeds=seeds, max_flows=1 << 20)
    cm.insert_headers(hb.hdr, hb.wirelen)
    cm.flush()
    st = cm.stats()
    assert st["unsupported"] == 0 and st["dropped"] == n_arp and st["inserted"] == n - n_arp
    orc = oracle.CountMin(65536, 4, 20000, 50, 37, seeds)
    assert orc.insert_hdr64(hb.hdr, hb.wirelen, FIVE) == n - n_arp
    _same_state(cm, orc)
    hh = cm.heavy_hitters()
    assert_same_list([(x.Flow, x.Count) for x in hh.Count], orc.heavy("count"))
    assert_same_list([(x.Flow, x.Size) for x in hh.Size], orc.heavy("size"))
    assert len(hh.Count) > 0 and len(hh.Size) > 0
    # the same capture as compact records (host packer), staged in several device batches,
    # and as compact records made on the device from the 64-byte records
    import torch
    from go2netspectra_amd import compact_headers, read_pcap_compact
    rec, cwl, side = read_pcap_compact(path)
    assert len(side) > 0 and np.array_equal(cwl, hb.wirelen)
    cm2 = CountMin(65536, 4, 20000, 50, flow_fields=FIVE, seeds=seeds, max_flows=1 << 20, batch_packets=70_000)
    cm2.insert_compact(rec, cwl, side)
    cm2.flush()
    assert cm2.stats() == st
    _same_state(cm2, orc)
    dh = torch.from_numpy(hb.hdr).cuda()
    dw = torch.from_numpy(hb.wirelen.view(np.int32)).cuda()
    drec, dside = compact_headers(dh, dw)
    cm3 = CountMin(65536, 4, 20000, 50, flow_fields=FIVE, seeds=seeds, max_flows=1 << 20)
    cm3.insert_compact(drec, dw, dside)
    cm3.flush()
    assert cm3.stats() == st
    _same_state(cm3, orc)
    # the 16-byte form (wire lengths inside the records): host packer through staged host
    # batches, device producer through device batches; IPv6 tuples escape to the side array
    rec16, none16, side16 = read_pcap_compact(path, rec_len=True)
    assert none16 is None and len(side16) >= len(side)
    assert np.array_equal(np.ascontiguousarray(rec16[:, 12:16]).view("<u4").reshape(-1) >> 16, hb.wirelen)
    cm5 = CountMin(65536, 4, 20000, 50, flow_fields=FIVE, seeds=seeds, max_flows=1 << 20, batch_packets=70_000)
    cm5.insert_compact(rec16, None, side16)
    cm5.flush()
    assert cm5.stats() == st
    _same_state(cm5, orc)
    drec16, dside16 = compact_headers(dh, dw, rec_len=True)
    dr, ds = drec16.cpu().numpy(), dside16.cpu().numpy()
    esc = rec16[:, 13] == 2  # the device numbers its escapes in wave order, the packer in file order
    assert np.array_equal(dr[:, 13], rec16[:, 13]) and np.array_equal(dr[~esc], rec16[~esc])
    assert np.array_equal(dr[esc, 4:], rec16[esc, 4:]) and len(ds) == len(side16)
    hi = np.ascontiguousarray(rec16[esc, :4]).view("<u4").reshape(-1)
    di = np.ascontiguousarray(dr[esc, :4]).view("<u4").reshape(-1)
    assert np.array_equal(ds[di], side16[hi])
    cm6 = CountMin(65536, 4, 20000, 50, flow_fields=FIVE, seeds=seeds, max_flows=1 << 20, batch_packets=70_000)
    cm6.insert_compact(drec16, None, dside16)
    cm6.flush()
    assert cm6.stats() == st
    _same_state(cm6, orc)
    # a short or missing side array (advisor r4): escapes past it are counted as
    # unsupported and never read; everything else is applied as before
    cls = rec[:, 13]
    idx = np.ascontiguousarray(rec[:, :4]).view("<u4").reshape(-1)
    for keep in (len(side) // 2, 0):
        lost = (cls == 2) & (idx >= keep)
        assert lost.any()
        cm4 = CountMin(65536, 4, 20000, 50, flow_fields=FIVE, seeds=seeds, max_flows=1 << 20, batch_packets=70_000)
        cm4.insert_compact(rec, cwl, side[:keep] if keep else None)
        cm4.flush()
        s4 = cm4.stats()
        assert s4["unsupported"] == int(lost.sum()) and s4["dropped"] == n_arp
        o4 = oracle.CountMin(65536, 4, 20000, 50, 37, seeds)
        o4.insert_hdr64(hb.hdr[~lost], hb.wirelen[~lost], FIVE)
        _same_state(cm4, o4)
