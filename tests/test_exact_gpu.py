"""Exact aggregator parity on the GPU: every flow's Go key string, StartTime,
EndTime, PacketCount and ByteCount from the engine (C ABI gns_ex_*) equal the
sequential C restatement of exact/task.go, which keys flows by the Go-formatted
string itself."""
import numpy as np
import pytest

from helpers import assert_same_flows, frames_from_tuples, random_tuples

pytestmark = pytest.mark.gpu

FIVE = ["SrcIP", "DstIP", "SrcPort", "DstPort", "Protocol"]


def gpu_flows(task):
    return {f.Key: (f.StartTime, f.EndTime, f.PacketCount, f.ByteCount) for f in task.flows()}


def tricky_tuples(rng, n, nflows):
    """IPv4 flows, the same flows arriving IPv4-mapped over IPv6 (same key string),
    and IPv6 addresses whose 16-byte slot equals an IPv4 slot (different string)."""
    t = random_tuples(rng, n, nflows, v6_frac=0.3, s=1.05)
    v6 = t["v6"].copy()
    ipver = np.where(v6, 6, 4).astype(np.uint8)
    sel = rng.random(n) < 0.15  # re-send some IPv4 packets as IPv4-mapped IPv6
    m = sel & ~v6
    for a in ("src16", "dst16"):
        x = t[a]
        x[m, 12:16] = x[m, 0:4]
        x[m, 0:10] = 0
        x[m, 10:12] = 0xFF
    ipver[m] = 6
    alias = (rng.random(n) < 0.05) & ~v6 & ~m  # IPv4 slot bytes, but a 16-byte IPv6 net.IP
    ipver[alias] = 6
    return t, ipver


def test_tuples_parity(gpu, oracle):
    from go2netspectra_amd import ExactTask, PacketBatch
    rng = np.random.default_rng(1)
    n = 300_000
    t, ipver = tricky_tuples(rng, n, 20_000)
    ts = rng.integers(-(1 << 40), 1 << 40, n).astype(np.int64)  # not monotonic: order is stream order
    b = PacketBatch(t["src16"], t["dst16"], t["sport"], t["dport"], t["proto"], t["length"], ipver, ts)
    task = ExactTask("per_five_tuple", FIVE, 128, batch_packets=65536)
    for part in np.array_split(np.arange(n), 3):
        task.process_packets(PacketBatch(*(None if a is None else a[part] for a in
                                           (b.src16, b.dst16, b.sport, b.dport, b.proto, b.length, b.ipver, b.ts))))
    task.flush()
    orc = oracle.Exact(FIVE)
    orc.insert_tuples(t["src16"], t["dst16"], t["sport"], t["dport"], t["proto"], ipver, t["length"], ts)
    want = orc.export()
    got = gpu_flows(task)
    assert len(got) == len(want)
    assert_same_flows(got, want)
    snap = task.snapshot()
    assert snap.TaskName == "per_five_tuple" and len(snap.Shards) == 128
    assert sum(len(s.Flows) for s in snap.Shards) == len(want)


@pytest.mark.parametrize("fields", [["SrcIP"], ["DstPort", "Protocol"], ["DstIP", "SrcIP", "SrcPort"]])
def test_headers_parity_and_reset(gpu, oracle, fields):
    from go2netspectra_amd import ExactTask, HeaderBatch
    rng = np.random.default_rng(len(fields))
    t = random_tuples(rng, 80_000, 3000, v6_frac=0.25)
    hdr = frames_from_tuples(t, rng, vlan_frac=0.3)
    hdr[rng.random(len(hdr)) < 0.02, 12:14] = [0x08, 0x06]  # ARP: dropped (parser.go:48-49)
    ts = np.cumsum(rng.integers(0, 5000, len(hdr))).astype(np.int64)
    task = ExactTask("x", fields)
    task.process_packets(HeaderBatch(hdr, t["length"], ts))
    task.flush()
    orc = oracle.Exact(fields)
    done = orc.insert_hdr64(hdr, t["length"], ts)
    assert task.agg.counters()["inserted"] == done
    assert_same_flows(gpu_flows(task), orc.export())
    task.reset()
    orc.reset()
    task.process_packets(HeaderBatch(hdr[:5000], t["length"][:5000], ts[:5000] + 7))
    orc.insert_hdr64(hdr[:5000], t["length"][:5000], ts[:5000] + 7)
    task.flush()
    assert_same_flows(gpu_flows(task), orc.export())


def test_query(gpu, oracle):
    """Query reads IP fields as 16-byte net.IPs (task.go:298-326): an IPv4 flow is found
    through its IPv4-mapped form, not through the left-aligned sketch slot."""
    from go2netspectra_amd import ExactTask, PacketBatch
    rng = np.random.default_rng(3)
    n = 50_000
    t, ipver = tricky_tuples(rng, n, 2000)
    ts = np.arange(n, dtype=np.int64)
    task = ExactTask("q", FIVE)
    task.process_packets(PacketBatch(t["src16"], t["dst16"], t["sport"], t["dport"], t["proto"], t["length"],
                                     ipver, ts))
    task.flush()
    orc = oracle.Exact(FIVE)
    orc.insert_tuples(t["src16"], t["dst16"], t["sport"], t["dport"], t["proto"], ipver, t["length"], ts)
    keys = PacketBatch(t["src16"], t["dst16"], t["sport"], t["dport"], t["proto"], t["length"]).keys(FIVE)[:3000]
    mapped = keys.copy()
    v4 = ipver[:3000] == 4
    for off in (0, 16):
        mapped[v4, off + 12:off + 16] = keys[v4, off:off + 4]
        mapped[v4, off:off + 10] = 0
        mapped[v4, off + 10:off + 12] = 0xFF
    for q in (keys, mapped):
        got = task.agg.query_many(q)
        want = np.array([orc.query(bytes(k)) for k in q], np.uint64)
        assert np.array_equal(got, want)
        import torch  # device keys in, device answers out (gns_ex_query_device)
        gd = task.agg.query_many(torch.from_numpy(np.ascontiguousarray(q)).cuda())
        assert gd.is_cuda and np.array_equal(gd.cpu().numpy().view(np.uint64), want)
    assert (task.agg.query_many(mapped[v4]) > 0).all()
    assert task.query(bytes(mapped[0])) == orc.query(bytes(mapped[0]))


def test_synthetic_device_resident(gpu, oracle):
    import torch
    from go2netspectra_amd import ExactTask, HeaderBatch, SyntheticTraffic
    syn = SyntheticTraffic()
    hdr, wl = syn.generate(2_000_000)
    ts = torch.arange(2_000_000, dtype=torch.int64, device="cuda") * 1000 + 1_700_000_000_000_000_000
    task = ExactTask("per_five_tuple", FIVE, max_flows=1 << 21)
    task.process_packets(HeaderBatch(hdr, wl, ts))
    task.flush()
    torch.cuda.synchronize()
    orc = oracle.Exact(FIVE)
    assert orc.insert_hdr64(hdr.cpu().numpy(), wl.cpu().numpy().view(np.uint32), ts.cpu().numpy()) == 2_000_000
    assert_same_flows(gpu_flows(task), orc.export())


def test_manager_exact_group(gpu, oracle):
    from go2netspectra_amd import HeaderBatch, Manager, parse_config
    cfg = parse_config("""
aggregator:
  types: ["exact"]
  exact:
    tasks:
      - name: "per_five_tuple"
        key_fields: ["SrcIP", "DstIP", "SrcPort", "DstPort", "Protocol"]
        num_shards: 128
""")
    rng = np.random.default_rng(9)
    t = random_tuples(rng, 20_000, 500)
    hdr = frames_from_tuples(t)
    ts = np.arange(20_000, dtype=np.int64)
    mgr = Manager(cfg)
    mgr.start()
    mgr.process(HeaderBatch(hdr, t["length"], ts))
    snaps = mgr.stop()
    orc = oracle.Exact(FIVE)
    orc.insert_hdr64(hdr, t["length"], ts)
    got = {k: (f.StartTime, f.EndTime, f.PacketCount, f.ByteCount)
           for s in snaps["per_five_tuple"].Shards for k, f in s.Flows.items()}
    assert_same_flows(got, orc.export())
    task = mgr.tasks()[0]
    msg = task.alerter_msg([{"name": "r", "task_name": "per_five_tuple", "metric": "total_packets",
                             "operator": ">", "threshold": 100}])
    assert "Observed Value:</b> <code>20000 packets" in msg


def test_dictionary_grows_instead_of_failing(gpu, oracle):
    """exact/task.go:135-148 keeps every flow of the period (a Go map grows): a
    dictionary sized for 32 flows doubles as the flows arrive (the batch that
    overflows is re-run on the grown table) and the result equals the oracle;
    reset then starts a clean period."""
    from go2netspectra_amd import ExactTask, HeaderBatch
    rng = np.random.default_rng(29)
    task = ExactTask("tiny", FIVE, max_flows=32, batch_packets=1 << 16)
    t = random_tuples(rng, 200_000, 60_000, s=0.5)
    hdr = frames_from_tuples(t, rng)
    ts = np.arange(len(hdr), dtype=np.int64)
    for part in np.array_split(np.arange(len(hdr)), 3):
        task.process_packets(HeaderBatch(hdr[part], t["length"][part], ts[part]))
    task.flush()
    orc = oracle.Exact(FIVE)
    orc.insert_hdr64(hdr, t["length"], ts)
    assert_same_flows(gpu_flows(task), orc.export())
    ds = task.agg.dict_stats()
    assert ds["growths"] >= 8 and ds["slots"] >= 1 << 16, ds
    assert task.agg.counters()["dict_full"] == 0
    task.reset()
    orc = oracle.Exact(FIVE)
    t2 = random_tuples(rng, 5000, 20)
    hdr2 = frames_from_tuples(t2, rng)
    ts2 = np.arange(len(hdr2), dtype=np.int64) + 99
    task.process_packets(HeaderBatch(hdr2, t2["length"], ts2))
    task.flush()
    orc.insert_hdr64(hdr2, t2["length"], ts2)
    assert_same_flows(gpu_flows(task), orc.export())


@pytest.mark.parametrize("batch", [16384, 1 << 24])
def test_wire_lengths_beyond_the_sort_word_field(gpu, oracle, batch):
    """X2 sorts one 64-bit word per packet (flow id | packet index | wire length): a
    length that does not fit the word's length field (>= 2^sb - 1, the escape value
    itself included) is read back from the batch's length array; ByteCount is a u64
    sum (task.go:154-212)."""
    from go2netspectra_amd import ExactTask, PacketBatch
    rng = np.random.default_rng(31)
    n = 120_000
    t = random_tuples(rng, n, 400)
    big = rng.random(n) < 0.2
    lens = t["length"].copy()
    lens[big] = rng.integers(1 << 12, 1 << 32, big.sum(), dtype=np.uint64).astype(np.uint32)
    edge = np.flatnonzero(~big)[:64]  # every power-of-two boundary a field width could have
    lens[edge] = (np.uint64(1) << (np.arange(64) % 32 + 1).astype(np.uint64)) - np.uint64(1) - (np.arange(64) // 32).astype(np.uint64)
    lens[-1] = 0xFFFFFFFF
    ts = rng.integers(-(1 << 50), 1 << 50, n).astype(np.int64)
    task = ExactTask("big", FIVE, batch_packets=batch, max_flows=1 << 12)
    ipver = np.where(t["v6"], 6, 4).astype(np.uint8)
    task.process_packets(PacketBatch(t["src16"], t["dst16"], t["sport"], t["dport"], t["proto"], lens, ipver, ts))
    task.flush()
    orc = oracle.Exact(FIVE)
    orc.insert_tuples(t["src16"], t["dst16"], t["sport"], t["dport"], t["proto"], ipver, lens, ts)
    assert_same_flows(gpu_flows(task), orc.export())


def test_pcapng_capture_drives_exact_and_countmin(gpu, oracle, tmp_path):
    """A pcapng capture (nanosecond if_tsresol, several interfaces, skipped blocks) read by the
    host packer feeds the exact aggregator (StartTime/EndTime from the capture timestamps) and
    Count-Min exactly as the restatements see the same records (reader.go:35-49 -> task.go)."""
    import go2netspectra_amd as g
    from go2netspectra_amd import CountMin, ExactTask
    rng = np.random.default_rng(41)
    t = random_tuples(rng, 30_000, 800, v6_frac=0.2)
    hdr = frames_from_tuples(t, rng, vlan_frac=0.2)
    ts = rng.integers(1 << 60, (1 << 60) + (1 << 40), len(hdr)).astype(np.uint64)
    path = str(tmp_path / "c.pcapng")
    g.write_pcapng(path, [bytes(r) for r in hdr], t["length"], ts_units=ts, tsresol=9,
                   iface_of=rng.integers(0, 2, len(hdr)), n_ifaces=2, extra_blocks=True)
    hb = g.read_pcap(path)
    from oracle import pyframe  # VLAN-tagged / IPv6 frames come back as host-decoded 0x88B5 records
    want = np.frombuffer(b"".join(pyframe.frame_record(bytes(r), int(w)) for r, w in zip(hdr, t["length"])),
                         np.uint8).reshape(-1, 64)
    assert np.array_equal(hb.hdr, want) and np.array_equal(hb.wirelen, t["length"])
    assert np.array_equal(hb.ts, ts.astype(np.int64))
    task = ExactTask("cap", FIVE)
    task.process_packets(hb)
    task.flush()
    orc = oracle.Exact(FIVE)
    orc.insert_hdr64(hb.hdr, hb.wirelen, hb.ts)
    assert_same_flows(gpu_flows(task), orc.export())
    seeds = np.array([0x9747B28C, 0x1B873593, 0xCC9E2D51], np.uint32)
    cm = CountMin(4096, 3, 1 << 20, 50, flow_fields=FIVE, seeds=seeds, max_flows=1 << 14)
    cm.insert_headers(hb.hdr, hb.wirelen)
    cm.flush()
    o = oracle.CountMin(4096, 3, 1 << 20, 50, 37, seeds)
    o.insert_hdr64(hb.hdr, hb.wirelen, FIVE)
    for a, b in zip(cm.export_state(), o.export()):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("batch,touched_list", [(4096, False), (300_000, False), (1_500_000, False), (300_000, True)])
def test_start_end_times_with_heavy_ties_across_sort_paths(gpu, oracle, monkeypatch, batch, touched_list):
    """StartTime / EndTime come from the merged smallest / largest stream index of
    every path (designated flows' LDS partials in X1 and X1b, the tail's per-bin
    aggregation with wave folding).  Batch sizes span the cold-start cap, one and
    several P3 sub-passes; 40 heavy flows are designated after the first batch
    (and fold in P4 before it); timestamps are random so any wrong first / last
    packet shows."""
    from go2netspectra_amd import ExactTask, PacketBatch
    if touched_list:  # T and D over the batch's touched-flow list (large tables) instead of a slot scan
        monkeypatch.setenv("GNS_EX_LIST", "1")
    rng = np.random.default_rng(batch)
    n = 3_000_000
    t = random_tuples(rng, n, 40, s=0.8)
    ts = rng.integers(-(1 << 60), 1 << 60, n).astype(np.int64)
    ipver = np.where(t["v6"], 6, 4).astype(np.uint8)
    task = ExactTask("ties", FIVE, batch_packets=batch, max_flows=1 << 10)
    task.process_packets(PacketBatch(t["src16"], t["dst16"], t["sport"], t["dport"], t["proto"], t["length"], ipver, ts))
    task.flush()
    orc = oracle.Exact(FIVE)
    orc.insert_tuples(t["src16"], t["dst16"], t["sport"], t["dport"], t["proto"], ipver, t["length"], ts)
    assert_same_flows(gpu_flows(task), orc.export())


@pytest.mark.parametrize("touched_list", [False, True])
def test_tail_bins_with_more_flows_than_the_table(gpu, oracle, monkeypatch, touched_list):
    """About 1.4M distinct tail flows in one batch: each of P4's 512 bins holds more
    flows than its LDS table takes before a flush (2048), so bins merge in several
    rounds; every flow's four fields must still equal the oracle's."""
    from go2netspectra_amd import ExactTask, PacketBatch
    if touched_list:
        monkeypatch.setenv("GNS_EX_LIST", "1")
    rng = np.random.default_rng(11)
    n = 3_000_000
    t = random_tuples(rng, n, 3_000_000, s=0.3)
    ts = rng.integers(0, 1 << 50, n).astype(np.int64)
    ipver = np.where(t["v6"], 6, 4).astype(np.uint8)
    task = ExactTask("wide", FIVE, batch_packets=1 << 22, max_flows=1 << 22)
    task.process_packets(PacketBatch(t["src16"], t["dst16"], t["sport"], t["dport"], t["proto"], t["length"], ipver, ts))
    task.flush()
    orc = oracle.Exact(FIVE)
    orc.insert_tuples(t["src16"], t["dst16"], t["sport"], t["dport"], t["proto"], ipver, t["length"], ts)
    want = orc.export()
    assert len(want) > 1_500_000
    assert_same_flows(gpu_flows(task), want)
