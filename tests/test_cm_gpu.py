"""Count-Min parity on the GPU: every test compares the device state exported
through the C ABI with the sequential C oracle fed the same stream
(bit-exact: C, S and both fingerprint arrays)."""
import numpy as np
import pytest

from helpers import assert_same_list, frames_from_tuples, random_tuples, sizes_u32, zipf_index, zipf_keys

pytestmark = pytest.mark.gpu


def assert_same_state(cm, orc):
    C, S, Fc, Fs = cm.export_state()
    oC, oS, oFc, oFs = orc.export()
    for name, a, b in (("C", C, oC), ("S", S, oS), ("FPc", Fc, oFc), ("FPs", Fs, oFs)):
        if not np.array_equal(a, b):
            bad = np.nonzero(a != b)[0] if a.ndim == 1 else np.nonzero((a != b).any(axis=1))[0]
            raise AssertionError(f"{name} differs in {len(bad)} cells, first {bad[:5]}: "
                                 f"gpu={a[bad[:3]]} oracle={b[bad[:3]]}")


def make_pair(oracle, w, d, K, st=1000, ct=10, seed=1, **kw):
    from go2netspectra_amd import CountMin
    seeds = np.random.default_rng(seed).integers(0, 2**32, d, dtype=np.uint64).astype(np.uint32)
    cm = CountMin(w, d, st, ct, key_bytes=K, seeds=seeds, **kw)
    orc = oracle.CountMin(w, d, st, ct, K, seeds)
    return cm, orc


@pytest.mark.parametrize("w,d,K,nflows,n,batch", [
    (256, 2, 16, 2000, 100_000, 0),        # heavy collisions: replay path
    (65536, 4, 37, 50_000, 1_000_000, 0),  # C1 geometry
    (1000, 3, 13, 5000, 200_000, 0),       # non power-of-two width, odd key
    (1, 1, 4, 50, 60_000, 0),              # every packet in one bucket
    (4096, 2, 16, 3000, 300_000, 32768),   # multi-batch (state carried across batches)
    (1 << 20, 4, 37, 1 << 18, 2_000_000, 0),
])
def test_insert_keys_parity(gpu, oracle, w, d, K, nflows, n, batch):
    rng = np.random.default_rng(w * 7 + d)
    cm, orc = make_pair(oracle, w, d, K, batch_packets=batch)
    keys, _, _ = zipf_keys(rng, n, nflows, K)
    sizes = sizes_u32(rng, n)
    cm.insert_keys(keys, sizes)
    cm.flush()
    orc.insert_keys(keys, sizes)
    assert_same_state(cm, orc)


def test_many_calls_and_reset(gpu, oracle):
    rng = np.random.default_rng(5)
    cm, orc = make_pair(oracle, 512, 3, 16, st=5000, ct=20)
    for _ in range(4):
        keys, _, _ = zipf_keys(rng, 20_000, 700, 16)
        sizes = sizes_u32(rng, 20_000)
        cm.insert_keys(keys, sizes)
        orc.insert_keys(keys, sizes)
    cm.flush()
    assert_same_state(cm, orc)
    cm.reset()
    orc.reset()
    assert_same_state(cm, orc)
    keys, _, _ = zipf_keys(rng, 30_000, 300, 16)
    sizes = sizes_u32(rng, 30_000)
    cm.insert_keys(keys, sizes)
    orc.insert_keys(keys, sizes)
    cm.flush()
    assert_same_state(cm, orc)


def test_stage_timing_mask(gpu, oracle):
    """set_timing(stages=...) times only those stages; the result is unchanged."""
    rng = np.random.default_rng(9)
    cm, orc = make_pair(oracle, 4096, 4, 37)
    keys, _, _ = zipf_keys(rng, 200_000, 5000, 37)
    sizes = sizes_u32(rng, 200_000)
    cm.set_timing(True, stages=["extract", "apply"])
    cm.stage_times(reset=True)
    cm.insert_keys(keys, sizes)
    cm.flush()
    st = cm.stage_times()
    assert st["extract"][1] >= 1 and st["apply"][1] >= 1
    assert all(st[k][1] == 0 for k in cm.STAGES if k not in ("extract", "apply"))
    cm.set_timing(True)
    cm.stage_times(reset=True)
    cm.insert_keys(keys, sizes)
    cm.flush()
    st = cm.stage_times()
    assert st["resolve"][1] >= 1 and st["insert"][1] >= 1
    orc.insert_keys(keys, sizes)
    orc.insert_keys(keys, sizes)
    assert_same_state(cm, orc)


def test_sizes_wrap_and_overflow(gpu, oracle):
    """sizes >= 2^20-1 take the overflow path; u32 wrap of S (count_min.go:110)."""
    rng = np.random.default_rng(9)
    cm, orc = make_pair(oracle, 128, 2, 8)
    keys, _, _ = zipf_keys(rng, 50_000, 40, 8, s=1.5)
    sizes = sizes_u32(rng, 50_000, big_frac=0.05)
    sizes[:100] = 0
    sizes[100:200] = 0xFFFFFFFF
    cm.insert_keys(keys, sizes)
    orc.insert_keys(keys, sizes)
    cm.flush()
    assert_same_state(cm, orc)


def test_query_and_heavy_hitters(gpu, oracle):
    rng = np.random.default_rng(11)
    cm, orc = make_pair(oracle, 4096, 3, 16, st=20_000, ct=50)
    keys, flows, _ = zipf_keys(rng, 200_000, 20_000, 16)
    sizes = sizes_u32(rng, 200_000)
    cm.insert_keys(keys, sizes)
    orc.insert_keys(keys, sizes)
    cm.flush()
    q = cm.query_many(flows[:5000])
    want = np.array([orc.query(bytes(f)) for f in flows[:5000]], dtype=np.uint64)
    assert np.array_equal(q, want)
    import torch  # device keys in, device answers out (gns_cm_query_device); a strided view of the keys
    k17 = np.zeros((5000, 17), np.uint8)
    k17[:, :16] = flows[:5000]
    qd = cm.query_many(torch.from_numpy(k17).cuda()[:, :16])
    assert qd.is_cuda and np.array_equal(qd.cpu().numpy().view(np.uint64), want)
    absent = rng.integers(0, 256, (100, 16), dtype=np.uint8)
    assert np.array_equal(cm.query_many(absent), np.array([orc.query(bytes(f)) for f in absent], np.uint64))
    hh = cm.heavy_hitters()
    assert_same_list([(h.Flow, h.Count) for h in hh.Count], orc.heavy("count"))
    assert_same_list([(h.Flow, h.Size) for h in hh.Size], orc.heavy("size"))
    assert hh.Size is not None


@pytest.mark.parametrize("K", [4, 8, 13, 16, 37])
def test_heavy_hitter_ties_beyond_first_bytes(gpu, oracle, K):
    """Equal counts AND equal first key bytes: the device orders ties by the full key
    (stable radix passes over every 8-byte chunk), value desc then bytes asc, as the
    oracle's canonical order of count_min.go:232-239."""
    rng = np.random.default_rng(K)
    cm, orc = make_pair(oracle, 65536, 3, K, st=1000, ct=10)
    base = rng.integers(0, 256, K, dtype=np.uint8)
    flows = np.repeat(base[None, :], 300, axis=0)
    for i in range(300):  # differ only in the last two bytes, or only in byte 5 / the middle
        if K >= 2:
            flows[i, K - 2] = (i >> 8) & 0xFF
            flows[i, K - 1] = i & 0xFF
        if K > 5 and i % 5 == 0:
            flows[i, 5] ^= 0x80
        if K > 12 and i % 7 == 0:
            flows[i, K // 2] ^= 0x40
    flows = np.unique(flows, axis=0)
    reps = 50 + np.arange(len(flows)) % 3  # three groups of equal counts
    keys = np.repeat(flows, reps, axis=0)
    keys = keys[rng.permutation(len(keys))]
    sizes = np.full(len(keys), 100, np.uint32)
    cm.insert_keys(keys, sizes)
    orc.insert_keys(keys, sizes)
    cm.flush()
    hh = cm.heavy_hitters()
    got_c = [(h.Flow, h.Count) for h in hh.Count]
    assert_same_list(got_c, orc.heavy("count"))
    assert_same_list([(h.Flow, h.Size) for h in hh.Size], orc.heavy("size"))
    assert len(got_c) > 100 and len({v for _, v in got_c}) <= 6  # many ties


@pytest.mark.parametrize("fields", [
    ["SrcIP"], ["SrcIP", "DstIP", "SrcPort", "DstPort", "Protocol"],
    ["DstIP", "SrcPort", "DstPort", "Protocol"], ["SrcPort", "SrcIP", "Protocol"], ["DstPort"],
])
def test_tuples_and_headers_parity(gpu, oracle, fields):
    from go2netspectra_amd import CountMin, PacketBatch
    rng = np.random.default_rng(len(fields))
    t = random_tuples(rng, 60_000, 3000, v6_frac=0.2)
    K = sum({"SrcIP": 16, "DstIP": 16, "SrcPort": 2, "DstPort": 2, "Protocol": 1}[f] for f in fields)
    seeds = np.array([0x1111, 0x2222, 0x3333], np.uint32)
    batch = PacketBatch(t["src16"], t["dst16"], t["sport"], t["dport"], t["proto"], t["length"])
    cm = CountMin(2048, 3, 10_000, 30, flow_fields=fields, seeds=seeds)
    cm.insert_tuples(batch)
    cm.flush()
    orc = oracle.CountMin(2048, 3, 10_000, 30, K, seeds)
    orc.insert_keys(batch.keys(fields), t["length"])
    assert_same_state(cm, orc)
    # same packets as 64-byte frame records through the fused parser
    hdr = frames_from_tuples(t, rng, vlan_frac=0.3)
    cm2 = CountMin(2048, 3, 10_000, 30, flow_fields=fields, seeds=seeds)
    cm2.insert_headers(hdr, t["length"])
    cm2.flush()
    orc2 = oracle.CountMin(2048, 3, 10_000, 30, K, seeds)
    done = orc2.insert_hdr64(hdr, t["length"], fields)
    assert done == 60_000 - cm2.stats()["unsupported"] - cm2.stats()["dropped"]
    assert_same_state(cm2, orc2)


def test_synthetic_device_resident_parity(gpu, oracle):
    """C2 geometry on device-resident synthetic Zipf headers (2M packets)."""
    import torch
    from go2netspectra_amd import CountMin, SyntheticTraffic
    fields = ["SrcIP", "DstIP", "SrcPort", "DstPort", "Protocol"]
    syn = SyntheticTraffic()
    hdr, wl = syn.generate(2_000_000)
    seeds = np.array([0xA1, 0xB2, 0xC3, 0xD4], np.uint32)
    cm = CountMin(1 << 20, 4, 1 << 20, 1000, flow_fields=fields, seeds=seeds, max_flows=1 << 21)
    cm.insert_headers(hdr, wl)
    cm.flush()
    torch.cuda.synchronize()
    orc = oracle.CountMin(1 << 20, 4, 1 << 20, 1000, 37, seeds)
    h = hdr.cpu().numpy()
    w = wl.cpu().numpy().view(np.uint32)
    assert orc.insert_hdr64(h, w, fields) == 2_000_000
    assert_same_state(cm, orc)
    assert cm.stats()["inserted"] == 2_000_000


@pytest.mark.parametrize("w", [1, 16, 4096])
def test_hot_designation_takeover(gpu, oracle, w):
    """Designated hot buckets whose owner changes between calls: the batch-level
    decision fails and the exact in-order fallback must reproduce the oracle."""
    rng = np.random.default_rng(w)
    cm, orc = make_pair(oracle, w, 2, 8, st=1 << 20, ct=100)
    flows = rng.integers(0, 256, (40, 8), dtype=np.uint8)
    for phase in range(5):
        n = 300_000
        # phase-dependent heavy flow (70%), the rest spread over the others
        heavy = np.full(n, phase % len(flows))
        idx = np.where(rng.random(n) < 0.7, heavy, rng.integers(0, len(flows), n))
        keys = np.ascontiguousarray(flows[idx])
        sizes = sizes_u32(rng, n)
        if phase == 3:
            sizes[::7] = rng.integers(1 << 21, 1 << 31, len(sizes[::7]))
        cm.insert_keys(keys, sizes)
        orc.insert_keys(keys, sizes)
        cm.flush()
        assert_same_state(cm, orc)
    st = cm.stage_times()
    assert "hot" in st


def test_golden_stream_fixture(gpu):
    """The committed oracle fixture (tests/golden/cm_stream.npz) through the engine."""
    import os
    from go2netspectra_amd import CountMin
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "cm_stream.npz"))
    w, d, st, ct, K = (int(x) for x in z["params"])
    cm = CountMin(w, d, st, ct, key_bytes=K, seeds=z["seeds"])
    cm.insert_keys(z["keys"], z["sizes"])
    cm.flush()
    C, S, Fc, Fs = cm.export_state()
    assert np.array_equal(C, z["C"]) and np.array_equal(S, z["S"])
    assert np.array_equal(Fc, z["FPc"]) and np.array_equal(Fs, z["FPs"])
    hh = cm.heavy_hitters()
    assert [h.Count for h in hh.Count] == z["hh_count"].tolist()
    assert [h.Flow for h in hh.Count] == [bytes(x).ljust(K, b"\0") for x in z["hh_count_flows"]]
    assert [h.Size for h in hh.Size] == z["hh_size"].tolist()


def test_manager_task_surface(gpu, oracle):
    """factory -> Manager -> SketchTask path (model.Task surface) on header batches."""
    from go2netspectra_amd import HeaderBatch, Manager, parse_config
    cfg = parse_config("""
aggregator:
  types: ["sketch"]
  sketch:
    tasks:
      - {name: cm5, skt_type: 0, flow_fields: [SrcIP, DstIP, SrcPort, DstPort, Protocol], width: 4096, depth: 4,
         size_thereshold: 100000, count_thereshold: 50}
      - {name: cmsrc, skt_type: 0, flow_fields: [SrcIP], width: 1000, depth: 2, size_thereshold: 200000,
         count_thereshold: 100}
""")
    seeds = np.array([11, 22, 33, 44], np.uint32)
    mgr = Manager(cfg, seeds=seeds)
    mgr.start()
    rng = np.random.default_rng(77)
    t = random_tuples(rng, 50_000, 2000)
    hdr = frames_from_tuples(t)
    mgr.process(HeaderBatch(hdr, t["length"]))
    snaps = mgr.stop()
    for task, K, w, d, st, ctr in (("cm5", 37, 4096, 4, 100000, 50), ("cmsrc", 16, 1000, 2, 200000, 100)):
        fields = [x.FlowFields for x in cfg.Aggregator.Sketch.Tasks if x.Name == task][0]
        o = oracle.CountMin(w, d, st, ctr, K, seeds)
        o.insert_hdr64(hdr, t["length"], fields)
        assert [(h.Flow, h.Count) for h in snaps[task].Count] == o.heavy("count")
        assert [(h.Flow, h.Size) for h in snaps[task].Size] == o.heavy("size")


def test_large_sizes_mixed_owner(gpu, oracle):
    """Sizes just below and above the 2^19-1 escape, one bucket shared by an owner
    and a foreign flow: the per-chunk size sums must not carry between halves."""
    rng = np.random.default_rng(77)
    cm, orc = make_pair(oracle, 1, 1, 8, st=1, ct=1)
    n = 200_000
    flows = rng.integers(0, 256, (2, 8), dtype=np.uint8)
    idx = (rng.random(n) < 0.02).astype(np.int64)
    keys = np.ascontiguousarray(flows[idx])
    sizes = np.where(idx == 0, (1 << 19) - 2, rng.integers(0, 1 << 19, n)).astype(np.uint32)
    sizes[::97] = (1 << 19) - 1
    sizes[::89] = (1 << 20) - 2
    for part in np.array_split(np.arange(n), 4):
        cm.insert_keys(keys[part], sizes[part])
        orc.insert_keys(keys[part], sizes[part])
    cm.flush()
    assert_same_state(cm, orc)


@pytest.mark.parametrize("w,d,K,nflows,n", [
    (1 << 24, 8, 4, 1 << 16, 2_000_000),   # C5 geometry: bins of 16 LDS tiles
    (1 << 22, 8, 8, 1 << 15, 1_000_000),   # d * tiles > 4096: bins of 2 tiles
    (5_000_000, 3, 13, 50_000, 1_000_000),  # non power-of-two wide row
    (20_000_000, 8, 4, 1 << 15, 1_000_000),  # bins of 16 tiles (k_subpart's 1024-thread variant)
])
@pytest.mark.parametrize("sparse", ["1", "0"])
def test_wide_rows_parity(gpu, oracle, monkeypatch, w, d, K, nflows, n, sparse):
    """Widths beyond 1024 LDS tiles per row: K3 bins hold 2^sub_bits tiles.  K4 takes a
    bin in stream order with only its touched buckets in LDS (k_apply_sparse, the
    default), or (GNS_K4_SPARSE=0) partitions each bin by tile before the in-order
    tile pass (k_subpart + k_apply)."""
    monkeypatch.setenv("GNS_K4_SPARSE", sparse)
    rng = np.random.default_rng(w % 1000 + d)
    cm, orc = make_pair(oracle, w, d, K, st=1 << 16, ct=100, max_flows=1 << 20)
    keys, flows, _ = zipf_keys(rng, n, nflows, K)
    sizes = sizes_u32(rng, n)
    sizes[::1001] = 70_000  # overflow side table
    half = n // 2
    for sl in (slice(0, half), slice(half, n)):
        cm.insert_keys(keys[sl], sizes[sl])
        orc.insert_keys(keys[sl], sizes[sl])
    cm.flush()
    assert_same_state(cm, orc)
    q = cm.query_many(flows[:2000])
    assert np.array_equal(q, np.array([orc.query(bytes(f)) for f in flows[:2000]], np.uint64))
    hh = cm.heavy_hitters()
    assert_same_list([(h.Flow, h.Count) for h in hh.Count], orc.heavy("count"))


@pytest.mark.parametrize("w,d,K,nflows,n", [
    (65536, 4, 37, 50_000, 1_000_000),
    (256, 2, 16, 2000, 100_000),
])
def test_ballot_rank_fallback_parity(gpu, oracle, monkeypatch, w, d, K, nflows, n):
    """K3's ballot multisplit (used when the LDS lane-order probe fails; forced
    here with GNS_K3_RANK=0) gives the same bit-exact state."""
    monkeypatch.setenv("GNS_K3_RANK", "0")
    rng = np.random.default_rng(w + 3 * d)
    cm, orc = make_pair(oracle, w, d, K, batch_packets=n // 3)
    keys, _, _ = zipf_keys(rng, n, nflows, K)
    sizes = sizes_u32(rng, n)
    cm.insert_keys(keys, sizes)
    cm.flush()
    orc.insert_keys(keys, sizes)
    assert_same_state(cm, orc)


@pytest.mark.parametrize("K,batch,w,d", [(16, 0, 5000, 4), (37, 40_000, 5000, 4),
                                         (8, 0, 5_000_000, 3)])  # super-bins: the sparse K4's slice check
def test_bucket_range_slices_are_the_global_sketch(gpu, oracle, K, batch, w, d):
    """SURVEY §8e exact global mode: G handles with disjoint bucket ranges, each
    fed the whole stream, together hold exactly the single sketch (hot
    designation, replay and multi-batch paths included)."""
    from go2netspectra_amd import CountMin
    from go2netspectra_amd.dist import assemble_slices, bucket_slice
    rng = np.random.default_rng(77 + K)
    seeds = rng.integers(0, 2**32, d, dtype=np.uint64).astype(np.uint32)
    keys, _, _ = zipf_keys(rng, 400_000, 20_000, K)
    sizes = sizes_u32(rng, 400_000)
    orc = oracle.CountMin(w, d, 1000, 10, K, seeds)
    orc.insert_keys(keys, sizes)
    world = 3
    states, ranges = [], []
    for r in range(world):
        rg = bucket_slice(r, world, w)
        cm = CountMin(w, d, 1000, 10, key_bytes=K, seeds=seeds, batch_packets=batch, bucket_range=rg)
        cm.insert_keys(keys, sizes)
        cm.flush()
        states.append(cm.export_state())
        ranges.append(rg)
        cm.close()
    got = assemble_slices(states, ranges, w, d)
    for name, a, b in zip(("C", "S", "FPc", "FPs"), got, orc.export()):
        assert np.array_equal(a, b), name


def test_bucket_range_rejects_bad_ranges(gpu):
    from go2netspectra_amd import CountMin
    for rg in [(10, 10), (20, 10), (0, 5001)]:
        with pytest.raises(Exception):
            CountMin(5000, 2, 1000, 10, key_bytes=16, bucket_range=rg)


def test_tiny_dictionary_grows_and_reset_restarts(gpu, oracle):
    """A 64-flow initial dictionary under a stream of thousands of flows: the table
    grows instead of failing (count_min.go:94-157 has no failure mode), the state
    stays bit-exact, and reset starts a clean period."""
    rng = np.random.default_rng(17)
    cm, orc = make_pair(oracle, 1024, 3, 16, max_flows=64)
    keys, _, _ = zipf_keys(rng, 20_000, 5000, 16, s=0.5)
    sizes = sizes_u32(rng, 20_000)
    cm.insert_keys(keys, sizes)
    orc.insert_keys(keys, sizes)
    cm.flush()
    assert_same_state(cm, orc)
    ds = cm.dict_stats()
    assert ds["growths"] > 0 and ds["slots"] > 128, ds
    assert cm.counters()["dict_full"] == 0
    cm.reset()
    orc.reset()
    for _ in range(3):
        small, _, _ = zipf_keys(rng, 5000, 20, 16)
        sizes = sizes_u32(rng, 5000)
        cm.insert_keys(small, sizes)
        orc.insert_keys(small, sizes)
    cm.flush()
    assert_same_state(cm, orc)


def test_view_answers_the_state_at_refresh_while_ingesting(gpu, oracle):
    """configs[4] read side: heavy hitters and queries of a snapshot view run on
    another thread while the handle keeps inserting, and equal the oracle at the
    refresh point (count_min.go:160-247), not at whatever the ingest reached."""
    import threading
    from go2netspectra_amd import GnsError
    rng = np.random.default_rng(21)
    cm, orc = make_pair(oracle, 8192, 4, 16, st=20_000, ct=50)
    keys, flows, _ = zipf_keys(rng, 600_000, 30_000, 16)
    sizes = sizes_u32(rng, 600_000)
    a, b = 200_000, 600_000
    cm.insert_keys(keys[:a], sizes[:a])
    orc.insert_keys(keys[:a], sizes[:a])
    want_q = np.array([orc.query(bytes(f)) for f in flows[:3000]], dtype=np.uint64)
    want_c, want_s = orc.heavy("count"), orc.heavy("size")
    view = cm.view()
    with pytest.raises(GnsError):
        view.heavy_hitters()          # never refreshed
    view.refresh()                    # state after packets [0, a)
    results, errors = [], []

    def reader():
        try:
            for _ in range(6):
                hh = view.heavy_hitters()
                results.append(([(h.Flow, h.Count) for h in hh.Count], [(h.Flow, h.Size) for h in hh.Size],
                                view.query_many(flows[:3000])))
        except Exception as e:  # pragma: no cover - reported below
            errors.append(e)

    t = threading.Thread(target=reader)
    t.start()
    for lo in range(a, b, 50_000):   # ingest continues while the reader runs
        cm.insert_keys(keys[lo:lo + 50_000], sizes[lo:lo + 50_000])
    t.join()
    assert not errors, errors
    assert len(results) == 6
    for c, s, q in results:
        assert c == want_c and s == want_s
        assert np.array_equal(q, want_q)
    orc.insert_keys(keys[a:b], sizes[a:b])
    view.refresh()                    # now the whole stream
    hh = view.heavy_hitters()
    assert_same_list([(h.Flow, h.Count) for h in hh.Count], orc.heavy("count"))
    assert_same_list([(h.Flow, h.Size) for h in hh.Size], orc.heavy("size"))
    cm.flush()
    assert_same_state(cm, orc)
    cm.reset()
    with pytest.raises(GnsError):
        view.query_many(flows[:10])   # stale after reset until refreshed
    view.refresh()
    assert not view.query_many(flows[:10]).any()
    view.close()


def test_gathered_heavy_rows_order_on_device(gpu):
    """dist._canonical_rows on a GPU tensor (the RCCL path of the per-window exchange)
    orders like the host merge, ties beyond the first four key bytes included."""
    import torch
    from go2netspectra_amd.dist import _canonical_rows, merge_heavy_arrays
    rng = np.random.default_rng(17)
    for K in (4, 16, 37):
        n = 50_000
        rows = rng.integers(0, 256, (n, K + 4), dtype=np.uint8)
        rows[:, :4] = rng.integers(0, 3, (n, 4))   # long runs tied on the first bytes
        rows[:, K + 1:] = 0                         # values < 256: many ties
        rows = np.unique(rows, axis=0)
        rows = rows[np.unique(rows[:, :K], axis=0, return_index=True)[1]]  # disjoint flows
        rows = rows[rng.permutation(len(rows))]
        got = _canonical_rows(torch.from_numpy(rows).to("cuda"), K)
        vals = np.ascontiguousarray(rows[:, K:]).view("<u4").reshape(-1)
        wf, wv = merge_heavy_arrays(rows[:, :K], vals)
        assert np.array_equal(got[:, :K], wf)
        assert np.array_equal(np.ascontiguousarray(got[:, K:]).view("<u4").reshape(-1), wv)


@pytest.mark.parametrize("batch,w,d,K,max_flows", [
    (0, 2048, 2, 16, 16384), (40_000, 2048, 2, 16, 16384),
    (40_000, 512, 8, 37, 16384),  # 32-word records: the bucket cache of rows 0..7 moves with them
])
def test_unbounded_distinct_flows_reclaim(gpu, oracle, batch, w, d, K, max_flows):
    """Memory bounded like the reference (count_min.go:66-81 is fixed-size): more
    than 50x max_flows distinct flows in one period.  Flows no bucket names are
    reclaimed between batches; a batch whose new flows overflow the dictionary is
    undone, the dictionary rebuilt and the batch re-run in halves.  The state stays
    bit-exact, no GNS_E_FULL, and a snapshot view taken mid-stream keeps answering
    the state at its refresh across the reclaims (its ids are remapped too)."""
    rng = np.random.default_rng(91 + batch + d)  # live ids <= 2*d*w <= max_flows / 2
    cm, orc = make_pair(oracle, w, d, K, st=20_000, ct=30, max_flows=max_flows, batch_packets=batch)
    view = cm.view()
    heavy = rng.integers(0, 256, (300, K), dtype=np.uint8)
    want_view = None
    for part in range(6):
        n = 200_000
        uniq = rng.integers(0, 256, (n, K), dtype=np.uint8)
        keys = np.where((rng.random(n) < 0.8)[:, None], uniq, heavy[zipf_index(rng, n, 300)])
        sizes = sizes_u32(rng, n)
        cm.insert_keys(keys, sizes)
        orc.insert_keys(keys, sizes)
        if part == 2:
            view.refresh()
            want_view = (orc.heavy("count"), orc.heavy("size"),
                         np.array([orc.query(bytes(f)) for f in heavy], np.uint64))
    cm.flush()
    assert_same_state(cm, orc)
    ds = cm.dict_stats()
    assert ds["reclaims"] > 0 and ds["dropped"] > 50 * max_flows, ds
    assert cm.counters()["dict_full"] == 0
    hh = view.heavy_hitters()
    assert_same_list([(h.Flow, h.Count) for h in hh.Count], want_view[0])
    assert_same_list([(h.Flow, h.Size) for h in hh.Size], want_view[1])
    assert np.array_equal(view.query_many(heavy), want_view[2])
    assert_same_list([(h.Flow, h.Count) for h in cm.heavy_hitters().Count], orc.heavy("count"))
    view.close()


def _hh_from_state(C, F):
    """HeavyHitters (threshold 1) derived from exported bucket state: every flow named
    by a bucket with a nonzero value, at its largest value; value desc, flow bytes asc."""
    nz = C > 0
    v = C[nz].astype(np.int64)
    k = F[nz]
    key = k.copy().view(">u4").reshape(-1).astype(np.int64)  # 4-byte flows: byte order = big-endian value
    o = np.lexsort((-v, key))
    key, v = key[o], v[o]
    first = np.ones(len(key), bool)
    first[1:] = key[1:] != key[:-1]
    key, v = key[first], v[first]
    o = np.lexsort((key, -v))
    return key[o], v[o]


def test_heavy_hitters_beyond_2p26_candidates(gpu):
    """Verdict r2 #10: the heavy-hitter candidate buffer has no 2^26 cap.  d=8, w=2^24,
    thresholds 1: 20M distinct 4-byte flows in bursts of 1-4 packets (so a bucket's
    majority-vote count seldom cancels to 0) leave > 2^26 nonempty buckets per list, all
    candidates; both lists equal the ones derived from the exported state."""
    from go2netspectra_amd import CountMin
    nf = 20_000_000
    rng = np.random.default_rng(11)
    flows = rng.permutation(nf).astype("<u4")
    keys = np.repeat(flows, rng.integers(1, 5, nf)).view(np.uint8).reshape(-1, 4)
    n = len(keys)
    sizes = rng.integers(1, 1500, n).astype(np.uint32)
    seeds = np.random.default_rng(1).integers(0, 2**32, 8, dtype=np.uint64).astype(np.uint32)
    cm = CountMin(1 << 24, 8, 1, 1, key_bytes=4, seeds=seeds, max_flows=1 << 25)
    cm.insert_keys(keys, sizes)
    cm.flush()
    C, S, Fc, Fs = cm.export_state()
    assert int((C > 0).sum()) > (1 << 26) and int((S > 0).sum()) > (1 << 26)
    fc, c, fs, s = cm.heavy_hitters_arrays()
    for (f, v), (F, V) in (((fc, c), (Fc, C)), ((fs, s), (Fs, S))):
        wk, wv = _hh_from_state(V, F)
        assert len(v) == len(wv)
        got = np.ascontiguousarray(f[:, :4]).view(">u4").reshape(-1).astype(np.int64)
        bad = np.flatnonzero((got != wk) | (v.astype(np.int64) != wv))
        assert len(bad) == 0, f"first difference at {bad[0]}: got {got[bad[0]]},{v[bad[0]]} want {wk[bad[0]]},{wv[bad[0]]}"


@pytest.mark.parametrize("w,d,K,nflows,n,batch", [
    (65536, 4, 37, 50_000, 1_000_000, 0),
    (256, 2, 16, 2000, 100_000, 0),
    (1000, 3, 13, 5000, 200_000, 70_000),
    (1 << 20, 4, 37, 1 << 18, 2_000_000, 0),
])
def test_compact_streams_parity(gpu, oracle, monkeypatch, w, d, K, nflows, n, batch):
    """K1's compact cold / hot streams and K3c (GNS_CMODE=1, the measured A/B variant of
    DESIGN §10): the same bit-exact state as the per-packet code array."""
    monkeypatch.setenv("GNS_CMODE", "1")
    rng = np.random.default_rng(w + 11 * d)
    cm, orc = make_pair(oracle, w, d, K, batch_packets=batch)
    keys, _, _ = zipf_keys(rng, n, nflows, K)
    sizes = sizes_u32(rng, n, big_frac=0.01)
    cm.insert_keys(keys, sizes)
    cm.flush()
    orc.insert_keys(keys, sizes)
    assert_same_state(cm, orc)
    hh = cm.heavy_hitters()
    assert_same_list([(x.Flow, x.Count) for x in hh.Count], orc.heavy("count"))


@pytest.mark.parametrize("w", [16, 4096])
def test_compact_streams_hot_fallbacks(gpu, oracle, monkeypatch, w):
    """Ownership changes of designated buckets with compact streams: the block checks and
    the exact entry path read K1's hot streams (k_hot_blockcheck, k_hot_scatter_cs)."""
    monkeypatch.setenv("GNS_CMODE", "1")
    rng = np.random.default_rng(100 + w)
    cm, orc = make_pair(oracle, w, 2, 8, st=1 << 20, ct=100)
    flows = rng.integers(0, 256, (40, 8), dtype=np.uint8)
    for phase in range(5):
        m = 300_000
        heavy = np.full(m, phase % len(flows))
        idx = np.where(rng.random(m) < 0.7, heavy, rng.integers(0, len(flows), m))
        keys = np.ascontiguousarray(flows[idx])
        sizes = sizes_u32(rng, m)
        if phase == 3:
            sizes[::7] = rng.integers(1 << 21, 1 << 31, len(sizes[::7]))
        cm.insert_keys(keys, sizes)
        orc.insert_keys(keys, sizes)
        cm.flush()
        assert_same_state(cm, orc)


def test_heavy_rows_device_and_device_merge(gpu, oracle):
    """gns_cm_heavy_rows (the lists as device rows) equals gns_cm_heavy_hitters, and
    gns_hh_order_rows puts shuffled rows with many ties back in canonical order (value
    desc, flow bytes asc: dist.merge_heavy_arrays on the host)."""
    import torch
    from go2netspectra_amd.dist import merge_heavy_arrays, order_rows_device
    rng = np.random.default_rng(77)
    cm, orc = make_pair(oracle, 4096, 3, 13, st=2000, ct=20)
    keys, _, _ = zipf_keys(rng, 400_000, 6000, 13)
    sizes = sizes_u32(rng, 400_000)
    cm.insert_keys(keys, sizes)
    cm.flush()
    cf, cv, sf, sv = cm.heavy_hitters_arrays()
    cr, sr = cm.heavy_hitters_rows_device()
    for f, v, r in ((cf, cv, cr), (sf, sv, sr)):
        g = r.cpu().numpy()
        assert len(g) == len(v) > 0
        assert np.array_equal(g[:, :13], f) and np.array_equal(np.ascontiguousarray(g[:, 13:]).view("<u4").reshape(-1), v)
    # ties on (value, first four bytes) beyond them, several key widths
    for K in (4, 8, 13, 16, 37):
        n = 50_000
        flows = rng.integers(0, 256, (n, K), dtype=np.uint8)
        flows[: n // 2, : min(K, 4)] = rng.integers(0, 3, (n // 2, min(K, 4)), dtype=np.uint8)
        flows = np.unique(flows, axis=0)
        vals = rng.integers(0, 40, len(flows)).astype(np.uint32)
        vals[::5] = rng.integers(0, 2**32, len(vals[::5]), dtype=np.uint64).astype(np.uint32)
        perm = rng.permutation(len(flows))
        rows = np.concatenate([flows[perm], vals[perm].view(np.uint8).reshape(-1, 4)], axis=1)
        got = order_rows_device(torch.from_numpy(np.ascontiguousarray(rows)).cuda(), K).cpu().numpy()
        wf, wv = merge_heavy_arrays(flows, vals)
        assert np.array_equal(got[:, :K], wf), K
        assert np.array_equal(np.ascontiguousarray(got[:, K:]).view("<u4").reshape(-1), wv), K


def _mm3_words(words, seed):
    """MurmurHash3 x86_32 of 4-byte keys (statistic/hash.go:13-53), vectorized."""
    M = np.uint64(0xFFFFFFFF)
    rotl = lambda x, r: ((x << np.uint64(r)) | (x >> np.uint64(32 - r))) & M
    k = (words.astype(np.uint64) * np.uint64(0xCC9E2D51)) & M
    k = (rotl(k, 15) * np.uint64(0x1B873593)) & M
    h = rotl(np.uint64(seed) ^ k, 13)
    h = (h * np.uint64(5) + np.uint64(0xE6546B64)) & M
    h ^= np.uint64(4)
    h ^= h >> np.uint64(16)
    h = (h * np.uint64(0x85EBCA6B)) & M
    h ^= h >> np.uint64(13)
    h = (h * np.uint64(0xC2B2AE35)) & M
    return h ^ (h >> np.uint64(16))


@pytest.mark.parametrize("n2", [2_500_000, 4_000_000])
def test_superbin_many_rounds(gpu, oracle, n2):
    """One super-bin (w=2^23: bins of two 4096-bucket tiles) takes millions of cold updates of
    one batch: k_subpart groups ~300 / ~460 rounds by tile; K4 reads each tile through its
    runs from a per-tile table (2.5M) or, past one table, in windows of rounds in the second
    launch (4M: state stored and reloaded between windows)."""
    rng = np.random.default_rng(2323)
    w, d, K = 1 << 23, 2, 4
    cm, orc = make_pair(oracle, w, d, K, st=1 << 30, ct=1 << 30, batch_packets=1 << 23, max_flows=1 << 16)
    seeds = np.random.default_rng(1).integers(0, 2**32, d, dtype=np.uint64).astype(np.uint32)
    cand = np.unique(rng.integers(0, 2**32, 6_000_000, dtype=np.uint64).astype(np.uint32))
    h0 = _mm3_words(cand, int(seeds[0])) & np.uint64(w - 1)
    pick = cand[h0 < 8192][:3000]  # row 0: super-bin 0
    assert len(pick) == 3000
    for x in pick[:3]:
        assert oracle.mm3(int(x).to_bytes(4, "little"), int(seeds[0])) % w < 8192
    flows = pick.view(np.uint8).reshape(-1, 4)
    other = rng.integers(0, 256, (20_000, 4), dtype=np.uint8)
    n1 = 1_000_000
    k1 = np.concatenate([flows, other])[rng.integers(0, 23_000, n1)]
    k2 = flows[rng.integers(0, 3000, n2)]
    for keys in (k1, k2):
        keys = np.ascontiguousarray(keys)
        sizes = sizes_u32(rng, len(keys))
        sizes[::997] = 70_000
        cm.insert_keys(keys, sizes)
        orc.insert_keys(keys, sizes)
    cm.flush()
    assert_same_state(cm, orc)


@pytest.mark.parametrize("w,d,nflows", [(4096, 2, 6000), (1 << 16, 4, 120_000)])
def test_tiny_sizes_drain_size_counters(gpu, oracle, w, d, nflows):
    """Sizes drawn from {0, 1, 2, 3}: the size halves keep reaching S == 0 (a foreign update
    with s == S drains the bucket, the next one takes it over; a foreign size-0 update takes
    over only an empty bucket), which the aggregate check must never apply linearly
    (count_min.go:99-128).  Several batches, so buckets carry S == 0 into later chunks."""
    rng = np.random.default_rng(w + d)
    cm, orc = make_pair(oracle, w, d, 16, st=4, ct=50, batch_packets=200_000)
    keys, _, _ = zipf_keys(rng, 1_000_000, nflows, 16, s=0.9)
    sizes = rng.integers(0, 4, len(keys), dtype=np.uint64).astype(np.uint32)
    cm.insert_keys(keys, sizes)
    cm.flush()
    orc.insert_keys(keys, sizes)
    assert_same_state(cm, orc)


@pytest.mark.parametrize("sparse", ["1", "0"])
def test_contested_superbins_parity(gpu, oracle, monkeypatch, sparse):
    """Super-bin geometry (w = 2^22, d = 8: bins of two tiles) under heavy contention:
    1.5M flows over 4M buckets per row, so buckets change owners all the time, most
    chunks replay, and a chunk's replay list can outgrow the LDS copy (the fallback that
    re-reads updates and, in k_apply_sparse, maps them to their slots again).  One device
    batch of 3M packets with sizes that take the overflow table, then a second batch."""
    monkeypatch.setenv("GNS_K4_SPARSE", sparse)
    rng = np.random.default_rng(4404)
    n = 3_000_000
    cm, orc = make_pair(oracle, 1 << 22, 8, 8, st=1 << 12, ct=3, max_flows=1 << 22, batch_packets=n)
    keys, _, _ = zipf_keys(rng, n, 1_500_000, 8, s=0.6)
    sizes = sizes_u32(rng, n)
    sizes[::997] = 100_000
    cm.insert_keys(keys, sizes)
    orc.insert_keys(keys, sizes)
    keys2, _, _ = zipf_keys(rng, n // 3, 1_500_000, 8, s=0.6)
    sizes2 = sizes_u32(rng, n // 3)
    cm.insert_keys(keys2, sizes2)
    orc.insert_keys(keys2, sizes2)
    cm.flush()
    assert_same_state(cm, orc)
    assert cm.counters()["replayed"] > 0
