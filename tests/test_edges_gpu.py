"""Edge cases of the insert / query surface on the GPU, each against the
sequential C oracle: empty batches, ragged batch sizes around every internal
block size (K1 blocks of 16384 packets, K3s sub-passes of 8192, 256-packet
waves), a sketch that saw nothing, and the same stream cut into batches in
different places (the result must not depend on where a batch ends)."""
import numpy as np
import pytest

from helpers import assert_same_flows, frames_from_tuples, random_tuples, sizes_u32, zipf_keys

pytestmark = pytest.mark.gpu

RAGGED = [1, 63, 64, 65, 255, 257, 8191, 8193, 16383, 16385, 40_000, 1]


def _cm_pair(oracle, w=4096, d=4, K=16, st=20_000, ct=40, **kw):
    from go2netspectra_amd import CountMin
    seeds = np.random.default_rng(7).integers(0, 2**32, d, dtype=np.uint64).astype(np.uint32)
    return CountMin(w, d, st, ct, key_bytes=K, seeds=seeds, **kw), oracle.CountMin(w, d, st, ct, K, seeds)


def _same_cm(cm, orc):
    got, want = cm.export_state(), orc.export()
    for name, a, b in zip(("C", "S", "FPc", "FPs"), got, want):
        assert np.array_equal(a, b), name


def test_cm_empty_batches_and_empty_sketch(gpu, oracle):
    cm, orc = _cm_pair(oracle)
    cm.insert_keys(np.zeros((0, 16), np.uint8), np.zeros(0, np.uint32))
    cm.flush()
    _same_cm(cm, orc)
    assert cm.query_many(np.zeros((0, 16), np.uint8)).shape == (0,)
    assert not cm.query_many(np.ones((5, 16), np.uint8)).any()
    hh = cm.heavy_hitters()
    assert hh.Count == [] and hh.Size == [] and hh.Size is not None  # count_min.go:210 non-nil Size
    view = cm.view()
    view.refresh()
    assert view.heavy_hitters().Count == []
    view.close()
    from go2netspectra_amd import PacketBatch
    t = random_tuples(np.random.default_rng(1), 10, 5)
    empty = PacketBatch(t["src16"][:0], t["dst16"][:0], t["sport"][:0], t["dport"][:0], t["proto"][:0],
                        t["length"][:0])
    cm2, _ = _cm_pair(oracle, K=37)
    cm2.insert_tuples(empty)
    cm2.insert_headers(np.zeros((0, 64), np.uint8), np.zeros(0, np.uint32))
    cm2.flush()


@pytest.mark.parametrize("batch", [0, 16384, 24576])
def test_cm_ragged_batches(gpu, oracle, batch):
    """Calls of ragged sizes (and device batches of 16384 / 24576 packets inside a call):
    the state equals one sequential pass over the concatenated stream."""
    rng = np.random.default_rng(batch + 3)
    cm, orc = _cm_pair(oracle, batch_packets=batch)
    n = sum(RAGGED)
    keys, _, _ = zipf_keys(rng, n, 3000, 16)
    sizes = sizes_u32(rng, n)
    off = 0
    for m in RAGGED:
        cm.insert_keys(keys[off:off + m], sizes[off:off + m])
        off += m
    cm.flush()
    orc.insert_keys(keys, sizes)
    _same_cm(cm, orc)


def test_cm_cut_points_do_not_matter(gpu, oracle):
    """The same 5-tuple header stream inserted as one call and as many ragged calls."""
    rng = np.random.default_rng(11)
    t = random_tuples(rng, 60_000, 2500)
    hdr, wl = frames_from_tuples(t), t["length"]
    fields = ["SrcIP", "DstIP", "SrcPort", "DstPort", "Protocol"]
    from go2netspectra_amd import CountMin
    seeds = np.arange(1, 5, dtype=np.uint32) * 0x9E3779B1
    a = CountMin(65536, 4, 50_000, 50, flow_fields=fields, seeds=seeds)
    b = CountMin(65536, 4, 50_000, 50, flow_fields=fields, seeds=seeds)
    a.insert_headers(hdr, wl)
    cuts = np.sort(rng.choice(np.arange(1, len(wl)), 17, replace=False))
    for lo, hi in zip(np.r_[0, cuts], np.r_[cuts, len(wl)]):
        b.insert_headers(hdr[lo:hi], wl[lo:hi])
    a.flush(); b.flush()
    for x, y in zip(a.export_state(), b.export_state()):
        assert np.array_equal(x, y)
    orc = oracle.CountMin(65536, 4, 50_000, 50, 37, seeds)
    orc.insert_hdr64(hdr, wl, fields)
    _same_cm(a, orc)


def test_ss_empty_and_ragged(gpu, oracle):
    from go2netspectra_amd import SuperSpread
    seeds = np.array([3, 5], np.uint32)
    ss = SuperSpread(512, 2, 20, 32, 5, 0.5, 1.08, flow_bytes=16, elem_bytes=16, seeds=seeds,
                     hll_master=1, rng_seed=2)
    orc = oracle.SuperSpread(512, 2, 20, 32, 5, 0.5, 1.08, 16, 16, seeds, 1, 2)
    ss.insert_keys(np.zeros((0, 16), np.uint8), np.zeros((0, 16), np.uint8))
    ss.flush()
    assert ss.heavy_hitters().Count == [] and ss.heavy_hitters().Size is None
    rng = np.random.default_rng(5)
    n = sum(RAGGED)
    fl, _, _ = zipf_keys(rng, n, 500, 16)
    el = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    off = 0
    for m in RAGGED:
        ss.insert_keys(fl[off:off + m], el[off:off + m])
        off += m
    ss.flush()
    orc.insert(fl, el)
    got, want = ss.export_state(), orc.export()
    for name, a, b in zip(("values", "keys", "regs", "pbits"), got, want):
        same = np.array_equal(a.view(np.uint64), b.view(np.uint64)) if name == "pbits" else np.array_equal(a, b)
        assert same, name


def test_exact_empty_and_ragged(gpu, oracle):
    from go2netspectra_amd import ExactTask, PacketBatch
    five = ["SrcIP", "DstIP", "SrcPort", "DstPort", "Protocol"]
    rng = np.random.default_rng(9)
    n = sum(RAGGED)
    t = random_tuples(rng, n, 3000)
    ts = np.arange(n, dtype=np.int64) * 7
    task = ExactTask("ragged", five)
    task.process_packets(PacketBatch(t["src16"][:0], t["dst16"][:0], t["sport"][:0], t["dport"][:0],
                                     t["proto"][:0], t["length"][:0], None, ts[:0]))
    task.flush()
    assert task.flows() == []
    off = 0
    for m in RAGGED:
        sl = slice(off, off + m)
        task.process_packets(PacketBatch(t["src16"][sl], t["dst16"][sl], t["sport"][sl], t["dport"][sl],
                                         t["proto"][sl], t["length"][sl], None, ts[sl]))
        off += m
    task.flush()
    orc = oracle.Exact(five)
    ipver = np.full(n, 4, np.uint8)
    orc.insert_tuples(t["src16"], t["dst16"], t["sport"], t["dport"], t["proto"], ipver, t["length"], ts)
    got = {f.Key: (f.StartTime, f.EndTime, f.PacketCount, f.ByteCount) for f in task.flows()}
    assert_same_flows(got, orc.export())
