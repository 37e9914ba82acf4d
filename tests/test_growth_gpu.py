"""The engine keeps counting wherever the reference does (count_min.go:47-81,94-157
and super_spread.go:182-235 have no failure mode), and the configuration the
bench times is itself parity-checked.

- uniform traffic shaped like scripts/pcapgen/main.go:17-97 (every packet a new
  flow) into sketches whose live ids outgrow the INITIAL dictionary: the table
  grows, no error, state bit-exact against the sequential oracle;
- one device batch with more than 2^22 packets whose size takes the overflow
  side table (>= 2^16-1): the table grows with the batch;
- the headline handle settings (d=4 w=2^20, 5-tuple key, max_flows 2^22,
  64M-packet device batches) over two consecutive 64M-packet windows of the
  synthetic Zipf stream: the heaviest flow's size counter wraps 2^32 inside a
  batch while its buckets are designated (the summary-path wrap proof of
  DESIGN.md §4) and designation carries across windows; full state and both
  heavy-hitter lists equal the oracle's.
"""
import numpy as np
import pytest

from helpers import assert_same_list, pcapgen_records, sizes_u32, zipf_keys

pytestmark = pytest.mark.gpu

FIVE = ["SrcIP", "DstIP", "SrcPort", "DstPort", "Protocol"]


def _bench_row_seeds(d):
    """bench.py row_seeds: splitmix64 stream from 0x9747B28C."""
    s, out = 0x9747B28C, []
    for _ in range(d):
        s = (s + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        z = ((s ^ (s >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        out.append((z ^ (z >> 31)) & 0xFFFFFFFF)
    return np.array(out, np.uint32)


def _same_cm(cm, orc):
    got, want = cm.export_state(), orc.export()
    for name, a, b in zip(("C", "S", "FPc", "FPs"), got, want):
        if not np.array_equal(a, b):
            bad = np.nonzero(a != b)[0] if a.ndim == 1 else np.nonzero((a != b).any(axis=1))[0]
            raise AssertionError(f"{name} differs in {len(bad)} cells, first {bad[:5]}")


def test_unique_flows_grow_countmin(gpu, oracle):
    """5.2M pcapgen-style packets (unique flows) into CM d=4 w=2^16 starting from a
    2^16-flow dictionary: live ids reach ~2*d*w = 512K, so the table must grow."""
    from go2netspectra_amd import CountMin
    rng = np.random.default_rng(404)
    seeds = np.array([0x9747B28C, 0x1B873593, 0xCC9E2D51, 0x85EBCA6B], np.uint32)
    cm = CountMin(1 << 16, 4, 1 << 20, 100, flow_fields=FIVE, seeds=seeds, max_flows=1 << 16)
    orc = oracle.CountMin(1 << 16, 4, 1 << 20, 100, 37, seeds)
    for part in range(4):
        hdr, wl = pcapgen_records(rng, 1_300_000)
        cm.insert_headers(hdr, wl)
        assert orc.insert_hdr64(hdr, wl, FIVE) == len(wl)
    cm.flush()
    _same_cm(cm, orc)
    ds = cm.dict_stats()
    assert ds["growths"] > 0 and ds["slots"] >= 1 << 19, ds
    assert ds["live"] > (1 << 17), ds          # live ids well past the initial 2^16 capacity
    assert cm.counters()["dict_full"] == 0
    assert cm.stats()["inserted"] == 5_200_000
    hh = cm.heavy_hitters()
    assert_same_list([(h.Flow, h.Count) for h in hh.Count], orc.heavy("count"))
    assert_same_list([(h.Flow, h.Size) for h in hh.Size], orc.heavy("size"))


def test_unique_flows_grow_superspread(gpu, oracle):
    """The default SuperSpread task (SrcIP -> DstIP, d=2, w=32768, m=128) under 5M
    packets from unique sources, starting from a 4096-flow dictionary: cell owners
    (up to d*w = 65536 live ids) outgrow it; the table grows; bit-exact."""
    from go2netspectra_amd import SuperSpread
    rng = np.random.default_rng(405)
    seeds = np.array([0x1234, 0x5678], np.uint32)
    hm, rs = 0x0123456789ABCDEF, 0x0DDBA11CAFEF00D5
    ss = SuperSpread(32768, 2, 4096, 128, 5, 0.5, 1.08, flow_fields=["SrcIP"], elem_fields=["DstIP"],
                     seeds=seeds, hll_master=hm, rng_seed=rs, max_flows=4096)
    orc = oracle.SuperSpread(32768, 2, 4096, 128, 5, 0.5, 1.08, 16, 16, seeds, hm, rs)
    for part in range(2):
        hdr, wl = pcapgen_records(rng, 2_500_000)
        ss.insert_headers(hdr, wl)
        assert orc.insert_hdr64(hdr, wl, ["SrcIP"], ["DstIP"]) == len(wl)
    ss.flush()
    got, want = ss.export_state(), orc.export()
    for name, a, b in zip(("values", "keys", "regs", "pbits"), got, want):
        same = np.array_equal(a.view(np.uint64), b.view(np.uint64)) if name == "pbits" else np.array_equal(a, b)
        assert same, name
    ds = ss.dict_stats()
    assert ds["growths"] > 0 and ds["live"] > 8192, ds
    assert ss.counters()["dict_full"] == 0
    assert_same_list([(h.Flow, h.Count) for h in ss.heavy_hitters().Count], orc.heavy())


def test_oversize_packets_beyond_old_batch_cap(gpu, oracle):
    """One device batch of 4.5M packets, every size >= 2^16-1 (TSO/GRO-sized), d=2:
    9M overflow-table updates, more than twice the old fixed 2^22 table."""
    from go2netspectra_amd import CountMin
    rng = np.random.default_rng(406)
    seeds = np.array([77, 88], np.uint32)
    cm = CountMin(4096, 2, 1 << 30, 100, key_bytes=8, seeds=seeds, batch_packets=8 << 20)
    orc = oracle.CountMin(4096, 2, 1 << 30, 100, 8, seeds)
    warm, _, _ = zipf_keys(rng, 1000, 50, 8)
    ws = sizes_u32(rng, 1000)
    cm.insert_keys(warm, ws)          # warm handle: the next call is ONE device batch
    orc.insert_keys(warm, ws)
    n = 4_500_000
    keys, _, _ = zipf_keys(rng, n, 20_000, 8)
    sizes = rng.integers(0xFFFF, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    sizes[::13] = 0xFFFF
    cm.insert_keys(keys, sizes)
    orc.insert_keys(keys, sizes)
    cm.flush()                        # GNS_E_RANGE before: more than 2^22 oversize updates
    _same_cm(cm, orc)
    assert cm.counters()["ovf_full"] == 0


def test_headline_configuration_two_full_windows(gpu, oracle):
    """BASELINE configs[1] as bench.py times it: d=4 w=2^20, 5-tuple (37 B), size /
    count thresholds 2^20 / 1000, bench row seeds, max_flows 2^22, 64M-packet device
    batches, two consecutive fresh 64M-packet windows of the synthetic Zipf(1.1)
    stream.  Full state + both heavy-hitter lists equal the oracle after each window."""
    import torch
    from go2netspectra_amd import CountMin, SyntheticTraffic
    n = 64 << 20
    seeds = _bench_row_seeds(4)
    syn = SyntheticTraffic()
    dev = torch.device("cuda", 0)
    hdr = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    wl = torch.empty((n,), dtype=torch.int32, device=dev)
    cm = CountMin(1 << 20, 4, 1 << 20, 1000, flow_fields=FIVE, seeds=seeds, max_flows=1 << 22, batch_packets=n)
    orc = oracle.CountMin(1 << 20, 4, 1 << 20, 1000, 37, seeds)
    for k in range(2):
        syn.fill(hdr, wl, first=k * n)
        torch.cuda.synchronize()
        # the heaviest flow's bytes in this window exceed 2^32: its S wraps inside the batch
        key = (hdr[:, 26:38].to(torch.int64) * torch.tensor([1 << (5 * i) for i in range(12)], device=dev)).sum(1)
        uniq, inv, cnt = torch.unique(key, return_inverse=True, return_counts=True)
        top = int(torch.argmax(cnt))
        top_bytes = int(wl.to(torch.int64)[inv == top].sum())
        del key, uniq, inv, cnt
        assert top_bytes > 1 << 32, top_bytes
        cm.insert_headers(hdr, wl)
        cm.flush()
        h = hdr.cpu().numpy()
        w = wl.cpu().numpy().view(np.uint32)
        assert orc.insert_hdr64(h, w, FIVE) == n
        del h, w
        _same_cm(cm, orc)
        hh = cm.heavy_hitters()
        assert_same_list([(x.Flow, x.Count) for x in hh.Count], orc.heavy("count"))
        assert_same_list([(x.Flow, x.Size) for x in hh.Size], orc.heavy("size"))
    assert cm.stats()["inserted"] == 2 * n
    assert cm.counters()["dict_full"] == 0
