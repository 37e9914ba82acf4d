"""configs[3] routing on the GPU: the device partition
(gns_route_partition) is the stable filter by owner shard
mm3(SrcIP slot, 0xA5A5A5A5) % G of the host restatement (dist.shard_of), and
each shard's stream through the engine equals the sequential oracle fed the
stable filter of the unsharded stream."""
import numpy as np
import pytest

from helpers import assert_same_list, frames_from_tuples, random_tuples

pytestmark = pytest.mark.gpu

FIVE = ["SrcIP", "DstIP", "SrcPort", "DstPort", "Protocol"]


def owner_of_records(oracle, hdr, wl, G):
    """Host owner shard per record: parse with the oracle; records it does not count go to 0."""
    from go2netspectra_amd.dist import shard_of
    src = np.zeros((len(wl), 16), np.uint8)
    ok = np.zeros(len(wl), bool)
    for i in range(len(wl)):
        st, s16, _, _, _, _ = oracle.parse_hdr64(bytes(hdr[i]), int(wl[i]))
        ok[i] = st == 0
        src[i] = np.frombuffer(s16, np.uint8)
    return np.where(ok, shard_of(src, G), 0)


@pytest.mark.parametrize("G", [1, 3, 8, 64])
def test_partition_is_the_stable_filter(gpu, oracle, G):
    import torch
    from go2netspectra_amd.dist import Router
    rng = np.random.default_rng(G)
    t = random_tuples(rng, 40_000, 3000, v6_frac=0.25)
    hdr = frames_from_tuples(t, rng, vlan_frac=0.3)
    hdr[rng.random(len(hdr)) < 0.02, 12:14] = [0x08, 0x06]  # ARP: dropped, owned by shard 0
    wl = t["length"]
    owner = owner_of_records(oracle, hdr, wl, G)
    r = Router(G)
    oh, ow, counts = r.partition(torch.from_numpy(hdr).cuda(), torch.from_numpy(wl.view(np.int32)).cuda())
    assert np.array_equal(counts, np.bincount(owner, minlength=G))
    order = np.argsort(owner, kind="stable")
    assert np.array_equal(oh.cpu().numpy(), hdr[order])
    assert np.array_equal(ow.cpu().numpy().view(np.uint32), wl[order])


def test_slices_exchanged_in_rank_order_are_the_filter(gpu, oracle):
    """The all-to-all of route_exchange, emulated in one process: G contiguous
    slices of the global stream, partitioned on the device, run g of every slice
    concatenated in slice order == stable filter of shard g."""
    import torch
    from go2netspectra_amd import SyntheticTraffic
    from go2netspectra_amd.dist import Router, shard_of
    G, n = 8, 3_000_000
    hdr, wl = SyntheticTraffic().generate(n)
    r = Router(G)
    runs = [[] for _ in range(G)]
    for sl in np.array_split(np.arange(n), G):
        oh, ow, counts = r.partition(hdr[sl[0]:sl[-1] + 1], wl[sl[0]:sl[-1] + 1])
        off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        for g in range(G):
            runs[g].append(oh[off[g]:off[g + 1]].cpu().numpy())
    h = hdr.cpu().numpy()
    owner = shard_of(np.pad(h[:, 26:30], ((0, 0), (0, 12))), G)
    for g in range(G):
        assert np.array_equal(np.concatenate(runs[g]), h[owner == g])


@pytest.mark.parametrize("g", [0, 5])
def test_shard_stream_through_engine_equals_oracle_on_filter(gpu, oracle, g):
    """verdict r2 #1b: SyntheticTraffic(shard=g, nshards=8), two consecutive windows
    through the engine == the oracle fed stream[shard_of(src) == g] of the unsharded
    stream (count_min.go:94-157 on the shard's sub-stream)."""
    import torch
    from go2netspectra_amd import CountMin, SyntheticTraffic
    from go2netspectra_amd.dist import shard_of
    G, n = 8, 400_000
    syn = SyntheticTraffic(shard=g, nshards=G)
    seeds = np.array([0xA1, 0xB2, 0xC3, 0xD4], np.uint32)
    cm = CountMin(1 << 16, 4, 1 << 20, 300, flow_fields=FIVE, seeds=seeds, max_flows=1 << 20)
    got = []
    for k in range(2):
        h, w = syn.generate(n, first=k * n)
        cm.insert_headers(h, w)
        got.append((h.cpu().numpy(), w.cpu().numpy().view(np.uint32)))
    cm.flush()
    gh, gw = SyntheticTraffic().generate(G * 2 * n + (1 << 21))  # enough of the global stream
    gh, gw = gh.cpu().numpy(), gw.cpu().numpy().view(np.uint32)
    owner = shard_of(np.pad(gh[:, 26:30], ((0, 0), (0, 12))), G)
    fh, fw = gh[owner == g][:2 * n], gw[owner == g][:2 * n]
    assert len(fw) == 2 * n
    assert np.array_equal(np.concatenate([x[0] for x in got]), fh)
    assert np.array_equal(np.concatenate([x[1] for x in got]), fw)
    orc = oracle.CountMin(1 << 16, 4, 1 << 20, 300, 37, seeds)
    assert orc.insert_hdr64(fh, fw, FIVE) == 2 * n
    C, S, Fc, Fs = cm.export_state()
    oC, oS, oFc, oFs = orc.export()
    assert np.array_equal(C, oC) and np.array_equal(S, oS)
    assert np.array_equal(Fc, oFc) and np.array_equal(Fs, oFs)
    hh = cm.heavy_hitters()
    assert_same_list([(x.Flow, x.Count) for x in hh.Count], orc.heavy("count"))


@pytest.mark.parametrize("owner_key", [["DstIP"], ["DstPort", "Protocol"], ["SrcIP", "DstIP", "SrcPort", "DstPort",
                                                                             "Protocol"]])
@pytest.mark.parametrize("G", [2, 7])
def test_keyed_partition_and_key_owners(gpu, oracle, owner_key, G):
    """A router built for an owner key other than [SrcIP] (the full key
    when SrcIP is not in the key): the device partition is the stable filter under
    dist.owner_of_tuples, and gns_route_owner_keys gives every flow key (host or
    device memory) the shard its packets went to; v4-mapped slots fold."""
    import torch
    from go2netspectra_amd.dist import Router, owner_of_keys, owner_of_tuples
    from go2netspectra_amd.packets import PacketBatch
    rng = np.random.default_rng(40 + G)
    t = random_tuples(rng, 30_000, 2000, v6_frac=0.25)
    hdr = frames_from_tuples(t, rng, vlan_frac=0.3)
    wl = t["length"]
    # the tuple the parser derives from each record (ports / protocol follow gopacket's
    # keep-on-error rules for short wire lengths, so they can differ from t's)
    ok = np.ones(len(wl), bool)
    pt = {"src16": np.zeros((len(wl), 16), np.uint8), "dst16": np.zeros((len(wl), 16), np.uint8),
          "sport": np.zeros(len(wl), np.uint16), "dport": np.zeros(len(wl), np.uint16), "proto": np.zeros(len(wl), np.uint8)}
    for i in range(len(wl)):
        st, s16, d16, sp, dp, pr = oracle.parse_hdr64(bytes(hdr[i]), int(wl[i]))
        ok[i] = st == 0
        pt["src16"][i], pt["dst16"][i] = np.frombuffer(s16, np.uint8), np.frombuffer(d16, np.uint8)
        pt["sport"][i], pt["dport"][i], pt["proto"][i] = sp, dp, pr
    own = np.where(ok, owner_of_tuples(pt["src16"], pt["dst16"], pt["sport"], pt["dport"], pt["proto"], G, owner_key), 0)
    r = Router(G, owner=owner_key)
    oh, ow, counts = r.partition(torch.from_numpy(hdr).cuda(), torch.from_numpy(wl.view(np.int32)).cuda())
    assert np.array_equal(counts, np.bincount(own, minlength=G))
    order = np.argsort(own, kind="stable")
    assert np.array_equal(oh.cpu().numpy(), hdr[order])
    # query keys of the 5-tuple task and of the owner key's own layout
    for fields in (owner_key, ["SrcIP", "DstIP", "SrcPort", "DstPort", "Protocol"], owner_key[::-1]):
        keys = PacketBatch(pt["src16"], pt["dst16"], pt["sport"], pt["dport"], pt["proto"], t["length"]).keys(fields)
        host = r.owner_of_keys(keys[ok], fields)
        assert np.array_equal(host, own[ok])
        assert np.array_equal(host, owner_of_keys(keys[ok], fields, G, owner_key))
        dev = r.owner_of_keys(torch.from_numpy(keys[ok]).cuda(), fields).cpu().numpy()
        assert np.array_equal(dev.astype(np.int64), host)
    mapped = np.zeros((50, 16), np.uint8)
    mapped[:, 10:12] = 0xFF
    mapped[:, 12:] = rng.integers(0, 256, (50, 4))
    v4 = np.zeros((50, 16), np.uint8)
    v4[:, :4] = mapped[:, 12:]
    if owner_key[0] == "DstIP":
        assert np.array_equal(r.owner_of_keys(mapped, ["DstIP"]), r.owner_of_keys(v4, ["DstIP"]))
    with pytest.raises(Exception, match="lacks owner field"):
        r.owner_of_keys(np.zeros((4, 2), np.uint8), ["SrcPort"])
