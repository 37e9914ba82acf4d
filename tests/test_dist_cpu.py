"""CPU, world_size 2..8 over gloo: the multi-GPU path's sharding + per-window
heavy-hitter all-gather.  Each rank runs an exact sketch of its flow shard
(the C oracle stands in for the GPU engine here) and the merged heavy-hitter
list must equal the union of the per-shard lists computed in one process."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _stream(n=20_000):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from helpers import random_tuples
    return random_tuples(np.random.default_rng(123), n, 400)


def _shard_sketch(batch, rank, world):
    from go2netspectra_amd.dist import split_batch
    from go2netspectra_amd.sketch import HeavyCount, HeavyRecord, HeavySize
    from oracle import oracle as orc
    part = split_batch(batch, world)[rank]
    cm = orc.CountMin(512, 3, 50_000, 40, 16, np.array([1, 2, 3], np.uint32))
    if len(part):
        cm.insert_keys(part.keys(["SrcIP"]), part.length)
    return HeavyRecord(Size=[HeavySize(f, v) for f, v in cm.heavy("size")],
                       Count=[HeavyCount(f, v) for f, v in cm.heavy("count")]), len(part)


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from go2netspectra_amd.dist import allgather_heavy, allgather_heavy_arrays
    from go2netspectra_amd.packets import PacketBatch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    t = _stream()
    batch = PacketBatch(t["src16"], t["dst16"], t["sport"], t["dport"], t["proto"], t["length"])
    hh, n = _shard_sketch(batch, rank, world)
    merged = allgather_heavy(hh, world)
    # the array form (CountMin.heavy_hitters_arrays -> bench.py's per-window exchange)
    def arr(items):
        f = np.array([np.frombuffer(x, np.uint8) for x, _ in items], np.uint8).reshape(len(items), 16)
        return f, np.array([v for _, v in items], np.uint32)
    cf, cv = arr([(h.Flow, h.Count) for h in hh.Count])
    sf, sv = arr([(h.Flow, h.Size) for h in hh.Size])
    ga = allgather_heavy_arrays((cf, cv, sf, sv), world)
    if rank == 0:
        q.put(([(h.Flow, h.Count) for h in merged.Count], [(h.Flow, h.Size) for h in merged.Size],
               [(bytes(f), int(v)) for f, v in zip(ga[0], ga[1])], [(bytes(f), int(v)) for f, v in zip(ga[2], ga[3])]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_shard_and_allgather(world):
    """world 8 = the node the driver's scaling run uses (8 x MI355X)."""
    import sys
    sys.path.insert(0, ROOT)
    from go2netspectra_amd.dist import merge_heavy
    from go2netspectra_amd.packets import PacketBatch
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got_c, got_s, arr_c, arr_s = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-process reference: union of the per-shard lists
    t = _stream()
    batch = PacketBatch(t["src16"], t["dst16"], t["sport"], t["dport"], t["proto"], t["length"])
    lists_c, lists_s, total = [], [], 0
    for r in range(world):
        hh, n = _shard_sketch(batch, r, world)
        lists_c.append([(h.Flow, h.Count) for h in hh.Count])
        lists_s.append([(h.Flow, h.Size) for h in hh.Size])
        total += n
    assert total == len(batch)
    assert got_c == merge_heavy(lists_c) and got_s == merge_heavy(lists_s)
    assert arr_c == got_c and arr_s == got_s
    assert len(got_c) > 0


# --- exact global mode: bucket-range slices, all-gathered -------
W_EX, D_EX, K_EX = 600, 3, 16   # width not divisible by the world size: uneven slices


def _full_state():
    from oracle import oracle as orc
    t = _stream(8_000)
    import sys
    sys.path.insert(0, ROOT)
    from go2netspectra_amd.packets import PacketBatch
    batch = PacketBatch(t["src16"], t["dst16"], t["sport"], t["dport"], t["proto"], t["length"])
    cm = orc.CountMin(W_EX, D_EX, 50_000, 40, K_EX, np.array([7, 8, 9], np.uint32))
    cm.insert_keys(batch.keys(["SrcIP"]), batch.length)
    return cm.export()


def _slice_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    from go2netspectra_amd.dist import allgather_slices, bucket_slice
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    # stand-in for CountMin(bucket_range=slice): the full sketch's columns inside
    # the slice, everything else untouched (zero)
    C, S, Fc, Fs = _full_state()
    lo, hi = bucket_slice(rank, world, W_EX)
    keep = np.zeros(D_EX * W_EX, bool)
    for r in range(D_EX):
        keep[r * W_EX + lo: r * W_EX + hi] = True
    mine = (np.where(keep, C, 0).astype(np.uint32), np.where(keep, S, 0).astype(np.uint32),
            np.where(keep[:, None], Fc, 0).astype(np.uint8), np.where(keep[:, None], Fs, 0).astype(np.uint8))
    g = allgather_slices(mine, rank, world, W_EX, D_EX)
    if rank == 0:
        q.put([a.copy() for a in g])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_bucket_slices_allgather(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_slice_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = _full_state()
    for g, w in zip(got, want):
        assert np.array_equal(g, w)
    assert want[0].any()


# --- configs[3] routing: each rank holds a contiguous slice of the stream, ----
# partitions it by owner shard and exchanges the runs (all-to-all); every rank
# must receive exactly the stable filter stream[shard_of(src) == rank] and its
# sketch must equal the oracle fed that filter.
def _route_stream(n=12_000):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from helpers import frames_from_tuples, random_tuples
    rng = np.random.default_rng(77)
    t = random_tuples(rng, n, 900)
    return frames_from_tuples(t), t["length"], t["src16"]


def _route_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from go2netspectra_amd.dist import exchange_runs, stable_split_records
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    hdr, wl, src = _route_stream()
    sl = np.array_split(np.arange(len(wl)), world)[rank]     # this rank's slice of the stream
    rh, rw, counts = stable_split_records(hdr[sl], wl[sl], world, src[sl])
    in_h, in_w = exchange_runs(torch.from_numpy(np.ascontiguousarray(rh)),
                               torch.from_numpy(np.ascontiguousarray(rw).view(np.int32)), counts, world)
    q.put((rank, in_h.numpy().copy(), in_w.numpy().view(np.uint32).copy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 8])
def test_route_exchange_delivers_the_stable_filter(world):
    import sys
    sys.path.insert(0, ROOT)
    from go2netspectra_amd.dist import shard_of
    from oracle import oracle as orc
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_route_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict((r, (h, w)) for r, h, w in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    hdr, wl, src = _route_stream()
    owner = shard_of(src, world)
    fields = ["SrcIP", "DstIP", "SrcPort", "DstPort", "Protocol"]
    seeds = np.array([5, 6, 7], np.uint32)
    total = 0
    for g in range(world):
        h, w = got[g]
        assert np.array_equal(h, hdr[owner == g]) and np.array_equal(w, wl[owner == g])
        total += len(w)
        a = orc.CountMin(1024, 3, 50_000, 20, 37, seeds)
        b = orc.CountMin(1024, 3, 50_000, 20, 37, seeds)
        a.insert_hdr64(h, w, fields)
        b.insert_hdr64(hdr[owner == g], wl[owner == g], fields)
        for x, y in zip(a.export(), b.export()):
            assert np.array_equal(x, y)
    assert total == len(wl)


# --- the owner key follows the tasks' flow keys, and queries are -----
# routed to the owner shard.  A key without SrcIP (legal, config.go:59) shards by
# the whole key; every rank's routed query must equal the answer of the shard
# holding the flow (the oracle fed that shard's stable filter).
def test_owner_fields_rule_c_equals_host():
    import ctypes as ct
    import sys
    sys.path.insert(0, ROOT)
    from go2netspectra_amd import _lib
    from go2netspectra_amd.dist import owner_fields
    L = _lib.load()
    cases = [[["SrcIP"]], [["SrcIP", "DstIP", "SrcPort", "DstPort", "Protocol"], ["SrcIP"]], [["DstIP"]],
             [["DstPort", "Protocol"]], [["Protocol", "DstPort", "DstIP"], ["DstPort", "Protocol"]],
             [["DstIP"], ["SrcIP"]], [["SrcPort"], ["DstPort"]], [["DstIP", "Bogus"], ["DstIP"]]]
    for tasks in cases:
        arr = (_lib.Layout * len(tasks))(*[_lib.Layout.of(t) for t in tasks])
        o = _lib.Layout()
        rc = L.gns_route_owner_fields(arr, len(tasks), ct.byref(o))
        try:
            want = owner_fields(tasks)
        except ValueError:
            want = None
        if want is None:
            assert rc == _lib.GNS_E_ARG and b"share no field" in L.gns_last_error()
        else:
            assert rc == 0 and o.names() == want, (tasks, o.names(), want)


def test_manager_owner_fields():
    import sys
    sys.path.insert(0, ROOT)
    from go2netspectra_amd.dist import owner_fields
    from go2netspectra_amd.factory import key_fields

    class T:  # stand-ins with the Task attributes the rule reads (no device needed)
        def __init__(self, f):
            self.flow_fields = f
    assert owner_fields([key_fields(T(["SrcIP", "DstIP"])), key_fields(T(["SrcIP"]))]) == ["SrcIP"]
    with pytest.raises(ValueError, match="share no field"):
        owner_fields([key_fields(T(["DstIP"])), key_fields(T(["SrcPort"]))])


def test_owner_folds_v4_mapped_slots():
    """An IPv4-mapped IPv6 slot and the IPv4 slot have one owner (the exact
    aggregator keys both as ::ffff:a.b.c.d, exact/task.go:330-366)."""
    import sys
    sys.path.insert(0, ROOT)
    from go2netspectra_amd.dist import owner_of_keys, owner_of_tuples, shard_of
    rng = np.random.default_rng(5)
    v4 = np.zeros((500, 16), np.uint8)
    v4[:, :4] = rng.integers(0, 256, (500, 4))
    mapped = np.zeros((500, 16), np.uint8)
    mapped[:, 10:12] = 0xFF
    mapped[:, 12:] = v4[:, :4]
    for G in (2, 3, 8):
        assert np.array_equal(shard_of(v4, G), shard_of(mapped, G))
        a = owner_of_keys(v4, ["DstIP"], G, ["DstIP"])
        b = owner_of_keys(mapped, ["DstIP"], G, ["DstIP"])
        c = owner_of_tuples(v4, mapped, None, None, None, G, ["DstIP"])
        assert np.array_equal(a, b) and np.array_equal(a, c)


KEYED_LAYOUTS = {"dstip": ["DstIP"], "dport_proto": ["DstPort", "Protocol"]}


def _keyed_stream(n=10_000):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from helpers import random_tuples
    return random_tuples(np.random.default_rng(91), n, 700)


def _keyed_queries(t, rank, fields):
    """rank's query batch: keys of stream packets (present flows) plus random keys."""
    import sys
    sys.path.insert(0, ROOT)
    from go2netspectra_amd.packets import PacketBatch
    b = PacketBatch(t["src16"], t["dst16"], t["sport"], t["dport"], t["proto"], t["length"])
    keys = b.keys(fields)
    rng = np.random.default_rng(1000 + rank)
    pick = keys[rng.integers(0, len(keys), 300 + 50 * rank)]
    junk = rng.integers(0, 256, (40, keys.shape[1]), dtype=np.uint8)
    return np.concatenate([pick, junk])


def _keyed_oracle(t, fields, world, g):
    """Oracle Count-Min fed shard g's stable filter under the task's owner key."""
    import sys
    sys.path.insert(0, ROOT)
    from go2netspectra_amd.dist import owner_fields, owner_of_tuples
    from go2netspectra_amd.packets import PacketBatch
    from oracle import oracle as orc
    own = owner_of_tuples(t["src16"], t["dst16"], t["sport"], t["dport"], t["proto"], world, owner_fields([fields]))
    m = own == g
    b = PacketBatch(t["src16"][m], t["dst16"][m], t["sport"][m], t["dport"][m], t["proto"][m], t["length"][m])
    keys = b.keys(fields)
    cm = orc.CountMin(256, 3, 50_000, 40, keys.shape[1], np.array([11, 12, 13], np.uint32))
    if len(b):
        cm.insert_keys(keys, b.length)
    return cm, m


def _keyed_worker(rank, world, port, layout, q):
    import sys
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from go2netspectra_amd.dist import exchange_runs, owner_fields, owner_of_tuples, routed_query
    from go2netspectra_amd.packets import PacketBatch
    from oracle import oracle as orc
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fields = KEYED_LAYOUTS[layout]
    owner = owner_fields([fields])
    t = _keyed_stream()
    sl = np.array_split(np.arange(len(t["length"])), world)[rank]  # this rank's slice of the stream
    own = owner_of_tuples(t["src16"][sl], t["dst16"][sl], t["sport"][sl], t["dport"][sl], t["proto"][sl], world, owner)
    order = np.argsort(own, kind="stable")
    counts = np.bincount(own, minlength=world)
    # the "records" exchanged are the packets' indices in the global stream (int64 rows)
    idx = torch.from_numpy(np.ascontiguousarray(sl[order]).astype(np.int64).view(np.uint8).reshape(-1, 8))
    got, _ = _exchange_rows(idx, counts, world)
    got = got.numpy().view(np.int64).reshape(-1)
    b = PacketBatch(t["src16"][got], t["dst16"][got], t["sport"][got], t["dport"][got], t["proto"][got],
                    t["length"][got])
    keys = b.keys(fields)
    cm = orc.CountMin(256, 3, 50_000, 40, keys.shape[1], np.array([11, 12, 13], np.uint32))
    if len(b):
        cm.insert_keys(keys, b.length)
    qk = _keyed_queries(t, rank, fields)
    ans = routed_query(lambda ks: np.array([cm.query(bytes(k)) for k in ks], np.uint64), qk, fields, world, owner)
    # a rank with nothing to ask still takes part in the collective
    empty = routed_query(lambda ks: np.array([cm.query(bytes(k)) for k in ks], np.uint64),
                         qk[:0] if rank == 0 else qk[:7], fields, world, owner)
    q.put((rank, got.copy(), ans.copy(), empty.copy()))
    dist.barrier()
    dist.destroy_process_group()


def _exchange_rows(rows, counts, world):
    """exchange_runs for fixed-width rows of any byte width (the index rows of the test)."""
    import torch
    import torch.distributed as dist
    send = torch.tensor([int(c) for c in counts], dtype=torch.int64)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send)
    sc, rc = send.tolist(), recv.tolist()
    out = torch.empty((sum(rc), rows.shape[1]), dtype=rows.dtype)
    dist.all_to_all_single(out, rows, output_split_sizes=rc, input_split_sizes=sc)
    return out, rc


@pytest.mark.parametrize("world", [2, 3, 8])
@pytest.mark.parametrize("layout", sorted(KEYED_LAYOUTS))
def test_keyed_sharding_and_routed_queries(world, layout):
    import sys
    sys.path.insert(0, ROOT)
    from go2netspectra_amd.dist import owner_fields, owner_of_keys
    fields = KEYED_LAYOUTS[layout]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_keyed_worker, args=(r, world, port, layout, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict((r, (g, a, e)) for r, g, a, e in (q.get(timeout=120) for _ in range(world)))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    t = _keyed_stream()
    shards = [_keyed_oracle(t, fields, world, g) for g in range(world)]
    total = 0
    for g in range(world):
        got, _, _ = res[g]
        assert np.array_equal(got, np.flatnonzero(shards[g][1]))  # the full-key stable filter, in order
        total += len(got)
    assert total == len(t["length"])
    owner = owner_fields([fields])
    nonzero = 0
    for r in range(world):
        qk = _keyed_queries(t, r, fields)
        own = owner_of_keys(qk, fields, world, owner)
        want = np.array([shards[o][0].query(bytes(k)) for o, k in zip(own, qk)], np.uint64)
        assert np.array_equal(res[r][1], want)
        nonzero += int((want != 0).sum())
        e = res[r][2]
        assert len(e) == (0 if r == 0 else 7) and np.array_equal(e, want[:len(e)])
    assert nonzero > 0
    # a flow never splits: every packet of one flow key went to one shard
    from go2netspectra_amd.packets import PacketBatch
    b = PacketBatch(t["src16"], t["dst16"], t["sport"], t["dport"], t["proto"], t["length"])
    keys = b.keys(fields)
    where = np.zeros(len(keys), np.int64)
    for g in range(world):
        where[shards[g][1]] = g
    _, inv = np.unique(keys, axis=0, return_inverse=True)
    for u in range(inv.max() + 1):
        assert len(set(where[inv.reshape(-1) == u])) == 1
