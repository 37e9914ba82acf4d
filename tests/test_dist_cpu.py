"""CPU, world_size 2 over gloo: the multi-GPU path's sharding + per-window
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


def test_two_rank_shard_and_allgather():
    import sys
    sys.path.insert(0, ROOT)
    from go2netspectra_amd.dist import merge_heavy
    from go2netspectra_amd.packets import PacketBatch
    world = 2
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


@pytest.mark.parametrize("world", [2, 3])
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
