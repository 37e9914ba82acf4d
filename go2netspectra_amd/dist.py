"""Multi-GPU sharding of the sketch path (one process per GPU, torch.distributed).

Count-Min buckets are (fingerprint, counter) pairs under order-dependent
majority-vote rules (count_min.go:99-155): they are NOT additive, so summing
counter rows across GPUs (all-reduce) would not produce the sketch of the
union stream.  The path therefore shards by flow: every packet
goes to the GPU that owns its flow, each GPU runs an exact sketch of its
sub-stream, queries go to the owner shard (routed_query), and the only
collective on the data path is the per-window all-gather of heavy-hitter
candidates (flows are disjoint across shards, so the global list is a union).

Ownership.  A flow key is the task's configured fields (task.go:265-300; any
non-empty field list is legal, config.go:59).  The owner key is a set of fields
that EVERY task of the Manager keys on, so that every flow of every task lands
on one shard (owner_fields):
  * [SrcIP] when every task's key contains SrcIP (the default tasks and
    BASELINE configs[3], "sharded by src-IP": every flow of a source shares a GPU);
  * otherwise the fields the tasks share, in canonical order -- for one task its
    whole flow key, e.g. ["DstIP"] or ["DstPort", "Protocol"];
  * no shared field: no owner exists, ValueError.
owner = mm3(owner key, 0xA5A5A5A5) % world, with every IP slot folded
(an IPv4-mapped IPv6 slot hashes as the IPv4 slot), so the owner is a function
of the EncodeFlow bytes and of the exact aggregator's To16 key alike.  The
device form is gns_route.hip (Router); the functions here are its host
restatement (CPU tests, host-side splits).
"""
from __future__ import annotations

import numpy as np

from .sketch import HeavyCount, HeavyRecord, HeavySize

SHARD_SEED = 0xA5A5A5A5
CANON_FIELDS = ["SrcIP", "DstIP", "SrcPort", "DstPort", "Protocol"]
_FIELD_SIZE = {"SrcIP": 16, "DstIP": 16, "SrcPort": 2, "DstPort": 2, "Protocol": 1}


def _mm3_rows(rows: np.ndarray, seed: int) -> np.ndarray:
    """MurmurHash3_x86_32 of every row of a [n, K] uint8 array (vectorised; hash.go:13-53)."""
    rows = np.ascontiguousarray(rows, np.uint8)
    n, K = rows.shape
    c1, c2 = np.uint32(0xCC9E2D51), np.uint32(0x1B873593)
    pad = np.zeros((n, (K + 3) // 4 * 4), np.uint8)
    pad[:, :K] = rows
    w = pad.view("<u4").reshape(n, pad.shape[1] // 4)
    h = np.full(n, seed, np.uint32)
    with np.errstate(over="ignore"):
        for i in range(K // 4):
            k = w[:, i].astype(np.uint32) * c1
            k = (k << np.uint32(15)) | (k >> np.uint32(17))
            k = k * c2
            h ^= k
            h = (h << np.uint32(13)) | (h >> np.uint32(19))
            h = h * np.uint32(5) + np.uint32(0xE6546B64)
        if K & 3:
            k = w[:, K // 4].astype(np.uint32) * c1
            k = (k << np.uint32(15)) | (k >> np.uint32(17))
            h ^= k * c2
        h ^= np.uint32(K)
        h ^= h >> np.uint32(16)
        h = h * np.uint32(0x85EBCA6B)
        h ^= h >> np.uint32(13)
        h = h * np.uint32(0xC2B2AE35)
        h ^= h >> np.uint32(16)
    return h


def _mm3_16(slots: np.ndarray, seed: int) -> np.ndarray:
    return _mm3_rows(np.asarray(slots, np.uint8).reshape(-1, 16), seed)


def canon_slots(a16: np.ndarray) -> np.ndarray:
    """[n, 16] IP slots with IPv4-mapped IPv6 (::ffff:a.b.c.d) folded to the IPv4 slot."""
    a = np.array(a16, np.uint8, copy=True).reshape(-1, 16)
    m = (a[:, :10] == 0).all(axis=1) & (a[:, 10] == 0xFF) & (a[:, 11] == 0xFF)
    a[m, :4] = a[m, 12:16]
    a[m, 4:] = 0
    return a


def owner_fields(task_fields) -> list:
    """The owner key of a set of tasks (gns_route_owner_fields): [SrcIP] when every
    task keys on SrcIP, else the fields all tasks share in canonical order.
    task_fields: one field list per task (sketch FlowFields / exact KeyFields)."""
    sets = [set(f for f in (fs or []) if f in _FIELD_SIZE) for fs in task_fields]
    if not sets:
        raise ValueError("no tasks to shard")
    if all("SrcIP" in fs for fs in sets):
        return ["SrcIP"]
    common = [f for f in CANON_FIELDS if all(f in fs for fs in sets)]
    if not common:
        raise ValueError(f"the tasks' flow keys {[list(fs or []) for fs in task_fields]} share no field: no shard "
                         "owns every flow of every task (shard each task set on its own router)")
    return common


def _owner_key(fields: dict, owner: list) -> np.ndarray:
    """Owner key rows from per-field byte arrays (IP slots folded)."""
    parts = []
    for f in owner:
        a = np.asarray(fields[f], np.uint8)
        parts.append(canon_slots(a) if f in ("SrcIP", "DstIP") else (a if a.ndim == 2 else a.reshape(-1, 1)))
    return np.ascontiguousarray(np.concatenate(parts, axis=1))


def owner_of_tuples(src16, dst16, sport, dport, proto, world: int, owner=("SrcIP",)) -> np.ndarray:
    """Owner shard of every packet (PacketInfo fields as EncodeFlow lays them out)."""
    n = len(np.asarray(src16).reshape(-1, 16))
    if world <= 1:
        return np.zeros(n, np.int64)
    fields = {"SrcIP": src16, "DstIP": dst16,
              "SrcPort": np.asarray(sport, ">u2").view(np.uint8).reshape(-1, 2) if sport is not None else None,
              "DstPort": np.asarray(dport, ">u2").view(np.uint8).reshape(-1, 2) if dport is not None else None,
              "Protocol": np.asarray(proto, np.uint8).reshape(-1, 1) if proto is not None else None}
    return (_mm3_rows(_owner_key(fields, list(owner)), SHARD_SEED) % np.uint32(world)).astype(np.int64)


def owner_of_keys(keys, key_fields, world: int, owner=("SrcIP",)) -> np.ndarray:
    """Owner shard of flow keys [n, K] laid out as key_fields (a task's EncodeFlow bytes):
    the shard whose sketch holds the flow (gns_route_owner_keys on the device)."""
    keys = np.ascontiguousarray(keys, np.uint8)
    if keys.ndim != 2:
        keys = keys.reshape(keys.shape[0], -1) if keys.size else np.zeros((len(keys), 0), np.uint8)
    fields, off = {}, 0
    for f in key_fields:
        sz = _FIELD_SIZE.get(f, 0)
        fields.setdefault(f, keys[:, off:off + sz])
        off += sz
    missing = [f for f in owner if f not in fields]
    if missing:
        raise ValueError(f"key fields {list(key_fields)} lack owner field(s) {missing}")
    if world <= 1:
        return np.zeros(keys.shape[0], np.int64)
    return (_mm3_rows(_owner_key(fields, list(owner)), SHARD_SEED) % np.uint32(world)).astype(np.int64)


def shard_of(src16: np.ndarray, world: int) -> np.ndarray:
    """Owner GPU of each packet under the [SrcIP] owner key: mm3(SrcIP slot, 0xA5A5A5A5) % world."""
    if world <= 1:
        return np.zeros(len(src16), np.int64)
    return (_mm3_16(canon_slots(src16), SHARD_SEED) % np.uint32(world)).astype(np.int64)


def split_batch(batch, world: int, owner=("SrcIP",)):
    """Stable split of a host PacketBatch into per-shard batches (order kept)."""
    from .packets import PacketBatch
    own = owner_of_tuples(batch.src16, batch.dst16, batch.sport, batch.dport, batch.proto, world, owner)
    out = []
    for g in range(world):
        m = own == g
        out.append(PacketBatch(batch.src16[m], batch.dst16[m], batch.sport[m], batch.dport[m],
                               batch.proto[m], batch.length[m],
                               None if batch.ipver is None else batch.ipver[m],
                               None if batch.ts is None else batch.ts[m]))
    return out


class Router:
    """Device-side stable partition of header records by owner shard
    (gns_route_partition; the device form of owner_of_tuples / split_batch) and
    the owner of query keys (gns_route_owner_keys)."""

    def __init__(self, nshards: int, device: int = 0, owner=("SrcIP",)):
        import ctypes as ct
        from . import _lib
        self._L = _lib.load()
        self.nshards = int(nshards)
        self.device = device
        self.owner = list(owner)
        h = ct.c_void_p()
        lay = _lib.Layout.of(self.owner)
        _lib.check(self._L.gns_route_create_keyed(self.nshards, ct.byref(lay), device, ct.byref(h)))
        self._h = h

    def owner_of_keys(self, keys, key_fields):
        """Owner shard of flow keys [n, K] laid out as key_fields (host numpy -> numpy int64;
        a device tensor -> a device int32 tensor)."""
        import ctypes as ct
        from . import _lib
        lay = _lib.Layout.of(list(key_fields))
        if hasattr(keys, "data_ptr") and getattr(keys, "is_cuda", False):
            import torch
            n = int(keys.shape[0])
            out = torch.empty((n,), dtype=torch.int32, device=keys.device)
            if n == 0:
                return out
            keys = keys.reshape(n, -1).contiguous()
            _lib.device_ready(keys)
            _lib.check(self._L.gns_route_owner_keys(self._h, ct.byref(lay), keys.data_ptr(), int(keys.shape[1]) if n else 1,
                                                    n, out.data_ptr(), _lib.MEM_DEVICE))
            return out
        keys = np.ascontiguousarray(keys, np.uint8)
        n = keys.shape[0]
        keys = keys.reshape(n, -1) if n else np.zeros((0, max(_lib.layout_bytes(key_fields), 1)), np.uint8)
        out = np.zeros(n, np.uint32)
        _lib.check(self._L.gns_route_owner_keys(self._h, ct.byref(lay), keys.ctypes.data, keys.shape[1], n,
                                                out.ctypes.data, _lib.MEM_HOST))
        return out.astype(np.int64)

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._L.gns_route_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _outputs(self, hdr, n, out_hdr, out_wl):
        import torch
        if (out_hdr is None) != (out_wl is None):
            raise ValueError("out_hdr and out_wl go together")
        if out_hdr is None:  # fresh tensors (torch's caching allocator): results never alias
            return (torch.empty((n, 64), dtype=torch.uint8, device=hdr.device),
                    torch.empty((n,), dtype=torch.int32, device=hdr.device))
        if out_hdr.shape[0] < n or out_wl.shape[0] < n or out_hdr.numel() < 64 * n:
            raise ValueError(f"output buffers hold fewer than {n} records")
        return out_hdr[:n], out_wl[:n]

    def partition(self, hdr, wirelen, out_hdr=None, out_wl=None):
        """hdr [n,64] uint8 / wirelen [n] (device tensors) -> (out_hdr, out_wl, counts):
        the records regrouped shard by shard, packet order kept inside each shard;
        counts[g] = packets of shard g (numpy uint64).  Returns after the device work."""
        from . import _lib
        n = int(wirelen.shape[0])
        out_hdr, out_wl = self._outputs(hdr, n, out_hdr, out_wl)
        counts = np.zeros(self.nshards, np.uint64)
        _lib.device_ready(hdr, wirelen)
        _lib.check(self._L.gns_route_partition(self._h, hdr.data_ptr(), wirelen.data_ptr(), n, out_hdr.data_ptr(),
                                               out_wl.data_ptr(), counts.ctypes.data))
        return out_hdr, out_wl, counts

    def partition_async(self, hdr, wirelen, out_hdr=None, out_wl=None):
        """As partition, queued on torch's current stream without a host wait: counts
        is a device int64 tensor [nshards] (the all-to-all's split sizes)."""
        import torch
        from . import _lib
        n = int(wirelen.shape[0])
        out_hdr, out_wl = self._outputs(hdr, n, out_hdr, out_wl)
        counts = torch.empty((self.nshards,), dtype=torch.int64, device=hdr.device)
        st = torch.cuda.current_stream(hdr.device).cuda_stream
        _lib.check(self._L.gns_route_partition_async(self._h, hdr.data_ptr(), wirelen.data_ptr(), n,
                                                     out_hdr.data_ptr(), out_wl.data_ptr(), counts.data_ptr(), st))
        return out_hdr, out_wl, counts


def exchange_runs(run_hdr, run_wl, counts, world: int):
    """All-to-all of shard runs (RCCL on the GPU, gloo on the CPU): run g of every
    rank goes to rank g; the received runs are concatenated in source-rank order,
    so with rank r holding slice r of the stream each rank receives exactly the
    stable filter stream[shard_of(src) == rank].

    counts: this rank's run lengths, a device int64 tensor (Router.partition_async)
    or host integers.  One all-to-all of the counts, ONE host read of the send and
    receive split sizes, then the record and wire-length all-to-alls issued back to
    back (asynchronous) and waited together."""
    import torch
    import torch.distributed as dist
    dev = run_hdr.device
    if torch.is_tensor(counts):
        send = counts.to(device=dev, dtype=torch.int64)
    else:
        send = torch.tensor([int(c) for c in counts], dtype=torch.int64, device=dev)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send)
    both = torch.cat([send, recv]).cpu().tolist()  # the one host read of the exchange
    sc, rc = [int(x) for x in both[:world]], [int(x) for x in both[world:]]
    in_h = torch.empty((sum(rc), 64), dtype=torch.uint8, device=dev)
    in_w = torch.empty((sum(rc),), dtype=run_wl.dtype, device=dev)
    w1 = dist.all_to_all_single(in_h, run_hdr[: sum(sc)], output_split_sizes=rc, input_split_sizes=sc,
                                async_op=True)
    w2 = dist.all_to_all_single(in_w, run_wl[: sum(sc)], output_split_sizes=rc, input_split_sizes=sc,
                                async_op=True)
    w1.wait()
    w2.wait()
    return in_h, in_w


def route_exchange(router: "Router", hdr, wirelen, world: int):
    """configs[3] routing step: partition this rank's slice of the stream on the
    device (counts stay on the device), then exchange the runs (exchange_runs).
    Returns this rank's shard stream (device tensors).  Under gloo (CPU
    rehearsal) the runs travel through host memory and come back to the device."""
    import torch.distributed as dist
    oh, ow, counts = router.partition_async(hdr, wirelen)
    if dist.get_backend() != "nccl":
        ih, iw = exchange_runs(oh.cpu(), ow.cpu(), counts.cpu(), world)
        return ih.to(hdr.device), iw.to(hdr.device)
    return exchange_runs(oh, ow, counts, world)


def stable_split_records(hdr: np.ndarray, wirelen: np.ndarray, world: int, src16: np.ndarray = None, own=None):
    """Host restatement of Router.partition for records whose owners are known
    (tests / CPU rehearsal): runs shard by shard in stream order, and their lengths.
    own: owner shard per record (owner_of_tuples); default: the SrcIP owner of src16."""
    if own is None:
        own = shard_of(src16, world)
    order = np.argsort(own, kind="stable")
    counts = np.bincount(own, minlength=world).astype(np.uint64)
    return hdr[order], wirelen[order], counts


def _coll_device():
    import torch
    import torch.distributed as dist
    return torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")


def routed_query(query_many, keys, key_fields, world: int, owner=("SrcIP",), router: "Router" = None):
    """Owner-routed batched Query ("queries are routed to the owner
    shard"; Sketch.Query count_min.go:160-174 / super_spread.go:238-249 answered
    by the shard whose sketch holds the flow).  Collective: every rank calls it
    with its own batch of flow keys [n, K] (laid out as key_fields, n may differ
    or be 0).  Keys go to their owners in one all-to-all, each owner answers the
    keys it received with its local query_many (CountMin / SuperSpread / exact
    .query_many), and the answers come back in a second all-to-all, in the
    caller's order.  router: a Router computes the owners on the GPU; without
    one, the host restatement owner_of_keys does."""
    import torch
    import torch.distributed as dist
    from . import _lib
    if dist.get_backend() == "nccl" or _lib.is_device(keys):
        return _routed_query_device(query_many, keys, key_fields, world, owner, router)
    keys = np.ascontiguousarray(keys, np.uint8)
    n = keys.shape[0]
    K = max(sum(_FIELD_SIZE.get(f, 0) for f in key_fields), 1)
    keys = keys.reshape(n, -1) if n else np.zeros((0, K), np.uint8)
    own = router.owner_of_keys(keys, key_fields) if router is not None else owner_of_keys(keys, key_fields, world, owner)
    order = np.argsort(own, kind="stable")
    sc = np.bincount(own, minlength=world).astype(np.int64)
    dev = _coll_device()
    send = torch.from_numpy(sc).to(dev)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send)
    rc = [int(x) for x in recv.cpu().tolist()]
    scl = [int(x) for x in sc]
    out_keys = torch.from_numpy(np.ascontiguousarray(keys[order])).to(dev)
    in_keys = torch.empty((sum(rc), keys.shape[1]), dtype=torch.uint8, device=dev)
    dist.all_to_all_single(in_keys, out_keys, output_split_sizes=rc, input_split_sizes=scl)
    mine = in_keys.cpu().numpy()
    ans = np.asarray(query_many(mine) if len(mine) else np.zeros(0, np.uint64), np.uint64)
    back = torch.empty((n,), dtype=torch.int64, device=dev)
    dist.all_to_all_single(back, torch.from_numpy(np.ascontiguousarray(ans).view(np.int64)).to(dev),
                           output_split_sizes=scl, input_split_sizes=rc)
    out = np.empty(n, np.uint64)
    out[order] = back.cpu().numpy().view(np.uint64)
    return out


_ROUTERS: dict = {}


def _routed_query_device(query_many, keys, key_fields, world: int, owner, router):
    """routed_query under RCCL: keys, owners, the permutation and the answers stay on
    the GPU.  Owners from the Router's device kernel (gns_route_owner_keys), a stable
    device argsort by owner, the two all-to-alls on device tensors and the owner's
    query_many on the keys it received (gns_*_query_device); the only host read is
    the split sizes the all-to-all needs.  Host keys are copied up once and the
    answers come back as numpy; device keys give a device int64 tensor (uint64 bits)."""
    import torch
    import torch.distributed as dist
    from . import _lib
    dev = torch.device("cuda", torch.cuda.current_device())
    host_in = not _lib.is_device(keys)
    K = max(sum(_FIELD_SIZE.get(f, 0) for f in key_fields), 1)
    if host_in:
        keys = torch.from_numpy(np.ascontiguousarray(keys, np.uint8).reshape(-1, K)).to(dev)
    n = int(keys.shape[0])
    keys = keys.reshape(n, -1) if n else keys.reshape(0, K)
    K = int(keys.shape[1])
    if router is None:  # one device router per (world, device, owner key), kept for later calls
        rk = (world, dev.index, tuple(owner))
        router = _ROUTERS.get(rk)
        if router is None:
            router = _ROUTERS[rk] = Router(world, dev.index, owner)
    own = router.owner_of_keys(keys, key_fields).to(torch.int64)
    order = torch.argsort(own, stable=True)
    sc = torch.bincount(own, minlength=world)
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc)
    both = torch.cat([sc, rc]).cpu().tolist()  # the split sizes: the one host read
    scl, rcl = [int(x) for x in both[:world]], [int(x) for x in both[world:]]
    in_keys = torch.empty((sum(rcl), K), dtype=torch.uint8, device=dev)
    dist.all_to_all_single(in_keys, keys.index_select(0, order), output_split_sizes=rcl, input_split_sizes=scl)
    ans = query_many(in_keys)
    if not torch.is_tensor(ans):  # a host-only query_many (e.g. a snapshot view)
        ans = torch.from_numpy(np.ascontiguousarray(np.asarray(ans, np.uint64)).view(np.int64)).to(dev)
    back = torch.empty((n,), dtype=torch.int64, device=dev)
    dist.all_to_all_single(back, ans.to(torch.int64), output_split_sizes=scl, input_split_sizes=rcl)
    out = torch.empty_like(back)
    out[order] = back
    return out.cpu().numpy().view(np.uint64) if host_in else out


def _pack(items, K: int) -> np.ndarray:
    buf = np.zeros((len(items), K + 4), np.uint8)
    for i, (f, v) in enumerate(items):
        buf[i, :K] = np.frombuffer(f, np.uint8)
        buf[i, K:] = np.frombuffer(np.uint32(v).tobytes(), np.uint8)
    return buf


def _unpack(buf: np.ndarray, K: int):
    return [(bytes(r[:K]), int(np.frombuffer(r[K:K + 4].tobytes(), np.uint32)[0])) for r in buf]


def _allgather_rows(rows: np.ndarray, world: int) -> np.ndarray:
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    n = torch.tensor([rows.shape[0]], dtype=torch.int64, device=dev)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    cap = max(int(x.item()) for x in ns)
    width = rows.shape[1]
    mine = torch.zeros((max(cap, 1), width), dtype=torch.uint8, device=dev)
    if rows.shape[0]:
        mine[: rows.shape[0]] = torch.from_numpy(rows).to(dev)
    parts = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine)
    out = [p[: int(c.item())].cpu().numpy() for p, c in zip(parts, ns)]
    return np.concatenate(out, axis=0) if out else rows


def merge_heavy(lists):
    """Union of disjoint per-shard lists, max per flow, sorted value desc / flow asc."""
    best = {}
    for items in lists:
        for f, v in items:
            best[f] = max(best.get(f, 0), v)
    return sorted(best.items(), key=lambda fv: (-fv[1], fv[0]))


def allgather_heavy(hh: HeavyRecord, world: int) -> HeavyRecord:
    """Per-window exchange: all-gather every shard's heavy hitters (RCCL on GPU)."""
    K = len(hh.Count[0].Flow) if hh.Count else (len(hh.Size[0].Flow) if hh.Size else 0)
    import torch
    import torch.distributed as dist
    kt = torch.tensor([K], dtype=torch.int64,
                      device="cuda" if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(kt, op=dist.ReduceOp.MAX)
    K = int(kt.item())
    cnt = _unpack(_allgather_rows(_pack([(h.Flow, h.Count) for h in hh.Count], K), world), K)
    merged_c = merge_heavy([cnt])
    if hh.Size is None:
        return HeavyRecord(Size=None, Count=[HeavyCount(f, v) for f, v in merged_c])
    sz = _unpack(_allgather_rows(_pack([(h.Flow, h.Size) for h in hh.Size], K), world), K)
    merged_s = merge_heavy([sz])
    return HeavyRecord(Size=[HeavySize(f, v) for f, v in merged_s], Count=[HeavyCount(f, v) for f, v in merged_c])


def _sort_key(flows: np.ndarray, vals: np.ndarray) -> np.ndarray:
    """One 64-bit key per row: inverted value (desc) over the first four key bytes."""
    K = flows.shape[1]
    head = np.zeros((len(vals), 4), np.uint8)
    head[:, : min(K, 4)] = flows[:, : min(K, 4)]
    return ((np.uint64(0xFFFFFFFF) - vals.astype(np.uint64)) << np.uint64(32)) | \
        head.view(">u4").reshape(-1).astype(np.uint64)


def _order_tie_runs(flows: np.ndarray, key_sorted: np.ndarray, o: np.ndarray) -> np.ndarray:
    """o orders the rows by the 64-bit key; order each run of equal keys by the full key bytes."""
    tie = np.flatnonzero(key_sorted[1:] == key_sorted[:-1])
    i = 0
    while i < len(tie):
        a = tie[i]
        b = a + 1
        while i < len(tie) and tie[i] == b - 1:
            b += 1
            i += 1
        run = o[a:b]
        o[a:b] = run[sorted(range(len(run)), key=lambda j: flows[run[j]].tobytes())]
    return o


def merge_heavy_arrays(flows: np.ndarray, vals: np.ndarray):
    """Union of flow-disjoint per-shard lists in canonical order: value desc, then
    flow bytes asc (the tie order of CountMin.heavy_hitters, count_min.go:232-239).
    Sorted on one 64-bit key (inverted value, first four key bytes); only runs
    that tie on both are ordered by their full key bytes.  Shards own disjoint
    flows (shard_of), so no flow appears twice."""
    flows = np.ascontiguousarray(flows, np.uint8)
    vals = np.asarray(vals, np.uint32)
    if len(vals) == 0:
        return flows, vals
    comp = _sort_key(flows, vals)
    o = np.argsort(comp)
    o = _order_tie_runs(flows, comp[o], o)
    return flows[o], vals[o]


def _allgather_rows_dev(rows: np.ndarray, world: int):
    """All-gather of packed rows; the result stays where the collective put it
    (the GPU under RCCL), concatenated in rank order."""
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    n = torch.tensor([rows.shape[0]], dtype=torch.int64, device=dev)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    counts = [int(x.item()) for x in ns]
    mine = torch.zeros((max(max(counts), 1), rows.shape[1]), dtype=torch.uint8, device=dev)
    if rows.shape[0]:
        mine[: rows.shape[0]] = torch.from_numpy(rows).to(dev)
    parts = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine)
    return torch.cat([p[:c] for p, c in zip(parts, counts)], dim=0)


def _canonical_rows(g, K: int) -> np.ndarray:
    """Gathered (flow | value) rows -> host rows in canonical order.  The order is
    built where the rows are (torch stable sorts: first four key bytes asc, then
    value desc), one copy to the host, then only runs tied on both are ordered by
    their full key bytes."""
    import torch
    n = g.shape[0]
    if n == 0:
        return np.zeros((0, K + 4), np.uint8)
    if g.device.type == "cpu":  # gloo rehearsal: numpy sorts faster than torch's CPU stable sort
        rows = g.numpy()
        vals = np.ascontiguousarray(rows[:, K:]).view("<u4").reshape(-1)
        comp = _sort_key(rows[:, :K], vals)
        o = np.argsort(comp)
        return rows[_order_tie_runs(rows[:, :K], comp[o], o)]
    wv = g[:, K:K + 4].to(torch.int64)
    val = wv[:, 0] | (wv[:, 1] << 8) | (wv[:, 2] << 16) | (wv[:, 3] << 24)
    wh = g[:, : min(K, 4)].to(torch.int64)
    head = torch.zeros(n, dtype=torch.int64, device=g.device)
    for b in range(4):
        head = (head << 8) | (wh[:, b] if b < K else 0)
    o1 = torch.sort(head, stable=True).indices
    o2 = torch.sort(-val[o1], stable=True).indices
    rows = g[o1[o2]].cpu().numpy()
    flows = rows[:, :K]
    vals = np.ascontiguousarray(rows[:, K:]).view("<u4").reshape(-1)
    comp = _sort_key(flows, vals)
    o = _order_tie_runs(flows, comp, np.arange(n))
    return rows[o]


def allgather_heavy_arrays(arrays, world: int):
    """Per-window exchange on the array form of HeavyHitters (CountMin.heavy_hitters_arrays:
    count flows [n,K], counts, size flows, sizes): two RCCL all-gathers of packed
    (flow | value) rows, ordered on the GPU, then one copy to the host.  Same
    result as allgather_heavy without per-flow Python objects (a 2^20-bucket window
    has ~10^5 per shard)."""
    cf, cv, sf, sv = arrays
    K = cf.shape[1] if cf.ndim == 2 else sf.shape[1]

    def pack(f, v):
        rows = np.zeros((len(v), K + 4), np.uint8)
        if len(v):
            rows[:, :K] = f[:, :K]
            rows[:, K:] = np.ascontiguousarray(v, "<u4").view(np.uint8).reshape(-1, 4)
        return rows

    out = []
    for f, v in ((cf, cv), (sf, sv)):
        rows = _canonical_rows(_allgather_rows_dev(pack(f, v), world), K)
        out.extend((rows[:, :K], np.ascontiguousarray(rows[:, K:]).view("<u4").reshape(-1).astype(np.uint32)))
    return tuple(out)


def order_rows_device(rows, K: int):
    """Canonical order (value desc, flow bytes asc) of device rows [flow (K) | u32 value] on
    the GPU (gns_hh_order_rows: the hand-written radix sort of the heavy-hitter lists)."""
    import torch
    from . import _lib
    n = int(rows.shape[0])
    out = torch.empty_like(rows)
    if n:
        L = _lib.load()
        rows = rows.contiguous()
        torch.cuda.current_stream(rows.device).synchronize()  # the rows are complete
        _lib.check(L.gns_hh_order_rows(rows.data_ptr(), K, n, out.data_ptr(), rows.device.index or 0))
    return out


def _allgather_dev_rows(rows, world: int):
    """All-gather of device rows [n_r, W] (RCCL), concatenated in rank order."""
    import torch
    import torch.distributed as dist
    dev = rows.device
    n = torch.tensor([rows.shape[0]], dtype=torch.int64, device=dev)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    counts = [int(x.item()) for x in ns]
    mine = torch.zeros((max(max(counts), 1), rows.shape[1]), dtype=torch.uint8, device=dev)
    if rows.shape[0]:
        mine[: rows.shape[0]] = rows
    parts = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(parts, mine)
    return torch.cat([p[:c] for p, c in zip(parts, counts)], dim=0)


def allgather_heavy_rows(cm, world: int, rows=None):
    """Per-window exchange with the lists kept on the device (RCCL): each shard's device
    heavy-hitter rows (CountMin.heavy_hitters_rows_device, or `rows` already taken), two
    all-gathers, the union put in canonical order on the GPU (order_rows_device; shards own
    disjoint flows), then one copy to the host.  Returns (count flows [n,K], counts, size
    flows, sizes) like allgather_heavy_arrays."""
    K = cm.key_bytes
    out = []
    for rows in (rows if rows is not None else cm.heavy_hitters_rows_device()):
        g = order_rows_device(_allgather_dev_rows(rows, world), K).cpu().numpy()
        out.extend((g[:, :K], np.ascontiguousarray(g[:, K:]).view("<u4").reshape(-1).astype(np.uint32)))
    return tuple(out)


# ---------------------------------------------------------------------------
# Exact global mode (SURVEY §8e "exact global alternative"): every GPU sees the
# whole stream but applies only the updates that fall in its slice of bucket
# columns [lo, hi) of every row (CountMin(bucket_range=...)).  Buckets are
# independent (count_min.go:94-157 touches one bucket per row), so the slices
# together are exactly the single-GPU sketch; the global state is an
# all-gather of the slices.  Input is replicated, so this mode does not scale
# throughput: it is the bit-exact correctness mode, flow sharding is the
# scaling mode.
# ---------------------------------------------------------------------------
def bucket_slice(rank: int, world: int, width: int):
    """[lo, hi) bucket columns owned by `rank` (contiguous, sizes differ by at most one)."""
    return (rank * width // world, (rank + 1) * width // world)


def assemble_slices(states, ranges, width: int, depth: int):
    """Global (C, S, FPc, FPs) from per-slice exports (each a full-size export
    whose columns outside its range are untouched)."""
    C = np.zeros(depth * width, np.uint32)
    S = np.zeros(depth * width, np.uint32)
    K = states[0][2].shape[1]
    Fc = np.zeros((depth * width, K), np.uint8)
    Fs = np.zeros((depth * width, K), np.uint8)
    for (c, s, fc, fs), (lo, hi) in zip(states, ranges):
        for r in range(depth):
            sl = slice(r * width + lo, r * width + hi)
            C[sl], S[sl], Fc[sl], Fs[sl] = c[sl], s[sl], fc[sl], fs[sl]
    return C, S, Fc, Fs


def allgather_slices(state, rank: int, world: int, width: int, depth: int):
    """All-gather of every rank's slice (RCCL on GPU, gloo on CPU) -> the global state."""
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    C, S, Fc, Fs = state
    K = Fc.shape[1]
    lo, hi = bucket_slice(rank, world, width)
    cap = max(bucket_slice(q, world, width)[1] - bucket_slice(q, world, width)[0] for q in range(world))
    # per row: C, S as 4 bytes each + the two fingerprints, padded to the widest slice
    rowb = 8 + 2 * K
    mine = np.zeros((depth, cap, rowb), np.uint8)
    for r in range(depth):
        sl = slice(r * width + lo, r * width + hi)
        mine[r, : hi - lo, 0:4] = C[sl].view(np.uint8).reshape(-1, 4)
        mine[r, : hi - lo, 4:8] = S[sl].view(np.uint8).reshape(-1, 4)
        mine[r, : hi - lo, 8:8 + K] = Fc[sl]
        mine[r, : hi - lo, 8 + K:] = Fs[sl]
    t = torch.from_numpy(mine).to(dev)
    parts = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(parts, t)
    states, ranges = [], []
    for q, part in enumerate(parts):
        a = part.cpu().numpy()
        qlo, qhi = bucket_slice(q, world, width)
        c = np.zeros(depth * width, np.uint32)
        s = np.zeros(depth * width, np.uint32)
        fc = np.zeros((depth * width, K), np.uint8)
        fs = np.zeros((depth * width, K), np.uint8)
        for r in range(depth):
            sl = slice(r * width + qlo, r * width + qhi)
            n = qhi - qlo
            c[sl] = np.ascontiguousarray(a[r, :n, 0:4]).view(np.uint32).reshape(-1)
            s[sl] = np.ascontiguousarray(a[r, :n, 4:8]).view(np.uint32).reshape(-1)
            fc[sl] = a[r, :n, 8:8 + K]
            fs[sl] = a[r, :n, 8 + K:]
        states.append((c, s, fc, fs))
        ranges.append((qlo, qhi))
    return assemble_slices(states, ranges, width, depth)
