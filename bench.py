#!/usr/bin/env python3
"""Benchmark: Count-Min update throughput on device-resident synthetic traffic.

Metric (BASELINE.json): "Mpackets/s CMS update (device-resident, d=4 w=2^20)
at 1/2/4/8 MI355X".  Workload = configs[1]: Count-Min d=4 w=2^20, 100M Zipf(1.1)
5-tuple header records (64 B + 4 B wire length) resident in HBM; one step =
one pass of the full hot path (parse -> flow key -> flow id -> 4 MurmurHash3
rows -> bucket updates) over the 100M-packet batch; the sketch state carries
over from step to step like a live measurement period.

Multi-GPU (torchrun, one rank per GPU over RCCL): each rank owns the flows
whose SrcIP hashes to it and processes its own 100M-packet shard stream (weak
scaling, no data-path collective); after the timed region the ranks
all-gather their heavy-hitter candidates (the per-window exchange).

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PACKETS = 100_000_000
WIDTH, DEPTH = 1 << 20, 4
FIELDS = ["SrcIP", "DstIP", "SrcPort", "DstPort", "Protocol"]
BYTES_PER_PKT = 68          # SURVEY §8d convention A: 64-B header + 4-B wire length
# stages timed (HIP events) inside the timed steps; GNS_BENCH_ALL_STAGES=1 times every stage
_ALL = os.environ.get("GNS_BENCH_ALL_STAGES") == "1"
TIMED_STAGES = None if _ALL else ["extract", "scatter", "apply", "insert"]  # Count-Min
SS_TIMED_STAGES = None if _ALL else ["extract", "total"]                    # SuperSpread
EX_TIMED_STAGES = None if _ALL else ["extract", "total"]                    # exact aggregator
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def row_seeds(d):
    s, out = 0x9747B28C, []
    for _ in range(d):
        s = (s + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
        z = s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        out.append((z ^ (z >> 31)) & 0xFFFFFFFF)
    return np.array(out, np.uint32)


def host_cpu():
    """The GPU box's host CPU as BASELINE.md asks it to be reported (nproc, lscpu model)."""
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:
        avail = None
    quota = None  # cgroup v2 CPU quota (the box's CPU share), in CPUs
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"nproc": os.cpu_count(), "affinity_cpus": avail, "cgroup_cpu_quota": quota, "model": model}


def cpu_baseline(hdr_dev, wl_dev, seconds: float = 8.0, width: int = WIDTH, depth: int = DEPTH, fields=FIELDS,
                 keep_state: bool = False):
    """Timed CPU restatements on a bounded prefix of the same stream (rank 0).
    keep_state: also return the sequential oracle (the parity check replays the
    same prefix through the engine)."""
    from oracle import oracle as orc
    n = min(int(wl_dev.shape[0]), 24_000_000)
    hdr = hdr_dev[:n].cpu().numpy()
    wl = wl_dev[:n].cpu().numpy().view(np.uint32)
    seeds = row_seeds(depth)
    # (1) sequential oracle, 1 thread
    K = 37 if len(fields) == 5 else 16
    cm = orc.CountMin(width, depth, 1 << 20, 1000, K, seeds)
    chunk, done, t0 = 1_000_000, 0, time.perf_counter()
    while done < n and time.perf_counter() - t0 < seconds:
        m = min(chunk, n - done)
        cm.insert_hdr64(hdr[done:done + m], wl[done:done + m], fields)
        done += m
    seq_rate = done / (time.perf_counter() - t0) / 1e6
    seq_n = done
    seq_state = cm if keep_state else None
    if not keep_state:
        del cm
    # (2) restatement of the Go worker pool (shared sketch, CAS loops, shared cursor)
    threads = int(os.environ.get("GNS_CPU_THREADS", min(16, os.cpu_count() or 1)))
    cm = orc.CountMin(width, depth, 1 << 20, 1000, K, seeds)
    done, t0 = 0, time.perf_counter()
    chunk = 4_000_000
    while done < n and time.perf_counter() - t0 < seconds / 2:
        m = min(chunk, n - done)
        cm.insert_hdr64_pool(hdr[done:done + m], wl[done:done + m], fields, threads)
        done += m
    pool_rate = done / (time.perf_counter() - t0) / 1e6
    # (3) the same pool on every core this process may use (all host cores) =
    # min(CPU affinity, cgroup CPU quota): more threads than the quota only time-slice
    host = host_cpu()
    allc = host["affinity_cpus"] or os.cpu_count() or 1
    if host["cgroup_cpu_quota"]:
        allc = max(1, min(allc, int(host["cgroup_cpu_quota"])))
    cm = orc.CountMin(width, depth, 1 << 20, 1000, K, seeds)
    done_all, t0 = 0, time.perf_counter()
    while done_all < n and time.perf_counter() - t0 < seconds / 2:
        m = min(chunk, n - done_all)
        cm.insert_hdr64_pool(hdr[done_all:done_all + m], wl[done_all:done_all + m], fields, allc)
        done_all += m
    all_rate = done_all / (time.perf_counter() - t0) / 1e6
    del cm
    out = {
        "value": round(pool_rate, 3), "unit": "Mpackets/s", "cores": threads, "kind": "port",
        "sample": f"first {done:,} packets of the same synthetic stream (window 0); C restatement of the Go "
                  f"worker pool (count_min.go CAS loops + parse/encode, {threads} threads = the reference's "
                  f"num_workers default, shared cursor)",
        "host": host,
        "sequential_oracle": {"value": round(seq_rate, 3), "cores": 1, "packets": seq_n},
        "all_cores_pool": {"value": round(all_rate, 3), "cores": allc, "packets": done_all,
                           "what": "BASELINE.md B1: the same worker-pool restatement with one thread per usable "
                                   "core = min(CPU affinity set, cgroup CPU quota) of this process"},
    }
    return (out, seq_state, seq_n) if keep_state else out


def cpu_baseline_ss(hdr_dev, wl_dev, seconds: float = 10.0):
    """Sequential SuperSpread oracle on a bounded prefix of the same stream (rank 0).
    Returns the baseline, the oracle (its state is the parity reference) and the
    number of packets it took."""
    from oracle import oracle as orc
    n = min(int(wl_dev.shape[0]), 8_000_000)
    hdr = hdr_dev[:n].cpu().numpy()
    wl = wl_dev[:n].cpu().numpy().view(np.uint32)
    ss = orc.SuperSpread(SS_W, SS_D, SS_THR, SS_M, 5, 0.5, 1.08, 16, 16, row_seeds(SS_D), SS_HLL, SS_RNG)
    chunk, done, t0 = 500_000, 0, time.perf_counter()
    while done < n and time.perf_counter() - t0 < seconds:
        m = min(chunk, n - done)
        ss.insert_hdr64(hdr[done:done + m], wl[done:done + m], ["SrcIP"], ["DstIP"])
        done += m
    rate = done / (time.perf_counter() - t0) / 1e6
    base = {"value": round(rate, 3), "unit": "Mpackets/s", "cores": 1, "kind": "port", "host": host_cpu(),
            "sample": f"first {done:,} packets of window 0; sequential C restatement of "
                      f"super_spread.go (parse + encode + HLL + MV), 1 thread"}
    return base, ss, done


def parity_check_ss(orc_ss, hdr, wl, local):
    """After the timed region: the CPU leg's prefix through a fresh SuperSpread handle,
    whole exported state (values, owner keys, every HLL register, pbits as bit patterns)
    and the heavy-hitter list compared with the sequential oracle."""
    from go2netspectra_amd import SuperSpread
    ss = SuperSpread(SS_W, SS_D, SS_THR, SS_M, 5, 0.5, 1.08, flow_fields=["SrcIP"], elem_fields=["DstIP"],
                     seeds=row_seeds(SS_D), hll_master=SS_HLL, rng_seed=SS_RNG, device=local)
    ss.insert_headers(hdr, wl)
    ss.flush()
    got = ss.export_state()
    want = orc_ss.export()
    same = {name: bool(np.array_equal(np.asarray(a).view(np.uint8), np.asarray(b).view(np.uint8)))
            for name, a, b in zip(("values", "keys", "registers", "pbits"), got, want)}
    same["heavy"] = [(h.Flow, h.Count) for h in ss.heavy_hitters().Count] == orc_ss.heavy()
    ss.close()
    return {"checked_packets": int(wl.shape[0]), "bit_exact": all(same.values()), "arrays": same,
            "how": "the cpu_baseline sequential oracle's prefix of window 0 through a fresh handle "
                   "(declared generator, DESIGN.md §2)"}


# configs[2] / SURVEY §8d C3: the reference's default SuperSpread task
# (configs/config.yaml:112-122): flow [SrcIP], element [DstIP], d=2, w=32768,
# m=128, size=5, base=0.5, b=1.08; per-source fan-out Zipf(1.1) over 2^20 dsts.
SS_W, SS_D, SS_M, SS_THR, SS_FANOUT = 32768, 2, 128, 4096, 1 << 20
SS_HLL, SS_RNG = 0x0123456789ABCDEF, 0x0DDBA11CAFEF00D5


def bench_superspread(args, torch, dist, world, rank, local):
    """configs[2]: SuperSpread over 100M-packet windows in HBM.  Every step is a
    fresh window of the stream (packets [k*n, (k+1)*n)), generated on the device
    between steps and excluded from the timed sum, so HLL encodes keep
    happening as they would on live traffic (replaying one window would make
    every later pass encode-free)."""
    from go2netspectra_amd import SuperSpread, SyntheticTraffic
    n = args.packets
    syn = SyntheticTraffic(shard=rank, nshards=world, device=local, fanout=SS_FANOUT)
    hdr = torch.empty((n, 64), dtype=torch.uint8, device=f"cuda:{local}")
    wl = torch.empty((n,), dtype=torch.int32, device=f"cuda:{local}")
    ss = SuperSpread(SS_W, SS_D, SS_THR, SS_M, 5, 0.5, 1.08, flow_fields=["SrcIP"], elem_fields=["DstIP"],
                     seeds=row_seeds(SS_D), hll_master=SS_HLL, rng_seed=SS_RNG,
                     batch_packets=args.batch or n, device=local)  # one device batch per step, as the CM bench
    elapsed = 0.0
    for k in range(args.warmup + args.steps):
        syn.fill(hdr, wl, first=k * n)
        if k == args.warmup:
            ss.set_timing(True, stages=SS_TIMED_STAGES)
            ss.stage_times(reset=True)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ss.insert_headers(hdr, wl)
        ss.flush()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        if k >= args.warmup:
            elapsed += time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    stages = {k: v for k, v in ss.stage_times().items() if v[1]}
    kern = {k: v for k, v in stages.items() if k in ("extract", "resolve", "encode", "apply")}
    dom = max(kern, key=lambda k: kern[k][0])
    dom_ms, dom_launches = kern[dom]
    avg_ms = dom_ms / max(dom_launches, 1)
    pkts_per_launch = n * args.steps / max(dom_launches, 1)
    achieved = BYTES_PER_PKT * pkts_per_launch / (avg_ms * 1e-3) / 1e9
    traffic = None  # PMC HBM bytes per launch of the dominant kernel (tools/pmc_ss.sh)
    tfile = os.path.join(ROOT, "profiles", f"traffic_ss_d{SS_D}_w{SS_W}.json")
    if os.path.exists(tfile):
        try:
            traffic = json.load(open(tfile)).get(dom)
        except Exception:
            traffic = None
    hh = ss.heavy_hitters()  # first call sizes the list's buffers; the next three are timed
    t_hh = time.perf_counter()
    for _ in range(3):
        hh_n = len(ss.heavy_hitters_arrays()[1])
    t_hh = (time.perf_counter() - t_hh) / 3
    line = {
        "metric": "Mpackets/s SuperSpread update (device-resident, d=2 w=32768 m=128)",
        "value": round(n * args.steps * world / elapsed / 1e6, 2), "unit": "Mpackets/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8/u32/f64",
        "data": "synthetic (Zipf 1.1 sources over 2^20 5-tuples, per-packet Zipf 1.1 DstIP over 2^20, "
                "on-device generator, fresh window per step)",
        "config": {"workload": "configs[2]: SuperSpread flow=SrcIP elem=DstIP (default task geometry), "
                               "100M headers in HBM per GPU per step, bit-exact registers/pbits/counters",
                   "packets_per_step_per_gpu": n},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "bytes_per_packet": BYTES_PER_PKT, "kernel_avg_ms": round(avg_ms, 4)},
        "stage_ms_per_step": {k: round(v[0] / args.steps, 3) for k, v in stages.items()},
        "heavy_hitters": len(hh.Count), "engine_counters": ss.counters(),
        "heavy_hitters_ms": round(t_hh * 1e3, 3),
        "heavy_hitters_how": f"{hh_n} flows; device list (candidates, per-flow max, radix order), one D2H; "
                             "mean of 3 calls after the sizing call, after the timed steps",
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        ph, pw = syn.generate(8_000_000)
        base, orc_ss, done = cpu_baseline_ss(ph, pw)
        line["cpu_baseline"] = base
        line["parity"] = parity_check_ss(orc_ss, ph[:done], pw[:done], local)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def cpu_baseline_exact(hdr_dev, wl_dev, ts_dev, seconds: float = 10.0):
    from oracle import oracle as orc
    n = min(int(wl_dev.shape[0]), 4_000_000)
    hdr = hdr_dev[:n].cpu().numpy()
    wl = wl_dev[:n].cpu().numpy().view(np.uint32)
    ts = ts_dev[:n].cpu().numpy()
    ex = orc.Exact(FIELDS)
    chunk, done, t0 = 250_000, 0, time.perf_counter()
    while done < n and time.perf_counter() - t0 < seconds:
        m = min(chunk, n - done)
        ex.insert_hdr64(hdr[done:done + m], wl[done:done + m], ts[done:done + m])
        done += m
    rate = done / (time.perf_counter() - t0) / 1e6
    return {"value": round(rate, 3), "unit": "Mpackets/s", "cores": 1, "kind": "port", "host": host_cpu(),
            "sample": f"first {done:,} packets; sequential C restatement of exact/task.go (parse, Go key "
                      f"string, hash map), 1 thread"}


def bench_exact(args, torch, dist, world, rank, local):
    """Exact aggregator (per 5-tuple) over 100M device-resident headers per step."""
    from go2netspectra_amd import ExactTask, HeaderBatch, SyntheticTraffic
    n = args.packets
    # every step inserts a FRESH window of the rank's shard stream (window k = packets
    # [k*n, (k+1)*n)), generated before the step's opening barrier, outside the timed sum
    syn = SyntheticTraffic(shard=rank, nshards=world, device=local)
    dev = f"cuda:{local}"
    hdr = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    wl = torch.empty((n,), dtype=torch.int32, device=dev)
    ts = torch.empty((n,), dtype=torch.int64, device=dev)
    win = [0]

    def next_window():
        k = win[0]
        win[0] += 1
        syn.fill(hdr, wl, first=k * n)
        torch.arange(k * n, (k + 1) * n, dtype=torch.int64, device=dev, out=ts)
        ts.mul_(100).add_(1_700_000_000_000_000_000)
        torch.cuda.synchronize()

    task = ExactTask("per_five_tuple", FIELDS, 128, device=local, max_flows=args.ex_max_flows,
                     batch_packets=args.batch or n)
    batch = HeaderBatch(hdr, wl, ts)
    for _ in range(args.warmup):
        next_window()
        task.process_packets(batch)
        task.flush()
    task.agg.set_timing(True, stages=EX_TIMED_STAGES)
    task.agg.stage_times(reset=True)
    elapsed = 0.0
    for _ in range(args.steps):
        next_window()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        task.process_packets(batch)
        task.flush()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed += time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    stages = {k: v for k, v in task.agg.stage_times().items() if v[1]}
    kern = {k: v for k, v in stages.items() if k in ("extract", "resolve", "partition", "aggregate")}
    dom = max(kern, key=lambda k: kern[k][0])
    dom_ms, dom_launches = kern[dom]
    avg_ms = dom_ms / max(dom_launches, 1)
    # algorithmic bytes per packet: X1 reads the 68-B record; the partition reads and writes
    # each 8-B word of the tail; the aggregation reads it (per packet of the whole batch these
    # are upper bounds: only the tail has words)
    bpp = {"extract": BYTES_PER_PKT, "partition": 16, "aggregate": 8, "resolve": BYTES_PER_PKT}[dom]
    achieved = bpp * (n * args.steps / max(dom_launches, 1)) / (avg_ms * 1e-3) / 1e9
    line = {
        "metric": "Mpackets/s exact per-5-tuple aggregation (device-resident)",
        "value": round(n * args.steps * world / elapsed / 1e6, 2), "unit": "Mpackets/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
        "data": "synthetic (Zipf 1.1 over 2^20 5-tuples, on-device generator, ts = 100 ns apart; a fresh "
                "window of the stream per step, generated outside the timed region)",
        "config": {"workload": "exact aggregator, key = 5-tuple, 100M headers in HBM per GPU, exact "
                               "per-flow packets/bytes/start/end", "packets_per_step_per_gpu": n,
                   "windows": f"steps use stream windows 0..{win[0] - 1} (warmup first), none replayed"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                     "bytes_per_packet": bpp, "kernel_avg_ms": round(avg_ms, 4)},
        "stage_ms_per_step": {k: round(v[0] / args.steps, 3) for k, v in stages.items()},
        "engine_counters": task.agg.counters(),
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline_exact(hdr, wl, ts)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def thrift_messages_device(hdr, wl, torch):
    """The live path's NATS payloads for the same packets, built on the device:
    MarshalPacketInfo (packetcodec.go:54-73) of IPv4 PacketInfo is a fixed
    70-byte TBinaryProtocol layout, so a batch is an [n, 70] byte tensor."""
    n = int(wl.shape[0])
    h = hdr.view(torch.uint8)
    m = torch.zeros((n, 70), dtype=torch.uint8, device=hdr.device)
    be = lambda x, nb: torch.stack([((x >> (8 * (nb - 1 - i))) & 0xFF).to(torch.uint8) for i in range(nb)], 1)
    ts = torch.arange(n, dtype=torch.int64, device=hdr.device) * 100 + 1_700_000_000_000_000_000
    m[:, 0:3] = torch.tensor([0x0A, 0x00, 0x01], dtype=torch.uint8, device=hdr.device)
    m[:, 3:11] = be(ts, 8)
    m[:, 11:14] = torch.tensor([0x0C, 0x00, 0x02], dtype=torch.uint8, device=hdr.device)
    m[:, 14:21] = torch.tensor([0x0B, 0x00, 0x01, 0, 0, 0, 4], dtype=torch.uint8, device=hdr.device)
    m[:, 21:25] = h[:, 26:30]
    m[:, 25:32] = torch.tensor([0x0B, 0x00, 0x02, 0, 0, 0, 4], dtype=torch.uint8, device=hdr.device)
    m[:, 32:36] = h[:, 30:34]
    m[:, 36:41] = torch.tensor([0x08, 0x00, 0x03, 0, 0], dtype=torch.uint8, device=hdr.device)
    m[:, 41:43] = h[:, 34:36]
    m[:, 43:48] = torch.tensor([0x08, 0x00, 0x04, 0, 0], dtype=torch.uint8, device=hdr.device)
    m[:, 48:50] = h[:, 36:38]
    m[:, 50:56] = torch.tensor([0x08, 0x00, 0x05, 0, 0, 0], dtype=torch.uint8, device=hdr.device)
    m[:, 56] = h[:, 23]
    m[:, 57] = 0  # FiveTuple stop
    m[:, 58:61] = torch.tensor([0x0A, 0x00, 0x03], dtype=torch.uint8, device=hdr.device)
    m[:, 61:69] = be(wl.to(torch.int64) & 0xFFFFFFFF, 8)
    m[:, 69] = 0  # PacketInfo stop
    offs = torch.arange(n + 1, dtype=torch.int64, device=hdr.device) * 70
    return m, offs


def bench_thrift(args, torch, dist, world, rank, local):
    """f3 live path: decode 100M device-resident PacketInfo messages (one NATS
    payload each) into records and run the Count-Min path on them."""
    from go2netspectra_amd import CountMin, SyntheticTraffic, _lib
    from go2netspectra_amd._lib import check
    import ctypes as ct
    n = args.packets
    syn = SyntheticTraffic(shard=rank, nshards=world, device=local)
    hdr, wl = syn.generate(n)
    msg, offs = thrift_messages_device(hdr, wl, torch)
    del hdr, wl
    rec = torch.empty((n, 64), dtype=torch.uint8, device=f"cuda:{local}")
    rwl = torch.empty((n,), dtype=torch.int32, device=f"cuda:{local}")
    rts = torch.empty((n,), dtype=torch.int64, device=f"cuda:{local}")
    L = _lib.load()
    cm = CountMin(WIDTH, DEPTH, 1 << 20, 1000, flow_fields=FIELDS, seeds=row_seeds(DEPTH), max_flows=args.max_flows,
                  batch_packets=n, device=local)
    bad = ct.c_uint64(0)

    def step():
        check(L.gns_thrift_decode(msg.data_ptr(), n * 70, offs.data_ptr(), n, rec.data_ptr(), rwl.data_ptr(),
                                  rts.data_ptr(), ct.byref(bad), _lib.MEM_DEVICE, local))
        cm.insert_headers(rec, rwl)

    for _ in range(args.warmup):
        step()
        cm.flush()
    dec = 0.0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ta = time.perf_counter()
        check(L.gns_thrift_decode(msg.data_ptr(), n * 70, offs.data_ptr(), n, rec.data_ptr(), rwl.data_ptr(),
                                  rts.data_ptr(), ct.byref(bad), _lib.MEM_DEVICE, local))
        dec += time.perf_counter() - ta  # the decode call synchronizes the device
        cm.insert_headers(rec, rwl)
    cm.flush()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    dec_ms = dec / args.steps * 1e3
    bpp = 70 + 8 + 64 + 4 + 8  # message + offset read, record + wire length + timestamp written
    line = {
        "metric": "Mpackets/s Thrift PacketInfo batch decode + CMS update (device-resident, d=4 w=2^20)",
        "value": round(n * args.steps * world / elapsed / 1e6, 2), "unit": "Mpackets/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8/u32",
        "data": "synthetic (the Count-Min bench stream, marshalled as 70-B IPv4 PacketInfo messages on the device)",
        "config": {"workload": "SURVEY f3: ns-engine ingest, 100M PacketInfo messages in HBM -> records -> Count-Min",
                   "packets_per_step_per_gpu": n, "rejected": int(bad.value)},
        "roofline": {"bound": "hbm", "kernel": "k_thrift_decode", "achieved": round(bpp * n / (dec_ms * 1e-3) / 1e9, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(bpp * n / (dec_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     "traffic": None, "bytes_per_packet": bpp, "kernel_avg_ms": round(dec_ms, 4),
                     "note": "decode time from the host clock around the synchronizing decode call"},
        "note": "not the headline metric",
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def bench_hybrid(args, torch, dist, world, rank, local):
    """configs[4]: hybrid exact + sketch.  Each step (one window of 100M packets per
    GPU) goes through BOTH the exact per-5-tuple aggregator and a Count-Min of the
    configs[4] geometry (d=8, w=2^24); at every window boundary the sketch's
    snapshot view is refreshed and a reader thread extracts the device-side
    heavy-hitter lists (count and size) and answers a batch of point queries
    from it while the next window is being ingested (queries concurrent with
    ingest).  value = packets ingested by both paths / time; the reader's work
    is inside the timed region (it is joined before the closing barrier)."""
    import threading
    from go2netspectra_amd import CountMin, ExactTask, HeaderBatch, SyntheticTraffic
    n = args.packets
    W, D = 1 << 24, 8
    syn = SyntheticTraffic(shard=rank, nshards=world, device=local)
    hdr, wl = syn.generate(n)
    ts = torch.arange(n, dtype=torch.int64, device=f"cuda:{local}") * 100 + 1_700_000_000_000_000_000
    batch = HeaderBatch(hdr, wl, ts)
    ex = ExactTask("per_five_tuple", FIELDS, 128, device=local, max_flows=args.ex_max_flows, batch_packets=args.batch or n)
    cm = CountMin(W, D, 1 << 20, 1000, flow_fields=FIELDS, seeds=row_seeds(D), max_flows=args.max_flows,
                  batch_packets=args.batch or n, device=local)
    view = cm.view()
    # point-query keys: the 5-tuple keys of 2^16 packets of the stream (host copy, made once)
    h = hdr[: 1 << 16].view(torch.uint8).cpu().numpy()
    qkeys = np.zeros((h.shape[0], 37), np.uint8)
    qkeys[:, 0:4], qkeys[:, 16:20], qkeys[:, 32:36], qkeys[:, 36] = h[:, 26:30], h[:, 30:34], h[:, 34:38], h[:, 23]

    # the two ingest paths run on their own streams from two host threads (each
    # engine synchronizes its own stream at batch boundaries)
    def ex_step():
        ex.process_packets(batch)
        ex.flush()

    def step():
        if args.hybrid_serial:  # one host thread: the exact path, then the sketch path
            ex_step()
            cm.insert_headers(hdr, wl)
            return
        te = threading.Thread(target=ex_step)
        te.start()
        cm.insert_headers(hdr, wl)
        te.join()

    for _ in range(args.warmup):
        step()
    ex.flush()
    cm.flush()
    cm.set_timing(True)
    cm.stage_times(reset=True)
    ex.agg.set_timing(True)
    ex.agg.stage_times(reset=True)
    windows = []
    lock = threading.Condition()
    pending = [0]
    stop = [False]
    lat = []

    def reader():
        while True:
            with lock:
                while pending[0] == 0 and not stop[0]:
                    lock.wait()
                if pending[0] == 0 and stop[0]:
                    return
                pending[0] = 0
            t0 = time.perf_counter()
            cf, cv, sf, sv = view.heavy_hitters_arrays()
            q = view.query_many(qkeys)
            lat.append(time.perf_counter() - t0)
            windows.append((len(cv), len(sv), int((q >> np.uint64(32)).max()) if len(q) else 0))

    th = threading.Thread(target=reader)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    th.start()
    for _ in range(args.steps):
        step()
        view.refresh()               # window boundary: snapshot for the reader
        with lock:
            pending[0] += 1
            lock.notify()
    ex.flush()
    cm.flush()
    with lock:
        stop[0] = True
        lock.notify()
    th.join()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    stages = cm.stage_times()
    ex_stages = ex.agg.stage_times()
    # dominant kernel over both engines' stages (HIP events on each engine's stream), at
    # SURVEY §8d convention A (68 B/packet: each engine reads every record once)
    kern = {f"cm.{k}": v for k, v in stages.items() if k in ("extract", "resolve", "scan", "scatter", "apply")}
    kern.update({f"exact.{k}": v for k, v in ex_stages.items() if k in ("extract", "resolve", "partition", "aggregate")})
    dom = max(kern, key=lambda k: kern[k][0])
    dom_ms, dom_launches = kern[dom]
    avg_ms = dom_ms / max(dom_launches, 1)
    achieved = BYTES_PER_PKT * (n * args.steps / max(dom_launches, 1)) / (avg_ms * 1e-3) / 1e9
    traffic = None  # PMC record of this workload (tools/r05_pmc.sh hybrid -> profiles/traffic_hybrid_*.json)
    tfile = os.path.join(ROOT, "profiles", f"traffic_hybrid_d{D}_w{W}_b{args.batch or n}.json")
    if os.path.exists(tfile):
        try:
            key = {"exact.extract": "k_ex_extract", "exact.resolve": "k_ex_resolve", "exact.partition": "k_ex_pscatter",
                   "exact.aggregate": "k_ex_pagg"}.get(dom, dom.split(".", 1)[1])
            traffic = json.load(open(tfile)).get(key)
        except Exception:
            traffic = None
    line = {
        "metric": "Mpackets/s hybrid exact + CMS d=8 w=2^24 ingest with concurrent heavy-hitter queries",
        "value": round(n * args.steps * world / elapsed / 1e6, 2), "unit": "Mpackets/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32/u64",
        "data": "synthetic (Zipf 1.1 over 2^20 5-tuples, 64-B records, on-device generator)",
        "config": {"workload": "configs[4]: exact per-5-tuple aggregator + Count-Min d=8 w=2^24 on the same "
                               "100M-packet window per GPU; per window a snapshot view, device-side heavy-hitter "
                               "extraction and 65,536 point queries on a reader thread concurrent with ingest",
                   "packets_per_step_per_gpu": n, "windows_queried": len(windows),
                   "ingest": "serial (one thread)" if args.hybrid_serial else "concurrent (two streams, two threads)"},
        "queries": {"windows": len(windows), "latency_ms_avg": round(1e3 * sum(lat) / max(len(lat), 1), 3),
                    "latency_ms_max": round(1e3 * max(lat), 3) if lat else None,
                    "last_window_heavy_hitters": {"count": windows[-1][0], "size": windows[-1][1]} if windows else None},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "bytes_per_packet": BYTES_PER_PKT, "kernel_avg_ms": round(avg_ms, 4),
                     "pipeline_frac": round(2 * BYTES_PER_PKT * n * args.steps / elapsed / 1e9 / HBM_PEAK_GBS, 4),
                     "note": "pipeline_frac counts the record stream twice (both engines read it)"},
        "stage_ms_per_step": {k: round(v[0] / args.steps, 3) for k, v in stages.items()},
        "exact_stage_ms_per_step": {k: round(v[0] / args.steps, 3) for k, v in ex_stages.items()},
        "note": "not the headline metric",
    }
    view.close()
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def bench_c1(args, torch, dist, world, rank, local):
    """configs[0]: the pcap-analyzer path (cmd/pcap-analyzer -> offline.RunAnalyzer ->
    pcap.Reader.ReadPackets -> workers -> Count-Min) on a 1M-packet capture in the
    reference generator's format (scripts/pcapgen/main.go), Count-Min d=4 w=65536.
    A step = the whole capture: the host packer reads the file into 64-byte records
    (gns_pack_pcap), the engine inserts them from host memory (H2D staging included)
    into a fresh period of the sketch.  The CPU legs time the C restatement of the Go
    worker pool and the sequential oracle on the same records (plus the same pack)."""
    from go2netspectra_amd import CountMin, read_pcap, write_pcapgen
    from oracle import oracle as orc
    n = args.c1_packets
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"gns_pcapgen_{n}.pcap")
    if not os.path.exists(path):
        write_pcapgen(path, n)
    W, D = 65536, 4
    seeds = row_seeds(D)
    cm = CountMin(W, D, 1 << 20, 1000, flow_fields=FIELDS, seeds=seeds, max_flows=1 << 21, batch_packets=n, device=local)
    t_pack = t_gpu = 0.0
    hb = None
    for k in range(args.warmup + args.steps):
        cm.reset()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        hb = read_pcap(path)
        t1 = time.perf_counter()
        cm.insert_headers(hb.hdr, hb.wirelen)
        cm.flush()
        t2 = time.perf_counter()
        if k >= args.warmup:
            t_pack += t1 - t0
            t_gpu += t2 - t1
    K = args.steps
    line = {
        "metric": "Mpackets/s pcap-analyzer Count-Min d=4 w=65536 (pcap file -> packer -> GPU), 1M-packet pcapgen capture",
        "value": round(n * K / (t_pack + t_gpu) / 1e6, 2), "unit": "Mpackets/s", "n_gpus": 1, "steps": K,
        "warmup": args.warmup, "ms_per_step": round((t_pack + t_gpu) / K * 1e3, 3), "higher_is_better": True,
        "scaling": "none", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic capture in scripts/pcapgen/main.go's format (go2netspectra_amd.write_pcapgen), "
                f"{os.path.getsize(path) / 1e6:.0f} MB on local disk (page cache warm after the warmup)",
        "config": {"workload": "configs[0]: pcap-analyzer, Count-Min d=4 w=65536, 5-tuple key, 1M packets",
                   "packets": n, "pack_ms": round(t_pack / K * 1e3, 3), "insert_ms_incl_h2d": round(t_gpu / K * 1e3, 3),
                   "insert_only_rate": round(n * K / t_gpu / 1e6, 2)},
        "note": "not the headline metric; the reference pcap-analyzer is a CPU path (BASELINE configs[0])",
    }
    if not args.no_cpu:
        o = orc.CountMin(W, D, 1 << 20, 1000, 37, seeds)
        t0 = time.perf_counter()
        o.insert_hdr64(hb.hdr, hb.wirelen, FIELDS)
        seq_s = time.perf_counter() - t0
        threads = int(os.environ.get("GNS_CPU_THREADS", 16))
        p = orc.CountMin(W, D, 1 << 20, 1000, 37, seeds)
        t0 = time.perf_counter()
        p.insert_hdr64_pool(hb.hdr, hb.wirelen, FIELDS, threads)
        pool_s = time.perf_counter() - t0
        pack_s = t_pack / K
        line["cpu_baseline"] = {
            "value": round(n / (pack_s + pool_s) / 1e6, 3), "unit": "Mpackets/s", "cores": threads, "kind": "port",
            "sample": f"the whole {n:,}-packet capture: the same packer, then the C restatement of the Go worker "
                      f"pool ({threads} threads, count_min.go CAS loops); pool alone "
                      f"{n / pool_s / 1e6:.2f} Mpkt/s",
            "host": host_cpu(),
            "sequential_oracle": {"value": round(n / (pack_s + seq_s) / 1e6, 3), "cores": 1,
                                  "insert_only": round(n / seq_s / 1e6, 3)},
        }
        got, want = cm.export_state(), o.export()
        line["parity"] = {"checked_packets": n, "bit_exact": all(bool(np.array_equal(a, b)) for a, b in zip(got, want)),
                          "how": "the last step's sketch vs the sequential oracle on the same records"}
    print(json.dumps(line), flush=True)


def bench_windows(args, torch, dist, world, cm, timed_step, n):
    """configs[3]'s per-window cycle, timed after the headline steps: each window
    inserts --window-steps fresh steps of packets (timed_step: generation outside
    the timed part), takes the shard's heavy hitters on the device
    (gns_cm_heavy_hitters: candidates, dedupe, order) and all-gathers every
    shard's list over RCCL (dist.allgather_heavy_arrays; flows are disjoint across
    shards, so the union is the global list).  Max over ranks, like the steps."""
    from go2netspectra_amd.dist import allgather_heavy_arrays, allgather_heavy_rows
    device_rows = world > 1 and dist.get_backend() == "nccl"  # RCCL: the lists never leave the GPUs
    t_ins = t_hh = t_x = 0.0
    per_hh = []
    # warm, twice: the read side's buffers and the sort's scratch.  The second list call
    # of a process has stalled 18-36 ms before its first kernel ran, with the GPU idle
    # (profiles/r06_hh_spike_kernel_trace.txt), once; the windows below are timed after it.
    for _ in range(2):
        if device_rows:
            allgather_heavy_rows(cm, world)
        else:
            arrs = cm.heavy_hitters_arrays()
            if world > 1:
                allgather_heavy_arrays(arrs, world)
    for _ in range(args.windows):
        for _ in range(args.window_steps):
            t_ins += timed_step()
        if world > 1:
            dist.barrier()
        b = time.perf_counter()
        if device_rows:  # the shard's device list, then all-gather + device merge + one D2H
            rows = cm.heavy_hitters_rows_device()
            torch.cuda.synchronize()
            c = time.perf_counter()
            arrs = allgather_heavy_rows(cm, world, rows)
            dist.barrier()
        else:
            arrs = cm.heavy_hitters_arrays()
            c = time.perf_counter()
            if world > 1:
                arrs = allgather_heavy_arrays(arrs, world)
                dist.barrier()
        e = time.perf_counter()
        t_hh += c - b
        t_x += e - c
        per_hh.append(round((c - b) * 1e3, 3))
    el = t_ins + t_hh + t_x
    if world > 1:
        tt = torch.tensor([el], dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    W = args.windows
    return {"windows": W, "steps_per_window": args.window_steps,
            "value": round(n * args.window_steps * W * world / el / 1e6, 2), "unit": "Mpackets/s",
            "ms_per_window": round(el / W * 1e3, 3), "insert_ms": round(t_ins / W * 1e3, 3),
            "heavy_hitters_ms": round(t_hh / W * 1e3, 3), "exchange_ms": round(t_x / W * 1e3, 3),
            "heavy_hitters_ms_per_window": per_hh, "heavy_hitters_ms_median": float(np.median(per_hh)),
            "global_heavy_hitters": {"count": int(len(arrs[1])), "size": int(len(arrs[3]))},
            "collective": ("all-gather of packed (flow | value) rows, " + dist.get_backend()
                           + (", lists kept on the GPUs, merged by the device sort" if device_rows else ""))
            if world > 1 else "none (one shard: the device list is already the global one)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--packets", type=int, default=PACKETS)
    ap.add_argument("--batch", type=int, default=0, help="device batch (packets); 0 = whole step")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--width", type=int, default=WIDTH, help="Count-Min width (2^24 = configs[4] geometry)")
    ap.add_argument("--depth", type=int, default=DEPTH, help="Count-Min depth (8 = configs[4] geometry)")
    ap.add_argument("--config", choices=["c1", "c2"], default="c2",
                    help="c1 = configs[0]: the pcap-analyzer path on a 1M-packet pcapgen capture (CM d=4 w=65536); "
                         "c2 = configs[1], the headline")
    ap.add_argument("--c1-packets", type=int, default=1_000_000)
    ap.add_argument("--sketch", choices=["countmin", "superspread", "exact", "thrift", "hybrid"], default="countmin",
                    help="superspread = configs[2]; hybrid = configs[4]; exact = the exact aggregator "
                         "(none of them is the headline metric)")
    ap.add_argument("--max-flows", type=int, default=1 << 22,
                    help="flow dictionary capacity (slots = next power of two >= 2x)")
    ap.add_argument("--ex-max-flows", type=int, default=1 << 21,
                    help="exact aggregator flow dictionary capacity (--sketch exact / hybrid)")
    ap.add_argument("--windows", type=int, default=3,
                    help="after the timed steps: W timed windows of insert + device heavy hitters + "
                         "all-gather of every shard's list (configs[3] per-window exchange); 0 = off")
    ap.add_argument("--window-steps", type=int, default=10,
                    help="steps per window (fresh 100M-packet windows; configs[3] says a 1 s window)")
    ap.add_argument("--hybrid-serial", action="store_true",
                    help="--sketch hybrid: run the exact and sketch paths one after the other from one host "
                         "thread instead of concurrently on two streams from two threads")
    ap.add_argument("--route", action="store_true",
                    help="configs[3] pipeline (N > 1): each GPU holds a contiguous slice of the unsharded stream; "
                         "the timed step partitions it on the device, all-to-alls the shard runs and inserts")
    ap.add_argument("--key", choices=["5tuple", "srcip"], default="5tuple",
                    help="flow key: full 5-tuple (37 B, primary) or [SrcIP] (16 B, the default task layout)")
    ap.add_argument("--flows", type=int, default=1 << 20,
                    help="distinct flows of the synthetic stream (experiments; the headline uses 2^20)")
    ap.add_argument("--host-input", nargs="?", const="headers", choices=["headers", "tuples", "compact", "compact16"], default=None,
                    help="time inserts from pinned host memory plus the per-window D2H of counters and heavy "
                         "hitters (PCIe-inclusive rate, for DESIGN.md): 64-B header records or 41-B PacketInfo "
                         "tuples (the live path's pre-parsed form)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # GNS_DIST_BACKEND=gloo: rehearsal of the N-rank path with several ranks on fewer
    # GPUs (RCCL needs one GPU per rank); the data path is the same, only the
    # barrier / max-reduce / heavy-hitter all-gather go over gloo
    backend = os.environ.get("GNS_DIST_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(torch.cuda.device_count(), 1)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
    torch.cuda.set_device(local)

    from go2netspectra_amd import CountMin, SyntheticTraffic

    if args.config == "c1":
        return bench_c1(args, torch, dist, world, rank, local)
    if args.sketch == "superspread":
        return bench_superspread(args, torch, dist, world, rank, local)
    if args.sketch == "exact":
        return bench_exact(args, torch, dist, world, rank, local)
    if args.sketch == "thrift":
        return bench_thrift(args, torch, dist, world, rank, local)
    if args.sketch == "hybrid":
        return bench_hybrid(args, torch, dist, world, rank, local)
    n = args.packets
    fields = FIELDS if args.key == "5tuple" else ["SrcIP"]
    K = 37 if args.key == "5tuple" else 16
    dev = torch.device("cuda", local)
    route = args.route and world > 1
    # Input windows.  Every step inserts a FRESH window of the stream, generated on
    # the device before the step's opening barrier and excluded from the timed sum:
    #  - default (weak scaling): rank r's window k = packets [k*n, (k+1)*n) of its
    #    shard stream, the stable filter stream[shard_of(src) == r] (what the
    #    routing step delivers; SyntheticTraffic(shard, nshards));
    #  - --route (configs[3] pipeline): rank r holds the contiguous slice
    #    [(k*world + r)*n, ...) of the UNSHARDED stream; the timed step partitions
    #    it on the device, all-to-alls the runs and inserts what it received.
    syn = SyntheticTraffic(flows=args.flows, shard=0 if route else rank, nshards=1 if route else world, device=local)
    hdr = torch.empty((n, 64), dtype=torch.uint8, device=dev)
    wl = torch.empty((n,), dtype=torch.int32, device=dev)
    win = [0]

    def next_window():
        k = win[0]
        win[0] += 1
        syn.fill(hdr, wl, first=(k * world + rank) * n if route else k * n)

    # host input: 16M-packet device batches, so the H2D copy of batch i+1 overlaps batch i
    batch = args.batch or (min(n, 1 << 24) if args.host_input else n)
    cm = CountMin(args.width, args.depth, 1 << 20, 1000, flow_fields=fields, seeds=row_seeds(args.depth),
                  max_flows=args.max_flows, batch_packets=batch, device=local)
    router = None
    if route:
        from go2netspectra_amd.dist import Router
        router = Router(world, local)
    torch.cuda.synchronize()

    def barrier():
        if world > 1:
            dist.barrier()

    tuples = None
    window_out = None
    pin = None
    if args.host_input:  # pinned host buffers; the engine stages them H2D per device batch
        def pinned(a):
            return torch.empty(a.shape, dtype=a.dtype, pin_memory=True)
        if args.host_input == "tuples":  # PacketInfo SoA (src16, dst16, ports, proto, length) = 41 B/packet
            from go2netspectra_amd.packets import PacketBatch
            pin = {"src16": pinned(torch.empty((n, 16), dtype=torch.uint8)),
                   "dst16": pinned(torch.empty((n, 16), dtype=torch.uint8)),
                   "sport": pinned(torch.empty((n,), dtype=torch.int16)), "dport": pinned(torch.empty((n,), dtype=torch.int16)),
                   "proto": pinned(torch.empty((n,), dtype=torch.uint8)), "length": pinned(torch.empty((n,), dtype=torch.int32))}
            tuples = PacketBatch(pin["src16"].numpy(), pin["dst16"].numpy(), pin["sport"].numpy().view(np.uint16),
                                 pin["dport"].numpy().view(np.uint16), pin["proto"].numpy(),
                                 pin["length"].numpy().view(np.uint32))
        elif args.host_input in ("compact", "compact16"):
            # 16-B compact records + wire length = 20 B/packet; compact16: the wire length inside
            # the record = 16 B/packet (+ side records either way)
            pin = {"rec": pinned(torch.empty((n, 16), dtype=torch.uint8)),
                   "wl": pinned(wl) if args.host_input == "compact" else None,
                   "side": pinned(torch.empty((max(1024, n // 256), 64), dtype=torch.uint8)), "ns": 0}
        else:
            pin = {"hdr": pinned(hdr), "wl": pinned(wl)}
        cnt_C = np.empty(args.depth * args.width, np.uint32)
        cnt_S = np.empty(args.depth * args.width, np.uint32)

        def window_out():  # per-window outputs back to the host: counter rows + heavy hitters (Snapshot)
            cm.export_counters(cnt_C, cnt_S)
            return cm.heavy_hitters_arrays()

    def stage_host():  # untimed: this step's window into the pinned host buffers
        if pin is None:
            return
        if tuples is not None:
            h = hdr.view(torch.uint8)
            src16 = torch.zeros((n, 16), dtype=torch.uint8, device=dev)
            dst16 = torch.zeros((n, 16), dtype=torch.uint8, device=dev)
            src16[:, :4] = h[:, 26:30]
            dst16[:, :4] = h[:, 30:34]
            pin["src16"].copy_(src16)
            pin["dst16"].copy_(dst16)
            pin["sport"].copy_((h[:, 34].to(torch.int32) << 8 | h[:, 35].to(torch.int32)).to(torch.int16))
            pin["dport"].copy_((h[:, 36].to(torch.int32) << 8 | h[:, 37].to(torch.int32)).to(torch.int16))
            pin["proto"].copy_(h[:, 23])
            pin["length"].copy_(wl)
        elif "rec" in pin:
            from go2netspectra_amd import compact_headers
            rec, side = compact_headers(hdr, wl, rec_len=pin["wl"] is None)
            pin["rec"].copy_(rec)
            if pin["wl"] is not None:
                pin["wl"].copy_(wl)
            pin["ns"] = int(side.shape[0])
            pin["side"][: pin["ns"]].copy_(side)
        else:
            pin["hdr"].copy_(hdr)
            pin["wl"].copy_(wl)

    def step():
        if route:
            from go2netspectra_amd.dist import route_exchange
            ih, iw = route_exchange(router, hdr, wl, world)
            cm.insert_headers(ih, iw)
        elif tuples is not None:
            cm.insert_tuples(tuples)
        elif pin is not None and "rec" in pin:
            cm.insert_compact(pin["rec"].numpy(), pin["wl"].numpy().view(np.uint32) if pin["wl"] is not None else None,
                              pin["side"][: pin["ns"]].numpy() if pin["ns"] else None)
        elif pin is not None:
            cm.insert_headers(pin["hdr"].numpy(), pin["wl"].numpy().view(np.uint32))
        else:
            cm.insert_headers(hdr, wl)
        if window_out is not None:
            window_out()

    def timed_step():
        """one fresh window: generated (untimed), then barrier + sync, the step, sync + barrier"""
        next_window()
        stage_host()
        torch.cuda.synchronize()
        barrier()
        t0 = time.perf_counter()
        step()
        cm.flush()
        torch.cuda.synchronize()
        barrier()
        return time.perf_counter() - t0

    for _ in range(args.warmup):
        timed_step()
    # HIP events around the three partition kernels and the whole batch only: each timed stage
    # puts two events into the batch's stream (timing every stage cost ~0.8% of the step,
    # profiles/r06_abh2); the small stages' times are in the rocprofv3 summaries under profiles/
    cm.set_timing(True, stages=TIMED_STAGES)
    cm.stage_times(reset=True)
    elapsed = 0.0
    for _ in range(args.steps):
        elapsed += timed_step()
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64, device="cuda" if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    stages = {k: v for k, v in cm.stage_times().items() if v[1]}
    counters = cm.counters()

    window = None
    if args.windows > 0 and not args.host_input and not route:
        window = bench_windows(args, torch, dist, world, cm, timed_step, n)

    # flow dictionary: reclaims during the run, and the cost of one reclaim at a
    # window boundary with this run's live set (untimed; inserts reclaim on their
    # own when the dictionary reaches max_flows)
    dict_run = cm.dict_stats()
    torch.cuda.synchronize()
    t_r = time.perf_counter()
    cm.reclaim()
    reclaim_ms = (time.perf_counter() - t_r) * 1e3
    dict_after = cm.dict_stats()
    dictionary = {"max_flows": args.max_flows, "reclaims_during_run": dict_run["reclaims"],
                  "retried_batches": dict_run["retried_batches"], "claimed_before_reclaim": dict_run["claimed"],
                  "live_flows": dict_after["live"], "one_reclaim_ms": round(reclaim_ms, 3)}

    hh = cm.heavy_hitters()
    if world > 1:
        from go2netspectra_amd.dist import allgather_heavy
        hh = allgather_heavy(hh, world)

    total_pkts = n * args.steps * world
    value = total_pkts / elapsed / 1e6
    # dominant kernel and its roofline (HIP events on the engine stream)
    kern = {k: v for k, v in stages.items() if k in ("extract", "resolve", "scan", "scatter", "apply")}
    dom = max(kern, key=lambda k: kern[k][0])
    dom_ms, dom_launches = kern[dom]
    avg_ms = dom_ms / max(dom_launches, 1)
    pkts_per_launch = n * args.steps / max(dom_launches, 1)
    achieved = BYTES_PER_PKT * pkts_per_launch / (avg_ms * 1e-3) / 1e9
    traffic = None  # PMC record of THIS geometry and device batch only (tools/pmc_cm.sh -> profiles/traffic_cm_*.json)
    tfile = os.path.join(ROOT, "profiles", f"traffic_cm_d{args.depth}_w{args.width}_k{K}_b{batch}.json")
    if os.path.exists(tfile) and not route and args.flows == 1 << 20:
        try:
            traffic = json.load(open(tfile)).get(dom)
        except Exception:
            traffic = None

    line = {
        "metric": "Mpackets/s CMS update (device-resident, d=4 w=2^20) at 1/2/4/8 MI355X",
        "value": round(value, 2), "unit": "Mpackets/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
        "data": "synthetic (Zipf 1.1 over 2^20 5-tuples, 64-B Ethernet/IPv4/TCP|UDP records, on-device generator; "
                "a fresh window of the stream per step, generated outside the timed region)",
        "config": {"workload": "configs[1]: Count-Min d=4 w=2^20, 100M Zipf(1.1) 5-tuple headers in HBM per GPU, "
                               "bit-exact counters", "packets_per_step_per_gpu": n, "device_batch": batch,
                   "key": "5-tuple (37 B)" if K == 37 else "[SrcIP] (16 B)",
                   "parallelism": f"owner-key shards x{world} (SrcIP slot; each GPU generates its shard of the stream)",
                   "windows": f"steps use stream windows 0..{win[0] - 1} (warmup first), none replayed"},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "bytes_per_packet": BYTES_PER_PKT, "kernel_avg_ms": round(avg_ms, 4),
                     "pipeline_frac": round(BYTES_PER_PKT * n * args.steps / elapsed / 1e9 / HBM_PEAK_GBS, 4),
                     # SURVEY §8d convention B: + one 32-B counter sector read + written per row
                     "pipeline_frac_b": round((BYTES_PER_PKT + args.depth * 64) * n * args.steps / elapsed / 1e9
                                              / HBM_PEAK_GBS, 4)},
        "stage_ms_per_step": {k: round(v[0] / args.steps, 3) for k, v in stages.items()},
        "heavy_hitters": {"count": len(hh.Count), "size": len(hh.Size or [])},
        "engine_counters": counters,
        "flow_dictionary": dictionary,
    }
    if window is not None:
        line["window_exchange"] = window
    if (args.width, args.depth) != (WIDTH, DEPTH):
        wl2 = f"2^{args.width.bit_length() - 1}" if args.width & (args.width - 1) == 0 else str(args.width)
        line["metric"] = f"Mpackets/s CMS update (device-resident, d={args.depth} w={wl2})"
        line["config"]["workload"] = (f"Count-Min d={args.depth} w={wl2} (configs[4] geometry when d=8 w=2^24), "
                                      f"{n / 1e6:g}M Zipf(1.1) 5-tuple headers in HBM per GPU per step (one device "
                                      f"batch), bit-exact counters")
        line["note"] = "not the headline metric (BASELINE.json metric is d=4 w=2^20)"
    if args.key != "5tuple":
        line["note"] = "secondary key layout (SURVEY §8d); the headline uses the 5-tuple key"
    if args.flows != 1 << 20:
        line["config"]["flows"] = args.flows
        line["note"] = "not the headline metric (BASELINE.json stream has 2^20 flows)"
    if route:
        line["metric"] = "Mpackets/s routed CMS update (device partition + RCCL all-to-all + insert), d=4 w=2^20"
        line["config"]["workload"] = ("configs[3]: each GPU holds a contiguous slice of the unsharded stream; a "
                                      "timed step partitions it by owner shard on the device, exchanges the runs "
                                      "(all-to-all) and inserts its shard's packets")
        line["note"] = "not the headline metric: includes the routing exchange"
    if args.host_input:
        line["metric"] = ("Mpackets/s CMS update, HOST-resident input (PCIe H2D of %s + per-window D2H of "
                          "counter rows and heavy hitters), d=4 w=2^20" % args.host_input)
        line["note"] = "not the headline metric: inputs start in pinned host memory, outputs end in host memory"
        line["config"]["host_input"] = args.host_input
    if rank == 0 and world == 1 and not args.no_cpu:
        # CPU legs on a bounded prefix of window 0, then the parity check: the same
        # prefix through a fresh engine handle must equal the sequential oracle
        m = min(n, 24_000_000)
        ph, pw = syn.generate(m, first=0)
        base, orc_state, seq_n = cpu_baseline(ph, pw, width=args.width, depth=args.depth, fields=fields,
                                              keep_state=True)
        line["cpu_baseline"] = base
        line["parity"] = parity_check(orc_state, ph[:seq_n], pw[:seq_n], args, fields)
    elif rank == 0:
        line["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def parity_check(orc_state, hdr, wl, args, fields):
    """After the timed region: the CPU leg's prefix (same packets, same seeds)
    through a fresh engine handle, whole exported state compared with the
    sequential oracle (C, S, both fingerprint arrays, both heavy-hitter lists)."""
    from go2netspectra_amd import CountMin
    cm = CountMin(args.width, args.depth, 1 << 20, 1000, flow_fields=fields, seeds=row_seeds(args.depth),
                  max_flows=args.max_flows, batch_packets=args.batch or args.packets, device=hdr.device.index or 0)
    cm.insert_headers(hdr, wl)
    cm.flush()
    got = cm.export_state()
    want = orc_state.export()
    same = {name: bool(np.array_equal(a, b)) for name, a, b in zip(("C", "S", "FPc", "FPs"), got, want)}
    hh = cm.heavy_hitters()
    same["heavy_count"] = [(h.Flow, h.Count) for h in hh.Count] == orc_state.heavy("count")
    same["heavy_size"] = [(h.Flow, h.Size) for h in hh.Size] == orc_state.heavy("size")
    cm.close()
    return {"checked_packets": int(wl.shape[0]), "bit_exact": all(same.values()), "arrays": same,
            "how": "the cpu_baseline sequential oracle's prefix of window 0 through a fresh handle"}


if __name__ == "__main__":
    main()
