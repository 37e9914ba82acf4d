"""Time CountMin.heavy_hitters_arrays at the headline geometry in the driver's
bench shape: `bench.py --steps 20 --warmup 5` inserts 25 fresh 100M-packet
windows, then the configs[3] window inserts 10 more and takes the lists
(130K count / 101K size entries on the driver box).  Usage:
    python tools/hh_probe.py [windows_before=25] [windows_after=10]
GNS_HH_TRACE=1 adds the engine's per-phase times on stderr."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from go2netspectra_amd import CountMin, SyntheticTraffic

FIELDS = ["SrcIP", "DstIP", "SrcPort", "DstPort", "Protocol"]
N = 100_000_000
before = int(sys.argv[1]) if len(sys.argv) > 1 else 25
after = int(sys.argv[2]) if len(sys.argv) > 2 else 10
syn = SyntheticTraffic(flows=1 << 20)
hdr = torch.empty((N, 64), dtype=torch.uint8, device="cuda")
wl = torch.empty((N,), dtype=torch.int32, device="cuda")
seeds = np.array([0x9747B28C, 0x1B873593, 0xCC9E2D51, 0x85EBCA6B], np.uint32)
cm = CountMin(1 << 20, 4, 1 << 20, 1000, flow_fields=FIELDS, seeds=seeds, max_flows=1 << 22, batch_packets=N)
win = 0


def windows(k):
    global win
    for _ in range(k):
        syn.fill(hdr, wl, first=win * N)
        win += 1
        cm.insert_headers(hdr, wl)
        cm.flush()
    torch.cuda.synchronize()


def timed(tag, reps):
    for i in range(reps):
        t = time.perf_counter()
        a = cm.heavy_hitters_arrays()
        dt = time.perf_counter() - t
        print(f"{tag} hh {i}: {dt * 1e3:.3f} ms  count {len(a[1])} size {len(a[3])}", flush=True)
    return a


windows(before)
timed(f"after {win} windows", 3)  # the bench's warm call, then repeats
windows(after)
a = timed(f"after {win} windows", 4)
# the C call alone into preallocated buffers
import ctypes as ct
from go2netspectra_amd import _lib
L = _lib.load()
nc, ns = len(a[1]), len(a[3])
cf = np.zeros((nc + 16, 37), np.uint8); cv = np.zeros(nc + 16, np.uint32)
sf = np.zeros((ns + 16, 37), np.uint8); sv = np.zeros(ns + 16, np.uint32)
for i in range(3):
    n1, n2 = ct.c_uint64(nc + 16), ct.c_uint64(ns + 16)
    t = time.perf_counter()
    L.gns_cm_heavy_hitters(cm._h, cf.ctypes.data, cv.ctypes.data, ct.byref(n1), sf.ctypes.data, sv.ctypes.data,
                           ct.byref(n2))
    print(f"C call {i}: {(time.perf_counter() - t) * 1e3:.3f} ms", flush=True)
