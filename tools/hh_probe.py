"""Time CountMin.heavy_hitters_arrays at the headline geometry (100M packets inserted)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from go2netspectra_amd import CountMin, SyntheticTraffic

FIELDS = ["SrcIP", "DstIP", "SrcPort", "DstPort", "Protocol"]
syn = SyntheticTraffic(flows=1 << 20)
hdr, wl = syn.generate(100_000_000)
seeds = np.array([0x9747B28C, 0x1B873593, 0xCC9E2D51, 0x85EBCA6B], np.uint32)
cm = CountMin(1 << 20, 4, 1 << 20, 1000, flow_fields=FIELDS, seeds=seeds, max_flows=1 << 22, batch_packets=100_000_000)
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 1
for _ in range(steps):
    cm.insert_headers(hdr, wl)
cm.flush()
torch.cuda.synchronize()
import ctypes as ct
from go2netspectra_amd import _lib
L = _lib.load()
for i in range(4):
    t = time.perf_counter()
    a = cm.heavy_hitters_arrays()
    dt = time.perf_counter() - t
    print(f"hh {i}: {dt*1e3:.3f} ms  count {len(a[1])} size {len(a[3])}", flush=True)
# the C call alone into preallocated buffers
nc, ns = len(a[1]), len(a[3])
cf = np.zeros((nc + 16, 37), np.uint8); cv = np.zeros(nc + 16, np.uint32)
sf = np.zeros((ns + 16, 37), np.uint8); sv = np.zeros(ns + 16, np.uint32)
for i in range(3):
    n1, n2 = ct.c_uint64(nc + 16), ct.c_uint64(ns + 16)
    t = time.perf_counter()
    L.gns_cm_heavy_hitters(cm._h, cf.ctypes.data, cv.ctypes.data, ct.byref(n1), sf.ctypes.data, sv.ctypes.data, ct.byref(n2))
    print(f"C call {i}: {(time.perf_counter() - t)*1e3:.3f} ms", flush=True)
