"""Phase A of tools/hh_spikes.py (the second heavy-hitter call after a burst of
inserts stalls 18-36 ms before its first kernel runs) with the HIP runtime log on
(AMD_LOG_LEVEL set by the caller), so the log's own timestamps show what the
runtime does during the stall.  usage: python tools/hh_spike_log.py [windows=35]"""
import ctypes as ct
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from go2netspectra_amd import CountMin, SyntheticTraffic, _lib

FIELDS = ["SrcIP", "DstIP", "SrcPort", "DstPort", "Protocol"]
N = 100_000_000
wins = int(sys.argv[1]) if len(sys.argv) > 1 else 35
syn = SyntheticTraffic(flows=1 << 20)
hdr = torch.empty((N, 64), dtype=torch.uint8, device="cuda")
wl = torch.empty((N,), dtype=torch.int32, device="cuda")
seeds = np.array([0x9747B28C, 0x1B873593, 0xCC9E2D51, 0x85EBCA6B], np.uint32)
cm = CountMin(1 << 20, 4, 1 << 20, 1000, flow_fields=FIELDS, seeds=seeds, max_flows=1 << 22, batch_packets=N)
for k in range(wins):
    syn.fill(hdr, wl, first=k * N)
    cm.insert_headers(hdr, wl)
    cm.flush()
torch.cuda.synchronize()
L = _lib.load()
print("MARK first call", flush=True)
a = cm.heavy_hitters_arrays()
nc, ns = len(a[1]) + 16, len(a[3]) + 16
cf = np.zeros((nc, 37), np.uint8); cv = np.zeros(nc, np.uint32)
sf = np.zeros((ns, 37), np.uint8); sv = np.zeros(ns, np.uint32)
for i in range(4):
    n1, n2 = ct.c_uint64(nc), ct.c_uint64(ns)
    L.gns_cm_version = None
    t = time.perf_counter()
    _lib.check(L.gns_cm_heavy_hitters(cm._h, cf.ctypes.data, cv.ctypes.data, ct.byref(n1), sf.ctypes.data,
                                      sv.ctypes.data, ct.byref(n2)))
    print(f"call {i}: {(time.perf_counter() - t) * 1e3:.3f} ms", flush=True)
