"""Where do the occasional 18-36 ms heavy-hitter calls come from?  The kernel
trace (profiles/r06_hh_spike_trace.txt) shows the first kernel of such a call
dispatched that late after the host launched it, with no host preemption.
Hypothesis: freeing a large host buffer (munmap) between calls -- the numpy
output arrays of the previous call -- stalls the process's GPU queues.
Phases, 20 calls each, at the driver's list sizes:
  A  C call into preallocated buffers, nothing freed in between
  B  as A, with a 16 MB numpy array allocated, touched and freed before each call
  C  as B, the array never touched
  D  heavy_hitters_arrays() (fresh output arrays each call)
  E  a one-key query (a tiny GPU op) after freeing a touched 16 MB array
  F  C calls 5 ms apart (the GPU idle in between)
  G  one 100M-packet window inserted before each C call (the bench's window shape)
usage: python tools/hh_spikes.py [windows=35]"""
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
a = cm.heavy_hitters_arrays()
nc, ns = len(a[1]) + 16, len(a[3]) + 16
cf = np.zeros((nc, 37), np.uint8); cv = np.zeros(nc, np.uint32)
sf = np.zeros((ns, 37), np.uint8); sv = np.zeros(ns, np.uint32)


def c_call():
    n1, n2 = ct.c_uint64(nc), ct.c_uint64(ns)
    _lib.check(L.gns_cm_heavy_hitters(cm._h, cf.ctypes.data, cv.ctypes.data, ct.byref(n1), sf.ctypes.data,
                                      sv.ctypes.data, ct.byref(n2)))


def churn(touch):
    x = np.empty(16 << 20, np.uint8)
    if touch:
        x[::4096] = 1
    del x


key = np.ascontiguousarray(a[0][:1])
phases = {"A": lambda: None, "B": lambda: churn(True), "C": lambda: churn(False)}
for name, pre in phases.items():
    ts = []
    for _ in range(20):
        pre()
        t = time.perf_counter()
        c_call()
        ts.append((time.perf_counter() - t) * 1e3)
    print(f"{name}: median {np.median(ts):.3f} max {max(ts):.3f} spikes(>8ms) {sum(t > 8 for t in ts)}  "
          + " ".join(f"{t:.1f}" for t in ts), flush=True)
ts = []
for _ in range(20):
    t = time.perf_counter()
    cm.heavy_hitters_arrays()
    ts.append((time.perf_counter() - t) * 1e3)
print(f"D: median {np.median(ts):.3f} max {max(ts):.3f} spikes(>8ms) {sum(t > 8 for t in ts)}  "
      + " ".join(f"{t:.1f}" for t in ts), flush=True)
ts = []
for _ in range(20):
    churn(True)
    t = time.perf_counter()
    cm.query_many(key)
    ts.append((time.perf_counter() - t) * 1e3)
print(f"E: median {np.median(ts):.3f} max {max(ts):.3f} spikes(>8ms) {sum(t > 8 for t in ts)}  "
      + " ".join(f"{t:.1f}" for t in ts), flush=True)
ts = []
for _ in range(20):
    time.sleep(0.005)
    t = time.perf_counter()
    c_call()
    ts.append((time.perf_counter() - t) * 1e3)
print(f"F: median {np.median(ts):.3f} max {max(ts):.3f} spikes(>8ms) {sum(t > 8 for t in ts)}  "
      + " ".join(f"{t:.1f}" for t in ts), flush=True)
ts = []
for k in range(12):
    syn.fill(hdr, wl, first=(wins + k) * N)
    cm.insert_headers(hdr, wl)
    cm.flush()
    torch.cuda.synchronize()
    t = time.perf_counter()
    c_call()
    ts.append((time.perf_counter() - t) * 1e3)
    nc, ns = nc + 4096, ns + 4096  # the lists grow with the windows
    cf = np.zeros((nc, 37), np.uint8); cv = np.zeros(nc, np.uint32)
    sf = np.zeros((ns, 37), np.uint8); sv = np.zeros(ns, np.uint32)
print(f"G: median {np.median(ts):.3f} max {max(ts):.3f} spikes(>8ms) {sum(t > 8 for t in ts)}  "
      + " ".join(f"{t:.1f}" for t in ts), flush=True)
