"""Is the 18-36 ms first-dispatch stall a power-state transition after sustained load?
H: 25-window burst, 200 ms idle, then 3 heavy-hitter calls.
I: 25-window burst, then 8 calls back to back, printing each call's start offset.
J: 25-window burst, 8 calls with 2 ms host sleeps between them.
The GPU's current SCLK (sysfs pp_dpm_sclk, read-only) is sampled around each phase."""
import ctypes as ct
import glob
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from go2netspectra_amd import CountMin, SyntheticTraffic, _lib

FIELDS = ["SrcIP", "DstIP", "SrcPort", "DstPort", "Protocol"]
N = 100_000_000
syn = SyntheticTraffic(flows=1 << 20)
hdr = torch.empty((N, 64), dtype=torch.uint8, device="cuda")
wl = torch.empty((N,), dtype=torch.int32, device="cuda")
seeds = np.array([0x9747B28C, 0x1B873593, 0xCC9E2D51, 0x85EBCA6B], np.uint32)
cm = CountMin(1 << 20, 4, 1 << 20, 1000, flow_fields=FIELDS, seeds=seeds, max_flows=1 << 22, batch_packets=N)
L = _lib.load()
win = 0


def sclk():
    out = []
    for p in glob.glob("/sys/class/drm/card*/device/pp_dpm_sclk"):
        try:
            cur = [l for l in open(p).read().splitlines() if l.endswith("*")]
            out.append(cur[0] if cur else "?")
        except OSError:
            pass
    return ";".join(out) or "n/a"


def burst(k=25):
    global win
    for _ in range(k):
        syn.fill(hdr, wl, first=win * N)
        win += 1
        cm.insert_headers(hdr, wl)
        cm.flush()
    torch.cuda.synchronize()
    return time.perf_counter()


burst(5)
a = cm.heavy_hitters_arrays()
nc, ns = len(a[1]) * 4 + 64, len(a[3]) * 4 + 64
cf = np.zeros((nc, 37), np.uint8); cv = np.zeros(nc, np.uint32)
sf = np.zeros((ns, 37), np.uint8); sv = np.zeros(ns, np.uint32)


def c_call():
    n1, n2 = ct.c_uint64(nc), ct.c_uint64(ns)
    _lib.check(L.gns_cm_heavy_hitters(cm._h, cf.ctypes.data, cv.ctypes.data, ct.byref(n1), sf.ctypes.data,
                                      sv.ctypes.data, ct.byref(n2)))


def series(label, t_end, k, gap):
    res = []
    for _ in range(k):
        if gap:
            time.sleep(gap)
        t = time.perf_counter()
        c_call()
        res.append(f"+{(t - t_end) * 1e3:.1f}:{(time.perf_counter() - t) * 1e3:.1f}")
    print(f"{label}: sclk_after={sclk()}  " + " ".join(res), flush=True)


for rep in range(2):
    t = burst()
    print(f"sclk right after burst: {sclk()}", flush=True)
    time.sleep(0.2)
    series(f"H{rep} (200 ms idle first)", t, 3, 0)
    series(f"I{rep} (back to back)", burst(), 8, 0)
    series(f"J{rep} (2 ms apart)", burst(), 8, 0.002)
