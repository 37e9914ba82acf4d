"""Heavy-hitter list calls on the handle's own stream vs through a snapshot view (its own
stream), after bursts of 100M-packet windows: do the 18-36 ms first-dispatch stalls follow
the stream?  usage: python tools/hh_view_probe.py [rounds=4]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from go2netspectra_amd import CountMin, SyntheticTraffic

FIELDS = ["SrcIP", "DstIP", "SrcPort", "DstPort", "Protocol"]
N = 100_000_000
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 4
syn = SyntheticTraffic(flows=1 << 20)
hdr = torch.empty((N, 64), dtype=torch.uint8, device="cuda")
wl = torch.empty((N,), dtype=torch.int32, device="cuda")
seeds = np.array([0x9747B28C, 0x1B873593, 0xCC9E2D51, 0x85EBCA6B], np.uint32)
cm = CountMin(1 << 20, 4, 1 << 20, 1000, flow_fields=FIELDS, seeds=seeds, max_flows=1 << 22, batch_packets=N)
view = cm.view()
win = 0


def burst(k):
    global win
    for _ in range(k):
        syn.fill(hdr, wl, first=win * N)
        win += 1
        cm.insert_headers(hdr, wl)
        cm.flush()
    torch.cuda.synchronize()


def timed(fn, k=6):
    out = []
    for _ in range(k):
        t = time.perf_counter()
        fn()
        out.append((time.perf_counter() - t) * 1e3)
    return out


def via_view():
    view.refresh()
    view.heavy_hitters_arrays()


burst(20)
cm.heavy_hitters_arrays()
via_view()
for r in range(rounds):
    burst(10)
    a = timed(cm.heavy_hitters_arrays)
    burst(10)
    b = timed(via_view)
    print(f"round {r}: handle stream {' '.join(f'{x:.1f}' for x in a)} | view stream {' '.join(f'{x:.1f}' for x in b)}",
          flush=True)
