"""Does the GPU stall new work at a fixed time after a burst of load ends?
After K windows of 100M-packet inserts (the bench's load), issue a tiny GPU op
(a one-key query, ~40 us) back to back for 400 ms and print every op slower than
2 ms with its start time relative to the end of the load.  Repeated for three
bursts, then once after an idle second (no load before).
usage: python tools/gpu_stall_probe.py [windows=10]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from go2netspectra_amd import CountMin, SyntheticTraffic

FIELDS = ["SrcIP", "DstIP", "SrcPort", "DstPort", "Protocol"]
N = 100_000_000
K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
syn = SyntheticTraffic(flows=1 << 20)
hdr = torch.empty((N, 64), dtype=torch.uint8, device="cuda")
wl = torch.empty((N,), dtype=torch.int32, device="cuda")
seeds = np.array([0x9747B28C, 0x1B873593, 0xCC9E2D51, 0x85EBCA6B], np.uint32)
cm = CountMin(1 << 20, 4, 1 << 20, 1000, flow_fields=FIELDS, seeds=seeds, max_flows=1 << 22, batch_packets=N)
win = 0
key = np.zeros((1, 37), np.uint8)


def burst():
    global win
    for _ in range(K):
        syn.fill(hdr, wl, first=win * N)
        win += 1
        cm.insert_headers(hdr, wl)
        cm.flush()
    torch.cuda.synchronize()
    return time.perf_counter()


def watch(t_end, label):
    slow, n = [], 0
    while time.perf_counter() - t_end < 0.4:
        t = time.perf_counter()
        cm.query_many(key)
        d = time.perf_counter() - t
        n += 1
        if d > 2e-3:
            slow.append(f"+{(t - t_end) * 1e3:.1f}ms:{d * 1e3:.1f}")
    print(f"{label}: {n} ops in 400 ms, slow: {' '.join(slow) or 'none'}", flush=True)


for b in range(3):
    watch(burst(), f"after burst {b}")
time.sleep(1.0)
watch(time.perf_counter(), "after 1 s idle")
