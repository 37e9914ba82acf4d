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
cm.insert_headers(hdr, wl)
cm.flush()
torch.cuda.synchronize()
for i in range(6):
    t = time.perf_counter()
    a = cm.heavy_hitters_arrays()
    dt = time.perf_counter() - t
    print(f"hh {i}: {dt*1e3:.3f} ms  count {len(a[1])} size {len(a[3])}", flush=True)
