import sys, time, os
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np, torch
from go2netspectra_amd import CountMin, SyntheticTraffic
import bench
syn = SyntheticTraffic()
hdr, wl = syn.generate(100_000_000)
cm = CountMin(1 << 20, 4, 1 << 20, 1000, flow_fields=bench.FIELDS, seeds=bench.row_seeds(4), max_flows=1 << 21, batch_packets=100_000_000)
cm.insert_headers(hdr, wl); cm.flush()
for f in ("export_counters", "heavy_hitters_arrays", "heavy_hitters"):
    t = time.perf_counter(); r = getattr(cm, f)(); dt = time.perf_counter() - t
    print(f, round(dt * 1e3, 2), "ms")
