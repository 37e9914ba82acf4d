#!/usr/bin/env python3
"""Dev probe (not part of the library): how much do two Count-Min pipelines
overlap on one GPU?  Two engines (own HIP streams) insert the same 100M
device-resident packets, first one after the other, then from two host
threads at once (ctypes drops the GIL during the C calls).  The ratio bounds
what pipelining K1 of one batch against K3/K4 of the previous one can gain.

usage: python tools/concurrency_probe.py [--packets N] [--steps K]
"""
import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--packets", type=int, default=100_000_000)
    ap.add_argument("--steps", type=int, default=4)
    args = ap.parse_args()
    import torch
    from go2netspectra_amd import CountMin, SyntheticTraffic
    from bench import FIELDS, row_seeds
    n = args.packets
    hdr, wl = SyntheticTraffic(flows=1 << 20, device=0).generate(n)
    cms = [CountMin(1 << 20, 4, 1 << 20, 1000, flow_fields=FIELDS, seeds=row_seeds(4), max_flows=1 << 21,
                    batch_packets=n, device=0) for _ in range(2)]
    for cm in cms:
        for _ in range(2):
            cm.insert_headers(hdr, wl)
        cm.flush()
    torch.cuda.synchronize()

    t0 = time.perf_counter()
    for _ in range(args.steps):
        for cm in cms:
            cm.insert_headers(hdr, wl)
    for cm in cms:
        cm.flush()
    torch.cuda.synchronize()
    seq = time.perf_counter() - t0

    def run(cm):
        for _ in range(args.steps):
            cm.insert_headers(hdr, wl)
        cm.flush()

    th = [threading.Thread(target=run, args=(cm,)) for cm in cms]
    t0 = time.perf_counter()
    for t in th:
        t.start()
    for t in th:
        t.join()
    torch.cuda.synchronize()
    par = time.perf_counter() - t0
    tot = 2 * args.steps * n
    print(json.dumps({"sequential_gpkt_s": round(tot / seq / 1e9, 2), "concurrent_gpkt_s": round(tot / par / 1e9, 2),
                      "speedup": round(seq / par, 3)}))


if __name__ == "__main__":
    main()
