#!/usr/bin/env python3
"""rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE counter CSVs -> per-kernel HBM traffic.

usage: pmc_traffic.py FETCH_CSV WRITE_CSV [out.json] [--median]

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (TCC_EA0_RDREQ/WRREQ x 64 B).
MI355X_MICROARCH.md (HBM section): on gfx950 FETCH_SIZE reports half of the
bytes of wide coalesced streaming reads, so reads are doubled.  The largest
dispatch of each kernel is taken: the bench's full 100M-packet batches (the
cold-start batch and the early-exit launches of the hot fallback path are
smaller).  --median takes the median dispatch instead (SuperSpread: the first
window's batch starts from empty registers, so every packet-row is a
candidate there; the steady-state batches are the median).  Output keys are
bench.py stage names.
"""
import collections
import csv
import json
import statistics
import sys

STAGE = {"k_extract": "extract", "k_resolve": "resolve", "k_scatter": "scatter", "k_scatter_st": "scatter", "k_apply": "apply",
         "k_hot_sum": "hot_sum", "k_hot_verify": "hot_verify", "k_tscan_down": "scan", "k_synth": "synth",
         "k_ss_extract_hdr": "extract", "k_ss_extract": "extract", "k_ss_walk_mv": "walk_mv"}


def load(path):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].split("<")[0].split("::")[-1].strip()
        d[name].append(float(r["Counter_Value"]) * 1024.0)
    return d


def main():
    median = "--median" in sys.argv
    argv = [a for a in sys.argv if a != "--median"]
    pick = (lambda v: statistics.median_low(v)) if median else max
    fetch, write = load(argv[1]), load(argv[2])
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f = pick(fetch.get(k, [0.0])) * 2.0
        w = pick(write.get(k, [0.0]))
        rec = {"fetch_bytes_x2": round(f), "write_bytes": round(w), "bytes": round(f + w),
               "dispatches": len(fetch.get(k, []))}
        out[STAGE.get(k, k)] = rec
        print(f"{k:24s} read {f / 1e9:8.3f} GB  write {w / 1e9:8.3f} GB  per dispatch")
    if len(argv) > 3:
        json.dump(out, open(argv[3], "w"), indent=1)


if __name__ == "__main__":
    main()
