#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace run (results .db or kernel_trace.csv)
into a per-kernel table: calls, avg/min/max/total device time.

usage: tools/prof_summary.py <dir-or-file> [--json out.json]
"""
import csv
import glob
import json
import os
import sqlite3
import sys
from collections import defaultdict


def rows_from_db(path):
    c = sqlite3.connect(path)
    for name, start, end in c.execute("select name, start, end from kernels"):
        yield name, int(end) - int(start)


def rows_from_csv(path):
    with open(path) as f:
        for r in csv.DictReader(f):
            yield r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"])


def main():
    src = sys.argv[1]
    files = [src] if os.path.isfile(src) else (glob.glob(os.path.join(src, "**", "*.db"), recursive=True) +
                                                 glob.glob(os.path.join(src, "**", "*kernel_trace.csv"), recursive=True))
    agg = defaultdict(list)
    for f in files:
        it = rows_from_db(f) if f.endswith(".db") else rows_from_csv(f)
        for name, ns in it:
            agg[name].append(ns)
    total = sum(sum(v) for v in agg.values())
    out = []
    print(f"{'kernel':70s} {'calls':>6s} {'avg_us':>10s} {'min_us':>10s} {'max_us':>10s} {'total_ms':>10s} {'pct':>6s}")
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        s = sum(v)
        out.append({"kernel": name, "calls": len(v), "avg_us": s / len(v) / 1e3, "min_us": min(v) / 1e3,
                    "max_us": max(v) / 1e3, "total_ms": s / 1e6, "pct": 100.0 * s / max(total, 1)})
        print(f"{name[:70]:70s} {len(v):6d} {s/len(v)/1e3:10.1f} {min(v)/1e3:10.1f} {max(v)/1e3:10.1f} "
              f"{s/1e6:10.2f} {100.0*s/max(total,1):6.1f}")
    if "--json" in sys.argv:
        json.dump(out, open(sys.argv[sys.argv.index("--json") + 1], "w"), indent=1)


if __name__ == "__main__":
    main()
