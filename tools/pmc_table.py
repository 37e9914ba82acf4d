#!/usr/bin/env python3
"""rocprofv3 --pmc counter CSVs -> per-kernel median counter values (one row per kernel).

usage: pmc_table.py CSV [CSV ...]
"""
import collections
import csv
import statistics
import sys


def main():
    d = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in sys.argv[1:]:
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"].split("(")[0].split("::")[-1].strip()
            d[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k in sorted(d):
        vals = {c: statistics.median(v) for c, v in d[k].items()}
        print(k)
        for c in sorted(vals):
            print(f"    {c:28s} {vals[c]:16.4g}")


if __name__ == "__main__":
    main()
