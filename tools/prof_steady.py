#!/usr/bin/env python3
"""Per-kernel device time of the full-batch launches only (rocprofv3 kernel trace CSV).

The bench's first batches are short (cold start: max(1M, B/32) packets) and its window-exchange
leg runs other batch sizes; roofline.kernel_avg_ms is the HIP-event average over the timed full
batches, so compare it with the launches of the largest grid of each kernel.

usage: tools/prof_steady.py [--last N] kernel_trace.csv [kernel-substring ...]
  --last N: only the last N launches of each kernel's largest grid (the timed steps
            of a bench run with warmup W and N steps: the cold first batches excluded)
"""
import csv
import statistics
import sys


def main():
    argv = sys.argv[1:]
    last = 0
    if argv and argv[0] == "--last":
        last = int(argv[1])
        argv = argv[2:]
    rows = list(csv.DictReader(open(argv[0])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    pats = argv[1:] or ["k_extract", "k_scatter_st", "k_apply", "k_ex_extract", "k_ex_pagg", "k_ex_pscatter"]
    print(f"{'kernel':58s} {'grid':>12s} {'launches':>9s} {'avg_us':>9s} {'median_us':>10s} {'min_us':>8s} {'max_us':>8s}")
    for p in pats:
        ks = [r for r in rows if p in r["Kernel_Name"]]
        if not ks:
            continue
        gmax = max(int(r["Grid_Size_X"]) for r in ks)
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in ks if int(r["Grid_Size_X"]) == gmax]
        if last:
            d = d[-last:]
        name = ks[0]["Kernel_Name"].split("(")[0][:58]
        print(f"{name:58s} {gmax:12d} {len(d):9d} {statistics.mean(d):9.1f} {statistics.median(d):10.1f} "
              f"{min(d):8.1f} {max(d):8.1f}")


if __name__ == "__main__":
    main()
