#!/usr/bin/env python
"""Aggregate rocprofv3 --pmc CSV output (counter_collection.csv files) per kernel (averaged per dispatch)."""
import collections
import csv
import sys


def main(paths, filt=""):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for p in paths:
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"]
            if filt and filt not in k:
                continue
            k = k.split("(")[0][:90]
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add((p, r["Dispatch_Id"]))
    for k, v in agg.items():
        n = max(1, len(disp[k]) // max(1, len(paths)))
        print(k, f"[{n} dispatches]")
        for c in sorted(v):
            print(f"    {c:28s} {v[c] / n:14.4g}")


if __name__ == "__main__":
    main([a for a in sys.argv[1:] if a.endswith(".csv")], next((a for a in sys.argv[1:] if not a.endswith(".csv")), ""))
