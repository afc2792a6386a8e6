#!/usr/bin/env python
"""Summarise a rocprofv3 --stats kernel_stats.csv: top kernels by total time (per-step if --steps)."""
import csv
import sys


def main(path, steps=1, top=30):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"{'total_ms':>9} {'calls':>6} {'avg_us':>9} {'pct':>6}  kernel")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        n = r["Name"]
        print(f"{float(r['TotalDurationNs']) / 1e6:9.3f} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.1f} "
              f"{float(r['TotalDurationNs']) / tot * 100:5.1f}%  {n[:140]}")
    print(f"total GPU kernel time {tot / 1e6:.3f} ms; per step (/{steps}) {tot / 1e6 / steps:.3f} ms")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 1)
