#!/usr/bin/env python
"""Summarise a rocprofv3 kernel trace: top kernels by total time (per step with ``steps``).

Accepts either ``--stats`` CSV output (``*kernel_stats.csv``) or the rocpd SQLite database
(``*_results.db``, rocprofv3's default output format).  With a database, kernels are also split by
grid size (``--by-grid``) so the per-layer launches of one template are told apart.
"""
import argparse
import csv
import sqlite3


def _rows_csv(path):
    for r in csv.DictReader(open(path)):
        yield r["Name"], int(r["Calls"]), float(r["TotalDurationNs"])


def _rows_db(path, by_grid):
    c = sqlite3.connect(path)
    key = "name, grid_x" if by_grid else "name"
    q = f"select name, {'grid_x' if by_grid else '0'}, count(*), sum(duration) from kernels group by {key}"
    for name, gx, n, tot in c.execute(q):
        yield (f"{name} [grid {gx}]" if by_grid else name), int(n), float(tot)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("steps", nargs="?", type=int, default=1)
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--by-grid", action="store_true")
    ap.add_argument("--skip-calls-below", type=int, default=0, help="drop kernels with fewer calls (one-time setup)")
    a = ap.parse_args(argv)
    rows = list(_rows_db(a.path, a.by_grid) if a.path.endswith(".db") else _rows_csv(a.path))
    rows = [r for r in rows if r[1] >= a.skip_calls_below]
    tot = sum(r[2] for r in rows)
    print(f"{'ms/step':>9} {'calls':>6} {'avg_us':>9} {'pct':>6}  kernel")
    for name, n, t in sorted(rows, key=lambda r: -r[2])[: a.top]:
        print(f"{t / 1e6 / a.steps:9.3f} {n:6d} {t / n / 1e3:9.1f} {t / tot * 100:5.1f}%  {name[:150]}")
    print(f"total GPU kernel time {tot / 1e6:.3f} ms; per step (/{a.steps}) {tot / 1e6 / a.steps:.3f} ms")


if __name__ == "__main__":
    main()
