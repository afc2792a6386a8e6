"""One training step of a rocprofv3 kernel trace as a per-stream Gantt list, with the step's
critical path marked: every kernel with its stream, start / end offset from the step start (us),
duration, and the idle gap before it on its own stream.

    python tools/step_gantt.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv [--marker conv1_fwd] [--step -2]

Steps are delimited by launches of the --marker kernel (default: the first-layer forward).
"""
import argparse
import csv
import re


def short(n):
    n = re.sub(r"^void ", "", n)
    n = n.split("(")[0]
    return n[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--marker", default="conv1_fwd")
    ap.add_argument("--step", type=int, default=-2, help="which step (python index over complete steps)")
    a = ap.parse_args()
    rows = []
    for r in csv.DictReader(open(a.trace)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Stream_Id") or r.get("Queue_Id"),
                     r["Kernel_Name"]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if a.marker in r[3]]
    if len(starts) < 3:
        raise SystemExit(f"fewer than 3 '{a.marker}' launches")
    k = a.step if a.step >= 0 else len(starts) - 1 + a.step
    lo, hi = starts[k], starts[k + 1]
    t0 = rows[lo][0]
    t_end = max(r[1] for r in rows[lo:hi])
    print(f"step {k}: {(t_end - t0) / 1000:.1f} us from the first {a.marker} to the last kernel end; "
          f"next step starts at {(rows[hi][0] - t0) / 1000:.1f} us")
    last_end = {}
    busy = {}
    print(f"{'stream':>6} {'start':>8} {'end':>8} {'dur':>7} {'gap':>6}  kernel")
    for s, e, st, name in rows[lo:hi]:
        gap = (s - last_end[st]) / 1000 if st in last_end else 0.0
        last_end[st] = e
        busy[st] = busy.get(st, 0) + (e - s)
        print(f"{st:>6} {(s - t0) / 1000:8.1f} {(e - t0) / 1000:8.1f} {(e - s) / 1000:7.1f} {gap:6.1f}  {short(name)}")
    for st, b in busy.items():
        print(f"stream {st}: busy {b / 1000:.1f} us")


if __name__ == "__main__":
    main()
