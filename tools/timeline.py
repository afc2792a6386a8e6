"""Per-stream timeline summary of a rocprofv3 kernel trace (run_kernel_trace.csv).

    python tools/timeline.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv --steps 10

Steps are delimited by the last kernel of the training step (the optimizer kernel: adam_k / sgd_k,
or --marker).  For the last --steps steps it prints: wall time per step, GPU-busy time (union of all
kernel intervals), busy time per HIP stream, overlap (sum of kernel times minus the union) and the
idle gaps, plus the kernels that run concurrently with the most other work.
"""
from __future__ import annotations

import argparse
import csv
from collections import defaultdict


def union_len(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--marker", default=None, help="substring of the step's last kernel")
    a = ap.parse_args()
    rows = []
    with open(a.trace) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"]))
    rows.sort()
    markers = [a.marker] if a.marker else ["adam_k", "sgd_k"]
    ends = [i for i, r in enumerate(rows) if any(r[3].startswith(m) for m in markers)]
    # a step may run several optimizer kernels back to back: keep the last of each run
    last = [i for j, i in enumerate(ends) if j + 1 == len(ends) or ends[j + 1] != i + 1]
    if len(last) < a.steps + 1:
        raise SystemExit(f"only {len(last)} step markers found")
    lo, hi = last[-a.steps - 1] + 1, last[-1] + 1
    sel = rows[lo:hi]
    t0 = min(r[0] for r in sel)
    t1 = max(r[1] for r in sel)
    n = a.steps
    iv = [(r[0], r[1]) for r in sel]
    busy = union_len(iv)
    per_stream = defaultdict(list)
    for r in sel:
        per_stream[r[2]].append((r[0], r[1]))
    ksum = sum(e - s for s, e in iv)
    print(f"{len(sel) / n:.0f} kernels per step over the last {n} steps")
    print(f"wall per step          {(t1 - t0) / n / 1e3:9.1f} us")
    print(f"GPU busy (union)       {busy / n / 1e3:9.1f} us   idle {(t1 - t0 - busy) / n / 1e3:.1f} us")
    print(f"sum of kernel times    {ksum / n / 1e3:9.1f} us   overlapped {(ksum - busy) / n / 1e3:.1f} us")
    for sid, v in sorted(per_stream.items()):
        print(f"  stream {sid:>3}: {len(v) / n:5.0f} kernels, busy {union_len(v) / n / 1e3:9.1f} us")
    # kernels per stream on the step's main stream vs the rest, by total time
    agg = defaultdict(float)
    for s, e, sid, k in sel:
        agg[(sid, k.split("(")[0][:70])] += (e - s) / n / 1e3
    print("top kernels (us/step, stream):")
    for (sid, k), v in sorted(agg.items(), key=lambda x: -x[1])[:25]:
        print(f"  {v:8.1f}  s{sid:<3} {k}")


if __name__ == "__main__":
    main()
