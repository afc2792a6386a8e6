#!/usr/bin/env python
"""Per-kernel MFMA / LDS / memory report from the three PMC passes of tools/gpu_pmc_evidence.sh.

usage: python tools/pmc_report.py <dir_a> <dir_b> [<dir_c>] [steps]   (dir_c: a WRITE_SIZE pass)

  MFMA util   SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs * 1024 SIMDs)  (busy fraction of
              every SIMD's matrix core over the kernel; GUI_ACTIVE reads high on sub-0.3 ms
              dispatches, which biases the ratio low there - MI355X_MICROARCH.md)
  LDS confl   SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS  (conflict cycles per LDS instruction)
  wait        SQ_WAIT_ANY / SQ_WAVE_CYCLES        (fraction of wave time stalled)
  rd/wr GB/s  FETCH_SIZE, WRITE_SIZE (KB) over the kernel time; on gfx950 FETCH_SIZE counts half the
              bytes of wide coalesced streaming reads, so rd is a lower bound (up to 2x)
"""
import collections
import csv
import os
import sys


def load(d):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    name = {}
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        k = int(r["Dispatch_Id"])
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        dur[k] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        name[k] = r["Kernel_Name"]
    return per, dur, name


def short(n):
    n = n.replace("void ", "")
    i = n.find("(")
    return (n[:i] if i > 0 else n)[:95]


def main():
    args = sys.argv[1:]
    dirs = [a for a in args if os.path.isdir(a)]
    rest = [a for a in args if not os.path.isdir(a)]
    da, db = dirs[0], dirs[1]
    dc = dirs[2] if len(dirs) > 2 else None
    steps = float(rest[0]) if rest else 1.0
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for d in [x for x in (da, db, dc) if x]:
        per, dur, name = load(d)
        for k, cs in per.items():
            a = agg[short(name[k])]
            for c, v in cs.items():
                a[c] += v
            if d == da:
                a["_t"] += dur[k]
                a["_n"] += 1
            elif d == db:
                a["_tb"] += dur[k]
            else:
                a["_tc"] += dur[k]
    rows = sorted(agg.items(), key=lambda kv: -kv[1]["_t"])
    tot = sum(a["_t"] for _, a in rows)
    print(f"{'ms/step':>8} {'%':>5} {'MFMA%':>6} {'LDScf':>6} {'wait%':>6} {'rdGB/s':>7} {'wrGB/s':>7}  kernel")
    for n, a in rows:
        if a["_t"] < 0.003 * tot:
            continue
        gui = a.get("GRBM_GUI_ACTIVE", 0.0)
        mf = a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) / (gui / 8 * 1024) * 100 if gui else 0.0
        lds = a.get("SQ_LDS_BANK_CONFLICT", 0.0) / max(a.get("SQ_INSTS_LDS", 0.0), 1.0)
        wt = a.get("SQ_WAIT_ANY", 0.0) / max(a.get("SQ_WAVE_CYCLES", 0.0), 1.0) * 100
        rd = a.get("FETCH_SIZE", 0.0) * 1024 / max(a["_tb"], 1e-12) / 1e9
        wr = a.get("WRITE_SIZE", 0.0) * 1024 / max(a["_tc"], 1e-12) / 1e9
        print(f"{a['_t'] / steps * 1e3:8.3f} {a['_t'] / tot * 100:5.1f} {mf:6.1f} {lds:6.2f} {wt:6.1f} {rd:7.0f} {wr:7.0f}  {n}")


if __name__ == "__main__":
    main()
