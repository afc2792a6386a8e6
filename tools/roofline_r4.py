#!/usr/bin/env python
"""Per-kernel roofline of one CNN-B1 training step (train_tf_ps.py:346-378, flat=True, 256x320x3,
batch B) from a rocprofv3 kernel trace, for the round-4 / round-5 kernel sets (uint8 input read by the
first layer's kernels, fused head, fused Dense dW + Adam; round 5: dense.hip forward / dX, the
multi-range Adam that also writes the flipped dgrad filters).

Each kernel of one steady-state step (between two consecutive conv1_fwd_rec_k launches) is mapped by
NAME to the op it implements; the three prelu_pool_bwd launches are told apart by their order (layers
4, 3, 2).  For every op: useful FLOPs (2 x MACs as written: layer 1 counts its 3 real channels),
COMPULSORY HBM bytes (each operand read once, each result written once), achieved TF/s and TB/s,
and the fraction of the binding roof (2.5 PF/s dense bf16 or 8 TB/s HBM).  Durations are the
kernels' own start->end times in the overlapped step (two streams), so a kernel slowed by a
concurrent one shows it.  Pass --serial to say the trace came from a serialized run.

    python tools/roofline_r4.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv [--batch 256]
"""
import argparse
import csv
import re
import sys

PEAK_TF = 2500.0
PEAK_TB = 8.0
L = [(256, 320, 3, 8, True), (128, 160, 8, 16, True), (64, 80, 16, 32, True), (32, 40, 32, 64, True),
     (16, 20, 64, 64, False)]


SPARSE: set = set()  # conv layers (2..5) running the sparse pool record (--sparse-layers)


def ops(B):
    bf, f32 = 2, 4
    o = {}

    def cf(i):
        H, W, ci, co, _ = L[i]
        return 2.0 * B * H * W * ci * co * 25

    H, W = 256, 320
    o["L1 fwd (u8 in, PReLU+pool, record)"] = (cf(0), B * H * W * 3 + B * (H // 2) * (W // 2) * 8 * (bf + bf + 1))
    o["L1 bwd (recompute, dW, dalpha, dbias)"] = (cf(0) * 2, B * H * W * 3 + B * (H // 2) * (W // 2) * 8 * (bf + bf + 1))
    for i in range(1, 5):
        H, W, ci, co, pool = L[i]
        out_hw = (H // 2) * (W // 2) if pool else H * W
        if i + 1 in SPARSE:  # sparse pool record (engine SPARSE_POOL): no full-resolution z / dZ
            o[f"L{i + 1} fwd"] = (cf(i), B * H * W * ci * bf + B * out_hw * co * (bf + bf + 1))
            o[f"L{i + 1} dgrad"] = (cf(i), B * out_hw * co * (bf + 1) + B * H * W * ci * bf)
            o[f"L{i + 1} wgrad"] = (cf(i), B * H * W * ci * bf + B * out_hw * co * (bf + 1))
            o[f"L{i + 1} PReLU+pool bwd"] = (0.0, B * out_hw * co * (bf + bf + 1 + bf))
            continue
        o[f"L{i + 1} fwd"] = (cf(i), B * H * W * ci * bf + B * H * W * co * bf + B * out_hw * co * bf)
        o[f"L{i + 1} dgrad"] = (cf(i), B * H * W * co * bf + B * H * W * ci * bf)
        o[f"L{i + 1} wgrad"] = (cf(i), B * H * W * ci * bf + B * H * W * co * bf)
        o[f"L{i + 1} PReLU{'+pool' if pool else ''} bwd"] = (0.0, B * out_hw * co * bf + 2 * B * H * W * co * bf)
    F = 16 * 20 * 64
    o["Dense fwd (split-K)"] = (2.0 * B * F * 2048, B * F * bf + 2048 * F * bf + B * 2048 * f32)
    o["head (Dense2 + MSE, fwd+bwd)"] = (8.0 * B * 2048, B * 2048 * f32 * 2)
    o["Dense dX"] = (2.0 * B * F * 2048, B * 2048 * bf + 2048 * F * bf + B * F * bf)
    o["Dense dW + Adam"] = (2.0 * B * F * 2048, B * 2048 * bf + B * F * bf + 2048 * F * (3 * f32 + 3 * f32 + bf))
    o["Adam (small params)"] = (0.0, 1.42e6 * 34)  # p, g, m, v read; p, m, v, bf16 p, g = 0 written
    o["dgrad filter flips"] = (0.0, 2 * 2 * 25 * (8 * 16 + 16 * 32 + 32 * 64 + 64 * 64))
    return o


def classify(name, ppb_seen):
    m = re.search(r"conv_fwd_strip_k<(\d+), 5, (\d+), \d+, \d+, (\d+)", name)
    if m:
        C, NF, E = int(m.group(1)), int(m.group(2)), int(m.group(3))
        if E in (1, 2, 3):
            return {8: "L2 fwd", 16: "L3 fwd", 32: "L4 fwd", 64: "L5 fwd"}.get(C)
        return {16: "L2 dgrad", 32: "L3 dgrad", 64: "L4 dgrad" if NF == 2 else "L5 dgrad"}.get(C)
    m = re.search(r"conv32_k<(\d+), (\d+), (\d+)", name)
    if m:
        C, CO, E = int(m.group(1)), int(m.group(2)), int(m.group(3))
        if E in (1, 2):
            return {16: "L3 fwd", 32: "L4 fwd", 64: "L5 fwd"}.get(C)
        return {(32, 16): "L3 dgrad", (64, 32): "L4 dgrad", (64, 64): "L5 dgrad"}.get((C, CO))
    m = re.search(r"conv_wgrad_strip_k<(\d+),", name)
    if m:
        return {8: "L2 wgrad", 16: "L3 wgrad", 32: "L4 wgrad", 64: "L5 wgrad"}.get(int(m.group(1)))
    if "prelu_pool_bwd" in name or "ppb_rows_k" in name:
        k = ["L4 PReLU+pool bwd", "L3 PReLU+pool bwd", "L2 PReLU+pool bwd"][min(ppb_seen[0], 2)]
        ppb_seen[0] += 1
        return k
    if "prelu_bwd" in name:
        return "L5 PReLU bwd"
    if "conv1_fwd" in name:
        return "L1 fwd (u8 in, PReLU+pool, record)"
    if "conv1_bwd" in name:
        return "L1 bwd (recompute, dW, dalpha, dbias)"
    if "EpiAdam" in name:
        return "Dense dW + Adam"
    if "dense_fwd_sk_k" in name:
        return "Dense fwd (split-K)"
    if "dense_dx" in name:
        return "Dense dX"
    if name.startswith("adam_multi_k"):
        return "Adam (small params)"
    if "EpiAtomic" in name:
        return "Dense fwd (split-K)"
    if "gemm_kernel<256, 80" in name or "gemm_kernel<256, 64" in name or "Cijk" in name:
        return "Dense dX"
    if "head_row" in name or "head_col" in name:
        return "head (Dense2 + MSE, fwd+bwd)"
    if name.startswith("adam_k"):
        return "Adam (small params)"
    if "flip" in name:
        return "dgrad filter flips"
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--step", type=int, default=-2)
    ap.add_argument("--serial", action="store_true", help="label: the trace is of a serialized run (PTG_SIDE_STREAM=0)")
    ap.add_argument("--sparse-layers", default=None,
                    help="conv layers on the sparse pool record (default: 2,3 from batch 128, as the engine)")
    a = ap.parse_args()
    sl = a.sparse_layers if a.sparse_layers is not None else ("2,3" if a.batch >= 128 else "")
    SPARSE.update(int(v) for v in sl.split(",") if v)
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if "conv1_fwd" in r["Kernel_Name"]]
    s, e = starts[a.step - 1], starts[a.step]
    ks = rows[s:e]
    table = ops(a.batch)
    t0 = int(ks[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in ks)
    print(f"CNN-B1 b{a.batch} ({'serialized, one stream' if a.serial else 'overlapped, two streams'}): {len(ks)} kernels in "
          f"one step, first start -> last end {(t1 - t0) / 1e3:.1f} us")
    print(f"{'op':40s} {'us':>7s} {'GFLOP':>7s} {'MB':>8s} {'TF/s':>7s} {'TB/s':>6s} {'bound':>7s} {'%roof':>6s} "
          f"{'floor us':>8s}")
    acc = {}
    ppb_seen = [0]
    other = []
    for r in ks:
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        name = r["Kernel_Name"].replace("void ", "")
        op = classify(name, ppb_seen)
        if op is None or op not in table:
            other.append((name[:60], us))
            continue
        acc[op] = acc.get(op, 0.0) + us
    tot = floor_tot = 0.0
    for op, (fl, by) in table.items():
        if op not in acc:
            continue
        us = acc[op]
        tf = fl / us / 1e6 if us else 0.0
        tb = by / us / 1e6 if us else 0.0
        floor = max(fl / (PEAK_TF * 1e6), by / (PEAK_TB * 1e6))
        bound = "compute" if fl / (PEAK_TF * 1e6) >= by / (PEAK_TB * 1e6) else "HBM"
        tot += us
        floor_tot += floor
        print(f"{op:40s} {us:7.1f} {fl / 1e9:7.2f} {by / 1e6:8.1f} {tf:7.1f} {tb:6.2f} {bound:>7s} "
              f"{100 * floor / us:6.1f} {floor:8.1f}")
    for n, us in other:
        print(f"{'other: ' + n:40s} {us:7.1f}")
        tot += us
    print(f"{'SUM of kernel times':40s} {tot:7.1f}   (roofline floor of the mapped ops {floor_tot:.1f} us)")
    return 0


if __name__ == "__main__":
    sys.exit(main())
