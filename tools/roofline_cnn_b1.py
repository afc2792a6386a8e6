#!/usr/bin/env python
"""Per-kernel roofline table of one CNN-B1 training step (train_tf_ps.py:346-378, flat=True,
256x320x3, batch B) from a rocprofv3 kernel trace.

Every kernel of one steady-state step (the dispatches between two consecutive input-pack kernels)
is matched IN LAUNCH ORDER to the op it implements (the engine's fixed op sequence: pack, 5 conv
forwards, Dense fwd, loss, Dense / conv backward, optimizer).  For each op the table gives useful
FLOPs (2 * MACs of the op as written — layer 1 counts its 3 real input channels, not the padded 4)
and COMPULSORY bytes (each operand the op must read once + each result it must write once; saved
activations re-read in backward count; anything a kernel re-reads beyond that is its own
inefficiency), achieved TF/s and TB/s, the arithmetic intensity, and which roof binds:
compute (2.5 PF/s dense bf16) or HBM (8 TB/s) at the op's intensity, with the achieved fraction
of that roof.  Kernels the map does not know are listed as "other".

    python tools/roofline_cnn_b1.py gpurun_out/prof_cnn_b1/run_kernel_trace.csv [--batch 256]
"""
import argparse
import csv
import sys

PEAK_TF = 2500.0  # dense bf16 MFMA, TFLOP/s
PEAK_TB = 8.0     # HBM3E, TB/s


def layer_shapes(B):
    """(H, W, Cin, Cout, pool) per conv layer; 5x5 same convs."""
    return [(256, 320, 3, 8, True), (128, 160, 8, 16, True), (64, 80, 16, 32, True), (32, 40, 32, 64, True),
            (16, 20, 64, 64, False)]


def op_table(B):
    L = layer_shapes(B)
    bf, f32 = 2, 4
    ops = []

    def conv_flops(H, W, ci, co):
        return 2.0 * B * H * W * ci * co * 25

    H0, W0 = 256, 320
    ops.append(("input pack u8 -> bf16 (4 ch)", "pack_u8rgb4", 0.0, B * H0 * W0 * 3 + B * H0 * W0 * 4 * bf))
    for i, (H, W, ci, co, pool) in enumerate(L):
        cin_b = 4 if i == 0 else ci
        out_hw = (H // 2) * (W // 2) if pool else H * W
        by = B * H * W * cin_b * bf + co * 25 * cin_b * bf + B * out_hw * co * bf
        if pool:
            by += B * out_hw * co  # u8 pool-selection mask saved for backward
        ops.append((f"L{i + 1} conv fwd + PReLU{' + pool' if pool else ''}", "conv", conv_flops(H, W, ci, co), by))
    F = 16 * 20 * 64
    ops.append(("zero split-K accumulator", "Fill", 0.0, B * 2048 * f32))
    ops.append(("Dense 20480->2048 fwd (split-K)", "gemm", 2.0 * B * F * 2048, B * F * bf + 2048 * F * bf + B * 2048 * f32))
    ops.append(("Dense bias + ReLU", "bias_act", 0.0, B * 2048 * (f32 + bf + f32)))
    ops.append(("Dense 2048->2 fwd", "dense_small_fwd", 2.0 * B * 2048 * 2, B * 2048 * bf + 2048 * 2 * f32))
    ops.append(("MSE loss + dpred", "mse", 0.0, B * 2 * f32 * 3))
    ops.append(("dgrad filter flips", "conv_flip", 0.0, sum(co * 25 * ci * bf * 2 for (_, _, ci, co, _) in L[1:])))
    ops.append(("Dense 2048->2 dW", "dense_small_dw", 2.0 * B * 2048 * 2, B * 2048 * bf + B * 2 * f32 + 2048 * 2 * f32))
    ops.append(("Dense 2048->2 dX (+ReLU')", "dense_small_dx", 2.0 * B * 2048 * 2, B * 2 * f32 + B * 2048 * (bf + bf)))
    ops.append(("Dense bias grad", "col_sum", 0.0, B * 2048 * bf + 2048 * f32))
    ops.append(("Dense 20480->2048 dX", "gemm", 2.0 * B * F * 2048, B * 2048 * bf + 2048 * F * bf + B * F * bf))
    ops.append(("Dense 20480->2048 dW + fused Adam", "gemm", 2.0 * B * F * 2048,
                B * 2048 * bf + B * F * bf + 2048 * F * (3 * f32 + 3 * f32 + bf)))
    for i in range(len(L) - 1, -1, -1):
        H, W, ci, co, pool = L[i]
        cin_b = 4 if i == 0 else ci
        out_hw = (H // 2) * (W // 2) if pool else H * W
        by_act = B * out_hw * co * bf + B * H * W * co * bf * 2  # dY (pooled), z read, dZ write
        if pool:
            by_act += B * out_hw * co
        ops.append((f"L{i + 1} PReLU{' + pool' if pool else ''} bwd", "prelu", 0.0, by_act))
        ops.append((f"L{i + 1} conv wgrad", "wgrad", conv_flops(H, W, ci, co),
                    B * H * W * cin_b * bf + B * H * W * co * bf + co * 25 * cin_b * f32))
        if i > 0:
            ops.append((f"L{i + 1} conv dgrad", "conv", conv_flops(H, W, ci, co),
                        B * H * W * co * bf + co * 25 * ci * bf + B * H * W * ci * bf))
    return ops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--step", type=int, default=-2, help="which pack->pack interval (default: second to last)")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("pack_u8rgb4")]
    s, e = starts[a.step - 1], starts[a.step]
    ks = rows[s:e]
    ops = op_table(a.batch)
    step_us = (int(ks[-1]["End_Timestamp"]) - int(ks[0]["Start_Timestamp"])) / 1e3
    print(f"CNN-B1 b{a.batch}: {len(ks)} kernels in one step, first start -> last end {step_us:.1f} us")
    print(f"{'op':44s} {'kernel':34s} {'us':>7s} {'GFLOP':>7s} {'MB':>8s} {'TF/s':>7s} {'TB/s':>6s} {'F/B':>6s} "
          f"{'bound':>7s} {'%roof':>6s}")
    tot_us = tot_f = tot_b = 0.0
    oi = 0
    for r in ks:
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        kshort = name.split("<")[0].split("::")[-1][:34]
        label, flops, by = "other (" + kshort + ")", 0.0, 0.0
        while oi < len(ops):
            lbl, key, f, b = ops[oi]
            if key in name or (key == "conv" and "conv" in name and "wgrad" not in name) or \
               (key == "prelu" and "prelu" in name) or (key == "Fill" and "Fill" in name):
                label, flops, by = lbl, f, b
                oi += 1
                break
            if key in ("Fill",):  # optional op: skip when its kernel is absent
                oi += 1
                continue
            break
        tf = flops / us / 1e6 if us else 0.0
        tb = by / us / 1e6 if us else 0.0
        ai = flops / by if by else 0.0
        roof_tf = min(PEAK_TF, ai * PEAK_TB) if flops else 0.0
        bound = ("compute" if ai * PEAK_TB >= PEAK_TF else "HBM") if flops else ("HBM" if by else "-")
        frac = (tf / roof_tf if flops else (tb / PEAK_TB if by else 0.0)) * 100
        tot_us += us; tot_f += flops; tot_b += by
        print(f"{label:44s} {kshort:34s} {us:7.1f} {flops / 1e9:7.2f} {by / 1e6:8.1f} {tf:7.1f} {tb:6.2f} {ai:6.0f} "
              f"{bound:>7s} {frac:6.1f}")
    print(f"{'TOTAL (sum of kernel times)':44s} {'':34s} {tot_us:7.1f} {tot_f / 1e9:7.2f} {tot_b / 1e6:8.1f} "
          f"{tot_f / tot_us / 1e6:7.1f} {tot_b / tot_us / 1e6:6.2f}")
    t_min = max(tot_f / (PEAK_TF * 1e12), 0) + 0.0
    print(f"roofline floor of the step (each op at its own roof, summed): "
          f"{sum(max(f / (PEAK_TF * 1e6), b / (PEAK_TB * 1e6)) for _, _, f, b in ops):.1f} us; "
          f"pure compute floor {t_min * 1e6:.1f} us")
    return 0


if __name__ == "__main__":
    sys.exit(main())
