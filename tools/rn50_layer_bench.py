#!/usr/bin/env python
"""Per-layer timing of the ResNet-50 conv GEMMs (fwd / dgrad / wgrad) and BN passes at batch B.

Every unique conv shape of keras.applications ResNet-50 v1 is timed once through the same dispatch
the graph engine uses (nn/graph_ops.py conv_forward / conv_wgrad / conv_dgrad) with HIP events;
the table shows us/call, TFLOP/s and the per-step total weighted by how often the shape occurs, so
GEMM-engine variants can be A/B'd in one GPU call.

    python tools/rn50_layer_bench.py [--batch 128] [--iters 10] [--only fwd,dgrad,wgrad,bn]
"""
from __future__ import annotations

import argparse
import collections
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from pyspark_tf_gke_amd.nn import graph_ops as G  # noqa: E402
from pyspark_tf_gke_amd.ops import bn as KB  # noqa: E402


def rn50_convs():
    """(H_in, Cin, Cout, k, stride, pad) of every conv, in network order."""
    out = [(224, 4, 64, 7, 2, 3)]
    h, cin = 56, 64
    for mid, cout, blocks, stride in [(64, 256, 3, 1), (128, 512, 4, 2), (256, 1024, 6, 2), (512, 2048, 3, 2)]:
        for b in range(blocks):
            s = stride if b == 0 else 1
            out.append((h, cin, mid, 1, s, 0))
            ho = h // s
            out.append((ho, mid, mid, 3, 1, 1))
            out.append((ho, mid, cout, 1, 1, 0))
            if b == 0:
                out.append((h, cin, cout, 1, s, 0))
            h, cin = ho, cout
    return out


def timeit(fn, iters):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="fwd,dgrad,wgrad,bn")
    a = ap.parse_args()
    kinds = set(a.only.split(","))
    B, dev = a.batch, "cuda"
    cnt = collections.Counter(rn50_convs())
    tot = collections.defaultdict(float)
    flops_tot = collections.defaultdict(float)
    print(f"{'layer':34s} {'n':>2s} {'kind':6s} {'us':>8s} {'TF/s':>7s}")
    for (H, C, Co, k, s, p), n in cnt.items():
        OH = (H + 2 * p - k) // s + 1
        x = (torch.randn(B, H, H, C, device=dev) * 0.5).to(torch.bfloat16)
        w = (torch.randn(Co, k, k, C, device=dev) * 0.05).to(torch.bfloat16)
        z = torch.empty(B, OH, OH, Co, device=dev, dtype=torch.bfloat16)
        dz = (torch.randn(B, OH, OH, Co, device=dev) * 0.1).to(torch.bfloat16)
        dw = torch.zeros(Co, k, k, C, device=dev)
        dx = torch.zeros(B, H, H, C, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * B * OH * OH * Co * k * k * C
        name = f"{H}x{H}x{C}->{Co} k{k}s{s}"
        cases = []
        if "fwd" in kinds:
            cases.append(("fwd", lambda: G.conv_forward(x, w, None, s, p, z)))
        if "wgrad" in kinds:
            cases.append(("wgrad", lambda: G.conv_wgrad(x, dz, s, p, dw)))
        if "dgrad" in kinds and C != 4:
            ws = _WS()
            cases.append(("dgrad", lambda ws=ws: G.conv_dgrad(dz, w, s, p, dx, s > 1, ws, "k")))
        for kind, fn in cases:
            us = timeit(fn, a.iters)
            tot[kind] += us * n
            flops_tot[kind] += fl * n
            print(f"{name:34s} {n:2d} {kind:6s} {us:8.1f} {fl / us / 1e6:7.1f}")
        if "bn" in kinds:
            M = B * OH * OH
            part = KB.part_buffer(Co, dev)
            zz = z.normal_().to(torch.bfloat16) if False else dz
            us = timeit(lambda: KB.bn_stats(zz, part), a.iters)
            tot["bn_stats"] += us * n
            print(f"{name:34s} {n:2d} {'bnst':6s} {us:8.1f} {M * Co * 2 / us / 1e6:7.1f} TB/s")
    print("per-step totals (ms):", {k: round(v / 1e3, 3) for k, v in tot.items()},
          "TF/s:", {k: round(flops_tot[k] / tot[k] / 1e6, 1) for k in flops_tot})


class _WS:
    def __init__(self):
        self.d = {}

    def get(self, key, shape, dtype, dev, zero=False):
        t = self.d.get(key)
        if t is None or tuple(t.shape) != tuple(shape):
            t = torch.zeros(shape, dtype=dtype, device=dev)
            self.d[key] = t
        return t


if __name__ == "__main__":
    main()
