#!/usr/bin/env python
"""Micro-benchmark of the conv kernels on the CNN-B1 layer shapes (batch 256 by default).

    python tools/bench_conv.py [--batch 256] [--iters 20] [--only fwd1,wgrad1,...]

Each case is timed with HIP events over ``iters`` launches; run it under
``rocprofv3 --pmc ... -- python tools/bench_conv.py --only fwd1`` for counters of one kernel.
"""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from pyspark_tf_gke_amd.ops import nn as K  # noqa: E402

# (name, H, W, Cin, Cout, pool)
LAYERS = [("1", 256, 320, 4, 8, True), ("2", 128, 160, 8, 16, True), ("3", 64, 80, 16, 32, True),
          ("4", 32, 40, 32, 64, True), ("5", 16, 20, 64, 64, False)]


def cases(B):
    dev = "cuda"
    for name, H, W, C, Co, pool in LAYERS:
        x = torch.randn(B, H, W, C, device=dev).to(torch.bfloat16)
        w = (torch.randn(Co, 5, 5, C, device=dev) * 0.1).to(torch.bfloat16)
        b = torch.randn(Co, device=dev)
        al = torch.rand(H, W, Co, device=dev) * 0.3
        z = torch.empty(B, H, W, Co, device=dev, dtype=torch.bfloat16)
        aux = torch.empty(B, H // 2, W // 2, Co, device=dev, dtype=torch.bfloat16) if pool else \
            torch.empty(B, H, W, Co, device=dev, dtype=torch.bfloat16)
        epi = "pool" if pool else "prelu"
        flops = 2.0 * B * H * W * Co * 25 * C
        yield "fwd" + name, flops, lambda x=x, w=w, b=b, z=z, al=al, aux=aux, epi=epi: \
            K.conv2d_fwd_fused(x, w, b, 2, z, al, aux, epi)
        dw = torch.empty(Co, 5, 5, C, device=dev)
        yield "wgrad" + name, flops, lambda x=x, z=z, dw=dw: K.conv2d_wgrad_halo(x, z, 2, dw)
        if name != "1":
            dx = torch.empty_like(x)
            wf = torch.empty(C, 5, 5, Co, device=dev, dtype=torch.bfloat16)
            yield "dgrad" + name, flops, lambda z=z, w=w, dx=dx, wf=wf: K.conv2d_dgrad_halo(z, w, 2, dx, wf)
        dp = aux
        dz = torch.empty_like(z)
        da, db = torch.zeros(H, W, Co, device=dev), torch.zeros(Co, device=dev)
        if pool:
            yield "pbwd" + name, 0.0, lambda dp=dp, z=z, al=al, dz=dz, da=da, db=db: \
                K.prelu_pool_bwd(dp, z, al, dz, da, db)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    only = set(a.only.split(",")) if a.only else None
    for name, flops, fn in cases(a.batch):
        if only and name not in only:
            continue
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        tf = flops / ms / 1e9 if flops else 0.0
        print(f"{name:8s} {ms * 1e3:8.1f} us  {tf:7.1f} TFLOP/s", flush=True)


if __name__ == "__main__":
    main()
