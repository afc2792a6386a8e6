"""Per-op timing of the CNN-B1 layer kernels at the bench shape (batch 256, 256x320x3).

Times each fused op of the reference CNN (train_tf_ps.py:351-363) in isolation with HIP events and
prints us/call and the effective HBM rate of its compulsory bytes, so kernel variants can be A/B'd
in one GPU call.  Usage: python tools/cnn_layer_bench.py [--batch 256] [--iters 20] [--only fwd1,...]
"""
from __future__ import annotations

import argparse
import json

import torch

from pyspark_tf_gke_amd.ops import nn as ops

SPEC = [(4, 8, 256, 320), (8, 16, 128, 160), (16, 32, 64, 80), (32, 64, 32, 40), (64, 64, 16, 20)]


def timeit(fn, iters):
    for _ in range(3):
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
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    only = set(a.only.split(",")) if a.only else None
    dev = "cuda"
    N = a.batch
    g = torch.Generator(device=dev).manual_seed(0)
    res = []
    for li, (C, Co, H, W) in enumerate(SPEC, 1):
        pool = li < 5
        x = (torch.rand((N, H, W, C), device=dev, generator=g) - 0.5).bfloat16()
        w = (torch.rand((Co, 5, 5, C), device=dev, generator=g) * 0.1 - 0.05).bfloat16()
        b = torch.zeros(Co, device=dev)
        al = torch.full((H, W, Co), 0.25, device=dev)
        z = torch.empty((N, H, W, Co), device=dev, dtype=torch.bfloat16)
        aux = torch.empty((N, H // 2, W // 2, Co) if pool else (N, H, W, Co), device=dev, dtype=torch.bfloat16)
        epi = "pool" if pool else "prelu"
        ops_ = {}
        ops_[f"fwd{li}"] = (lambda x=x, w=w, b=b, z=z, al=al, aux=aux, epi=epi: ops.conv2d_fwd_fused(
            x, w, b, 2, z, alpha=al, aux_out=aux, epi=epi),
            x.numel() * 2 + z.numel() * 2 + aux.numel() * 2)
        dp = torch.randn(aux.shape, device=dev, generator=g).bfloat16()
        dz = torch.empty_like(z)
        da = torch.zeros_like(al)
        db = torch.zeros(Co, device=dev)
        if pool:
            ops_[f"ppbwd{li}"] = (lambda dp=dp, z=z, al=al, dz=dz, da=da, db=db: ops.prelu_pool_bwd(dp, z, al, dz, da, db),
                                  dp.numel() * 2 + z.numel() * 4)
        else:
            ops_[f"pbwd{li}"] = (lambda dp=dp, z=z, al=al, dz=dz, da=da, db=db: ops.prelu_bwd(dp, z, al, dz, da, db),
                                 dp.numel() * 2 + z.numel() * 4)
        dw = torch.zeros((Co, 5, 5, C), device=dev)
        ops_[f"wgrad{li}"] = (lambda x=x, dz=dz, dw=dw: ops.conv2d_wgrad_halo(x, dz, 2, dw),
                              x.numel() * 2 + dz.numel() * 2)
        if li > 1:
            dx = torch.empty_like(x)
            wf = torch.empty((C, 5, 5, Co), device=dev, dtype=torch.bfloat16)
            ops_[f"dgrad{li}"] = (lambda dz=dz, w=w, dx=dx, wf=wf: ops.conv2d_dgrad_halo(dz, w, 2, dx, wf),
                                  dz.numel() * 2 + dx.numel() * 2)
            if ops.conv32_supported(H, W, Co, C, 5, 2, None):  # conv32.hip data gradient (flipped filters)
                ops_[f"dgrad32_{li}"] = (lambda dz=dz, wf=wf, dx=dx: ops.conv32(dz, wf, None, dx),
                                         dz.numel() * 2 + dx.numel() * 2)
            if ops.conv32_supported(H, W, C, Co, 5, 2, epi):
                ops_[f"fwd32_{li}"] = (lambda x=x, w=w, b=b, z=z, al=al, aux=aux, epi=epi: ops.conv32(
                    x, w, b, z, al, aux, epi), x.numel() * 2 + z.numel() * 2 + aux.numel() * 2)
            # the implicit-GEMM weight gradient of gemm.hip (split-K over the pixels, fp32 atomics)
            dwg = torch.zeros_like(dw)
            for sp in (0, 8, 32, 128):
                ops_[f"wgradG{li}_s{sp}"] = (lambda x=x, dz=dz, dwg=dwg, sp=sp: ops.conv2d_wgrad(x, dz, 1, 2, dwg, splits=sp),
                                             x.numel() * 2 + dz.numel() * 2)
            # the implicit-GEMM path of gemm.hip for the same dgrad / forward (A/B reference)
            ops_[f"dgradG{li}"] = (lambda dz=dz, w=w, dx=dx: ops.conv2d_dgrad(dz, w, 2, dx),
                                   dz.numel() * 2 + dx.numel() * 2)
            ops_[f"fwdG{li}"] = (lambda x=x, w=w, b=b, z=z: ops.conv2d_fwd(x, w, b, 1, 2, z),
                                 x.numel() * 2 + z.numel() * 2)
        for name, (fn, nbytes) in ops_.items():
            if only and name not in only:
                continue
            us = timeit(fn, a.iters)
            r = {"op": name, "us": round(us, 1), "GBps": round(nbytes / us / 1e3, 1)}
            res.append(r)
            print(json.dumps(r), flush=True)
    print(json.dumps({"total_us": round(sum(r["us"] for r in res), 1)}))


if __name__ == "__main__":
    main()
