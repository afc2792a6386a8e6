"""Isolated timing of the PReLU+pool backward kernels at the CNN-B1 layer 2-4 shapes (b256):
dense prelu_pool_bwd (sg) vs the sparse-record prelu_pool_bwd_sel.  Usage: python tools/sel_bench.py [--batch 256]"""
import argparse
import json

import torch

from pyspark_tf_gke_amd.ops import nn as K


def timeit(fn, iters=20):
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
    ap.add_argument("--nper", default="0")
    a = ap.parse_args()
    N, dev = a.batch, "cuda"
    for li, (C, H, W) in ((2, (16, 128, 160)), (3, (32, 64, 80)), (4, (64, 32, 40))):
        PH, PW = H // 2, W // 2
        dp = torch.randn(N, PH, PW, C, device=dev).bfloat16()
        z = torch.randn(N, H, W, C, device=dev).bfloat16()
        al = torch.full((H, W, C), 0.25, device=dev)
        dz = torch.empty_like(z)
        da = torch.zeros_like(al)
        db = torch.zeros(C, device=dev)
        zs = torch.randn(N, PH, PW, C, device=dev).bfloat16()
        arg = torch.randint(0, 4, (N, PH, PW, C), device=dev, dtype=torch.uint8)
        dzs = torch.empty_like(zs)
        dense = timeit(lambda: K.prelu_pool_bwd(dp, z, al, dz, da, db))
        for nper in [int(v) for v in a.nper.split(",")]:
            sel = timeit(lambda: K.prelu_pool_bwd_sel(dp, zs, arg, al, dzs, da, db, nper=nper))
            mb_sel = (dp.numel() * 2 + zs.numel() * 2 + arg.numel() + dzs.numel() * 2) / 1e6
            print(json.dumps({"layer": li, "nper": nper, "dense_us": round(dense, 1), "sel_us": round(sel, 1),
                              "sel_MB": round(mb_sel, 1), "sel_TBps": round(mb_sel / sel / 1e6 * 1e6 / 1e6, 2)}), flush=True)


if __name__ == "__main__":
    main()
