"""Time the CNN-B1 Dense 20480->2048 GEMMs (batch 256) on the GPU: forward at several split-K
factors, dX, dW, dW+Adam, and hipBLASLt (torch.matmul) for the same shapes as a yardstick."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pyspark_tf_gke_amd.ops import nn as K  # noqa: E402


def timeit(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1000 / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=256)
    ap.add_argument("--k", type=int, default=20480)
    ap.add_argument("--n", type=int, default=2048)
    a = ap.parse_args()
    M, Kd, N = a.m, a.k, a.n
    dev = "cuda"
    x = torch.randn(M, Kd, device=dev).bfloat16()
    w = torch.randn(N, Kd, device=dev).bfloat16() * 0.01
    b = torch.zeros(N, device=dev)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    wsp = torch.empty(M * N, device=dev)
    dy = torch.randn(M, N, device=dev).bfloat16()
    dx = torch.empty(M, Kd, device=dev, dtype=torch.bfloat16)
    g = torch.empty(N, Kd, device=dev)
    p, m, v = torch.randn(N, Kd, device=dev), torch.zeros(N, Kd, device=dev), torch.zeros(N, Kd, device=dev)
    pb = torch.empty(N, Kd, device=dev, dtype=torch.bfloat16)
    res = {}
    for s in (0, 1, 4, 8, 16, 20, 25, 32, 40):
        res[f"fwd_splits{s}"] = timeit(lambda: K.linear_fwd(x, w, b, "relu", y, workspace=wsp, splits=s))
    from pyspark_tf_gke_amd import _native

    lib = _native.hip_lib()
    K.BLASLT_DX = False
    for bn in (-1, 0, 64, 80, 81, 82):
        lib.ptg_gemm_skinny_set(bn)
        res[f"dx_skinny{bn}"] = timeit(lambda: K.linear_dx(dy, w, dx))
        if bn == -1:
            ref = torch.matmul(dy.float(), w.float())
            res["dx_maxrel"] = float(((dx.float() - ref).abs().max() / ref.abs().max()).item())
    lib.ptg_gemm_skinny_set(-1)
    res["dx"] = timeit(lambda: K.linear_dx(dy, w, dx))
    res["dw"] = timeit(lambda: K.linear_dw(dy, x, g))
    res["dw_adam"] = timeit(lambda: K.linear_dw_adam(dy, x, p, m, v, pb, 1e-3, 0.9, 0.999, 1e-7))
    res["torch_fwd"] = timeit(lambda: torch.matmul(x, w.t()))
    res["torch_dx"] = timeit(lambda: torch.matmul(dy, w))
    res["torch_dw"] = timeit(lambda: torch.matmul(dy.t(), x))
    print(json.dumps({k: (round(v_, 1) if v_ > 0.01 else v_) for k, v_ in res.items()}))


if __name__ == "__main__":
    main()
