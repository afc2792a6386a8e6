"""HBM rate of the fused Adam update at CNN-B1's Dense size (41.9M params): the flat adam_k pass
(p, m, v, g read; p, m, v, bf16 p written: 30 B/param) and the dW GEMM with Adam in its epilogue
(linear_dw_adam: 26 B/param, the gradient never stored) at batch 32 / 256, each timed alone after a
read that evicts the Infinity Cache."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyspark_tf_gke_amd.ops import nn as K  # noqa: E402


def timed(fn, flush, iters=10):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        flush.sum()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        ts.append((a, b))
    torch.cuda.synchronize()
    us = sorted(x.elapsed_time(y) * 1000 for x, y in ts)
    return us[len(us) // 2]


def main():
    dev = "cuda"
    N, Kd = 2048, 20480
    n = N * Kd
    flush = torch.empty(128 << 20, device=dev)
    p, m, v, g = (torch.randn(n, device=dev) * 0.01 for _ in range(4))
    pb = torch.empty(n, device=dev, dtype=torch.bfloat16)
    res = {}
    t = timed(lambda: K.adam(p, g, m, v, pb, 1e-3, 0.9, 0.999, 1e-7), flush)
    res["adam_k_us"] = round(t, 1)
    res["adam_k_TBs"] = round(30 * n / t / 1e6, 2)
    for B in (32, 64, 128, 256):
        dz = torch.randn(B, N, device=dev).bfloat16()
        x = torch.randn(B, Kd, device=dev).bfloat16()
        t = timed(lambda: K.linear_dw_adam(dz, x, p.view(N, Kd), m.view(N, Kd), v.view(N, Kd), pb.view(N, Kd),
                                           1e-3, 0.9, 0.999, 1e-7), flush)
        res[f"dw_adam_b{B}_us"] = round(t, 1)
        res[f"dw_adam_b{B}_TBs"] = round(26 * n / t / 1e6, 2)
    copy_src = torch.empty(n * 2, device=dev)
    copy_dst = torch.empty(n * 2, device=dev)
    t = timed(lambda: copy_dst.copy_(copy_src), flush)
    res["copy_336MB_us"] = round(t, 1)
    res["copy_TBs"] = round(2 * 8 * n / t / 1e6, 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
