"""Time the big-Dense GEMMs of CNN-B1 (x[M, 20480] . W[2048, 20480]^T and its dX) on one MI355X:
the weight-streaming kernels of dense.hip, the older gemm.hip split-K paths and hipBLASLt
(torch.matmul) as a yardstick.  Each call is timed alone with events, after a 512 MB write that
evicts the weight from the 256 MB Infinity Cache ("cold", as inside a training step where GBs of
activations pass between two uses of the weight) and back to back ("warm").

  python tools/dense_bench.py --m 256 32 64
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pyspark_tf_gke_amd.ops import nn as K  # noqa: E402


def timed(fn, flush, iters=30, cold=True):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        if cold:
            flush.sum()  # reads 512 MB: evicts the weight, leaves clean lines (no write-back in the timing)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        ts.append((a, b))
    torch.cuda.synchronize()
    us = sorted(a.elapsed_time(b) * 1000 for a, b in ts)
    return round(us[len(us) // 2], 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[256, 64, 32])
    ap.add_argument("--k", type=int, default=20480)
    ap.add_argument("--n", type=int, default=2048)
    a = ap.parse_args()
    dev = "cuda"
    flush = torch.empty(128 << 20, device=dev)  # 512 MB
    Kd, N = a.k, a.n
    w = (torch.randn(N, Kd, device=dev) * 0.01).bfloat16()
    for M in a.m:
        x = torch.randn(M, Kd, device=dev).bfloat16()
        dy = torch.randn(M, N, device=dev).bfloat16()
        dx = torch.empty(M, Kd, device=dev, dtype=torch.bfloat16)
        res = {"M": M, "N": N, "K": Kd}
        S = K.dense_fwd_splits(M, N, Kd)
        part = torch.empty(max(S, 1), M, N, device=dev)
        acc = torch.zeros(M, N, device=dev)
        ref = x.float() @ w.float().t()
        if S:
            K.dense_fwd_parts(x, w, part, S)
            res["fwd_parts_maxrel"] = float(((part.sum(0) - ref).abs().max() / ref.abs().max()).item())
            for cold in (True, False):
                res[f"fwd_parts_{'cold' if cold else 'warm'}_us"] = timed(lambda: K.dense_fwd_parts(x, w, part, S),
                                                                        flush, cold=cold)
        res["splits"] = S
        res["read84MB_cold_us"] = timed(lambda: w.view(torch.int32).sum(), flush)
        if 128 < M <= 256 and S:
            from pyspark_tf_gke_amd import _native
            from pyspark_tf_gke_amd.ops._util import ptr, stream_handle

            lib = _native.hip_lib()
            for mode, nm in ((3, "dma_only"), (5, "tiledB"), (7, "tiledB_dma_only"), (8, "m32tile_tiledB_dma"),
                             (9, "m32tile_dma")):
                for ss in (16,):
                    pp = torch.empty(ss, M, N, device=dev)
                    fn = lambda: lib.ptg_dense_fwd_sk_dbg(ptr(x), ptr(w), ptr(pp), M, N, Kd, ss, mode, stream_handle())
                    res[f"dbg_{nm}_s{ss}_cold_us"] = timed(fn, flush)

        tiles = -(-M // 128) * -(-N // 128)
        so = max(1, min(32, 512 // max(tiles, 1), Kd // 640))
        res["fwd_atomic_cold_us"] = timed(lambda: K.gemm(M, N, Kd, x, Kd, 1, w, Kd, 1, 3, acc, N, None, 0, so), flush)
        res["fwd_blaslt_cold_us"] = timed(lambda: torch.mm(x, w.t(), out_dtype=torch.float32), flush)
        res["dx_gemm_cold_us"] = timed(lambda: K.gemm(M, Kd, N, dy, N, 1, w, Kd, 0, 0, dx, Kd), flush)
        res["dx_blaslt_cold_us"] = timed(lambda: torch.matmul(dy, w, out=dx), flush)
        if hasattr(K, "dense_dx"):
            K.dense_dx(dy, w, dx)
            refx = dy.float() @ w.float()
            res["dx_dense_maxrel"] = float(((dx.float() - refx).abs().max() / refx.abs().max()).item())
            res["dx_dense_cold_us"] = timed(lambda: K.dense_dx(dy, w, dx), flush)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
