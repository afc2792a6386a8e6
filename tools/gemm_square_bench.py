#!/usr/bin/env python
"""Square bf16 GEMM C[M][N] = A[M][K] B[N][K]^T (bf16 out) on uniform random [-1, 1) operands:
the 256x256 LDS-DMA kernel, the 128x128 register-staged kernel, and hipBLASLt (torch.matmul) —
TFLOP/s of each, max error vs an fp32 reference on a sampled block.

    python tools/gemm_square_bench.py [--sizes 4096,8192] [--iters 20]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyspark_tf_gke_amd import _native  # noqa: E402
from pyspark_tf_gke_amd.ops import nn as K  # noqa: E402


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
    return a.elapsed_time(b) / iters  # ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="4096,8192")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    lib = _native.hip_lib()
    out = []
    for S in [int(x) for x in a.sizes.split(",")]:
        A = (torch.rand(S, S, device="cuda") * 2 - 1).bfloat16()
        B = (torch.rand(S, S, device="cuda") * 2 - 1).bfloat16()
        C = torch.empty(S, S, device="cuda", dtype=torch.bfloat16)
        flops = 2.0 * S ** 3
        row = {"M=N=K": S}
        for name, on in (("ptg_256x256_ldsdma", 1), ("ptg_128x128_regstage", 0)):
            lib.ptg_gemm256_set(on)
            ms = timeit(lambda: K.gemm(S, S, S, A, S, True, B, S, True, 0, C, S), a.iters)
            row[name + "_tflops"] = round(flops / ms / 1e9, 1)
            ref = A[:256].float() @ B[:512].float().t()
            row[name + "_maxerr"] = round(float((C[:256, :512].float() - ref).abs().max()), 4)
        lib.ptg_gemm256_set(1)
        ms = timeit(lambda: torch.matmul(A, B.t()), a.iters)
        row["hipblaslt_tflops"] = round(flops / ms / 1e9, 1)
        out.append(row)
        print(json.dumps(row), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
