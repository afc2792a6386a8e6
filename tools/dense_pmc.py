"""Driver for PMC passes over the big-Dense kernels (rocprofv3 --pmc ... -- python tools/dense_pmc.py):
dense.hip forward and dX and hipBLASLt's dX at CNN-B1's b256 shape, 10 calls each, every call after a
512 MB read that evicts the weight from the Infinity Cache."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pyspark_tf_gke_amd.ops import nn as K  # noqa: E402


def main():
    dev = "cuda"
    M, N, Kd = int(os.environ.get("DM", 256)), 2048, 20480
    flush = torch.empty(128 << 20, device=dev)
    w = (torch.randn(N, Kd, device=dev) * 0.01).bfloat16()
    x = torch.randn(M, Kd, device=dev).bfloat16()
    dy = torch.randn(M, N, device=dev).bfloat16()
    dx = torch.empty(M, Kd, device=dev, dtype=torch.bfloat16)
    S = K.dense_fwd_splits(M, N, Kd)
    part = torch.empty(S, M, N, device=dev)
    for _ in range(10):
        flush.sum()
        K.dense_fwd_parts(x, w, part, S)
        flush.sum()
        K.dense_dx(dy, w, dx)
        flush.sum()
        torch.matmul(dy, w, out=dx)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
