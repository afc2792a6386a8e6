"""Locate mismatches of the first-layer kernels (conv1.hip) against the fp32 reference: prints, per
(sample, pooled row, pooled column block, channel), where the forward's pooled output differs.
Usage: python tools/conv1_debug.py [N H W]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pyspark_tf_gke_amd.ops import nn as K  # noqa: E402
from pyspark_tf_gke_amd.ops import reference as R  # noqa: E402


def main():
    N, H, W = (int(a) for a in sys.argv[1:4]) if len(sys.argv) >= 4 else (7, 256, 320)
    torch.manual_seed(0)
    x = torch.randint(0, 256, (N, H, W, 3), dtype=torch.uint8)
    w = (torch.randn(8, 5, 5, 4) * 0.2).to(torch.bfloat16)
    w[..., 3] = 0
    b = torch.randn(8) * 0.1
    alpha = torch.rand(H, W, 8) * 0.5
    p = torch.empty(N, H // 2, W // 2, 8, dtype=torch.bfloat16, device="cuda")
    K.conv1_fwd_pm(x.cuda(), w.cuda(), b.cuda(), alpha.cuda(), p)
    torch.cuda.synchronize()
    pr = torch.empty(N, H // 2, W // 2, 8)
    R.conv1_fwd_pm(x, w, b, alpha, pr)
    err = (p.float().cpu() - pr).abs()
    bad = err > 0.05
    print(f"N={N} H={H} W={W} wave={os.environ.get('PTG_CONV1_WAVE', '1')} max err {err.max().item():.4g} "
          f"bad {int(bad.sum())} of {bad.numel()}")
    if bad.any():
        idx = bad.nonzero()
        print("samples with errors:", sorted(set(idx[:, 0].tolist())))
        print("pooled rows (mod 2 = row pair in tile):", sorted(set(idx[:, 1].tolist()))[:40])
        print("pooled cols:", sorted(set(idx[:, 2].tolist()))[:80])
        print("channels:", sorted(set(idx[:, 3].tolist())))
        for r in idx[:10].tolist():
            print("  ", r, float(p[tuple(r)]), float(pr[tuple(r)]))


if __name__ == "__main__":
    main()
