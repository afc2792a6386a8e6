"""Where the chunked KMeans assignment (ml.hip kmeans_chunk_k, D > 576) differs from the host path:
prints the rows with the largest min-distance difference and their fp64 reference distances.
Usage: python tools/kmeans_debug.py [n k D]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pyspark_tf_gke_amd.ops import df as D  # noqa: E402


def main():
    n, k, Dm = (int(a) for a in sys.argv[1:4]) if len(sys.argv) >= 4 else (4000, 25, 2048)
    g = torch.Generator().manual_seed(k)
    X = torch.randn(n, Dm, generator=g)
    X[:, : Dm // 3] = (X[:, : Dm // 3] > 1.0).float()
    C = X[torch.randperm(n, generator=g)[:k]].clone() + 0.01 * torch.randn(k, Dm, generator=g)
    out = {}
    for dev in ("cuda", "cpu"):
        Xd, Cd = X.to(dev), C.to(dev)
        a = torch.empty(n, dtype=torch.int32, device=dev)
        md = torch.empty(n, dtype=torch.float32, device=dev)
        s = torch.zeros(k, Dm, dtype=torch.float32, device=dev)
        c = torch.zeros(k, dtype=torch.float32, device=dev)
        cost = torch.zeros(1, dtype=torch.float64, device=dev)
        D.kmeans_assign_accum(Xd, Cd, assign=a, sums=s, counts=c, cost=cost, mind=md)
        out[dev] = [t.cpu() for t in (a, md, s, c, cost)]
    ag, mg = out["cuda"][0], out["cuda"][1]
    ah, mh = out["cpu"][0], out["cpu"][1]
    d = ((X.double()[:, None, :] - C.double()[None]) ** 2).sum(2)
    diff = (mg - mh).abs()
    print(f"n={n} k={k} D={Dm}: max |mind diff| {diff.max():.4g}, rows > 0.1: {int((diff > 0.1).sum())}, "
          f"assign agree {(ag == ah).float().mean():.5f}")
    for r in torch.argsort(diff, descending=True)[:8].tolist():
        print(f"  row {r} (tile {r // 64}, in-tile {r % 64}): gpu {mg[r]:.4f} a={int(ag[r])} cpu {mh[r]:.4f} a={int(ah[r])} "
              f"fp64 gpu-center {d[r, int(ag[r])]:.4f} cpu-center {d[r, int(ah[r])]:.4f}")
    for name, i in (("sums", 2), ("counts", 3), ("cost", 4)):
        a_, b_ = out["cuda"][i].double(), out["cpu"][i].double()
        print(f"  {name}: max abs diff {(a_ - b_).abs().max():.4g} (scale {b_.abs().max():.4g})")


if __name__ == "__main__":
    main()
