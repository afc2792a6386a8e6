"""Where the CSV-MLP step time goes at the reference's batch sizes: per-step wall time of
(a) Model.train_step_fast (the bench / fit path), (b) the cached native launch alone (MlpStep.run),
(c) the same launches with steps=8 per launch (kernel time per step, launch cost amortised).
python tools/mlp_overhead.py [--batch 32]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pyspark_tf_gke_amd.models import build_deep_model  # noqa: E402
from pyspark_tf_gke_amd.ops import nn as K  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--iters", type=int, default=500)
a = ap.parse_args()
B = a.batch
dev = torch.device("cuda")
m = build_deep_model(3, 15, device=dev)
g = torch.Generator().manual_seed(0)
x = torch.randn(8 * B, 3, generator=g).to(dev)
y = torch.randint(0, 15, (8 * B,), generator=g).to(torch.int32).to(dev)
st = m._stats_buf()


def timeit(fn, iters):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


xb, yb = x[:B], y[:B]
us_step = timeit(lambda: m.train_step_fast(xb, yb, st), a.iters)
ms = next(iter(m._mlp_steps.values()))
it = [m.optimizer.iterations]


def run(xx, yy, k):
    ms.run(xx, yy, k, it[0])
    it[0] += k


us_run = timeit(lambda: run(xb, yb, 1), a.iters)
us_run8 = timeit(lambda: run(x, y, 8), a.iters // 4) / 8
print(json.dumps({"batch": B, "train_step_fast_us": round(us_step, 2), "cached_launch_us": round(us_run, 2),
                  "kernel_us_per_step_8_per_launch": round(us_run8, 2)}), flush=True)
