"""Host-side (Python) cost of the training step: cProfile over K train_step_fast calls of the bench
model, with no device sync inside the loop, so the per-call host time shows where the launch path
spends it.  When the host enqueues slower than the GPU executes (small batches), these are the
step's idle gaps on the GPU timeline.
    python tools/host_profile.py [--workload cnn_b1] [--batch 32] [--steps 200] [--top 30]"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402
from pyspark_tf_gke_amd.distribute import MultiWorkerMirroredStrategy  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="cnn_b1")
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--steps", type=int, default=200)
ap.add_argument("--top", type=int, default=30)
a = ap.parse_args()
st = MultiWorkerMirroredStrategy()
with st.scope():
    model, _, xs, ys = bench._build(a.workload, a.batch, st.device, 1234, 0, 1)
stats = model._stats_buf()
for i in range(20):
    model.train_step_fast(xs[i % 2], ys[i % 2], stats)
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(a.steps):
    model.train_step_fast(xs[i % 2], ys[i % 2], stats)
t_host = time.perf_counter() - t0
torch.cuda.synchronize()
t_all = time.perf_counter() - t0
print(f"host enqueue {t_host / a.steps * 1e6:.1f} us/step, wall {t_all / a.steps * 1e6:.1f} us/step")
pr = cProfile.Profile()
pr.enable()
for i in range(a.steps):
    model.train_step_fast(xs[i % 2], ys[i % 2], stats)
pr.disable()
torch.cuda.synchronize()
s = io.StringIO()
ps = pstats.Stats(pr, stream=s).sort_stats("tottime")
ps.print_stats(a.top)
print(s.getvalue())
s = io.StringIO()
ps = pstats.Stats(pr, stream=s).sort_stats("cumulative")
ps.print_stats(a.top)
print(s.getvalue())
