"""The reference's training loop (ParameterServerStrategy + ClusterCoordinator scheduling the
GradientTape closure, train_tf_ps.py:612-645 / :734-765) on N ranks, sync vs async PS mode.

Launch N ranks on one node (on the 1-GPU box they share cuda:0 over a gloo control group; HIP IPC
maps the async windows exactly as over xGMI):

    PTG_DIST_BACKEND=gloo python -m pyspark_tf_gke_amd.runtime.launcher --nproc 2 -- \\
        python tools/ps_modes_bench.py --batch 64 --steps 40

Per mode: the job's samples/s over the timed epoch (every closure is one worker step of --batch
samples), the mean closure time on each worker, and how many closures each worker ran.  Rank 0
prints one JSON line per mode."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--steps", type=int, default=40, help="closures per epoch (whole job)")
ap.add_argument("--epochs", type=int, default=2, help="the first epoch is warm-up")
ap.add_argument("--modes", default="sync,async")
ap.add_argument("--shape", default="256,320")
a = ap.parse_args()
H, W = (int(x) for x in a.shape.split(","))

from pyspark_tf_gke_amd import distribute as ds  # noqa: E402
from pyspark_tf_gke_amd import nn  # noqa: E402
from pyspark_tf_gke_amd.distribute.ps import ParameterServerStrategy  # noqa: E402
from pyspark_tf_gke_amd.models import build_cnn_model  # noqa: E402
from pyspark_tf_gke_amd.parallel import comm  # noqa: E402


def run(mode):
    strategy = ParameterServerStrategy(mode=mode)
    dev = strategy.device
    g = torch.Generator().manual_seed(strategy.rank)
    xs = [torch.randint(0, 256, (a.batch, H, W, 3), generator=g, dtype=torch.uint8).to(dev) for _ in range(2)]
    ys = [(torch.rand((a.batch, 2), generator=g) * 200).to(dev) for _ in range(2)]
    with strategy.scope():
        torch.manual_seed(1)
        model = build_cnn_model((H, W, 3), flat=True, summary=False, device=dev)
        optimizer = nn.optimizers.Adam(learning_rate=1e-4)
        loss_obj = nn.losses.MeanSquaredError()
    coordinator = ds.ClusterCoordinator(strategy)

    def per_worker_fn(ctx=None):
        def gen():
            i = 0
            while True:
                yield xs[i % 2], ys[i % 2]
                i += 1
        return gen()

    it = iter(coordinator.create_per_worker_dataset(per_worker_fn))
    busy = [0.0]

    def step_fn(inputs):
        t0 = time.perf_counter()
        features, labels = inputs
        with nn.GradientTape() as tape:
            preds = model(features, training=True)
            loss = loss_obj(labels, preds)
        grads = tape.gradient(loss, model.trainable_variables)
        optimizer.apply_gradients(zip(grads, model.trainable_variables))
        busy[0] += time.perf_counter() - t0
        return loss

    def per_worker_train_step(iterator):
        return strategy.run(step_fn, args=(next(iterator),))

    res = None
    for epoch in range(a.epochs):
        busy[0] = 0.0
        ran0 = coordinator.closures_run
        if dev.type == "cuda":
            torch.cuda.synchronize()
        comm.barrier()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            coordinator.schedule(per_worker_train_step, args=(it,))
        coordinator.join()
        if dev.type == "cuda":
            torch.cuda.synchronize()
        dt = comm.all_reduce_max_scalar(time.perf_counter() - t0)
        ran = comm.all_gather_int(coordinator.closures_run - ran0)
        busy_ms = [x * 1e3 for x in comm.all_reduce_float(
            [busy[0] if r == strategy.rank else 0.0 for r in range(strategy.world_size)])]
        res = {"mode": mode, "ranks": strategy.world_size, "batch": a.batch, "closures": a.steps,
               "job_samples_per_s": round(a.steps * a.batch / dt, 1), "epoch_s": round(dt, 4),
               "job_ms_per_closure": round(dt / a.steps * 1e3, 4), "closures_per_worker": ran,
               "worker_ms_per_closure": [round(b / max(n, 1), 3) for b, n in zip(busy_ms, ran)]}
    if mode == "async":
        strategy.shutdown()
    return res


for mode in a.modes.split(","):
    r = run(mode)
    if comm.rank() == 0:
        print(json.dumps(r), flush=True)
