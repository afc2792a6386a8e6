"""CNN-B1 training step on one GPU through the reference's primary call stack vs fit()'s step:

  ps   ParameterServerStrategy (1 worker, 1 PS task) + ClusterCoordinator.schedule of the
       GradientTape closure (train_tf_ps.py:612-645 / cli/train.py _ps_loop), join() per epoch
  fit  Model.train_step_fast (the fused Sequential step fit() runs)

Same model, batch, synthetic uint8 images resident on the device.  Prints one JSON line per path:
python tools/ps_vs_fit.py [--batch 256] [--steps 20] [--epochs 2]."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--steps", type=int, default=20, help="closures per epoch")
ap.add_argument("--epochs", type=int, default=2, help="the first epoch is warm-up")
ap.add_argument("--shape", default="256,320")
ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
a = ap.parse_args()
H, W = (int(x) for x in a.shape.split(","))
dev = torch.device(a.device)

from pyspark_tf_gke_amd import distribute as ds  # noqa: E402
from pyspark_tf_gke_amd import nn  # noqa: E402
from pyspark_tf_gke_amd.cli.train import make_parameter_server_strategy  # noqa: E402
from pyspark_tf_gke_amd.models import build_cnn_model  # noqa: E402

g = torch.Generator().manual_seed(0)
xs = [torch.randint(0, 256, (a.batch, H, W, 3), generator=g, dtype=torch.uint8).to(dev) for _ in range(2)]
ys = [(torch.rand((a.batch, 2), generator=g) * 200).to(dev) for _ in range(2)]


def sync():
    if dev.type == "cuda":
        torch.cuda.synchronize()


# ---- fit()'s fused step
torch.manual_seed(1)
m = build_cnn_model((H, W, 3), flat=True, summary=False, device=dev)
st = m._stats_buf()
for i in range(3):
    m.train_step_fast(xs[i % 2], ys[i % 2], st)
sync()
t0 = time.perf_counter()
for i in range(a.steps):
    m.train_step_fast(xs[i % 2], ys[i % 2], st)
sync()
fit_ms = (time.perf_counter() - t0) / a.steps * 1e3
print(json.dumps({"path": "fit (train_step_fast)", "ms_per_step": round(fit_ms, 4),
                  "samples_per_s": round(a.batch / fit_ms * 1e3, 1), "batch": a.batch}), flush=True)
del m

# ---- the same GradientTape step without a strategy / coordinator: splits the PS path's overhead
# into the tape step itself (separate loss, unfused optimizer launch) and the PS dispatch
torch.manual_seed(1)
mt_ = build_cnn_model((H, W, 3), flat=True, summary=False, device=dev)
opt_ = nn.optimizers.Adam(learning_rate=1e-4)
lo_ = nn.losses.MeanSquaredError()


def tape_step(xb, yb):
    with nn.GradientTape() as tape:
        p = mt_(xb, training=True)
        lv = lo_(yb, p)
    gr = tape.gradient(lv, mt_.trainable_variables)
    opt_.apply_gradients(zip(gr, mt_.trainable_variables))


for i in range(3):
    tape_step(xs[i % 2], ys[i % 2])
sync()
t0 = time.perf_counter()
for i in range(a.steps):
    tape_step(xs[i % 2], ys[i % 2])
sync()
tape_ms = (time.perf_counter() - t0) / a.steps * 1e3
print(json.dumps({"path": "GradientTape loop, no strategy", "ms_per_step": round(tape_ms, 4),
                  "samples_per_s": round(a.batch / tape_ms * 1e3, 1), "batch": a.batch,
                  "vs_fit": round(tape_ms / fit_ms, 3)}), flush=True)
del mt_, opt_

# ---- ParameterServerStrategy + ClusterCoordinator (the reference's loop)
strategy = make_parameter_server_strategy(1, 1)
with strategy.scope():
    torch.manual_seed(1)
    model = build_cnn_model((H, W, 3), flat=True, summary=False, device=dev)
    optimizer = nn.optimizers.Adam(learning_rate=1e-4)
    loss_obj = nn.losses.MeanSquaredError()
    metrics = [nn.metrics.Mean("loss"), nn.metrics.MeanAbsoluteError("mae")]
coordinator = ds.ClusterCoordinator(strategy)


def per_worker_fn(ctx=None):
    def gen():
        i = 0
        while True:
            yield xs[i % 2], ys[i % 2]
            i += 1
    return gen()


it = iter(coordinator.create_per_worker_dataset(per_worker_fn))


def step_fn(inputs):
    features, labels = inputs
    with nn.GradientTape() as tape:
        preds = model(features, training=True)
        loss = loss_obj(labels, preds)
    grads = tape.gradient(loss, model.trainable_variables)
    optimizer.apply_gradients(zip(grads, model.trainable_variables))
    for mt in metrics[1:]:
        mt.update_state(labels, preds)
    metrics[0].update_state(loss)
    return loss


def per_worker_train_step(iterator):
    return strategy.run(step_fn, args=(next(iterator),))


times = []
for epoch in range(a.epochs):
    for mt in metrics:
        mt.reset_state()
    sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        coordinator.schedule(per_worker_train_step, args=(it,))
    coordinator.join()
    vals = [float(mt.result()) for mt in metrics]
    sync()
    times.append((time.perf_counter() - t0) / a.steps * 1e3)
ps_ms = times[-1]
print(json.dumps({"path": "ParameterServerStrategy + ClusterCoordinator (GradientTape closure)",
                  "ms_per_step": round(ps_ms, 4), "samples_per_s": round(a.batch / ps_ms * 1e3, 1),
                  "batch": a.batch, "epoch_ms_per_step": [round(t, 3) for t in times], "loss": vals[0],
                  "vs_fit": round(ps_ms / fit_ms, 3)}), flush=True)
