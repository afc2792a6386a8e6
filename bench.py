#!/usr/bin/env python
"""Headline benchmark (driver contract): ``python bench.py --gpus N --steps K --warmup W``.

Default workload = the reference's CNN-B1 regressor (train_tf_ps.py:346-378 with flat=True, the
model ``__main__`` trains, :883): 256x320x3 input, 5 x [Conv5x5 + PReLU (+ MaxPool)], Dense(2048,
relu), Dense(2); MSE + MAE/MSE metrics; Adam.  Synthetic data of that shape (random uint8 images,
random pixel targets), random-init weights, bf16 compute / fp32 master weights.  N>1 ranks run
MultiWorkerMirroredStrategy (gradient buckets reduce-scattered over RCCL during backward, sharded
Adam, bf16 all-gather overlapped with the next forward) with a fixed per-GPU batch (weak scaling).
Every timed step is a full train step: input pack (decoded uint8 images resident in HBM ->
normalised, channel-padded bf16), forward, loss, backward, gradient reduce-scatter / all-gather,
Adam update.

``--gpus N`` without a torch.distributed launcher (no ``WORLD_SIZE`` in the environment) spawns N
fresh rank processes through :func:`pyspark_tf_gke_amd.runtime.launcher.launch` before anything
touches the GPU; under ``torch.distributed.run`` the ranks come from the environment.  Either way
the job asserts ``world_size == --gpus``.

``--workload groupby`` measures the Spark DataFrame groupBy-aggregate over 1B synthetic rows per
GPU instead (rows/s).  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="cnn_b1", choices=["cnn_b1", "groupby", "sort", "mlp", "cnn_a1", "mnist", "resnet50"])
    ap.add_argument("--batch-size", type=int, default=int(os.environ.get("PTG_BENCH_BATCH", "0")),
                    help="per-GPU batch (weak scaling); 0 = the workload default")
    ap.add_argument("--rows", type=int, default=1_000_000_000, help="groupby: rows per GPU")
    ap.add_argument("--keys", type=int, default=1_000_000, help="groupby: distinct keys")
    ap.add_argument("--graph", type=int, default=int(os.environ.get("PTG_BENCH_GRAPH", "0")),
                    help="capture the train step in a HIP graph")
    ap.add_argument("--groupby-extra", type=int, default=int(os.environ.get("PTG_BENCH_GROUPBY", "1")),
                    help="after the CNN timing, also time the Spark groupBy half of the BASELINE metric and "
                         "report it under extra.groupby (1B rows per GPU)")
    ap.add_argument("--extra-batches", default=os.environ.get("PTG_BENCH_EXTRA_BATCHES", "32,64"),
                    help="cnn_b1: also time these per-GPU batches (the reference's 32 and 64) into extra")
    ap.add_argument("--mlp-batches", default=os.environ.get("PTG_BENCH_MLP_BATCHES", "32,64"),
                    help="cnn_b1: also time the reference's CSV-MLP step (train_tf_ps.py build_deep_model) at these "
                         "batches into extra.mlp_b<B> (the fused one-launch step)")
    ap.add_argument("--sim-world", type=int, default=int(os.environ.get("PTG_BENCH_SIM_WORLD", "8")),
                    help="cnn_b1 on 1 GPU: also time rank 0's kernel sequence of an N-rank sharded data-parallel "
                         "step (PTG_SIM_WORLD: collectives replaced by local kernels of the same HBM bytes) into "
                         "extra.sim_world<N>; 0 = off")
    ap.add_argument("--seed", type=int, default=1234)
    return ap.parse_args(argv)


DEFAULT_BATCH = {"cnn_b1": 256, "cnn_a1": 256, "resnet50": 128, "mnist": 512, "mlp": 4096}


def _sync():
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def _build(workload, B, dev, seed, rank, world):
    """Model + two synthetic global batches; this rank keeps its [rank*B, (rank+1)*B) slice, so a
    1-rank run at batch B*world sees exactly the union of what the N ranks see."""
    from pyspark_tf_gke_amd.models import build_cnn_a1, build_cnn_model, build_deep_model, build_mnist_cnn
    from pyspark_tf_gke_amd.models.resnet import build_resnet50

    torch.manual_seed(seed)  # identical initial weights on every rank and every world size
    G = B * world
    g = torch.Generator(device="cpu")
    g.manual_seed(seed)
    sl = slice(rank * B, (rank + 1) * B)

    def img(h, w, c):
        return [torch.randint(0, 256, (G, h, w, c), generator=g, dtype=torch.uint8)[sl].to(dev) for _ in range(2)]

    if workload == "cnn_b1":
        model = build_cnn_model((256, 320, 3), flat=True, summary=False)
        meta = ("samples/sec TF CNN train", "CNN-B1 (train_tf_ps.py build_cnn_model flat=True, 256x320x3, 43.37M params)",
                "256x320x3")
        xs = img(256, 320, 3)
        ys = [(torch.rand((G, 2), generator=g) * torch.tensor([320.0, 256.0]))[sl].to(dev) for _ in range(2)]
    elif workload == "cnn_a1":
        model = build_cnn_a1((256, 320, 3))
        meta = ("samples/sec TF CNN train", "CNN-A1 (3-conv 32/64/128 + GAP, 4.86M params)", "256x320x3")
        xs = img(256, 320, 3)
        ys = [(torch.rand((G, 2), generator=g) * 256)[sl].to(dev) for _ in range(2)]
    elif workload == "resnet50":
        model = build_resnet50()
        meta = ("samples/sec TF ResNet-50 train",
                "ResNet-50 (keras.applications v1, 224x224x3, 1000 classes, 25.6M params)", "224x224x3")
        xs = img(224, 224, 3)
        ys = [torch.randint(0, 1000, (G,), generator=g)[sl].to(torch.int32).to(dev) for _ in range(2)]
    elif workload == "mnist":
        model = build_mnist_cnn()
        meta = ("samples/sec TF CNN train", "MNIST CNN (28x28x1, conv32/conv64/dense128)", "28x28x1")
        xs = [torch.rand((G, 28, 28, 1), generator=g)[sl].to(dev) for _ in range(2)]
        ys = [torch.randint(0, 10, (G,), generator=g)[sl].to(torch.int32).to(dev) for _ in range(2)]
    else:  # mlp: the reference's CSV MLP (train_tf_ps.py:328-343), 3 features -> 15 classes
        model = build_deep_model(3, 15)
        meta = ("samples/sec TF MLP train", "CSV-MLP (train_tf_ps.py build_deep_model 3->16->32->64->15, 3,695 params)",
                "3 features")
        xs = [torch.randn((G, 3), generator=g)[sl].to(dev) for _ in range(2)]
        ys = [torch.randint(0, 15, (G,), generator=g)[sl].to(torch.int32).to(dev) for _ in range(2)]
    return model, meta, xs, ys


def _input_note(workload: str) -> str:
    if workload == "mlp":
        return "fp32 features resident in HBM"
    if workload == "mnist":
        return "fp32 28x28x1 images in [0, 1) resident in HBM"
    if workload == "cnn_b1":
        return ("in the timed step: uint8 NHWC images resident in HBM, read by the first conv's forward and "
                "weight-gradient kernels themselves (/255 + channel pad in registers, no packed copy)")
    return "in the timed step: uint8 NHWC images resident in HBM -> /255, channel-padded bf16 (pack_u8rgb4_k)"


def _time_steps(model, xs, ys, steps, warmup):
    from pyspark_tf_gke_amd.ops import nn as K
    from pyspark_tf_gke_amd.parallel import comm

    import contextlib

    stats = model._stats_buf()
    # PTG_STEP_PRIORITY=-1 (A/B): the step's own kernels on a high-priority stream, so the command
    # processor hands freed CUs to them ahead of the side stream's weight-gradient kernels
    prio = int(os.environ.get("PTG_STEP_PRIORITY", "0") or 0)
    scope = (torch.cuda.stream(torch.cuda.Stream(priority=prio)) if prio and torch.cuda.is_available()
             else contextlib.nullcontext())
    with scope:
        for i in range(warmup):
            model.train_step_fast(xs[i % 2], ys[i % 2], stats)
        _sync()
        comm.barrier()
        _sync()
        K.fill_(stats, 0.0)
        t0 = time.perf_counter()
        for i in range(steps):
            model.train_step_fast(xs[i % 2], ys[i % 2], stats)
    _sync()
    comm.barrier()
    _sync()
    dt = comm.all_reduce_max_scalar(time.perf_counter() - t0)
    return dt, model._logs_from(stats)


def _comm_probe(model, strategy, reps=5):
    """The collectives of one training step (every gradient bucket's reduce-scatter and every
    parameter bucket's all-gather, the exact sizes and dtypes of the step), timed alone: an upper
    bound on the step's exposed communication (in the real step they overlap backward/forward)."""
    from pyspark_tf_gke_amd.parallel import comm

    plan = getattr(model, "_shard_plan", None)
    if plan is None or strategy.world_size == 1:
        return None
    st = model.store
    outs = {b.idx: torch.empty(b.shi - b.slo, dtype=torch.float32, device=st.flat.device) for b in plan.buckets}
    strategy.wait_parameters(model)

    def once():
        for b in plan.buckets:
            comm.reduce_scatter_flat(outs[b.idx], st.flat_grad[b.lo:b.hi])
        for b in plan.buckets:
            buf = st.flat if b.fp32 else st.flat_bf16
            comm.all_gather_flat(buf[b.lo:b.hi], buf[b.slo:b.shi].clone())

    once()
    _sync()
    comm.barrier()
    t0 = time.perf_counter()
    for _ in range(reps):
        once()
    _sync()
    dt = comm.all_reduce_max_scalar(time.perf_counter() - t0) / reps
    nbytes = sum((b.hi - b.lo) * 4 + (b.hi - b.lo) * (4 if b.fp32 else 2) for b in plan.buckets)
    return {"comm_ms_isolated": round(dt * 1e3, 4), "buckets": len(plan.buckets),
            "bytes_per_step": int(nbytes), "note": "reduce-scatter + all-gather of one step run alone"}


def bench_train(args, strategy, rank, world):
    dev = strategy.device
    B = args.batch_size or DEFAULT_BATCH[args.workload]
    with strategy.scope():
        model, (name, cfg_model, shape), xs, ys = _build(args.workload, B, dev, args.seed, rank, world)
    if args.graph:
        model.jit_compile = True
    dt, logs = _time_steps(model, xs, ys, args.steps, args.warmup)
    ms = dt / args.steps * 1e3
    opt = {"resnet50": "SGD(0.1, momentum 0.9)"}.get(args.workload, "Adam(1e-3)") + " fused flat"
    res = {"metric": name, "value": round(B * world * args.steps / dt, 2), "unit": "samples/s",
           "ms_per_step": round(ms, 4),
           "config": {"model": cfg_model, "global_batch": B * world, "per_gpu_batch": B, "input": shape,
                      "parallelism": f"dp{world}" + (" (MultiWorkerMirroredStrategy, RCCL reduce-scatter/all-gather)"
                                                     if world > 1 else ""),
                      "optimizer": opt, "final_loss": round(logs["loss"], 6),
                      "input_pipeline": _input_note(args.workload)}}
    probe = _comm_probe(model, strategy)
    if probe is not None:
        res["comm"] = probe
    del model, xs, ys
    return res


def bench_mlp_fit(B: int, steps_per_epoch: int = 2048, epochs: int = 3) -> dict:
    """The reference's CSV-MLP ``model.fit`` loop (train_tf_ps.py:651-672) at batch B over a column
    dataset: fit() keeps the columns in HBM and runs groups of 64 consecutive batches per launch of
    the fused step (mlp.hip).  Every batch is a full forward/backward/Adam step; the time covers
    whole epochs (including each epoch's metric readback), divided by the number of steps."""
    import numpy as np

    from pyspark_tf_gke_amd.data.dataset import Dataset
    from pyspark_tf_gke_amd.models import build_deep_model

    rng = np.random.default_rng(7)
    X = rng.normal(size=(B * steps_per_epoch, 3)).astype(np.float32)
    y = rng.integers(0, 15, B * steps_per_epoch).astype(np.int32)
    ds = Dataset.from_tensor_slices((X, y)).batch(B)
    model = build_deep_model(3, 15)
    model.fit(ds, epochs=1, verbose=0)  # columns to HBM, plan + launch descriptors built
    _sync()
    t0 = time.perf_counter()
    model.fit(ds, epochs=epochs, verbose=0)
    _sync()
    dt = time.perf_counter() - t0
    n = steps_per_epoch * epochs
    return {"value": round(B * n / dt, 2), "unit": "samples/s", "ms_per_step": round(dt / n * 1e3, 5),
            "per_gpu_batch": B, "steps": n, "grouped": model._mlp_fit_plan(ds, None, None) is not None,
            "model": "CSV-MLP 3->16->32->64->15 via model.fit over a Dataset (grouped fused steps)"}


def bench_groupby(args, strategy, rank, world):
    from pyspark_tf_gke_amd.sql import bench_groupby as bg

    return bg.run(rows_per_gpu=args.rows, num_keys=args.keys, steps=args.steps, warmup=args.warmup,
                  device=strategy.device)


def _self_launch(args) -> int | None:
    """``--gpus N`` with no launcher around us: run N fresh ranks and return their exit code."""
    if "WORLD_SIZE" in os.environ or args.gpus <= 1:
        return None
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from pyspark_tf_gke_amd.runtime.launcher import launch

    cmd = [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    return launch(cmd, args.gpus, master_addr="127.0.0.1", prefix_output=False)


def main():
    args = parse()
    rc = _self_launch(args)
    if rc is not None:
        return rc
    from pyspark_tf_gke_amd.distribute import MultiWorkerMirroredStrategy
    from pyspark_tf_gke_amd.parallel import comm

    strategy = MultiWorkerMirroredStrategy()
    rank, world = strategy.rank, strategy.world_size
    if world != args.gpus:
        raise RuntimeError(f"--gpus {args.gpus} but the job has {world} ranks (WORLD_SIZE="
                           f"{os.environ.get('WORLD_SIZE')})")
    extra = {}
    if args.workload == "groupby":
        res = bench_groupby(args, strategy, rank, world)
        dtype, data = "fp64", "synthetic (bigint keys = hash(row) % keys, double values), resident in HBM"
    elif args.workload == "sort":
        from pyspark_tf_gke_amd.sql import bench_groupby as bg

        res = bg.run_sort(rows_per_gpu=args.rows, steps=args.steps, warmup=args.warmup, device=strategy.device)
        dtype, data = "int64 keys / fp64 values", "synthetic (random full-range bigint keys, double values), resident in HBM"
    else:
        res = bench_train(args, strategy, rank, world)
        dtype = "bf16" if strategy.device.type == "cuda" else "fp32 (host reference path, no GPU)"
        data = ("synthetic (random features / labels of the reference shape; random-init weights)"
                if args.workload == "mlp" else
                "synthetic (random uint8 images / targets of the reference shape; random-init weights)")
        if args.workload == "cnn_b1" and args.extra_batches:
            for b in [int(x) for x in args.extra_batches.split(",") if x.strip()]:
                a2 = argparse.Namespace(**{**vars(args), "batch_size": b})
                r2 = bench_train(a2, strategy, rank, world)
                extra[f"batch{b}"] = {"value": r2["value"], "unit": "samples/s", "ms_per_step": r2["ms_per_step"],
                                      "per_gpu_batch": b, "global_batch": b * world}
        if args.workload == "cnn_b1" and args.mlp_batches and world == 1:
            for b in [int(x) for x in args.mlp_batches.split(",") if x.strip()]:
                a2 = argparse.Namespace(**{**vars(args), "batch_size": b, "workload": "mlp", "steps": 200,
                                           "warmup": 20})
                r2 = bench_train(a2, strategy, rank, world)
                extra[f"mlp_b{b}"] = {"value": r2["value"], "unit": "samples/s", "ms_per_step": r2["ms_per_step"],
                                      "per_gpu_batch": b, "global_batch": b * world,
                                      "model": "CSV-MLP 3->16->32->64->15 (train_tf_ps.py:328-343), Adam, fp32"}
            if torch.cuda.is_available():
                for b in [int(x) for x in args.mlp_batches.split(",") if x.strip()]:
                    extra[f"mlp_fit_b{b}"] = bench_mlp_fit(b)
        if args.workload == "cnn_b1" and args.sim_world > 1 and world == 1 and torch.cuda.is_available():
            # the N>1 compute path on one GPU: dW into flat_grad, per-bucket reduce-scatter stand-in,
            # shard Adam, all-gather stand-in + bf16 re-cast (MultiWorkerMirroredStrategy sim mode)
            from pyspark_tf_gke_amd import config as _cfg

            _cfg.set_cli("sim_world", args.sim_world)
            try:
                sst = MultiWorkerMirroredStrategy()
                a2 = argparse.Namespace(**vars(args))
                r2 = bench_train(a2, sst, rank, world)
                extra[f"sim_world{args.sim_world}"] = {
                    "ms_per_step": r2["ms_per_step"], "value": r2["value"], "unit": "samples/s",
                    "per_gpu_batch": r2["config"]["per_gpu_batch"],
                    "vs_n1_step": round(r2["ms_per_step"] / res["ms_per_step"], 4),
                    "note": "rank 0's kernels of a dp%d sharded step on 1 GPU, collectives replaced by local "
                            "kernels moving the same local bytes (no xGMI time)" % args.sim_world}
            finally:
                _cfg._cli.pop("sim_world", None)
        if args.workload == "cnn_b1" and args.groupby_extra and torch.cuda.is_available():
            # second half of BASELINE.json's metric ("rows/sec Spark groupBy + samples/sec TF CNN
            # train"); timed separately, after the CNN steps, so it cannot perturb them.  With N > 1
            # ranks the shuffle's collectives run here for the first time in the job: a watchdog
            # prints the headline line without the groupBy extra and ends the process if they hang
            # (PTG_BENCH_EXTRA_TIMEOUT seconds), so a stuck extra can never take the CNN number down.
            watchdog = None
            if world > 1:
                import threading

                done = threading.Event()

                def _expire(limit=float(os.environ.get("PTG_BENCH_EXTRA_TIMEOUT", "240"))):
                    if done.wait(limit):
                        return
                    extra["groupby"] = {"error": f"multi-rank groupBy extra did not finish in {limit:.0f} s"}
                    if rank == 0:
                        print(json.dumps(_bench_line(res, extra, world, args, dtype, data)), flush=True)
                    os._exit(0)

                watchdog = threading.Thread(target=_expire, daemon=True)
                watchdog.start()
            try:
                import gc

                gc.collect()
                torch.cuda.empty_cache()
                gb = bench_groupby(argparse.Namespace(rows=args.rows, keys=args.keys, steps=3, warmup=1), strategy,
                                   rank, world)
                extra["groupby"] = {"metric": gb["metric"], "value": gb["value"], "unit": gb["unit"],
                                    "ms_per_step": gb["ms_per_step"], "rows_per_gpu": gb["config"]["rows_per_gpu"],
                                    "distinct_keys": gb["config"]["distinct_keys"], "keys": gb["config"]["keys"],
                                    "counts_check": gb["config"]["counts_check"],
                                    "sums_check": gb["config"]["sums_check"],
                                    "groups_check": gb["config"]["groups_check"], "dtype": "fp64"}
                from pyspark_tf_gke_amd.sql import bench_groupby as bg

                gc.collect()
                torch.cuda.empty_cache()
                gs = bg.run(rows_per_gpu=args.rows, num_keys=args.keys, steps=3, warmup=1, device=strategy.device,
                            sparse=True)
                extra["groupby_sparse"] = {"value": gs["value"], "unit": gs["unit"], "ms_per_step": gs["ms_per_step"],
                                           "distinct_keys": gs["config"]["distinct_keys"], "keys": gs["config"]["keys"],
                                           "groups_out": gs["config"]["groups_out"],
                                           "counts_check": gs["config"]["counts_check"],
                                           "sums_check": gs["config"]["sums_check"],
                                           "groups_check": gs["config"]["groups_check"], "dtype": "fp64"}
            except Exception as e:  # noqa: BLE001 - never lose the headline line
                extra["groupby"] = {"error": repr(e)[:300]}
            if watchdog is not None:
                done.set()
    out = _bench_line(res, extra, world, args, dtype, data)
    if rank == 0:
        print(json.dumps(out), flush=True)
    comm.destroy()
    return 0


def _bench_line(res, extra, world, args, dtype, data) -> dict:
    out = {"metric": res["metric"], "value": res["value"], "unit": res["unit"], "n_gpus": world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": res["ms_per_step"],
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": dtype, "data": data,
           "config": res["config"]}
    if "comm" in res:
        out["comm"] = res["comm"]
    if extra:
        out["extra"] = dict(extra)
    return out


if __name__ == "__main__":
    sys.exit(main())
