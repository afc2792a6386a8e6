"""Trainer for the BASELINE.json model families that are not in the reference repo (SURVEY.md §0,
finding 6): ``--model resnet50`` (keras.applications ResNet-50, "MultiWorkerMirroredStrategy ->
RCCL all-reduce on 8xMI355X") and ``--model mnist`` (the MNIST-shaped CNN, "bf16 training on 1
MI355X").  No datasets can be downloaded here, so both train on synthetic data of the real shape:
ResNet-50 on uniform-noise 224x224x3 images with random labels (a throughput workload), MNIST on
procedurally drawn class-dependent 28x28 strokes (learnable, so the loss curve is meaningful).

Every rank runs this script (SPMD, one rank per GPU); with WORLD_SIZE > 1 the model is built under
MultiWorkerMirroredStrategy and each rank draws its own shard of the synthetic stream.  Artifacts
(rank 0): ``model.keras``, ``history.json``, ``train_report.json`` (samples/s per epoch).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch


def synthetic_mnist(n: int, seed: int, device):
    """Class c = a stroke at a class-specific angle/offset + noise (28x28x1 in [0,1])."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    y = torch.randint(0, 10, (n,), generator=g)
    yy, xx = torch.meshgrid(torch.arange(28.0), torch.arange(28.0), indexing="ij")
    ang = (y.float() * (3.14159 / 10)).view(n, 1, 1)
    off = ((y % 3).float() - 1.0).view(n, 1, 1) * 4.0
    d = (xx - 14) * torch.sin(ang) - (yy - 14) * torch.cos(ang) - off
    img = torch.exp(-(d ** 2) / 4.0) + 0.15 * torch.rand(n, 28, 28, generator=g)
    return img.clamp(0, 1).unsqueeze(-1).to(device), y.to(torch.int32).to(device)


def parse_args(argv):
    env = os.environ.get
    p = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    p.add_argument("--model", choices=["resnet50", "mnist"], default="resnet50")
    p.add_argument("--epochs", type=int, default=int(env("EPOCHS", "1")))
    p.add_argument("--steps-per-epoch", type=int, default=int(env("STEPS_PER_EPOCH", "20")))
    p.add_argument("--batch-size", type=int, default=int(env("BATCH_SIZE", "0")), help="per-worker batch")
    p.add_argument("--output-dir", default=env("OUTPUT_DIR", "./tf-model"))
    p.add_argument("--optimizer", choices=["sgd", "adam"], default=None)
    p.add_argument("--lr", type=float, default=None)
    p.add_argument("--seed", type=int, default=1337)
    return p.parse_args(argv)


def main(argv=None) -> int:
    args = parse_args(sys.argv[1:] if argv is None else argv)
    from .. import nn
    from ..data import Dataset
    from ..distribute import MultiWorkerMirroredStrategy
    from ..models import build_mnist_cnn
    from ..models.resnet import ResNet50
    from ..parallel import comm
    from ..utils.logging import configure

    configure()
    strategy = MultiWorkerMirroredStrategy()
    dev, rank, world = strategy.device, strategy.rank, strategy.world_size
    bs = args.batch_size or (128 if args.model == "resnet50" else 256)
    steps = args.steps_per_epoch
    with strategy.scope():
        if args.model == "resnet50":
            model = ResNet50()
            opt = (nn.optimizers.Adam(args.lr or 1e-3) if args.optimizer == "adam"
                   else nn.optimizers.SGD(args.lr or 0.1, momentum=0.9))
            model.compile(optimizer=opt, loss=nn.losses.SparseCategoricalCrossentropy(), metrics=["accuracy"])
        else:
            model = build_mnist_cnn(compile=False)
            opt = (nn.optimizers.SGD(args.lr or 0.05, momentum=0.9) if args.optimizer == "sgd"
                   else nn.optimizers.Adam(args.lr or 1e-3))
            model.compile(optimizer=opt, loss="sparse_categorical_crossentropy", metrics=["accuracy"])
    if args.model == "resnet50":
        g = torch.Generator(device=dev).manual_seed(args.seed + rank)
        n = bs * 2
        x = torch.rand((n, 224, 224, 3), generator=g, device=dev)
        y = torch.randint(0, 1000, (n,), generator=g, device=dev).to(torch.int32)
    else:
        x, y = synthetic_mnist(bs * steps, args.seed + rank, dev)
    ds = Dataset.from_tensor_slices((x, y)).shuffle(len(x), seed=args.seed + rank).batch(bs, drop_remainder=True).repeat()
    t0 = time.perf_counter()
    per_epoch = []

    class _Timer:
        def on_epoch_end(self, epoch, logs=None):
            if dev.type == "cuda":
                torch.cuda.synchronize()
            per_epoch.append(time.perf_counter())

    hist = model.fit(ds, epochs=args.epochs, steps_per_epoch=steps, verbose=1 if rank == 0 else 0, callbacks=[_Timer()])
    times = [b - a for a, b in zip([t0] + per_epoch[:-1], per_epoch)]
    rates = [round(bs * world * steps / t, 1) for t in times]
    report = {"model": args.model, "workers": world, "per_worker_batch": bs, "steps_per_epoch": steps,
              "samples_per_s_by_epoch": rates, "history": hist.history,
              "data": "synthetic (" + ("uniform images, random labels" if args.model == "resnet50"
                                        else "procedural class-dependent strokes") + ")"}
    if rank == 0:
        os.makedirs(args.output_dir, exist_ok=True)
        model.save(os.path.join(args.output_dir, "model.keras"))
        model.export(os.path.join(args.output_dir, "saved_model"))
        with open(os.path.join(args.output_dir, "history.json"), "w") as fh:
            json.dump(hist.history, fh)
        with open(os.path.join(args.output_dir, "train_report.json"), "w") as fh:
            json.dump(report, fh, indent=2)
        print(json.dumps({k: report[k] for k in ("model", "workers", "samples_per_s_by_epoch")}), flush=True)
    comm.barrier()
    return 0


if __name__ == "__main__":
    sys.exit(main())
