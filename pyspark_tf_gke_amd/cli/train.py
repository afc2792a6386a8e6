"""Training CLI with the flag/env surface of the reference's ``train_tf_ps.py`` (:822-840):

  --data-path/DATA_PATH  --data-url/DATA_URL  --data-is-images  --img-height/IMG_HEIGHT=256
  --img-width/IMG_WIDTH=320  --output-dir/OUTPUT_DIR=./tf-model  --epochs/EPOCHS=1
  --batch-size/BATCH_SIZE=32  --use-ps  --worker-replicas/WORKER_REPLICAS=2
  --ps-replicas/PS_REPLICAS=1  --port/TF_GRPC_PORT=2222  --worker-addrs/WORKER_ADDRS
  --ps-addrs/PS_ADDRS  --chief-addr/CHIEF_ADDR  --chief-port/CHIEF_PORT=2223

Additions: ``--strategy {auto,ps,mirrored,none}``, ``--synthetic N`` (generate a laser-spot-shaped
image set), ``--flat/--gap`` (CNN head; the reference's __main__ hard-codes flat=True, :883),
``--interactive`` (the reference's blocking ``input()`` at :857 becomes opt-in), ``--plot``
(the reference's blocking ``plt.show()`` at :806-808 becomes a saved PNG), ``--checkpoint-every``.

Behaviour per mode (same artifacts as the reference: label_map.json, model.keras, history.json):
  * CSV (MLP): local path = seeded 80/20 split + fit(validation_data) with Adam(1e-3)
    (:651-672); PS path = ClusterCoordinator schedule/join loop with Adam(1e-4) (:587-650).
  * images (CNN): local path = fit on the training subset with validation (:773-808); PS path as
    above with MSE/MAE/MSE metrics (:707-772).
Every rank of a multi-GPU launch runs this script (SPMD); rank 0 writes artifacts and prints.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from typing import List, Optional

import numpy as np


def parse_args(argv: List[str]):
    env = os.environ.get
    p = argparse.ArgumentParser(description="Train the MLP (CSV) or CNN (images) on MI355X, optionally with "
                                            "ParameterServerStrategy / MultiWorkerMirroredStrategy")
    p.add_argument("--data-path", default=env("DATA_PATH", "/app/infra/local/mysql-database/datasets/image-datasets/laser-spots"))
    p.add_argument("--data-url", default=env("DATA_URL", ""))
    p.add_argument("--data-is-images", action="store_true")
    p.add_argument("--img-height", type=int, default=int(env("IMG_HEIGHT", "256")))
    p.add_argument("--img-width", type=int, default=int(env("IMG_WIDTH", "320")))
    p.add_argument("--output-dir", default=env("OUTPUT_DIR", "./tf-model"))
    p.add_argument("--epochs", type=int, default=int(env("EPOCHS", "1")))
    p.add_argument("--batch-size", type=int, default=int(env("BATCH_SIZE", "32")))
    p.add_argument("--use-ps", action="store_true")
    p.add_argument("--worker-replicas", type=int, default=int(env("WORKER_REPLICAS", "2")))
    p.add_argument("--ps-replicas", type=int, default=int(env("PS_REPLICAS", "1")))
    p.add_argument("--port", type=int, default=int(env("TF_GRPC_PORT", "2222")))
    p.add_argument("--worker-addrs", default=env("WORKER_ADDRS", ""))
    p.add_argument("--ps-addrs", default=env("PS_ADDRS", ""))
    p.add_argument("--chief-addr", default=env("CHIEF_ADDR", ""))
    p.add_argument("--chief-port", type=int, default=int(env("CHIEF_PORT", "2223")))
    # additions
    p.add_argument("--strategy", default=env("PTG_STRATEGY", "auto"), choices=["auto", "ps", "mirrored", "none"])
    p.add_argument("--ps-mode", default=env("PTG_PS_MODE", "sync"), choices=["sync", "async"],
                   help="ParameterServerStrategy update mode: 'async' is TF's (workers push gradients that the "
                        "owning ranks apply as they arrive, train_tf_ps.py:505-510); 'sync' commits one "
                        "update per coordinator round")
    p.add_argument("--cache-decoded", action="store_true",
                   help="keep decoded images in host RAM after the first epoch (Dataset.cache)")
    p.add_argument("--synthetic", type=int, default=int(env("PTG_SYNTHETIC", "0")),
                   help="generate N synthetic laser-spot images into --data-path first")
    head = p.add_mutually_exclusive_group()
    head.add_argument("--flat", dest="flat", action="store_true", default=True)
    head.add_argument("--gap", dest="flat", action="store_false")
    p.add_argument("--interactive", action="store_true")
    p.add_argument("--plot", action="store_true")
    p.add_argument("--checkpoint-every", type=int, default=0, help="save a resumable checkpoint every N epochs")
    p.add_argument("--resume", action="store_true")
    p.add_argument("--seed", type=int, default=1337)
    return p.parse_args(argv)


def _is_chief() -> bool:
    from ..parallel import comm

    return comm.rank() == 0


def make_parameter_server_strategy(worker_replicas: int, ps_replicas: int, port: int = 2222, worker_addrs=None,
                                   ps_addrs=None, chief_addr=None, chief_port: int = 2223, mode: str | None = None):
    """Same contract as train_tf_ps.py:440-511: print the ClusterSpec, validate the chief IPv4, export
    TF_CONFIG (task=chief), build the resolver/partitioner/strategy."""
    from .. import distribute as ds

    cluster = ds.build_cluster_def(worker_replicas, ps_replicas, port, worker_addrs, ps_addrs, chief_addr, chief_port)
    if _is_chief():
        print("Computed ClusterSpec:", json.dumps(cluster), flush=True)
    if chief_addr:
        ds.validate_chief_addr(chief_addr)
        os.environ["TF_CONFIG"] = ds.make_tf_config(cluster, "chief", 0)
        if _is_chief():
            print("TF_CONFIG set:", os.environ["TF_CONFIG"], flush=True)
    resolver = ds.SimpleClusterResolver(ds.ClusterSpec(cluster), rpc_layer="grpc")
    part = ds.MinSizePartitioner(min_shard_bytes=256 << 10, max_shards=max(ps_replicas, 1))
    return ds.ParameterServerStrategy(cluster_resolver=resolver, variable_partitioner=part, mode=mode)


def _strategy_for(args, use_ps: bool):
    from .. import distribute as ds

    mode = args.strategy
    if mode == "auto":
        mode = "ps" if use_ps else ("mirrored" if int(os.environ.get("WORLD_SIZE", "1")) > 1 else "none")
    if mode == "ps":
        wa = [s.strip() for s in args.worker_addrs.split(",") if s.strip()] or None
        pa = [s.strip() for s in args.ps_addrs.split(",") if s.strip()] or None
        return "ps", make_parameter_server_strategy(args.worker_replicas, args.ps_replicas, args.port, wa, pa,
                                                    args.chief_addr or None, args.chief_port,
                                                    mode=getattr(args, "ps_mode", None))
    if mode == "mirrored":
        return "mirrored", ds.MultiWorkerMirroredStrategy()
    return "none", None


def _save_artifacts(model, history: dict, output_dir: str) -> None:
    if not _is_chief():
        return
    path = os.path.join(output_dir, "model.keras")
    model.save(path)
    print(f"Model saved to: {path}", flush=True)
    with open(os.path.join(output_dir, "history.json"), "w") as fh:
        json.dump({k: [float(x) for x in v] for k, v in history.items()}, fh)


def _ps_loop(model, strategy, per_worker_fn, steps_per_epoch, epochs, loss_obj, optimizer, metrics, fmt):
    """The reference's coordinator loop: schedule steps_per_epoch closures, join() per epoch."""
    from .. import distribute as ds
    from ..nn import GradientTape, add_n

    coordinator = ds.ClusterCoordinator(strategy)
    it = iter(coordinator.create_per_worker_dataset(per_worker_fn))

    def step_fn(inputs):
        features, labels = inputs
        with GradientTape() as tape:
            preds = model(features, training=True)
            loss = loss_obj(labels, preds)
            # Add possible regularization losses (train_tf_ps.py:624)
            loss += add_n(model.losses) if model.losses else 0.0
        grads = tape.gradient(loss, model.trainable_variables)
        optimizer.apply_gradients(zip(grads, model.trainable_variables))
        for m in metrics[1:]:
            m.update_state(labels, preds)
        metrics[0].update_state(loss)
        return loss

    def per_worker_train_step(iterator):
        return strategy.run(step_fn, args=(next(iterator),))

    history = {}
    for epoch in range(epochs):
        if _is_chief():
            print(f"Starting epoch {epoch + 1}/{epochs}...", flush=True)
        for m in metrics:
            m.reset_state()
        for _ in range(steps_per_epoch):
            coordinator.schedule(per_worker_train_step, args=(it,))
        coordinator.join()
        vals = [float(m.result()) for m in metrics]
        if _is_chief():
            print(fmt(epoch, vals), flush=True)
        for m, v in zip(metrics, vals):
            history.setdefault(m.name, []).append(v)
    return history


def run_deep_training(data_source: str, output_dir: str, epochs: int, batch_size: int, use_parameter_server: bool,
                      worker_replicas: int, ps_replicas: int, args=None, seed: int = 1337) -> dict:
    from .. import nn
    from ..data import Dataset
    from ..data.loaders import load_csv
    from ..models import build_deep_model

    os.makedirs(output_dir, exist_ok=True)
    if _is_chief():
        print(f"Loading dataset from: {data_source}", flush=True)
    X, y, vocab = load_csv(data_source)
    num_classes, input_dim = int(y.max()) + 1, X.shape[1]
    if _is_chief():
        with open(os.path.join(output_dir, "label_map.json"), "w", encoding="utf-8") as fh:
            json.dump({int(i): s for i, s in enumerate(vocab)}, fh, ensure_ascii=False, indent=2)
    steps_per_epoch = max(1, len(X) // batch_size)
    mode, strategy = _strategy_for(args, use_parameter_server and worker_replicas > 0)
    if mode == "ps":
        if _is_chief():
            print("Using ParameterServerStrategy with workers and ps.", flush=True)

        def per_worker_dataset_fn(ctx=None):
            ds = Dataset.from_tensor_slices((X, y))
            if ctx is not None:
                ds = ds.shard(ctx.num_input_pipelines, ctx.input_pipeline_id)
            return ds.shuffle(min(3000, len(X)), seed=seed).batch(batch_size).repeat()

        with strategy.scope():
            model = build_deep_model(input_dim, num_classes)
            optimizer = nn.optimizers.Adam(learning_rate=1e-4)
            loss_obj = nn.losses.SparseCategoricalCrossentropy()
            metrics = [nn.metrics.Mean("loss"), nn.metrics.SparseCategoricalAccuracy("accuracy")]
        hist = _ps_loop(model, strategy, per_worker_dataset_fn, steps_per_epoch, epochs, loss_obj, optimizer, metrics,
                        lambda e, v: f"Epoch {e + 1} - loss: {v[0]:.4f} - accuracy: {v[1]:.4f}")
        history = {"accuracy": hist["accuracy"][-1:]}
    else:
        if _is_chief():
            print("Running single-process (no distributed strategy)." if mode == "none"
                  else "Running MultiWorkerMirroredStrategy (RCCL all-reduce).", flush=True)
        idx = np.arange(len(X))
        np.random.default_rng(seed).shuffle(idx)
        val = max(1, int(len(X) * 0.2))
        tr, va = idx[:-val], idx[-val:]
        ctx = strategy.scope() if strategy is not None else _null()
        with ctx:
            model = build_deep_model(input_dim, num_classes)
        ds_train = Dataset.from_tensor_slices((X[tr], y[tr]))
        if strategy is not None and strategy.world_size > 1:
            ds_train = ds_train.shard(strategy.world_size, strategy.rank)
        ds_train = ds_train.shuffle(min(3000, len(tr)), seed=seed).batch(batch_size).repeat().prefetch(1)
        ds_val = Dataset.from_tensor_slices((X[va], y[va])).batch(batch_size).prefetch(1)
        h = model.fit(ds_train, epochs=epochs, steps_per_epoch=max(1, len(tr) // batch_size // max(1, getattr(strategy, "world_size", 1))),
                      validation_data=ds_val, verbose=1 if _is_chief() else 0)
        history = h.history
    _save_artifacts(model, history, output_dir)
    return history


class _null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def run_image_training(data_dir: str, output_dir: str, epochs: int, batch_size: int, use_parameter_server: bool,
                       worker_replicas: int, ps_replicas: int, img_height: int, img_width: int, flat_layer: bool = True,
                       args=None, seed: int = 1337, plot: bool = False) -> dict:
    from .. import nn
    from ..data.loaders import count_images, make_image_dataset
    from ..models import build_cnn_model

    os.makedirs(output_dir, exist_ok=True)
    shape = (img_height, img_width, 3)
    total = count_images(data_dir)
    mode, strategy = _strategy_for(args, use_parameter_server and worker_replicas > 0)
    if mode == "ps":
        if _is_chief():
            print("Using ParameterServerStrategy with workers and ps for image training.", flush=True)
        steps_per_epoch = max(1, total // batch_size)

        def per_worker_dataset_fn(ctx=None):
            return make_image_dataset(data_dir, (img_height, img_width), batch_size, shuffle=True, input_context=ctx,
                                      seed=seed)

        with strategy.scope():
            model = build_cnn_model(shape, num_outputs=2, flat=flat_layer, summary=True,
                                    print_fn=print if _is_chief() else (lambda *a: None))
            optimizer = nn.optimizers.Adam(learning_rate=1e-4)
            loss_obj = nn.losses.MeanSquaredError()
            metrics = [nn.metrics.Mean("loss"), nn.metrics.MeanAbsoluteError("mae"), nn.metrics.MeanSquaredError("mse")]
        hist = _ps_loop(model, strategy, per_worker_dataset_fn, steps_per_epoch, epochs, loss_obj, optimizer, metrics,
                        lambda e, v: f"Epoch {e + 1} - loss: {v[0]:.4f} - mae: {v[1]:.4f} - mse: {v[2]:.4f}")
        history = {"mae": hist["mae"][-1:], "mse": hist["mse"][-1:], "loss": hist["loss"][-1:]}
    else:
        if _is_chief():
            print("Running single-process image training." if mode == "none"
                  else "Running MultiWorkerMirroredStrategy image training.", flush=True)
        val_split = 0.2
        train_count = max(1, total - int(total * val_split))
        world = getattr(strategy, "world_size", 1) if strategy is not None else 1
        steps_per_epoch = max(1, train_count // batch_size // world)
        ictx = strategy.input_context() if strategy is not None and world > 1 else None
        cache = bool(getattr(args, "cache_decoded", False))
        ds_train = make_image_dataset(data_dir, (img_height, img_width), batch_size, shuffle=True, input_context=ictx,
                                      validation_split=val_split, subset="training", seed=seed, repeat=True,
                                      cache=cache)
        ds_val = make_image_dataset(data_dir, (img_height, img_width), batch_size, shuffle=False,
                                    validation_split=val_split, subset="validation", seed=seed, repeat=False,
                                    cache=cache)
        ctx = strategy.scope() if strategy is not None else _null()
        with ctx:
            model = build_cnn_model(shape, num_outputs=2, flat=flat_layer, summary=True,
                                    print_fn=print if _is_chief() else (lambda *a: None))
        cbs = []
        if args is not None and args.checkpoint_every:
            from ..utils.checkpoint import CheckpointCallback

            cbs.append(CheckpointCallback(os.path.join(output_dir, "ckpt"), every=args.checkpoint_every,
                                          resume=args.resume))
        h = model.fit(ds_train, epochs=epochs, steps_per_epoch=steps_per_epoch, validation_data=ds_val,
                      verbose=1 if _is_chief() else 0, callbacks=cbs)
        history = h.history
        if plot and _is_chief():
            _plot_mae(history, os.path.join(output_dir, "mae.png"))
    _save_artifacts(model, history, output_dir)
    return history


def _plot_mae(history: dict, path: str) -> None:
    try:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt

        for k in ("mae", "val_mae"):
            if history.get(k):
                plt.plot(range(1, len(history[k]) + 1), history[k], label=k)
        plt.xlabel("epoch")
        plt.ylabel("MAE (px)")
        plt.yscale("log")
        plt.legend()
        plt.savefig(path)
        plt.close()
    except ImportError:
        _plot_curves_pil({k: history[k] for k in ("mae", "val_mae") if history.get(k)}, path)
    except Exception as e:  # noqa: BLE001
        print(f"plot skipped: {e}")


def _plot_curves_pil(curves: dict, path: str, size=(640, 400)) -> None:
    """Line plot of per-epoch curves with PIL only (matplotlib is not in the image): log-scale y,
    axes with min / max labels, one colour per curve and a legend."""
    from PIL import Image, ImageDraw

    import math

    W, H = size
    L, R, T, B = 60, 20, 20, 40
    img = Image.new("RGB", size, "white")
    d = ImageDraw.Draw(img)
    vals = [v for c in curves.values() for v in c if v > 0]
    if not vals:
        return
    lo, hi = math.log10(min(vals)), math.log10(max(vals))
    hi = hi if hi > lo else lo + 1.0
    n = max(len(c) for c in curves.values())
    d.rectangle([L, T, W - R, H - B], outline="black")
    for frac, v in ((0.0, lo), (1.0, hi)):
        y = H - B - frac * (H - T - B)
        d.text((4, y - 6), f"{10 ** v:.3g}", fill="black")
    d.text((L, H - B + 6), "1", fill="black")
    d.text((W - R - 30, H - B + 6), str(n), fill="black")
    d.text(((W - L) // 2, H - B + 20), "epoch", fill="black")
    colours = ["#1f77b4", "#d62728", "#2ca02c", "#9467bd"]
    for k, (name, c) in enumerate(curves.items()):
        pts = [(L + (i / max(n - 1, 1)) * (W - L - R), H - B - (math.log10(max(v, 1e-12)) - lo) / (hi - lo) * (H - T - B))
               for i, v in enumerate(c)]
        if len(pts) > 1:
            d.line(pts, fill=colours[k % len(colours)], width=2)
        d.text((W - R - 120, T + 6 + 14 * k), name, fill=colours[k % len(colours)])
    img.save(path)


def main(argv: Optional[List[str]] = None) -> int:
    args = parse_args(sys.argv[1:] if argv is None else argv)
    if args.interactive:
        input("Press enter to continue...")
    from ..utils.logging import configure

    configure()
    data_source = args.data_path
    if args.synthetic:
        from ..data.loaders import write_synthetic_image_dataset
        from ..parallel import comm

        if comm.rank() == 0 and not os.path.exists(os.path.join(data_source, "clean_labels.jsonl")):
            write_synthetic_image_dataset(data_source, n=args.synthetic, size=(args.img_height, args.img_width))
        comm.init()
        comm.barrier()
    is_images = bool(args.data_is_images) or os.path.isdir(data_source)
    t0 = time.time()
    if is_images:
        run_image_training(data_source, args.output_dir, args.epochs, args.batch_size, args.use_ps,
                           args.worker_replicas, args.ps_replicas, args.img_height, args.img_width,
                           flat_layer=args.flat, args=args, seed=args.seed, plot=args.plot)
    else:
        run_deep_training(data_source, args.output_dir, args.epochs, args.batch_size, args.use_ps,
                          args.worker_replicas, args.ps_replicas, args=args, seed=args.seed)
    if _is_chief():
        print(f"done in {time.time() - t0:.1f}s", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
