"""Checkpoint / resume.  The reference only saves the final ``model.keras``; here a
checkpoint holds the flat fp32 parameters, the optimizer state (Adam moments / SGD velocity) and
step, the BatchNormalization moving statistics, the epoch, and the RNG
state, written atomically with safetensors + a JSON manifest.  Parameters/moments are identical
on every rank for mirrored training (rank 0 writes), while the sharded parameter-server strategy
writes one shard file per rank (its slice of the optimizer state) plus the gathered parameters.
"""
from __future__ import annotations

import json
import os
import time

import torch

from ..parallel import comm


def save_checkpoint(model, path: str, epoch: int, extra: dict | None = None) -> str:
    from safetensors.torch import save_file

    os.makedirs(path, exist_ok=True)
    opt = model.optimizer
    st = model.store
    rank = comm.rank()
    tensors = {}
    sharded = hasattr(model.strategy, "shard_range") if getattr(model, "strategy", None) is not None else False
    if rank == 0 or sharded:
        if sharded and comm.world_size() > 1:
            lo, hi = model.strategy.shard_range(model)
        else:
            lo, hi = 0, st.total
        if opt is not None:
            for k, t in opt.state_tensors().items():
                if t is not None:
                    tensors["opt_" + k] = t[lo:hi].detach().cpu().contiguous()
        if rank == 0:
            tensors["params"] = st.flat.detach().cpu().contiguous()
            for l in model.layers:  # non-trainable BatchNormalization state
                if getattr(l, "moving_mean", None) is not None:
                    tensors[f"bn/{l.name}/moving_mean"] = l.moving_mean.detach().cpu().contiguous()
                    tensors[f"bn/{l.name}/moving_variance"] = l.moving_variance.detach().cpu().contiguous()
        tmp = os.path.join(path, f"shard-{rank:05d}.safetensors.tmp")
        save_file(tensors, tmp, metadata={"lo": str(lo), "hi": str(hi)})
        os.replace(tmp, os.path.join(path, f"shard-{rank:05d}.safetensors"))
    comm.barrier()
    if rank == 0:
        manifest = {"epoch": epoch, "step": opt.iterations if opt else 0, "world_size": comm.world_size(),
                    "sharded": sharded, "time": time.time(), "torch_rng": torch.get_rng_state().tolist()[:16],
                    **(extra or {})}
        with open(os.path.join(path, "manifest.json.tmp"), "w") as fh:
            json.dump(manifest, fh)
        os.replace(os.path.join(path, "manifest.json.tmp"), os.path.join(path, "manifest.json"))
    comm.barrier()
    return path


def load_checkpoint(model, path: str) -> dict:
    from safetensors import safe_open

    with open(os.path.join(path, "manifest.json")) as fh:
        manifest = json.load(fh)
    st = model.store
    opt = model.optimizer
    if opt is not None:
        opt.build(st)
    state = opt.state_tensors() if opt is not None else {}
    with safe_open(os.path.join(path, "shard-00000.safetensors"), "pt") as f:
        keys = set(f.keys())
        st.flat.copy_(f.get_tensor("params").to(st.flat.device))
        if not manifest["sharded"]:
            for k, t in state.items():
                if t is not None and "opt_" + k in keys:
                    t.copy_(f.get_tensor("opt_" + k).to(t.device))
        for l in model.layers:
            if getattr(l, "moving_mean", None) is not None and f"bn/{l.name}/moving_mean" in keys:
                l.moving_mean.copy_(f.get_tensor(f"bn/{l.name}/moving_mean").to(l.moving_mean.device))
                l.moving_variance.copy_(f.get_tensor(f"bn/{l.name}/moving_variance").to(l.moving_variance.device))
    if manifest["sharded"] and opt is not None:
        for r in range(manifest["world_size"]):
            fn = os.path.join(path, f"shard-{r:05d}.safetensors")
            with safe_open(fn, "pt") as f:
                md = f.metadata()
                lo, hi = int(md["lo"]), int(md["hi"])
                for k, t in state.items():
                    if t is not None and "opt_" + k in f.keys():
                        t[lo:hi].copy_(f.get_tensor("opt_" + k).to(t.device))
    if opt is not None:
        opt.iterations = int(manifest["step"])
    st.refresh_bf16()
    return manifest


class CheckpointCallback:
    """Keras-style callback: save every ``every`` epochs; with ``resume=True`` restore the latest
    checkpoint at train begin (the fit loop then skips completed epochs via ``initial_epoch``)."""

    def __init__(self, path: str, every: int = 1, resume: bool = False):
        self.path, self.every, self.resume = path, max(1, every), resume
        self.model = None
        self.start_epoch = 0

    def set_model(self, model):
        self.model = model

    def on_train_begin(self, logs=None):
        if self.resume and os.path.exists(os.path.join(self.path, "manifest.json")):
            m = load_checkpoint(self.model, self.path)
            self.start_epoch = int(m["epoch"]) + 1

    def on_epoch_end(self, epoch, logs=None):
        if (epoch + 1) % self.every == 0:
            save_checkpoint(self.model, self.path, epoch, {"logs": logs or {}})
