"""Checkpoint / resume.  The reference only saves the final ``model.keras``; here a
checkpoint holds the fp32 parameters (per parameter name), the optimizer state (Adam moments / SGD velocity) and
step, the BatchNormalization moving statistics, the epoch, and every rank's RNG state, written
atomically with safetensors + a JSON manifest.  Parameters/moments are stored once, per parameter
name, in the full layout (rank 0 writes them after the strategy gathered any sharded state); each
rank writes its own RNG file.
"""
from __future__ import annotations

import json
import os
import time

import torch

from ..parallel import comm


def _rng_file(path: str, rank: int) -> str:
    return os.path.join(path, f"rng-{rank:05d}.safetensors")


def save_checkpoint(model, path: str, epoch: int, extra: dict | None = None) -> str:
    """Collective (every rank calls it).  Parameters and optimizer state are stored per parameter
    name (``param/<name>``, ``opt_<slot>/<name>``) by rank 0, so a checkpoint loads into any
    flat-buffer layout (1 GPU, N GPUs with the sharded data-parallel update's re-laid-out store, or
    the parameter-server placement): strategies that shard the state (MWMS sharded update, PS owners)
    first gather it into the full layout (``synchronize_state``).  Every rank writes its own RNG
    state (``rng-<rank>.safetensors``) and restores its own on load, so data-parallel ranks keep
    distinct random streams across a resume."""
    from safetensors.torch import save_file

    os.makedirs(path, exist_ok=True)
    opt = model.optimizer
    st = model.store
    strat = getattr(model, "strategy", None)
    if strat is not None and hasattr(strat, "synchronize_state"):
        strat.synchronize_state(model)  # sharded update / PS owners: full fp32 master + optimizer moments
    rank = comm.rank()
    rng = {"rng/cpu": torch.get_rng_state().contiguous()}
    if torch.cuda.is_available() and st.flat.device.type == "cuda":
        rng["rng/cuda"] = torch.cuda.get_rng_state(st.flat.device).contiguous()
    save_file(rng, _rng_file(path, rank) + ".tmp")
    os.replace(_rng_file(path, rank) + ".tmp", _rng_file(path, rank))
    if rank == 0:
        tensors = {}
        if opt is not None:
            for k, t in opt.state_tensors().items():
                if t is None:
                    continue
                for p in st.params:
                    tensors[f"opt_{k}/{p.name}"] = t[p.offset:p.offset + p.numel].detach().cpu().contiguous()
        for p in st.params:
            tensors["param/" + p.name] = p.data.detach().reshape(-1).cpu().contiguous()
        for l in model.layers:  # non-trainable BatchNormalization state
            if getattr(l, "moving_mean", None) is not None:
                tensors[f"bn/{l.name}/moving_mean"] = l.moving_mean.detach().cpu().contiguous()
                tensors[f"bn/{l.name}/moving_variance"] = l.moving_variance.detach().cpu().contiguous()
        tmp = os.path.join(path, "shard-00000.safetensors.tmp")
        save_file(tensors, tmp)
        os.replace(tmp, os.path.join(path, "shard-00000.safetensors"))
    comm.barrier()
    if rank == 0:
        manifest = {"epoch": epoch, "step": opt.iterations if opt else 0, "world_size": comm.world_size(),
                    "sharded": False, "layout": "per-param", "total": int(st.total), "time": time.time(),
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
    if manifest.get("sharded") or manifest.get("layout", "per-param") != "per-param":
        # round-1/2 parameter-server checkpoints stored flat [lo:hi] optimizer slices per rank; every
        # checkpoint is now written per parameter name
        raise ValueError(f"checkpoint {path}: layout {manifest.get('layout')!r} (flat per-rank optimizer "
                         "shards) is no longer readable; checkpoints are stored per parameter name")
    strat = getattr(model, "strategy", None)
    st = model.store
    if strat is not None and hasattr(strat, "wait_parameters"):
        strat.wait_parameters(model)  # no parameter gather still in flight may land on the loaded values
    opt = model.optimizer
    if opt is not None:
        opt.build(st)
    state = opt.state_tensors() if opt is not None else {}
    with safe_open(os.path.join(path, "shard-00000.safetensors"), "pt") as f:
        keys = set(f.keys())
        for p in st.params:
            key = "param/" + p.name
            if key not in keys:
                raise KeyError(f"checkpoint {path} has no parameter {p.name!r}")
            p.data.copy_(f.get_tensor(key).to(st.flat.device).view(p.shape))
            for k, t in state.items():
                if t is not None and f"opt_{k}/{p.name}" in keys:
                    t[p.offset:p.offset + p.numel].copy_(f.get_tensor(f"opt_{k}/{p.name}").to(t.device))
        for l in model.layers:
            if getattr(l, "moving_mean", None) is not None and f"bn/{l.name}/moving_mean" in keys:
                l.moving_mean.copy_(f.get_tensor(f"bn/{l.name}/moving_mean").to(l.moving_mean.device))
                l.moving_variance.copy_(f.get_tensor(f"bn/{l.name}/moving_variance").to(l.moving_variance.device))
        legacy_rng = {k: f.get_tensor(k) for k in ("rng/cpu", "rng/cuda") if k in keys}
    rank = comm.rank()
    rng = legacy_rng
    if os.path.exists(_rng_file(path, rank)):
        with safe_open(_rng_file(path, rank), "pt") as f:
            rng = {k: f.get_tensor(k) for k in f.keys()}
    if "rng/cpu" in rng:
        torch.set_rng_state(rng["rng/cpu"])
    if "rng/cuda" in rng and st.flat.device.type == "cuda":
        torch.cuda.set_rng_state(rng["rng/cuda"], st.flat.device)
    if opt is not None:
        opt.set_iterations(int(manifest["step"]))
    st.refresh_bf16()
    st.master_stale = False
    if strat is not None and hasattr(strat, "on_state_loaded"):
        strat.on_state_loaded(model)  # parameter server: re-pack the owned shards
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
