"""Checkpoint / resume.  The reference only saves the final ``model.keras``; here a
checkpoint holds the fp32 parameters (per parameter name), the optimizer state (Adam moments / SGD velocity) and
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


def _ps_sharded(model) -> bool:
    st = getattr(model, "strategy", None)
    return st is not None and hasattr(st, "shard_range") and comm.world_size() > 1


def save_checkpoint(model, path: str, epoch: int, extra: dict | None = None) -> str:
    """Collective (every rank calls it).  Parameters and mirrored optimizer state are stored per
    parameter name (``param/<name>``, ``opt_<slot>/<name>``), so a checkpoint loads into any
    flat-buffer layout (1 GPU, or N GPUs with the sharded data-parallel update's re-laid-out store).
    The parameter-server strategy keeps its per-rank flat optimizer shards (``opt_<slot>`` + lo/hi)."""
    from safetensors.torch import save_file

    os.makedirs(path, exist_ok=True)
    opt = model.optimizer
    st = model.store
    strat = getattr(model, "strategy", None)
    if strat is not None and hasattr(strat, "synchronize_state"):
        strat.synchronize_state(model)  # sharded update: full fp32 master + optimizer moments
    rank = comm.rank()
    tensors = {}
    sharded = _ps_sharded(model)
    if rank == 0 or sharded:
        lo, hi = model.strategy.shard_range(model) if sharded else (0, st.total)
        if opt is not None:
            for k, t in opt.state_tensors().items():
                if t is None:
                    continue
                if sharded:
                    tensors["opt_" + k] = t[lo:hi].detach().cpu().contiguous()
                elif rank == 0:
                    for p in st.params:
                        tensors[f"opt_{k}/{p.name}"] = t[p.offset:p.offset + p.numel].detach().cpu().contiguous()
        if rank == 0:
            for p in st.params:
                tensors["param/" + p.name] = p.data.detach().reshape(-1).cpu().contiguous()
            for l in model.layers:  # non-trainable BatchNormalization state
                if getattr(l, "moving_mean", None) is not None:
                    tensors[f"bn/{l.name}/moving_mean"] = l.moving_mean.detach().cpu().contiguous()
                    tensors[f"bn/{l.name}/moving_variance"] = l.moving_variance.detach().cpu().contiguous()
            tensors["rng/cpu"] = torch.get_rng_state().contiguous()
            if torch.cuda.is_available() and st.flat.device.type == "cuda":
                tensors["rng/cuda"] = torch.cuda.get_rng_state(st.flat.device).contiguous()
        tmp = os.path.join(path, f"shard-{rank:05d}.safetensors.tmp")
        save_file(tensors, tmp, metadata={"lo": str(lo), "hi": str(hi)})
        os.replace(tmp, os.path.join(path, f"shard-{rank:05d}.safetensors"))
    comm.barrier()
    if rank == 0:
        manifest = {"epoch": epoch, "step": opt.iterations if opt else 0, "world_size": comm.world_size(),
                    "sharded": sharded, "layout": "ps-flat" if sharded else "per-param",
                    "total": int(st.total), "time": time.time(),
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
    strat = getattr(model, "strategy", None)
    st = model.store
    if manifest["sharded"] and (int(manifest.get("total", -1)) != int(st.total)
                                or int(manifest["world_size"]) != comm.world_size()
                                or not _ps_sharded(model)):
        # flat [lo:hi] optimizer slices only mean something in the layout that wrote them
        raise ValueError(f"checkpoint {path}: parameter-server optimizer shards were written for "
                         f"world {manifest['world_size']} / flat size {manifest.get('total')}; this model "
                         f"has world {comm.world_size()} / flat size {st.total} (load it with the same layout)")
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
            if not manifest["sharded"]:
                for k, t in state.items():
                    if t is not None and f"opt_{k}/{p.name}" in keys:
                        t[p.offset:p.offset + p.numel].copy_(f.get_tensor(f"opt_{k}/{p.name}").to(t.device))
        for l in model.layers:
            if getattr(l, "moving_mean", None) is not None and f"bn/{l.name}/moving_mean" in keys:
                l.moving_mean.copy_(f.get_tensor(f"bn/{l.name}/moving_mean").to(l.moving_mean.device))
                l.moving_variance.copy_(f.get_tensor(f"bn/{l.name}/moving_variance").to(l.moving_variance.device))
        if "rng/cpu" in keys:
            torch.set_rng_state(f.get_tensor("rng/cpu"))
        if "rng/cuda" in keys and st.flat.device.type == "cuda":
            torch.cuda.set_rng_state(f.get_tensor("rng/cuda"), st.flat.device)
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
