"""Optimizers over the flat parameter store.

``Adam`` reproduces ``tf.keras.optimizers.Adam`` (train_tf_ps.py:339,374 with lr 1e-3; the PS
loops use 1e-4, :606,728): m/v moments, epsilon 1e-7, bias correction folded into the step size
lr_t = lr * sqrt(1 - b2^t) / (1 - b1^t).  The whole model is updated by ONE fused kernel launch
(``ptg_adam``) that also refreshes the bf16 compute copy.  ``apply(lo, hi)`` updates a byte range
only: that is how the sharded parameter-server strategy gives each rank its shard of the update.
"""
from __future__ import annotations

import math

import torch

from ..ops import nn as K
from . import streams as S


class Optimizer:
    def __init__(self, learning_rate: float):
        self.learning_rate = float(learning_rate)
        self.iterations = 0
        from ..distribute.strategy import current_strategy

        st = current_strategy()
        if st is not None:
            # created under strategy.scope(): every rank registers its optimizers in the same
            # order, so coordinator rounds can name the optimizer of an update by index
            st.optimizers.append(self)

    def get_config(self) -> dict:
        return {"name": type(self).__name__.lower(), "learning_rate": self.learning_rate}

    def set_iterations(self, n: int) -> None:
        """Set the step counter everywhere it lives: the host count and, after HIP-graph capture,
        the on-device counter the replayed graphs read for Adam's bias correction."""
        self.iterations = int(n)
        ds = getattr(self, "dev_state", None)
        if ds is not None:
            ds[0] = float(self.iterations)

    def apply_gradients(self, grads_and_vars) -> None:
        from .tape import apply_gradients

        apply_gradients(self, grads_and_vars)


class Adam(Optimizer):
    def __init__(self, learning_rate: float = 1e-3, beta_1: float = 0.9, beta_2: float = 0.999,
                 epsilon: float = 1e-7, name: str = "adam"):
        super().__init__(learning_rate)
        self.beta_1, self.beta_2, self.epsilon = beta_1, beta_2, epsilon
        self.name = name
        self.m = None
        self.v = None

    def build(self, store) -> None:
        if self.m is None or self.m.numel() != store.total or self.m.device != store.flat.device:
            self.m = K.zeros(store.total, torch.float32, store.flat.device)
            self.v = K.zeros(store.total, torch.float32, store.flat.device)
            self.dev_state = None

    def use_device_step(self, store) -> None:
        """Keep the step counter / bias-corrected step size on the device (HIP-graph capture)."""
        self.build(store)
        if getattr(self, "dev_state", None) is None:
            self.dev_state = torch.tensor([float(self.iterations), 0.0], dtype=torch.float32, device=store.flat.device)

    def lr_t(self, step: int) -> float:
        b1, b2 = self.beta_1, self.beta_2
        return self.learning_rate * math.sqrt(1.0 - b2 ** step) / (1.0 - b1 ** step)

    def apply(self, store, gscale: float = 1.0, lo: int = 0, hi: int | None = None, advance: bool = True) -> None:
        self.build(store)
        step = self.iterations + 1
        hi = store.total if hi is None else hi
        ds = getattr(self, "dev_state", None)
        if ds is not None and advance:
            K.adam_step(ds, self.learning_rate, self.beta_1, self.beta_2)
        if hi > lo:
            sl = slice(lo, hi)
            K.adam(store.flat[sl], store.flat_grad[sl], self.m[sl], self.v[sl], store.flat_bf16[sl],
                   self.lr_t(step), self.beta_1, self.beta_2, self.epsilon, gscale, lr_dev=ds, clear_grad=True)
        if lo == 0 and hi >= store.total:
            store.grad_clean = True  # the update consumed and zeroed every gradient
        if advance:
            self.iterations = step

    def apply_shard(self, store, grad_shard, lo: int, hi: int, gscale: float = 1.0, advance: bool = True) -> None:
        """Update params[lo:hi] from an already-reduced gradient shard (sharded PS / sharded
        data-parallel update).  ``advance=False`` lets one step update several shards."""
        self.build(store)
        step = self.iterations + 1
        if hi > lo:
            K.adam(store.flat[lo:hi], grad_shard, self.m[lo:hi], self.v[lo:hi], store.flat_bf16[lo:hi],
                   self.lr_t(step), self.beta_1, self.beta_2, self.epsilon, gscale)
        if advance:
            self.iterations = step

    # ---- fused update: the gradient producer applies Adam in its epilogue (one local replica) ----
    def begin_fused(self, store) -> "FusedAdamStep":
        self.build(store)
        ds = getattr(self, "dev_state", None)
        if ds is not None:
            K.adam_step(ds, self.learning_rate, self.beta_1, self.beta_2)
        return FusedAdamStep(self, store, self.iterations + 1, ds)

    def finish_fused(self, ctx: "FusedAdamStep") -> None:
        """Plain fused-flat Adam over every range no gradient producer has updated: one launch for
        all the gaps, which also writes the flipped dgrad filters of the conv kernels in them
        (``ctx.flips``) so the next backward skips its flip pass."""
        st = ctx.store
        lo, gaps = 0, []
        for a, b in sorted(ctx.done) + [(st.total, st.total)]:
            if a > lo:
                gaps.append((lo, a))
            lo = max(lo, b)
        flips = [(nm, f) for nm, f in ctx.flips if any(a <= f[1] and f[1] + f[2] * f[3] * f[3] * f[4] <= b
                                                       for a, b in gaps)]
        if gaps and st.flat.is_cuda and len(gaps) <= 4 and len(flips) <= 4:
            self.build(st)
            K.adam_multi(st.flat, st.flat_grad, self.m, self.v, st.flat_bf16, gaps, self.lr_t(ctx.step), self.beta_1,
                         self.beta_2, self.epsilon, 1.0, lr_dev=getattr(self, "dev_state", None), clear_grad=True,
                         flips=[f for _, f in flips])
            st.flip_token = (id(self), ctx.step) if flips else None
            st.flip_names = frozenset(nm for nm, _ in flips)
        else:
            for a, b in gaps:
                self.apply(st, lo=a, hi=b, advance=False)
            st.flip_token = None
        # the gaps were cleared by their updates; the fused producers' ranges were never written
        ctx.store.grad_clean = True
        self.iterations = ctx.step

    def get_config(self):
        return {"name": self.name, "learning_rate": self.learning_rate, "beta_1": self.beta_1,
                "beta_2": self.beta_2, "epsilon": self.epsilon}

    def state_tensors(self) -> dict:
        return {"m": self.m, "v": self.v}


class FusedAdamStep:
    """One training step's Adam state for gradient producers that update their own parameter
    (``DenseOp`` runs :func:`ops.nn.linear_dw_adam`); ``done`` collects the flat ranges they took."""

    def __init__(self, opt: Adam, store, step: int, lr_dev):
        self.opt, self.store, self.step, self.lr_dev = opt, store, step, lr_dev
        self.done: list = []
        self.flips: list = []  # (op name, ConvOp.flip_spec()) the finishing pass may write

    def linear_dw(self, dz, x, param) -> None:
        o, n = param.offset, param.numel
        st, opt = self.store, self.opt
        shp = param.grad.shape
        lr_t = opt.lr_t(self.step)
        # a weight-gradient producer: overlaps the rest of the backward on the side stream (streams.py)
        fn = lambda: K.linear_dw_adam(dz, x, st.flat[o:o + n].view(shp), opt.m[o:o + n].view(shp),  # noqa: E731
                                      opt.v[o:o + n].view(shp), st.flat_bf16[o:o + n].view(shp), lr_t,
                                      opt.beta_1, opt.beta_2, opt.epsilon, 1.0, lr_dev=self.lr_dev)
        S.launch(fn, dz.device, aux=True)
        self.done.append((o, o + n))


class SGD(Optimizer):
    """``tf.keras.optimizers.SGD(learning_rate, momentum, nesterov)`` as one fused flat kernel
    (the usual ResNet-50 optimizer)."""

    def __init__(self, learning_rate: float = 0.01, momentum: float = 0.0, nesterov: bool = False, name: str = "SGD"):
        super().__init__(learning_rate)
        self.momentum, self.nesterov, self.name = float(momentum), bool(nesterov), name
        self.velocity = None

    def build(self, store) -> None:
        if self.momentum > 0 and (self.velocity is None or self.velocity.numel() != store.total
                                  or self.velocity.device != store.flat.device):
            self.velocity = K.zeros(store.total, torch.float32, store.flat.device)

    def apply(self, store, gscale: float = 1.0, lo: int = 0, hi: int | None = None, advance: bool = True) -> None:
        self.build(store)
        hi = store.total if hi is None else hi
        if hi > lo:
            sl = slice(lo, hi)
            K.sgd(store.flat[sl], store.flat_grad[sl], self.velocity[sl] if self.velocity is not None else None,
                  store.flat_bf16[sl], self.learning_rate, self.momentum, self.nesterov, gscale, clear_grad=True)
        if lo == 0 and hi >= store.total:
            store.grad_clean = True
        if advance:
            self.iterations += 1

    def apply_shard(self, store, grad_shard, lo: int, hi: int, gscale: float = 1.0, advance: bool = True) -> None:
        self.build(store)
        if hi > lo:
            K.sgd(store.flat[lo:hi], grad_shard, self.velocity[lo:hi] if self.velocity is not None else None,
                  store.flat_bf16[lo:hi], self.learning_rate, self.momentum, self.nesterov, gscale)
        if advance:
            self.iterations += 1

    def get_config(self):
        return {"name": self.name, "learning_rate": self.learning_rate, "momentum": self.momentum,
                "nesterov": self.nesterov}

    def state_tensors(self) -> dict:
        return {"velocity": self.velocity} if self.velocity is not None else {}

    def use_device_step(self, store) -> None:
        self.build(store)  # SGD has no step-dependent scalars: its launch is capturable as is


def get(identifier) -> Optimizer:
    if isinstance(identifier, Optimizer):
        return identifier
    if isinstance(identifier, str) and identifier.lower() == "adam":
        return Adam()
    if isinstance(identifier, str) and identifier.lower() == "sgd":
        return SGD()
    raise ValueError(f"unknown optimizer {identifier!r}")
