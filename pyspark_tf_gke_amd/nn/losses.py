"""Keras-compatible loss objects (train_tf_ps.py:340,375,607,729).

In ``fit()`` the loss runs as one fused device kernel that also produces the output gradient and
the metric sums (``ops.nn.mse`` / ``ops.nn.softmax_xent``).  Calling a loss object directly
(custom training loops, :mod:`.tape`) returns the scalar loss and, under a GradientTape, records
which fused kernel to run for the backward pass.
"""
from __future__ import annotations

import torch


class Loss:
    name = "loss"
    kind = "none"

    def __call__(self, y_true, y_pred):
        from .tape import _active_tape

        from .tape import _HeadPred

        y_true = torch.as_tensor(y_true, device=y_pred.device)
        tape = _active_tape()
        val = None
        hd = getattr(y_pred, "_lz", None) if isinstance(y_pred, _HeadPred) else None
        if hd is not None and hd.state == "pending" and self.kind == "mse" and tape is not None and tape.out is y_pred:
            val = hd.fused_loss(self, y_true)  # fit()'s fused regression head (nn/tape.py)
        fused = val is not None
        if val is None:
            val = self.compute(y_true, y_pred)
        if tape is not None:
            # a differentiable scalar: tape.gradient() accepts it and linear combinations of it
            val = tape.record_loss(self, y_true, y_pred, val)
            if fused:
                hd.record = val._terms[0][0]
        return val

    def compute(self, y_true, y_pred):
        raise NotImplementedError

    def get_config(self):
        return {"name": self.name}


class MeanSquaredError(Loss):
    name = "mean_squared_error"
    kind = "mse"

    def compute(self, y_true, y_pred):
        d = y_pred.float() - y_true.float()
        return (d * d).mean()


class SparseCategoricalCrossentropy(Loss):
    name = "sparse_categorical_crossentropy"
    kind = "sparse_xent"

    def __init__(self, from_logits: bool = False):
        self.from_logits = from_logits

    def compute(self, y_true, y_pred):
        p = y_pred.float()
        if self.from_logits:
            p = torch.softmax(p, -1)
        p = p.gather(1, y_true.long().view(-1, 1)).clamp(1e-7, 1 - 1e-7)
        return (-p.log()).mean()


def get(identifier) -> Loss:
    if isinstance(identifier, Loss):
        return identifier
    key = str(identifier).lower()
    if key in ("mse", "mean_squared_error", "meansquarederror"):
        return MeanSquaredError()
    if key in ("sparse_categorical_crossentropy", "sparsecategoricalcrossentropy"):
        return SparseCategoricalCrossentropy()
    raise ValueError(f"unknown loss {identifier!r}")
