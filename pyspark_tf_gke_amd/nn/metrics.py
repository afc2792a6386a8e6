"""Keras-compatible streaming metrics (train_tf_ps.py:608-609,627-628,730-732,748-750).

State is two device scalars (total, count); ``result()`` is the only host sync.  Under a
distribution strategy ``result()`` all-reduces the pair across ranks, which is what TF's
PS-hosted metric variables give the reference (M3 in SURVEY §2.2.c).
"""
from __future__ import annotations

import torch


_MT = {torch.float32: 0, torch.float64: 1, torch.bfloat16: 2, torch.int32: 3, torch.int64: 4}


class Metric:
    def __init__(self, name: str):
        from ..distribute import current_strategy

        self.name = name
        self._state = None  # f64[2] = (total, count) on the data's device
        self._total = None
        self._count = None
        self._strategy = current_strategy()  # metrics created under strategy.scope() stay bound to it

    def _ensure(self, device):
        if self._state is None or self._state.device != torch.device(device):
            self._state = torch.zeros(2, dtype=torch.float64, device=device)
            self._total, self._count = self._state[0], self._state[1]

    def _fused(self, kind: int, yp, yt=None, C: int = 0) -> bool:
        """One-launch update on the GPU (nn_eltwise.hip metric_update_k); False: use the torch ops."""
        if not (isinstance(yp, torch.Tensor) and yp.is_cuda and yp.dtype in _MT and yp.is_contiguous()):
            return False
        if yt is not None:
            if not (isinstance(yt, torch.Tensor) and yt.is_cuda and yt.dtype in _MT and yt.is_contiguous()):
                return False
            n = yt.numel() if kind == 3 else yp.numel()
            if (kind == 3 and yp.numel() != n * C) or (kind != 3 and yt.numel() != n):
                return False
        else:
            n = yp.numel()
        from ..ops._util import hip
        from .tape import _Deferred

        for t in (yp, yt):  # a deferred prediction (nn/tape.py) is computed before the kernel reads it
            if isinstance(t, _Deferred) and getattr(t, "_lz", None) is not None:
                t._lz.materialize()
        self._ensure(yp.device)
        hip("ptg_metric_update", kind, yp.data_ptr(), _MT[yp.dtype], yt.data_ptr() if yt is not None else None,
            _MT[yt.dtype] if yt is not None else 0, n, C, float(n), self._state.data_ptr())
        return True

    def reset_state(self):
        if self._state is not None:
            self._state.zero_()

    def _add(self, total, count, device):
        self._ensure(device)
        self._total += total
        self._count += count

    def result(self):
        if self._total is None:
            self._ensure("cpu" if self._strategy is None else self._strategy.device)
        from ..distribute import current_strategy

        t = self._state.clone()
        st = self._strategy or current_strategy()
        if st is not None:
            t = st.all_reduce_sum(t)
        tot, cnt = t[0].item(), t[1].item()
        return torch.tensor(tot / cnt if cnt else 0.0, dtype=torch.float32)


class Mean(Metric):
    def __init__(self, name: str = "mean"):
        super().__init__(name)

    def update_state(self, values, sample_weight=None):
        if sample_weight is None and self._fused(0, values):
            return
        v = torch.as_tensor(values)
        self._add(v.double().sum(), float(v.numel()), v.device)


class MeanAbsoluteError(Metric):
    def __init__(self, name: str = "mean_absolute_error"):
        super().__init__(name)

    def update_state(self, y_true, y_pred, sample_weight=None):
        if sample_weight is None and self._fused(1, y_pred, y_true):
            return
        yp = torch.as_tensor(y_pred)
        yt = torch.as_tensor(y_true, device=yp.device)
        d = (yp.double() - yt.double()).abs()
        self._add(d.sum(), float(d.numel()), yp.device)


class MeanSquaredError(Metric):
    def __init__(self, name: str = "mean_squared_error"):
        super().__init__(name)

    def update_state(self, y_true, y_pred, sample_weight=None):
        if sample_weight is None and self._fused(2, y_pred, y_true):
            return
        yp = torch.as_tensor(y_pred)
        yt = torch.as_tensor(y_true, device=yp.device)
        d = yp.double() - yt.double()
        self._add((d * d).sum(), float(d.numel()), yp.device)


class SparseCategoricalAccuracy(Metric):
    def __init__(self, name: str = "sparse_categorical_accuracy"):
        super().__init__(name)

    def update_state(self, y_true, y_pred, sample_weight=None):
        if (sample_weight is None and isinstance(y_pred, torch.Tensor) and y_pred.dim() == 2
                and self._fused(3, y_pred, y_true, y_pred.shape[-1])):
            return
        yp = torch.as_tensor(y_pred)
        yt = torch.as_tensor(y_true, device=yp.device)
        c = (yp.argmax(-1) == yt.long().view(-1)).double()
        self._add(c.sum(), float(c.numel()), yp.device)


def canonical_name(m) -> str:
    if isinstance(m, Metric):
        return m.name
    key = str(m).lower()
    return {"mean_absolute_error": "mae", "mean_squared_error": "mse", "acc": "accuracy",
            "sparse_categorical_accuracy": "accuracy"}.get(key, key)
