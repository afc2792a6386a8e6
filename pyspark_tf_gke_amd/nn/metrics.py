"""Keras-compatible streaming metrics (train_tf_ps.py:608-609,627-628,730-732,748-750).

State is two device scalars (total, count); ``result()`` is the only host sync.  Under a
distribution strategy ``result()`` all-reduces the pair across ranks, which is what TF's
PS-hosted metric variables give the reference (M3 in SURVEY §2.2.c).
"""
from __future__ import annotations

import torch


class Metric:
    def __init__(self, name: str):
        from ..distribute import current_strategy

        self.name = name
        self._total = None
        self._count = None
        self._strategy = current_strategy()  # metrics created under strategy.scope() stay bound to it

    def _ensure(self, device):
        if self._total is None or self._total.device != torch.device(device):
            self._total = torch.zeros((), dtype=torch.float64, device=device)
            self._count = torch.zeros((), dtype=torch.float64, device=device)

    def reset_state(self):
        if self._total is not None:
            self._total.zero_()
            self._count.zero_()

    def _add(self, total, count, device):
        self._ensure(device)
        self._total += total
        self._count += count

    def result(self):
        if self._total is None:
            self._ensure("cpu" if self._strategy is None else self._strategy.device)
        from ..distribute import current_strategy

        t = torch.stack([self._total, self._count])
        st = self._strategy or current_strategy()
        if st is not None:
            t = st.all_reduce_sum(t)
        tot, cnt = t[0].item(), t[1].item()
        return torch.tensor(tot / cnt if cnt else 0.0, dtype=torch.float32)


class Mean(Metric):
    def __init__(self, name: str = "mean"):
        super().__init__(name)

    def update_state(self, values, sample_weight=None):
        v = torch.as_tensor(values)
        self._add(v.double().sum(), float(v.numel()), v.device)


class MeanAbsoluteError(Metric):
    def __init__(self, name: str = "mean_absolute_error"):
        super().__init__(name)

    def update_state(self, y_true, y_pred, sample_weight=None):
        yp = torch.as_tensor(y_pred)
        yt = torch.as_tensor(y_true, device=yp.device)
        d = (yp.double() - yt.double()).abs()
        self._add(d.sum(), float(d.numel()), yp.device)


class MeanSquaredError(Metric):
    def __init__(self, name: str = "mean_squared_error"):
        super().__init__(name)

    def update_state(self, y_true, y_pred, sample_weight=None):
        yp = torch.as_tensor(y_pred)
        yt = torch.as_tensor(y_true, device=yp.device)
        d = yp.double() - yt.double()
        self._add((d * d).sum(), float(d.numel()), yp.device)


class SparseCategoricalAccuracy(Metric):
    def __init__(self, name: str = "sparse_categorical_accuracy"):
        super().__init__(name)

    def update_state(self, y_true, y_pred, sample_weight=None):
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
