"""GradientTape-style custom training loops on the fused engine.

The reference's ParameterServerStrategy step (train_tf_ps.py:616-631, :738-753) is::

    with tf.GradientTape() as tape:
        preds = model(features, training=True)
        loss = loss_obj(labels, preds)
    grads = tape.gradient(loss, model.trainable_variables)
    optimizer.apply_gradients(zip(grads, model.trainable_variables))

The same code runs here.  The tape does not trace Python ops: it records the model forward
(the engine already keeps every activation its fused backward needs) and the loss object, and
``gradient()`` runs the fused loss kernel + fused backward into the flat gradient buffer.
``apply_gradients`` then performs the active strategy's collective (all-reduce / reduce-scatter)
and the single fused Adam launch.
"""
from __future__ import annotations

import torch

_TAPES: list = []


def _active_tape():
    return _TAPES[-1] if _TAPES else None


class GradientTape:
    def __init__(self, persistent: bool = False):
        self.model = None
        self.out = None
        self.x = None
        self.loss_obj = None
        self.y_true = None

    def __enter__(self):
        _TAPES.append(self)
        return self

    def __exit__(self, *exc):
        _TAPES.remove(self)
        return False

    def record_forward(self, model, out):
        self.model, self.out = model, out

    def record_loss(self, loss_obj, y_true, y_pred, value):
        self.loss_obj, self.y_true = loss_obj, y_true

    def gradient(self, target, sources):
        from . import engine as E
        from . import losses as LS

        m = self.model
        if m is None or self.loss_obj is None:
            raise RuntimeError("GradientTape.gradient: no model forward / loss recorded")
        out = self.out
        last = m._last_op()
        if isinstance(self.loss_obj, LS.SparseCategoricalCrossentropy) and isinstance(last, E.DenseOp) \
                and last.act == "softmax" and not last.logits_only:
            raise RuntimeError("compile() the model with the loss (or build with from_logits) before a tape loop")
        stats = torch.zeros(8, dtype=torch.float32, device=out.device)
        saved_loss = m.loss
        m.loss = self.loss_obj
        try:
            yb = self.y_true
            if isinstance(self.loss_obj, LS.SparseCategoricalCrossentropy):
                yb = yb.to(torch.int32).view(-1).contiguous()
            else:
                yb = yb.float().contiguous()
                if yb.dim() == 1:
                    yb = yb.view(-1, 1)
            m.store.zero_grad()
            dpred = m._loss_grad(out, yb, stats)
        finally:
            m.loss = saved_loss
        m._run_backward(dpred)
        m._pending_grads = True
        return [v.param.grad for v in sources]


def apply_gradients(optimizer, grads_and_vars) -> None:
    gv = list(grads_and_vars)
    if not gv:
        return
    model = gv[0][1].model
    from ..distribute import current_strategy

    st = getattr(model, "strategy", None) or current_strategy()
    if st is not None:
        st.finish_gradients(model)
        st.apply_update(model, optimizer)
    else:
        optimizer.apply(model.store)
    model._pending_grads = False
