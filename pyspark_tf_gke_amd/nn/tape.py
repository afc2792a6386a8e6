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

from .. import config

_TAPES: list = []
OVERLAP = config.get("tape_overlap")


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
        from ..distribute import current_strategy
        from . import streams as S

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
        # the same side-stream overlap as fit()'s step (streams.py): every wgrad forks off the dgrad
        # chain and the step's stream joins it before returning, so the gradients handed back are
        # stream-ordered complete, exactly as with the serial backward
        st = getattr(m, "strategy", None) or current_strategy()
        side = S.for_step(m.store, st)
        ready: list = []

        def dense_done(op):
            # a big Dense layer's dW has just been forked onto the side stream: an event there lets
            # apply_gradients start that layer's Adam while the conv backward below still runs
            if side is not None and isinstance(op, E.DenseOp) and op.big:
                p = op.dense.kernel
                ev = torch.cuda.Event()
                ev.record(S._stream(p.grad.device))
                ready.append((p.offset, p.offset + p.numel, ev))

        with S.active(side):
            m._run_backward(dpred, on_op_done=dense_done)
        # one local replica (no strategy, or a one-worker parameter server) can overlap its update
        m._tape_ready = ready if st is None or getattr(st, "world_size", 2) == 1 else None
        m._pending_grads = True
        return [v.param.grad for v in sources]


def apply_gradients(optimizer, grads_and_vars) -> None:
    gv = list(grads_and_vars)
    if not gv:
        return
    model = gv[0][1].model
    from ..distribute import current_strategy

    st = getattr(model, "strategy", None) or current_strategy()
    ready = getattr(model, "_tape_ready", None)
    model._tape_ready = None
    if st is not None:
        # a one-worker ParameterServerStrategy applies the update itself (possibly at round commit)
        # and takes the overlapped form from here (ps.py _apply_local)
        model._tape_overlap = ready if ready and _overlap_ok(optimizer, gv) else None
        st.finish_gradients(model)
        st.apply_update(model, optimizer)
    elif ready and _overlap_ok(optimizer, gv):
        _apply_overlapped(optimizer, model.store, ready)
    else:
        optimizer.apply(model.store)
    model._pending_grads = False


_AUX: dict = {}


def _overlap_ok(optimizer, gv) -> bool:
    """The gradients handed in are the tape's own buffers, untouched (no clipping / scaling in
    between), and the optimizer is plain flat Adam with a host-side step counter."""
    from .optimizers import Adam

    return (OVERLAP and type(optimizer) is Adam and getattr(optimizer, "dev_state", None) is None
            and all(getattr(v, "param", None) is not None and g is v.param.grad for g, v in gv))


def _apply_overlapped(optimizer, store, ready) -> None:
    """Adam over the big Dense ranges on an auxiliary stream, each waiting only for its layer's dW
    (so the HBM-bound update overlaps the rest of the backward), then the remaining gaps on the
    step's stream, which joins the auxiliary stream before returning."""
    dev = store.flat.device
    aux = _AUX.get(dev)
    if aux is None:
        aux = _AUX[dev] = torch.cuda.Stream(device=dev)
    cur = torch.cuda.current_stream(dev)
    # aux deliberately does not wait for the step's stream: each range's event already follows
    # everything that reads or writes that range before its update (this step's forward and dX
    # read the bf16 weights before the dW fork; the previous update was joined into the step's
    # stream).  The gradients of those ranges are cleared by the update, so code that reads them
    # between gradient() and apply_gradients() must turn this off (PTG_TAPE_OVERLAP=0).
    step = optimizer.iterations + 1
    # a fresh optimizer allocates and zero-fills its moments HERE, on the step's stream; the aux
    # stream must not read them before that fill (it otherwise never waits for the step's stream)
    before = optimizer.m
    optimizer.build(store)
    if optimizer.m is not before:
        aux.wait_stream(cur)
    with torch.cuda.stream(aux):
        for lo, hi, ev in ready:
            aux.wait_event(ev)
            optimizer.apply(store, lo=lo, hi=hi, advance=False)
    lo = 0
    for a, b in sorted((r[0], r[1]) for r in ready) + [(store.total, store.total)]:
        if a > lo:
            optimizer.apply(store, lo=lo, hi=a, advance=False)
        lo = max(lo, b)
    cur.wait_stream(aux)
    store.grad_clean = True
    optimizer.iterations = step
