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

On one local replica (no strategy, or a one-worker parameter server) a model ending in
[Dense(relu, big), Dense(N <= 4)] returns its prediction from the tape forward as a deferred tensor
held at the big layer's split-K sums; an MSE loss object called on it runs fit()'s two-kernel fused
head instead of the seven-kernel tail + loss + loss gradient.  The same replica defers each big Dense layer's
weight-gradient GEMM: ``gradient()`` hands back a :class:`_LazyGrad` for that kernel, which computes
the gradient the moment anything reads it.  When it reaches ``apply_gradients`` untouched, the
update runs Adam inside that GEMM's epilogue (``ops.nn.linear_dw_adam``, as fit() does) on an
auxiliary stream, so the [2048, 20480] fp32 gradient is never written nor read back.
"""
from __future__ import annotations

import torch

from .. import config

_TAPES: list = []
OVERLAP = config.get("tape_overlap")
LAZY_DW = config.get("tape_lazy_dw")
TAPE_HEAD = config.get("tape_fused_head")


def _active_tape():
    return _TAPES[-1] if _TAPES else None


_META = {"shape", "dtype", "device", "is_cuda", "ndim", "size", "dim", "numel", "layout", "requires_grad",
         "is_floating_point", "element_size", "__len__"}


def _func_name(func) -> str:
    n = getattr(func, "__name__", "")
    if n == "__get__":  # a property getter: the descriptor carries the name
        n = getattr(getattr(func, "__self__", None), "__name__", "")
    return n


class _Deferred(torch.Tensor):
    """A tensor whose contents a deferred kernel still has to produce (``_lz.materialize()``).  It
    aliases the buffer that kernel writes; any torch operation on it (metadata queries aside)
    first runs the kernel, so user code sees an ordinary tensor."""

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if _func_name(func) not in _META:
            _materialize_in(args)
            _materialize_in(kwargs.values())
        with torch._C.DisableTorchFunctionSubclass():
            return func(*args, **kwargs)


class _LazyGrad(_Deferred):
    """The gradient of a big Dense kernel whose GEMM has not run yet (``_lz``: a :class:`_LazyDW`)."""


# ---------------------------------------------------------------------------------------------
# Differentiable targets.  The tape does not trace arbitrary torch code; what it can differentiate
# is a LINEAR combination of the loss values it recorded (train_tf_ps.py:620-625 builds
# ``loss = loss_obj(labels, preds); loss += tf.add_n(model.losses) if model.losses else 0.0``).
# A loss object called under a tape returns a _TapeLoss: the scalar value plus its terms
# ((record, coefficient), ...).  +, -, unary -, * and / by a constant, add_n and sum keep the
# terms; any other operation returns a plain tensor, which gradient() refuses.
# ---------------------------------------------------------------------------------------------
class _LossRecord:
    """One loss-object call under a tape: its gradient is d(loss_obj(y_true, y_pred)) / d(params)."""

    def __init__(self, tape, loss_obj, y_true, y_pred):
        self.tape, self.loss_obj, self.y_true, self.y_pred = tape, loss_obj, y_true, y_pred


_ADD = {"add", "__add__", "__radd__", "__iadd__", "add_"}
_SUB = {"sub", "__sub__", "__isub__", "sub_", "subtract"}
_RSUB = {"__rsub__", "rsub"}
_MUL = {"mul", "__mul__", "__rmul__", "__imul__", "mul_", "multiply"}
_DIV = {"div", "__truediv__", "__itruediv__", "div_", "true_divide", "divide"}
_NEG = {"neg", "__neg__", "negative"}
_SAME = {"float", "to", "clone", "contiguous", "reshape", "view", "squeeze", "unsqueeze", "sum", "mean",
         "__pos__", "positive"}


def _terms(x):
    """Terms of a tape loss, () for a constant (a number or a tensor the tape does not track)."""
    return getattr(x, "_terms", ()) if isinstance(x, _TapeLoss) else ()


def _const(x) -> float | None:
    if isinstance(x, _TapeLoss):
        return None
    if isinstance(x, (int, float)):
        return float(x)
    if isinstance(x, torch.Tensor) and x.numel() == 1:
        return float(x)
    return None


def _scaled(ts, c: float):
    return tuple((r, k * c) for r, k in ts)


def _lin_terms(name: str, args, kwargs):
    """The terms of func(*args) for a linear func of tape losses and constants, or None."""
    a = args[0] if args else None
    b = args[1] if len(args) > 1 else kwargs.get("other")
    alpha = kwargs.get("alpha", 1)
    if any(isinstance(x, _TapeLoss) and getattr(x, "_terms", ()) is None for x in (a, b)):
        return None  # an operand an in-place op already took out of the linear family
    if name in _SAME:
        return _terms(a)
    if name in _NEG:
        return _scaled(_terms(a), -1.0)
    if name in _ADD:
        return _terms(a) + _scaled(_terms(b), float(alpha))
    if name in _SUB:
        return _terms(a) + _scaled(_terms(b), -float(alpha))
    if name in _RSUB:  # b - a
        return _terms(b) + _scaled(_terms(a), -1.0)
    if name in _MUL:
        ta, tb = _terms(a), _terms(b)
        if ta and tb:
            return None  # loss * loss is not linear
        if not ta and not tb:
            return ()
        c = _const(b if ta else a)
        return None if c is None else _scaled(ta or tb, c)
    if name in _DIV:
        if _terms(b):
            return None
        c = _const(b)
        return None if not c else _scaled(_terms(a), 1.0 / c)
    return None


class _TapeLoss(torch.Tensor):
    """A scalar loss value the tape can differentiate (``_terms``)."""

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        name = _func_name(func)
        with torch._C.DisableTorchFunctionSubclass():
            out = func(*args, **kwargs)
        if name in _META or not isinstance(out, torch.Tensor):
            return out
        ts = _lin_terms(name, args, kwargs)
        if ts is None or out.numel() != 1:
            if isinstance(out, _TapeLoss):  # an in-place op that left the linear family
                out._terms = None
            return out.as_subclass(torch.Tensor) if isinstance(out, _TapeLoss) else out
        res = out if isinstance(out, _TapeLoss) else out.as_subclass(_TapeLoss)
        res._terms = ts
        return res


def _tape_loss(value, record) -> _TapeLoss:
    v = torch.as_tensor(value)
    t = v.as_subclass(_TapeLoss)
    t._terms = ((record, 1.0),)
    return t


def add_n(inputs):
    """``tf.add_n``: the sum of a list of (tape) losses, keeping what the tape can differentiate."""
    inputs = list(inputs)
    if not inputs:
        raise ValueError("add_n of an empty list")
    out = inputs[0]
    for x in inputs[1:]:
        out = out + x
    return out


def _param_of(src):
    p = getattr(src, "param", None)
    if p is not None:
        return p
    if hasattr(src, "offset") and hasattr(src, "grad"):
        return src  # a Param of the flat store
    raise TypeError(f"GradientTape.gradient: source {src!r} is not a model variable")


class _HeadPred(_Deferred):
    """The prediction of a [..., Dense(relu, big), Dense(N <= 4)] tail under a tape, held at the
    big layer's split-K sums (``_lz``: a :class:`_HeadState`): an MSE loss object called on it runs
    fit()'s fused head (forward, loss, head backward in two launches); anything else runs the
    plain tail first."""


class _HeadState:
    def __init__(self, model, acc, pred):
        self.model, self.acc, self.pred = model, acc, pred
        self.state = "pending"  # -> "plain" (unfused tail ran) or "fused" (head_mse ran for the loss)
        self.dz1 = None
        self.loss_obj = None
        self.record = None  # the tape's _LossRecord of the fused loss call

    def discard(self) -> None:
        """An abandoned pending prediction (a failed closure, a second forward before the loss):
        the split-K sums it holds must not leak into the next forward, which adds onto them."""
        if self.state == "pending":
            self.acc.zero_()
            self.state = "dropped"

    def redo_plain(self) -> None:
        """The fused head ran for a loss, but the tape is asked for the gradient of another target:
        recompute the big layer's sums (the head consumed them) and run the plain tail instead."""
        if self.state != "fused":
            return
        d1 = self.model.ops[-2]
        d1.forward_splitk_sums(d1._x, self.model.ws)
        self.state, self.dz1, self.loss_obj, self.record = "pending", None, None, None
        self.materialize()

    def scale_grads(self, c: float) -> None:
        """The target is c x the fused loss: scale what the head kernels produced (dz1 and the
        Dense2 / Dense1-bias gradients); the backward below is linear in dz1."""
        d1, d2 = self.model.ops[-2], self.model.ops[-1]
        self.dz1.mul_(c)
        for g in (d2.dense.kernel.grad, d2.dense.bias.grad, d1.dense.bias.grad):
            g.mul_(c)

    def materialize(self) -> None:
        """The unfused tail: Dense1 bias + ReLU from the split-K sums (re-zeroing them), Dense2."""
        if self.state != "pending":
            return
        from ..ops import nn as K

        self.state = "plain"
        m = self.model
        d1, d2 = m.ops[-2], m.ops[-1]
        B, N1 = self.acc.shape[-2:]
        y1 = m.ws.get(d1.name + "/y", (B, N1), torch.bfloat16, self.acc.device)
        K.bias_act(self.acc, d1.dense.bias.data, "relu", out_bf16=y1, clear=True)
        d1._y = y1
        if d2.mask_for_prev:
            d2._prev_y = y1
        y2 = d2.forward(y1, m.ws, True)
        self.pred.copy_(y2)

    def fused_loss(self, loss_obj, y_true):
        """The loss value of an MSE loss object, computed by fit()'s fused head kernels, which also
        leave dz1 (Dense1's pre-activation gradient) and the Dense2 / Dense1-bias gradients."""
        from ..ops import nn as K

        m = self.model
        d1, d2 = m.ops[-2], m.ops[-1]
        B, K1 = self.acc.shape[-2:]
        N2 = d2.dense.units
        yb = y_true.float()
        if yb.dim() == 1:
            yb = yb.view(-1, 1)
        if tuple(yb.shape) != (B, N2):
            return None
        yb = yb.contiguous()
        flush_lazy(m)
        m.store.zero_grad()  # the head accumulates the Dense2 and Dense1-bias gradients
        dev = self.acc.device
        dz1 = m.ws.get(d1.name + "/dz", (B, K1), torch.bfloat16, dev)
        scratch = m.ws.get(d1.name + "/headscratch", (B * (N2 + 2),), torch.float32, dev)
        stats = m.ws.get("__tape_head_stats", (8,), torch.float32, dev)
        stats.zero_()
        K.head_mse(self.acc, d1.dense.bias.data, d2.dense.kernel.data, d2.dense.bias.data, yb, dz1,
                   d2.dense.kernel.grad, d2.dense.bias.grad, d1.dense.bias.grad, stats, pred_out=self.pred,
                   scratch=scratch)
        self.state, self.dz1, self.loss_obj = "fused", dz1, loss_obj
        return stats[2] / float(B * N2)


def _materialize_in(xs) -> None:
    for a in xs:
        if isinstance(a, _Deferred):
            lz = getattr(a, "_lz", None)
            if lz is not None:
                lz.materialize()
        elif isinstance(a, (list, tuple)):
            _materialize_in(a)
        elif isinstance(a, dict):
            _materialize_in(a.values())


def _event(dev):
    if dev.type != "cuda":
        return None
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(dev))
    return ev


class _LazyDW:
    """One deferred Dense weight gradient dW = dz^T @ x: the bf16 operands stay in the model's
    workspace until ``materialize()`` (the plain GEMM into the gradient buffer) or ``fused_adam()``
    (Adam in the GEMM epilogue) consumes them; the model flushes pending ones before its next
    forward rewrites that workspace."""

    def __init__(self, dz, x, param):
        self.dz, self.x, self.param = dz, x, param
        self.pending = True
        self.ev = _event(dz.device)  # after dz, x are final (and this layer's dX has read the weights)
        self.view = None

    def materialize(self) -> None:
        if not self.pending:
            return
        self.pending = False
        from ..ops import nn as K

        K.linear_dw(self.dz, self.x, self.param.grad)
        self.ev = _event(self.dz.device)

    def fused_adam(self, opt, store, step: int) -> None:
        from ..ops import nn as K

        self.pending = False
        p = self.param
        o, n = p.offset, p.numel
        shp = p.grad.shape
        K.linear_dw_adam(self.dz, self.x, store.flat[o:o + n].view(shp), opt.m[o:o + n].view(shp),
                         opt.v[o:o + n].view(shp), store.flat_bf16[o:o + n].view(shp), opt.lr_t(step),
                         opt.beta_1, opt.beta_2, opt.epsilon, 1.0)


class _DeferDW:
    """Stands in for fit()'s FusedAdamStep during a tape backward (DenseOp.backward calls
    ``linear_dw``): it records the GEMM's operands instead of launching it."""

    cpu_ok = True

    def __init__(self):
        self.items: list = []

    def linear_dw(self, dz, x, param) -> None:
        self.items.append(_LazyDW(dz, x, param))


def flush_lazy(model) -> None:
    """Compute every deferred weight gradient of ``model`` (on the current stream)."""
    lz = getattr(model, "_lazy_dw", None)
    if lz:
        model._lazy_dw = None
        for d in lz:
            d.materialize()


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
        self.model, self.out, self.ret = model, out, out

    def record_loss(self, loss_obj, y_true, y_pred, value):
        self.loss_obj, self.y_true = loss_obj, y_true
        rec = _LossRecord(self, loss_obj, y_true, y_pred)
        self.records = getattr(self, "records", []) + [rec]
        return _tape_loss(value, rec)

    def _target_terms(self, target):
        """Merge the target's terms per loss record; raise for anything the tape cannot differentiate."""
        ts = getattr(target, "_terms", None) if isinstance(target, _TapeLoss) else None
        if ts is None:
            raise ValueError("GradientTape.gradient: the target is not a linear combination of loss values "
                             "recorded by this tape (loss objects called on the model output inside the "
                             "`with` block, combined by +, -, * / constant, add_n)")
        merged: dict = {}
        for rec, c in ts:
            if rec.tape is not self:
                raise ValueError("GradientTape.gradient: the target depends on a loss recorded by another tape")
            if rec.y_pred is not self.out and rec.y_pred is not self.ret:
                raise ValueError("GradientTape.gradient: the target depends on a loss of a prediction other than "
                                 "this tape's last model forward")
            r0, c0 = merged.get(id(rec), (rec, 0.0))
            merged[id(rec)] = (rec, c0 + c)
        return [(r, c) for r, c in merged.values() if c != 0.0]

    @staticmethod
    def _labels(loss_obj, y_true):
        from . import losses as LS

        if isinstance(loss_obj, LS.SparseCategoricalCrossentropy):
            return y_true.to(torch.int32).view(-1).contiguous()
        yb = y_true.float().contiguous()
        return yb.view(-1, 1) if yb.dim() == 1 else yb

    def _dpred(self, m, out, terms):
        """d(target)/d(prediction) = sum of coefficient x the fused loss kernels' output gradients."""
        stats = torch.zeros(8, dtype=torch.float32, device=out.device)
        saved_loss = m.loss
        dpred = None
        try:
            for rec, c in terms:
                m.loss = rec.loss_obj
                dp = m._loss_grad(out, self._labels(rec.loss_obj, rec.y_true), stats, gscale=c)
                if dpred is None:
                    dpred = dp.clone() if len(terms) > 1 else dp  # dp is the model's reused workspace
                else:
                    dpred.add_(dp)
        finally:
            m.loss = saved_loss
        return dpred

    def gradient(self, target, sources):
        from . import engine as E
        from . import losses as LS
        from ..distribute import current_strategy
        from . import streams as S

        m = self.model
        if m is None or self.loss_obj is None:
            raise RuntimeError("GradientTape.gradient: no model forward / loss recorded")
        single = not isinstance(sources, (list, tuple))
        srcs = [sources] if single else list(sources)
        params = [_param_of(s) for s in srcs]
        own = {id(p) for p in m.store.params}
        for p in params:
            if id(p) not in own:
                raise ValueError(f"GradientTape.gradient: source {p.name!r} is not a variable of the recorded model")
        terms = self._target_terms(target)
        flush_lazy(m)
        out = self.out
        last = m._last_op()
        if any(isinstance(r.loss_obj, LS.SparseCategoricalCrossentropy) for r, _ in terms) \
                and isinstance(last, E.DenseOp) and last.act == "softmax" and not last.logits_only:
            raise RuntimeError("compile() the model with the loss (or build with from_logits) before a tape loop")
        hd = getattr(out, "_lz", None) if isinstance(out, _HeadPred) else None
        head = (hd is not None and hd.state == "fused" and len(terms) == 1 and terms[0][0].loss_obj is hd.loss_obj
                and terms[0][0] is getattr(hd, "record", None))
        if hd is not None and hd.state == "fused" and not head:
            hd.redo_plain()  # the fused head's gradients are those of one unscaled loss: run the plain tail
        if head and terms[0][1] != 1.0:
            hd.scale_grads(terms[0][1])
        if not head:
            m.store.zero_grad()
            if not terms:  # e.g. loss - loss: every gradient is zero
                return self._result([p.grad for p in params], single)
            dpred = self._dpred(m, out, terms)
        # the same side-stream overlap as fit()'s step (streams.py): every wgrad forks off the dgrad
        # chain and the step's stream joins it before returning, so the gradients handed back are
        # stream-ordered complete, exactly as with the serial backward
        st = getattr(m, "strategy", None) or current_strategy()
        side = S.for_step(m.store, st)
        ready: list = []
        local = _update_takes_overlap(st)
        # one local replica whose update consumes the tape's overlap list (no strategy, or a one-worker
        # parameter server, ps.py _apply_local): defer the big Dense dW
        defer = _DeferDW() if (OVERLAP and LAZY_DW and local) else None
        big = [op for op in m.ops if isinstance(op, E.DenseOp) and op.big] if defer is not None else []
        for op in big:
            op.fused_update = defer

        def dense_done(op):
            # a big Dense layer's dW has just been forked onto the side stream: an event there lets
            # apply_gradients start that layer's Adam while the conv backward below still runs
            if side is not None and defer is None and isinstance(op, E.DenseOp) and op.big:
                p = op.dense.kernel
                ev = torch.cuda.Event()
                ev.record(S._stream(p.grad.device))
                ready.append((p.offset, p.offset + p.numel, ev, None))

        try:
            with S.active(side):
                if head:  # the head kernels already produced dz1 and the head's own gradients
                    d1 = m.ops[-2]
                    dx = d1.backward_dz(hd.dz1, m.ws)
                    dense_done(d1)
                    E.run_backward(m.ops[:-2], dx, m.ws, on_op_done=dense_done)
                else:
                    m._run_backward(dpred, on_op_done=dense_done)
        finally:
            for op in big:
                op.fused_update = None
        grads = {}
        if defer is not None and defer.items:
            m._lazy_dw = defer.items
            for d in defer.items:
                p = d.param
                d.view = p.grad.as_subclass(_LazyGrad)
                d.view._lz = d
                grads[id(p)] = d.view
                ready.append((p.offset, p.offset + p.numel, None, d))
        m._tape_ready = ready if local else None
        m._pending_grads = True
        return self._result([grads.get(id(p), p.grad) for p in params], single)

    def _result(self, grads, single):
        self.model._pending_grads = True
        return grads[0] if single else grads


def _update_takes_overlap(st) -> bool:
    """Whether the update after a tape backward consumes the tape's overlap list (deferred Dense dW
    fused with Adam, per-range Adam events): with no strategy (apply_gradients runs it) or a
    one-worker ParameterServerStrategy (ps.py _apply_local).  Any other strategy reads the whole flat
    gradient buffer, so nothing may be deferred."""
    if st is None:
        return True
    from ..distribute.ps import ParameterServerStrategy
    from ..parallel import comm

    # the same gate as ps.py's apply_update / commit_round: a one-worker group that still runs its
    # collectives (PTG_FORCE_PG + PTG_COLLECTIVES_WORLD1) pushes the flat gradient buffer, so a
    # deferred Dense dW would be pushed before it exists
    return isinstance(st, ParameterServerStrategy) and not comm.distributed()


def _var_model(v):
    m = getattr(v, "model", None)
    if m is None:
        raise TypeError(f"apply_gradients: {v!r} is not a model variable (model.trainable_variables)")
    return m


def apply_gradients(optimizer, grads_and_vars) -> None:
    gv = [(g, v) for g, v in grads_and_vars if g is not None]  # TF skips variables without a gradient
    if not gv:
        return
    model = _var_model(gv[0][1])
    from ..distribute import current_strategy

    st = getattr(model, "strategy", None) or current_strategy()
    ready = getattr(model, "_tape_ready", None)
    model._tape_ready = None
    params = [_param_of(v) for _, v in gv]
    subset = {id(p) for p in params} != {id(p) for p in model.store.params}
    ok = bool(ready) and not subset and _overlap_ok(optimizer, gv, ready)
    if not ok:
        flush_lazy(model)  # the update below reads every gradient from the flat buffer
        _stage_grads(gv)
    if subset:
        # only the listed variables move (and only their optimizer slots)
        if st is not None and (getattr(st, "world_size", 1) > 1 or st.in_round()):
            raise NotImplementedError("apply_gradients on a subset of the variables under a distribution "
                                      "strategy's collective update")
        if not hasattr(optimizer, "build"):
            raise NotImplementedError(f"apply_gradients on a subset of the variables with {type(optimizer).__name__}")
        optimizer.build(model.store)
        if getattr(optimizer, "dev_state", None) is not None:
            from ..ops import nn as K

            K.adam_step(optimizer.dev_state, optimizer.learning_rate, optimizer.beta_1, optimizer.beta_2)
        for lo, hi in _ranges(params):
            optimizer.apply(model.store, lo=lo, hi=hi, advance=False)
        optimizer.iterations += 1
        model._pending_grads = False
        return
    if st is not None:
        # a one-worker ParameterServerStrategy applies the update itself (possibly at round commit)
        # and takes the overlapped form from here (ps.py _apply_local)
        model._tape_overlap = ready if ok else None
        st.finish_gradients(model)
        st.apply_update(model, optimizer)
    elif ok:
        _apply_overlapped(optimizer, model.store, ready, model)
    else:
        optimizer.apply(model.store)
    model._pending_grads = False


def _stage_grads(gv) -> None:
    """Gradients the caller replaced (clipped, scaled, computed elsewhere) go into the flat gradient
    buffer the fused update reads; the tape's own buffers are already there."""
    for g, v in gv:
        p = _param_of(v)
        if g is p.grad:
            continue
        if not isinstance(g, torch.Tensor):
            g = torch.as_tensor(g, dtype=torch.float32)
        with torch._C.DisableTorchFunctionSubclass():
            same = g.device == p.grad.device and g.data_ptr() == p.grad.data_ptr() and g.numel() == p.grad.numel()
            if not same:
                if g.numel() != p.grad.numel():
                    raise ValueError(f"apply_gradients: gradient of {p.name!r} has {g.numel()} elements, "
                                     f"the variable {p.grad.numel()}")
                p.grad.copy_(g.reshape(p.grad.shape))


def _ranges(params) -> list:
    out: list = []
    for a, b in sorted((p.offset, p.offset + p.numel) for p in params):
        if out and a <= out[-1][1]:
            out[-1] = (out[-1][0], max(out[-1][1], b))
        else:
            out.append((a, b))
    return out


_AUX: dict = {}


def _overlap_ok(optimizer, gv, ready) -> bool:
    """The gradients handed in are the tape's own buffers, untouched (no clipping / scaling in
    between: a deferred Dense gradient that something has read counts as touched), and the
    optimizer is plain flat Adam with a host-side step counter."""
    from .optimizers import Adam

    if not (OVERLAP and type(optimizer) is Adam and getattr(optimizer, "dev_state", None) is None):
        return False
    lazy = {id(r[3].param): r[3] for r in ready if r[3] is not None}
    for g, v in gv:
        p = getattr(v, "param", None)
        if p is None:
            return False
        d = lazy.get(id(p))
        if d is None:
            if g is not p.grad:
                return False
        elif g is not d.view or not d.pending:
            return False
    return True


def _apply_overlapped(optimizer, store, ready, model=None) -> None:
    """Adam over the big Dense ranges on an auxiliary stream, each waiting only for its layer's dW
    (so the HBM-bound update overlaps the rest of the backward), then the remaining gaps on the
    step's stream, which joins the auxiliary stream before returning."""
    dev = store.flat.device
    step = optimizer.iterations + 1
    if dev.type != "cuda":  # CPU: the same update, in order
        optimizer.build(store)
        _update_ranges(optimizer, store, ready, step)
        if model is not None:
            model._lazy_dw = None
        store.grad_clean = True
        optimizer.iterations = step
        return
    aux = _AUX.get(dev)
    if aux is None:
        aux = _AUX[dev] = torch.cuda.Stream(device=dev)
    cur = torch.cuda.current_stream(dev)
    # aux deliberately does not wait for the step's stream: each range's event already follows
    # everything that reads or writes that range before its update (this step's forward and dX
    # read the bf16 weights before the dW fork; the previous update was joined into the step's
    # stream).  The gradients of those ranges are cleared by the update, so code that reads them
    # between gradient() and apply_gradients() must turn this off (PTG_TAPE_OVERLAP=0).
    # a fresh optimizer allocates and zero-fills its moments HERE, on the step's stream; the aux
    # stream must not read them before that fill (it otherwise never waits for the step's stream)
    before = optimizer.m
    optimizer.build(store)
    if optimizer.m is not before:
        aux.wait_stream(cur)
    with torch.cuda.stream(aux):
        for lo, hi, ev, lazy in ready:
            ev = lazy.ev if lazy is not None else ev
            if ev is not None:
                aux.wait_event(ev)
            _update_range(optimizer, store, lo, hi, lazy, step)
    _update_gaps(optimizer, store, ready)
    cur.wait_stream(aux)
    if model is not None:
        model._lazy_dw = None
    store.grad_clean = True
    optimizer.iterations = step


def _update_range(optimizer, store, lo, hi, lazy, step) -> None:
    if lazy is not None and lazy.pending:
        lazy.fused_adam(optimizer, store, step)  # dW never stored: Adam in the GEMM epilogue
    else:
        optimizer.apply(store, lo=lo, hi=hi, advance=False)


def _update_gaps(optimizer, store, ready) -> None:
    lo = 0
    for a, b in sorted((r[0], r[1]) for r in ready) + [(store.total, store.total)]:
        if a > lo:
            optimizer.apply(store, lo=lo, hi=a, advance=False)
        lo = max(lo, b)


def _update_ranges(optimizer, store, ready, step) -> None:
    for lo, hi, _, lazy in ready:
        _update_range(optimizer, store, lo, hi, lazy, step)
    _update_gaps(optimizer, store, ready)
