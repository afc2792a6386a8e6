"""``Sequential`` model with the Keras surface the reference uses (train_tf_ps.py:328-378, :651-679,
:773-814): ``compile / fit / evaluate / predict / summary / save``, History dicts, plus
``train_on_batch`` and GradientTape-style custom loops (:mod:`.tape`).

A training step is: zero the (accumulated) gradient ranges -> fused forward ops -> fused
loss kernel (output gradient + metric sums) -> fused backward ops (the active distribution
strategy gets a callback as each op's gradients complete, to launch bucketed RCCL collectives
while the rest of backward runs) -> strategy gradient sync -> ONE fused Adam launch (or the
strategy's sharded update).  Host syncs happen only at epoch boundaries (metric readout).
"""
from __future__ import annotations

import contextlib
import json
import math
import os
import sys
import time
import zipfile

import numpy as np
import torch

from ..ops import nn as K
from ..runtime import fault as _fault
from ..runtime import heartbeat as _heartbeat
from . import engine as E
from . import streams as S
from . import layers as L
from . import losses as LS
from . import metrics as MT
from . import optimizers as OPT
from .params import ParamStore
from .. import config

# Adam fused into the weight-gradient GEMM of big Dense layers on one replica (gemm.hip EpiAdam):
# the 168 MB CNN-B1 Dense kernel gradient is never written or re-read.  PTG_FUSED_ADAM=0 disables.
FUSED_ADAM = config.get("fused_adam")
DEVICE_FEED = config.get("device_feed")
FUSED_HEAD = config.get("fused_head")
FLIP_IN_ADAM = config.get("flip_in_adam")
# A model that is only a small Dense stack (the reference's CSV MLP) trains one whole step per launch
# (mlp.hip): forward, loss, backward and Adam in one workgroup, everything in LDS.
MLP_FUSED = config.get("mlp_fused")


def default_device() -> torch.device:
    from ..distribute import current_strategy

    st = current_strategy()
    if st is not None:
        return st.device
    if torch.cuda.is_available():
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


class History:
    def __init__(self):
        self.history: dict = {}
        self.epoch: list = []


class Variable:
    """Handle on one parameter of the flat store (what ``model.trainable_variables`` returns)."""

    def __init__(self, param, model=None):
        self.param = param
        self.model = model
        self.name = param.name

    @property
    def shape(self):
        return self.param.shape

    def numpy(self):
        return self.param.data.detach().cpu().numpy()

    def assign(self, value):
        self.param.data.copy_(torch.as_tensor(value, dtype=torch.float32))


class Sequential:
    def __init__(self, layers=None, name: str = "sequential"):
        self.name = name
        self._layers: list = []
        self.input_shape = None
        self.built = False
        self.store: ParamStore | None = None
        self.ops: list = []
        self.ws = E.Workspace()
        self.optimizer = None
        self.loss = None
        self.metric_names: list = []
        self.device = None
        self._stats = None
        self._eval_stats = None
        self.stop_training = False
        self.strategy = None
        for l in layers or []:
            self.add(l)

    # ---------------------------------------------------------------- structure
    def add(self, layer) -> None:
        if isinstance(layer, L.Input):
            self.input_shape = layer.shape
        self._layers.append(layer)

    @property
    def layers(self):
        return [l for l in self._layers if not isinstance(l, L.Input)]

    def build(self, input_shape=None, device=None, seed: int | None = None) -> None:
        if self.built:
            return
        if input_shape is not None:
            self.input_shape = tuple(int(s) for s in (input_shape[1:] if input_shape[0] is None else input_shape))
        if self.input_shape is None:
            raise ValueError("Sequential needs an Input layer or build(input_shape)")
        self.device = torch.device(device) if device is not None else default_device()
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.store = ParamStore()
        shape = self.input_shape
        for l in self.layers:
            shape = l.build(shape, self.store)
        self.output_shape = shape
        if seed is None:
            seed = config.get("seed")
        self.store.finalize(self.device, seed=seed)
        self.ops = E.lower(self._layers)
        self.store.update_zero_ranges()
        self.built = True
        from ..distribute import current_strategy

        st = current_strategy()
        if st is not None:
            st.register_model(self)

    def count_params(self) -> int:
        return self.store.num_params() if self.store else 0

    @property
    def trainable_variables(self):
        return [Variable(p, self) for l in self.layers for p in l.params]

    weights = trainable_variables

    @property
    def losses(self):
        return []  # no regularizers (reference: `model.losses` is empty, train_tf_ps.py:624)

    def get_weights(self):
        self._check_master()
        return [w for l in self.layers for w in l.keras_weights()]

    def set_weights(self, ws):
        i = 0
        for l in self.layers:
            n = len(l.keras_weights())
            if n:
                l.set_keras_weights(ws[i:i + n])
                i += n
        self.store.refresh_bf16()

    # ---------------------------------------------------------------- compile
    def compile(self, optimizer="adam", loss=None, metrics=None, jit_compile=None, steps_per_execution: int = 1) -> None:
        """``jit_compile=True`` (or env PTG_HIP_GRAPH=1) captures the whole training step - forward,
        loss, backward, optimizer - into one HIP graph after two eager warm-up steps and replays it
        (single-GPU training; multi-rank strategies stay eager because their collectives are
        launched from host hooks)."""
        if jit_compile is None:
            jit_compile = config.get("hip_graph")
        self.jit_compile = bool(jit_compile)
        # Keras' steps_per_execution: batches run per device launch where the step allows it (the
        # fused small-MLP step: fit() hands it this many consecutive batches of a column dataset)
        self.steps_per_execution = max(1, int(steps_per_execution))
        self._graphs = {}
        self._graph_warm = {}
        self.optimizer = OPT.get(optimizer)
        self.loss = LS.get(loss) if loss is not None else None
        self.metric_names = [MT.canonical_name(m) for m in (metrics or [])]
        if not self.built and self.input_shape is not None:
            self.build()
        self._configure_loss()

    def _configure_loss(self):
        if not self.built or self.loss is None:
            return
        last = self._last_op()
        if isinstance(self.loss, LS.SparseCategoricalCrossentropy) and isinstance(last, E.DenseOp):
            # softmax is folded into the fused softmax-crossentropy kernel
            last.logits_only = last.act == "softmax" or self.loss.from_logits

    # ---------------------------------------------------------------- execution plan hooks
    def _run_forward(self, xb, training: bool):
        if getattr(self, "_lazy_dw", None):
            from .tape import flush_lazy

            flush_lazy(self)  # a deferred tape dW still reads this workspace
        return E.run_forward(self.ops, xb, self.ws, training, pre_op=self._pre_op_hook())

    def _pre_op_hook(self):
        """Per-op forward hook of the sharded data-parallel update (waits for the op's parameter
        all-gather right before the op runs); None when the model is not sharded."""
        if getattr(self, "_shard_plan", None) is None:
            return None
        st = self.strategy
        return lambda op: st.before_forward_op(self, op)

    def _sync_master(self) -> None:
        """Collective: make the fp32 master weights current on every rank (sharded update)."""
        st = getattr(self, "strategy", None)
        if st is not None and hasattr(st, "synchronize_master"):
            st.synchronize_master(self)

    def _check_master(self) -> None:
        if getattr(self.store, "master_stale", False):
            raise RuntimeError("after sharded data-parallel steps only this rank's slice of the fp32 master "
                               "weights is current: call strategy.synchronize_master(model) on every rank "
                               "first (fit() and train_on_batch() do it for you)")

    def _run_backward(self, dpred, on_op_done=None):
        return E.run_backward(self.ops, dpred, self.ws, on_op_done=on_op_done, flips_ready=self._flips_ready())

    def _flips_ready(self) -> frozenset:
        """Conv ops whose flipped dgrad filter the last update wrote from the current weights."""
        st, opt = self.store, getattr(self, "optimizer", None)
        if opt is None or st.flip_token is None or st.flip_token != (id(opt), opt.iterations):
            return frozenset()
        return st.flip_names

    def _last_op(self):
        return self.ops[-1]

    def first_op(self):
        return self.ops[0]

    # ---------------------------------------------------------------- device helpers
    def _to_device(self, a, dtype=None):
        if isinstance(a, torch.Tensor):
            t = a
        else:
            a = np.asarray(a)
            t = torch.from_numpy(np.ascontiguousarray(a))
        if dtype is not None and t.dtype != dtype:
            t = t.to(dtype)
        if t.device != self.device:
            if t.device.type == "cpu" and self.device.type == "cuda":
                t = t.pin_memory().to(self.device, non_blocking=True)
            else:
                t = t.to(self.device)
        return t

    def _x_dtype(self, x):
        if isinstance(x, torch.Tensor):
            return None if x.dtype in (torch.uint8, torch.bfloat16, torch.float32) else torch.float32
        a = np.asarray(x)
        return None if a.dtype in (np.uint8, np.float32) else torch.float32

    def _prep_batch(self, x, y):
        xb = self._to_device(x, self._x_dtype(x))
        yb = None
        if y is not None:
            if isinstance(self.loss, LS.SparseCategoricalCrossentropy):
                yb = self._to_device(y, torch.int32).view(-1)
            else:
                yb = self._to_device(y, torch.float32)
                if yb.dim() == 1:
                    yb = yb.view(-1, 1)
        return xb, yb

    def _stats_buf(self, which="train"):
        if which == "train":
            if self._stats is None or self._stats.device != self.device:
                self._stats = K.zeros(8, torch.float32, self.device)
            return self._stats
        if self._eval_stats is None or self._eval_stats.device != self.device:
            self._eval_stats = K.zeros(8, torch.float32, self.device)
        return self._eval_stats

    # ---------------------------------------------------------------- forward / loss / step
    def __call__(self, x, training: bool = False):
        if not self.built:
            self.build()
        xb = self._to_device(x, self._x_dtype(x))
        from .tape import _active_tape

        tape = _active_tape()
        if tape is not None and training and self._tape_head_ok():
            out = self._tape_head_forward(xb)
            tape.record_forward(self, out)
            return out
        out = self._run_forward(xb, training)
        if tape is not None:
            tape.record_forward(self, out)
        if isinstance(self._last_op(), E.DenseOp) and self._last_op().logits_only:
            out = torch.softmax(out.float(), -1)
            if tape is not None:
                tape.ret = out  # the probabilities handed to the caller stand for this forward too
        return out

    def _loss_grad(self, out, yb, stats, gscale=1.0):
        dev = out.device
        pred = out if out.dtype == torch.float32 else out.float()
        dpred = self.ws.get("__dpred", pred.shape, torch.float32, dev)
        if isinstance(self.loss, LS.MeanSquaredError):
            K.mse(pred.contiguous(), yb, dpred, stats, gscale)
        elif isinstance(self.loss, LS.SparseCategoricalCrossentropy):
            K.softmax_xent(pred.contiguous(), yb, dpred, stats, gscale)
        else:
            raise ValueError(f"unsupported loss {self.loss}")
        return dpred

    def _strategy(self):
        if getattr(self, "strategy", None) is not None:
            return self.strategy
        from ..distribute import current_strategy

        return current_strategy()

    def backward_and_update(self, dpred, strategy=None) -> None:
        """Backward from d(loss)/d(output) + gradient sync + optimizer update."""
        st = strategy
        fused = self._begin_fused_update(st)
        if fused is not None:
            # one local replica: big Dense layers apply Adam in their weight-gradient epilogue,
            # the rest of the flat store gets the usual fused Adam pass afterwards
            try:
                with S.active(S.for_step(self.store, st)):
                    self._run_backward(dpred)
            finally:
                for op in self._fusable_ops:
                    op.fused_update = None
            self.optimizer.finish_fused(fused)
            return
        hook = st.on_op_grads_ready if st is not None else None
        with S.active(S.for_step(self.store, st)):  # joined before the gradient sync / update
            self._run_backward(dpred, on_op_done=(lambda op: hook(self, op)) if hook else None)
        if st is not None:
            st.finish_gradients(self)
            st.apply_update(self)
        else:
            self.optimizer.apply(self.store)

    def _begin_fused_update(self, st):
        """FusedAdamStep when this step can update big Dense kernels inside their wgrad GEMM: Adam,
        one replica (no gradient collective between backward and update), GPU, PTG_FUSED_ADAM != 0."""
        if not FUSED_ADAM or not isinstance(self.optimizer, OPT.Adam) or not self.store.flat.is_cuda:
            return None
        if st is not None and (st.dp_degree != 1 or getattr(st, "sharded_update", False)):
            return None
        all_ops = getattr(self, "ops", None) or []
        if getattr(self, "_fusable_key", None) is not all_ops:
            self._fusable_key = all_ops
            self._fusable_ops = [op for op in all_ops if isinstance(op, E.DenseOp) and op.big]
        ops = self._fusable_ops
        if not ops:
            return None
        ctx = self.optimizer.begin_fused(self.store)
        for op in ops:
            op.fused_update = ctx
        if FLIP_IN_ADAM:
            for op in all_ops:
                spec = op.flip_spec() if isinstance(op, E.ConvOp) else None
                if spec is not None:
                    ctx.flips.append((op.name, spec))
        return ctx

    def _head_fusable(self, xb, st) -> bool:
        """[..., Dense(relu, big), Dense(N <= 4, linear)] + MSE on the GPU: the head runs as two fused
        kernels (head_row_k + head_col_k) instead of seven small ones, on one replica or under a
        data-parallel strategy (its gradient hooks fire for the two Dense ops as usual)."""
        if not FUSED_HEAD or not xb.is_cuda:
            return False
        if st is not None and st.world_size != 1 and not hasattr(st, "on_op_grads_ready"):
            return False
        return isinstance(self.loss, LS.MeanSquaredError) and self._head_ops_ok()

    def _head_ops_ok(self) -> bool:
        ops = getattr(self, "ops", None) or []
        if len(ops) < 3:
            return False
        d1, d2 = ops[-2], ops[-1]
        return (isinstance(d1, E.DenseOp) and isinstance(d2, E.DenseOp) and d1.big and not d2.big
                and d1.act == "relu" and d2.act in (None, "linear") and d1.dense.bias is not None
                and d2.dense.bias is not None and d2.dense.units <= 4 and not d1.first)

    def _tape_head_ok(self) -> bool:
        """A GradientTape forward on one local replica whose tail the fused head covers (the loss is
        only known when the loss object is called: nn/tape.py _HeadPred)."""
        from . import tape as T

        if not (T.TAPE_HEAD and FUSED_HEAD and self._head_ops_ok()):
            return False
        st = self._strategy()
        return st is None or getattr(st, "world_size", 2) == 1

    def _tape_head_forward(self, xb):
        from .tape import _HeadPred, _HeadState, flush_lazy

        if getattr(self, "_lazy_dw", None):
            flush_lazy(self)
        self._drop_pending_head()
        d1, d2 = self.ops[-2], self.ops[-1]
        x = E.run_forward(self.ops[:-2], xb, self.ws, True, pre_op=self._pre_op_hook())
        acc = d1.forward_splitk_sums(x, self.ws)
        pred = self.ws.get(d2.name + "/tapepred", (acc.shape[-2], d2.dense.units), torch.float32, acc.device)
        out = pred.as_subclass(_HeadPred)
        out._lz = self._head_state = _HeadState(self, acc, pred)
        return out

    def _drop_pending_head(self) -> None:
        """A tape prediction still held at the split-K sums (its loss never ran) is abandoned: clear
        the sums so the next big-Dense forward does not add onto them."""
        prev = getattr(self, "_head_state", None)
        if prev is not None:
            prev.discard()
            self._head_state = None

    def _train_step_fused_head(self, xb, yb, stats, st) -> None:
        self._drop_pending_head()
        d1, d2 = self.ops[-2], self.ops[-1]
        pre = self._pre_op_hook()
        x = E.run_forward(self.ops[:-2], xb, self.ws, True, pre_op=pre)
        if pre is not None:  # sharded update: the two Dense ops' parameter all-gathers
            pre(d1)
            pre(d2)
        acc = d1.forward_splitk_sums(x, self.ws)
        B, K1 = acc.shape[-2:]
        dz1 = self.ws.get(d1.name + "/dz", (B, K1), torch.bfloat16, acc.device)
        N2 = d2.dense.units
        scratch = self.ws.get(d1.name + "/headscratch", (B * (N2 + 2),), torch.float32, acc.device)
        K.head_mse(acc, d1.dense.bias.data, d2.dense.kernel.data, d2.dense.bias.data, yb.contiguous(), dz1,
                   d2.dense.kernel.grad, d2.dense.bias.grad, d1.dense.bias.grad, stats, scratch=scratch)
        hook = st.on_op_grads_ready if st is not None else None
        fused = self._begin_fused_update(st)
        try:
            with S.active(S.for_step(self.store, st)):
                if hook is not None:
                    hook(self, d2)  # Dense2 weights/bias and Dense1 bias gradients exist now
                dx = d1.backward_dz(dz1, self.ws)
                if hook is not None:
                    hook(self, d1)
                E.run_backward(self.ops[:-2], dx, self.ws, on_op_done=(lambda op: hook(self, op)) if hook else None,
                               flips_ready=self._flips_ready())
        finally:
            for op in getattr(self, "_fusable_ops", []):
                op.fused_update = None
        if fused is not None:
            self.optimizer.finish_fused(fused)
        elif st is not None:
            st.finish_gradients(self)
            st.apply_update(self)
        else:
            self.optimizer.apply(self.store)

    # ---------------------------------------------------------------- fused small-MLP step
    def _mlp_plan(self, st):
        """(dims, acts, woffs, boffs, loss kind) when the whole model is a small Dense stack that the
        one-launch training step (mlp.hip) covers, else None.  Cached per (ops, loss)."""
        key = (id(self.ops), id(self.loss), id(self.optimizer))
        if getattr(self, "_mlp_key", None) != key:
            self._mlp_key = key
            self._mlp_cached = self._build_mlp_plan()
        plan = self._mlp_cached
        if plan is None:
            return None
        if st is not None and (st.world_size != 1 or st.dp_degree != 1 or getattr(st, "sharded_update", False)
                               or st.in_round() or hasattr(st, "variable_partitioner")):
            return None
        return plan

    def _build_mlp_plan(self):
        if not MLP_FUSED or not self.ops or self.device is None or self.device.type != "cuda":
            return None
        opt = self.optimizer
        if type(opt) is not OPT.Adam or getattr(opt, "dev_state", None) is not None:
            return None
        if not all(isinstance(op, E.DenseOp) for op in self.ops) or len(self.ops) > 6:
            return None
        last = self.ops[-1]
        if isinstance(self.loss, LS.SparseCategoricalCrossentropy) and last.act == "softmax" and last.logits_only:
            kind = 0
        elif isinstance(self.loss, LS.MeanSquaredError) and last.act in (None, "linear"):
            kind = 1
        else:
            return None
        acts = []
        for op in self.ops[:-1]:
            if op.act not in (None, "linear", "relu"):
                return None
            acts.append(1 if op.act == "relu" else 0)
        acts.append(0)
        dims = [self.ops[0].dense.fan_in] + [op.dense.units for op in self.ops]
        woffs = [op.dense.kernel.offset for op in self.ops]
        boffs = [op.dense.bias.offset if op.dense.bias is not None else -1 for op in self.ops]
        if max(w + dims[l + 1] * dims[l] for l, w in enumerate(woffs)) > self.store.total:
            return None
        return dims, acts, woffs, boffs, kind, K.mlp_desc(dims, acts, woffs, boffs)

    def _mlp_fit_plan(self, x, y, st):
        """(iterator factory over (batch group, batches), MLP plan) when fit() can feed the fused
        MLP step groups of batches from a device-resident column dataset, else None."""
        from ..data.dataset import Dataset

        if self.device is None or self.device.type != "cuda" or getattr(self, "jit_compile", False):
            return None
        plan = self._mlp_plan(st)
        if plan is None:
            return None
        if isinstance(x, Dataset):
            cp = getattr(x, "_plan", None)
            if cp is None or "batch" not in cp.names():
                return None
        elif isinstance(x, (np.ndarray, torch.Tensor)) and y is not None:
            return None  # array inputs keep the per-batch path (its shuffle order is _iter_batches')
        else:
            return None
        if sum(int(np.prod(getattr(a, "shape", (0,)))) * 4 for a in cp.arrays) > (1 << 30):
            return None  # large datasets stay host-resident
        dev_plans = getattr(self, "_dev_plans", None)
        if dev_plans is None:
            dev_plans = self._dev_plans = {}
        key = id(cp)
        dp = dev_plans.get(key)
        if dp is None or dp[0] is not cp:
            dp = dev_plans[key] = (cp, cp.on_device(self.device))
        group = self.steps_per_execution if getattr(self, "steps_per_execution", 1) > 1 else 64
        return (lambda: dp[1].iter_groups(group, with_count=True)), plan

    def _mlp_fusable(self, xb, yb, st):
        if xb.dtype != torch.float32 or not xb.is_cuda or xb.dim() != 2:
            return None
        plan = self._mlp_plan(st)
        if plan is None or xb.shape[1] != plan[0][0]:
            return None
        B = xb.shape[0]
        ok = getattr(self, "_mlp_lds_ok", None)
        if ok is None:
            ok = self._mlp_lds_ok = {}
        if B not in ok:
            ok[B] = 0 < K.mlp_lds_bytes(plan[0], B) <= 160 * 1024
        return plan if ok[B] else None

    def _train_step_mlp(self, xb, yb, stats, plan, steps: int = 1) -> None:
        dims, acts, woffs, boffs, kind, desc = plan
        opt, store = self.optimizer, self.store
        opt.build(store)
        if not getattr(store, "grad_clean", False):
            store.zero_grad()  # (the fused step writes no gradient; leave the buffer clean)
        y = yb.view(-1).contiguous() if kind == 0 else yb.contiguous()
        x = xb.contiguous()
        if x.is_cuda and x.dtype == torch.float32 and y.dtype == (torch.int32 if kind == 0 else torch.float32):
            B = x.shape[0] // steps
            key = (id(plan), B, store.flat.data_ptr(), opt.m.data_ptr(), opt.v.data_ptr(), stats.data_ptr(),
                   opt.learning_rate, opt.beta_1, opt.beta_2, opt.epsilon)
            ms = self._mlp_steps.get(key) if hasattr(self, "_mlp_steps") else None
            if ms is None:
                if not hasattr(self, "_mlp_steps") or len(self._mlp_steps) > 8:
                    self._mlp_steps = {}
                ms = self._mlp_steps[key] = K.MlpStep(store.flat, opt.m, opt.v, store.flat_bf16, stats, dims, acts,
                                                      woffs, boffs, B, kind, opt.learning_rate, opt.beta_1,
                                                      opt.beta_2, opt.epsilon, opt.iterations, desc=desc)
            ms.run(x, y, steps, opt.iterations)
        else:
            K.mlp_train(x, y, store.flat, opt.m, opt.v, store.flat_bf16, stats, dims, acts, woffs, boffs, steps, kind,
                        opt.learning_rate, opt.beta_1, opt.beta_2, opt.epsilon, opt.iterations, desc=desc)
        opt.iterations += steps
        store.grad_clean = True

    def train_step(self, xb, yb, stats=None) -> None:
        _fault.maybe_fail()
        _heartbeat.progress()
        st = self._strategy()
        stats = self._stats_buf() if stats is None else stats
        plan = self._mlp_fusable(xb, yb, st)
        if plan is not None:
            return self._train_step_mlp(xb, yb, stats, plan)
        if self._head_fusable(xb, st):
            self.store.zero_grad()
            return self._train_step_fused_head(xb, yb, stats, st)
        self.store.zero_grad()
        out = self._run_forward(xb, True)
        dpred = self._loss_grad(out, yb, stats)
        self.backward_and_update(dpred, st)

    # ---------------------------------------------------------------- HIP-graph step
    def _graph_usable(self, xb) -> bool:
        if not getattr(self, "jit_compile", False) or not xb.is_cuda:
            return False
        st = self._strategy()
        return st is None or st.dp_degree == 1

    def train_step_fast(self, xb, yb, stats=None) -> None:
        """One training step; replays a captured HIP graph when ``jit_compile`` is on (same batch
        shape/dtype as the captured step), otherwise runs eagerly."""
        stats = self._stats_buf() if stats is None else stats
        if not self._graph_usable(xb):
            return self.train_step(xb, yb, stats)
        key = (tuple(xb.shape), xb.dtype, tuple(yb.shape), yb.dtype, stats.data_ptr())
        ent = self._graphs.get(key)
        if ent is None:
            n = self._graph_warm.get(key, 0)
            if n < 2:  # eager warm-up: kernels selected, workspace buffers allocated
                self._graph_warm[key] = n + 1
                return self.train_step(xb, yb, stats)
            self.optimizer.use_device_step(self.store)
            sx, sy = xb.clone(), yb.clone()
            torch.cuda.synchronize(xb.device)
            graph = torch.cuda.CUDAGraph()
            it0 = self.optimizer.iterations
            with torch.cuda.graph(graph):
                self.train_step(sx, sy, stats)  # recorded, not executed
            self.optimizer.iterations = it0
            ent = self._graphs[key] = (graph, sx, sy)
        graph, sx, sy = ent
        sx.copy_(xb, non_blocking=True)
        sy.copy_(yb, non_blocking=True)
        graph.replay()
        self.optimizer.iterations += 1

    def train_on_batch(self, x, y, return_dict: bool = False):
        xb, yb = self._prep_batch(x, y)
        stats = self._stats_buf()
        K.fill_(stats, 0.0)
        self.train_step(xb, yb, stats)
        self._sync_master()
        logs = self._logs_from(stats)
        return logs if return_dict else [logs["loss"]] + [logs[m] for m in self.metric_names if m in logs]

    def test_step(self, xb, yb, stats) -> None:
        out = self._run_forward(xb, False)
        self._loss_grad(out, yb, stats)

    # ---------------------------------------------------------------- logs
    def _logs_from(self, stats, prefix="") -> dict:
        s = stats.detach()
        st = self._strategy()
        if st is not None and st.world_size > 1:
            s = st.all_reduce_sum(s.clone())
        s = s.double().cpu().numpy()
        logs = {}
        nsamp = max(s[4], 1.0)
        logs[prefix + "loss"] = float(s[0] / nsamp)
        for m in self.metric_names:
            if m == "accuracy":
                logs[prefix + "accuracy"] = float(s[1] / nsamp)
            elif m == "mae":
                logs[prefix + "mae"] = float(s[1] / max(s[3], 1.0))
            elif m == "mse":
                logs[prefix + "mse"] = float(s[2] / max(s[3], 1.0))
        return logs

    # ---------------------------------------------------------------- fit / evaluate / predict
    def _iter_batches(self, x, y, batch_size, shuffle, seed=None):
        from ..data.dataset import Dataset

        if isinstance(x, Dataset) or hasattr(x, "__iter__") and not isinstance(x, (np.ndarray, torch.Tensor)):
            if (self.device.type == "cuda" and DEVICE_FEED and isinstance(x, Dataset)
                    and getattr(x, "_plan", None) is None and not getattr(x, "_on_device", False)):
                # host batches (decoded images, CSV rows): pinned ring + side-stream H2D, overlapped
                # with the train step (data/device_feed.py)
                from ..data.device_feed import DeviceFeeder

                return DeviceFeeder(x, self.device)
            return iter(x)
        n = len(x)
        bs = batch_size or 32
        idx = np.arange(n)
        if shuffle:
            np.random.default_rng(seed).shuffle(idx)

        def gen():
            for i in range(0, n, bs):
                j = idx[i:i + bs]
                yield (x[j], None if y is None else y[j])

        return gen()

    def fit(self, x=None, y=None, batch_size=None, epochs: int = 1, verbose="auto", callbacks=None,
            validation_data=None, shuffle: bool = True, steps_per_epoch=None, validation_steps=None,
            initial_epoch: int = 0):
        if not self.built:
            self.build()
        if self.optimizer is None:
            raise RuntimeError("call compile() before fit()")
        verbose = 1 if verbose == "auto" else verbose
        st = self._strategy()
        is_chief = st is None or st.is_chief
        hist = History()
        callbacks = list(callbacks or [])
        for cb in callbacks:
            if hasattr(cb, "set_model"):
                cb.set_model(self)
            if hasattr(cb, "on_train_begin"):
                cb.on_train_begin()
            initial_epoch = max(initial_epoch, int(getattr(cb, "start_epoch", 0) or 0))
        persistent_it = None
        # the fused small-MLP step (mlp.hip) over a column dataset: the columns go to the device once
        # and fit() takes groups of consecutive full batches per launch (no per-batch callbacks exist,
        # so this changes nothing but the launch count; steps_per_execution sets the group size)
        mlp_group = self._mlp_fit_plan(x, y, st)
        if steps_per_epoch is not None:
            persistent_it = mlp_group[0]() if mlp_group else self._iter_batches(x, y, batch_size, shuffle)
        stash = None
        stats = self._stats_buf()
        for epoch in range(initial_epoch, epochs):
            if verbose and is_chief:
                print(f"Epoch {epoch + 1}/{epochs}", flush=True)
            K.fill_(stats, 0.0)
            t0 = time.perf_counter()
            if persistent_it is not None:
                it = persistent_it
            elif mlp_group:
                it = mlp_group[0]()
            else:
                it = self._iter_batches(x, y, batch_size, shuffle, seed=epoch)
            nsteps = 0
            while steps_per_epoch is None or nsteps < steps_per_epoch:
                if mlp_group:
                    if stash is not None:
                        (xb, yb, k), stash = stash, None
                    else:
                        try:
                            batch, k = next(it)
                        except StopIteration:
                            break
                        xb, yb = self._prep_batch(batch[0], batch[1])
                    if steps_per_epoch is not None and nsteps + k > steps_per_epoch:
                        k1 = steps_per_epoch - nsteps  # the rest of the group opens the next epoch
                        B = xb.shape[0] // k
                        stash = (xb[k1 * B:], yb[k1 * B:], k - k1)
                        xb, yb, k = xb[:k1 * B], yb[:k1 * B], k1
                    B = xb.shape[0] // k
                    self._last_batch = int(B)
                    if self._mlp_fusable(xb[:B], yb[:B], st) is not None:
                        for _ in range(k):  # fault injection counts every step of the group
                            _fault.maybe_fail()
                        _heartbeat.progress(k)
                        self._train_step_mlp(xb, yb, stats, mlp_group[1], steps=k)
                    else:
                        for j in range(k):
                            self.train_step_fast(xb[j * B:(j + 1) * B], yb[j * B:(j + 1) * B], stats)
                    nsteps += k
                    continue
                try:
                    batch = next(it)
                except StopIteration:
                    break
                xb, yb = self._prep_batch(batch[0], batch[1])
                self._last_batch = int(xb.shape[0])
                self.train_step_fast(xb, yb, stats)
                nsteps += 1
            logs = self._logs_from(stats)
            dt_train = time.perf_counter() - t0  # the logs readback synchronised the device
            self._sync_master()  # every rank is here: the full fp32 master for callbacks / saving
            if validation_data is not None:
                vlogs = self.evaluate(*(validation_data if isinstance(validation_data, tuple) else (validation_data,)),
                                      batch_size=batch_size, steps=validation_steps, verbose=0, return_dict=True,
                                      _prefix="val_")
                logs.update(vlogs)
            dt = time.perf_counter() - t0
            for k_, v_ in logs.items():
                hist.history.setdefault(k_, []).append(v_)
            hist.epoch.append(epoch)
            if verbose and is_chief:
                per = dt / max(nsteps, 1)
                body = " - ".join(f"{k_}: {v_:.4f}" for k_, v_ in sorted(logs.items()))
                bs = getattr(self, "_last_batch", 0)
                rate = f" - {bs * nsteps / max(dt_train, 1e-9):.0f} samples/s (train)" if bs else ""
                print(f"{nsteps}/{nsteps} - {dt:.0f}s {per * 1e3:.0f}ms/step{rate} - {body}", flush=True)
            for cb in callbacks:
                if hasattr(cb, "on_epoch_end"):
                    cb.on_epoch_end(epoch, logs)
            if self.stop_training:
                break
        for cb in callbacks:
            if hasattr(cb, "on_train_end"):
                cb.on_train_end()
        self.history = hist
        return hist

    def evaluate(self, x=None, y=None, batch_size=None, steps=None, verbose="auto", return_dict=False,
                 _prefix=""):
        stats = self._stats_buf("eval")
        K.fill_(stats, 0.0)
        it = self._iter_batches(x, y, batch_size, False)
        n = 0
        while steps is None or n < steps:
            try:
                batch = next(it)
            except StopIteration:
                break
            xb, yb = self._prep_batch(batch[0], batch[1])
            self.test_step(xb, yb, stats)
            n += 1
        logs = self._logs_from(stats, prefix=_prefix)
        if return_dict:
            return logs
        vals = [logs[_prefix + "loss"]] + [logs[_prefix + m] for m in self.metric_names if _prefix + m in logs]
        return vals if len(vals) > 1 else vals[0]

    def predict(self, x, batch_size=None, verbose=0, steps=None):
        outs = []
        it = self._iter_batches(x, None, batch_size, False)
        n = 0
        for batch in it:
            xb = batch[0] if isinstance(batch, (tuple, list)) else batch
            outs.append(self(xb, training=False).float().cpu().numpy().copy())
            n += 1
            if steps is not None and n >= steps:
                break
        return np.concatenate(outs, 0) if outs else np.zeros((0,) + tuple(self.output_shape), np.float32)

    # ---------------------------------------------------------------- summary / save
    def summary(self, print_fn=None):
        pf = print_fn or print
        rows = []
        for l in self.layers:
            rows.append((f"{l.name} ({l.keras_class})", str((None, *l.out_shape)), f"{l.param_count():,}"))
        w = [max(31, max(len(r[0]) for r in rows) + 1), 22, 13]
        line = lambda a, b, c, d: a + b * (w[0] + 2) + c + b * (w[1] + 2) + c + b * (w[2] + 2) + d  # noqa: E731
        pf(f'Model: "{self.name}"')
        pf(line("┏", "━", "┳", "┓"))
        pf(f"┃ {'Layer (type)':<{w[0]}} ┃ {'Output Shape':<{w[1]}} ┃ {'Param #':>{w[2]}} ┃")
        pf(line("┡", "━", "╇", "┩"))
        for i, r in enumerate(rows):
            pf(f"│ {r[0]:<{w[0]}} │ {r[1]:<{w[1]}} │ {r[2]:>{w[2]}} │")
            pf(line("├", "─", "┼", "┤") if i + 1 < len(rows) else line("└", "─", "┴", "┘"))
        total = self.count_params()
        mb = total * 4 / 2 ** 20
        pf(f" Total params: {total:,} ({mb:.2f} MB)")
        pf(f" Trainable params: {total:,} ({mb:.2f} MB)")
        pf(" Non-trainable params: 0 (0.00 B)")

    def get_config(self) -> dict:
        layers = [{"class_name": "InputLayer",
                   "config": {"name": "input_layer", "batch_shape": [None, *self.input_shape], "dtype": "float32"}}]
        for l in self.layers:
            layers.append({"class_name": l.keras_class, "config": l.get_config()})
        return {"name": self.name, "layers": layers}

    def _save_class_name(self) -> str:
        return "Sequential"

    def export(self, filepath: str, assets: dict | None = None) -> str:
        """Keras-3 ``model.export``: write the SavedModel-layout directory (:mod:`.saved_model`)."""
        from . import saved_model

        return saved_model.save(self, filepath, assets=assets)

    def save(self, filepath: str) -> None:
        """Keras-v3-shaped zip: config.json + metadata.json + model.weights.safetensors (weights in Keras
        layouts, keyed ``layers/<name>/vars/<i>``; safetensors instead of HDF5 because h5py is absent)."""
        from safetensors.numpy import save as st_save

        st = self._strategy()
        if st is not None and not st.is_chief:
            return
        self._check_master()
        cfg = {"module": "pyspark_tf_gke_amd.nn", "class_name": self._save_class_name(), "config": self.get_config(),
               "compile_config": {"optimizer": self.optimizer.get_config() if self.optimizer else None,
                                  "loss": self.loss.name if self.loss else None, "metrics": self.metric_names}}
        meta = {"keras_version": "3-compatible", "framework": "pyspark_tf_gke_amd",
                "date_saved": time.strftime("%Y-%m-%d@%H:%M:%S"), "weights_format": "safetensors"}
        tensors = {}
        for l in self.layers:
            for i, w in enumerate(l.keras_weights()):
                tensors[f"layers/{l.name}/vars/{i}"] = np.ascontiguousarray(w.astype(np.float32))
        os.makedirs(os.path.dirname(os.path.abspath(filepath)) or ".", exist_ok=True)
        tmp = filepath + ".tmp"
        with zipfile.ZipFile(tmp, "w") as zf:
            zf.writestr("config.json", json.dumps(cfg, indent=2))
            zf.writestr("metadata.json", json.dumps(meta, indent=2))
            zf.writestr("model.weights.safetensors", st_save(tensors))
        os.replace(tmp, filepath)


def load_model(filepath: str, compile: bool = True, device=None) -> Sequential:
    from safetensors.numpy import load as st_load

    with zipfile.ZipFile(filepath) as zf:
        cfg = json.loads(zf.read("config.json"))
        tensors = st_load(zf.read("model.weights.safetensors"))
    if cfg.get("class_name") == "Functional":
        from .functional import model_from_config

        m = model_from_config(cfg["config"])
    else:
        L.reset_name_counters()
        m = Sequential(name=cfg["config"].get("name", "sequential"))
        for lc in cfg["config"]["layers"]:
            m.add(L.layer_from_config(lc["class_name"], lc["config"]))
    m.build(device=device)
    for l in m.layers:
        ws = []
        i = 0
        while f"layers/{l.name}/vars/{i}" in tensors:
            ws.append(tensors[f"layers/{l.name}/vars/{i}"])
            i += 1
        if ws:
            l.set_keras_weights(ws)
    m.store.refresh_bf16()
    cc = cfg.get("compile_config") or {}
    if compile and cc.get("loss"):
        opt = cc.get("optimizer") or {}
        m.compile(optimizer=OPT.Adam(learning_rate=opt.get("learning_rate", 1e-3)), loss=cc["loss"],
                  metrics=cc.get("metrics"))
    return m


_ = (math, sys)
