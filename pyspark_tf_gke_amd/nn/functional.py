"""Keras functional API (``Model(inputs, outputs)``) and its fused graph execution plan.

This is what the BASELINE.json ResNet-50 config needs beyond the reference's ``Sequential`` models
(train_tf_ps.py:328-378): a DAG of layers with residual ``Add`` joins and ``BatchNormalization``.

Lowering fuses the DAG into device ops (:mod:`.graph_ops`):

* ``Conv2D -> BatchNormalization [-> Add(residual)] [-> Activation('relu')]`` becomes ONE
  :class:`~.graph_ops.ConvBNOp`: MFMA conv (GEMM for 1x1, implicit GEMM / halo-tiled direct conv
  otherwise), a batch-statistics pass, and one apply pass that also adds the residual branch and
  applies the ReLU.  The residual ``Add`` is fused into whichever branch is computed *last*, so the
  other branch is already available.
* ``ZeroPadding2D`` is folded into the padding of the following conv or max-pool.
* everything else maps to the Sequential engine's ops (Dense, GAP, Flatten, PReLU...) or generic
  BN / Add / ReLU / MaxPool ops.

Backward walks the plan in reverse; a tensor consumed by several ops (a bottleneck block's input
feeds both the main branch and the shortcut) accumulates its gradient, preferably inside the
second producer's dgrad GEMM epilogue (``accumulate``) rather than with a separate add pass.
"""
from __future__ import annotations

import time

import numpy as np

from . import engine as E
from . import graph_ops as G
from . import layers as L
from .model import Sequential
from .params import ParamStore
from .. import config


class KerasTensor:
    """Symbolic output of a layer call (shape excludes the batch dimension)."""

    def __init__(self, shape, layer, inputs):
        self.shape = tuple(shape)
        self.layer = layer
        self.inputs = list(inputs)

    def __repr__(self):
        return f"<KerasTensor shape={(None, *self.shape)} from {self.layer.name}>"


def _as_tensor(t):
    return t.output if isinstance(t, L.Input) else t


def _topo(outputs) -> list:
    order, seen = [], set()

    def visit(t):
        if id(t) in seen:
            return
        seen.add(id(t))
        for i in t.inputs:
            visit(i)
        order.append(t)

    for o in outputs:
        visit(o)
    return order


class GraphPlan:
    """Fused op list in execution order over integer tensor ids (indices of the topo order)."""

    def __init__(self, nodes: list, input_idx: int, output_idx: int):
        self.nodes = nodes
        self.input_idx = input_idx
        self.output_idx = output_idx
        self.ops = _lower(nodes, input_idx)
        for op in self.ops:
            op.first = all(i == input_idx for i in op.inputs)

    def forward(self, x, ws, training, pre_op=None):
        vals = {self.input_idx: x}
        for op in self.ops:
            if pre_op is not None:
                pre_op(op)
            vals[op.output] = op.forward([vals[i] for i in op.inputs], ws, training)
        return vals[self.output_idx]

    def backward(self, dy, ws, on_op_done=None):
        from ..ops import bn as KB

        grads = {self.output_idx: dy}
        for op in reversed(self.ops):
            g = grads.pop(op.output, None)
            if g is None:
                continue
            existing = [grads.get(i) for i in op.inputs]
            res = op.backward(g, ws, existing)
            for i, gi, ex in zip(op.inputs, res, existing):
                if gi is None or i == self.input_idx:
                    continue
                if ex is None:
                    grads[i] = gi
                elif gi is not ex:
                    KB.add_(ex, gi, ex)
            if on_op_done is not None:
                on_op_done(op)
        return grads.get(self.input_idx)


def _lower(nodes: list, input_idx: int) -> list:
    idx = {id(t): k for k, t in enumerate(nodes)}
    consumers: dict = {k: [] for k in range(len(nodes))}
    for k, t in enumerate(nodes):
        for i in t.inputs:
            consumers[idx[id(i)]].append(k)

    def sole(k, cls):
        c = consumers[k]
        if len(c) == 1 and isinstance(nodes[c[0]].layer, cls):
            return c[0]
        return None

    alias: dict = {}  # folded node -> tensor id it forwards
    pad_of: dict = {}  # conv/pool node -> extra zero padding folded from a ZeroPadding2D producer
    claimed: set = set()
    ops = []

    def src(k):
        while k in alias:
            k = alias[k]
        return k

    for k, t in enumerate(nodes):
        if k == input_idx or k in claimed:
            continue
        layer = t.layer
        ins = [idx[id(i)] for i in t.inputs]
        if isinstance(layer, L.ZeroPadding2D):
            c = consumers[k]
            tgt = nodes[c[0]].layer if len(c) == 1 else None
            ok = (isinstance(tgt, L.Conv2D) and tgt.padding == "valid") or isinstance(tgt, L.MaxPooling2D)
            if not ok:
                raise NotImplementedError("ZeroPadding2D must feed a single 'valid' Conv2D or MaxPooling2D")
            alias[k] = ins[0]
            pad_of[c[0]] = pad_of.get(c[0], 0) + layer.pad
            continue
        if isinstance(layer, (L.Conv2D, L.BatchNormalization)):
            conv = layer if isinstance(layer, L.Conv2D) else None
            bn_k = sole(k, L.BatchNormalization) if conv is not None else k
            if conv is not None and bn_k is None:
                # Conv2D without BN: the Sequential engine's conv (+PReLU +pool) op
                prelu_k = sole(k, L.PReLU) if conv.activation in ("linear", None) else None
                last = prelu_k if prelu_k is not None else k
                pool_k = sole(last, L.MaxPooling2D)
                if pool_k is not None and nodes[pool_k].layer.pool_size != (2, 2):
                    pool_k = None
                if pad_of.get(k):
                    raise NotImplementedError("ZeroPadding2D before a Conv2D without BatchNormalization")
                inner = E.ConvOp(conv, nodes[prelu_k].layer if prelu_k is not None else None,
                                 nodes[pool_k].layer if pool_k is not None else None)
                out = pool_k if pool_k is not None else last
                for c in (prelu_k, pool_k):
                    if c is not None:
                        claimed.add(c)
                ops.append(G.Adapter(inner, [src(ins[0])], out))
                continue
            bn = nodes[bn_k].layer
            if bn_k != k:
                claimed.add(bn_k)
            end, relu, res = bn_k, False, None
            add_k = sole(bn_k, L.Add)
            if add_k is not None:
                other = [idx[id(i)] for i in nodes[add_k].inputs if idx[id(i)] != bn_k]
                if len(other) == 1 and src(other[0]) < k:
                    res = src(other[0])
                    end = add_k
                    claimed.add(add_k)
            act_k = sole(end, L.Activation)
            if act_k is not None and nodes[act_k].layer.activation == "relu":
                relu, end = True, act_k
                claimed.add(act_k)
            elif act_k is None:
                relu_k = sole(end, L.ReLU)
                if relu_k is not None:
                    relu, end = True, relu_k
                    claimed.add(relu_k)
            x_in = src(ins[0])
            if conv is not None:
                op = G.ConvBNOp(conv, bn, relu, res is not None, extra_pad=pad_of.get(k, 0))
            else:
                op = G.BNOp(bn, relu, res is not None)
            ops.append(G.GraphOp(op, [x_in] + ([res] if res is not None else []), end))
            continue
        if isinstance(layer, L.MaxPooling2D):
            ops.append(G.GraphOp(G.MaxPoolOp(layer, pad_of.get(k, 0)), [src(ins[0])], k))
            continue
        if isinstance(layer, L.Add):
            relu = False
            end = k
            act_k = sole(k, L.Activation)
            if act_k is not None and nodes[act_k].layer.activation == "relu":
                relu, end = True, act_k
                claimed.add(act_k)
            if len(ins) != 2:
                raise NotImplementedError("Add of exactly two tensors")
            ops.append(G.GraphOp(G.AddOp(layer, relu), [src(i) for i in ins], end))
            continue
        if isinstance(layer, L.Activation):
            if layer.activation == "linear":
                alias[k] = ins[0]
                continue
            if layer.activation == "relu":
                ops.append(G.Adapter(E.ReLUOp(layer), [src(ins[0])], k))
                continue
            raise NotImplementedError("standalone Activation('softmax'): use Dense(activation='softmax')")
        inner = {L.Dense: E.DenseOp, L.Flatten: E.FlattenOp, L.GlobalAveragePooling2D: E.GAPOp,
                 L.PReLU: E.PReLUOp, L.ReLU: E.ReLUOp}.get(type(layer))
        if inner is None:
            raise NotImplementedError(f"functional lowering of {type(layer).__name__}")
        ops.append(G.Adapter(inner(layer), [src(ins[0])], k))
    _bn_bwd_links(ops)
    # dense relu-mask hand-off as in the Sequential engine
    for a, b in zip(ops, ops[1:]):
        ia, ib = getattr(a, "inner", None), getattr(b, "inner", None)
        if isinstance(ia, E.DenseOp) and isinstance(ib, E.DenseOp) and not ib.big and ia.act == "relu" \
                and b.inputs == [a.output]:
            ib.mask_for_prev, ib._prev_big, ib._prev_op = True, ia.big, ia
            ia.grad_masked_by_next = True
    return ops


def _bn_bwd_links(ops) -> None:
    """Conv -> BN -> ReLU (no residual) feeding exactly one ConvBNOp: that consumer's dgrad epilogue
    computes the producer's BN backward sums (graph_ops.BN_BWD_EPI)."""
    uses: dict = {}
    for op in ops:
        for i in op.inputs:
            uses.setdefault(i, []).append(op)
    for a in ops:
        pa = getattr(a, "op", None)
        if not isinstance(pa, G.ConvBNOp) or not pa.relu or pa.residual:
            continue
        cons = uses.get(a.output, [])
        if len(cons) != 1 or not isinstance(getattr(cons[0], "op", None), G.ConvBNOp):
            continue
        b = cons[0]
        if b.inputs[0] != a.output or a.output in b.inputs[1:]:
            continue
        b.op.bwd_bn_op = pa


class Model(Sequential):
    """``keras.Model(inputs=..., outputs=...)`` on the fused graph plan.  Training/eval/predict/save
    come from :class:`~.model.Sequential`; only the execution plan differs."""

    def __init__(self, inputs=None, outputs=None, name: str = "functional"):
        super().__init__(None, name=name)
        ins = inputs if isinstance(inputs, (list, tuple)) else [inputs]
        outs = outputs if isinstance(outputs, (list, tuple)) else [outputs]
        if len(ins) != 1 or len(outs) != 1:
            raise NotImplementedError("Model with exactly one input and one output")
        self._in = _as_tensor(ins[0])
        self._out = _as_tensor(outs[0])
        self.nodes = _topo([self._out])
        if self._in not in self.nodes:
            raise ValueError("outputs are not connected to inputs")
        self._layers = [t.layer for t in self.nodes]
        self.input_shape = self._in.shape
        self.plan = None

    def build(self, input_shape=None, device=None, seed: int | None = None) -> None:
        if self.built:
            return
        import os

        import torch

        from .model import default_device

        self.device = torch.device(device) if device is not None else default_device()
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.store = ParamStore()
        shapes = {}
        for t in self.nodes:
            if isinstance(t.layer, L.Input):
                shapes[id(t)] = t.layer.shape
                continue
            ins = [shapes[id(i)] for i in t.inputs]
            shapes[id(t)] = t.layer.build(ins[0] if len(ins) == 1 else tuple(ins), self.store)
        self.output_shape = shapes[id(self._out)]
        if seed is None:
            seed = config.get("seed")
        self.store.finalize(self.device, seed=seed)
        for l in self.layers:
            if isinstance(l, L.BatchNormalization):
                l.init_state(self.device)
        self.plan = GraphPlan(self.nodes, self.nodes.index(self._in), self.nodes.index(self._out))
        self.ops = self.plan.ops
        self.store.update_zero_ranges()
        self.built = True
        from ..distribute import current_strategy

        st = current_strategy()
        if st is not None:
            st.register_model(self)

    # ---- execution plan hooks
    def _run_forward(self, xb, training: bool):
        return self.plan.forward(xb, self.ws, training, pre_op=self._pre_op_hook())

    def _run_backward(self, dpred, on_op_done=None):
        return self.plan.backward(dpred, self.ws, on_op_done=on_op_done)

    def _last_op(self):
        last = self.ops[-1]
        return getattr(last, "inner", last)

    def _tape_head_ok(self) -> bool:
        return False  # the deferred-prediction head (nn/tape.py) follows the Sequential plan only

    def first_op(self):
        first = self.ops[0]
        return getattr(first, "op", getattr(first, "inner", first))

    # ---- introspection / persistence
    def summary(self, print_fn=None):
        pf = print_fn or print
        rows = []
        for t in self.nodes:
            l = t.layer
            conn = ", ".join(f"{i.layer.name}" for i in t.inputs) or "-"
            pc = l.param_count() if not isinstance(l, L.Input) else 0
            rows.append((f"{l.name} ({l.keras_class})", str((None, *t.shape)), f"{pc:,}", conn))
        w = [max(31, max(len(r[0]) for r in rows) + 1), 22, 11, 28]
        pf(f'Model: "{self.name}"')
        pf("┏" + "┳".join("━" * (x + 2) for x in w) + "┓")
        pf(f"┃ {'Layer (type)':<{w[0]}} ┃ {'Output Shape':<{w[1]}} ┃ {'Param #':>{w[2]}} ┃ {'Connected to':<{w[3]}} ┃")
        pf("┡" + "╇".join("━" * (x + 2) for x in w) + "┩")
        for r in rows:
            pf(f"│ {r[0]:<{w[0]}} │ {r[1]:<{w[1]}} │ {r[2]:>{w[2]}} │ {r[3]:<{w[3]}} │")
        pf("└" + "┴".join("─" * (x + 2) for x in w) + "┘")
        trainable = self.store.num_params()
        nontrain = sum(l.non_trainable_count() for l in self.layers if isinstance(l, L.BatchNormalization))
        total = trainable + nontrain
        pf(f" Total params: {total:,} ({total * 4 / 2 ** 20:.2f} MB)")
        pf(f" Trainable params: {trainable:,} ({trainable * 4 / 2 ** 20:.2f} MB)")
        pf(f" Non-trainable params: {nontrain:,} ({nontrain * 4 / 2 ** 20:.2f} MB)")

    def count_params(self) -> int:
        nontrain = sum(l.non_trainable_count() for l in self.layers if isinstance(l, L.BatchNormalization))
        return (self.store.num_params() if self.store else 0) + nontrain

    def get_config(self) -> dict:
        layers = []
        for t in self.nodes:
            l = t.layer
            layers.append({"class_name": l.keras_class, "config": l.get_config(), "name": l.name,
                           "inbound_nodes": [i.layer.name for i in t.inputs]})
        return {"name": self.name, "layers": layers, "input_layers": [self._in.layer.name],
                "output_layers": [self._out.layer.name]}

    def _save_class_name(self) -> str:
        return "Functional"


def model_from_config(cfg: dict) -> Model:
    L.reset_name_counters()
    tensors = {}
    for lc in cfg["layers"]:
        layer = L.layer_from_config(lc["class_name"], lc["config"])
        if isinstance(layer, L.Input):
            tensors[layer.name] = layer.output
            continue
        ins = [tensors[n] for n in lc["inbound_nodes"]]
        tensors[layer.name] = layer(ins if len(ins) > 1 else ins[0])
    return Model(tensors[cfg["input_layers"][0]], tensors[cfg["output_layers"][0]], name=cfg.get("name", "functional"))


_ = (time, np)
