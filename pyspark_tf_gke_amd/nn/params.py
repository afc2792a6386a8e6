"""Flat parameter store.

All parameters of a model live in ONE fp32 master buffer (plus one fp32 gradient buffer and one
bf16 compute mirror at identical offsets).  This is the MI355X-native layout for the reference's
per-variable Keras weights (train_tf_ps.py:328-378): the fused Adam kernel updates every
parameter in a single launch, the data-parallel strategies all-reduce / reduce-scatter
contiguous byte ranges (a handful of large RCCL collectives instead of one per variable), and the
parameter-server strategy shards the buffer by byte range (the role of TF's
``MinSizePartitioner``, train_tf_ps.py:505-507).

Parameters are laid out in *reverse* layer order, so gradients complete front-to-back of the
buffer during backward and bucketed all-reduce can start on the head while the tail is still
being computed.  Every parameter starts on a 64-element boundary (16-byte vector access for the
fp32 and bf16 views).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable

import numpy as np
import torch

ALIGN = 64


def glorot_uniform(fan_in: int, fan_out: int):
    def init(shape, rng: np.random.Generator):
        limit = math.sqrt(6.0 / (fan_in + fan_out))
        return rng.uniform(-limit, limit, size=shape).astype(np.float32)

    return init


def zeros(shape, rng):
    return np.zeros(shape, np.float32)


def ones(shape, rng):
    return np.ones(shape, np.float32)


@dataclass
class Param:
    name: str
    shape: tuple
    init: Callable
    overwrite_grad: bool = False  # backward writes (not accumulates) this gradient
    logical_numel: int | None = None  # count shown by summary() (padding excluded)
    order: int = 0
    offset: int = -1
    data: torch.Tensor | None = None
    grad: torch.Tensor | None = None
    bf16: torch.Tensor | None = None
    mask_fn: Callable | None = None  # zero padded entries after init (e.g. padded input channels)
    fwd_bf16: bool = False  # forward reads only the bf16 mirror (matmul/conv weights): the sharded
    #                         update may all-gather just the bf16 copy of it

    @property
    def numel(self) -> int:
        return int(np.prod(self.shape))


@dataclass
class ParamStore:
    params: list = field(default_factory=list)
    flat: torch.Tensor | None = None
    flat_grad: torch.Tensor | None = None
    flat_bf16: torch.Tensor | None = None
    total: int = 0
    device: torch.device | None = None
    _zero_ranges: list = field(default_factory=list)
    # (id(optimizer), iterations) after an update that also wrote the conv ops' flipped dgrad
    # filters (nn.optimizers.Adam.finish_fused); any other write to the weights clears it
    flip_token: tuple | None = None
    flip_names: frozenset = frozenset()

    def add(self, name: str, shape, init, overwrite_grad=False, logical_numel=None, mask_fn=None) -> Param:
        p = Param(name, tuple(int(s) for s in shape), init, overwrite_grad, logical_numel, len(self.params),
                  mask_fn=mask_fn)
        self.params.append(p)
        return p

    def finalize(self, device, seed: int = 0) -> None:
        rng = np.random.default_rng(seed)
        host_vals = {}
        for p in self.params:  # init in declaration order (deterministic)
            v = p.init(p.shape, rng)
            if p.mask_fn is not None:
                v = p.mask_fn(v)
            host_vals[p.name] = v
        off = 0
        for p in reversed(self.params):  # reverse layer order = backward completion order
            p.offset = off
            off += int(math.ceil(p.numel / ALIGN) * ALIGN)
        self.total = max(off, ALIGN)
        self.device = torch.device(device)
        flat_host = np.zeros(self.total, np.float32)
        for p in self.params:
            flat_host[p.offset:p.offset + p.numel] = host_vals[p.name].reshape(-1)
        self.flat = torch.from_numpy(flat_host).to(self.device)
        from ..ops import nn as K

        self.flat_grad = K.zeros(self.total, torch.float32, self.device)
        from .engine import host_fp32

        mirror = torch.float32 if (host_fp32() and self.device.type == "cpu") else torch.bfloat16
        self.flat_bf16 = self.flat.to(mirror)
        self._bind_views()
        self.update_zero_ranges()

    def update_zero_ranges(self) -> None:
        """Contiguous ranges whose gradient must be zeroed before each backward (every parameter
        whose backward accumulates).  Re-run after the engine lowers the model, since lowering
        decides which gradients are written whole (``overwrite_grad``)."""
        ranges = []
        for p in sorted(self.params, key=lambda q: q.offset):
            if p.overwrite_grad:
                continue
            lo, hi = p.offset, p.offset + int(math.ceil(p.numel / ALIGN) * ALIGN)
            if ranges and ranges[-1][1] == lo:
                ranges[-1][1] = hi
            else:
                ranges.append([lo, hi])
        self._zero_ranges = [tuple(r) for r in ranges]

    def relayout(self, groups: list, align: int) -> list:
        """Re-place the parameters: ``groups`` (lists of Params, each in the order wanted) are laid
        out one after another, every group starting on and padded to a multiple of ``align``
        elements.  Values (fp32 master and bf16 mirror) move with their parameters; gradients are
        zero.  Returns the [lo, hi) element range of each group.  Used by the sharded data-parallel
        update, whose reduce-scatter / all-gather buckets need world-divisible ranges."""
        seen = {id(p) for g in groups for p in g}
        assert len(seen) == len(self.params), "relayout must place every parameter exactly once"
        old = {id(p): (p.offset, p.numel) for p in self.params}
        ranges, off = [], 0
        for g in groups:
            off = int(math.ceil(off / align) * align)
            lo = off
            for p in g:
                p.offset = off
                off += int(math.ceil(p.numel / ALIGN) * ALIGN)
            off = int(math.ceil(off / align) * align)
            ranges.append((lo, off))
        total = max(off, ALIGN)
        from ..ops import nn as K

        flat = K.zeros(total, self.flat.dtype, self.flat.device)
        mirror = K.zeros(total, self.flat_bf16.dtype, self.flat.device)
        for p in self.params:
            o, n = old[id(p)]
            flat[p.offset:p.offset + n] = self.flat[o:o + n]
            mirror[p.offset:p.offset + n] = self.flat_bf16[o:o + n]
        self.flat, self.flat_bf16 = flat, mirror
        self.flat_grad = K.zeros(total, torch.float32, flat.device)
        self.total = total
        self._bind_views()
        self.update_zero_ranges()
        return ranges

    def _bind_views(self) -> None:
        self.flip_token = None
        for p in self.params:
            sl = slice(p.offset, p.offset + p.numel)
            p.data = self.flat[sl].view(p.shape)
            p.grad = self.flat_grad[sl].view(p.shape)
            p.bf16 = self.flat_bf16[sl].view(p.shape)

    def zero_grad(self) -> None:
        """Zero every accumulated gradient before a backward.  Skipped when the last optimizer
        update consumed the whole gradient buffer and stored zeros back (``grad_clean``, set by the
        clearing Adam/SGD kernels): the per-step fill pass then disappears from the step."""
        if getattr(self, "grad_clean", False):
            self.grad_clean = False
            return
        from ..ops import nn as K

        for lo, hi in self._zero_ranges:
            K.fill_(self.flat_grad[lo:hi], 0.0)

    def refresh_bf16(self) -> None:
        from ..ops import nn as K

        self.flip_token = None
        if self.flat.is_cuda and self.flat_bf16.dtype == torch.bfloat16:
            K.cast_f32_bf16(self.flat, self.flat_bf16)
        else:
            self.flat_bf16.copy_(self.flat.to(self.flat_bf16.dtype))

    def by_name(self, name: str) -> Param:
        for p in self.params:
            if p.name == name:
                return p
        raise KeyError(name)

    def num_params(self) -> int:
        return sum(p.logical_numel if p.logical_numel is not None else p.numel for p in self.params)

    def to(self, device) -> None:
        self.device = torch.device(device)
        self.flat = self.flat.to(self.device)
        self.flat_grad = self.flat_grad.to(self.device)
        self.flat_bf16 = self.flat_bf16.to(self.device)
        self._bind_views()
