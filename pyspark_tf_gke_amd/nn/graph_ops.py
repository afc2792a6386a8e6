"""Fused device ops of the functional-graph engine (:mod:`.functional`).

* :class:`ConvBNOp` — ``Conv2D -> BatchNormalization [-> Add(residual)] [-> ReLU]`` (ResNet's
  unit).  Forward: conv into bf16 ``z`` (1x1/stride-1 = plain MFMA GEMM over the NHWC pixel rows;
  3x3 with C <= 64 = halo-tiled direct conv; otherwise implicit GEMM), batch statistics of ``z``
  (``bn_stats``, training) or moving statistics (inference), then ONE apply pass
  ``y = relu(z*scale + shift + residual)``.  Backward: one reduction pass (sum g, sum g*z with the
  ReLU mask applied on the fly), a per-channel finalize that also writes d(gamma)/d(beta), one
  apply pass producing ``dz`` and ``d(residual)``, then MFMA wgrad and dgrad of the conv.  The conv
  bias gradient of a conv feeding a training-mode BN is identically zero (BN removes the mean), so
  it is never computed.
* :class:`BNOp`, :class:`MaxPoolOp` (k x k / stride s / folded zero padding), :class:`AddOp`.
* :class:`Adapter` runs the Sequential engine's single-input ops (Dense, GAP, Flatten, PReLU...)
  inside a graph.

Gradient accumulation: ``backward(dy, ws, existing)`` receives the gradient buffers already
produced for each input (a tensor with several consumers); the 1x1 and implicit-GEMM dgrads add
into them inside the GEMM epilogue instead of running a separate add.
"""
from __future__ import annotations

import math

import torch

from ..ops import bn as KB
from ..ops import nn as K
from . import engine as E
from . import layers as L
from . import streams as S
from .. import config


def _bf16(x, ws, key):
    return E._bf16(x, ws, key)


class Adapter:
    """Graph node around a single-input Sequential-engine op."""

    def __init__(self, inner, inputs, output):
        self.inner = inner
        self.inputs = inputs
        self.output = output
        self.params = inner.params
        self.name = inner.name

    @property
    def first(self):
        return self.inner.first

    @first.setter
    def first(self, v):
        self.inner.first = v

    def forward(self, xs, ws, training):
        inner = self.inner
        if isinstance(inner, E.DenseOp) and inner.mask_for_prev:
            inner._prev_y = inner._prev_op._y
        return inner.forward(xs[0], ws, training)

    def backward(self, dy, ws, existing):
        return [self.inner.backward(dy, ws)]


class GraphOp:
    """Graph node around a multi-input fused op."""

    def __init__(self, op, inputs, output):
        self.op = op
        self.inputs = inputs
        self.output = output
        self.params = op.params
        self.name = op.name

    @property
    def first(self):
        return self.op.first

    @first.setter
    def first(self, v):
        self.op.first = v

    def forward(self, xs, ws, training):
        return self.op.forward(xs, ws, training)

    def backward(self, dy, ws, existing):
        return self.op.backward(dy, ws, existing)

    def _prep_input(self, x, ws):
        return self.op._prep_input(x, ws)


# ------------------------------------------------------------------------------------------------
# convolution dispatch (shared by ConvBNOp)
# ------------------------------------------------------------------------------------------------
# The halo-tiled direct conv (csrc/kernels/conv.hip) is tuned for the reference CNN's 5x5 layers
# with 4-64 channels; measured on ResNet-50's 3x3/64-channel layers (56x56, batch 128) the
# implicit-GEMM path is faster, so graph ops use the halo kernels for 5x5 only.
HALO_KS = (5,)
# BatchNormalization fusion: every ConvBNOp's batch statistics come out of its conv GEMM's epilogue
# (PTG_BN_EPI_STATS; no bn_stats pass over z; gemm.hip EpiBf16 stats).  (Applying the previous BN + ReLU
# in the next conv's operand loaders instead of a bn_apply pass measured slower - 8.04k vs 8.75k img/s
# - and was removed in round 5.)
BN_EPI_STATS = config.get("bn_epi_stats")
# Backward: a Conv -> BN -> ReLU block whose output feeds exactly one ConvBNOp gets its BN backward
# sums (sum g, sum g*z) from the epilogue of that consumer's dgrad GEMM, which also applies the ReLU
# mask to the gradient it stores (gemm.hip EpiBf16 backward form): the bn_bwd_reduce pass over dy and
# z disappears.  PTG_BN_BWD_EPI_STATS=0 keeps the separate reduction.
BN_BWD_EPI = config.get("bn_bwd_epi_stats")
# Residual BN + ReLU: bn_apply_k also writes a 1-bit ReLU mask of y; the backward reads it instead of
# y (PTG_BN_RELU_BITS=0: read y).
RELU_BITS = config.get("bn_relu_bits")


def _pow2(v):
    return v > 0 and (v & (v - 1)) == 0


def conv_forward(x, w, bias, stride, pad, z, stats=None) -> bool:
    """z = conv(x) (+ bias).  ``stats``: [64,2,Cout] partial sums for this op's BN, filled by the conv
    epilogue when it can.  Returns True when ``stats`` were produced."""
    N, H, W, C = x.shape
    Co, KH, KW, _ = w.shape
    if stats is not None:
        same = pad == KH // 2 and KH == KW and stride == 1
        halo = KH in HALO_KS and K.halo_eligible(C, Co, KH, stride, same)
        if not halo and _pow2(C) and C >= 4 and Co % 8 == 0:
            K.conv_bn_fwd(x, w, bias, stride, pad, z, stats)
            return True
    if not K.on_device(x):
        K.conv2d_fwd(x, w, bias, stride, pad, z, None)
        return False
    if KH == KW == 1 and stride == 1 and pad == 0:
        M = N * H * W
        K.gemm(M, Co, C, x, C, 1, w, C, 1, 0, z, Co, bias, 0, 1)
        return False
    same = pad == KH // 2 and KH == KW and stride == 1
    if KH in HALO_KS and K.halo_eligible(C, Co, KH, stride, same):
        K.conv2d_fwd_fused(x, w, bias, pad, z)
        return False
    K.conv2d_fwd(x, w, bias, stride, pad, z, None)
    return False


def conv_wgrad(x, dz, stride, pad, dw):
    """dw (fp32, already zeroed by the store) += d(conv)/dw."""
    N, H, W, C = x.shape
    _, OH, OW, Co = dz.shape
    _, KH, KW, _ = dw.shape
    if not K.on_device(x):
        return K.conv2d_wgrad(x, dz, stride, pad, dw, accumulate=True)
    if KH == KW == 1 and stride == 1 and pad == 0:
        M = N * H * W
        tiles = math.ceil(Co / 128) * math.ceil(C / 128)
        splits = max(1, min(math.ceil(512 / tiles), M // 512))  # ~2 blocks/CU; atomics cost bytes
        K.gemm(Co, C, M, dz, Co, 0, x, C, 0, 3, dw, C, None, 0, splits)
        return dw
    same = pad == KH // 2 and KH == KW and stride == 1
    if KH in HALO_KS and K.halo_eligible(C, Co, KH, stride, same):
        return K.conv2d_wgrad_halo(x, dz, pad, dw, zeroed=True)  # dw zeroed by the store
    return K.conv2d_wgrad(x, dz, stride, pad, dw, accumulate=True)


def conv_dgrad(dz, w, stride, pad, dx, accumulate, ws, key):
    """dx (+)= d(conv)/dx.  Returns True when the result was accumulated into ``dx`` in place."""
    Co, KH, KW, Cin = w.shape
    if KH == KW == 1 and pad == 0:
        K.conv1x1_dgrad(dz, w, stride, dx, accumulate)
        return True
    if stride != 1:
        raise NotImplementedError("dgrad of a strided KxK (K > 1) convolution that is not the first layer")
    same = pad == KH // 2 and KH == KW
    if K.on_device(dz) and KH in HALO_KS and K.halo_eligible(Co, Cin, KH, 1, same) and not accumulate:
        wf = ws.get(key + "/wflip", (Cin, KH, KW, Co), torch.bfloat16, dz.device)
        K.conv2d_dgrad_halo(dz, w, pad, dx, wf)
        return True
    K.conv2d_dgrad(dz, w, pad, dx, accumulate)
    return True


class _BNState:
    """Per-op BN scratch: statistics, coefficients, partial sums (zeroed by the finalize kernels)."""

    def __init__(self, bn: L.BatchNormalization, name: str):
        self.bn = bn
        self.name = name

    def bufs(self, ws, C, dev):
        f = torch.float32
        return (ws.get(self.name + "/bn_part", (KB.BN_G, 2, C), f, dev, zero=True),
                ws.get(self.name + "/bn_scale", (C,), f, dev), ws.get(self.name + "/bn_shift", (C,), f, dev),
                ws.get(self.name + "/bn_mean", (C,), f, dev), ws.get(self.name + "/bn_rstd", (C,), f, dev),
                ws.get(self.name + "/bn_coef", (3, C), f, dev))

    def forward(self, z, res, relu, y, ws, training, stats_done=False, apply=True):
        """Statistics (unless the conv epilogue produced them), finalize, and - unless the consumer
        applies it on load - the apply pass into y."""
        bn = self.bn
        C = z.shape[-1]
        M = z.numel() // C
        part, scale, shift, mean, rstd, _ = self.bufs(ws, C, z.device)
        g = bn.gamma.data if bn.gamma is not None else None
        b = bn.beta.data if bn.beta is not None else None
        if training and not stats_done:
            KB.bn_stats(z, part)
        KB.bn_finalize(part, M, g, b, bn.epsilon, bn.momentum if training else -1.0, bn.moving_mean,
                       bn.moving_variance, scale, shift, mean, rstd, training)
        if not K.on_device(z) and training:
            part.zero_()
        if not apply:
            return z
        # residual + ReLU on the GPU: the backward's ReLU mask comes from a bit mask written here
        # (1 bit instead of re-reading the 16-bit y in bn_bwd_reduce and bn_bwd_apply)
        mask = None
        if relu and res is not None and K.on_device(z) and RELU_BITS:
            mask = ws.get(self.name + "/relu_bits", (z.numel() // 8,), torch.uint8, z.device)
        self._mask = mask
        return KB.bn_apply(z, scale, shift, res, relu, y, mask)

    def backward(self, dy, y, z, relu, dz, dres, ws, stats_done=False):
        bn = self.bn
        C = z.shape[-1]
        M = z.numel() // C
        part, scale, shift, mean, rstd, coef = self.bufs(ws, C, z.device)
        # no residual was added before the ReLU: its mask is z*scale+shift > 0, y need not be read
        sc, sh = (scale, shift) if (relu and dres is None) else (None, None)
        mask = getattr(self, "_mask", None) if (relu and dres is not None) else None
        if not stats_done:  # else: the producing dgrad's epilogue summed (g, g*z) into part already
            KB.bn_bwd_reduce(dy, y, z, relu, part, sc, sh, mask)
        KB.bn_bwd_finalize(part, M, bn.gamma.data if bn.gamma is not None else None, mean, rstd,
                           bn.gamma.grad if bn.gamma is not None else None,
                           bn.beta.grad if bn.beta is not None else None, coef)
        if not K.on_device(z):
            part.zero_()
        return KB.bn_bwd_apply(dy, y, z, coef, relu, dz, dres, sc, sh, mask)


class ConvBNOp:
    first = False

    def __init__(self, conv: L.Conv2D, bn: L.BatchNormalization, relu: bool, residual: bool, extra_pad: int = 0):
        self.conv, self.bn, self.relu, self.residual = conv, bn, relu, residual
        self.params = list(conv.params) + list(bn.params)
        conv.kernel.fwd_bf16 = True
        self.stride = conv.strides[0]
        if conv.strides[0] != conv.strides[1]:
            raise NotImplementedError("non-square strides")
        self.pad = conv.pad_amount() + extra_pad
        self.name = conv.name
        self.state = _BNState(bn, conv.name)
        # the Conv -> BN -> ReLU producer whose BN backward sums our dgrad epilogue computes (set by
        # functional._bn_bwd_links); _bwd_stats_done marks a step in which it did
        self.bwd_bn_op = None
        self._bwd_stats_done = False
        if conv.activation not in ("linear", None):
            raise NotImplementedError("Conv2D(activation=...) followed by BatchNormalization")

    def _prep_input(self, x, ws):
        cp = self.conv.cin_p
        if x.shape[-1] == cp and (x.dtype == torch.bfloat16 or (E.host_fp32() and not x.is_cuda)):
            return x
        xi = ws.get(self.name + "/xin", (*x.shape[:-1], cp), torch.bfloat16, x.device)
        if x.shape[-1] == 3 and cp == 4 and x.dtype == torch.float32:
            return K.pack_rgb4(x.contiguous(), xi)
        xi.zero_()
        xi[..., : x.shape[-1]] = x
        return xi

    def forward(self, xs, ws, training):
        x = self._prep_input(xs[0], ws)
        res = xs[1] if self.residual else None
        if res is not None:
            res = _bf16(res, ws, self.name + "/res16")
        B = x.shape[0]
        OH, OW, Co = self.conv.out_shape
        dev = x.device
        z = ws.get(self.name + "/z", (B, OH, OW, Co), torch.bfloat16, dev)
        b = self.conv.bias.data if self.conv.bias is not None else None
        part = self.state.bufs(ws, Co, dev)[0] if (training and BN_EPI_STATS) else None
        stats_done = conv_forward(x, self.conv.kernel.bf16, b, self.stride, self.pad, z, part)
        self._x, self._z = x, z
        y = ws.get(self.name + "/y", z.shape, torch.bfloat16, dev)
        self.state.forward(z, res, self.relu, y, ws, training, stats_done)
        self._y = y
        return y

    def backward(self, dy, ws, existing):
        x, z, y = self._x, self._z, self._y
        dev = z.device
        dy = _bf16(dy, ws, self.name + "/dy16")
        dz = ws.get(self.name + "/dz", z.shape, torch.bfloat16, dev)
        dres = ws.get(self.name + "/dres", z.shape, torch.bfloat16, dev) if self.residual else None
        done, self._bwd_stats_done = self._bwd_stats_done, False
        self.state.backward(dy, y, z, self.relu, dz, dres, ws, stats_done=done)
        g = self.conv.kernel.grad
        S.launch(lambda: conv_wgrad(x, dz, self.stride, self.pad, g), dev)
        dx = None
        if not self.first:
            ex = existing[0]
            if ex is not None and ex.dtype == x.dtype and tuple(ex.shape) == tuple(x.shape):
                conv_dgrad(dz, self.conv.kernel.bf16, self.stride, self.pad, ex, True, ws, self.name)
                dx = ex
            else:
                dx = ws.get(self.name + "/dx", x.shape, torch.bfloat16, dev)
                p = self.bwd_bn_op
                if (p is not None and BN_BWD_EPI and self.stride == 1 and ex is None and p.relu and not p.residual
                        and getattr(p, "_z", None) is not None and tuple(p._z.shape) == tuple(x.shape)):
                    pc = p.conv.out_shape[-1]
                    part, scale, shift = p.state.bufs(ws, pc, dev)[:3]
                    if K.conv_dgrad_bnstats(dz, self.conv.kernel.bf16, self.pad, dx, part, p._z, scale, shift):
                        p._bwd_stats_done = True
                        return [dx] + ([dres] if self.residual else [])
                conv_dgrad(dz, self.conv.kernel.bf16, self.stride, self.pad, dx, False, ws, self.name)
        return [dx] + ([dres] if self.residual else [])


class BNOp:
    """Standalone BatchNormalization [+ residual Add] [+ ReLU] (input not produced by a Conv2D)."""

    first = False

    def __init__(self, bn: L.BatchNormalization, relu: bool, residual: bool):
        self.bn, self.relu, self.residual = bn, relu, residual
        self.params = list(bn.params)
        self.name = bn.name
        self.state = _BNState(bn, bn.name)

    def _prep_input(self, x, ws):
        return _bf16(x, ws, self.name + "/x16")

    def forward(self, xs, ws, training):
        z = self._prep_input(xs[0], ws)
        res = _bf16(xs[1], ws, self.name + "/res16") if self.residual else None
        y = ws.get(self.name + "/y", z.shape, torch.bfloat16, z.device)
        self.state.forward(z, res, self.relu, y, ws, training)
        self._z, self._y = z, y
        return y

    def backward(self, dy, ws, existing):
        z, y = self._z, self._y
        dy = _bf16(dy, ws, self.name + "/dy16")
        dz = ws.get(self.name + "/dz", z.shape, torch.bfloat16, z.device)
        dres = ws.get(self.name + "/dres", z.shape, torch.bfloat16, z.device) if self.residual else None
        self.state.backward(dy, y, z, self.relu, dz, dres, ws)
        return [None if self.first else dz] + ([dres] if self.residual else [])


class MaxPoolOp:
    first = False

    def __init__(self, layer: L.MaxPooling2D, pad: int = 0):
        self.layer = layer
        self.k, self.s, self.p = layer.pool_size[0], layer.strides[0], pad
        self.params = []
        self.name = layer.name

    def forward(self, xs, ws, training):
        x = _bf16(xs[0], ws, self.name + "/x16")
        B, H, W, C = x.shape
        OH, OW = KB.pool_out_size(H, self.k, self.s, self.p), KB.pool_out_size(W, self.k, self.s, self.p)
        out = ws.get(self.name + "/y", (B, OH, OW, C), torch.bfloat16, x.device)
        arg = ws.get(self.name + "/arg", (B, OH, OW, C), torch.uint8, x.device)
        KB.maxpool_fwd(x, out, arg, self.k, self.s, self.p)
        self._xshape, self._arg = x.shape, arg
        return out

    def backward(self, dy, ws, existing):
        if self.first:
            return [None]
        dy = _bf16(dy, ws, self.name + "/dy16")
        ex = existing[0]
        if ex is not None and ex.dtype == dy.dtype and tuple(ex.shape) == tuple(self._xshape):
            KB.maxpool_bwd(dy, self._arg, ex, self.k, self.s, self.p, accumulate=True)
            return [ex]
        dx = ws.get(self.name + "/dx", self._xshape, torch.bfloat16, dy.device)
        KB.maxpool_bwd(dy, self._arg, dx, self.k, self.s, self.p)
        return [dx]


class AddOp:
    first = False

    def __init__(self, layer: L.Add, relu: bool):
        self.layer, self.relu = layer, relu
        self.params = []
        self.name = layer.name

    def forward(self, xs, ws, training):
        a = _bf16(xs[0], ws, self.name + "/a16")
        b = _bf16(xs[1], ws, self.name + "/b16")
        y = ws.get(self.name + "/y", a.shape, torch.bfloat16, a.device)
        KB.add_(a, b, y)
        if self.relu:
            K.relu_bwd(y, y, y)
        self._y = y
        return y

    def backward(self, dy, ws, existing):
        dy = _bf16(dy, ws, self.name + "/dy16")
        if self.relu:
            g = ws.get(self.name + "/g", dy.shape, torch.bfloat16, dy.device)
            K.relu_bwd(dy, self._y, g)
        else:
            g = dy
        g2 = ws.get(self.name + "/g2", g.shape, torch.bfloat16, g.device)
        g2.copy_(g)  # each branch owns its gradient buffer (it may be accumulated into)
        return [g, g2]
