"""Fused execution plan for Sequential models (the training "step engine").

Keras layers (:mod:`.layers`) are lowered to device ops that own their forward/backward:

* ``ConvOp``   Conv2D [+ PReLU] [+ MaxPooling2D]: implicit-GEMM MFMA conv with bias in the
  epilogue, then ONE fused PReLU+max-pool kernel; backward = fused PReLU/pool gradient (also
  accumulating d(alpha) and d(bias)) -> MFMA wgrad (split-K) -> MFMA dgrad.
* ``DenseOp``  Dense: MFMA GEMM with bias+ReLU epilogue for wide layers, a VALU "skinny" kernel
  for narrow ones (N <= 64: the MLP and the 2-output regression head).  A narrow Dense also
  applies the previous layer's ReLU mask inside its dX kernel.
* ``FlattenOp`` (a view), ``GAPOp``, ``PReLUOp``/``PoolOp`` (unfused fallbacks).

Activations live in a :class:`Workspace` keyed by op and shape, so every step reuses the same
device buffers (stable addresses; capturable into a HIP graph).  Reference: the model builders of
train_tf_ps.py:328-378 and the GradientTape step of :616-631 / :738-753.
"""
from __future__ import annotations

import os

import torch

from ..ops import nn as K
from . import layers as L
from . import streams as S
from .. import config


# Host-path debug precision: with PTG_HOST_FP32=1 (or ``host_fp32(True)``) CPU models keep their
# "bf16" activations and compute-weight mirror in fp32, so the CPU engine can be checked against
# an fp32 autograd oracle exactly (the GPU path is always bf16).
_HOST_FP32 = [config.get("host_fp32")]

# Sparse PReLU+pool record (conv.hip EPI_POOLS: z at the argmax + argmax index instead of the full
# z) for layers 2-4 as well was measured and rejected (README): its longer epilogue makes those
# latency-bound forward kernels slower than the backward saves.
# The FIRST conv layer (no data gradient) keeps its whole backward sparse: forward writes the record,
# prelu_pool_bwd_sel turns it into dZ's record (dZ at the argmax) and the weight gradient expands it in
# LDS, so the full-resolution z and dZ (335 MB each for CNN-B1 at batch 256) never exist.  Measured
# on CNN-B1 b256: 118.6k vs 116.6k samples/s with the dense first-layer record.
SPARSE_FIRST = config.get("sparse_first")
# Pooled layers after the first: sparse pool record end to end (forward record, sparse dZ record,
# weight and data gradients expanding it in their loaders) - no full-resolution z / dZ in HBM.
SPARSE_POOL = config.get("sparse_pool")
SPARSE_POOL_MIN_BATCH = config.get("sparse_pool_min_batch")
# That first layer reads the raw uint8 [N,H,W,3] image batch itself (conv.hip U8 loaders: /255 and
# the zero 4th channel applied in registers) in both its forward and its weight gradient, so the
# packed bf16 copy of the input (pack_u8rgb4_k: 3 B read + 8 B written per pixel, 8 B read twice
# more) is never made.  PTG_RAW_U8_INPUT=0 restores the pack.
RAW_U8 = config.get("raw_u8_input")
# With CONV1_FUSED (default) that first layer runs as two position-major kernels instead
# (conv1.hip): the forward writes only the pooled output, and ONE backward kernel recomputes z, the
# PReLU and the pool argmax from x and accumulates dW, dalpha and dbias from the pooled gradient -
# no record, no dZ, no separate prelu/pool backward.  PTG_CONV1_FUSED=0 restores the sparse-record
# pipeline above for A/B.
CONV1_FUSED = config.get("conv1_fused")
# ... and by default (CONV1_REC) its forward keeps the pool record (z at each window's argmax + the
# argmax: 3 bytes per pooled element) so the backward kernel needs no conv recompute and no argmax
# search; PTG_CONV1_REC=0 runs the recomputing backward.
CONV1_REC = config.get("conv1_rec")


def host_fp32(enabled: bool | None = None) -> bool:
    if enabled is not None:
        _HOST_FP32[0] = bool(enabled)
    return _HOST_FP32[0]


class Workspace:
    def __init__(self):
        self.bufs: dict = {}

    def get(self, key, shape, dtype, device, zero=False):
        shape = tuple(int(s) for s in shape)
        if dtype == torch.bfloat16 and _HOST_FP32[0] and torch.device(device).type == "cpu":
            dtype = torch.float32
        t = self.bufs.get(key)
        if t is None or tuple(t.shape) != shape or t.dtype != dtype or t.device != torch.device(device):
            t = K.zeros(shape, dtype, device) if zero else torch.empty(shape, dtype=dtype, device=device)
            self.bufs[key] = t
        return t

    def clear(self):
        self.bufs.clear()


class Op:
    first = False  # no dX needed

    def __init__(self):
        self.params = []
        self.mask_for_prev = False  # this op applies the previous op's ReLU mask in its dX
        self.grad_masked_by_next = False  # our output gradient arrives already ReLU-masked

    def forward(self, x, ws, training):
        raise NotImplementedError

    def backward(self, dy, ws):
        raise NotImplementedError


def _const_buf(ws, key, shape, value, dev):
    """A workspace buffer filled with ``value`` once per (re)allocation (the per-element alphas of a
    ReLU / identity layer run through the PReLU kernels): the fill used to run at every forward and
    backward - a framework fill kernel per call in the MNIST step."""
    t = ws.get(key, shape, torch.float32, dev)
    if getattr(t, "_ptg_const", None) != value:
        K.fill_(t, value)
        t._ptg_const = value
    return t


def _bf16(x, ws, key):
    if x.dtype == torch.bfloat16 or (_HOST_FP32[0] and x.device.type == "cpu"):
        return x
    out = ws.get(key, x.shape, torch.bfloat16, x.device)
    out.copy_(x)
    return out


class ConvOp(Op):
    def __init__(self, conv: L.Conv2D, prelu: L.PReLU | None, pool: L.MaxPooling2D | None):
        super().__init__()
        self.conv, self.prelu, self.pool = conv, prelu, pool
        self.params = list(conv.params) + (list(prelu.params) if prelu else [])
        conv.kernel.fwd_bf16 = True
        # the kernel gradient is NOT overwrite_grad: the store's single per-step fill zeroes it
        # together with the biases/alphas, and the wgrad kernels accumulate onto it
        self.stride = conv.strides[0]
        self.pad = conv.pad_amount()
        self.name = conv.name
        if conv.activation not in ("linear", None, "relu"):
            raise NotImplementedError(f"Conv2D activation {conv.activation}")
        if conv.activation == "relu" and prelu:
            raise NotImplementedError("Conv2D(activation='relu') followed by PReLU")
        # Conv2D(activation='relu') -> MaxPooling2D fuses as PReLU with alpha 0 + pool (the MNIST
        # convnet): the pooled output comes out of the conv epilogue, its backward is one kernel

    def _prep_input(self, x, ws):
        cp = self.conv.cin_p
        if x.shape[-1] == cp and x.dtype == torch.bfloat16:
            return x
        if x.dtype == torch.uint8 and x.shape[-1] == 3 and cp == 4:
            # raw decoded images: bilinear resize + /255 + channel pad in one device pass
            H, W = self.conv.in_shape[0], self.conv.in_shape[1]
            xi = ws.get(self.name + "/xin", (x.shape[0], H, W, cp), torch.bfloat16, x.device)
            return K.resize_norm(x.contiguous(), xi, H, W)
        xi = ws.get(self.name + "/xin", (*x.shape[:-1], cp), torch.bfloat16, x.device)
        if x.shape[-1] == 3 and cp == 4 and x.dtype == torch.float32:
            return K.pack_rgb4(x.contiguous(), xi)
        xi.zero_()
        xi[..., : x.shape[-1]] = x
        return xi

    def _halo(self):
        """(fwd/wgrad eligible, dgrad eligible) for the halo-tiled direct-conv kernels."""
        H, W, _ = self.conv.in_shape
        OH, OW, Co = self.conv.out_shape
        KS = self.conv.kernel_size[0]
        same = (OH, OW) == (H, W) and self.conv.kernel_size[0] == self.conv.kernel_size[1] and self.pad == KS // 2
        fwd = K.halo_eligible(self.conv.cin_p, Co, KS, self.stride, same)
        dgrad = K.halo_eligible(Co, self.conv.cin_p, KS, self.stride, same)
        return fwd, dgrad

    def _alpha_const(self, ws, value, dev):
        key = self.name + ("/ones" if value else "/zeros")
        return _const_buf(ws, key, self.conv.out_shape, value, dev)

    def _raw_u8_ok(self, x) -> bool:
        """Raw uint8 images straight into the sparse first-layer kernels (same size, no resize)."""
        OH, OW, Co = self.conv.out_shape
        return (RAW_U8 and SPARSE_FIRST and self.first and x.is_cuda and x.dtype == torch.uint8 and x.dim() == 4
                and x.shape[-1] == 3 and self.conv.cin_p == 4 and tuple(x.shape[1:3]) == tuple(self.conv.in_shape[:2])
                and self.conv.kernel_size == (5, 5) and self.stride == 1 and self.pad == 2 and Co == 8
                and self.pool is not None and OH % 2 == 0 and OW % 2 == 0 and self.conv.activation != "relu"
                and self._halo()[0])

    def _fused1_ok(self, x) -> bool:
        """First layer served by conv1.hip (5x5, 3(+pad) -> 8, pad 2, PReLU/ReLU/identity + 2x2 pool)."""
        OH, OW, Co = self.conv.out_shape
        if not (CONV1_FUSED and self.first and x.is_cuda and x.dim() == 4 and self.pool is not None
                and self.conv.cin_p == 4 and self.conv.kernel_size == (5, 5) and self.stride == 1
                and self.pad == 2 and Co == 8 and OH % 2 == 0 and OW % 2 == 0 and self._halo()[0]):
            return False
        if x.dtype == torch.uint8:  # raw images: only at the layer's own size (no resize pass)
            return RAW_U8 and x.shape[-1] == 3 and tuple(x.shape[1:3]) == tuple(self.conv.in_shape[:2])
        return True

    def forward(self, x, ws, training):
        self._fused1 = False
        if self._fused1_ok(x):
            x = x.contiguous() if x.dtype == torch.uint8 else self._prep_input(x, ws)
            OH, OW, Co = self.conv.out_shape
            p = ws.get(self.name + "/p", (x.shape[0], OH // 2, OW // 2, Co), torch.bfloat16, x.device)
            b = self.conv.bias.data if self.conv.bias is not None else None
            self._fused1, self._x, self._sel, self._sparse = True, x, False, False
            if CONV1_REC:
                shp = (x.shape[0], OH // 2, OW // 2, Co)
                self._zs = ws.get(self.name + "/zsel", shp, torch.bfloat16, x.device)
                self._arg = ws.get(self.name + "/arg", shp, torch.uint8, x.device)
                return K.conv1_fwd_rec(x, self.conv.kernel.bf16, b, self._pool_alpha(ws, x.device), p, self._zs,
                                       self._arg)
            self._zs = self._arg = None
            return K.conv1_fwd_pm(x, self.conv.kernel.bf16, b, self._pool_alpha(ws, x.device), p)
        if self._raw_u8_ok(x):
            x = x.contiguous()
            B = x.shape[0]
            OH, OW, Co = self.conv.out_shape
            b = self.conv.bias.data if self.conv.bias is not None else None
            self._sel = True
            self._x, self._sparse = x, True
            return self._forward_pool_sparse(x, b, ws, B, OH, OW, Co, x.device)
        x = self._prep_input(x, ws)
        B = x.shape[0]
        OH, OW, Co = self.conv.out_shape
        dev = x.device
        b = self.conv.bias.data if self.conv.bias is not None else None
        self._sparse = self._sp2 = False
        halo_ok = self._halo()[0] and not (self.pool is not None and (OH % 2 or OW % 2))
        if (SPARSE_POOL and B >= SPARSE_POOL_MIN_BATCH and halo_ok and self.pool is not None and x.is_cuda
                and not self.first and self.stride == 1
                and self.conv.kernel_size == (5, 5) and self._halo()[1]
                and K.dgrad_sparse_supported(Co, self.conv.cin_p, 5)):
            self._sel, self._sp2 = False, True
            self._x = x
            return self._forward_pool_sparse(x, b, ws, B, OH, OW, Co, dev)
        self._sel = halo_ok and self.pool is not None and x.is_cuda and self.first and SPARSE_FIRST \
            and self.conv.kernel_size[0] == 5
        if halo_ok and self.pool is not None and x.is_cuda and self._sel:
            # sparse pool record: pooled output + z at the argmax + argmax position (no full z)
            self._x, self._sparse = x, True
            return self._forward_pool_sparse(x, b, ws, B, OH, OW, Co, dev)
        z = ws.get(self.name + "/z", (B, OH, OW, Co), torch.bfloat16, dev)
        self._x, self._z = x, z
        if halo_ok:
            return self._forward_halo(x, z, b, ws, B, OH, OW, Co, dev)
        act = "relu" if self.conv.activation == "relu" else None
        K.conv2d_fwd(x, self.conv.kernel.bf16, b, self.stride, self.pad, z, act)
        if self.prelu is not None and self.pool is not None:
            p = ws.get(self.name + "/p", (B, OH // 2, OW // 2, Co), torch.bfloat16, dev)
            return K.prelu_pool_fwd(z, self.prelu.alpha.data, p)
        if self.prelu is not None:
            a = ws.get(self.name + "/a", (B, OH, OW, Co), torch.bfloat16, dev)
            return K.prelu_fwd(z, self.prelu.alpha.data, a)
        if self.pool is not None:
            ones = _const_buf(ws, self.name + "/ones", (OH, OW, Co), 1.0, dev)
            p = ws.get(self.name + "/p", (B, OH // 2, OW // 2, Co), torch.bfloat16, dev)
            return K.prelu_pool_fwd(z, ones, p)
        return z

    def _pool_alpha(self, ws, dev):
        if self.prelu is not None:
            return self.prelu.alpha.data
        if self.conv.activation == "relu":
            return self._alpha_const(ws, 0.0, dev)  # ReLU == PReLU with alpha 0
        return self._alpha_const(ws, 1.0, dev)  # identity

    def _forward_pool_sparse(self, x, b, ws, B, OH, OW, Co, dev):
        shp = (B, OH // 2, OW // 2, Co)
        p = ws.get(self.name + "/p", shp, torch.bfloat16, dev)
        zs = ws.get(self.name + "/zsel", shp, torch.bfloat16, dev)
        arg = ws.get(self.name + "/arg", shp, torch.uint8, dev)
        K.conv2d_fwd_fused(x, self.conv.kernel.bf16, b, self.pad, zs, self._pool_alpha(ws, dev), p, "pools", arg)
        self._zs, self._arg, self._zshape = zs, arg, (B, OH, OW, Co)
        return p

    def _wflip_buf(self, ws, dev):
        """This op's flipped dgrad filter [Cin][KS][KS][Cout] (bf16): owned by the op, not the
        workspace, so a fused Adam step can write it for the next backward (``flip_spec``)."""
        KS, Co = self.conv.kernel_size[0], self.conv.out_shape[-1]
        shp = (self.conv.cin_p, KS, KS, Co)
        b = getattr(self, "_wf_buf", None)
        if b is None or tuple(b.shape) != shp or b.device != torch.device(dev):
            b = self._wf_buf = torch.empty(shp, dtype=torch.bfloat16, device=dev)
        return b

    def _flips(self) -> bool:
        return not self.first and self.stride == 1 and self.conv.kernel.bf16.is_cuda and self._halo()[1]

    def dgrad_flip_job(self, ws):
        """(weights, flip buffer) when this op's backward runs the halo dgrad on the GPU, else None."""
        if not self._flips():
            return None
        return self.conv.kernel.bf16, self._wflip_buf(ws, self.conv.kernel.bf16.device)

    def flip_spec(self):
        """(flip buffer, flat offset, Cout, KS, Cin) for an optimizer pass that writes this op's
        flipped dgrad filter from the updated weights (ops.nn.adam_multi), else None."""
        if not self._flips():
            return None
        k = self.conv.kernel
        Cout, KS, _, Cin = k.shape
        return self._wflip_buf(None, k.bf16.device), k.offset, Cout, KS, Cin

    def _backward_sel(self, x, dy, ws, dev):
        """First layer: sparse record -> dZ record -> weight gradient (no dense z / dZ, no dgrad)."""
        C = self._zshape[-1]
        bias_g = self.conv.bias.grad if self.conv.bias is not None else \
            ws.get(self.name + "/nobias", (C,), torch.float32, dev)
        dalpha = self.prelu.alpha.grad if self.prelu is not None else \
            ws.get(self.name + "/dalpha_dummy", self._zshape[1:], torch.float32, dev)
        dzs = ws.get(self.name + "/dzsel", self._zs.shape, torch.bfloat16, dev)
        K.prelu_pool_bwd_sel(dy, self._zs, self._arg, self._pool_alpha(ws, dev), dzs, dalpha, bias_g)
        K.conv2d_wgrad_halo_sparse(x, dzs, self._arg, self.pad, self.conv.kernel.grad, zeroed=True)
        return None

    def _backward_sparse_record(self, x, dy, ws, dev):
        """Pooled layer with a sparse record (SPARSE_POOL): dZ at each window's argmax, then the
        weight gradient (side stream) and the data gradient both expand it in their loaders."""
        C = self._zshape[-1]
        bias_g = self.conv.bias.grad if self.conv.bias is not None else \
            ws.get(self.name + "/nobias", (C,), torch.float32, dev)
        dalpha = self.prelu.alpha.grad if self.prelu is not None else \
            ws.get(self.name + "/dalpha_dummy", self._zshape[1:], torch.float32, dev)
        dzs = ws.get(self.name + "/dzsel", self._zs.shape, torch.bfloat16, dev)
        arg = self._arg
        K.prelu_pool_bwd_sel(dy, self._zs, arg, self._pool_alpha(ws, dev), dzs, dalpha, bias_g)
        g = self.conv.kernel.grad
        S.launch(lambda: K.conv2d_wgrad_halo_sparse(x, dzs, arg, self.pad, g, zeroed=True), dev)
        dx = ws.get(self.name + "/dx", x.shape, torch.bfloat16, dev)
        K.conv2d_dgrad_halo_sparse(dzs, arg, self.conv.kernel.bf16, self.pad, dx, self._wflip_buf(ws, dev),
                                   flipped=getattr(self, "_wf_ready", False))
        return dx

    def _backward_fused1(self, x, dy, ws, dev):
        """First layer, conv1.hip: one kernel from the pooled gradient to dW / dalpha / dbias."""
        OH, OW, Co = self.conv.out_shape
        bias_g = self.conv.bias.grad if self.conv.bias is not None else \
            ws.get(self.name + "/nobias", (Co,), torch.float32, dev)
        dalpha = self.prelu.alpha.grad if self.prelu is not None else \
            ws.get(self.name + "/dalpha_dummy", (OH, OW, Co), torch.float32, dev)
        if getattr(self, "_zs", None) is not None:
            K.conv1_bwd_rec(x, self._pool_alpha(ws, dev), dy, self._zs, self._arg, self.conv.kernel.grad, dalpha, bias_g)
            return None
        b = self.conv.bias.data if self.conv.bias is not None else None
        K.conv1_bwd_pm(x, self.conv.kernel.bf16, b, self._pool_alpha(ws, dev), dy, self.conv.kernel.grad, dalpha,
                       bias_g)
        return None

    def _forward_halo(self, x, z, b, ws, B, OH, OW, Co, dev):
        """One kernel: conv + bias, and the PReLU/ReLU (+ 2x2 max-pool) epilogue fused in."""
        w = self.conv.kernel.bf16
        if self.prelu is not None:
            alpha = self.prelu.alpha.data
        elif self.conv.activation == "relu":
            alpha = self._alpha_const(ws, 0.0, dev)  # ReLU == PReLU with alpha 0
        elif self.pool is not None:
            alpha = self._alpha_const(ws, 1.0, dev)  # identity
        else:
            return K.conv2d_fwd_fused(x, w, b, self.pad, z)
        if self.pool is not None:
            p = ws.get(self.name + "/p", (B, OH // 2, OW // 2, Co), torch.bfloat16, dev)
            K.conv2d_fwd_fused(x, w, b, self.pad, z, alpha, p, "pool")
            return p
        a = ws.get(self.name + "/a", (B, OH, OW, Co), torch.bfloat16, dev)
        K.conv2d_fwd_fused(x, w, b, self.pad, z, alpha, a, "prelu")
        return a

    def backward(self, dy, ws):
        x = self._x
        dev = x.device
        dy = _bf16(dy, ws, self.name + "/dy16")
        if getattr(self, "_fused1", False):
            return self._backward_fused1(x, dy, ws, dev)
        if getattr(self, "_sel", False):
            return self._backward_sel(x, dy, ws, dev)
        if getattr(self, "_sp2", False):
            return self._backward_sparse_record(x, dy, ws, dev)
        zshape = self._zshape if self._sparse else self._z.shape
        dz = ws.get(self.name + "/dz", zshape, torch.bfloat16, dev)
        bias_g = self.conv.bias.grad if self.conv.bias is not None else \
            ws.get(self.name + "/nobias", (zshape[-1],), torch.float32, dev)
        z = self._z if not self._sparse else None
        if self._sparse:
            if self.prelu is not None:
                dalpha = self.prelu.alpha.grad
            else:
                dalpha = ws.get(self.name + "/dalpha_dummy", zshape[1:], torch.float32, dev)
            K.prelu_pool_bwd_sparse(dy, self._zs, self._arg, self._pool_alpha(ws, dev), dz, dalpha, bias_g)
        elif self.prelu is not None and self.pool is not None:
            K.prelu_pool_bwd(dy, z, self.prelu.alpha.data, dz, self.prelu.alpha.grad, bias_g)
        elif self.prelu is not None:
            K.prelu_bwd(dy, z, self.prelu.alpha.data, dz, self.prelu.alpha.grad, bias_g)
        elif self.pool is not None:
            # identity (alpha 1) or ReLU (alpha 0: z is pre-activation on the halo path, post-ReLU on the
            # generic one - the same mask and argmax either way)
            dummy = ws.get(self.name + "/dalpha_dummy", z.shape[1:], torch.float32, dev)
            K.prelu_pool_bwd(dy, z, self._pool_alpha(ws, dev), dz, dummy, bias_g)
        elif self.conv.activation == "relu":
            zeros = ws.get(self.name + "/zeros", z.shape[1:], torch.float32, dev, zero=True)
            dummy = ws.get(self.name + "/dalpha_dummy", z.shape[1:], torch.float32, dev)
            K.prelu_bwd(dy, z, zeros, dz, dummy, bias_g)
        else:
            dz = dy
            K.col_sum(dz.reshape(-1, dz.shape[-1]), bias_g)
        halo_fwd, halo_dgrad = self._halo()
        g = self.conv.kernel.grad
        if halo_fwd:
            S.launch(lambda: K.conv2d_wgrad_halo(x, dz, self.pad, g, zeroed=True), dev)
        else:
            S.launch(lambda: K.conv2d_wgrad(x, dz, self.stride, self.pad, g, accumulate=True), dev)
        if self.first:
            return None
        return self._dgrad(x, dz, ws, dev, halo_dgrad)

    def _dgrad(self, x, dz, ws, dev, halo_dgrad):
        if self.stride != 1:
            raise NotImplementedError("dgrad for strided convolutions")
        dx = ws.get(self.name + "/dx", x.shape, torch.bfloat16, dev)
        if halo_dgrad:
            wf = self._wflip_buf(ws, dev)
            K.conv2d_dgrad_halo(dz, self.conv.kernel.bf16, self.pad, dx, wf,
                                flipped=getattr(self, "_wf_ready", False))
        else:
            K.conv2d_dgrad(dz, self.conv.kernel.bf16, self.pad, dx)
        return dx


class DenseOp(Op):
    def __init__(self, dense: L.Dense):
        super().__init__()
        self.dense = dense
        self.params = list(dense.params)
        self.name = dense.name
        N, Kd = dense.units, dense.fan_in
        self.big = N > 64 and N % 8 == 0 and Kd % 8 == 0
        if self.big:
            dense.kernel.overwrite_grad = True
            dense.kernel.fwd_bf16 = True
        self.act = dense.activation
        self.logits_only = False  # softmax folded into the loss
        self.fused_update = None  # optimizers.FusedAdamStep during a fused-update training step

    def forward(self, x, ws, training):
        x = x.reshape(x.shape[0], -1)
        B = x.shape[0]
        N = self.dense.units
        dev = x.device
        b = self.dense.bias.data if self.dense.bias is not None else None
        act = None if (self.logits_only and self.act == "softmax") else self.act
        if self.big:
            x = _bf16(x, ws, self.name + "/x16")
            y = ws.get(self.name + "/y", (B, N), torch.bfloat16, dev)
            # created zeroed and cleared again by the bias/activation pass after each use
            wsp = ws.get(self.name + "/splitk", (B * N,), torch.float32, dev, zero=True)
            K.linear_fwd(x, self.dense.kernel.bf16, b, act, y, workspace=wsp, workspace_zeroed=True)
        else:
            y = ws.get(self.name + "/y", (B, N), torch.float32, dev)
            K.dense_small_fwd(x, self.dense.kernel.data, b, act, y)
        self._x, self._y = x, y
        return y

    def forward_splitk_sums(self, x, ws):
        """Big Dense forward that stops at the fp32 split-K sums (no bias / activation): the fused
        regression head (head_mse_k) finishes the layer and re-zeroes the buffer for the next step."""
        x = x.reshape(x.shape[0], -1)
        B = x.shape[0]
        N, Kd = self.dense.units, self.dense.fan_in
        x = _bf16(x, ws, self.name + "/x16")
        # zeroed when (re)allocated; afterwards the head kernel leaves it zero after every step
        acc = ws.get(self.name + "/headacc", (B, N), torch.float32, x.device, zero=True)
        if not x.is_cuda:
            acc.add_(x.float() @ self.dense.kernel.bf16.float().t())
            self._x = x
            return acc
        w = self.dense.kernel.bf16
        S = K.dense_fwd_splits(B, N, Kd) if (DENSE_FWD_SPLITS <= 0 and x.dtype == torch.bfloat16
                                             and x.is_contiguous()) else 0
        if S > 0:
            # weight-streaming forward: S split-K partial slices with plain stores (no zeroed
            # accumulator, no atomics); the head / bias pass sums them
            part = ws.get(self.name + "/headparts", (S, B, N), torch.float32, x.device)
            K.dense_fwd_parts(x, w, part, S)
            self._x = x
            return part
        tiles = -(-B // 128) * -(-N // 128)
        # ~512 workgroups, <= 32 splits of >= 640 (CNN-B1 b32: 32 splits 0.645/0.657 vs 16 splits
        # 0.660/0.667 ms; b256 keeps 16 - 8/12 within noise, 4/6/20/32 slower: r4_ab_dense_fwd_splits.txt)
        splits = 1 if Kd < 4096 else max(1, min(32, 512 // max(tiles, 1), Kd // 640))
        if DENSE_FWD_SPLITS > 0:
            splits = min(int(DENSE_FWD_SPLITS), max(1, Kd // 64))
        K.gemm(B, N, Kd, x, Kd, 1, self.dense.kernel.bf16, Kd, 1, 3, acc, N, None, 0, splits)
        self._x = x
        return acc

    def backward_dz(self, dz, ws):
        """Big Dense backward from the pre-activation gradient dz (bias gradient already summed):
        dX (unless first) then dW, or Adam fused into the dW GEMM."""
        x = self._x
        dx = None
        if not self.first:
            dx = ws.get(self.name + "/dx", x.shape, torch.bfloat16, x.device)
            K.linear_dx(dz, self.dense.kernel.bf16, dx)
        fused = self.fused_update
        if fused is not None and (dz.is_cuda or getattr(fused, "cpu_ok", False)):
            fused.linear_dw(dz, x, self.dense.kernel)
        else:
            g = self.dense.kernel.grad
            S.launch(lambda: K.linear_dw(dz, x, g), dz.device)
        return dx

    def backward(self, dy, ws):
        x, y = self._x, self._y
        dev = y.device
        B, N = y.shape
        if self.big:
            if self.act == "relu" and not self.grad_masked_by_next:
                dz = ws.get(self.name + "/dz", (B, N), torch.bfloat16, dev)
                K.relu_bwd(dy, y, dz)
            else:
                dz = _bf16(dy, ws, self.name + "/dz16")
            if self.dense.bias is not None:
                K.col_sum(dz, self.dense.bias.grad)
            fused = self.fused_update
            dx = None
            if not self.first:
                # before the weight update below: dX reads this step's (pre-update) bf16 weights
                dx = ws.get(self.name + "/dx", x.shape, torch.bfloat16, dev)
                K.linear_dx(dz, self.dense.kernel.bf16, dx)
            if fused is not None and (dz.is_cuda or getattr(fused, "cpu_ok", False)):
                fused.linear_dw(dz, x, self.dense.kernel)  # Adam in the wgrad epilogue
            else:
                g = self.dense.kernel.grad
                S.launch(lambda: K.linear_dw(dz, x, g), dev)
            return dx
        # skinny path (fp32 math)
        if self.act == "relu" and not self.grad_masked_by_next:
            dz = ws.get(self.name + "/dz", (B, N), torch.float32, dev)
            K.relu_bwd(dy, y, dz)
        elif dy.dtype != torch.float32:
            dz = dy.float()
        else:
            dz = dy
        db = self.dense.bias.grad if self.dense.bias is not None else None
        K.dense_small_dw(dz, x, self.dense.kernel.grad, db)
        if self.first:
            return None
        mask = self._prev_y if self.mask_for_prev else None
        out_dtype = torch.bfloat16 if getattr(self, "_prev_big", False) or x.dtype == torch.bfloat16 else torch.float32
        dx = ws.get(self.name + "/dx", x.shape, out_dtype, dev)
        K.dense_small_dx(dz, self.dense.kernel.data, mask, dx)
        return dx


DENSE_FWD_SPLITS = config.get("dense_fwd_splits")


class FlattenOp(Op):
    def __init__(self, layer):
        super().__init__()
        self.name = layer.name

    def forward(self, x, ws, training):
        self._shape = x.shape
        return x.reshape(x.shape[0], -1)

    def backward(self, dy, ws):
        return dy.reshape(self._shape)


class GAPOp(Op):
    def __init__(self, layer):
        super().__init__()
        self.name = layer.name

    def forward(self, x, ws, training):
        x = _bf16(x, ws, self.name + "/x16")
        self._xshape = x.shape
        out = ws.get(self.name + "/y", (x.shape[0], x.shape[-1]), torch.float32, x.device)
        return K.gap_fwd(x, out)

    def backward(self, dy, ws):
        dx = ws.get(self.name + "/dx", self._xshape, torch.bfloat16, dy.device)
        return K.gap_bwd(dy.float().contiguous(), dx)


class PReLUOp(Op):
    def __init__(self, layer: L.PReLU):
        super().__init__()
        self.layer = layer
        self.params = list(layer.params)
        self.name = layer.name

    def forward(self, x, ws, training):
        x = _bf16(x, ws, self.name + "/x16")
        self._z = x
        a = ws.get(self.name + "/a", x.shape, torch.bfloat16, x.device)
        return K.prelu_fwd(x, self.layer.alpha.data, a)

    def backward(self, dy, ws):
        z = self._z
        dy = _bf16(dy, ws, self.name + "/dy16")
        dz = ws.get(self.name + "/dz", z.shape, torch.bfloat16, z.device)
        dummy_b = ws.get(self.name + "/db", (z.shape[-1],), torch.float32, z.device)
        return K.prelu_bwd(dy, z, self.layer.alpha.data, dz, self.layer.alpha.grad, dummy_b)


class PoolOp(Op):
    def __init__(self, layer):
        super().__init__()
        self.name = layer.name

    def forward(self, x, ws, training):
        x = _bf16(x, ws, self.name + "/x16")
        self._z = x
        B, H, W, C = x.shape
        ones = _const_buf(ws, self.name + "/ones", (H, W, C), 1.0, x.device)
        p = ws.get(self.name + "/p", (B, H // 2, W // 2, C), torch.bfloat16, x.device)
        return K.prelu_pool_fwd(x, ones, p)

    def backward(self, dy, ws):
        z = self._z
        dy = _bf16(dy, ws, self.name + "/dy16")
        ones = ws.get(self.name + "/ones", z.shape[1:], torch.float32, z.device)
        dummy = ws.get(self.name + "/dalpha", z.shape[1:], torch.float32, z.device)
        dummy_b = ws.get(self.name + "/db", (z.shape[-1],), torch.float32, z.device)
        dz = ws.get(self.name + "/dz", z.shape, torch.bfloat16, z.device)
        return K.prelu_pool_bwd(dy, z, ones, dz, dummy, dummy_b)


class ReLUOp(Op):
    def __init__(self, layer):
        super().__init__()
        self.name = layer.name

    def forward(self, x, ws, training):
        y = ws.get(self.name + "/y", x.shape, x.dtype, x.device)
        y.copy_(torch.relu(x)) if not x.is_cuda else K.relu_bwd(x, x, y)
        self._y = y
        return y

    def backward(self, dy, ws):
        dz = ws.get(self.name + "/dz", dy.shape, dy.dtype, dy.device)
        return K.relu_bwd(dy, self._y, dz)


def lower(layers: list) -> list:
    """Fuse a built layer list into device ops."""
    ops = []
    i = 0
    seq = [l for l in layers if not isinstance(l, L.Input)]
    while i < len(seq):
        l = seq[i]
        if isinstance(l, L.Conv2D):
            prelu = pool = None
            j = i + 1
            if j < len(seq) and isinstance(seq[j], L.PReLU) and l.activation in ("linear", None):
                prelu = seq[j]; j += 1
            if j < len(seq) and isinstance(seq[j], L.MaxPooling2D) and l.activation in ("linear", None, "relu") \
                    and tuple(seq[j].pool_size) == (2, 2) and tuple(seq[j].strides) == (2, 2):
                pool = seq[j]; j += 1
            ops.append(ConvOp(l, prelu, pool))
            i = j
        elif isinstance(l, L.Dense):
            ops.append(DenseOp(l)); i += 1
        elif isinstance(l, L.Flatten):
            ops.append(FlattenOp(l)); i += 1
        elif isinstance(l, L.GlobalAveragePooling2D):
            ops.append(GAPOp(l)); i += 1
        elif isinstance(l, L.PReLU):
            ops.append(PReLUOp(l)); i += 1
        elif isinstance(l, L.MaxPooling2D):
            ops.append(PoolOp(l)); i += 1
        elif isinstance(l, L.ReLU):
            ops.append(ReLUOp(l)); i += 1
        else:
            raise NotImplementedError(type(l).__name__)
    if ops:
        ops[0].first = True
    for k in range(1, len(ops)):
        ops[k].below = ops[k - 1]
    # ReLU-mask hand-off: a skinny Dense applies the previous relu-Dense's mask in its dX
    for k in range(1, len(ops)):
        cur, prev = ops[k], ops[k - 1]
        if isinstance(cur, DenseOp) and not cur.big and isinstance(prev, DenseOp) and prev.act == "relu":
            cur.mask_for_prev = True
            cur._prev_big = prev.big
            prev.grad_masked_by_next = True
            cur._prev_op = prev
    return ops


def run_forward(ops, x, ws, training=True, pre_op=None):
    for k, op in enumerate(ops):
        if pre_op is not None:
            pre_op(op)  # e.g. wait for this op's parameter all-gather (sharded data-parallel update)
        if isinstance(op, DenseOp) and op.mask_for_prev:
            op._prev_y = op._prev_op._y if hasattr(op, "_prev_op") else None
        x = op.forward(x, ws, training)
        if isinstance(op, DenseOp) and k + 1 < len(ops):
            nxt = ops[k + 1]
            if isinstance(nxt, DenseOp) and nxt.mask_for_prev:
                nxt._prev_y = op._y
    return x


def run_backward(ops, dy, ws, on_op_done=None, flips_ready=()):
    # every halo dgrad filter of this pass flipped by one launch up front (weights are fixed until
    # the optimizer step that follows the backward); ``flips_ready``: ops whose flipped filter the
    # last optimizer pass already wrote from these very weights (ops.nn.adam_multi)
    jobs = []
    for op in ops:
        if isinstance(op, ConvOp):
            job = op.dgrad_flip_job(ws)
            op._wf_ready = job is not None
            if job is not None and op.name not in flips_ready:
                jobs.append(job)
    if jobs:
        K.conv_flip_weights_multi(jobs)
    for op in reversed(ops):
        dy = op.backward(dy, ws)
        if on_op_done is not None:
            on_op_done(op)
    return dy
