"""Neural-network ops: GPU tensors run the hand-written gfx950 kernels (csrc/kernels/*.hip);
CPU tensors run the fp32 PyTorch reference in :mod:`.reference` (the ``local`` host path and
the numerics oracle of the tests).  There is no silent fallback: a GPU tensor with the HIP
library missing raises.

Layouts: activations NHWC bf16; conv filters [Cout][KH][KW][Cin]; dense weights [out][in];
master parameters / gradients fp32.
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch

from . import reference as ref
from ._util import hip, need, on_device, ptr, stream_handle
from .. import config

# prelu+pool backward kernel: "sg" = sample-parallel blocks with an in-LDS dalpha reduction
# (prelu_pool_bwd_sg_k), "chunk" = position-parallel blocks adding dalpha partials with atomics

ACT = {None: 0, "linear": 0, "none": 0, "relu": 1, "softmax": 2}


def conv_out_size(h: int, k: int, stride: int, pad: int) -> int:
    return (h + 2 * pad - k) // stride + 1


# ----------------------------------------------------------------------------------------------
# Convolution (implicit GEMM on MFMA)
# ----------------------------------------------------------------------------------------------
def conv2d_fwd(x, w, bias, stride: int, pad: int, out, act: str | None = None):
    """out[N,OH,OW,Cout] (bf16) = act(conv(x, w) + bias)."""
    if not on_device(x):
        return ref.conv2d_fwd(x, w, bias, stride, pad, out, act)
    N, H, W, C = x.shape
    Cout, KH, KW, Cw = w.shape
    assert Cw == C, (w.shape, x.shape)
    OH, OW = conv_out_size(H, KH, stride, pad), conv_out_size(W, KW, stride, pad)
    assert tuple(out.shape) == (N, OH, OW, Cout), (out.shape, (N, OH, OW, Cout))
    need(x, torch.bfloat16, "conv2d_fwd.x"); need(w, torch.bfloat16, "conv2d_fwd.w")
    need(out, torch.bfloat16, "conv2d_fwd.out")
    hip("ptg_conv2d_fwd", ptr(x), ptr(w), ptr(bias), ptr(out), N, H, W, C, Cout, KH, KW, stride, pad,
        OH, OW, ACT[act])
    return out


def conv2d_dgrad(dz, w, pad: int, out, accumulate: bool = False):
    """out[N,H,W,Cin] (+)= d(conv)/dx for a stride-1 convolution."""
    if not on_device(dz):
        if accumulate:
            tmp = torch.empty_like(out, dtype=torch.float32)
            ref.conv2d_dgrad(dz, w, pad, tmp)
            out.copy_((out.float() + tmp).to(out.dtype))
            return out
        return ref.conv2d_dgrad(dz, w, pad, out)
    N, H, W, Cout = dz.shape
    Cw, KH, KW, Cin = w.shape
    assert Cw == Cout and tuple(out.shape) == (N, H, W, Cin)
    need(dz, torch.bfloat16, "dgrad.dz"); need(out, torch.bfloat16, "dgrad.out")
    hip("ptg_conv2d_dgrad", ptr(dz), ptr(w), ptr(out), N, H, W, Cin, Cout, KH, KW, pad, int(accumulate))
    return out


def conv_dgrad_bnstats(dz, w, pad: int, out, part, z_blk, scale=None, shift=None) -> bool:
    """Stride-1 data gradient whose output feeds a Conv -> BN (-> ReLU) block (gemm.hip EpiBf16
    backward form): ``out`` = the gradient masked by the block's ReLU (relu(z_blk*scale + shift) > 0;
    no mask when ``scale`` is None) and ``part`` ([64, 2, Cin] fp32, accumulated into) += the block's BN
    backward sums (sum g, sum g*z_blk), i.e. what bn_bwd_reduce would compute.  Returns False (nothing
    launched) when the shape is not served by the fused GEMM paths."""
    if not on_device(dz):
        return False
    N, H, W, Cout = dz.shape
    Cw, KH, KW, Cin = w.shape
    if (tuple(out.shape) != (N, H, W, Cin) or tuple(z_blk.shape) != tuple(out.shape) or Cin % 8 or Cin >= 4096
            or Cw != Cout or part.dtype != torch.float32):
        return False
    for t in (dz, out, z_blk):
        if t.dtype != torch.bfloat16 or not t.is_contiguous():
            return False
    sc, sh = (ptr(scale), ptr(shift)) if scale is not None else (None, None)
    if KH == KW == 1 and pad == 0:
        if Cout % 8:
            return False
        hip("ptg_conv1x1_dgrad_bnstats", ptr(dz), ptr(w), ptr(out), N, H, W, Cin, Cout, ptr(part), ptr(z_blk), sc, sh)
        return True
    if Cout < 8 or Cout & (Cout - 1):
        return False
    hip("ptg_conv2d_dgrad_bnstats", ptr(dz), ptr(w), ptr(out), N, H, W, Cin, Cout, KH, KW, pad, ptr(part),
        ptr(z_blk), sc, sh)
    return True


def conv1x1_dgrad(dz, w, stride: int, out, accumulate: bool = False):
    """out[N,H,W,Cin] (+)= d/dx of a 1x1 convolution with stride ``stride`` (pad 0).  With
    stride > 1 and accumulate=False the off-lattice pixels are zeroed here."""
    N, OH, OW, Cout = dz.shape
    Cw, KH, KW, Cin = w.shape
    _, H, W, _ = out.shape
    assert KH == KW == 1 and Cw == Cout and out.shape[-1] == Cin
    if not on_device(dz):
        g = (_f32(dz).reshape(-1, Cout) @ _f32(w).reshape(Cout, Cin)).reshape(N, OH, OW, Cin)
        full = torch.zeros(out.shape, dtype=torch.float32)
        full[:, : OH * stride: stride, : OW * stride: stride] = g
        if accumulate:
            full += out.float()
        out.copy_(full.to(out.dtype))
        return out
    need(dz, torch.bfloat16, "dgrad1x1.dz"); need(out, torch.bfloat16, "dgrad1x1.out")
    if stride > 1 and not accumulate:
        out.zero_()  # the remapped epilogue then writes only the stride lattice
    hip("ptg_conv1x1_dgrad", ptr(dz), ptr(w), ptr(out), N, OH, OW, H, W, Cin, Cout, stride, int(accumulate))
    return out


def _f32(t):
    return t.float()


def conv2d_wgrad(x, dz, stride: int, pad: int, out, accumulate: bool = False, splits: int = 0):
    """out[Cout,KH,KW,C] (fp32) (+)= d(conv)/dw."""
    if not on_device(x):
        return ref.conv2d_wgrad(x, dz, stride, pad, out, accumulate)
    N, H, W, C = x.shape
    _, OH, OW, Cout = dz.shape
    Co, KH, KW, Cw = out.shape
    assert Co == Cout and Cw == C
    need(out, torch.float32, "wgrad.out")
    if not accumulate:
        out.zero_()
    hip("ptg_conv2d_wgrad", ptr(x), ptr(dz), ptr(out), N, H, W, C, Cout, KH, KW, stride, pad, OH, OW, splits)
    return out


HALO_C = (4, 8, 16, 32, 64)


def halo_eligible(C: int, Cout: int, KS: int, stride: int, same: bool) -> bool:
    """Shapes served by the halo-tiled direct-conv kernels (csrc/kernels/conv.hip)."""
    return same and stride == 1 and KS in (3, 5) and C in HALO_C and Cout % 8 == 0 and Cout <= 64


EPI = {None: 0, "pool": 1, "prelu": 2, "pools": 3, "ppb": 4}


def conv2d_fwd_fused(x, w, bias, pad: int, z_out, alpha=None, aux_out=None, epi=None, arg_out=None):
    """Halo-tiled 'same' conv: z = conv(x, w) + bias; epi='pool' also writes
    aux = maxpool2x2(prelu(z, alpha)); epi='prelu' writes aux = prelu(z, alpha).  epi='pools'
    (sparse pool, GPU only) writes aux = the pooled output, z_out = z at each window's argmax
    ([N,H/2,W/2,C]) and arg_out = the argmax position q = 2*dh + dw (uint8) instead of full z."""
    if not on_device(x) and epi == "pools":
        N, H, W, _ = x.shape
        full = torch.empty((N, H, W, w.shape[0]), dtype=z_out.dtype)
        ref.conv2d_fwd(x, w, bias, 1, pad, full, None)
        return ref.prelu_pool_fwd_sparse(full, alpha, aux_out, z_out, arg_out)
    if not on_device(x):
        ref.conv2d_fwd(x, w, bias, 1, pad, z_out, None)
        if epi == "pool":
            ref.prelu_pool_fwd(z_out, alpha, aux_out)
        elif epi == "prelu":
            ref.prelu_fwd(z_out, alpha, aux_out)
        return z_out
    N, H, W, C = x.shape
    Cout, KS, _, Cw = w.shape
    if x.dtype == torch.uint8:  # raw [N,H,W,3] images: the first-layer kernel packs them itself
        if not (epi == "pools" and C == 3 and Cw == 4 and KS == 5 and Cout == 8 and pad == 2):
            raise ValueError("conv2d_fwd_fused: uint8 input only for the 5x5 -> 8 sparse-pool first layer")
        assert tuple(z_out.shape) == (N, H // 2, W // 2, Cout) and tuple(arg_out.shape) == tuple(z_out.shape)
        need(w, torch.bfloat16, "conv1_u8.w")
        hip("ptg_conv1_pool_sparse_u8", ptr(x), ptr(w), ptr(bias), ptr(alpha), ptr(z_out), ptr(aux_out), ptr(arg_out),
            N, H, W)
        return aux_out
    if epi == "pools":
        assert tuple(z_out.shape) == (N, H // 2, W // 2, Cout) and arg_out is not None
        assert arg_out.dtype == torch.uint8 and tuple(arg_out.shape) == tuple(z_out.shape)
        assert tuple(aux_out.shape) == tuple(z_out.shape)
    else:
        assert tuple(z_out.shape) == (N, H, W, Cout)
    assert Cw == C
    need(x, torch.bfloat16, "conv_halo.x"); need(w, torch.bfloat16, "conv_halo.w")
    if (CONV32 and epi in (None, "pool", "prelu") and KS == 5 and pad == 2 and _conv32_ok(H, W, C, Cout, epi)
            and W > 0 and N * (H // max(1, 320 // W)) >= CONV32_MIN_WG):
        # channel-rich 5x5 layers (and data gradients): the 32x32x16-MFMA implicit GEMM (conv32.hip)
        return conv32(x, w, bias, z_out, alpha, aux_out, epi)
    hip("ptg_conv2d_fwd_halo", ptr(x), ptr(w), ptr(bias), ptr(alpha), ptr(z_out), ptr(aux_out), ptr(arg_out), N, H, W,
        C, Cout, KS, pad, EPI[epi])
    return z_out


EPI32 = {None: 0, "z": 0, "pool": 1, "prelu": 2}
CONV32 = config.get("conv32")
CONV32_MINCH = config.get("conv32_min_ch")
# conv32 runs one workgroup per 320-pixel tile (N * H / (320 / W) of them): below one per CU (CNN-B1
# layer 5 at batch < 256) the persistent strip kernels fill the GPU better (b32: 91 vs ~12 us)
CONV32_MIN_WG = config.get("conv32_min_wg")
_C32_OK: dict = {}


def _conv32_ok(H, W, C, Cout, epi) -> bool:
    key = (H, W, C, Cout, epi)
    v = _C32_OK.get(key)
    if v is None:
        v = _C32_OK[key] = min(C, Cout) >= CONV32_MINCH and conv32_supported(H, W, C, Cout, 5, 2, epi)
    return v


def conv32_supported(H: int, W: int, C: int, Cout: int, KS: int, pad: int, epi=None) -> bool:
    """The 32x32x16-MFMA implicit-GEMM conv (conv32.hip) covers this 5x5 'same' shape."""
    from .. import _native

    return bool(_native.hip_lib().ptg_conv32_supported(H, W, C, Cout, KS, pad, EPI32[epi]))


def conv32(x, w, bias, z_out, alpha=None, aux_out=None, epi=None):
    """z = conv5x5(x, w) + bias (stride 1, pad 2) on the 32x32x16 MFMA kernel (conv32.hip);
    epi "pool": aux = maxpool2x2(prelu(z, alpha)); "prelu": aux = prelu(z, alpha).  For a data
    gradient pass dz as x and the flipped filter [Cin][5][5][Cout] as w."""
    if not on_device(x):
        ref.conv2d_fwd(x, w, bias, 1, 2, z_out, None)
        if epi == "pool":
            ref.prelu_pool_fwd(z_out, alpha, aux_out)
        elif epi == "prelu":
            ref.prelu_fwd(z_out, alpha, aux_out)
        return z_out
    N, H, W, C = x.shape
    Cout = w.shape[0]
    assert tuple(w.shape) == (Cout, 5, 5, C) and tuple(z_out.shape) == (N, H, W, Cout), (x.shape, w.shape, z_out.shape)
    need(x, torch.bfloat16, "conv32.x"); need(w, torch.bfloat16, "conv32.w"); need(z_out, torch.bfloat16, "conv32.z")
    if epi == "pool":
        assert aux_out is not None and tuple(aux_out.shape) == (N, H // 2, W // 2, Cout)
    elif epi == "prelu":
        assert aux_out is not None and tuple(aux_out.shape) == (N, H, W, Cout)
    hip("ptg_conv32", ptr(x), ptr(w), ptr(bias), ptr(alpha), ptr(z_out), ptr(aux_out), N, H, W, C, Cout, EPI32[epi])
    return z_out


def conv2d_wgrad_halo(x, dz, pad: int, out, zeroed: bool = False):
    """out[Cout,KS,KS,C] (fp32) = d(conv)/dw for a stride-1 'same' conv (halo-tiled MFMA).
    ``zeroed``: ``out`` already holds zeros (the parameter store's one per-step gradient fill), so
    the kernel's atomic partial sums land on it directly."""
    if not on_device(x):
        return ref.conv2d_wgrad(x, dz, 1, pad, out, False)
    N, H, W, C = x.shape
    Cout, KS, _, _ = out.shape
    if not zeroed:
        out.zero_()
    hip("ptg_conv2d_wgrad_halo", ptr(x), ptr(dz), ptr(out), N, H, W, C, Cout, KS, pad)
    return out


def conv2d_wgrad_halo_sparse(x, dzsel, arg, pad: int, out, zeroed: bool = False):
    """out[Cout,KS,KS,C] (fp32) = d(conv)/dw with dZ given as its sparse pool record (dzsel / arg of
    shape [N,H/2,W/2,Cout]: dZ at each 2x2 window's argmax, zero elsewhere)."""
    N, H, W, C = x.shape
    Cout, KS, _, _ = out.shape
    if not on_device(x):
        dz = ref.expand_pool_record(dzsel, arg, (N, H, W, Cout)).to(dzsel.dtype)
        return ref.conv2d_wgrad(x, dz, 1, pad, out, zeroed)
    assert tuple(dzsel.shape) == (N, H // 2, W // 2, Cout) and tuple(arg.shape) == tuple(dzsel.shape)
    if x.dtype == torch.uint8:  # raw [N,H,W,3] images (first layer, see conv2d_fwd_fused)
        if not (C == 3 and KS == 5 and Cout == 8 and pad == 2 and out.shape[-1] == 4):
            raise ValueError("conv2d_wgrad_halo_sparse: uint8 input only for the 5x5 -> 8 first layer")
        need(dzsel, torch.bfloat16, "wgrad_u8.dzsel"); need(arg, torch.uint8, "wgrad_u8.arg")
        need(out, torch.float32, "wgrad_u8.out")
        if not zeroed:
            out.zero_()
        hip("ptg_conv1_wgrad_sparse_u8", ptr(x), ptr(dzsel), ptr(arg), ptr(out), N, H, W, Cout)
        return out
    need(x, torch.bfloat16, "wgrad_sparse.x"); need(dzsel, torch.bfloat16, "wgrad_sparse.dzsel")
    need(arg, torch.uint8, "wgrad_sparse.arg"); need(out, torch.float32, "wgrad_sparse.out")
    if not zeroed:
        out.zero_()
    hip("ptg_conv2d_wgrad_halo_sparse", ptr(x), ptr(dzsel), ptr(arg), ptr(out), N, H, W, C, Cout, KS, pad)
    return out


def _conv_shape(x, w, stride, pad):
    N, H, W, C = x.shape
    Co, KH, KW, Cw = w.shape
    assert Cw == C, (w.shape, x.shape)
    return N, H, W, C, Co, KH, KW, (H + 2 * pad - KH) // stride + 1, (W + 2 * pad - KW) // stride + 1


def conv_bn_fwd(x, w, bias, stride: int, pad: int, z, stats=None):
    """z = conv(x, w) + bias (implicit-GEMM MFMA conv, gemm.hip ptg_conv_bn_fwd); ``stats`` ([64, 2,
    Cout] fp32): the batch statistics (sum, sum of squares) of the stored z are added in the epilogue."""
    N, H, W, C, Co, KH, KW, OH, OW = _conv_shape(x, w, stride, pad)
    assert tuple(z.shape) == (N, OH, OW, Co), (z.shape, (N, OH, OW, Co))
    if not on_device(x):
        ref.conv2d_fwd(x, w, bias, stride, pad, z, None)
        if stats is not None:
            zf = z.float().reshape(-1, Co)
            stats[0, 0] += zf.sum(0)
            stats[0, 1] += (zf * zf).sum(0)
        return z
    need(x, torch.bfloat16, "conv_bn.x"); need(w, torch.bfloat16, "conv_bn.w"); need(z, torch.bfloat16, "conv_bn.z")
    if stats is not None:
        need(stats, torch.float32, "conv_bn.stats")
        assert tuple(stats.shape) == (64, 2, Co), stats.shape
    hip("ptg_conv_bn_fwd", ptr(x), ptr(w), ptr(bias), ptr(z), N, H, W, C, Co, KH, KW, stride, pad, OH, OW,
        ptr(stats))
    return z



def _conv1_check(x, w, alpha, N, H, W):
    if x.dtype == torch.uint8:
        assert x.shape[-1] == 3, "conv1: uint8 input is the [N,H,W,3] image batch"
    else:
        need(x, torch.bfloat16, "conv1.x")
        assert x.shape[-1] == 4, "conv1: bf16 input is the channel-padded [N,H,W,4] batch"
    assert x.is_contiguous(), "conv1: x must be contiguous"
    need(w, torch.bfloat16, "conv1.w")
    assert tuple(w.shape) == (8, 5, 5, 4), w.shape
    need(alpha, torch.float32, "conv1.alpha")
    assert tuple(alpha.shape) == (H, W, 8), alpha.shape
    if H % 2 or W % 2:
        raise ValueError("conv1: H and W must be even (2x2 pool)")


def conv1_fwd_pm(x, w, bias, alpha, pooled):
    """First conv layer of the reference CNN in one kernel (conv1.hip conv1_fwd_pm_k): pooled =
    maxpool2x2(prelu(conv5x5(x, w, pad 2) + bias, alpha)), nothing else written.  x is the raw
    uint8 [N,H,W,3] image batch (/255 in registers) or bf16 [N,H,W,4]; w bf16 [8,5,5,4]."""
    if not on_device(x):
        return ref.conv1_fwd_pm(x, w, bias, alpha, pooled)
    N, H, W, _ = x.shape
    _conv1_check(x, w, alpha, N, H, W)
    need(pooled, torch.bfloat16, "conv1.pooled")
    assert tuple(pooled.shape) == (N, H // 2, W // 2, 8), pooled.shape
    if bias is not None:
        need(bias, torch.float32, "conv1.bias")
    hip("ptg_conv1_fwd_pm", ptr(x), int(x.dtype == torch.uint8), ptr(w), ptr(bias), ptr(alpha), ptr(pooled), N, H, W)
    return pooled


def conv1_fwd_rec(x, w, bias, alpha, pooled, zsel, argq):
    """First conv layer forward keeping the pool record (conv1.hip conv1_fwd_rec_k): pooled =
    maxpool2x2(prelu(conv5x5(x) + bias, alpha)), zsel = z at each 2x2 window's argmax (bf16) and
    argq = the argmax q = 2*dh + dw (uint8), all [N,H/2,W/2,8].  uint8 images enter the MFMA as
    exact integers with the 1/255 applied to the accumulators."""
    if not on_device(x):
        return ref.conv1_fwd_rec(x, w, bias, alpha, pooled, zsel, argq)
    N, H, W, _ = x.shape
    _conv1_check(x, w, alpha, N, H, W)
    shp = (N, H // 2, W // 2, 8)
    need(pooled, torch.bfloat16, "conv1.pooled"); need(zsel, torch.bfloat16, "conv1.zsel"); need(argq, torch.uint8, "conv1.argq")
    assert tuple(pooled.shape) == shp and tuple(zsel.shape) == shp and tuple(argq.shape) == shp
    if bias is not None:
        need(bias, torch.float32, "conv1.bias")
    hip("ptg_conv1_fwd_rec", ptr(x), int(x.dtype == torch.uint8), ptr(w), ptr(bias), ptr(alpha), ptr(pooled), ptr(zsel),
        ptr(argq), N, H, W)
    return pooled


def conv1_bwd_rec(x, alpha, dp, zsel, argq, dw, dalpha, dbias):
    """Backward of :func:`conv1_fwd_rec` from its record (conv1.hip conv1_bwd_rec_k): dZ at each
    window's argmax from (dp, zsel, argq, alpha), then dw [8,5,5,4], dalpha [H,W,8], dbias [8]
    (fp32, accumulated atomically into what the buffers hold)."""
    if not on_device(x):
        return ref.conv1_bwd_rec(x, alpha, dp, zsel, argq, dw, dalpha, dbias)
    N, H, W, _ = x.shape
    if x.dtype == torch.uint8:
        assert x.shape[-1] == 3
    else:
        need(x, torch.bfloat16, "conv1.x")
        assert x.shape[-1] == 4
    shp = (N, H // 2, W // 2, 8)
    for t, nm in ((dp, "dp"), (zsel, "zsel")):
        need(t, torch.bfloat16, "conv1." + nm)
        assert tuple(t.shape) == shp, (nm, t.shape)
    need(argq, torch.uint8, "conv1.argq"); need(alpha, torch.float32, "conv1.alpha")
    need(dw, torch.float32, "conv1.dw"); need(dalpha, torch.float32, "conv1.dalpha"); need(dbias, torch.float32, "conv1.dbias")
    assert tuple(argq.shape) == shp and tuple(alpha.shape) == (H, W, 8) and tuple(dalpha.shape) == (H, W, 8)
    assert tuple(dw.shape) == (8, 5, 5, 4) and dbias.numel() == 8
    hip("ptg_conv1_bwd_rec", ptr(x), int(x.dtype == torch.uint8), ptr(alpha), ptr(dp), ptr(zsel), ptr(argq), ptr(dw),
        ptr(dalpha), ptr(dbias), N, H, W)
    return dw


def conv1_bwd_pm(x, w, bias, alpha, dp, dw, dalpha, dbias):
    """Backward of :func:`conv1_fwd_pm` in one kernel (conv1.hip conv1_bwd_pm_k): z, the PReLU and
    the pool argmax are recomputed from x; dw [8,5,5,4], dalpha [H,W,8] and dbias [8] (fp32)
    accumulate atomically (the caller provides them zeroed or holding the sum so far)."""
    if not on_device(x):
        return ref.conv1_bwd_pm(x, w, bias, alpha, dp, dw, dalpha, dbias)
    N, H, W, _ = x.shape
    _conv1_check(x, w, alpha, N, H, W)
    need(dp, torch.bfloat16, "conv1.dp")
    assert tuple(dp.shape) == (N, H // 2, W // 2, 8), dp.shape
    need(dw, torch.float32, "conv1.dw"); need(dalpha, torch.float32, "conv1.dalpha")
    need(dbias, torch.float32, "conv1.dbias")
    assert tuple(dw.shape) == (8, 5, 5, 4) and tuple(dalpha.shape) == (H, W, 8) and dbias.numel() == 8
    if bias is not None:
        need(bias, torch.float32, "conv1.bias")
    hip("ptg_conv1_bwd_pm", ptr(x), int(x.dtype == torch.uint8), ptr(w), ptr(bias), ptr(alpha), ptr(dp), ptr(dw),
        ptr(dalpha), ptr(dbias), N, H, W)
    return dw


def set_persist_mode(dynamic: bool | None) -> None:
    """Persistent conv kernels: True = claim tile chunks from a work queue (robust when another
    stream's kernels, e.g. RCCL collectives overlapping the backward, hold CUs), False = static
    per-workgroup ranges (fastest on an idle GPU), None = the PTG_PERSIST_DYNAMIC default."""
    if not torch.cuda.is_available():
        return
    hip("ptg_set_persist_mode", -1 if dynamic is None else int(bool(dynamic)))


def conv_flip_weights(w, out):
    """out[Cin][KS][KS][Cout] = w[Cout][KS-1-kh][KS-1-kw][Cin] (dgrad filter)."""
    Cout, KS, _, Cin = w.shape
    if not on_device(w):
        out.copy_(torch.flip(w, dims=(1, 2)).permute(3, 1, 2, 0))
        return out
    hip("ptg_conv_flip_weights", ptr(w), ptr(out), Cout, KS, Cin)
    return out


def conv_flip_weights_multi(jobs):
    """conv_flip_weights for up to 4 (w, out) pairs in ONE launch (every dgrad filter of a backward
    pass is flipped up front instead of by one ~5 us launch per layer)."""
    jobs = list(jobs)
    if not jobs:
        return
    if not on_device(jobs[0][0]):
        for w, out in jobs:
            conv_flip_weights(w, out)
        return
    for k in range(0, len(jobs), 4):
        args = []
        part = jobs[k:k + 4]
        for w, out in part:
            need(w, torch.bfloat16, "flip.w"); need(out, torch.bfloat16, "flip.out")
            Cout, KS, _, Cin = w.shape
            assert tuple(out.shape) == (Cin, KS, KS, Cout)
            args += [ptr(w), ptr(out), Cout, KS, Cin]
        for _ in range(4 - len(part)):
            args += [None, None, 0, 0, 0]
        hip("ptg_conv_flip_weights4", len(part), *args)


def conv2d_dgrad_halo(dz, w, pad: int, out, wflip_buf, flipped: bool = False):
    """dx = d(conv)/dx (stride-1 'same') via the halo fwd kernel on flipped weights (``flipped``:
    ``wflip_buf`` already holds them, see conv_flip_weights_multi)."""
    if not on_device(dz):
        return ref.conv2d_dgrad(dz, w, pad, out)
    if not flipped:
        conv_flip_weights(w, wflip_buf)
    KS = w.shape[1]
    return conv2d_fwd_fused(dz, wflip_buf, None, KS - 1 - pad, out)


def conv2d_dgrad_halo_sparse(dzsel, arg, w, pad: int, out, wflip_buf, flipped: bool = False):
    """dx = d(conv)/dx (stride-1 'same', 5x5) of a layer whose output was 2x2-pooled, with dZ given
    as its sparse pool record (dzsel / arg [N,H/2,W/2,Cout], see conv2d_wgrad_halo_sparse): the halo
    loader of the strip kernel expands it, so the full-resolution dZ is never materialised."""
    N, H, W, Cin = out.shape
    Cout, KS, _, Cw = w.shape
    assert Cw == Cin and tuple(dzsel.shape) == (N, H // 2, W // 2, Cout) and tuple(arg.shape) == tuple(dzsel.shape)
    if not on_device(dzsel):
        dz = ref.expand_pool_record(dzsel, arg, (N, H, W, Cout)).to(dzsel.dtype)
        return ref.conv2d_dgrad(dz, w, pad, out)
    need(dzsel, torch.bfloat16, "dgrad_sparse.dzsel"); need(arg, torch.uint8, "dgrad_sparse.arg")
    need(out, torch.bfloat16, "dgrad_sparse.out")
    if not flipped:
        conv_flip_weights(w, wflip_buf)
    hip("ptg_conv2d_dgrad_halo_sparse", ptr(dzsel), ptr(arg), ptr(wflip_buf), ptr(out), N, H, W, Cout, Cin, KS,
        KS - 1 - pad)
    return out


def dgrad_sparse_supported(Cout: int, Cin: int, KS: int) -> bool:
    """ptg_conv2d_dgrad_halo_sparse covers this layer (dZ channels Cout, dx channels Cin)."""
    return KS == 5 and Cout in (16, 32) and Cin % 8 == 0 and Cin <= 64


def gemm(M, N, K, a, lda, a_kcontig, b, ldb, b_kcontig, epi, c, ldc, bias=None, act=0, splits=1):
    hip("ptg_gemm_bf16", M, N, K, ptr(a), lda, int(a_kcontig), ptr(b), ldb, int(b_kcontig), epi, ptr(c), ldc,
        ptr(bias), act, splits)


_DFS: dict = {}


def dense_fwd_splits(M: int, N: int, K: int) -> int:
    """K-split count of the weight-streaming forward (dense.hip) for this shape, 0 if it does not
    apply (M > 256, N % 128, K % 64, ...)."""
    key = (M, N, K)
    s = _DFS.get(key)
    if s is None:
        from .. import _native

        s = _DFS[key] = int(_native.hip_lib().ptg_dense_fwd_splits(M, N, K))
    return s


def dense_fwd_parts(x, w, part, splits: int):
    """part[s] (fp32 [S, M, N]) = x[M, K] @ w[N, K]^T over K-split s (dense.hip): every slice is
    written with plain stores; consumers sum the S slices (head_mse / bias_act on a 3-D tensor)."""
    M, K = x.shape
    N = w.shape[0]
    need(x, torch.bfloat16, "dense_fwd.x")
    need(w, torch.bfloat16, "dense_fwd.w")
    assert part.dtype == torch.float32 and part.is_contiguous() and part.numel() >= splits * M * N
    hip("ptg_dense_fwd_sk", ptr(x), ptr(w), ptr(part), M, N, K, splits)
    return part


def linear_fwd(x, w, bias, act, out, workspace=None, splits: int = 0, workspace_zeroed: bool = False):
    """out[M,N] bf16 = act(x[M,K] @ w[N,K]^T + bias).  A batch-sized M with a big weight takes the
    weight-streaming split-K kernel (dense.hip, S partial slices summed by the bias/activation
    pass); otherwise split-K with an fp32 workspace when the output tile grid alone cannot fill the
    256 CUs.  ``workspace_zeroed``: the workspace holds zeros (a persistent buffer created zeroed):
    the atomic split-K sums land on it directly and the bias/activation pass clears it again."""
    if not on_device(x):
        return ref.linear_fwd(x, w, bias, act, out)
    M, K = x.shape
    N = w.shape[0]
    S = dense_fwd_splits(M, N, K) if (splits == 0 and K >= 4096 and x.dtype == torch.bfloat16
                                       and w.dtype == torch.bfloat16 and x.is_contiguous()) else 0
    if S > 0:
        if workspace is None or workspace.numel() < S * M * N:
            workspace = torch.empty(S * M * N, device=x.device, dtype=torch.float32)
        part = workspace[: S * M * N].view(S, M, N)
        dense_fwd_parts(x, w, part, S)
        hip("ptg_bias_act_parts", ptr(part), S, ptr(bias), ptr(out), None, M, N, ACT[act])
        return out
    if splits == 0:
        tiles = math.ceil(M / 128) * math.ceil(N / 128)
        splits = 1 if tiles >= 192 or K < 4096 else min(16, max(1, 512 // max(tiles, 1)), K // 1024)
    if splits > 1:
        if workspace is None or workspace.numel() < M * N:
            workspace = torch.empty(M * N, device=x.device, dtype=torch.float32)
            workspace_zeroed = False
        ws = workspace[: M * N]
        if not workspace_zeroed:
            ws.zero_()
        gemm(M, N, K, x, K, 1, w, K, 1, 3, ws, N, None, 0, splits)
        hip("ptg_bias_act", ptr(ws), ptr(bias), ptr(out), None, M, N, ACT[act], int(workspace_zeroed))
    else:
        gemm(M, N, K, x, K, 1, w, K, 1, 0, out, N, bias, ACT[act], 1)
    return out


def dense_dx_ok(dy, w, out) -> bool:
    """Shapes the weight-streaming dX kernel (dense.hip dense_dx_k) takes: batch M <= 256, the
    reduction (units) a multiple of 64, the input width a multiple of 80, bf16 contiguous."""
    M, N = dy.shape
    K = w.shape[1]
    return (M <= 256 and N % 64 == 0 and K % 80 == 0 and K >= 4096 and dy.dtype == torch.bfloat16
            and w.dtype == torch.bfloat16 and out.dtype == torch.bfloat16 and dy.is_contiguous()
            and w.is_contiguous() and out.is_contiguous())


def dense_dx(dy, w, out):
    """out[M,K] bf16 = dy[M,N] @ w[N,K] on dense.hip's weight-streaming kernel (GPU only)."""
    M, N = dy.shape
    K = w.shape[1]
    assert tuple(out.shape) == (M, K) and dense_dx_ok(dy, w, out)
    hip("ptg_dense_dx", ptr(dy), ptr(w), ptr(out), M, N, K)
    return out


# The big Dense layer's dX (M = batch <= 256, N = 2048 units, K = 20480 inputs) streams the weight
# through dense.hip (dy fragments straight into registers, W tiles by LDS-DMA + transposed LDS
# reads); PTG_BLASLT_DX=1 routes it to hipBLASLt for A/B runs only (tools/dense_bench.py).
BLASLT_DX = config.get("blaslt_dx")


def linear_dx(dy, w, out):
    """out[M,K] bf16 = dy[M,N] @ w[N,K]."""
    if not on_device(dy):
        return ref.linear_dx(dy, w, out)
    M, N = dy.shape
    K = w.shape[1]
    if BLASLT_DX and dy.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and out.dtype == torch.bfloat16 \
            and M <= 512 and K >= 8192:
        torch.matmul(dy, w, out=out)
        return out
    if dense_dx_ok(dy, w, out):
        return dense_dx(dy, w, out)
    gemm(M, K, N, dy, N, 1, w, K, 0, 0, out, K)
    return out


def linear_dw(dy, x, out, accumulate: bool = False):
    """out[N,K] fp32 (+)= dy[M,N]^T @ x[M,K]."""
    if not on_device(dy):
        return ref.linear_dw(dy, x, out, accumulate)
    M, N = dy.shape
    K = x.shape[1]
    gemm(N, K, M, dy, N, 0, x, K, 0, 2 if accumulate else 1, out, K)
    return out


def linear_dw_adam(dy, x, p, m, v, pbf, lr_t: float, b1: float, b2: float, eps: float, gscale: float = 1.0,
                   lr_dev=None):
    """Adam step on a Dense kernel straight from its gradient dy[M,N]^T @ x[M,K]: p/m/v ([N,K] fp32)
    and the bf16 mirror pbf are updated in the GEMM epilogue; the gradient is never stored."""
    if not on_device(dy):
        g = torch.zeros(p.shape, dtype=torch.float32, device=p.device)
        ref.linear_dw(dy, x, g, False)
        return adam(p, g, m, v, pbf, lr_t, b1, b2, eps, gscale, lr_dev=lr_dev)
    M, N = dy.shape
    K = x.shape[1]
    for t in (p, m, v, pbf):
        if t.numel() != N * K or not t.is_contiguous():
            raise ValueError("linear_dw_adam: optimizer state must be contiguous [N, K]")
    hip("ptg_gemm_adam", N, K, M, ptr(dy), N, 0, ptr(x), K, 0, ptr(p), ptr(m), ptr(v), ptr(pbf), K,
        float(lr_t), float(b1), float(b2), float(eps), float(gscale), ptr(lr_dev))


def head_mse(acc, b1, w2, b2, tgt, dz1, dw2, db2, db1, stats, pred_out=None, gscale: float = 1.0, scratch=None):
    """Fused Dense(relu) -> Dense(N2) -> MSE head on the Dense1 split-K sums ``acc`` [B, K1] (fp32,
    re-zeroed): stats / dpred as mse_k, dz1 [B, K1] bf16, dw2 / db2 / db1 accumulated (GPU only)."""
    if not on_device(acc):
        return ref.head_mse(acc, b1, w2, b2, tgt, dz1, dw2, db2, db1, stats, pred_out, gscale)
    B, K1 = acc.shape[-2:]
    nparts = acc.shape[0] if acc.dim() == 3 else 0  # dense_fwd_parts slices, else atomic sums
    N2 = w2.shape[0]
    if scratch is None or scratch.numel() < B * (N2 + 2):
        scratch = torch.empty(B * (N2 + 2), dtype=torch.float32, device=acc.device)
    hip("ptg_head_mse", ptr(acc), ptr(b1), ptr(w2), ptr(b2), ptr(tgt), ptr(dz1), ptr(dw2), ptr(db2), ptr(db1),
        ptr(stats), ptr(pred_out), ptr(scratch), B, K1, N2, float(gscale), nparts)


def col_sum(g, out):
    """out[N] += sum over rows of g[M,N]."""
    if not on_device(g):
        return ref.col_sum(g, out)
    M, N = g.shape
    hip("ptg_col_sum", ptr(g), int(g.dtype == torch.bfloat16), ptr(out), M, N)
    return out


def bias_act(acc, bias, act, out_bf16=None, out32=None, clear: bool = False):
    """act(acc + bias) into out_bf16 / out32; ``clear`` re-zeroes acc (a split-K accumulator).  A 3-D
    ``acc`` holds dense_fwd_parts slices [S, M, N], summed here (nothing to clear)."""
    if not on_device(acc):
        ref.bias_act(acc, bias, act, out_bf16, out32)
        if clear:
            acc.zero_()
        return
    if acc.dim() == 3:
        S, M, N = acc.shape
        hip("ptg_bias_act_parts", ptr(acc), S, ptr(bias), ptr(out_bf16), ptr(out32), M, N, ACT[act])
        return
    M, N = acc.shape
    hip("ptg_bias_act", ptr(acc), ptr(bias), ptr(out_bf16), ptr(out32), M, N, ACT[act], int(clear))


def dense_small_fwd(x, w, b, act, out, out_bf16=None):
    """out[M,N] fp32 = act(x[M,K] @ w[N,K]^T + b) for narrow layers (N <= 64)."""
    if not on_device(x):
        return ref.dense_small_fwd(x, w, b, act, out, out_bf16)
    M, K = x.shape
    N = w.shape[0]
    hip("ptg_dense_small_fwd", ptr(x), int(x.dtype == torch.bfloat16), ptr(w), ptr(b), ptr(out), ptr(out_bf16),
        M, K, N, ACT[act])
    return out


def dense_small_dx(dy, w, mask, out):
    """out[M,K] = (dy[M,N] @ w[N,K]) * (mask > 0 if mask is given)."""
    if not on_device(dy):
        return ref.dense_small_dx(dy, w, mask, out)
    M, N = dy.shape
    K = w.shape[1]
    mk = 0 if mask is None else (2 if mask.dtype == torch.bfloat16 else 1)
    hip("ptg_dense_small_dx", ptr(dy), ptr(w), ptr(mask), mk, ptr(out), int(out.dtype == torch.bfloat16), M, K, N)
    return out


def dense_small_dw(dy, x, dw, db):
    """dw[N,K] += dy^T x ; db[N] += sum_m dy (fp32)."""
    if not on_device(dy):
        return ref.dense_small_dw(dy, x, dw, db)
    M, N = dy.shape
    K = x.shape[1]
    hip("ptg_dense_small_dw", ptr(dy), ptr(x), int(x.dtype == torch.bfloat16), ptr(dw), ptr(db), M, K, N)


# ----------------------------------------------------------------------------------------------
# PReLU / pooling
# ----------------------------------------------------------------------------------------------
def prelu_pool_fwd(z, alpha, out):
    if not on_device(z):
        return ref.prelu_pool_fwd(z, alpha, out)
    N, H, W, C = z.shape
    hip("ptg_prelu_pool_fwd", ptr(z), ptr(alpha), ptr(out), N, H, W, C)
    return out


def prelu_pool_bwd(dp, z, alpha, dz_out, dalpha, dbias, nper: int = 0):
    """dz_out = d/dz of maxpool2x2(prelu(z)); dalpha, dbias accumulate (fp32).  ``nper``: samples
    per workgroup (0 = auto).  ``dz_out`` None: dalpha / dbias only."""
    if not on_device(z):
        return ref.prelu_pool_bwd(dp, z, alpha, dz_out, dalpha, dbias)
    N, H, W, C = z.shape
    hip("ptg_prelu_pool_bwd2", ptr(dp), ptr(z), ptr(alpha), ptr(dz_out), ptr(dalpha), ptr(dbias), N, H, W, C, nper)
    return dz_out


def prelu_pool_bwd_sparse(dp, zsel, arg, alpha, dz_out, dalpha, dbias, nper: int = 0):
    """Backward of maxpool2x2(prelu(z)) from the sparse forward record (zsel, arg)."""
    if not on_device(dp):
        return ref.prelu_pool_bwd_sparse(dp, zsel, arg, alpha, dz_out, dalpha, dbias)
    N, H, W, C = dz_out.shape
    hip("ptg_prelu_pool_bwd_sparse", ptr(dp), ptr(zsel), ptr(arg), ptr(alpha), ptr(dz_out), ptr(dalpha), ptr(dbias),
        N, H, W, C, nper)
    return dz_out


def prelu_pool_bwd_sel(dp, zsel, arg, alpha, dzsel_out, dalpha, dbias, nper: int = 0):
    """Sparse-in / sparse-out backward of maxpool2x2(prelu(z)): from the forward record (zsel, arg)
    write dzsel = dZ at each window's argmax ([N,H/2,W/2,C]); dalpha, dbias accumulate."""
    if not on_device(dp):
        return ref.prelu_pool_bwd_sel(dp, zsel, arg, alpha, dzsel_out, dalpha, dbias)
    N, PH, PW, C = dzsel_out.shape
    for t, nm in ((dp, "dp"), (zsel, "zsel"), (dzsel_out, "dzsel")):
        need(t, torch.bfloat16, "prelu_pool_bwd_sel." + nm)
        assert tuple(t.shape) == (N, PH, PW, C), (nm, t.shape)
    need(arg, torch.uint8, "prelu_pool_bwd_sel.arg")
    assert tuple(alpha.shape) == (2 * PH, 2 * PW, C) and tuple(dalpha.shape) == tuple(alpha.shape)
    hip("ptg_prelu_pool_bwd_sel", ptr(dp), ptr(zsel), ptr(arg), ptr(alpha), ptr(dzsel_out), ptr(dalpha), ptr(dbias),
        N, 2 * PH, 2 * PW, C, nper)
    return dzsel_out


def prelu_fwd(z, alpha, out):
    if not on_device(z):
        return ref.prelu_fwd(z, alpha, out)
    N = z.shape[0]
    hip("ptg_prelu_fwd", ptr(z), ptr(alpha), ptr(out), N, z[0].numel())
    return out


def prelu_bwd(da, z, alpha, dz_out, dalpha, dbias, nper: int = 0):
    if not on_device(z):
        return ref.prelu_bwd(da, z, alpha, dz_out, dalpha, dbias)
    N = z.shape[0]
    C = z.shape[-1]
    # dz_out None: dalpha / dbias only
    hip("ptg_prelu_bwd2", ptr(da), ptr(z), ptr(alpha), ptr(dz_out),
        ptr(dalpha), ptr(dbias), N, z[0].numel(), C, nper)
    return dz_out


def gap_fwd(x, out):
    """Global average pool NHWC -> [N, C] fp32."""
    if not on_device(x):
        return ref.gap_fwd(x, out)
    N, H, W, C = x.shape
    hip("ptg_gap_fwd", ptr(x), ptr(out), N, H * W, C)
    return out


def gap_bwd(dy, out):
    if not on_device(dy):
        return ref.gap_bwd(dy, out)
    N, H, W, C = out.shape
    hip("ptg_gap_bwd", ptr(dy), ptr(out), N, H * W, C)
    return out


# ----------------------------------------------------------------------------------------------
# Losses, optimizer, conversions
# ----------------------------------------------------------------------------------------------
def mse(pred, y, dpred, stats, gscale: float = 1.0):
    if not on_device(pred):
        return ref.mse(pred, y, dpred, stats, gscale)
    B, D = pred.shape
    hip("ptg_mse", ptr(pred), ptr(y), ptr(dpred), ptr(stats), B, D, float(gscale))


def softmax_xent(logits, labels, dlogits, stats, gscale: float = 1.0):
    if not on_device(logits):
        return ref.softmax_xent(logits, labels, dlogits, stats, gscale)
    B, C = logits.shape
    hip("ptg_softmax_xent", ptr(logits), ptr(labels), ptr(dlogits), ptr(stats), B, C, float(gscale))


def adam(p, g, m, v, pbf, lr_t: float, b1: float, b2: float, eps: float, gscale: float = 1.0, lr_dev=None,
         clear_grad: bool = False):
    """Fused Adam; with ``lr_dev`` (the device step state of :func:`adam_step`) the step size is read
    on the device, so the launch can be captured once into a HIP graph and replayed every step.
    ``clear_grad``: store zeros into ``g`` after reading it (replaces the next step's zero fill)."""
    if not on_device(p):
        if lr_dev is not None:
            lr_t = float(lr_dev[1])
        ref.adam(p, g, m, v, pbf, lr_t, b1, b2, eps, gscale)
        if clear_grad:
            g.zero_()
        return
    hip("ptg_adam", ptr(p), ptr(g), ptr(m), ptr(v), ptr(pbf), p.numel(), float(lr_t), float(b1), float(b2),
        float(eps), float(gscale), ptr(lr_dev), int(clear_grad))


def adam_multi(p, g, m, v, pbf, ranges, lr_t: float, b1: float, b2: float, eps: float, gscale: float = 1.0,
               lr_dev=None, clear_grad: bool = False, flips=()):
    """:func:`adam` over several [lo, hi) ranges of flat 1-D tensors in ONE launch (<= 4 ranges).
    ``flips``: (wf, offset, Cout, KS, Cin) records of conv kernels inside the ranges whose flipped
    bf16 dgrad filter ``wf`` [Cin][KS][KS][Cout] is written from the updated weights (what
    :func:`conv_flip_weights` would make of the new bf16 mirror)."""
    ranges = [(int(lo), int(hi)) for lo, hi in ranges if hi > lo]
    flips = list(flips)
    if not ranges:
        return
    if not on_device(p) or len(ranges) > 4 or len(flips) > 4:
        for lo, hi in ranges:
            adam(p[lo:hi], g[lo:hi], m[lo:hi], v[lo:hi], None if pbf is None else pbf[lo:hi], lr_t, b1, b2, eps,
                 gscale, lr_dev=lr_dev, clear_grad=clear_grad)
        for wf, off, Cout, KS, Cin in flips:
            n = Cout * KS * KS * Cin
            conv_flip_weights(pbf[off:off + n].view(Cout, KS, KS, Cin), wf)
        return
    import ctypes

    rr = (ctypes.c_long * (2 * len(ranges)))(*[x for r in ranges for x in r])
    ff = (ctypes.c_long * max(1, 5 * len(flips)))(*[int(x) for wf, off, co, ks, ci in flips
                                                    for x in (wf.data_ptr(), off, co, ks, ci)])
    for wf, off, co, ks, ci in flips:
        need(wf, torch.bfloat16, "adam_multi.wf")
        assert wf.numel() == co * ks * ks * ci
    hip("ptg_adam_multi", ptr(p), ptr(g), ptr(m), ptr(v), ptr(pbf), len(ranges), rr, float(lr_t), float(b1),
        float(b2), float(eps), float(gscale), ptr(lr_dev), int(clear_grad), len(flips), ff)


def _mlp_desc(dims, acts, woffs, boffs):
    import ctypes

    vals = list(dims) + list(acts) + list(woffs) + list(boffs)
    return (ctypes.c_long * len(vals))(*[int(v) for v in vals])


def mlp_lds_bytes(dims, B: int) -> int:
    """LDS bytes the fused MLP step (mlp.hip) needs for these layer widths at batch B (0: no)."""
    import ctypes

    from .. import _native

    L = len(dims) - 1
    desc = _mlp_desc(dims, [0] * L, [0] * L, [0] * L)
    out = ctypes.c_long(0)
    _native.check(_native.hip_lib().ptg_mlp_lds_bytes(ctypes.addressof(desc), L, B, ctypes.byref(out)),
                  "ptg_mlp_lds_bytes")
    return int(out.value)


def mlp_desc(dims, acts, woffs, boffs):
    """The host descriptor of a fused MLP step (build once per model, pass as ``desc=``)."""
    return _mlp_desc(dims, acts, woffs, boffs)


def mlp_train(x, y, flat, m, v, flat_bf16, stats, dims, acts, woffs, boffs, steps: int, loss_kind: int,
              lr: float, b1: float, b2: float, eps: float, t0: int, desc=None):
    """``steps`` full training steps of a small MLP (Dense stack) in ONE launch (mlp.hip): x holds
    steps x B rows (fp32), y the labels (int32, loss_kind 0 = softmax + sparse categorical
    cross-entropy) or targets (fp32, loss_kind 1 = MSE); the Adam update goes straight into the
    flat master store, its moments and the bf16 copy; metric sums into ``stats``."""
    if not on_device(flat):
        return ref.mlp_train(x, y, flat, m, v, flat_bf16, stats, dims, acts, woffs, boffs, steps, loss_kind, lr,
                             b1, b2, eps, t0)
    import ctypes

    L = len(dims) - 1
    B = x.shape[0] // steps
    need(x, torch.float32, "mlp_train.x")
    need(y, torch.int32 if loss_kind == 0 else torch.float32, "mlp_train.y")
    assert x.numel() == steps * B * dims[0] and y.shape[0] == steps * B, (x.shape, y.shape, steps, dims)
    if desc is None:  # (a cached descriptor was checked against the store when it was built)
        assert max(woffs[l] + dims[l + 1] * dims[l] for l in range(L)) <= flat.numel()
        desc = _mlp_desc(dims, acts, woffs, boffs)
    pbf = flat_bf16 if flat_bf16 is not None and flat_bf16.data_ptr() != flat.data_ptr() else None
    hip("ptg_mlp_train", x.data_ptr(), y.data_ptr(), flat.data_ptr(), m.data_ptr(), v.data_ptr(), ptr(pbf),
        stats.data_ptr(), ctypes.addressof(desc), L, B, steps, loss_kind, lr, b1, b2, eps, t0)


class MlpStep:
    """A cached launch of :func:`mlp_train` for one model, batch size and optimizer state (mlp.hip
    ``ptg_mlp_ctx_*``): pointers, LDS plan and hyper-parameters are bound once, the Adam step counter
    lives on the device, and a step is one short native call with the batch pointers."""

    def __init__(self, flat, m, v, flat_bf16, stats, dims, acts, woffs, boffs, B: int, loss_kind: int, lr: float,
                 b1: float, b2: float, eps: float, t0: int, desc=None):
        import ctypes

        from .. import _native

        self.lib = _native.hip_lib()
        L = len(dims) - 1
        desc = desc if desc is not None else _mlp_desc(dims, acts, woffs, boffs)
        pbf = flat_bf16 if flat_bf16 is not None and flat_bf16.data_ptr() != flat.data_ptr() else None
        self.tstep = torch.full((1,), float(t0), dtype=torch.float32, device=flat.device)
        h = ctypes.c_void_p()
        _native.check(self.lib.ptg_mlp_ctx_create(flat.data_ptr(), m.data_ptr(), v.data_ptr(), ptr(pbf),
                                                  stats.data_ptr(), self.tstep.data_ptr(), ctypes.addressof(desc), L,
                                                  B, loss_kind, lr, b1, b2, eps, ctypes.byref(h)), "ptg_mlp_ctx_create")
        self.h = h.value
        self._keep = (flat, m, v, pbf, stats, desc)
        self.t = int(t0)
        self.B, self.in_dim, self.kind = B, int(dims[0]), loss_kind

    def run(self, x, y, steps: int, t0: int) -> None:
        """``steps`` fused steps on x (steps*B rows, fp32) / y; ``t0`` = optimizer steps so far."""
        if t0 != self.t:  # the host counter moved (set_iterations, a checkpoint): resync the device one
            self.tstep.fill_(float(t0))
        rc = self.lib.ptg_mlp_ctx_run(self.h, x.data_ptr(), y.data_ptr(), steps, stream_handle())
        if rc:
            raise RuntimeError(f"native kernel ptg_mlp_ctx_run failed: hipError_t={rc}")
        self.t = t0 + steps

    def __del__(self):
        h, self.h = getattr(self, "h", None), None
        if h:
            try:
                self.lib.ptg_mlp_ctx_free(h)
            except Exception:  # noqa: BLE001 - interpreter shutdown
                pass


def adam_step(state, lr: float, b1: float, b2: float):
    """state[0] += 1; state[1] = bias-corrected step size (on the device)."""
    if not on_device(state):
        t = float(state[0]) + 1.0
        state[0] = t
        state[1] = lr * math.sqrt(1.0 - b2 ** t) / (1.0 - b1 ** t)
        return state
    hip("ptg_adam_step", ptr(state), float(lr), float(b1), float(b2))
    return state


def sgd(p, g, vel, pbf, lr: float, momentum: float, nesterov: bool, gscale: float = 1.0, clear_grad: bool = False):
    """Keras SGD: v = momentum*v - lr*g; p += v (Nesterov: p += momentum*v - lr*g); refreshes pbf.
    ``clear_grad`` as in :func:`adam`."""
    if not on_device(p):
        gg = g * gscale
        if vel is not None:
            vel.mul_(momentum).sub_(lr * gg)
            p.add_(momentum * vel - lr * gg if nesterov else vel)
        else:
            p.sub_(lr * gg)
        if pbf is not None:
            pbf.copy_(p.to(pbf.dtype))
        if clear_grad:
            g.zero_()
        return
    hip("ptg_sgd", ptr(p), ptr(g), ptr(vel), ptr(pbf), p.numel(), float(lr), float(momentum), int(nesterov),
        float(gscale), int(clear_grad))


def sim_reduce_scatter(g, out, nchunks: int, own_scale: float, w_peer: float):
    """Simulated-world reduce-scatter (see distribute/strategy.py): out = own_scale * chunk 0 of ``g``
    + w_peer * (chunks 1..n-1), every chunk read (the local bytes of a ring reduce-scatter)."""
    cnt = out.numel()
    if not on_device(g):
        ch = g[: nchunks * cnt].view(nchunks, cnt)
        out.copy_(own_scale * ch[0] + (w_peer * ch[1:].sum(0) if nchunks > 1 else 0.0))
        return out
    hip("ptg_sim_reduce_scatter", ptr(g), ptr(out), cnt, int(nchunks), float(own_scale), float(w_peer))
    return out


def sim_all_gather(bucket, cnt: int):
    """Simulated-world all-gather: rewrite the peer chunks [cnt, numel) of ``bucket`` in place."""
    if not on_device(bucket):
        return bucket
    es = bucket.element_size()
    hip("ptg_sim_all_gather", ptr(bucket), cnt * es, bucket.numel() * es)
    return bucket


def fill_(t: torch.Tensor, value: float = 0.0) -> torch.Tensor:
    """t[:] = value with the HIP fill kernel (GPU, 4-byte elements or zero fills of 16-byte aligned
    buffers whose size is a multiple of 4 bytes); torch's fill elsewhere."""
    nbytes = t.numel() * t.element_size()
    if not on_device(t) or not t.is_contiguous() or nbytes % 4 or t.data_ptr() % 16 or \
            (value != 0.0 and t.element_size() != 4):
        return t.fill_(value)
    if t.dtype == torch.float32:
        word = int(np.float32(value).view(np.uint32))
    elif value == 0.0:
        word = 0
    else:
        word = int(np.int32(int(value)).view(np.uint32))
    hip("ptg_fill_u32", ptr(t), nbytes // 4, word)
    return t


def zeros(shape, dtype=torch.float32, device=None) -> torch.Tensor:
    """torch.zeros without the framework fill kernel on the GPU."""
    t = torch.empty(shape, dtype=dtype, device=device)
    return fill_(t, 0.0)


def cast_f32_bf16(x, out):
    if not on_device(x):
        # host mode: the "bf16" mirror may be fp32 (PTG_HOST_FP32, possibly aliasing ``x``)
        if out.data_ptr() != x.data_ptr():
            out.copy_(x.to(out.dtype))
        return out
    hip("ptg_cast_f32_bf16", ptr(x), ptr(out), x.numel())
    return out


def resize_norm(images_u8, out, H: int, W: int):
    """uint8 [N,Hin,Win,3] -> bf16 [N,H,W,4] bilinear (half-pixel) resize, /255, zero 4th channel."""
    if not on_device(images_u8):
        return ref.resize_norm(images_u8, out, H, W)
    N, Hin, Win, _ = images_u8.shape
    if (Hin, Win) == (H, W) and (N * H * W) % 4 == 0:
        # no resize: a pure byte -> bf16 pack (bilinear weights would all be 0/1)
        hip("ptg_pack_u8rgb4", ptr(images_u8), ptr(out), N * H * W)
        return out
    hip("ptg_resize_norm", ptr(images_u8), ptr(out), N, Hin, Win, H, W)
    return out


def pack_rgb4(images_f32, out):
    """float [N,H,W,3] -> bf16 [N,H,W,4]."""
    if not on_device(images_f32):
        out.zero_()
        out[..., :3] = images_f32.to(out.dtype)
        return out
    npix = images_f32.numel() // 3
    hip("ptg_pack_rgb4", ptr(images_f32), ptr(out), npix)
    return out


def relu_bwd(dy, y, out):
    """out = (y > 0) * dy."""
    if not on_device(dy):
        out.copy_((dy.float() * (y.float() > 0)).to(out.dtype))
        return out
    flags = int(dy.dtype == torch.bfloat16) | (int(y.dtype == torch.bfloat16) << 1) | \
        (int(out.dtype == torch.bfloat16) << 2)
    hip("ptg_relu_bwd", ptr(dy), ptr(y), ptr(out), out.numel(), flags)
    return out
