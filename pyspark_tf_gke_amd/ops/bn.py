"""BatchNormalization / MaxPooling2D(k, s, zero-pad) / add ops (csrc/kernels/bn.hip).

Every function takes device buffers (NHWC bf16 activations, fp32 per-channel vectors) and runs the
HIP kernel for GPU tensors, the fp32 PyTorch reference for CPU tensors (host path + test oracle).
Batch statistics go through a [BN_G][2][C] fp32 partial-sum buffer that the caller zeroes.

Semantics follow Keras ``BatchNormalization`` in training mode: normalise with the biased batch
variance, moving stats updated as ``moving = moving * momentum + batch * (1 - momentum)``; inference
mode normalises with the moving statistics.
"""
from __future__ import annotations

import torch

from ._util import hip, need, on_device, ptr

BN_G = 64


def part_buffer(C: int, device) -> torch.Tensor:
    return torch.zeros((BN_G, 2, C), dtype=torch.float32, device=device)


def bn_stats(z, part):
    """part[g][0] += sum(z), part[g][1] += sum(z^2) over rows of z[M, C]."""
    C = z.shape[-1]
    M = z.numel() // C
    if not on_device(z):
        zf = z.reshape(M, C).float()
        part[0, 0] += zf.sum(0)
        part[0, 1] += (zf * zf).sum(0)
        return part
    need(z, torch.bfloat16, "bn_stats.z")
    hip("ptg_bn_stats", ptr(z), M, C, ptr(part))
    return part


def bn_finalize(part, M: int, gamma, beta, eps: float, momentum: float, mmean, mvar, scale, shift, mean_out,
                rstd_out, training: bool):
    C = scale.shape[0]
    if not on_device(scale):
        if training:
            s = part[:, 0].double().sum(0)
            q = part[:, 1].double().sum(0)
            mean = s / M
            var = (q / M - mean * mean).clamp_min(0.0)
            mean, var = mean.float(), var.float()
            if momentum >= 0 and mmean is not None:
                mmean.mul_(momentum).add_(mean * (1 - momentum))
                mvar.mul_(momentum).add_(var * (1 - momentum))
        else:
            mean, var = mmean.clone(), mvar.clone()
        rstd = torch.rsqrt(var + eps)
        sc = (gamma if gamma is not None else 1.0) * rstd
        scale.copy_(sc)
        shift.copy_((beta if beta is not None else 0.0) - mean * sc)
        if mean_out is not None:
            mean_out.copy_(mean)
            rstd_out.copy_(rstd)
        return
    hip("ptg_bn_finalize", ptr(part), C, M, ptr(gamma), ptr(beta), float(eps), float(momentum), ptr(mmean),
        ptr(mvar), ptr(scale), ptr(shift), ptr(mean_out), ptr(rstd_out), int(training))


def bn_apply(z, scale, shift, res, relu: bool, y, mask=None):
    """``mask`` (device, uint8 [M*C/8]): also write the ReLU bit mask of y (bit j of byte i: y[8i+j] >
    0) for :func:`bn_bwd_reduce` / :func:`bn_bwd_apply` ``mask=`` (1 bit read instead of 16)."""
    C = z.shape[-1]
    M = z.numel() // C
    if not on_device(z):
        v = z.float() * scale + shift
        if res is not None:
            v = v + res.float()
        if relu:
            v = torch.relu(v)
        y.copy_(v.to(y.dtype))
        return y
    hip("ptg_bn_apply", ptr(z), ptr(scale), ptr(shift), ptr(res), int(relu), ptr(y), M, C, ptr(mask))
    return y


def _relu_mask(y, z, scale, shift, M, C):
    """ReLU mask of the BN output: from y, or (mask_from_z) recomputed as z*scale+shift > 0."""
    if scale is not None:
        zf = z.float().reshape(M, C)
        return torch.addcmul(shift.view(1, C), zf, scale.view(1, C)) > 0
    return y.float().reshape(M, C) > 0


def bn_bwd_reduce(dy, y, z, relu: bool, part, scale=None, shift=None, mask=None):
    """part += (sum g, sum g*z) with g = dy masked by the ReLU.  With ``scale``/``shift`` (a BN with
    no residual input) the mask is recomputed from z and ``y`` is not read."""
    C = z.shape[-1]
    M = z.numel() // C
    if not on_device(z):
        g = dy.float().reshape(M, C)
        if relu:
            g = g * _relu_mask(y, z, scale, shift, M, C)
        part[0, 0] += g.sum(0)
        part[0, 1] += (g * z.float().reshape(M, C)).sum(0)
        return part
    mode = 0 if not relu else (2 if scale is not None else (3 if mask is not None else 1))
    hip("ptg_bn_bwd_reduce", ptr(dy), ptr(y), ptr(z), M, C, mode, ptr(part), ptr(scale), ptr(shift), ptr(mask))
    return part


def bn_bwd_finalize(part, M: int, gamma, mean, rstd, dgamma, dbeta, coef):
    C = mean.shape[0]
    if not on_device(mean):
        sg = part[:, 0].double().sum(0)
        sgz = part[:, 1].double().sum(0)
        db = sg.float()
        dg = ((sgz - mean.double() * sg) * rstd.double()).float()
        if dgamma is not None:
            dgamma.add_(dg)
        if dbeta is not None:
            dbeta.add_(db)
        a = (gamma if gamma is not None else torch.ones_like(mean)) * rstd
        c1 = -a * dg * rstd / M
        c0 = -a * db / M - c1 * mean
        coef[0].copy_(a)
        coef[1].copy_(c1)
        coef[2].copy_(c0)
        return coef
    hip("ptg_bn_bwd_finalize", ptr(part), C, M, ptr(gamma), ptr(mean), ptr(rstd), ptr(dgamma), ptr(dbeta),
        ptr(coef))
    return coef


def bn_bwd_apply(dy, y, z, coef, relu: bool, dz, dres=None, scale=None, shift=None, mask=None):
    C = z.shape[-1]
    M = z.numel() // C
    if not on_device(z):
        g = dy.float()
        if relu:
            g = g * _relu_mask(y, z, scale, shift, M, C).reshape(g.shape)
        if dres is not None:
            dres.copy_(g.to(dres.dtype))
        dz.copy_((coef[0] * g + coef[1] * z.float() + coef[2]).to(dz.dtype))
        return dz
    mode = 0 if not relu else (2 if scale is not None else (3 if mask is not None else 1))
    hip("ptg_bn_bwd_apply", ptr(dy), ptr(y), ptr(z), ptr(coef), mode, ptr(dz), ptr(dres), M, C, ptr(scale),
        ptr(shift), ptr(mask))
    return dz


def pool_out_size(h: int, k: int, s: int, p: int) -> int:
    return (h + 2 * p - k) // s + 1


def maxpool_fwd(x, out, arg, k: int, s: int, p: int):
    """out = MaxPooling2D(k, s) of x zero-padded by p (Keras ZeroPadding2D + MaxPooling2D 'valid');
    arg (uint8, same shape as out) receives the argmax window position."""
    N, H, W, C = x.shape
    OH, OW = out.shape[1], out.shape[2]
    if not on_device(x):
        xp = torch.nn.functional.pad(x.float().permute(0, 3, 1, 2), (p, p, p, p))
        o, idx = torch.nn.functional.max_pool2d(xp, k, s, return_indices=True)
        out.copy_(o.permute(0, 2, 3, 1).to(out.dtype))
        if arg is not None:
            Wp = W + 2 * p
            ih, iw = idx // Wp, idx % Wp
            oh = torch.arange(OH).view(1, 1, OH, 1)
            ow = torch.arange(OW).view(1, 1, 1, OW)
            pos = (ih - oh * s) * k + (iw - ow * s)
            arg.copy_(pos.permute(0, 2, 3, 1).to(torch.uint8))
        return out
    need(x, torch.bfloat16, "maxpool.x")
    hip("ptg_maxpool_fwd", ptr(x), ptr(out), ptr(arg), N, H, W, C, OH, OW, k, s, p)
    return out


def maxpool_bwd(dy, arg, dx, k: int, s: int, p: int, accumulate: bool = False):
    N, H, W, C = dx.shape
    OH, OW = dy.shape[1], dy.shape[2]
    if not on_device(dy):
        g = torch.zeros((N, H + 2 * p, W + 2 * p, C), dtype=torch.float32)
        a = arg.long()
        dyf = dy.float()
        for oh in range(OH):
            for ow in range(OW):
                kh, kw = a[:, oh, ow] // k, a[:, oh, ow] % k  # [N, C]
                ih, iw = oh * s + kh, ow * s + kw
                n_idx = torch.arange(N).view(N, 1).expand(N, C)
                c_idx = torch.arange(C).view(1, C).expand(N, C)
                g.index_put_((n_idx, ih, iw, c_idx), dyf[:, oh, ow], accumulate=True)
        g = g[:, p: p + H, p: p + W]
        if accumulate:
            g = g + dx.float()
        dx.copy_(g.to(dx.dtype))
        return dx
    hip("ptg_maxpool_bwd", ptr(dy), ptr(arg), ptr(dx), N, H, W, C, OH, OW, k, s, p, int(accumulate))
    return dx


def add_(a, b, out):
    """out = a + b (bf16, same shape)."""
    if not on_device(a):
        out.copy_((a.float() + b.float()).to(out.dtype))
        return out
    hip("ptg_add_bf16", ptr(a), ptr(b), ptr(out), a.numel())
    return out
