"""fp32 PyTorch reference implementations of every NN op (CPU).

These serve two roles: the host execution path for CPU tensors (``local`` mode, the CPU test
suite) and the numerics oracle the GPU tests compare the HIP kernels against.  Each function has
the same in/out contract as its counterpart in :mod:`.nn` (NHWC activations, [Cout,KH,KW,Cin]
filters, [out,in] dense weights, results written into the provided ``out`` tensors).
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _f(t):
    return t.float()


def _act(y, act):
    if act == "relu":
        return torch.relu(y)
    if act == "softmax":
        return torch.softmax(y, dim=-1)
    return y


def conv2d_fwd(x, w, bias, stride, pad, out, act=None):
    xn = _f(x).permute(0, 3, 1, 2)
    wn = _f(w).permute(0, 3, 1, 2)
    y = F.conv2d(xn, wn, None if bias is None else _f(bias), stride=stride, padding=pad)
    out.copy_(_act(y.permute(0, 2, 3, 1), act).to(out.dtype))
    return out


def conv2d_dgrad(dz, w, pad, out):
    N, H, W, Cin = out.shape
    wn = _f(w).permute(0, 3, 1, 2)  # [Cout, Cin, KH, KW]
    dx = torch.nn.grad.conv2d_input((N, Cin, H, W), wn, _f(dz).permute(0, 3, 1, 2), stride=1, padding=pad)
    out.copy_(dx.permute(0, 2, 3, 1).to(out.dtype))
    return out


def conv2d_wgrad(x, dz, stride, pad, out, accumulate=False):
    Cout, KH, KW, C = out.shape
    xn = _f(x).permute(0, 3, 1, 2)
    dw = torch.nn.grad.conv2d_weight(xn, (Cout, C, KH, KW), _f(dz).permute(0, 3, 1, 2), stride=stride,
                                     padding=pad)
    dw = dw.permute(0, 2, 3, 1)
    if accumulate:
        out.add_(dw)
    else:
        out.copy_(dw)
    return out


def linear_fwd(x, w, bias, act, out):
    y = _f(x) @ _f(w).t()
    if bias is not None:
        y = y + _f(bias)
    out.copy_(_act(y, act).to(out.dtype))
    return out


def linear_dx(dy, w, out):
    out.copy_((_f(dy) @ _f(w)).to(out.dtype))
    return out


def linear_dw(dy, x, out, accumulate=False):
    dw = _f(dy).t() @ _f(x)
    if accumulate:
        out.add_(dw)
    else:
        out.copy_(dw)
    return out


def col_sum(g, out):
    out.add_(_f(g).sum(0))
    return out


def bias_act(acc, bias, act, out_bf16=None, out32=None):
    y = _f(acc) + (0 if bias is None else _f(bias))
    y = _act(y, act)
    if out_bf16 is not None:
        out_bf16.copy_(y.to(out_bf16.dtype))
    if out32 is not None:
        out32.copy_(y)


def dense_small_fwd(x, w, b, act, out, out_bf16=None):
    y = _f(x) @ _f(w).t()
    if b is not None:
        y = y + _f(b)
    y = _act(y, act)
    out.copy_(y)
    if out_bf16 is not None:
        out_bf16.copy_(y.to(out_bf16.dtype))
    return out


def dense_small_dx(dy, w, mask, out):
    dx = _f(dy) @ _f(w)
    if mask is not None:
        dx = dx * (_f(mask) > 0)
    out.copy_(dx.to(out.dtype))
    return out


def dense_small_dw(dy, x, dw, db):
    dw.add_(_f(dy).t() @ _f(x))
    if db is not None:
        db.add_(_f(dy).sum(0))


def _prelu(z, alpha):
    return torch.where(z > 0, z, alpha * z)


def prelu_pool_fwd(z, alpha, out):
    y = _prelu(_f(z), _f(alpha))
    p = F.max_pool2d(y.permute(0, 3, 1, 2), 2, 2).permute(0, 2, 3, 1)
    out.copy_(p.to(out.dtype))
    return out


def prelu_pool_bwd(dp, z, alpha, dz_out, dalpha, dbias):
    zf = _f(z).detach().requires_grad_(True)
    af = _f(alpha).detach().requires_grad_(True)
    p = F.max_pool2d(_prelu(zf, af).permute(0, 3, 1, 2), 2, 2).permute(0, 2, 3, 1)
    p.backward(_f(dp))
    if dz_out is not None:
        dz_out.copy_(zf.grad.to(dz_out.dtype))
    dalpha.add_(af.grad)
    dbias.add_(zf.grad.sum((0, 1, 2)))
    return dz_out


def _windows(t):
    """[N,H,W,C] -> [N,H/2,W/2,4,C] with window position q = 2*dh + dw."""
    N, H, W, C = t.shape
    return t.reshape(N, H // 2, 2, W // 2, 2, C).permute(0, 1, 3, 2, 4, 5).reshape(N, H // 2, W // 2, 4, C)


def prelu_pool_fwd_sparse(z, alpha, pout, zsel_out, arg_out):
    zf = _f(z)
    y = _prelu(zf, _f(alpha))
    yw, zw = _windows(y), _windows(zf)
    q = torch.argmax(yw, dim=3)  # first maximum in q order
    pout.copy_(torch.gather(yw, 3, q.unsqueeze(3)).squeeze(3).to(pout.dtype))
    zsel_out.copy_(torch.gather(zw, 3, q.unsqueeze(3)).squeeze(3).to(zsel_out.dtype))
    arg_out.copy_(q.to(torch.uint8))
    return zsel_out


def prelu_pool_bwd_sparse(dp, zsel, arg, alpha, dz_out, dalpha, dbias):
    N, H, W, C = dz_out.shape
    g, zs, q = _f(dp), _f(zsel), arg.long()
    aw = _windows(_f(alpha).unsqueeze(0).expand(N, H, W, C))       # [N,PH,PW,4,C]
    hit = torch.nn.functional.one_hot(q, 4).permute(0, 1, 2, 4, 3).bool()  # [N,PH,PW,4,C]
    gq = torch.where(hit, g.unsqueeze(3), torch.zeros_like(aw))
    pos = (zs > 0).unsqueeze(3)
    dzw = torch.where(pos, gq, gq * aw)
    daw = torch.where(pos, torch.zeros_like(gq), gq * zs.unsqueeze(3))
    def unw(t):
        return t.reshape(N, H // 2, W // 2, 2, 2, C).permute(0, 1, 3, 2, 4, 5).reshape(N, H, W, C)
    dz = unw(dzw)
    dz_out.copy_(dz.to(dz_out.dtype))
    dalpha.add_(unw(daw).sum(0))
    dbias.add_(dz.reshape(-1, C).sum(0))
    return dz_out


def expand_pool_record(vsel, arg, out_shape):
    """Dense [N,H,W,C] tensor holding vsel[n,ph,pw,c] at window position arg (q = 2*dh + dw) and
    zero elsewhere in each 2x2 window (the sparse pool record's dense form)."""
    N, H, W, C = out_shape
    hit = torch.nn.functional.one_hot(arg.long(), 4).permute(0, 1, 2, 4, 3)  # [N,PH,PW,4,C]
    vw = _f(vsel).unsqueeze(3) * hit.float()
    return vw.reshape(N, H // 2, W // 2, 2, 2, C).permute(0, 1, 3, 2, 4, 5).reshape(N, H, W, C)


def prelu_pool_bwd_sel(dp, zsel, arg, alpha, dzsel_out, dalpha, dbias):
    """Sparse-in / sparse-out backward of maxpool2x2(prelu(z)): dzsel = dZ at each window's argmax."""
    N, PH, PW, C = dzsel_out.shape
    H, W = 2 * PH, 2 * PW
    g, zs, q = _f(dp), _f(zsel), arg.long()
    aw = _windows(_f(alpha).unsqueeze(0).expand(N, H, W, C))  # [N,PH,PW,4,C]
    a = torch.gather(aw, 3, q.unsqueeze(3)).squeeze(3)
    pos = zs > 0
    o = torch.where(pos, g, g * a)
    dzsel_out.copy_(o.to(dzsel_out.dtype))
    d = torch.where(pos, torch.zeros_like(g), g * zs)
    dalpha.add_(expand_pool_record(d, arg, (N, H, W, C)).sum(0))
    dbias.add_(o.reshape(-1, C).sum(0))
    return dzsel_out


def conv1_input(x):
    """The first-layer kernels' view of their input: uint8 [N,H,W,3] images -> /255, bf16-rounded,
    zero 4th channel; bf16 [N,H,W,4] as is."""
    if x.dtype == torch.uint8:
        xf = (x.float() * (1.0 / 255.0)).to(torch.bfloat16).float()
        return torch.cat([xf, torch.zeros_like(xf[..., :1])], dim=-1)
    return _f(x)


def _conv1_z(x, w, bias):
    """bf16-rounded z = conv5x5(x) + bias of the first layer (fp32 math)."""
    xn = conv1_input(x).permute(0, 3, 1, 2)
    z = F.conv2d(xn, _f(w).permute(0, 3, 1, 2), None if bias is None else _f(bias), padding=2)
    return z.permute(0, 2, 3, 1).to(torch.bfloat16).float()


def conv1_fwd_pm(x, w, bias, alpha, pooled):
    """pooled = maxpool2x2(prelu(conv5x5(x) + bias, alpha)) (conv1.hip conv1_fwd_pm_k)."""
    return prelu_pool_fwd(_conv1_z(x, w, bias), alpha, pooled)


def conv1_fwd_rec(x, w, bias, alpha, pooled, zsel, argq):
    """pooled + the pool record (z at each window's argmax, argmax q) (conv1.hip conv1_fwd_rec_k)."""
    return prelu_pool_fwd_sparse(_conv1_z(x, w, bias), alpha, pooled, zsel, argq)


def conv1_bwd_rec(x, alpha, dp, zsel, argq, dw, dalpha, dbias):
    """Backward of conv1_fwd_rec from its record: dw, dalpha, dbias accumulate."""
    N, PH, PW, C = zsel.shape
    dzs = torch.empty((N, PH, PW, C))
    prelu_pool_bwd_sel(dp, zsel, argq, alpha, dzs, dalpha, dbias)
    dz = expand_pool_record(dzs.to(torch.bfloat16), argq, (N, 2 * PH, 2 * PW, C))
    xin = conv1_input(x)
    g = torch.nn.grad.conv2d_weight(xin.permute(0, 3, 1, 2), (C, xin.shape[-1], 5, 5), dz.permute(0, 3, 1, 2),
                                    padding=2)
    dw.add_(g.permute(0, 2, 3, 1))
    return dw


def conv1_bwd_pm(x, w, bias, alpha, dp, dw, dalpha, dbias):
    """Backward of conv1_fwd_pm from the pooled gradient: dw, dalpha, dbias accumulate."""
    z = _conv1_z(x, w, bias)
    N, H, W, C = z.shape
    zsel = torch.empty((N, H // 2, W // 2, C))
    arg = torch.empty((N, H // 2, W // 2, C), dtype=torch.uint8)
    prelu_pool_fwd_sparse(z, alpha, torch.empty_like(zsel), zsel, arg)
    dzs = torch.empty_like(zsel)
    prelu_pool_bwd_sel(dp, zsel, arg, alpha, dzs, dalpha, dbias)
    dz = expand_pool_record(dzs.to(torch.bfloat16), arg, (N, H, W, C))
    xin = conv1_input(x)
    g = torch.nn.grad.conv2d_weight(xin.permute(0, 3, 1, 2), (C, xin.shape[-1], 5, 5), dz.permute(0, 3, 1, 2),
                                    padding=2)
    dw.add_(g.permute(0, 2, 3, 1))
    return dw


def prelu_fwd(z, alpha, out):
    out.copy_(_prelu(_f(z), _f(alpha)).to(out.dtype))
    return out


def prelu_bwd(da, z, alpha, dz_out, dalpha, dbias):
    zf, af, g = _f(z), _f(alpha), _f(da)
    dz = torch.where(zf > 0, g, g * af)
    if dz_out is not None:
        dz_out.copy_(dz.to(dz_out.dtype))
    dalpha.add_(torch.where(zf > 0, torch.zeros_like(g), g * zf).sum(0))
    dbias.add_(dz.reshape(-1, dz.shape[-1]).sum(0))
    return dz_out


def gap_fwd(x, out):
    out.copy_(_f(x).mean((1, 2)))
    return out


def gap_bwd(dy, out):
    N, H, W, C = out.shape
    out.copy_((_f(dy) / (H * W)).reshape(N, 1, 1, C).expand(N, H, W, C).to(out.dtype))
    return out


def mse(pred, y, dpred, stats, gscale=1.0):
    d = _f(pred) - _f(y)
    B = pred.shape[0]
    n = d.numel()
    dpred.copy_(2.0 * d / n * gscale)
    sse = (d * d).sum()
    stats[0] += sse / n * B
    stats[1] += d.abs().sum()
    stats[2] += sse
    stats[3] += n
    stats[4] += B


def head_mse(acc, b1, w2, b2, tgt, dz1, dw2, db2, db1, stats, pred_out=None, gscale=1.0):
    """Dense(relu) -> Dense(N2) -> MSE on the Dense1 split-K sums (head_row_k / head_col_k)."""
    h = torch.relu(_f(acc) + _f(b1))
    pred = h @ _f(w2).t() + _f(b2)
    B, N2 = pred.shape
    dp = torch.empty_like(pred)
    mse(pred, tgt, dp, stats, gscale)
    dz1.copy_(((dp @ _f(w2)) * (h > 0)).to(dz1.dtype))
    dw2.add_(dp.t() @ h)
    db2.add_(dp.sum(0))
    db1.add_(_f(dz1).sum(0))
    if pred_out is not None:
        pred_out.copy_(pred)
    acc.zero_()


def softmax_xent(logits, labels, dlogits, stats, gscale=1.0):
    lg = _f(logits)
    B, C = lg.shape
    p = torch.softmax(lg, dim=-1)
    onehot = F.one_hot(labels.long(), C).float()
    dlogits.copy_((p - onehot) / B * gscale)
    pl = p.gather(1, labels.long().view(-1, 1)).clamp(1e-7, 1 - 1e-7)
    stats[0] += (-pl.log()).sum()
    stats[1] += (lg.argmax(-1) == labels.long()).float().sum()
    stats[4] += B


def adam(p, g, m, v, pbf, lr_t, b1, b2, eps, gscale=1.0):
    gg = g * gscale
    m.mul_(b1).add_(gg, alpha=1 - b1)
    v.mul_(b2).addcmul_(gg, gg, value=1 - b2)
    p.sub_(lr_t * m / (v.sqrt() + eps))
    if pbf is not None:
        pbf.copy_(p.to(pbf.dtype))


def resize_norm(images_u8, out, H, W):
    x = images_u8.float().permute(0, 3, 1, 2)
    y = F.interpolate(x, size=(H, W), mode="bilinear", align_corners=False, antialias=False) / 255.0
    out.zero_()
    out[..., :3] = y.permute(0, 2, 3, 1).to(out.dtype)
    return out


def mlp_train(x, y, flat, m, v, flat_bf16, stats, dims, acts, woffs, boffs, steps, loss_kind, lr, b1, b2, eps, t0):
    """fp32 oracle of mlp.hip's fused step (forward, softmax-xent / MSE, backward, Adam per step)."""
    import math

    L = len(dims) - 1
    B = x.shape[0] // steps
    for s in range(steps):
        xs = _f(x[s * B:(s + 1) * B]).reshape(B, dims[0])
        Ws = [flat[woffs[l]:woffs[l] + dims[l + 1] * dims[l]].view(dims[l + 1], dims[l]) for l in range(L)]
        bs = [flat[boffs[l]:boffs[l] + dims[l + 1]] if boffs[l] >= 0 else None for l in range(L)]
        a = [xs]
        for l in range(L):
            z = a[-1] @ Ws[l].t()
            if bs[l] is not None:
                z = z + bs[l]
            if l < L - 1 and acts[l] == 1:
                z = torch.relu(z)
            a.append(z)
        g = torch.empty_like(a[-1])
        if loss_kind == 0:
            softmax_xent(a[-1], y[s * B:(s + 1) * B], g, stats)
        else:
            mse(a[-1], y[s * B:(s + 1) * B].reshape(B, -1), g, stats)
        t = t0 + s + 1
        lr_t = lr * math.sqrt(1.0 - b2 ** t) / (1.0 - b1 ** t)
        grads = []
        for l in range(L - 1, -1, -1):
            gw = g.t() @ a[l]
            gb = g.sum(0)
            if l > 0:
                g = g @ Ws[l]
                if acts[l - 1] == 1:
                    g = g * (a[l] > 0).float()
            grads.append((l, gw, gb))
        for l, gw, gb in grads:
            sl = slice(woffs[l], woffs[l] + gw.numel())
            adam(flat[sl], gw.reshape(-1), m[sl], v[sl], None, lr_t, b1, b2, eps)
            if boffs[l] >= 0:
                sb = slice(boffs[l], boffs[l] + gb.numel())
                adam(flat[sb], gb, m[sb], v[sb], None, lr_t, b1, b2, eps)
    if flat_bf16 is not None and flat_bf16.data_ptr() != flat.data_ptr():
        flat_bf16.copy_(flat.to(flat_bf16.dtype))
