"""Numerics of every HIP training kernel vs the fp32 PyTorch reference of the same op (run on the
MI355X box).  Inputs are bf16-rounded first, so the only differences are accumulation order and
output rounding."""
import numpy as np
import pytest
import torch

from pyspark_tf_gke_amd.ops import nn as K
from pyspark_tf_gke_amd.ops import reference as R

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _close(a, b, rtol=2e-2, atol=2e-2, name=""):
    a, b = a.float().cpu(), b.float().cpu()
    err = (a - b).abs().max().item()
    scale = b.abs().max().item() + 1e-6
    assert err <= atol + rtol * scale, f"{name}: max err {err:.4g} vs scale {scale:.4g}"


def rnd(*shape, dtype=torch.bfloat16, scale=1.0):
    return (torch.randn(*shape) * scale).to(dtype)


@pytest.fixture(autouse=True)
def _seed(hip_built):
    torch.manual_seed(0)


@pytest.mark.parametrize("M,N,KD", [(256, 2048, 1024), (104, 72, 40), (64, 256, 2048), (512, 16, 96)])
@pytest.mark.parametrize("layout", ["kk", "kmn", "mnmn", "mnk"])
def test_gemm_layouts(M, N, KD, layout):
    a = rnd(M, KD) if layout in ("kk", "kmn") else rnd(KD, M)
    b = rnd(N, KD) if layout in ("kk", "mnk") else rnd(KD, N)
    A = a.float() if layout in ("kk", "kmn") else a.float().t()
    Bm = b.float().t() if layout in ("kk", "mnk") else b.float()
    ref = A @ Bm
    c = torch.empty(M, N, device=DEV, dtype=torch.float32)
    ak = layout in ("kk", "kmn")
    bk = layout in ("kk", "mnk")
    K.gemm(M, N, KD, a.to(DEV), KD if ak else M, ak, b.to(DEV), KD if bk else N, bk, 1, c, N)
    _close(c, ref, 1e-3, 1e-3, "gemm")


def test_gemm_splitk_atomic_and_bias_relu():
    M, N, Kd = 64, 2048, 20480
    x, w = rnd(M, Kd, scale=0.1), rnd(N, Kd, scale=0.1)
    b = torch.randn(N)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    K.linear_fwd(x.to(DEV), w.to(DEV), b.to(DEV), "relu", out)
    ref = torch.relu(x.float() @ w.float().t() + b)
    _close(out, ref, 2e-2, 2e-2, "linear_fwd")


@pytest.mark.parametrize("M,N,Kd,bn", [(128, 2048, 20480 // 8, -1), (256, 2048, 20480, -1), (256, 2048, 20480, 64),
                                       (200, 512, 64 * 200, -1), (256, 2048, 20480, 0)])
def test_linear_dx_dw(M, N, Kd, bn, monkeypatch):
    """dX on gemm_kernel: the CNN-B1 shape (M = 256, K = 20480) on the skinny-M 256x80 tiles (bn -1),
    forced 256x64 tiles, a ragged M with 256x64, and the 128x128 tiling (bn 0); the hipBLASLt route
    (an off-by-default A/B knob, PTG_BLASLT_DX) is pinned off so our kernel is the one checked."""
    from pyspark_tf_gke_amd import _native

    monkeypatch.setattr(K, "BLASLT_DX", False)
    dy, w, x = rnd(M, N), rnd(N, Kd), rnd(M, Kd)
    dx = torch.empty(M, Kd, device=DEV, dtype=torch.bfloat16)
    _native.hip_lib().ptg_gemm_skinny_set(bn)
    try:
        K.linear_dx(dy.to(DEV), w.to(DEV), dx)
    finally:
        _native.hip_lib().ptg_gemm_skinny_set(-1)
    _close(dx, dy.float() @ w.float(), 2e-2, 2e-2, "dx")
    dw = torch.empty(N, Kd, device=DEV)
    K.linear_dw(dy.to(DEV), x.to(DEV), dw)
    _close(dw, dy.float().t() @ x.float(), 1e-3, 1e-3, "dw")


def test_adam_sgd_clear_grad():
    """clear_grad: same update, and the gradient buffer holds zeros afterwards."""
    n = 8192
    p, g, m, v = torch.randn(n), torch.randn(n), torch.randn(n).abs() * 0.1, torch.rand(n) * 0.1
    P, G, Mm, V = (t.clone().to(DEV) for t in (p, g, m, v))
    K.adam(P, G, Mm, V, None, 1e-3, 0.9, 0.999, 1e-7, 1.0, clear_grad=True)
    R.adam(p, g, m, v, None, 1e-3, 0.9, 0.999, 1e-7, 1.0)
    _close(P, p, 1e-6, 1e-6, "adam_p")
    assert not G.any()
    p, g, vel = torch.randn(n), torch.randn(n), torch.randn(n)
    P, G, VE = p.clone().to(DEV), g.clone().to(DEV), vel.clone().to(DEV)
    K.sgd(P, G, VE, None, 0.1, 0.9, False, 1.0, clear_grad=True)
    vel = 0.9 * vel - 0.1 * g
    _close(P, p + vel, 1e-6, 1e-6, "sgd_p")
    assert not G.any()


CONV_CASES = [(2, 16, 20, 4, 8, 5), (2, 16, 20, 8, 16, 5), (2, 12, 10, 16, 32, 5), (3, 8, 10, 32, 64, 5),
              (2, 8, 8, 64, 64, 5), (2, 9, 7, 16, 64, 3), (1, 6, 6, 8, 128, 3)]


@pytest.mark.parametrize("N,H,W,C,Co,KS", CONV_CASES)
def test_conv_fwd(N, H, W, C, Co, KS):
    x, w, b = rnd(N, H, W, C), rnd(Co, KS, KS, C, scale=0.2), torch.randn(Co)
    pad = KS // 2
    out = torch.empty(N, H, W, Co, device=DEV, dtype=torch.bfloat16)
    K.conv2d_fwd(x.to(DEV), w.to(DEV), b.to(DEV), 1, pad, out)
    ref = torch.empty(N, H, W, Co, dtype=torch.bfloat16)
    R.conv2d_fwd(x, w, b, 1, pad, ref)
    _close(out, ref, 2e-2, 2e-2, "conv_fwd")


def test_conv_fwd_strided_valid():
    x, w = rnd(2, 15, 13, 8), rnd(16, 3, 3, 8, scale=0.2)
    out = torch.empty(2, 7, 6, 16, device=DEV, dtype=torch.bfloat16)
    K.conv2d_fwd(x.to(DEV), w.to(DEV), None, 2, 0, out)
    ref = torch.empty(2, 7, 6, 16, dtype=torch.bfloat16)
    R.conv2d_fwd(x, w, None, 2, 0, ref)
    _close(out, ref, 2e-2, 2e-2, "conv_fwd_s2")


@pytest.mark.parametrize("N,H,W,C,Co,KS", [c for c in CONV_CASES if c[3] % 8 == 0])
def test_conv_dgrad(N, H, W, C, Co, KS):
    dz, w = rnd(N, H, W, Co), rnd(Co, KS, KS, C, scale=0.2)
    pad = KS // 2
    out = torch.empty(N, H, W, C, device=DEV, dtype=torch.bfloat16)
    K.conv2d_dgrad(dz.to(DEV), w.to(DEV), pad, out)
    ref = torch.empty(N, H, W, C, dtype=torch.bfloat16)
    R.conv2d_dgrad(dz, w, pad, ref)
    _close(out, ref, 2e-2, 2e-2, "dgrad")


@pytest.mark.parametrize("N,H,W,C,Co,KS", CONV_CASES)
def test_conv_wgrad(N, H, W, C, Co, KS):
    x, dz = rnd(N, H, W, C), rnd(N, H, W, Co)
    pad = KS // 2
    out = torch.empty(Co, KS, KS, C, device=DEV)
    K.conv2d_wgrad(x.to(DEV), dz.to(DEV), 1, pad, out)
    ref = torch.empty(Co, KS, KS, C)
    R.conv2d_wgrad(x, dz, 1, pad, ref)
    _close(out, ref, 1e-3, 1e-3, "wgrad")


def test_conv_wgrad_large_splitk():
    x, dz = rnd(8, 64, 80, 16), rnd(8, 64, 80, 32, scale=0.1)
    out = torch.empty(32, 5, 5, 16, device=DEV)
    K.conv2d_wgrad(x.to(DEV), dz.to(DEV), 1, 2, out)
    ref = torch.empty(32, 5, 5, 16)
    R.conv2d_wgrad(x, dz, 1, 2, ref)
    _close(out, ref, 1e-3, 1e-3, "wgrad_big")


HALO_CASES = [(2, 16, 20, 4, 8, 5), (2, 18, 22, 8, 16, 5), (2, 12, 10, 16, 32, 5), (3, 8, 10, 32, 64, 5),
              (2, 8, 8, 64, 64, 5), (2, 10, 14, 64, 24, 3), (2, 6, 70, 4, 8, 3), (1, 64, 80, 16, 32, 5),
              (2, 256, 320, 4, 8, 5), (2, 9, 7, 16, 64, 3),
              (3, 18, 70, 4, 8, 5), (5, 30, 130, 4, 8, 5)]  # first-layer pair kernel: partial tiles


# more tiles than resident workgroups: exercises the persistent tile ranges, the ring-buffer halo
# reuse across tiles of a strip and strip changes inside one workgroup's range
BIG_HALO = [(16, 256, 320, 4, 8, 5), (32, 128, 160, 8, 16, 5), (64, 64, 80, 16, 32, 5), (128, 32, 40, 32, 64, 5),
            (256, 16, 20, 64, 64, 5), (160, 32, 40, 64, 32, 5), (40, 66, 70, 16, 16, 3)]


@pytest.mark.parametrize("N,H,W,C,Co,KS", HALO_CASES + BIG_HALO)
@pytest.mark.parametrize("epi", [None, "pool", "prelu"])
def test_conv_halo_fwd(N, H, W, C, Co, KS, epi):
    if epi == "pool" and (H % 2 or W % 2):
        pytest.skip("fused pool epilogue needs even H, W (engine falls back)")
    x, w, b = rnd(N, H, W, C), rnd(Co, KS, KS, C, scale=0.2), torch.randn(Co)
    alpha = torch.rand(H, W, Co) * 0.5
    pad = KS // 2
    z = torch.empty(N, H, W, Co, device=DEV, dtype=torch.bfloat16)
    aux = None
    if epi == "pool":
        aux = torch.empty(N, H // 2, W // 2, Co, device=DEV, dtype=torch.bfloat16)
    elif epi == "prelu":
        aux = torch.empty(N, H, W, Co, device=DEV, dtype=torch.bfloat16)
    K.conv2d_fwd_fused(x.to(DEV), w.to(DEV), b.to(DEV), pad, z, alpha.to(DEV), aux, epi)
    zr = torch.empty(N, H, W, Co, dtype=torch.bfloat16)
    R.conv2d_fwd(x, w, b, 1, pad, zr)
    _close(z, zr, 2e-2, 2e-2, "halo_z")
    if epi == "pool":
        pr = torch.empty(N, H // 2, W // 2, Co, dtype=torch.bfloat16)
        R.prelu_pool_fwd(zr, alpha, pr)
        _close(aux, pr, 2e-2, 2e-2, "halo_pool")
    elif epi == "prelu":
        ar = torch.empty(N, H, W, Co, dtype=torch.bfloat16)
        R.prelu_fwd(zr, alpha, ar)
        _close(aux, ar, 2e-2, 2e-2, "halo_prelu")


@pytest.mark.parametrize("N,H,W,C,Co,KS", [c for c in HALO_CASES + BIG_HALO if c[1] % 2 == 0 and c[2] % 2 == 0])
def test_conv_halo_pool_sparse(N, H, W, C, Co, KS):
    """epi='pools': pooled output + z at the argmax + argmax position instead of the full z."""
    x, w, b = rnd(N, H, W, C), rnd(Co, KS, KS, C, scale=0.2), torch.randn(Co)
    alpha = torch.rand(H, W, Co) * 0.5
    pad = KS // 2
    shp = (N, H // 2, W // 2, Co)
    zs = torch.empty(shp, device=DEV, dtype=torch.bfloat16)
    p = torch.empty(shp, device=DEV, dtype=torch.bfloat16)
    arg = torch.full(shp, 255, device=DEV, dtype=torch.uint8)
    K.conv2d_fwd_fused(x.to(DEV), w.to(DEV), b.to(DEV), pad, zs, alpha.to(DEV), p, "pools", arg)
    zr = torch.empty(N, H, W, Co, dtype=torch.bfloat16)
    R.conv2d_fwd(x, w, b, 1, pad, zr)
    pr = torch.empty(shp, dtype=torch.bfloat16)
    R.prelu_pool_fwd(zr, alpha, pr)
    _close(p, pr, 2e-2, 2e-2, "pools_p")
    q = arg.cpu().long()
    assert int(q.max()) <= 3
    zw = R._windows(zr.float())
    z_at = torch.gather(zw, 3, q.unsqueeze(3)).squeeze(3)
    _close(zs, z_at, 2e-2, 2e-2, "pools_zsel")  # zsel is z at the reported argmax
    yw = R._windows(torch.where(zr.float() > 0, zr.float(), zr.float() * alpha))
    y_at = torch.gather(yw, 3, q.unsqueeze(3)).squeeze(3)
    _close(y_at, yw.max(3).values, 2e-2, 2e-2, "pools_argmax_is_max")


@pytest.mark.parametrize("C,N,H,W,nper", [(8, 3, 8, 12, 0), (16, 5, 16, 20, 2), (64, 3, 8, 12, 0), (32, 9, 6, 6, 4)])
def test_prelu_pool_bwd_sparse(C, N, H, W, nper):
    z = rnd(N, H, W, C)
    alpha = torch.randn(H, W, C) * 0.3
    shp = (N, H // 2, W // 2, C)
    pr, zs, arg = torch.empty(shp), torch.empty(shp, dtype=torch.bfloat16), torch.empty(shp, dtype=torch.uint8)
    R.prelu_pool_fwd_sparse(z, alpha, pr, zs, arg)
    dp = rnd(*shp)
    dz = torch.empty(N, H, W, C, device=DEV, dtype=torch.bfloat16)
    da, db = torch.zeros(H, W, C, device=DEV), torch.zeros(C, device=DEV)
    K.prelu_pool_bwd_sparse(dp.to(DEV), zs.to(DEV), arg.to(DEV), alpha.to(DEV), dz, da, db, nper)
    dzr = torch.empty(N, H, W, C, dtype=torch.bfloat16)
    dar, dbr = torch.zeros(H, W, C), torch.zeros(C)
    R.prelu_pool_bwd_sparse(dp, zs, arg, alpha, dzr, dar, dbr)
    _close(dz, dzr, 1e-2, 1e-2, "sparse_dz")
    _close(da, dar, 1e-2, 1e-2, "sparse_dalpha")
    _close(db, dbr, 1e-2, 1e-2, "sparse_dbias")


@pytest.mark.parametrize("C,N,H,W,nper", [(8, 3, 8, 12, 0), (16, 5, 16, 20, 2), (64, 3, 8, 12, 0), (8, 130, 6, 10, 0),
                                          (32, 9, 6, 6, 4)])
def test_prelu_pool_bwd_sel(C, N, H, W, nper):
    """Sparse record in, dZ record out (first conv layer): dzsel, dalpha, dbias vs the fp32 reference,
    and dzsel expanded == the dense sparse-record backward's dZ."""
    z = rnd(N, H, W, C)
    alpha = torch.randn(H, W, C) * 0.3
    shp = (N, H // 2, W // 2, C)
    pr, zs, arg = torch.empty(shp), torch.empty(shp, dtype=torch.bfloat16), torch.empty(shp, dtype=torch.uint8)
    R.prelu_pool_fwd_sparse(z, alpha, pr, zs, arg)
    dp = rnd(*shp)
    dzs = torch.empty(shp, device=DEV, dtype=torch.bfloat16)
    da, db = torch.zeros(H, W, C, device=DEV), torch.zeros(C, device=DEV)
    K.prelu_pool_bwd_sel(dp.to(DEV), zs.to(DEV), arg.to(DEV), alpha.to(DEV), dzs, da, db, nper)
    dzr = torch.empty(N, H, W, C, dtype=torch.bfloat16)
    dar, dbr = torch.zeros(H, W, C), torch.zeros(C)
    R.prelu_pool_bwd_sparse(dp, zs, arg, alpha, dzr, dar, dbr)
    _close(R.expand_pool_record(dzs.cpu(), arg, (N, H, W, C)), dzr, 1e-2, 1e-2, "sel_dz")
    _close(da, dar, 1e-2, 1e-2, "sel_dalpha")
    _close(db, dbr, 1e-2, 1e-2, "sel_dbias")


@pytest.mark.parametrize("N,H,W,C,Co", [(2, 16, 20, 4, 8), (3, 18, 70, 4, 8), (16, 256, 320, 4, 8),
                                        (2, 18, 22, 8, 16), (4, 12, 10, 16, 32), (3, 8, 10, 32, 64)])
def test_conv_halo_wgrad_sparse(N, H, W, C, Co):
    """Weight gradient from dZ's sparse pool record == the dense weight gradient of the expanded dZ."""
    x = rnd(N, H, W, C)
    shp = (N, H // 2, W // 2, Co)
    dzs = rnd(*shp, scale=0.1)
    arg = torch.randint(0, 4, shp, dtype=torch.uint8)
    out = torch.full((Co, 5, 5, C), 7.0, device=DEV)
    K.conv2d_wgrad_halo_sparse(x.to(DEV), dzs.to(DEV), arg.to(DEV), 2, out)
    dz = R.expand_pool_record(dzs, arg, (N, H, W, Co)).to(torch.bfloat16)
    ref = torch.empty(Co, 5, 5, C)
    R.conv2d_wgrad(x, dz, 1, 2, ref)
    _close(out, ref, 1e-3, 1e-3, "wgrad_sparse")


def test_first_layer_sparse_chain_matches_dense(monkeypatch):
    """CNN first layer end to end: sparse forward record + sel backward + sparse wgrad give the same
    pooled output and gradients (weights, bias, alpha) as the dense path."""
    from pyspark_tf_gke_amd.models import build_cnn_model
    from pyspark_tf_gke_amd.nn import engine as E

    torch.manual_seed(3)
    x = torch.rand(4, 64, 80, 3)
    y = torch.rand(4, 2) * 50
    grads = {}
    monkeypatch.setattr(E, "CONV1_FUSED", False)
    for mode in (False, True):
        monkeypatch.setattr(E, "SPARSE_FIRST", mode)
        m = build_cnn_model((64, 80, 3), flat=True, summary=False, device=DEV)
        xb, yb = m._prep_batch(x, y)
        m.store.zero_grad()
        out = m._run_forward(xb, True)
        d = m._loss_grad(out, yb, m._stats_buf())
        m._run_backward(d)
        torch.cuda.synchronize()
        assert m.ops[0]._sel == mode
        grads[mode] = {p.name: p.grad.detach().float().cpu().clone() for p in m.store.params}
    for name, g in grads[False].items():
        _close(grads[True][name], g, 2e-2, 1e-3, "sel_grad_" + name)


def _conv1_inputs(N, H, W, u8):
    if u8:
        x = torch.randint(0, 256, (N, H, W, 3), dtype=torch.uint8)
    else:
        x = torch.cat([rnd(N, H, W, 3), torch.zeros(N, H, W, 1, dtype=torch.bfloat16)], -1)
    w = rnd(8, 5, 5, 4, scale=0.2)
    w[..., 3] = 0
    b = torch.randn(8) * 0.1
    alpha = torch.rand(H, W, 8) * 0.5
    dp = rnd(N, H // 2, W // 2, 8, scale=0.1)
    return x, w, b, alpha, dp


@pytest.mark.parametrize("N,H,W,u8", [(3, 12, 140, True), (2, 14, 64, False), (5, 20, 70, False),
                                      (7, 256, 320, True)])
def test_conv1_fused_vs_reference(N, H, W, u8):
    """conv1.hip: pooled output and dW / dalpha / dbias of the recomputing backward vs the fp32
    reference (z rounded to bf16 as the kernels do)."""
    x, w, b, alpha, dp = _conv1_inputs(N, H, W, u8)
    p = torch.empty(N, H // 2, W // 2, 8, dtype=torch.bfloat16, device=DEV)
    K.conv1_fwd_pm(x.to(DEV), w.to(DEV), b.to(DEV), alpha.to(DEV), p)
    pr = torch.empty(N, H // 2, W // 2, 8)
    R.conv1_fwd_pm(x, w, b, alpha, pr)
    _close(p, pr, 2e-2, 2e-2, "conv1_pooled")
    dw = torch.full((8, 5, 5, 4), 1.5, device=DEV)  # accumulates onto what is there
    da = torch.full((H, W, 8), 0.25, device=DEV)
    db = torch.full((8,), -1.0, device=DEV)
    K.conv1_bwd_pm(x.to(DEV), w.to(DEV), b.to(DEV), alpha.to(DEV), dp.to(DEV), dw, da, db)
    dwr, dar, dbr = torch.full((8, 5, 5, 4), 1.5), torch.full((H, W, 8), 0.25), torch.full((8,), -1.0)
    R.conv1_bwd_pm(x, w, b, alpha, dp, dwr, dar, dbr)
    _close(dw, dwr, 2e-2, 1e-2, "conv1_dw")
    _close(db, dbr, 2e-2, 1e-2, "conv1_db")
    # an argmax flip from a 1-ulp z difference moves one element's gradient: compare in the mean
    assert (da.cpu() - dar).abs().mean().item() < 1e-3, "conv1_dalpha"


@pytest.mark.parametrize("N,H,W,u8", [(4, 12, 140, True), (3, 16, 80, False), (16, 256, 320, True)])
def test_conv1_fused_matches_sparse_record_pipeline(N, H, W, u8):
    """Same MFMA math for z in both pipelines, so the argmax agrees exactly: the fused kernels must
    reproduce the sparse-record pipeline (forward record -> sel backward -> sparse wgrad) up to
    summation order."""
    x, w, b, alpha, dp = _conv1_inputs(N, H, W, u8)
    xd, wd, bd, ad, dpd = x.to(DEV), w.to(DEV), b.to(DEV), alpha.to(DEV), dp.to(DEV)
    shp = (N, H // 2, W // 2, 8)
    p1 = torch.empty(shp, dtype=torch.bfloat16, device=DEV)
    K.conv1_fwd_pm(xd, wd, bd, ad, p1)
    p0 = torch.empty(shp, dtype=torch.bfloat16, device=DEV)
    zs = torch.empty(shp, dtype=torch.bfloat16, device=DEV)
    arg = torch.empty(shp, dtype=torch.uint8, device=DEV)
    K.conv2d_fwd_fused(xd, wd, bd, 2, zs, ad, p0, "pools", arg)
    assert torch.equal(p1.cpu(), p0.cpu()), "pooled outputs differ"
    dw1, da1, db1 = torch.zeros(8, 5, 5, 4, device=DEV), torch.zeros(H, W, 8, device=DEV), torch.zeros(8, device=DEV)
    K.conv1_bwd_pm(xd, wd, bd, ad, dpd, dw1, da1, db1)
    dw0, da0, db0 = torch.zeros(8, 5, 5, 4, device=DEV), torch.zeros(H, W, 8, device=DEV), torch.zeros(8, device=DEV)
    dzs = torch.empty(shp, dtype=torch.bfloat16, device=DEV)
    K.prelu_pool_bwd_sel(dpd, zs, arg, ad, dzs, da0, db0)
    K.conv2d_wgrad_halo_sparse(xd, dzs, arg, 2, dw0, zeroed=True)
    _close(dw1, dw0, 1e-3, 1e-4, "fused_dw")
    _close(da1, da0, 1e-4, 1e-5, "fused_dalpha")
    _close(db1, db0, 1e-3, 1e-4, "fused_dbias")


@pytest.mark.parametrize("N,H,W,u8", [(3, 12, 140, True), (2, 14, 64, False), (5, 20, 70, False),
                                      (7, 256, 320, True), (24, 256, 320, True)])
def test_conv1_record_kernels_vs_reference(N, H, W, u8):
    """conv1.hip record pipeline: the forward's pooled output / z at the argmax / argmax vs the fp32
    reference, and the backward from the GPU's own record vs the reference backward of that record.
    N = 24 gives every work item several samples, so the forward's prefetch ring (PTG_CONV1_PD deep)
    wraps and ends mid-ring."""
    x, w, b, alpha, dp = _conv1_inputs(N, H, W, u8)
    shp = (N, H // 2, W // 2, 8)
    p = torch.empty(shp, dtype=torch.bfloat16, device=DEV)
    zs = torch.empty(shp, dtype=torch.bfloat16, device=DEV)
    q = torch.empty(shp, dtype=torch.uint8, device=DEV)
    K.conv1_fwd_rec(x.to(DEV), w.to(DEV), b.to(DEV), alpha.to(DEV), p, zs, q)
    pr, zr, qr = torch.empty(shp), torch.empty(shp), torch.empty(shp, dtype=torch.uint8)
    R.conv1_fwd_rec(x, w, b, alpha, pr, zr, qr)
    _close(p, pr, 2e-2, 2e-2, "rec_pooled")
    agree = (q.cpu() == qr).float().mean().item()
    assert agree > 0.995, f"argmax agreement {agree}"  # ties / 1-ulp z differences may flip a few
    same = q.cpu() == qr
    _close(zs.cpu()[same], zr[same], 2e-2, 2e-2, "rec_zsel")
    dw = torch.full((8, 5, 5, 4), 0.5, device=DEV)
    da = torch.full((H, W, 8), 0.25, device=DEV)
    db = torch.full((8,), -1.0, device=DEV)
    K.conv1_bwd_rec(x.to(DEV), alpha.to(DEV), dp.to(DEV), zs, q, dw, da, db)
    dwr, dar, dbr = torch.full((8, 5, 5, 4), 0.5), torch.full((H, W, 8), 0.25), torch.full((8,), -1.0)
    R.conv1_bwd_rec(x, alpha, dp, zs.cpu(), q.cpu(), dwr, dar, dbr)
    _close(dw, dwr, 1e-2, 1e-3, "rec_dw")
    _close(db, dbr, 1e-3, 1e-3, "rec_db")
    _close(da, dar, 1e-3, 1e-4, "rec_dalpha")


@pytest.mark.parametrize("u8", [False, True])
def test_first_layer_fused_model_grads(monkeypatch, u8):
    """CNN first layer inside the model: conv1.hip path vs the sparse-record pipeline of conv.hip
    (weights, bias, alpha gradients of every layer).  Packed bf16 input: the same MFMA math on both
    sides, so the same argmaxes - equal up to summation order.  Raw uint8 input: conv1.hip takes the
    pixels as exact integers (1/255 on the accumulators) where conv.hip rounds x/255 to bf16, so a few
    window argmaxes flip and the first layer's weight gradient moves with them: directions only."""
    from pyspark_tf_gke_amd.models import build_cnn_model
    from pyspark_tf_gke_amd.nn import engine as E

    torch.manual_seed(4)
    x = torch.randint(0, 256, (4, 64, 80, 3), dtype=torch.uint8) if u8 else torch.rand(4, 64, 80, 3)
    y = torch.rand(4, 2) * 50
    grads = {}
    for mode in (False, True):
        monkeypatch.setattr(E, "CONV1_FUSED", mode)
        m = build_cnn_model((64, 80, 3), flat=True, summary=False, device=DEV)
        xb, yb = m._prep_batch(x, y)
        m.store.zero_grad()
        out = m._run_forward(xb, True)
        d = m._loss_grad(out, yb, m._stats_buf())
        m._run_backward(d)
        torch.cuda.synchronize()
        assert m.ops[0]._fused1 == mode
        grads[mode] = {p.name: p.grad.detach().float().cpu().clone() for p in m.store.params}
    for name, g in grads[False].items():
        g1 = grads[True][name]
        if not u8:
            _close(g1, g, 1e-2, 1e-4, "fused1_grad_" + name)
            continue
        cos = float(torch.dot(g1.flatten(), g.flatten()) / (g1.norm() * g.norm() + 1e-20))
        # the first layer's own parameters and the per-element PReLU alphas downstream (their gradient
        # follows each pool window's argmax) move the most
        sensitive = name.startswith("conv2d/") or "alpha" in name
        assert cos > (0.9 if sensitive else 0.99), ("fused1_grad_" + name, cos)


@pytest.mark.parametrize("N,H,W,C,Co,epi", [(16, 256, 320, 4, 8, "pools"), (32, 128, 160, 8, 16, "pool"),
                                             (64, 64, 80, 16, 32, "pool"), (256, 16, 20, 64, 64, "prelu")])
def test_persistent_work_queue_matches_static(N, H, W, C, Co, epi):
    """Work-queue (dynamic chunk) mode of the persistent conv kernels == static ranges: identical
    forward outputs, weight gradients equal up to summation order."""
    x, w, b = rnd(N, H, W, C).to(DEV), rnd(Co, 5, 5, C, scale=0.2).to(DEV), torch.randn(Co).to(DEV)
    alpha = (torch.rand(H, W, Co) * 0.3).to(DEV)
    dz = rnd(N, H, W, Co, scale=0.1).to(DEV)
    outs = {}
    try:
        for dyn in (False, True):
            K.set_persist_mode(dyn)
            shp = (N, H // 2, W // 2, Co) if epi in ("pool", "pools") else (N, H, W, Co)
            zs = torch.empty(shp if epi == "pools" else (N, H, W, Co), device=DEV, dtype=torch.bfloat16)
            aux = torch.empty(shp, device=DEV, dtype=torch.bfloat16)
            arg = torch.empty(shp, device=DEV, dtype=torch.uint8) if epi == "pools" else None
            K.conv2d_fwd_fused(x, w, b, 2, zs, alpha, aux, epi, arg)
            dw = torch.zeros(Co, 5, 5, C, device=DEV)
            K.conv2d_wgrad_halo(x, dz, 2, dw)
            torch.cuda.synchronize()
            outs[dyn] = (zs.cpu(), aux.cpu(), dw.cpu())
    finally:
        K.set_persist_mode(None)
    assert torch.equal(outs[False][0], outs[True][0]) and torch.equal(outs[False][1], outs[True][1])
    _close(outs[True][2], outs[False][2], 1e-4, 1e-4, "wq_wgrad")


def test_conv_flip_weights_multi():
    """One launch flipping several dgrad filters == the per-layer flip (and the reference permute)."""
    shapes = [(8, 5, 5, 4), (16, 5, 5, 8), (32, 5, 5, 16), (64, 5, 5, 32), (64, 3, 3, 64)]
    ws = [rnd(*s_).to(DEV) for s_ in shapes]
    outs = [torch.empty(s_[3], s_[1], s_[2], s_[0], device=DEV, dtype=torch.bfloat16) for s_ in shapes]
    K.conv_flip_weights_multi(list(zip(ws, outs)))
    for w, o in zip(ws, outs):
        ref = torch.flip(w.cpu(), dims=(1, 2)).permute(3, 1, 2, 0)
        assert torch.equal(o.cpu(), ref)


@pytest.mark.parametrize("N,H,W,C,Co,KS", HALO_CASES + BIG_HALO)
def test_conv_halo_wgrad(N, H, W, C, Co, KS):
    x, dz = rnd(N, H, W, C), rnd(N, H, W, Co, scale=0.1)
    pad = KS // 2
    out = torch.empty(Co, KS, KS, C, device=DEV)
    K.conv2d_wgrad_halo(x.to(DEV), dz.to(DEV), pad, out)
    ref = torch.empty(Co, KS, KS, C)
    R.conv2d_wgrad(x, dz, 1, pad, ref)
    _close(out, ref, 1e-3, 1e-3, "halo_wgrad")


@pytest.mark.parametrize("N,H,W,C,Co,KS", [c for c in HALO_CASES + BIG_HALO if c[4] in K.HALO_C and c[3] % 8 == 0])
def test_conv_halo_dgrad(N, H, W, C, Co, KS):
    dz, w = rnd(N, H, W, Co), rnd(Co, KS, KS, C, scale=0.2)
    pad = KS // 2
    out = torch.empty(N, H, W, C, device=DEV, dtype=torch.bfloat16)
    wf = torch.empty(C, KS, KS, Co, device=DEV, dtype=torch.bfloat16)
    K.conv2d_dgrad_halo(dz.to(DEV), w.to(DEV), pad, out, wf)
    ref = torch.empty(N, H, W, C, dtype=torch.bfloat16)
    R.conv2d_dgrad(dz, w, pad, ref)
    _close(out, ref, 2e-2, 2e-2, "halo_dgrad")


@pytest.mark.parametrize("C,N,H,W,nper", [(8, 3, 8, 12, 0), (16, 3, 8, 12, 0), (64, 3, 8, 12, 0), (128, 3, 8, 12, 0),
                                          (24, 7, 10, 14, 3), (8, 9, 7, 9, 4), (32, 5, 6, 6, 2),
                                          (8, 40, 6, 10, 0), (16, 130, 4, 4, 0), (8, 67, 7, 9, 0),
                                          (64, 9, 32, 40, 0), (256, 5, 4, 6, 2), (16, 33, 18, 22, 0)])
def test_prelu_pool_fwd_bwd(C, N, H, W, nper):
    z = rnd(N, H, W, C)
    alpha = torch.randn(H, W, C) * 0.3
    alpha[0, 0, :] = 0.0  # exercise ties of zeros
    z[0, :2, :2, :] = -1.0
    p = torch.empty(N, H // 2, W // 2, C, device=DEV, dtype=torch.bfloat16)
    K.prelu_pool_fwd(z.to(DEV), alpha.to(DEV), p)
    pr = torch.empty(N, H // 2, W // 2, C, dtype=torch.bfloat16)
    R.prelu_pool_fwd(z, alpha, pr)
    _close(p, pr, 1e-2, 1e-2, "prelu_pool_fwd")
    dp = rnd(N, H // 2, W // 2, C)
    dz = torch.empty(N, H, W, C, device=DEV, dtype=torch.bfloat16)
    da = torch.zeros(H, W, C, device=DEV)
    db = torch.zeros(C, device=DEV)
    K.prelu_pool_bwd(dp.to(DEV), z.to(DEV), alpha.to(DEV), dz, da, db, nper)
    dzr = torch.empty(N, H, W, C, dtype=torch.bfloat16)
    dar, dbr = torch.zeros(H, W, C), torch.zeros(C)
    R.prelu_pool_bwd(dp, z, alpha, dzr, dar, dbr)
    _close(dz, dzr, 1e-2, 1e-2, "dz")
    _close(da, dar, 1e-2, 1e-2, "dalpha")
    _close(db, dbr, 1e-2, 1e-2, "dbias")


@pytest.mark.parametrize("N,H,W,C,nper", [(4, 16, 20, 64, 0), (7, 5, 6, 24, 3), (5, 4, 4, 8, 2), (96, 16, 20, 64, 0)])
def test_prelu_fwd_bwd(N, H, W, C, nper):
    z, alpha, da = rnd(N, H, W, C), torch.randn(H, W, C) * 0.2, rnd(N, H, W, C)
    a = torch.empty_like(z, device=DEV)
    K.prelu_fwd(z.to(DEV), alpha.to(DEV), a)
    ar = torch.empty_like(z)
    R.prelu_fwd(z, alpha, ar)
    _close(a, ar, 1e-2, 1e-2, "prelu_fwd")
    dz = torch.empty_like(z, device=DEV)
    dal, db = torch.zeros(H, W, C, device=DEV), torch.zeros(C, device=DEV)
    K.prelu_bwd(da.to(DEV), z.to(DEV), alpha.to(DEV), dz, dal, db, nper)
    dzr, dalr, dbr = torch.empty_like(z), torch.zeros(H, W, C), torch.zeros(C)
    R.prelu_bwd(da, z, alpha, dzr, dalr, dbr)
    _close(dz, dzr, 1e-2, 1e-2, "dz")
    _close(dal, dalr, 1e-2, 1e-2, "dalpha")
    _close(db, dbr, 1e-2, 1e-2, "dbias")


@pytest.mark.parametrize("M,Kd,N,act", [(32, 3, 16, "relu"), (64, 64, 15, "softmax"), (128, 2048, 2, None),
                                        (8192, 3, 16, "relu"), (8192, 32, 64, "relu"), (20000, 64, 15, None)])
def test_dense_small(M, Kd, N, act):
    x, w, b = torch.randn(M, Kd), torch.randn(N, Kd) * 0.1, torch.randn(N)
    y = torch.empty(M, N, device=DEV)
    K.dense_small_fwd(x.to(DEV), w.to(DEV), b.to(DEV), act, y)
    yr = torch.empty(M, N)
    R.dense_small_fwd(x, w, b, act, yr)
    _close(y, yr, 1e-4, 1e-4, "small_fwd")
    dy = torch.randn(M, N)
    mask = torch.randn(M, Kd)
    dx = torch.empty(M, Kd, device=DEV)
    K.dense_small_dx(dy.to(DEV), w.to(DEV), mask.to(DEV), dx)
    dxr = torch.empty(M, Kd)
    R.dense_small_dx(dy, w, mask, dxr)
    _close(dx, dxr, 1e-4, 1e-4, "small_dx")
    dw, db = torch.zeros(N, Kd, device=DEV), torch.zeros(N, device=DEV)
    K.dense_small_dw(dy.to(DEV), x.to(DEV), dw, db)
    dwr, dbr = torch.zeros(N, Kd), torch.zeros(N)
    R.dense_small_dw(dy, x, dwr, dbr)
    tol = 1e-4 if M <= 1024 else 2e-3  # split-M atomics: different summation order over 8k+ rows
    _close(dw, dwr, tol, tol, "small_dw")
    _close(db, dbr, tol, tol, "small_db")


def test_losses_and_adam():
    B = 64
    pred, y = torch.randn(B, 2) * 10, torch.randn(B, 2) * 10
    d = torch.empty(B, 2, device=DEV)
    st = torch.zeros(8, device=DEV)
    K.mse(pred.to(DEV), y.to(DEV), d, st)
    dr, sr = torch.empty(B, 2), torch.zeros(8)
    R.mse(pred, y, dr, sr)
    _close(d, dr, 1e-5, 1e-5, "mse_grad")
    _close(st[:5], sr[:5], 1e-4, 1e-4, "mse_stats")
    logits, lab = torch.randn(B, 15), torch.randint(0, 15, (B,), dtype=torch.int32)
    dl = torch.empty(B, 15, device=DEV)
    st.zero_()
    K.softmax_xent(logits.to(DEV), lab.to(DEV), dl, st)
    dlr, sr = torch.empty(B, 15), torch.zeros(8)
    R.softmax_xent(logits, lab, dlr, sr)
    _close(dl, dlr, 1e-5, 1e-5, "xent_grad")
    _close(st[:5], sr[:5], 1e-4, 1e-4, "xent_stats")
    n = 4096
    p, g, m, v = torch.randn(n), torch.randn(n), torch.randn(n).abs() * 0.1, torch.rand(n) * 0.1
    P, G, Mm, V = (t.clone().to(DEV) for t in (p, g, m, v))
    pb = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    K.adam(P, G, Mm, V, pb, 1e-3, 0.9, 0.999, 1e-7, 0.5)
    R.adam(p, g, m, v, None, 1e-3, 0.9, 0.999, 1e-7, 0.5)
    _close(P, p, 1e-6, 1e-6, "adam_p")
    _close(V, v, 1e-6, 1e-6, "adam_v")
    _close(pb, p, 1e-2, 1e-2, "adam_bf16")


@pytest.mark.parametrize("N,H,W,C", [(5, 64, 80, 128), (3, 7, 7, 2048), (256, 16, 20, 64), (2, 3, 5, 8)])
def test_gap_fwd_bwd(N, H, W, C):
    x = rnd(N, H, W, C)
    g = torch.full((N, C), 3.0, device=DEV)
    K.gap_fwd(x.to(DEV), g)
    _close(g, x.float().mean((1, 2)), 1e-3, 1e-3, "gap_fwd")
    dy = torch.randn(N, C)
    dx = torch.empty(N, H, W, C, device=DEV, dtype=torch.bfloat16)
    K.gap_bwd(dy.to(DEV), dx)
    _close(dx, (dy / (H * W)).view(N, 1, 1, C).expand(N, H, W, C), 1e-2, 1e-6, "gap_bwd")


def test_resize_norm_and_gap():
    imgs = torch.randint(0, 256, (2, 37, 45, 3), dtype=torch.uint8)
    out = torch.empty(2, 32, 40, 4, device=DEV, dtype=torch.bfloat16)
    K.resize_norm(imgs.to(DEV), out, 32, 40)
    ref = torch.empty(2, 32, 40, 4, dtype=torch.bfloat16)
    R.resize_norm(imgs, ref, 32, 40)
    _close(out, ref, 1e-2, 1e-2, "resize")
    x = rnd(3, 4, 5, 128)
    g = torch.empty(3, 128, device=DEV)
    K.gap_fwd(x.to(DEV), g)
    _close(g, x.float().mean((1, 2)), 1e-3, 1e-3, "gap")


@pytest.mark.parametrize("B,N,Kd", [(256, 2048, 1024), (64, 136, 40), (32, 72, 200)])
def test_linear_dw_adam(B, N, Kd):
    """Adam in the wgrad epilogue == wgrad GEMM + adam_k (fp32 reference of both)."""
    dy, x = rnd(B, N), rnd(B, Kd)
    p, m, v = torch.randn(N, Kd), torch.randn(N, Kd) * 0.01, torch.rand(N, Kd) * 0.01
    P, Mm, V = (t.clone().to(DEV) for t in (p, m, v))
    pb = torch.empty(N, Kd, device=DEV, dtype=torch.bfloat16)
    K.linear_dw_adam(dy.to(DEV), x.to(DEV), P, Mm, V, pb, 1e-3, 0.9, 0.999, 1e-7, 0.5)
    g = dy.float().t() @ x.float()
    R.adam(p, g, m, v, None, 1e-3, 0.9, 0.999, 1e-7, 0.5)
    _close(Mm, m, 1e-4, 1e-6, "m")
    _close(V, v, 1e-4, 1e-8, "v")
    _close(P, p, 1e-5, 1e-5, "p")
    _close(pb, p, 1e-2, 1e-2, "p_bf16")
    # device step state overrides the host step size
    lr_dev = torch.tensor([0.0, 0.0], device=DEV)
    P2 = p.clone().to(DEV)
    K.linear_dw_adam(dy.to(DEV), x.to(DEV), P2, m.clone().to(DEV), v.clone().to(DEV), pb, 5.0, 0.9, 0.999, 1e-7,
                     0.5, lr_dev=lr_dev)
    _close(P2, p, 0, 0, "lr_dev_zero_step")


def test_fused_adam_training_matches_unfused(monkeypatch):
    """A few Adam steps of an MLP with big Dense layers: fused-epilogue update == plain fused-flat
    Adam pass (same weights, moments and bf16 mirror)."""
    from pyspark_tf_gke_amd.nn import layers as L
    from pyspark_tf_gke_amd.nn import model as MD

    torch.manual_seed(5)
    x = torch.randn(64, 256)
    y = torch.randn(64, 2)
    res = {}
    for fused in (False, True):
        monkeypatch.setattr(MD, "FUSED_ADAM", fused)
        m = MD.Sequential([L.Input((256,)), L.Dense(512, activation="relu"), L.Dense(128, activation="relu"),
                           L.Dense(2)])
        m.build(device=DEV, seed=11)
        m.compile(optimizer="adam", loss="mse")
        for _ in range(3):
            m.train_on_batch(x, y)
        torch.cuda.synchronize()
        assert bool(getattr(m, "_fusable_ops", None)) == fused
        res[fused] = (m.store.flat.cpu().clone(), m.optimizer.m.cpu().clone(), m.optimizer.v.cpu().clone(),
                      m.store.flat_bf16.float().cpu().clone())
    for i, name in enumerate(("p", "m", "v", "pbf")):
        _close(res[True][i], res[False][i], 1e-4, 1e-6, "fused_" + name)


@pytest.mark.parametrize("M,N,KD", [(4000, 3300, 1000), (4096, 4096, 512)])
@pytest.mark.parametrize("epi", ["bf16_bias_relu", "f32"])
def test_gemm256_lds_dma(M, N, KD, epi):
    """The 256x256 LDS-DMA kernel (>= 200 tiles): ragged M/N/K edges zero-filled by the range
    check, source-swizzled fragments, 4-pass LDS epilogue — vs fp32 torch; and the same call with
    the kernel switched off (128x128 register-staged path) agrees."""
    from pyspark_tf_gke_amd import _native

    a, b = rnd(M, KD), rnd(N, KD)
    bias = torch.randn(N)
    ref = a.float() @ b.float().t()
    outs = []
    for on in (1, 0):
        _native.hip_lib().ptg_gemm256_set(on)
        if epi == "f32":
            c = torch.empty(M, N, device=DEV, dtype=torch.float32)
            K.gemm(M, N, KD, a.to(DEV), KD, True, b.to(DEV), KD, True, 1, c, N)
            _close(c, ref, 1e-3, 1e-3, f"gemm256 f32 on={on}")
        else:
            c = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
            K.linear_fwd(a.to(DEV), b.to(DEV), bias.to(DEV), "relu", c, splits=1)
            _close(c, torch.relu(ref + bias), 2e-2, 2e-2, f"gemm256 bf16 on={on}")
        outs.append(c.float().cpu())
    _native.hip_lib().ptg_gemm256_set(1)
    _close(outs[0], outs[1], 1e-2, 1e-2, "256 vs 128 kernel")


@pytest.mark.parametrize("M,N,KD,splits", [(256, 2048, 20480, 16), (200, 1000, 9000, 8), (64, 640, 4096, 12)])
def test_gemm_split_major_xcd_mapping(M, N, KD, splits):
    """Split-K GEMM (fp32 atomic epilogue) with the split-major XCD mapping (ptg_gemm_set_split_xcd)
    == the tile mapping and the fp32 reference: every (tile, split) item is covered exactly once,
    including grids whose tile count is not a multiple of 8 (then the tile mapping is kept)."""
    from pyspark_tf_gke_amd import _native

    a, b = rnd(M, KD), rnd(N, KD)
    ref = a.float() @ b.float().t()
    outs = []
    try:
        for on in (1, 0):
            _native.hip_lib().ptg_gemm_set_split_xcd(on)
            c = torch.zeros(M, N, device=DEV, dtype=torch.float32)
            K.gemm(M, N, KD, a.to(DEV), KD, 1, b.to(DEV), KD, 1, 3, c, N, None, 0, splits)
            torch.cuda.synchronize()
            _close(c, ref, 1e-3, 1e-3, f"split-K on={on}")
            outs.append(c.cpu())
    finally:
        _native.hip_lib().ptg_gemm_set_split_xcd(1)  # the default
    _close(outs[0], outs[1], 1e-4, 1e-4, "split-major vs tile mapping")


def test_conv_fwd_gemm256_resnet_layer():
    """A ResNet-50 stage-1 3x3 conv at batch 32 (M = 100352 output pixels, 392 tiles) through the
    LDS-DMA kernel's im2col loader vs the fp32 reference."""
    N, H, W, C, Co, KS = 32, 56, 56, 64, 256, 3
    x, w, b = rnd(N, H, W, C), rnd(Co, KS, KS, C, scale=0.1), torch.randn(Co)
    out = torch.empty(N, H, W, Co, device=DEV, dtype=torch.bfloat16)
    K.conv2d_fwd(x.to(DEV), w.to(DEV), b.to(DEV), 1, 1, out)
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b, padding=1)
    _close(out, ref.permute(0, 2, 3, 1), 2e-2, 2e-2, "conv_fwd_256")

@pytest.mark.parametrize("n", [64, 300_000])
def test_metric_update_kernel_matches_torch(n):
    """nn/metrics.py one-launch updates (metric_update_k) == the fp64 torch formulas: Mean of a
    loss scalar / vector, MAE and MSE over fp32 and bf16 predictions, sparse categorical accuracy;
    n = 300K takes the multi-workgroup atomic form."""
    from pyspark_tf_gke_amd.nn import metrics as MT

    g = torch.Generator().manual_seed(n)
    yp = torch.randn(n, 2, generator=g)
    yt = torch.randn(n, 2, generator=g)
    logits = torch.randn(n, 15, generator=g)
    lab = torch.randint(0, 15, (n,), generator=g, dtype=torch.int32)
    for dt in (torch.float32, torch.bfloat16):
        p, t = yp.to(dt), yt.to(dt)
        m1, m2 = MT.MeanAbsoluteError(), MT.MeanSquaredError()
        for _ in range(2):
            m1.update_state(t.cuda(), p.cuda())
            m2.update_state(t.cuda(), p.cuda())
        d = p.double() - t.double()
        assert abs(float(m1.result()) - float(d.abs().mean())) <= 1e-5 * max(1.0, float(d.abs().mean()))
        assert abs(float(m2.result()) - float((d * d).mean())) <= 1e-5 * max(1.0, float((d * d).mean()))
        assert float(m1._state[1]) == 2 * p.numel()
    mean = MT.Mean()
    mean.update_state(torch.tensor(2.5, device="cuda"))
    mean.update_state(yp[:, 0].cuda())
    want = (2.5 + float(yp[:, 0].double().sum())) / (n + 1)
    assert abs(float(mean.result()) - want) <= 1e-5 * max(1.0, abs(want))
    acc = MT.SparseCategoricalAccuracy()
    acc.update_state(lab.cuda(), logits.cuda())
    want = float((logits.argmax(-1) == lab.long()).double().mean())
    assert abs(float(acc.result()) - want) <= 1e-6


def test_adam_multi_ranges_and_flips():
    """adam_multi_k: several ranges in one launch == adam_k per range (bitwise), untouched elements
    stay untouched, and the flipped filters equal conv_flip_weights of the updated bf16 mirror."""
    n = 4096 + 3 * 5 * 5 * 8 + 16 * 5 * 5 * 8
    g0 = torch.randn(n)
    p0, m0, v0 = torch.randn(n), torch.randn(n) * 0.01, torch.rand(n) * 0.01
    ranges = [(0, 1024), (1536, n)]
    flips = [(1536, 3, 5, 8), (1536 + 3 * 200, 16, 5, 8)]
    outs = []
    for multi in (True, False):
        p, g, m, v = (t.clone().to(DEV) for t in (p0, g0, m0, v0))
        pb = torch.zeros(n, device=DEV, dtype=torch.bfloat16)
        wfs = [torch.zeros(ci, ks, ks, co, device=DEV, dtype=torch.bfloat16) for _, co, ks, ci in flips]
        if multi:
            K.adam_multi(p, g, m, v, pb, ranges, 1e-3, 0.9, 0.999, 1e-7, 0.5, clear_grad=True,
                         flips=[(wf, off, co, ks, ci) for wf, (off, co, ks, ci) in zip(wfs, flips)])
        else:
            for lo, hi in ranges:
                K.adam(p[lo:hi], g[lo:hi], m[lo:hi], v[lo:hi], pb[lo:hi], 1e-3, 0.9, 0.999, 1e-7, 0.5,
                       clear_grad=True)
            for wf, (off, co, ks, ci) in zip(wfs, flips):
                K.conv_flip_weights(pb[off:off + co * ks * ks * ci].view(co, ks, ks, ci), wf)
        torch.cuda.synchronize()
        outs.append([t.cpu() for t in (p, g, m, v, pb, *wfs)])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    assert torch.equal(outs[0][0][1024:1536], p0[1024:1536]) and torch.equal(outs[0][1][1024:1536], g0[1024:1536])
    assert outs[0][1][:1024].abs().max() == 0


@pytest.mark.parametrize("N,H,W,Co,Ci", [(3, 16, 40, 16, 8), (2, 32, 48, 32, 16), (5, 12, 20, 16, 16)])
def test_dgrad_halo_sparse_matches_dense(N, H, W, Co, Ci):
    """conv.hip SPIN loader: the data gradient from the sparse pool record (dzsel / argq, expanded in
    the halo loader) equals the dense data gradient of the expanded dZ - the same MFMA math on the
    same values, so the outputs are identical - and both match the fp32 reference."""
    torch.manual_seed(7)
    shp = (N, H // 2, W // 2, Co)
    dzs = rnd(*shp)
    arg = torch.randint(0, 4, shp, dtype=torch.uint8)
    w = rnd(Co, 5, 5, Ci, scale=0.1)
    dz = R.expand_pool_record(dzs.float(), arg, (N, H, W, Co)).bfloat16()
    d_dense = torch.empty(N, H, W, Ci, dtype=torch.bfloat16, device=DEV)
    d_sparse = torch.empty_like(d_dense)
    wf = torch.empty(Ci, 5, 5, Co, dtype=torch.bfloat16, device=DEV)
    K.conv2d_dgrad_halo(dz.to(DEV), w.to(DEV), 2, d_dense, wf)
    K.conv2d_dgrad_halo_sparse(dzs.to(DEV), arg.to(DEV), w.to(DEV), 2, d_sparse, wf, flipped=True)
    torch.cuda.synchronize()
    assert torch.equal(d_sparse.cpu(), d_dense.cpu()), "sparse-record dgrad differs from the dense one"
    ref = torch.empty(N, H, W, Ci)
    R.conv2d_dgrad(dz.float(), w.float(), 2, ref)
    _close(d_sparse, ref, 2e-2, 2e-2, "dgrad_sparse")


def test_sparse_pool_record_model_grads(monkeypatch):
    """CNN-B1-shaped model with the sparse pool record on layers 2-3 (engine.SPARSE_POOL) vs the dense
    z / dZ path: the same argmaxes and dZ values, so every parameter gradient agrees up to summation
    order."""
    from pyspark_tf_gke_amd.models import build_cnn_model
    from pyspark_tf_gke_amd.nn import engine as E

    torch.manual_seed(5)
    x = torch.rand(4, 64, 80, 3)
    y = torch.rand(4, 2) * 50
    grads = {}
    for mode in (False, True):
        monkeypatch.setattr(E, "SPARSE_POOL", mode)
        monkeypatch.setattr(E, "SPARSE_POOL_MIN_BATCH", 1)
        m = build_cnn_model((64, 80, 3), flat=True, summary=False, device=DEV)
        xb, yb = m._prep_batch(x, y)
        m.store.zero_grad()
        out = m._run_forward(xb, True)
        d = m._loss_grad(out, yb, m._stats_buf())
        m._run_backward(d)
        torch.cuda.synchronize()
        assert sum(bool(getattr(op, "_sp2", False)) for op in m.ops) == (2 if mode else 0)
        grads[mode] = {p.name: p.grad.detach().float().cpu().clone() for p in m.store.params}
    for name, g in grads[False].items():
        _close(grads[True][name], g, 1e-2, 1e-4, "sparse_pool_grad_" + name)
