"""ResNet-family kernels (bn.hip, strided/accumulating dgrad, SGD) and the functional graph engine on
the MI355X, each compared against the fp32 PyTorch reference of the same op."""
import pytest
import torch

from graph_oracle import oracle_grads
from pyspark_tf_gke_amd import nn
from pyspark_tf_gke_amd.ops import bn as KB
from pyspark_tf_gke_amd.ops import nn as K

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-12))


@pytest.fixture(scope="module", autouse=True)
def _lib(hip_built):
    return hip_built


@pytest.mark.parametrize("M,C", [(4096, 64), (1000, 256), (392, 2048), (50176, 128), (6272, 2048), (25088, 512), (300, 96), (100000, 256)])
def test_bn_forward_backward(M, C):
    torch.manual_seed(0)
    z = (torch.randn(M, C) * 2 + 0.5).to(torch.bfloat16)
    res = torch.randn(M, C).to(torch.bfloat16)
    dy = torch.randn(M, C).to(torch.bfloat16)
    gamma, beta = torch.rand(C) + 0.5, torch.randn(C)
    out = {}
    for dev in ("cpu", DEV):
        zz, rr, dd = z.to(dev), res.to(dev), dy.to(dev)
        g, b = gamma.to(dev), beta.to(dev)
        part = KB.part_buffer(C, dev)
        f = lambda: torch.empty(C, device=dev)  # noqa: E731
        scale, shift, mean, rstd = f(), f(), f(), f()
        mm, mv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
        KB.bn_stats(zz, part)
        KB.bn_finalize(part, M, g, b, 1e-3, 0.9, mm, mv, scale, shift, mean, rstd, True)
        if dev == "cpu":
            part.zero_()
        assert float(part.abs().sum()) == 0.0  # finalize re-zeroes the partial sums
        y = torch.empty(M, C, dtype=torch.bfloat16, device=dev)
        KB.bn_apply(zz, scale, shift, rr, True, y)
        dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
        coef = torch.empty(3, C, device=dev)
        KB.bn_bwd_reduce(dd, y, zz, True, part)
        KB.bn_bwd_finalize(part, M, g, mean, rstd, dg, db, coef)
        dz = torch.empty_like(zz)
        dres = torch.empty_like(zz)
        KB.bn_bwd_apply(dd, y, zz, coef, True, dz, dres)
        out[dev] = dict(y=y, mm=mm, mv=mv, dg=dg, db=db, dz=dz, dres=dres, scale=scale)
    for k in out["cpu"]:
        assert _rel(out[DEV][k], out["cpu"][k]) < 2e-2, k


@pytest.mark.parametrize("M,C", [(4096, 64), (1000, 256), (392, 2048), (6272, 1024), (300, 96)])
def test_bn_backward_mask_from_z(M, C):
    """BN without a residual: the ReLU mask recomputed from z (y not read) == the mask from y."""
    torch.manual_seed(5)
    z = (torch.randn(M, C) * 2 + 0.3).to(torch.bfloat16).to(DEV)
    dy = torch.randn(M, C).to(torch.bfloat16).to(DEV)
    gamma, beta = (torch.rand(C) + 0.5).to(DEV), torch.randn(C).to(DEV)
    f = lambda: torch.empty(C, device=DEV)  # noqa: E731
    part = KB.part_buffer(C, DEV)
    scale, shift, mean, rstd = f(), f(), f(), f()
    KB.bn_stats(z, part)
    KB.bn_finalize(part, M, gamma, beta, 1e-3, -1.0, None, None, scale, shift, mean, rstd, True)
    y = torch.empty_like(z)
    KB.bn_apply(z, scale, shift, None, True, y)
    outs = []
    for sc, sh in ((None, None), (scale, shift)):
        coef = torch.empty(3, C, device=DEV)
        dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        KB.bn_bwd_reduce(dy, y, z, True, part, sc, sh)
        KB.bn_bwd_finalize(part, M, gamma, mean, rstd, dg, db, coef)
        dz = torch.empty_like(z)
        KB.bn_bwd_apply(dy, y if sc is None else None, z, coef, True, dz, None, sc, sh)
        outs.append((dz.cpu(), dg.cpu(), db.cpu()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("M,C", [(4096, 64), (1000, 256), (392, 2048), (300, 96)])
def test_bn_backward_relu_bits(M, C):
    """Residual BN + ReLU: the backward with the 1-bit ReLU mask bn_apply wrote (relu mode 3) gives
    the same bits as with the mask from y (mode 1); the mask bits are y > 0."""
    torch.manual_seed(6)
    z = (torch.randn(M, C) * 2 + 0.3).to(torch.bfloat16).to(DEV)
    res = torch.randn(M, C).to(torch.bfloat16).to(DEV)
    res[0, :8] = 0.0  # exact zeros through the ReLU
    dy = torch.randn(M, C).to(torch.bfloat16).to(DEV)
    gamma, beta = (torch.rand(C) + 0.5).to(DEV), torch.randn(C).to(DEV)
    f = lambda: torch.empty(C, device=DEV)  # noqa: E731
    part = KB.part_buffer(C, DEV)
    scale, shift, mean, rstd = f(), f(), f(), f()
    KB.bn_stats(z, part)
    KB.bn_finalize(part, M, gamma, beta, 1e-3, -1.0, None, None, scale, shift, mean, rstd, True)
    y = torch.empty_like(z)
    bits = torch.empty(M * C // 8, dtype=torch.uint8, device=DEV)
    KB.bn_apply(z, scale, shift, res, True, y, bits)
    want = (y.float() > 0).reshape(-1, 8).cpu()
    got = ((bits.cpu().long().unsqueeze(1) >> torch.arange(8)) & 1).bool()
    assert torch.equal(got, want)
    outs = []
    for m in (None, bits):
        coef = torch.empty(3, C, device=DEV)
        dg, db = torch.zeros(C, device=DEV), torch.zeros(C, device=DEV)
        KB.bn_bwd_reduce(dy, y if m is None else None, z, True, part, mask=m)
        KB.bn_bwd_finalize(part, M, gamma, mean, rstd, dg, db, coef)
        dz, dres = torch.empty_like(z), torch.empty_like(z)
        KB.bn_bwd_apply(dy, y if m is None else None, z, coef, True, dz, dres, mask=m)
        outs.append((dz.cpu(), dres.cpu(), dg.cpu(), db.cpu()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.parametrize("shape,k,s,p", [((2, 112, 112, 64), 3, 2, 1), ((3, 17, 19, 16), 3, 2, 0),
                                         ((2, 32, 40, 8), 2, 2, 0)])
def test_maxpool(shape, k, s, p):
    torch.manual_seed(1)
    x = torch.randn(shape).to(torch.bfloat16)
    N, H, W, C = shape
    OH, OW = KB.pool_out_size(H, k, s, p), KB.pool_out_size(W, k, s, p)
    dy = torch.randn(N, OH, OW, C).to(torch.bfloat16)
    res = {}
    for dev in ("cpu", DEV):
        o = torch.empty(N, OH, OW, C, dtype=torch.bfloat16, device=dev)
        a = torch.empty(N, OH, OW, C, dtype=torch.uint8, device=dev)
        KB.maxpool_fwd(x.to(dev), o, a, k, s, p)
        dx = torch.empty(shape, dtype=torch.bfloat16, device=dev)
        KB.maxpool_bwd(dy.to(dev), a, dx, k, s, p)
        res[dev] = (o, a, dx)
    assert torch.equal(res[DEV][0].cpu(), res["cpu"][0])
    assert torch.equal(res[DEV][1].cpu(), res["cpu"][1])
    assert _rel(res[DEV][2], res["cpu"][2]) < 1e-2


@pytest.mark.parametrize("stride,acc", [(1, False), (2, False), (2, True), (1, True)])
def test_conv1x1_dgrad(stride, acc):
    torch.manual_seed(2)
    N, H, W, Cin, Cout = 4, 28, 28, 64, 128
    OH, OW = (H - 1) // stride + 1, (W - 1) // stride + 1
    dz = torch.randn(N, OH, OW, Cout).to(torch.bfloat16)
    w = (torch.randn(Cout, 1, 1, Cin) * 0.1).to(torch.bfloat16)
    init = torch.randn(N, H, W, Cin).to(torch.bfloat16)
    res = {}
    for dev in ("cpu", DEV):
        dx = init.clone().to(dev)
        K.conv1x1_dgrad(dz.to(dev), w.to(dev), stride, dx, acc)
        res[dev] = dx
    assert _rel(res[DEV], res["cpu"]) < 1e-2


def test_conv3x3_dgrad_accumulate():
    torch.manual_seed(3)
    N, H, W, Cin, Cout = 2, 14, 14, 128, 128
    dz = torch.randn(N, H, W, Cout).to(torch.bfloat16)
    w = (torch.randn(Cout, 3, 3, Cin) * 0.05).to(torch.bfloat16)
    init = torch.randn(N, H, W, Cin).to(torch.bfloat16)
    res = {}
    for dev in ("cpu", DEV):
        dx = init.clone().to(dev)
        K.conv2d_dgrad(dz.to(dev), w.to(dev), 1, dx, accumulate=True)
        res[dev] = dx
    assert _rel(res[DEV], res["cpu"]) < 1e-2


@pytest.mark.parametrize("nesterov", [False, True])
def test_sgd_kernel(nesterov):
    torch.manual_seed(4)
    n = 10_000
    p, g, v = torch.randn(n), torch.randn(n), torch.randn(n)
    res = {}
    for dev in ("cpu", DEV):
        pp, vv = p.clone().to(dev), v.clone().to(dev)
        pb = torch.empty(n, dtype=torch.bfloat16, device=dev)
        K.sgd(pp, g.to(dev), vv, pb, 0.1, 0.9, nesterov, 0.5)
        res[dev] = (pp, vv, pb)
    for a, b in zip(res[DEV], res["cpu"]):
        assert _rel(a, b) < 1e-5 or a.dtype == torch.bfloat16 and _rel(a, b) < 1e-2


def test_small_resnet_grads_vs_autograd():
    from pyspark_tf_gke_amd.models.resnet import ResNet

    torch.manual_seed(0)
    m = ResNet((1, 1), input_shape=(64, 64, 3), classes=10, width=16, device=DEV)
    m.compile(optimizer=nn.optimizers.SGD(0.0), loss="sparse_categorical_crossentropy")
    x = torch.rand(16, 64, 64, 3)
    y = torch.randint(0, 10, (16,))
    stats = m._stats_buf()
    stats.zero_()
    m.store.zero_grad()
    xb, yb = m._prep_batch(x, y)
    out = m._run_forward(xb, True)
    dpred = m._loss_grad(out, yb, stats)
    m._run_backward(dpred)
    torch.cuda.synchronize()
    loss = m._logs_from(stats)["loss"]
    ref_loss, ref = oracle_grads(m, x, y)
    assert abs(loss - ref_loss) < 3e-2 * max(1.0, abs(ref_loss))
    g = {p.name: p.grad.detach().float().cpu() for p in m.store.params}
    for name, rg in ref.items():
        if name.endswith("kernel"):
            eg = g[name].reshape(rg.shape).flatten()
            cos = float(torch.dot(eg, rg.flatten()) / (eg.norm() * rg.norm()))
            assert cos > 0.9, (name, cos)


def test_resnet50_train_steps():
    from pyspark_tf_gke_amd.models.resnet import build_resnet50

    torch.manual_seed(0)
    m = build_resnet50(device=DEV, optimizer=nn.optimizers.SGD(0.01, momentum=0.9))
    x = torch.rand(8, 224, 224, 3, device=DEV)
    y = torch.randint(0, 1000, (8,), device=DEV).to(torch.int32)
    l0 = m.train_on_batch(x, y, return_dict=True)["loss"]
    for _ in range(3):
        l1 = m.train_on_batch(x, y, return_dict=True)["loss"]
    assert l0 == l0 and l1 == l1 and l1 < l0  # fits the fixed batch
    p = m.predict(x[:2].cpu().numpy(), batch_size=2)
    assert p.shape == (2, 1000) and abs(float(p.sum()) - 2.0) < 1e-2


def _bn_pair(C):
    return (torch.rand(C) * 1.5 + 0.25).to(DEV), (torch.randn(C) * 0.5).to(DEV)


@pytest.mark.parametrize("N,H,W,C,Co,KS,stride,pad", [
    (4, 14, 14, 64, 256, 1, 1, 0),     # 1x1 GEMM
    (4, 14, 14, 64, 64, 3, 1, 1),      # 3x3 implicit GEMM
    (2, 28, 28, 128, 256, 1, 2, 0),    # 1x1 stride 2 (implicit GEMM)
    (2, 38, 38, 4, 64, 7, 2, 0),       # stem (C = 4)
    (64, 28, 28, 256, 512, 1, 1, 0),   # big enough for the 256x256 LDS-DMA kernel: stats there
    (3, 7, 7, 512, 2048, 1, 1, 0),
])
def test_conv_bn_fwd_stats(N, H, W, C, Co, KS, stride, pad):
    """gemm.hip ptg_conv_bn_fwd vs the fp32 reference, and the epilogue's batch statistics of the
    stored z."""
    x = torch.randn(N, H, W, C).to(torch.bfloat16).to(DEV)
    w = (torch.randn(Co, KS, KS, C) * (1.0 / (KS * KS * C) ** 0.5)).to(torch.bfloat16).to(DEV)
    OH, OW = (H + 2 * pad - KS) // stride + 1, (W + 2 * pad - KS) // stride + 1
    z = torch.empty(N, OH, OW, Co, dtype=torch.bfloat16, device=DEV)
    stats = torch.zeros(64, 2, Co, device=DEV)
    K.conv_bn_fwd(x, w, None, stride, pad, z, stats)
    zr = torch.empty(N, OH, OW, Co, dtype=torch.bfloat16)
    from pyspark_tf_gke_amd.ops import reference as R
    R.conv2d_fwd(x.cpu(), w.cpu(), None, stride, pad, zr, None)
    assert _rel(z, zr) < 1e-2
    zf = z.float().reshape(-1, Co).cpu()  # statistics of exactly what was stored
    st = stats.sum(0).cpu()
    assert _rel(st[0], zf.sum(0)) < 1e-4 and _rel(st[1], (zf * zf).sum(0)) < 1e-4


def test_resnet_bn_epilogue_stats_match_bn_stats(monkeypatch):
    """Small ResNet on the GPU: BN batch statistics from the conv epilogues (PTG_BN_EPI_STATS) give
    the separate bn_stats pass's loss and gradients."""
    from pyspark_tf_gke_amd.models.resnet import ResNet
    from pyspark_tf_gke_amd.nn import graph_ops as G

    x = torch.rand(16, 64, 64, 3)
    y = torch.randint(0, 10, (16,))
    res = {}
    for epi in (False, True):
        monkeypatch.setattr(G, "BN_EPI_STATS", epi)
        torch.manual_seed(0)
        m = ResNet((2, 1), input_shape=(64, 64, 3), classes=10, width=16, device=DEV)
        m.compile(optimizer=nn.optimizers.SGD(0.0), loss="sparse_categorical_crossentropy")
        stats = m._stats_buf()
        stats.zero_()
        m.store.zero_grad()
        xb, yb = m._prep_batch(x, y)
        out = m._run_forward(xb, True)
        m._run_backward(m._loss_grad(out, yb, stats))
        torch.cuda.synchronize()
        res[epi] = (m._logs_from(stats)["loss"], {p.name: p.grad.detach().float().cpu().clone() for p in m.store.params})
    assert abs(res[True][0] - res[False][0]) < 1e-2 * max(1.0, abs(res[False][0]))
    # two bf16 plans differ in fp32 summation order (atomics) only, but every bf16 rounding / ReLU /
    # max-pool decision downstream can flip with it: compare directions, loosely magnitudes
    for name, g0 in res[False][1].items():
        if name.endswith("_conv/bias"):
            continue
        g1 = res[True][1][name]
        cos = float(torch.dot(g1.flatten(), g0.flatten()) / (g1.norm() * g0.norm() + 1e-20))
        assert cos > 0.99 and _rel(g1, g0) < 0.15, (name, cos, _rel(g1, g0))


def test_resnet_bn_backward_epilogue_sums_match_reduce(monkeypatch):
    """Small ResNet: the BN backward sums of every Conv -> BN -> ReLU -> Conv link come from the
    consumer's dgrad epilogue (gemm.hip EpiBf16 backward form; no bn_bwd_reduce for that BN) and
    give the separate-reduction plan's loss and gradients."""
    from pyspark_tf_gke_amd.models.resnet import ResNet
    from pyspark_tf_gke_amd.nn import graph_ops as G

    x = torch.rand(16, 64, 64, 3)
    y = torch.randint(0, 10, (16,))
    res = {}
    calls = {}
    real = KB.bn_bwd_reduce

    def counting(*a, **k):
        calls[cur] = calls.get(cur, 0) + 1
        return real(*a, **k)

    monkeypatch.setattr(KB, "bn_bwd_reduce", counting)
    for cur in (False, True):
        monkeypatch.setattr(G, "BN_BWD_EPI", cur)
        torch.manual_seed(0)
        m = ResNet((2, 1), input_shape=(64, 64, 3), classes=10, width=16, device=DEV)
        m.compile(optimizer=nn.optimizers.SGD(0.0), loss="sparse_categorical_crossentropy")
        links = sum(1 for op in m.ops if getattr(getattr(op, "op", None), "bwd_bn_op", None) is not None)
        assert links >= 6  # two per bottleneck (1x1 -> 3x3 -> 1x1), three bottlenecks
        stats = m._stats_buf()
        stats.zero_()
        m.store.zero_grad()
        xb, yb = m._prep_batch(x, y)
        out = m._run_forward(xb, True)
        m._run_backward(m._loss_grad(out, yb, stats))
        torch.cuda.synchronize()
        res[cur] = (m._logs_from(stats)["loss"], {p.name: p.grad.detach().float().cpu().clone() for p in m.store.params})
    assert calls[False] - calls[True] == links  # one bn_bwd_reduce pass fewer per link
    assert abs(res[True][0] - res[False][0]) < 1e-3 * max(1.0, abs(res[False][0]))
    for name, g0 in res[False][1].items():
        if name.endswith("_conv/bias"):  # ~0 in exact arithmetic (a per-channel shift before BN)
            continue
        g1 = res[True][1][name]
        cos = float(torch.dot(g1.flatten(), g0.flatten()) / (g1.norm() * g0.norm() + 1e-20))
        assert cos > 0.99 and _rel(g1, g0) < 0.1, (name, cos, _rel(g1, g0))


@pytest.mark.parametrize("N,H,W,Cin,Cout,KS", [(64, 28, 28, 512, 256, 1), (8, 28, 28, 128, 64, 1), (8, 14, 14, 64, 64, 3)])
def test_dgrad_bnstats_matches_reduce(N, H, W, Cin, Cout, KS):
    """gemm.hip EpiBf16 backward form on both GEMM kernels (the first shape takes the 256x256 LDS-DMA
    kernel): the masked data gradient equals conv dgrad + ReLU mask, and the partial sums equal
    bn_bwd_reduce's over the same (dy, z)."""
    torch.manual_seed(N + Cin)
    dz = (torch.randn(N, H, W, Cout) * 0.3).to(torch.bfloat16).cuda()
    w = (torch.randn(Cout, KS, KS, Cin) * 0.05).to(torch.bfloat16).cuda()
    zb = torch.randn(N, H, W, Cin).to(torch.bfloat16).cuda()
    sc, sh = _bn_pair(Cin)
    dx_ref = torch.empty(N, H, W, Cin, dtype=torch.bfloat16, device=DEV)
    if KS == 1:
        K.conv1x1_dgrad(dz, w, 1, dx_ref)
    else:
        K.conv2d_dgrad(dz, w, KS // 2, dx_ref)
    part_ref = KB.part_buffer(Cin, DEV)
    KB.bn_bwd_reduce(dx_ref, None, zb, True, part_ref, sc, sh)
    dx = torch.empty_like(dx_ref)
    part = KB.part_buffer(Cin, DEV)
    assert K.conv_dgrad_bnstats(dz, w, KS // 2, dx, part, zb, sc, sh)
    torch.cuda.synchronize()
    mask = (zb.float() * sc + sh) > 0
    want = torch.where(mask, dx_ref, torch.zeros_like(dx_ref))
    bad = int((dx != want).sum())  # (fma vs mul+add can flip a mask bit exactly at 0)
    assert bad <= max(2, dx.numel() // 1_000_000), bad
    s_ref, s = part_ref.sum(0), part.sum(0)
    assert torch.allclose(s, s_ref, rtol=1e-3, atol=1e-2 * float(s_ref.abs().max()) / 100 + 1e-3)
