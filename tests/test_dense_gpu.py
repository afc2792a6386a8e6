"""Weight-streaming Dense kernels (csrc/kernels/dense.hip) vs fp32 PyTorch on the MI355X box.

The big Dense layer of CNN-B1 (Flatten(20480) -> Dense(2048), train_tf_ps.py:366-367) at the
reference's batch sizes (32, 64) and the bench's (256), plus ragged M: the forward's split-K partial
slices (plain stores, summed by the consumer), the fused head and bias/activation pass reading them.
Inputs are bf16-rounded first, so the only differences are accumulation order and output rounding.
"""
import pytest
import torch

from pyspark_tf_gke_amd.ops import nn as K

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _seed(hip_built):
    torch.manual_seed(0)


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return float((a - b).abs().max() / (b.abs().max() + 1e-12))


@pytest.mark.parametrize("M,N,Kd", [(256, 2048, 20480), (64, 2048, 20480), (32, 2048, 20480), (200, 1024, 8192),
                                    (100, 256, 4096), (17, 2048, 20480)])
def test_dense_fwd_parts_vs_fp32(M, N, Kd):
    S = K.dense_fwd_splits(M, N, Kd)
    assert S > 0
    x = (torch.randn(M, Kd) * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, Kd) * 0.02).to(torch.bfloat16)
    ref = x.float() @ w.float().t()
    part = torch.full((S, M, N), float("nan"), device=DEV)  # every element must be written
    K.dense_fwd_parts(x.to(DEV), w.to(DEV), part, S)
    torch.cuda.synchronize()
    assert torch.isfinite(part).all()
    got = part.sum(0)
    assert _rel(got, ref) < 2e-5, _rel(got, ref)
    # each slice is its own K range
    kc = Kd // S
    s = S - 1
    ref_s = x[:, s * kc:(s + 1) * kc].float() @ w[:, s * kc:(s + 1) * kc].float().t()
    assert _rel(part[s], ref_s) < 2e-5


@pytest.mark.parametrize("act", [None, "relu"])
def test_linear_fwd_big_dense_uses_parts(act):
    M, N, Kd = 128, 2048, 20480
    x = (torch.randn(M, Kd) * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, Kd) * 0.02).to(torch.bfloat16)
    b = torch.randn(N) * 0.1
    ref = x.float() @ w.float().t() + b
    if act == "relu":
        ref = torch.relu(ref)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    K.linear_fwd(x.to(DEV), w.to(DEV), b.to(DEV), act, out)
    torch.cuda.synchronize()
    assert _rel(out, ref) < 1e-2


def test_head_mse_on_partial_slices_vs_fp32():
    """The fused regression head summing S partial slices == the same head on summed fp32 sums."""
    B, K1, N2, S = 256, 2048, 2, 16
    g = torch.Generator().manual_seed(1)
    parts = torch.randn(S, B, K1, generator=g) * 0.25
    acc = parts.sum(0)
    b1 = torch.randn(K1, generator=g) * 0.1
    w2 = torch.randn(N2, K1, generator=g) * 0.02
    b2 = torch.randn(N2, generator=g)
    t = torch.randn(B, N2, generator=g) * 3
    h = torch.relu(acc + b1)
    pred = h @ w2.t() + b2
    d = pred - t
    dp = 2 * d / (B * N2)
    dz = (dp @ w2) * (h > 0)
    dz1 = torch.empty(B, K1, device=DEV, dtype=torch.bfloat16)
    dw2 = torch.zeros(N2, K1, device=DEV)
    db2 = torch.zeros(N2, device=DEV)
    db1 = torch.zeros(K1, device=DEV)
    stats = torch.zeros(8, device=DEV)
    pred_out = torch.empty(B, N2, device=DEV)
    K.head_mse(parts.to(DEV).contiguous(), b1.to(DEV), w2.to(DEV), b2.to(DEV), t.to(DEV), dz1, dw2, db2, db1, stats,
               pred_out=pred_out)
    torch.cuda.synchronize()
    assert torch.allclose(pred_out.cpu(), pred, rtol=1e-4, atol=1e-4)
    assert torch.allclose(dz1.float().cpu(), dz, rtol=1e-2, atol=1e-6)
    assert torch.allclose(dw2.cpu(), dp.t() @ h, rtol=1e-4, atol=1e-5)
    assert torch.allclose(db2.cpu(), dp.sum(0), rtol=1e-4, atol=1e-6)
    assert torch.allclose(db1.cpu(), dz.sum(0), rtol=1e-4, atol=1e-6)
    st = stats.cpu()
    assert abs(float(st[2]) - float((d * d).sum())) <= 1e-4 * float((d * d).sum())


def test_bias_act_on_partial_slices():
    S, M, N = 8, 64, 2048
    parts = torch.randn(S, M, N)
    b = torch.randn(N)
    ref = torch.relu(parts.sum(0) + b)
    out = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    out32 = torch.empty(M, N, device=DEV)
    K.bias_act(parts.to(DEV), b.to(DEV), "relu", out_bf16=out, out32=out32)
    torch.cuda.synchronize()
    assert torch.allclose(out32.cpu(), ref, rtol=1e-5, atol=1e-5)
    assert _rel(out, ref) < 1e-2


@pytest.mark.parametrize("M,N,Kd", [(256, 2048, 20480), (64, 2048, 20480), (32, 2048, 20480), (200, 1024, 8000),
                                    (17, 128, 4160)])
def test_dense_dx_vs_fp32(M, N, Kd):
    """dX = dy @ W through dense_dx_k (register A fragments, LDS-DMA W with transposed reads),
    including batches that leave waves with no rows and widths that are not multiples of 128."""
    dy = (torch.randn(M, N) * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, Kd) * 0.02).to(torch.bfloat16)
    ref = dy.float() @ w.float()
    out = torch.full((M, Kd), float("nan"), device=DEV).to(torch.bfloat16)
    K.dense_dx(dy.to(DEV), w.to(DEV), out)
    torch.cuda.synchronize()
    assert torch.isfinite(out.float()).all()
    assert _rel(out, ref) < 8e-3, _rel(out, ref)
    # linear_dx takes this path by default for the CNN-B1 shape
    out2 = torch.empty(M, Kd, device=DEV, dtype=torch.bfloat16)
    K.linear_dx(dy.to(DEV), w.to(DEV), out2)
    torch.cuda.synchronize()
    assert torch.equal(out2.cpu(), out.cpu())

