"""conv32.hip (5x5 'same' conv as an implicit GEMM on v_mfma_f32_32x32x16_bf16) against the fp32
PyTorch reference of the same op (F.conv2d on the bf16 operands), for the CNN-B1 layer shapes it
serves (train_tf_ps.py:357-364) and their data gradients (flipped filters), with the fused
PReLU + 2x2 max-pool / PReLU epilogues."""
import pytest
import torch
import torch.nn.functional as F

from pyspark_tf_gke_amd.ops import nn as K

pytestmark = pytest.mark.gpu

# (H, W, C, Cout, epi): forward layers 3-5 and the data gradients of layers 3-5
CASES = [(64, 80, 16, 32, "pool"), (32, 40, 32, 64, "pool"), (16, 20, 64, 64, "prelu"),
         (64, 80, 32, 16, None), (32, 40, 64, 32, None), (16, 20, 64, 64, None), (16, 20, 64, 24, None)]


@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")
@pytest.mark.parametrize("N", [3, 160])  # 160: 320-pixel tiles (C = 64: two half-channel passes); 3: 160-pixel tiles
@pytest.mark.parametrize("H,W,C,Co,epi", CASES)
def test_conv32_matches_fp32_reference(hip_built, H, W, C, Co, epi, N):
    g = torch.Generator(device="cuda").manual_seed(H * 100 + C + Co)
    x = (torch.randn((N, H, W, C), device="cuda", generator=g)).bfloat16()
    w = (torch.randn((Co, 5, 5, C), device="cuda", generator=g) * 0.05).bfloat16()
    b = torch.randn(Co, device="cuda", generator=g) * 0.1 if epi else None
    al = (torch.rand((H, W, Co), device="cuda", generator=g) * 0.5) if epi else None
    assert K.conv32_supported(H, W, C, Co, 5, 2, epi)
    z = torch.empty((N, H, W, Co), device="cuda", dtype=torch.bfloat16)
    aux = None
    if epi == "pool":
        aux = torch.empty((N, H // 2, W // 2, Co), device="cuda", dtype=torch.bfloat16)
    elif epi == "prelu":
        aux = torch.empty_like(z)
    K.conv32(x, w, b, z, al, aux, epi)
    torch.cuda.synchronize()
    ref = F.conv2d(x.float().permute(0, 3, 1, 2), w.float().permute(0, 3, 1, 2), b, padding=2).permute(0, 2, 3, 1)
    zf = z.float()
    err = (zf - ref).abs().max().item()
    assert err <= 2e-2 * max(1.0, ref.abs().max().item()), err
    # the epilogue sees the bf16-rounded z
    if epi is not None:
        zr = z.float()
        y = torch.where(zr > 0, zr, al * zr)
        if epi == "pool":
            yr = F.max_pool2d(y.permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1)
        else:
            yr = y
        assert torch.allclose(aux.float(), yr.bfloat16().float(), atol=1e-2, rtol=1e-2)
