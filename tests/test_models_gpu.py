"""End-to-end model steps on the MI355X vs the same model on the CPU reference path (same seed,
same data): the fused HIP engine must track the fp32 reference within bf16 tolerance."""
import numpy as np
import pytest
import torch

from pyspark_tf_gke_amd import _native
from pyspark_tf_gke_amd.models import build_cnn_model, build_deep_model, build_mnist_cnn

pytestmark = pytest.mark.gpu


def test_native_library_is_loaded(hip_built):
    assert _native.HIP_LIB_PATH.exists()
    assert str(_native.HIP_LIB_PATH) in _native.loaded_paths()


def _steps(model, x, y, n):
    out = []
    for _ in range(n):
        out.append(model.train_on_batch(x, y, return_dict=True))
    return out


def test_cnn_small_input_tracks_reference(hip_built):
    torch.manual_seed(0)
    x = torch.rand(4, 32, 40, 3)
    y = torch.rand(4, 2) * 30
    mg = build_cnn_model((32, 40, 3), flat=True, summary=False, device="cuda")
    mc = build_cnn_model((32, 40, 3), flat=True, summary=False, device="cpu")
    lg = _steps(mg, x, y, 3)
    lc = _steps(mc, x, y, 3)
    for a, b in zip(lg, lc):
        assert abs(a["loss"] - b["loss"]) <= 0.05 * abs(b["loss"]) + 1e-3, (a, b)
    pg = mg.store.flat.cpu()
    pc = mc.store.flat
    assert torch.allclose(pg, pc, atol=5e-3, rtol=5e-2)


def test_cnn_b1_full_size_step(hip_built):
    torch.manual_seed(0)
    m = build_cnn_model((256, 320, 3), flat=True, summary=False, device="cuda")
    x = torch.rand(8, 256, 320, 3)
    y = torch.rand(8, 2) * 200
    logs = _steps(m, x, y, 5)
    assert all(np.isfinite(l["loss"]) for l in logs)
    assert logs[-1]["loss"] < logs[0]["loss"]


def test_mlp_tracks_reference(hip_built):
    torch.manual_seed(0)
    x = torch.randn(64, 3)
    y = torch.randint(0, 15, (64,), dtype=torch.int32)
    mg = build_deep_model(3, 15, device="cuda")
    mc = build_deep_model(3, 15, device="cpu")
    lg, lc = _steps(mg, x, y, 5), _steps(mc, x, y, 5)
    for a, b in zip(lg, lc):
        assert abs(a["loss"] - b["loss"]) < 1e-3, (a, b)
        assert abs(a["accuracy"] - b["accuracy"]) < 1e-6


def test_mnist_cnn_learns(hip_built):
    torch.manual_seed(0)
    m = build_mnist_cnn(device="cuda")
    x = torch.rand(64, 28, 28, 1)
    y = torch.randint(0, 10, (64,), dtype=torch.int32)
    logs = _steps(m, x, y, 20)
    assert logs[-1]["loss"] < logs[0]["loss"]
