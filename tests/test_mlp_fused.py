"""The reference's CSV MLP (train_tf_ps.py:328-343: 3 -> 16 -> 32 -> 64 -> C softmax, Adam,
SparseCategoricalCrossentropy) trained one whole step per launch (csrc/kernels/mlp.hip).

CPU: the fp32 oracle of the fused step (ops/reference.py ``mlp_train``) equals the layer-by-layer
engine step (fused-softmax loss kernel, dense backward, flat Adam) over several steps.
GPU: the HIP kernel equals that fp32 oracle (one launch per step, and ``steps`` > 1 per launch),
metric sums included, for the classifier and an MSE regressor; ``fit()`` of the MLP goes through
the fused kernel."""
import pytest
import torch

from pyspark_tf_gke_amd import nn
from pyspark_tf_gke_amd.models import build_deep_model
from pyspark_tf_gke_amd.ops import nn as K
from pyspark_tf_gke_amd.ops import reference as ref


def _plan(m):
    ops = m.ops
    dims = [ops[0].dense.fan_in] + [op.dense.units for op in ops]
    acts = [1 if op.act == "relu" else 0 for op in ops[:-1]] + [0]
    return dims, acts, [op.dense.kernel.offset for op in ops], [op.dense.bias.offset for op in ops]


def _data(B, steps, C=15, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(steps * B, 3, generator=g)
    y = torch.randint(0, C, (steps * B,), generator=g).to(torch.int32)
    return x, y


def test_mlp_oracle_matches_engine_step_cpu():
    torch.manual_seed(0)
    m = build_deep_model(3, 15, device="cpu")
    ref_m = build_deep_model(3, 15, device="cpu")
    ref_m.store.flat.copy_(m.store.flat)
    B, steps = 32, 4
    x, y = _data(B, steps)
    stats = torch.zeros(8)
    for s in range(steps):
        xb, yb = m._prep_batch(x[s * B:(s + 1) * B], y[s * B:(s + 1) * B])
        m.train_step(xb, yb, stats)
    dims, acts, wo, bo = _plan(ref_m)
    opt = ref_m.optimizer
    opt.build(ref_m.store)
    st2 = torch.zeros(8)
    ref.mlp_train(x, y, ref_m.store.flat, opt.m, opt.v, None, st2, dims, acts, wo, bo, steps, 0, opt.learning_rate,
                  opt.beta_1, opt.beta_2, opt.epsilon, 0)
    assert torch.allclose(m.store.flat, ref_m.store.flat, atol=1e-6, rtol=1e-5)
    assert torch.allclose(stats, st2, rtol=1e-4, atol=1e-4)


gpu = pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a GPU")


@pytest.mark.gpu
@gpu
@pytest.mark.parametrize("B,steps,kind", [(32, 1, 0), (64, 1, 0), (64, 3, 0), (128, 2, 0), (7, 2, 0), (32, 2, 1)])
def test_mlp_kernel_matches_fp32_oracle(hip_built, B, steps, kind):
    torch.manual_seed(1)
    C = 15 if kind == 0 else 2
    m = build_deep_model(3, C, device="cuda")
    if kind == 1:  # the same stack as a regressor: linear head + MSE
        m.ops[-1].dense.activation = "linear"
        m.ops[-1].act = "linear"
        m.ops[-1].logits_only = False
    dims, acts, wo, bo = _plan(m)
    x, y = _data(B, steps, C)
    if kind == 1:
        y = torch.randn(steps * B, C)
    flat0 = m.store.flat.clone()
    mm = torch.rand_like(flat0) * 1e-3
    vv = torch.rand_like(flat0) * 1e-6
    # GPU kernel
    p, m1, v1 = flat0.clone(), mm.clone(), vv.clone()
    pbf = torch.zeros_like(p, dtype=torch.bfloat16)
    st1 = torch.zeros(8, device="cuda")
    xd, yd = x.cuda(), y.cuda()
    K.mlp_train(xd, yd, p, m1, v1, pbf, st1, dims, acts, wo, bo, steps, kind, 1e-3, 0.9, 0.999, 1e-7, 5)
    torch.cuda.synchronize()
    # fp32 oracle
    p2, m2, v2 = flat0.cpu(), mm.cpu(), vv.cpu()
    st2 = torch.zeros(8)
    ref.mlp_train(x, y, p2, m2, v2, None, st2, dims, acts, wo, bo, steps, kind, 1e-3, 0.9, 0.999, 1e-7, 5)
    n = sum(d1 * d0 for d0, d1 in zip(dims[:-1], dims[1:])) + sum(dims[1:])
    assert torch.allclose(p.cpu(), p2, atol=2e-6, rtol=1e-5), float((p.cpu() - p2).abs().max())
    assert torch.allclose(m1.cpu(), m2, atol=1e-7, rtol=1e-4)
    assert torch.allclose(v1.cpu(), v2, atol=1e-10, rtol=1e-4)
    used = torch.zeros_like(p2, dtype=torch.bool)
    for l in range(len(wo)):
        used[wo[l]:wo[l] + dims[l + 1] * dims[l]] = True
        used[bo[l]:bo[l] + dims[l + 1]] = True
    assert int(used.sum()) == n
    assert torch.equal(pbf.cpu()[used], p.cpu()[used].to(torch.bfloat16))
    assert torch.allclose(st1.cpu(), st2, rtol=1e-4, atol=1e-3)


@pytest.mark.gpu
@gpu
def test_mlp_fit_uses_fused_step(hip_built, monkeypatch):
    torch.manual_seed(2)
    m = build_deep_model(3, 15, device="cuda")
    calls = []
    orig, orig_run = K.mlp_train, K.MlpStep.run
    monkeypatch.setattr(K, "mlp_train", lambda *a, **k: (calls.append(1), orig(*a, **k))[1])
    monkeypatch.setattr(K.MlpStep, "run", lambda self, *a, **k: (calls.append(a[2]), orig_run(self, *a, **k))[1])
    x, y = _data(64, 20)
    h = m.fit(x.numpy(), y.numpy(), batch_size=64, epochs=2, verbose=0)
    # every one of the 40 steps ran inside a fused launch (cached launches count their steps)
    assert sum(calls) >= 2 * 20 and all(v == v for v in h.history["loss"])
    assert h.history["loss"][-1] < h.history["loss"][0] + 1e-3


@pytest.mark.gpu
@gpu
def test_mlp_fit_dataset_grouped_launches_match_per_batch_engine(hip_built, monkeypatch):
    """The reference's local MLP fit (cli/train.py: from_tensor_slices -> shuffle(3000) -> batch -> repeat,
    steps_per_epoch): columns uploaded once, groups of full batches per fused launch (with a group
    split across the epoch boundary) == the layer-by-layer engine step per batch."""
    from pyspark_tf_gke_amd.data import Dataset
    from pyspark_tf_gke_amd.nn import model as M

    g = torch.Generator().manual_seed(4)
    X = torch.randn(1000, 3, generator=g).numpy()
    y = torch.randint(0, 15, (1000,), generator=g).to(torch.int32).numpy()

    def run(fused):
        monkeypatch.setattr(M, "MLP_FUSED", fused)
        torch.manual_seed(5)
        m = build_deep_model(3, 15, device="cuda")
        m.compile(optimizer=nn.optimizers.Adam(1e-3), loss=nn.losses.SparseCategoricalCrossentropy(),
                  metrics=["accuracy"], steps_per_execution=5)
        ds = Dataset.from_tensor_slices((X, y)).shuffle(300, seed=1).batch(32).repeat().prefetch(1)
        calls = []
        orig, orig_run = K.mlp_train, K.MlpStep.run
        monkeypatch.setattr(K, "mlp_train", lambda *a, **k: (calls.append(a[11]), orig(*a, **k))[1])
        monkeypatch.setattr(K.MlpStep, "run", lambda self, *a, **k: (calls.append(a[2]), orig_run(self, *a, **k))[1])
        h = m.fit(ds, epochs=3, steps_per_epoch=13, verbose=0)
        monkeypatch.setattr(K, "mlp_train", orig)
        monkeypatch.setattr(K.MlpStep, "run", orig_run)
        torch.cuda.synchronize()
        return m.store.flat.clone(), h.history["loss"], calls, m.optimizer.iterations

    fa, la, ca, ia = run(True)
    fb, lb, cb, ib = run(False)
    assert ia == ib == 39 and not cb and sum(ca) == 39 and max(ca) == 5, (ia, ib, ca)
    assert torch.allclose(fa, fb, rtol=1e-3, atol=1e-5), float((fa - fb).abs().max())
    assert all(abs(a - b) <= 1e-3 * max(1.0, abs(b)) for a, b in zip(la, lb)), (la, lb)


@pytest.mark.gpu
@gpu
@pytest.mark.parametrize("B", [32, 128])
def test_mlp_cached_launch_matches_direct_launch(hip_built, B):
    """MlpStep (bound pointers, device-side Adam step counter) == ptg_mlp_train with the host
    counter, bit for bit, over 3 cached launches of 2 steps each (the counter advances on the
    device) and a resync after the host counter moves."""
    torch.manual_seed(3)
    m = build_deep_model(3, 15, device="cuda")
    dims, acts, wo, bo = _plan(m)
    x, y = _data(B, 2, 15)
    xd, yd = x.cuda(), y.cuda()
    flat0 = m.store.flat.clone()
    outs = []
    for cached in (True, False):
        p = flat0.clone()
        mm, vv = torch.zeros_like(p), torch.zeros_like(p)
        pbf = torch.zeros_like(p, dtype=torch.bfloat16)
        st = torch.zeros(8, device="cuda")
        t = 0
        ms = K.MlpStep(p, mm, vv, pbf, st, dims, acts, wo, bo, B, 0, 1e-3, 0.9, 0.999, 1e-7, 0) if cached else None
        for rep in range(4):
            if rep == 3:
                t += 5  # the host counter moved (e.g. set_iterations): the device counter resyncs
            if cached:
                ms.run(xd, yd, 2, t)
            else:
                K.mlp_train(xd, yd, p, mm, vv, pbf, st, dims, acts, wo, bo, 2, 0, 1e-3, 0.9, 0.999, 1e-7, t)
            t += 2
        torch.cuda.synchronize()
        outs.append((p.cpu(), mm.cpu(), vv.cpu(), st.cpu()))
    for a, b in zip(*outs):
        assert torch.equal(a, b)
