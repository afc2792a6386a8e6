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


def test_mlp_lds_resident_adam_state_matches_hbm(hip_built, monkeypatch):
    """mlp.hip with the p / m / v span brought into LDS by one DMA burst (and the HBM copies written
    only at a launch's last step) == the per-element HBM path, bit for bit, over single- and
    multi-step launches at batch 32 and 64."""
    from pyspark_tf_gke_amd.nn import optimizers

    for B in (32, 64):
        g = torch.Generator().manual_seed(B)
        x = torch.randn(8 * B, 3, generator=g).cuda()
        y = torch.randint(0, 15, (8 * B,), generator=g, dtype=torch.int32).cuda()
        out = []
        for res in ("1", "0"):
            monkeypatch.setenv("PTG_MLP_RES", res)
            torch.manual_seed(0)
            m = build_deep_model(3, 15, device="cuda")
            m.compile(optimizer=optimizers.Adam(1e-2), loss=m.loss, metrics=m.metric_names)
            st = m._stats_buf()
            plan = m._mlp_fusable(x[:B], y[:B], m._strategy())
            assert plan is not None
            for steps, r0 in ((4, 0), (1, 4), (3, 5)):
                m._train_step_mlp(x[r0 * B:(r0 + steps) * B], y[r0 * B:(r0 + steps) * B], st, plan, steps=steps)
            torch.cuda.synchronize()
            out.append((m.store.flat.clone(), m.optimizer.m.clone(), m.optimizer.v.clone(), st.clone()))
        for a, b in zip(out[0], out[1]):
            assert torch.equal(a, b), (B, (a - b).abs().max().item())


def test_mnist_cnn_tracks_reference(hip_built):
    """The MNIST convnet (Conv(relu) -> MaxPool fused into one ConvOp: PReLU alpha 0 + pool epilogue,
    one-kernel backward) vs the fp32 CPU reference path: losses, accuracy and parameters."""
    from pyspark_tf_gke_amd.nn import engine as E

    torch.manual_seed(0)
    x = torch.rand(64, 28, 28, 1)
    y = torch.randint(0, 10, (64,), dtype=torch.int32)
    mg = build_mnist_cnn(device="cuda")
    mc = build_mnist_cnn(device="cpu")
    assert sum(isinstance(op, E.ConvOp) and op.pool is not None for op in mg.ops) == 2
    lg, lc = _steps(mg, x, y, 4), _steps(mc, x, y, 4)
    for a, b in zip(lg, lc):
        assert abs(a["loss"] - b["loss"]) <= 0.02 * abs(b["loss"]) + 1e-3, (a, b)
    pg, pc = mg.store.flat.cpu(), mc.store.flat
    assert torch.allclose(pg, pc, atol=5e-3, rtol=5e-2), float((pg - pc).abs().max())


def test_mnist_cnn_learns(hip_built):
    torch.manual_seed(0)
    m = build_mnist_cnn(device="cuda")
    x = torch.rand(64, 28, 28, 1)
    y = torch.randint(0, 10, (64,), dtype=torch.int32)
    logs = _steps(m, x, y, 20)
    assert logs[-1]["loss"] < logs[0]["loss"]


def test_device_feed_matches_plain_upload(hip_built):
    """fit() over a host Dataset through the pinned-ring / side-stream device feed gives the same
    parameters as the plain per-batch upload (same data, same order), and the feed overlaps: it
    reuses its staging slots."""
    import numpy as np

    from pyspark_tf_gke_amd.data import device_feed as F
    from pyspark_tf_gke_amd.data.dataset import Dataset
    from pyspark_tf_gke_amd.models import build_deep_model
    from pyspark_tf_gke_amd.nn import model as M

    rng = np.random.default_rng(0)
    X = rng.normal(size=(4096, 3)).astype(np.float32)
    y = rng.integers(0, 15, 4096).astype(np.int32)

    def ds():  # a generator source: not the columnar plan, so fit() takes the host path
        return Dataset.from_generator(lambda: ((X[i:i + 256], y[i:i + 256]) for i in range(0, 4096, 256)))

    params = []
    for feed in (True, False):
        M.DEVICE_FEED = feed
        torch.manual_seed(0)
        m = build_deep_model(3, 15, device="cuda")
        m.fit(ds(), epochs=2, verbose=0)
        params.append(m.store.flat.detach().cpu().clone())
    M.DEVICE_FEED = True
    # same batches in the same order; the Dense kernels' atomic split-K reductions are not
    # bitwise deterministic run to run, so compare to fp32 reduction noise
    assert torch.allclose(params[0], params[1], rtol=1e-4, atol=1e-6)
    assert F.STATS["batches"] >= 32


def test_fused_regression_head_matches_unfused(hip_built):
    """CNN-B1 (flat) head as one head_mse_k launch vs the seven-kernel path over 3 steps: same
    losses / metrics, and the parameter updates point the same way (Adam normalises each element's
    step, so elements whose gradient is ~0 can move by +-lr either way: compare the update vectors'
    cosine, not elementwise values)."""
    from pyspark_tf_gke_amd.nn import model as M

    g = torch.Generator().manual_seed(0)
    X = torch.randint(0, 256, (3, 16, 64, 80, 3), generator=g, dtype=torch.uint8)
    Y = torch.rand(3, 16, 2, generator=g) * 60
    res = []
    for fused in (True, False):
        M.FUSED_HEAD = fused
        torch.manual_seed(0)
        m = build_cnn_model((64, 80, 3), flat=True, summary=False, device="cuda")
        p0 = m.store.flat.detach().cpu().clone()
        assert m._head_fusable(X[0].cuda(), None) == fused
        logs = [m.train_on_batch(X[i], Y[i], return_dict=True) for i in range(3)]
        res.append((logs, m.store.flat.detach().cpu() - p0))
    M.FUSED_HEAD = True
    for a, b in zip(res[0][0], res[1][0]):
        for k in ("loss", "mae", "mse"):
            assert abs(a[k] - b[k]) <= 2e-2 * max(1.0, abs(b[k])), (k, a, b)
    u, v = res[0][1], res[1][1]
    cos = float((u * v).sum() / (u.norm() * v.norm()))
    assert cos > 0.98, cos


def test_head_mse_kernel_vs_fp32_reference(hip_built):
    """head_mse_k against fp32 torch on the same split-K sums: dz1, dW2, db2, db1, stats, and the
    accumulator left zeroed."""
    from pyspark_tf_gke_amd.ops import nn as K

    B, K1, N2 = 256, 2048, 2
    g = torch.Generator().manual_seed(1)
    acc = torch.randn(B, K1, generator=g)
    b1 = torch.randn(K1, generator=g) * 0.1
    w2 = torch.randn(N2, K1, generator=g) * 0.02
    b2 = torch.randn(N2, generator=g)
    t = torch.randn(B, N2, generator=g) * 3
    h = torch.relu(acc + b1)
    pred = h @ w2.t() + b2
    d = pred - t
    dp = 2 * d / (B * N2)
    dz = (dp @ w2) * (h > 0)
    dev = "cuda"
    acc_d = acc.to(dev).contiguous()
    dz1 = torch.empty(B, K1, device=dev, dtype=torch.bfloat16)
    dw2 = torch.zeros(N2, K1, device=dev)
    db2 = torch.zeros(N2, device=dev)
    db1 = torch.zeros(K1, device=dev)
    stats = torch.zeros(8, device=dev)
    K.head_mse(acc_d, b1.to(dev), w2.to(dev), b2.to(dev), t.to(dev), dz1, dw2, db2, db1, stats)
    torch.cuda.synchronize()
    assert float(acc_d.abs().max()) == 0.0
    assert torch.allclose(dz1.float().cpu(), dz, rtol=1e-2, atol=1e-6)
    assert torch.allclose(dw2.cpu(), dp.t() @ h, rtol=1e-4, atol=1e-5)
    assert torch.allclose(db2.cpu(), dp.sum(0), rtol=1e-4, atol=1e-6)
    assert torch.allclose(db1.cpu(), dz.sum(0), rtol=1e-4, atol=1e-6)
    st = stats.cpu()
    assert abs(float(st[0]) - float((d * d).mean()) * B) <= 1e-4 * float((d * d).mean()) * B
    assert abs(float(st[1]) - float(d.abs().sum())) <= 1e-4 * float(d.abs().sum())
    assert float(st[3]) == B * N2 and float(st[4]) == B


def test_raw_uint8_first_layer_matches_packed_input(hip_built):
    """The first conv layer reading the raw uint8 [N,H,W,3] batch itself (U8 loaders of
    conv1_pair_pool_k / conv_wgrad_strip_k) == the packed-bf16 path: identical forward (same /255
    rounding), same first-layer weight gradient up to atomic-order noise, same losses.  W = 80 leaves
    a partial 64-pixel tile; H = 62 a partial 4-row tile."""
    from pyspark_tf_gke_amd.nn import engine as E

    g = torch.Generator().manual_seed(1)
    X = torch.randint(0, 256, (3, 16, 62, 80, 3), generator=g, dtype=torch.uint8)
    Y = torch.rand(3, 16, 2, generator=g) * 60
    res = []
    for raw in (True, False):
        E.RAW_U8 = raw
        torch.manual_seed(0)
        m = build_cnn_model((62, 80, 3), flat=True, summary=False, device="cuda")
        pred = m.predict(X[0].cuda()) if hasattr(m, "predict") else None
        first = m.ops[0]
        m.store.zero_grad()
        logs = [m.train_on_batch(X[i], Y[i], return_dict=True) for i in range(3)]
        assert first._raw_u8_ok(X[0].cuda()) == raw
        res.append((torch.as_tensor(pred).float().cpu(), logs, first.conv.kernel.data.detach().cpu().clone()))
    E.RAW_U8 = True
    if not E.CONV1_FUSED:
        assert torch.equal(res[0][0], res[1][0])
    else:
        # conv1.hip takes raw pixels as exact integers with the 1/255 on the accumulators; the packed
        # path rounds x/255 to bf16 first, so the two agree to bf16 rounding, not bitwise
        assert torch.allclose(res[0][0], res[1][0], rtol=2e-2, atol=2e-3)
    for a, b in zip(res[0][1], res[1][1]):
        assert abs(a["loss"] - b["loss"]) <= 1e-2 * max(1.0, abs(b["loss"])), (a, b)
    if not E.CONV1_FUSED:
        assert torch.allclose(res[0][2], res[1][2], rtol=1e-3, atol=1e-5)
    else:  # Adam moves a weight by ~lr per step whatever the gradient's size: 3 steps of 1e-3 at most
        assert (res[0][2] - res[1][2]).abs().max().item() <= 6.5e-3


def _same_training(m0, m1, init, l0, l1):
    """Two runs of the same steps agree: per-step losses, and the parameters up to the run-order noise
    of the fp32-atomic weight-gradient sums (Adam turns noise-level gradients of tiny parameters into
    full-size steps, so the check is on the whole update: |p1 - p0| <= 5% of |p0 - init|; a skipped
    or misplaced update differs by its whole size)."""
    np.testing.assert_allclose(l1, l0, rtol=2e-3)
    d = (m1.store.flat - m0.store.flat).norm().item()
    u = (m0.store.flat - init).norm().item()
    assert u > 0 and d <= 0.05 * u, (d, u)
    for p0, p1 in zip(m0.ops[-2].dense.params, m1.ops[-2].dense.params):
        dd = (p1.data - p0.data).norm().item()
        assert dd <= 0.05 * max((p0.data - init[p0.offset:p0.offset + p0.numel].view(p0.data.shape)).norm().item(),
                                1e-12), (p0.name, dd)


def test_persistent_work_queue_mode_matches_static(hip_built):
    """Work-queue mode of the persistent conv kernels (tile chunks claimed from per-stream counters)
    computes the same training step as static per-workgroup ranges, with the side-stream weight
    gradients running concurrently with the dgrad chain (a shared counter would make each kernel skip
    the chunks the other claimed)."""
    from pyspark_tf_gke_amd.ops import nn as K

    torch.manual_seed(0)
    xs = [torch.randint(0, 256, (64, 128, 160, 3), dtype=torch.uint8, device="cuda") for _ in range(2)]
    ys = [torch.rand(64, 2, device="cuda") * 100 for _ in range(2)]

    def run(dynamic):
        K.set_persist_mode(dynamic)
        try:
            torch.manual_seed(1)
            m = build_cnn_model((128, 160, 3), flat=True, summary=False, device="cuda")
            init = m.store.flat.clone()
            st = m._stats_buf()
            losses = []
            for i in range(5):
                st.zero_()
                m.train_step_fast(xs[i % 2], ys[i % 2], st)
                losses.append(m._logs_from(st)["loss"])
            torch.cuda.synchronize()
            return m, losses, init
        finally:
            K.set_persist_mode(None)

    m0, l0, init = run(False)
    m1, l1, _ = run(True)
    _same_training(m0, m1, init, l0, l1)


def test_tape_loop_overlapped_adam_same_training(hip_built):
    """The reference's GradientTape loop (train_tf_ps.py:616-631): with the side-stream backward
    and the big Dense Adam on an auxiliary stream waiting only for its dW (tape.py), the weights,
    moments and losses match the serial tape loop (PTG_TAPE_OVERLAP=0) up to run-order noise."""
    from pyspark_tf_gke_amd import nn
    from pyspark_tf_gke_amd.nn import tape as T

    torch.manual_seed(0)
    xs = [torch.randint(0, 256, (16, 64, 80, 3), dtype=torch.uint8, device="cuda") for _ in range(2)]
    ys = [torch.rand(16, 2, device="cuda") * 60 for _ in range(2)]

    def run(overlap):
        torch.manual_seed(1)
        m = build_cnn_model((64, 80, 3), flat=True, summary=False, device="cuda")
        init = m.store.flat.clone()
        opt = nn.optimizers.Adam(learning_rate=1e-3)
        lo = nn.losses.MeanSquaredError()
        losses, used = [], []
        old = T.OVERLAP
        T.OVERLAP = overlap
        try:
            for i in range(6):
                with nn.GradientTape() as tape:
                    p = m(xs[i % 2], training=True)
                    lv = lo(ys[i % 2], p)
                g = tape.gradient(lv, m.trainable_variables)
                used.append(bool(m._tape_ready) and T._overlap_ok(opt, list(zip(g, m.trainable_variables)), m._tape_ready))
                opt.apply_gradients(zip(g, m.trainable_variables))
                losses.append(float(lv))
        finally:
            T.OVERLAP = old
        torch.cuda.synchronize()
        assert opt.iterations == 6 and m.store.grad_clean
        return m, losses, init, used

    m0, l0, init, u0 = run(False)
    m1, l1, _, u1 = run(True)
    assert not any(u0) and all(u1), (u0, u1)  # the overlapped path really ran
    _same_training(m0, m1, init, l0, l1)


def test_tape_fused_head_lazy_dw_matches_fit(hip_built):
    """The tape loop on CNN-B1 (flat) takes fit()'s fused head (MSE on the _HeadPred) and the big
    Dense dW fused with Adam at apply_gradients (_LazyDW): same training as train_step_fast, and
    both deferred paths really ran."""
    from pyspark_tf_gke_amd import nn
    from pyspark_tf_gke_amd.nn import tape as T

    torch.manual_seed(0)
    xs = [torch.randint(0, 256, (16, 64, 80, 3), dtype=torch.uint8, device="cuda") for _ in range(2)]
    ys = [torch.rand(16, 2, device="cuda") * 60 for _ in range(2)]
    torch.manual_seed(1)
    mf = build_cnn_model((64, 80, 3), flat=True, summary=False, device="cuda")
    init = mf.store.flat.clone()
    st = mf._stats_buf()
    lf = []
    for i in range(6):
        st.zero_()
        mf.train_step_fast(xs[i % 2], ys[i % 2], st)
        lf.append(float(st[0] / st[4]))
    torch.manual_seed(1)
    mt = build_cnn_model((64, 80, 3), flat=True, summary=False, device="cuda")
    assert torch.equal(mt.store.flat, init)
    opt = nn.optimizers.Adam(learning_rate=1e-3)
    lo = nn.losses.MeanSquaredError()
    lt, kinds = [], []
    for i in range(6):
        with nn.GradientTape() as tape:
            p = mt(xs[i % 2], training=True)
            lv = lo(ys[i % 2], p)
        g = tape.gradient(lv, mt.trainable_variables)
        kinds.append((isinstance(p, T._HeadPred) and p._lz.state == "fused",
                      any(isinstance(t, T._LazyGrad) and t._lz.pending for t in g)))
        opt.apply_gradients(zip(g, mt.trainable_variables))
        lt.append(float(lv))
    torch.cuda.synchronize()
    assert all(a and b for a, b in kinds), kinds
    assert mt._lazy_dw is None and opt.iterations == 6
    _same_training(mf, mt, init, lf, lt)


def test_ps_one_worker_tape_overlap_same_training(hip_built):
    """The reference's primary loop (ParameterServerStrategy + ClusterCoordinator.schedule of the
    GradientTape closure, train_tf_ps.py:612-645) with one worker: the round-commit update takes the
    overlapped Dense Adam (ps.py _apply_local) and trains exactly like the serial update."""
    from pyspark_tf_gke_amd import distribute as ds
    from pyspark_tf_gke_amd import nn
    from pyspark_tf_gke_amd.cli.train import make_parameter_server_strategy
    from pyspark_tf_gke_amd.nn import tape as T

    torch.manual_seed(0)
    xs = [torch.randint(0, 256, (16, 64, 80, 3), dtype=torch.uint8, device="cuda") for _ in range(2)]
    ys = [torch.rand(16, 2, device="cuda") * 60 for _ in range(2)]

    def run(overlap):
        strategy = make_parameter_server_strategy(1, 1)
        with strategy.scope():
            torch.manual_seed(1)
            m = build_cnn_model((64, 80, 3), flat=True, summary=False, device="cuda")
            opt = nn.optimizers.Adam(learning_rate=1e-3)
            lo = nn.losses.MeanSquaredError()
        init = m.store.flat.clone()
        coord = ds.ClusterCoordinator(strategy)
        losses, used = [], []

        def step_fn(i):
            with nn.GradientTape() as tape:
                p = m(xs[i % 2], training=True)
                lv = lo(ys[i % 2], p)
            g = tape.gradient(lv, m.trainable_variables)
            opt.apply_gradients(zip(g, m.trainable_variables))
            return lv

        old, orig = T.OVERLAP, T._apply_overlapped

        def counted(*a):
            used.append(1)
            return orig(*a)

        T.OVERLAP, T._apply_overlapped = overlap, counted
        try:
            for i in range(6):
                r = coord.schedule(lambda i=i: strategy.run(step_fn, args=(i,)))
                coord.join()
                losses.append(float(r.fetch()))
        finally:
            T.OVERLAP, T._apply_overlapped = old, orig
        torch.cuda.synchronize()
        assert opt.iterations == 6 and len(used) == (6 if overlap else 0), used
        return m, losses, init

    m0, l0, init = run(False)
    m1, l1, _ = run(True)
    _same_training(m0, m1, init, l0, l1)


def test_flip_in_adam_matches_flip_kernel(hip_built, monkeypatch):
    """The fused step's Adam pass writes the conv layers' flipped dgrad filters (adam_multi_k): after
    the first step no flip kernel runs, and five CNN-B1 steps train as with the per-backward flip.
    A weight write outside the optimizer (set_weights) invalidates the written filters."""
    from pyspark_tf_gke_amd.nn import model as M
    from pyspark_tf_gke_amd.nn import engine as E
    from pyspark_tf_gke_amd.ops import nn as K

    torch.manual_seed(0)
    xs = [torch.randint(0, 256, (32, 128, 160, 3), dtype=torch.uint8, device="cuda") for _ in range(2)]
    ys = [torch.rand(32, 2, device="cuda") * 100 for _ in range(2)]
    calls = []
    orig = K.conv_flip_weights_multi
    monkeypatch.setattr(K, "conv_flip_weights_multi", lambda jobs: (calls.append(len(jobs)), orig(jobs)))

    def run(flag):
        monkeypatch.setattr(M, "FLIP_IN_ADAM", flag)
        calls.clear()
        torch.manual_seed(1)
        m = build_cnn_model((128, 160, 3), flat=True, summary=False, device="cuda")
        init = m.store.flat.clone()
        st = m._stats_buf()
        losses = []
        for i in range(5):
            st.zero_()
            m.train_step_fast(xs[i % 2], ys[i % 2], st)
            losses.append(m._logs_from(st)["loss"])
        torch.cuda.synchronize()
        return m, losses, init, list(calls)

    m0, l0, init, c0 = run(False)
    m1, l1, _, c1 = run(True)
    assert len(c0) == 5 and all(c == 4 for c in c0), c0
    assert c1 == [4], c1  # only the first backward flips; every later one reads the Adam-written filters
    _same_training(m0, m1, init, l0, l1)
    # the written filters are exactly what the flip kernel makes of the current bf16 weights
    for op in m1.ops:
        if isinstance(op, E.ConvOp) and op.flip_spec() is not None:
            ref = torch.empty_like(op._wf_buf)
            K.conv_flip_weights(op.conv.kernel.bf16, ref)
            torch.cuda.synchronize()
            assert torch.equal(ref, op._wf_buf), op.name
    assert m1._flips_ready()
    m1.set_weights(m1.get_weights())
    assert not m1._flips_ready()
