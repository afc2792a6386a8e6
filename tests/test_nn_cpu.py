"""Keras-surface behaviour of the training runtime on the CPU (reference) path."""
import json
import zipfile

import numpy as np
import pytest
import torch

from pyspark_tf_gke_amd import nn
from pyspark_tf_gke_amd.data import Dataset
from pyspark_tf_gke_amd.models import (CNN_A1_PARAMS, CNN_B1_PARAMS, build_cnn_a1, build_cnn_model,
                                       build_deep_model, build_mnist_cnn)


def test_param_counts_match_reference_summaries(capsys):
    m = build_cnn_model((256, 320, 3), flat=True, summary=True, device="cpu")
    assert m.count_params() == CNN_B1_PARAMS  # 150-320-by-256-B1-model.txt:38
    out = capsys.readouterr().out
    assert "p_re_lu_4 (PReLU)" in out and "41,945,088" in out and "Total params: 43,368,850" in out
    a1 = build_cnn_a1((256, 320, 3), device="cpu")
    assert a1.count_params() == CNN_A1_PARAMS  # 100-320-by-256-A1-model.txt:27
    mlp = build_deep_model(3, 15, device="cpu")
    assert mlp.count_params() == 3695  # SURVEY §2.1 derived facts


def test_layer_names_follow_keras():
    m = build_cnn_model((32, 40, 3), flat=False, summary=False, device="cpu")
    names = [l.name for l in m.layers]
    assert names[:3] == ["conv2d", "p_re_lu", "max_pooling2d"]
    assert "global_average_pooling2d" in names and names[-1] == "dense_1"


def test_mlp_fit_history_and_validation():
    rng = np.random.default_rng(0)
    X = rng.normal(size=(400, 3)).astype(np.float32)
    y = (X[:, 0] > 0).astype(np.int32) + 2 * (X[:, 1] > 0).astype(np.int32)
    m = build_deep_model(3, 4, device="cpu")
    ds = Dataset.from_tensor_slices((X[:320], y[:320])).shuffle(300, seed=1).batch(32).repeat()
    val = Dataset.from_tensor_slices((X[320:], y[320:])).batch(32)
    h = m.fit(ds, epochs=8, steps_per_epoch=10, validation_data=val, verbose=0)
    assert set(h.history) == {"loss", "accuracy", "val_loss", "val_accuracy"}
    assert len(h.history["loss"]) == 8
    assert h.history["loss"][-1] < h.history["loss"][0]
    assert h.history["accuracy"][-1] > 0.5
    p = m.predict(X[:5])
    assert p.shape == (5, 4) and np.allclose(p.sum(1), 1.0, atol=1e-5)


def test_cnn_fit_mse_metrics():
    x = np.random.default_rng(0).random((16, 32, 40, 3)).astype(np.float32)
    y = (np.random.default_rng(1).random((16, 2)) * 30).astype(np.float32)
    m = build_cnn_model((32, 40, 3), flat=True, summary=False, device="cpu")
    h = m.fit(x, y, batch_size=8, epochs=3, verbose=0)
    assert set(h.history) == {"loss", "mae", "mse"}
    assert abs(h.history["loss"][0] - h.history["mse"][0]) < 1e-3 * h.history["mse"][0]
    assert h.history["loss"][-1] < h.history["loss"][0]


def test_save_and_load_roundtrip(tmp_path):
    m = build_cnn_model((32, 40, 3), flat=True, summary=False, device="cpu")
    x = np.random.default_rng(0).random((4, 32, 40, 3)).astype(np.float32)
    before = m.predict(x)
    path = str(tmp_path / "model.keras")
    m.save(path)
    with zipfile.ZipFile(path) as zf:
        cfg = json.loads(zf.read("config.json"))
        assert {"config.json", "metadata.json", "model.weights.safetensors"} <= set(zf.namelist())
    assert cfg["config"]["layers"][1]["class_name"] == "Conv2D"
    m2 = nn.load_model(path, device="cpu")
    after = m2.predict(x)
    assert np.allclose(before, after, atol=1e-4)
    w = m2.get_weights()
    assert w[0].shape == (5, 5, 3, 8)  # Keras kernel layout [KH, KW, Cin, Cout]


def test_gradient_tape_custom_loop_matches_fit_step():
    """The reference's PS step body (train_tf_ps.py:616-631) runs unchanged on the engine."""
    rng = np.random.default_rng(0)
    X = rng.normal(size=(64, 3)).astype(np.float32)
    y = rng.integers(0, 5, 64).astype(np.int32)
    m1 = build_deep_model(3, 5, device="cpu")
    m2 = build_deep_model(3, 5, device="cpu")
    opt = nn.optimizers.Adam(learning_rate=1e-3)
    loss_obj = nn.losses.SparseCategoricalCrossentropy()
    acc = nn.metrics.SparseCategoricalAccuracy()
    for _ in range(3):
        with nn.GradientTape() as tape:
            logits = m1(X, training=True)
            loss = loss_obj(y, logits)
        grads = tape.gradient(loss, m1.trainable_variables)
        opt.apply_gradients(zip(grads, m1.trainable_variables))
        acc.update_state(y, logits)
        m2.train_on_batch(X, y)
    assert torch.allclose(m1.store.flat, m2.store.flat, atol=1e-6)
    assert 0.0 <= float(acc.result()) <= 1.0


def test_mnist_cnn_cpu_learns():
    m = build_mnist_cnn(device="cpu")
    x = torch.rand(32, 28, 28, 1)
    y = torch.randint(0, 10, (32,), dtype=torch.int32)
    l0 = m.train_on_batch(x, y, return_dict=True)["loss"]
    for _ in range(10):
        l1 = m.train_on_batch(x, y, return_dict=True)["loss"]
    assert l1 < l0


def test_odd_spatial_pooling_floor():
    m = build_cnn_model((36, 44, 3), flat=True, summary=False, device="cpu")
    assert m.layers[-4].out_shape == (2, 2, 64)
    x = torch.rand(2, 36, 44, 3)
    y = torch.rand(2, 2)
    assert np.isfinite(m.train_on_batch(x, y, return_dict=True)["loss"])


def test_conv1_reference_matches_autograd():
    """The fp32 oracle of the fused first-layer kernels (ops/reference.py conv1_fwd_pm / conv1_bwd_pm,
    which the conv1.hip GPU tests compare against) equals autograd through
    conv -> bias -> PReLU -> 2x2 max-pool on the same bf16-rounded z."""
    from pyspark_tf_gke_amd.ops import reference as R

    torch.manual_seed(0)
    N, H, W = 2, 8, 12
    x = torch.randint(0, 256, (N, H, W, 3), dtype=torch.uint8)
    w = (torch.randn(8, 5, 5, 4) * 0.2).to(torch.bfloat16)
    b, alpha = torch.randn(8) * 0.1, torch.rand(H, W, 8) * 0.5
    dp = torch.randn(N, H // 2, W // 2, 8).to(torch.bfloat16)
    p = torch.empty(N, H // 2, W // 2, 8)
    R.conv1_fwd_pm(x, w, b, alpha, p)
    dw, da, db = torch.zeros(8, 5, 5, 4), torch.zeros(H, W, 8), torch.zeros(8)
    R.conv1_bwd_pm(x, w, b, alpha, dp, dw, da, db)

    xin = R.conv1_input(x).permute(0, 3, 1, 2)
    wf = w.float().detach().requires_grad_(True)
    bf = b.clone().requires_grad_(True)
    af = alpha.clone().requires_grad_(True)
    z = torch.nn.functional.conv2d(xin, wf.permute(0, 3, 1, 2), bf, padding=2).permute(0, 2, 3, 1)
    z = z + (z.to(torch.bfloat16).float() - z).detach()  # the kernels' bf16 rounding, straight-through
    y = torch.where(z > 0, z, af * z)
    pool = torch.nn.functional.max_pool2d(y.permute(0, 3, 1, 2), 2, 2).permute(0, 2, 3, 1)
    pool.backward(dp.float())
    assert torch.allclose(p, pool.detach(), atol=1e-6)
    # dZ is bf16 in the kernels (and their oracle): 2^-8 relative per term of dW / dbias
    assert torch.allclose(dw, wf.grad, rtol=1e-2, atol=1e-2)
    assert torch.allclose(db, bf.grad, rtol=1e-2, atol=1e-2)
    assert torch.allclose(da, af.grad, rtol=1e-3, atol=1e-3)


def _tape_step(m, opt, x, y, touch=None):
    loss_obj = nn.losses.MeanSquaredError()
    with nn.GradientTape() as tape:
        pred = m(x, training=True)
        loss = loss_obj(y, pred)
    grads = tape.gradient(loss, m.trainable_variables)
    if touch is not None:
        touch(grads)
    opt.apply_gradients(zip(grads, m.trainable_variables))
    return grads


def test_tape_lazy_dense_dw_matches_train_on_batch():
    """A CNN-B1-shaped tape loop (flat head, big Dense): the deferred Dense dW fused with Adam at
    apply_gradients (nn/tape.py _LazyDW) gives the train_on_batch weights."""
    from pyspark_tf_gke_amd.nn import tape as T

    torch.manual_seed(0)
    x = torch.rand(4, 32, 40, 3)
    y = torch.rand(4, 2)
    m1 = build_cnn_model((32, 40, 3), flat=True, summary=False, device="cpu")
    m2 = build_cnn_model((32, 40, 3), flat=True, summary=False, device="cpu")
    m2.set_weights(m1.get_weights())
    m2.compile(optimizer=nn.optimizers.Adam(1e-3), loss="mse")
    opt = nn.optimizers.Adam(1e-3)
    lazies = []
    saved = T.TAPE_HEAD
    T.TAPE_HEAD = False  # the same unfused tail as train_on_batch on the CPU: bitwise-equal inputs to Adam
    try:
        for _ in range(3):
            _tape_step(m1, opt, x, y, touch=lambda g: lazies.extend(t for t in g if isinstance(t, T._LazyGrad)))
            m2.train_on_batch(x, y)
    finally:
        T.TAPE_HEAD = saved
    assert lazies, "the big Dense kernel gradient should be deferred"
    assert all(not t._lz.pending for t in lazies)
    assert m1._lazy_dw is None
    assert torch.allclose(m1.store.flat, m2.store.flat, atol=1e-5)


def test_tape_lazy_dense_dw_materializes_on_read():
    """Reading a deferred gradient computes it (the plain update path then runs), and a gradient()
    followed by another forward without apply_gradients flushes it before the workspace is reused."""
    from pyspark_tf_gke_amd.nn import tape as T

    torch.manual_seed(1)
    x = torch.rand(4, 32, 40, 3)
    y = torch.rand(4, 2)
    m1 = build_cnn_model((32, 40, 3), flat=True, summary=False, device="cpu")
    m2 = build_cnn_model((32, 40, 3), flat=True, summary=False, device="cpu")
    m2.set_weights(m1.get_weights())
    o1, o2 = nn.optimizers.Adam(1e-3), nn.optimizers.Adam(1e-3)
    seen = {}

    def norms(grads):
        seen["n"] = [float(torch.linalg.vector_norm(g)) for g in grads]

    saved = T.LAZY_DW
    try:
        _tape_step(m1, o1, x, y, touch=norms)
        T.LAZY_DW = False
        _tape_step(m2, o2, x, y, touch=lambda g: seen.setdefault("ref", [float(torch.linalg.vector_norm(t)) for t in g]))
    finally:
        T.LAZY_DW = saved
    assert np.allclose(seen["n"], seen["ref"], rtol=1e-5)
    assert torch.allclose(m1.store.flat, m2.store.flat, atol=1e-6)
    # gradient() then a forward: the pending dW is computed first
    with nn.GradientTape() as tape:
        loss = nn.losses.MeanSquaredError()(y, m1(x, training=True))
    g = tape.gradient(loss, m1.trainable_variables)
    lz = [t for t in g if isinstance(t, T._LazyGrad)]
    assert lz and lz[0]._lz.pending
    m1(x)
    assert not lz[0]._lz.pending and float(torch.linalg.vector_norm(lz[0])) > 0


def test_tape_fused_head_matches_unfused_tail():
    """Under a tape, MSE on the CNN-B1 tail runs the fused head (nn/tape.py _HeadPred): same loss,
    predictions and gradients as the unfused tail + loss + loss-gradient path (bf16 rounding aside)."""
    from pyspark_tf_gke_amd.nn import tape as T

    torch.manual_seed(0)
    x = torch.rand(4, 32, 40, 3)
    y = torch.rand(4, 2)
    m = build_cnn_model((32, 40, 3), flat=True, summary=False, device="cpu")
    res = {}
    saved = T.TAPE_HEAD
    try:
        for head in (True, False):
            T.TAPE_HEAD = head
            with nn.GradientTape() as tape:
                p = m(x, training=True)
                loss = nn.losses.MeanSquaredError()(y, p)
            if head:
                assert isinstance(p, T._HeadPred) and p._lz.state == "fused"
            g = tape.gradient(loss, m.trainable_variables)
            res[head] = ([t.float().clone() for t in g], float(loss), p.float().clone())
    finally:
        T.TAPE_HEAD = saved
    assert abs(res[True][1] - res[False][1]) <= 1e-4 * abs(res[False][1])
    assert torch.allclose(res[True][2], res[False][2], atol=1e-4)
    for a, b in zip(res[True][0], res[False][0]):
        assert float((a - b).abs().max()) <= 1e-2 * max(float(b.abs().max()), 1e-3)


def test_tape_head_pred_read_first_runs_plain_tail():
    """A prediction read before the loss (a metric on it) runs the plain tail; the loss then takes
    the ordinary path and the training matches the unfused run."""
    from pyspark_tf_gke_amd.nn import tape as T

    torch.manual_seed(2)
    x = torch.rand(4, 32, 40, 3)
    y = torch.rand(4, 2)
    m1 = build_cnn_model((32, 40, 3), flat=True, summary=False, device="cpu")
    m2 = build_cnn_model((32, 40, 3), flat=True, summary=False, device="cpu")
    m2.set_weights(m1.get_weights())
    o1, o2 = nn.optimizers.Adam(1e-3), nn.optimizers.Adam(1e-3)
    mae = nn.metrics.MeanAbsoluteError()
    for m, o in ((m1, o1), (m2, o2)):
        saved = T.TAPE_HEAD
        T.TAPE_HEAD = m is m1
        try:
            with nn.GradientTape() as tape:
                p = m(x, training=True)
                mae.update_state(y, p)
                loss = nn.losses.MeanSquaredError()(y, p)
            if m is m1:
                assert p._lz.state == "plain"
            g = tape.gradient(loss, m.trainable_variables)
            o.apply_gradients(zip(g, m.trainable_variables))
        finally:
            T.TAPE_HEAD = saved
    assert torch.equal(m1.store.flat, m2.store.flat)


def test_ps_one_worker_tape_lazy_path_matches_plain_loop():
    """The reference's primary loop with one worker (ParameterServerStrategy + ClusterCoordinator
    scheduling the GradientTape closure) on the CNN-B1 shape: the deferred Dense dW, the fused
    head and the round commit (ps.py _apply_local -> tape._apply_overlapped) train exactly like
    a plain tape loop."""
    from pyspark_tf_gke_amd import distribute as ds
    from pyspark_tf_gke_amd.cli.train import make_parameter_server_strategy
    from pyspark_tf_gke_amd.nn import tape as T

    torch.manual_seed(4)
    xs = [torch.rand(4, 32, 40, 3) for _ in range(2)]
    ys = [torch.rand(4, 2) for _ in range(2)]
    m0 = build_cnn_model((32, 40, 3), flat=True, summary=False, device="cpu")
    init = m0.get_weights()
    o0 = nn.optimizers.Adam(1e-3)
    for i in range(4):
        _tape_step(m0, o0, xs[i % 2], ys[i % 2])
    strategy = make_parameter_server_strategy(1, 1)
    with strategy.scope():
        m1 = build_cnn_model((32, 40, 3), flat=True, summary=False, device="cpu")
        o1 = nn.optimizers.Adam(1e-3)
        lo = nn.losses.MeanSquaredError()
    m1.set_weights(init)
    coord = ds.ClusterCoordinator(strategy)
    seen = []

    def step_fn(i):
        with nn.GradientTape() as tape:
            p = m1(xs[i % 2], training=True)
            lv = lo(ys[i % 2], p)
        g = tape.gradient(lv, m1.trainable_variables)
        seen.append(any(isinstance(t, T._LazyGrad) for t in g))
        o1.apply_gradients(zip(g, m1.trainable_variables))
        return lv

    for i in range(4):
        coord.schedule(lambda i=i: strategy.run(step_fn, args=(i,)))
    coord.join()
    assert all(seen) and o1.iterations == 4
    assert torch.allclose(m0.store.flat, m1.store.flat, atol=1e-6)


# ---------------------------------------------------------------------------------------------
# GradientTape.gradient(target, sources): the reference's step_fn (train_tf_ps.py:616-631,
# :738-753) with `loss += tf.add_n(model.losses) if model.losses else 0.0`, scaled targets, sums
# of recorded losses and subsets of the variables, against torch autograd.
# ---------------------------------------------------------------------------------------------
def _mlp_autograd(m, X, y, coef):
    """d(coef * SCCE(y, softmax(mlp(X)))) / d(params) by torch autograd from the engine's weights."""
    ps = [p for l in m.layers for p in l.params]
    ts = [p.data.detach().clone().requires_grad_(True) for p in ps]
    h = torch.as_tensor(X)
    for i in range(0, len(ts), 2):
        h = h @ ts[i].t() + ts[i + 1]
        if i + 2 < len(ts):
            h = torch.relu(h)
    loss = torch.nn.functional.cross_entropy(h, torch.as_tensor(y).long()) * coef
    loss.backward()
    return {id(p): t.grad for p, t in zip(ps, ts)}


def test_tape_reference_step_fn_scaled_target_matches_autograd():
    rng = np.random.default_rng(3)
    X = rng.normal(size=(32, 3)).astype(np.float32)
    y = rng.integers(0, 5, 32).astype(np.int32)
    m = build_deep_model(3, 5, device="cpu")
    loss_obj = nn.losses.SparseCategoricalCrossentropy()
    ref = _mlp_autograd(m, X, y, 2.5)
    with nn.GradientTape() as tape:
        logits = m(X, training=True)
        loss = loss_obj(y, logits)
        # Add possible regularization losses (the reference's exact line)
        loss += nn.add_n(m.losses) if m.losses else 0.0
        loss = 2.5 * loss
    vs = m.trainable_variables
    grads = tape.gradient(loss, vs)
    for g, v in zip(grads, vs):
        assert torch.allclose(g, ref[id(v.param)], rtol=1e-4, atol=1e-6), v.name
    # the loss value follows the arithmetic
    with nn.GradientTape() as tape:
        plain = loss_obj(y, m(X, training=True))
    assert abs(float(loss) - 2.5 * float(plain)) < 1e-5


def test_tape_sources_subset_in_caller_order_and_partial_update():
    rng = np.random.default_rng(4)
    X = rng.normal(size=(32, 3)).astype(np.float32)
    y = rng.integers(0, 5, 32).astype(np.int32)
    m = build_deep_model(3, 5, device="cpu")
    ref = _mlp_autograd(m, X, y, 1.0)
    vs = m.trainable_variables
    sub = [vs[5], vs[0], vs[3]]
    before = [v.param.data.clone() for v in vs]
    opt = nn.optimizers.Adam(1e-2)
    with nn.GradientTape() as tape:
        loss = nn.losses.SparseCategoricalCrossentropy()(y, m(X, training=True))
    grads = tape.gradient(loss, sub)
    assert len(grads) == 3
    for g, v in zip(grads, sub):
        assert tuple(g.shape) == tuple(v.param.shape)
        assert torch.allclose(g, ref[id(v.param)], rtol=1e-4, atol=1e-6), v.name
    single = None
    with nn.GradientTape() as tape:
        loss = nn.losses.SparseCategoricalCrossentropy()(y, m(X, training=True))
    single = tape.gradient(loss, vs[2])
    assert torch.allclose(single, ref[id(vs[2].param)], rtol=1e-4, atol=1e-6)
    with nn.GradientTape() as tape:
        loss = nn.losses.SparseCategoricalCrossentropy()(y, m(X, training=True))
    grads = tape.gradient(loss, sub)
    opt.apply_gradients(zip(grads, sub))
    moved = {id(v.param) for v in sub}
    for v, b in zip(vs, before):
        changed = not torch.equal(v.param.data, b)
        assert changed == (id(v.param) in moved), v.name
    assert opt.iterations == 1


def test_tape_replaced_gradients_are_applied():
    """Gradients the caller rescales before apply_gradients are the ones the update uses."""
    rng = np.random.default_rng(5)
    X = rng.normal(size=(32, 3)).astype(np.float32)
    y = rng.integers(0, 5, 32).astype(np.int32)
    m1 = build_deep_model(3, 5, device="cpu")
    m2 = build_deep_model(3, 5, device="cpu")
    m2.set_weights(m1.get_weights())
    o1, o2 = nn.optimizers.SGD(0.1), nn.optimizers.SGD(0.1)
    lo = nn.losses.SparseCategoricalCrossentropy()
    with nn.GradientTape() as tape:
        l1 = lo(y, m1(X, training=True))
    g1 = [g * 0.5 for g in tape.gradient(l1, m1.trainable_variables)]
    o1.apply_gradients(zip(g1, m1.trainable_variables))
    with nn.GradientTape() as tape:
        l2 = lo(y, m2(X, training=True)) * 0.5
    o2.apply_gradients(zip(tape.gradient(l2, m2.trainable_variables), m2.trainable_variables))
    assert torch.allclose(m1.store.flat, m2.store.flat, atol=1e-6)


def test_tape_untracked_target_raises():
    rng = np.random.default_rng(6)
    X = rng.normal(size=(16, 3)).astype(np.float32)
    y = rng.integers(0, 5, 16).astype(np.int32)
    m = build_deep_model(3, 5, device="cpu")
    lo = nn.losses.SparseCategoricalCrossentropy()
    with nn.GradientTape() as tape:
        loss = lo(y, m(X, training=True))
    with pytest.raises(ValueError):
        tape.gradient(loss * loss, m.trainable_variables)  # not linear
    with pytest.raises(ValueError):
        tape.gradient(torch.tensor(1.0), m.trainable_variables)  # not a recorded loss
    with pytest.raises(ValueError):
        tape.gradient(torch.sqrt(loss), m.trainable_variables)
    alias = loss
    loss.clamp_(max=1e9)  # in place: every reference to this loss leaves the linear family
    with pytest.raises(ValueError):
        tape.gradient(alias + 1, m.trainable_variables)  # was a TypeError
    with nn.GradientTape() as other:
        l2 = lo(y, m(X, training=True))
    with pytest.raises(ValueError):
        tape.gradient(l2, m.trainable_variables)  # another tape's loss
    m2 = build_deep_model(3, 5, device="cpu")
    with pytest.raises(ValueError):
        other.gradient(l2, m2.trainable_variables)  # a variable of another model


def test_tape_sum_of_losses_on_fused_head_matches_scaled_single():
    """CNN-B1-shaped model (fused MSE head on the tape): loss_a + 0.5 * loss_b on the same prediction
    (the head's fused gradients are redone through the plain tail) equals 1.5 * loss_a, and
    0.25 * loss (scaled fused head) equals loss with a quarter of the gradient."""
    from pyspark_tf_gke_amd.nn import tape as T

    torch.manual_seed(2)
    x = torch.rand(4, 32, 40, 3)
    y = torch.rand(4, 2) * 10
    m = build_cnn_model((32, 40, 3), flat=True, summary=False, device="cpu")
    mse = nn.losses.MeanSquaredError()
    saved = T.LAZY_DW
    T.LAZY_DW = False  # plain gradient tensors to compare
    try:
        def grads(fn):
            with nn.GradientTape() as tape:
                pred = m(x, training=True)
                tgt = fn(pred)
            return [g.clone() for g in tape.gradient(tgt, m.trainable_variables)]

        g_sum = grads(lambda p: mse(y, p) + 0.5 * mse(y, p))
        g_15 = grads(lambda p: 1.5 * mse(y, p))
        g_1 = grads(lambda p: mse(y, p))
        g_q = grads(lambda p: mse(y, p) * 0.25)
    finally:
        T.LAZY_DW = saved
    def rel(a, b):
        return float(torch.linalg.vector_norm(a - b) / (torch.linalg.vector_norm(b) + 1e-12))

    # the plain tail and the fused head round dZ / activations to bf16 at different points: compare at
    # that precision; a power-of-two scale of the fused head is exact
    for a, b, c, q in zip(g_sum, g_15, g_1, g_q):
        assert rel(a, 1.5 * c) < 2e-2
        assert rel(b, 1.5 * c) < 1e-2
        assert rel(q, 0.25 * c) < 1e-5


def test_tape_mwms_one_worker_trains_big_dense_like_fit():
    """under a one-worker MultiWorkerMirroredStrategy the big Dense kernel's gradient must
    not be deferred (its update reads the flat buffer): the tape loop equals train_on_batch."""
    from pyspark_tf_gke_amd import distribute as ds

    torch.manual_seed(0)
    x = torch.rand(4, 32, 40, 3)
    y = torch.rand(4, 2)
    st = ds.MultiWorkerMirroredStrategy()
    with st.scope():
        m1 = build_cnn_model((32, 40, 3), flat=True, summary=False, device="cpu")
        opt = nn.optimizers.Adam(1e-3)
    m2 = build_cnn_model((32, 40, 3), flat=True, summary=False, device="cpu")
    m2.set_weights(m1.get_weights())
    m2.compile(optimizer=nn.optimizers.Adam(1e-3), loss="mse")
    big = next(l for l in m1.layers if isinstance(l, nn.Dense) and l.units == 2048)
    w0 = big.kernel.data.clone()
    from pyspark_tf_gke_amd.nn import tape as T

    saved = T.TAPE_HEAD
    T.TAPE_HEAD = False  # train_on_batch's unfused CPU tail: the same roundings
    try:
        for _ in range(2):
            with st.scope():
                _tape_step(m1, opt, x, y)
            m2.train_on_batch(x, y)
    finally:
        T.TAPE_HEAD = saved
    assert not torch.equal(big.kernel.data, w0), "the big Dense kernel never trained"
    # (MWMS re-lays the flat store out in buckets: compare per variable)
    for a, b in zip(m1.get_weights(), m2.get_weights()):
        assert np.allclose(a, b, atol=1e-5)


def test_tape_abandoned_head_prediction_does_not_leak():
    """a tape forward whose prediction is abandoned (a closure that fails between the
    forward and the loss) leaves split-K sums behind; the next forward must not add onto them."""
    from pyspark_tf_gke_amd.nn import tape as T

    torch.manual_seed(3)
    x = torch.rand(4, 32, 40, 3)
    y = torch.rand(4, 2)
    m1 = build_cnn_model((32, 40, 3), flat=True, summary=False, device="cpu")
    m2 = build_cnn_model((32, 40, 3), flat=True, summary=False, device="cpu")
    m2.set_weights(m1.get_weights())
    with nn.GradientTape():
        p = m1(x, training=True)
    assert isinstance(p, T._HeadPred) and p._lz.state == "pending"  # the sums are held, never consumed
    mse = nn.losses.MeanSquaredError()
    with nn.GradientTape():
        l1 = mse(y, m1(x, training=True))
    with nn.GradientTape():
        l2 = mse(y, m2(x, training=True))
    assert abs(float(l1) - float(l2)) <= 1e-6 * max(1.0, abs(float(l2)))


def test_sparse_pool_record_dgrad_cpu_fallback_matches_dense():
    """ops.nn.conv2d_dgrad_halo_sparse off the GPU: the data gradient of the expanded sparse pool
    record equals the dense data gradient (the reference the GPU kernel is tested against)."""
    from pyspark_tf_gke_amd.ops import nn as K
    from pyspark_tf_gke_amd.ops import reference as R

    torch.manual_seed(3)
    N, H, W, Co, Ci = 2, 8, 12, 16, 8
    dzs = torch.randn(N, H // 2, W // 2, Co).bfloat16()
    arg = torch.randint(0, 4, (N, H // 2, W // 2, Co), dtype=torch.uint8)
    w = (torch.randn(Co, 5, 5, Ci) * 0.1).bfloat16()
    out = torch.empty(N, H, W, Ci)
    K.conv2d_dgrad_halo_sparse(dzs, arg, w, 2, out, None)
    ref = torch.empty(N, H, W, Ci)
    R.conv2d_dgrad(R.expand_pool_record(dzs, arg, (N, H, W, Co)), w, 2, ref)
    assert torch.allclose(out, ref, atol=1e-5)
    # the record keeps exactly one value per window and channel
    dense = R.expand_pool_record(dzs, arg, (N, H, W, Co))
    win = dense.reshape(N, H // 2, 2, W // 2, 2, Co)
    assert int((win != 0).sum(dim=(2, 4)).max()) <= 1
