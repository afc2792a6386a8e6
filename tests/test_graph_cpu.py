"""Functional-graph engine (ResNet family) on the CPU host path vs an fp32 torch-autograd oracle."""
import os

import numpy as np
import pytest
import torch

from graph_oracle import oracle_grads
from pyspark_tf_gke_amd import nn
from pyspark_tf_gke_amd.models.resnet import RESNET50_PARAMS, RESNET50_TRAINABLE, ResNet, ResNet50


def _engine_grads(m, x, y):
    stats = m._stats_buf()
    stats.zero_()
    m.store.zero_grad()
    xb, yb = m._prep_batch(x, y)
    out = m._run_forward(xb, True)
    dpred = m._loss_grad(out, yb, stats)
    m._run_backward(dpred)
    return m._logs_from(stats)["loss"], {p.name: p.grad.detach().float().clone() for p in m.store.params}


def _rel(a, b):
    return float((a - b).norm() / max(b.norm(), 1e-6))


def test_resnet50_param_count_matches_keras():
    m = ResNet50(device="cpu")
    assert m.count_params() == RESNET50_PARAMS
    assert m.store.num_params() == RESNET50_TRAINABLE
    names = [l.name for l in m.layers]
    assert "conv2_block1_0_conv" in names and "conv5_block3_out" in names and names[-1] == "predictions"
    # every Conv2D+BN(+Add)(+ReLU) unit is one fused op; stem pool + GAP + Dense are the others
    assert len(m.ops) == 53 + 3


@pytest.fixture
def fp32_host():
    from pyspark_tf_gke_amd.nn import engine

    old = engine.host_fp32()
    engine.host_fp32(True)
    yield
    engine.host_fp32(old)


@pytest.mark.parametrize("blocks", [(1, 1), (2, 1)])
def test_resnet_small_grads_match_autograd(blocks, fp32_host):
    """Engine plumbing + BN/pool/residual math, exact up to fp32 rounding (host fp32 mode)."""
    torch.manual_seed(0)
    m = ResNet(blocks, input_shape=(32, 32, 3), classes=10, width=8, device="cpu")
    m.compile(optimizer=nn.optimizers.SGD(0.0), loss="sparse_categorical_crossentropy", metrics=["accuracy"])
    x = torch.rand(4, 32, 32, 3)
    y = torch.randint(0, 10, (4,))
    loss, g = _engine_grads(m, x, y)
    ref_loss, ref = oracle_grads(m, x, y)
    assert abs(loss - ref_loss) < 1e-4 * max(1.0, abs(ref_loss))
    for name, rg in ref.items():
        if name.endswith("_conv/bias") and "predictions" not in name:
            # conv bias before a training-mode BN: analytically zero gradient (the engine skips it)
            assert float(rg.abs().max()) < 1e-4
            continue
        eg = g[name].reshape(rg.shape)
        assert _rel(eg, rg) < 1e-3, (name, _rel(eg, rg))


def test_resnet_small_bf16_close_to_autograd():
    """The real (bf16-activation) host path: same directions, bf16-level deviations."""
    torch.manual_seed(0)
    m = ResNet((1, 1), input_shape=(32, 32, 3), classes=10, width=8, device="cpu")
    m.compile(optimizer=nn.optimizers.SGD(0.0), loss="sparse_categorical_crossentropy")
    x = torch.rand(16, 32, 32, 3)
    y = torch.randint(0, 10, (16,))
    loss, g = _engine_grads(m, x, y)
    ref_loss, ref = oracle_grads(m, x, y)
    assert abs(loss - ref_loss) < 2e-2 * max(1.0, abs(ref_loss))
    for name, rg in ref.items():
        if name.endswith("kernel"):
            eg = g[name].reshape(rg.shape).flatten()
            cos = float(torch.dot(eg, rg.flatten()) / (eg.norm() * rg.norm()))
            assert cos > 0.9, (name, cos)


def test_resnet_train_loss_decreases_and_saves(tmp_path):
    torch.manual_seed(0)
    m = ResNet((1, 1), input_shape=(32, 32, 3), classes=4, width=8, device="cpu")
    m.compile(optimizer=nn.optimizers.Adam(1e-2), loss="sparse_categorical_crossentropy", metrics=["accuracy"])
    x = torch.rand(8, 32, 32, 3)
    y = torch.randint(0, 4, (8,))
    first = m.train_on_batch(x, y, return_dict=True)["loss"]
    for _ in range(15):
        last = m.train_on_batch(x, y, return_dict=True)["loss"]
    assert last < first
    # moving statistics moved away from their (0, 1) init
    bn = [l for l in m.layers if isinstance(l, nn.BatchNormalization)][0]
    assert float(bn.moving_mean.abs().sum()) > 0
    p_train = m.predict(x.numpy(), batch_size=8)
    path = str(tmp_path / "model.keras")
    m.save(path)
    m2 = nn.load_model(path, device="cpu")
    assert m2.count_params() == m.count_params()
    p_load = m2.predict(x.numpy(), batch_size=8)
    np.testing.assert_allclose(p_load, p_train, atol=2e-2)


def test_functional_mlp_and_sgd():
    inp = nn.Input((3,))
    h = nn.Dense(16, activation="relu")(inp)
    h = nn.Dense(8, activation="relu")(h)
    out = nn.Dense(3, activation="softmax")(h)
    m = nn.Model(inp, out)
    m.build(device="cpu")
    m.compile(optimizer=nn.optimizers.SGD(0.1, momentum=0.9, nesterov=True), loss="sparse_categorical_crossentropy",
              metrics=["accuracy"])
    rng = np.random.default_rng(0)
    x = rng.normal(size=(64, 3)).astype(np.float32)
    y = (x[:, 0] > 0).astype(np.int32) + (x[:, 1] > 0)
    h0 = m.fit(x, y, batch_size=16, epochs=1, verbose=0).history["loss"][0]
    h1 = m.fit(x, y, batch_size=16, epochs=10, verbose=0).history["loss"][-1]
    assert h1 < h0


def test_saved_model_export_load(tmp_path):
    from pyspark_tf_gke_amd.models import build_cnn_model

    torch.manual_seed(0)
    for m, x in ((ResNet((1, 1), input_shape=(32, 32, 3), classes=4, width=8, device="cpu"),
                  np.random.rand(3, 32, 32, 3).astype(np.float32)),
                 (build_cnn_model((32, 40, 3), flat=True, summary=False, device="cpu"),
                  np.random.rand(3, 32, 40, 3).astype(np.float32))):
        d = str(tmp_path / m.name)
        m.export(d, assets={"label_map.json": {"0": "a"}})
        for f in ("saved_model.pb", "saved_model.json", "fingerprint.json", "variables/variables.safetensors",
                  "variables/variables.index.json", "assets/label_map.json"):
            assert os.path.exists(os.path.join(d, f)), f
        loaded = nn.saved_model.load(d, device="cpu")
        out = loaded.signatures["serving_default"](input_layer=x)["output_0"]
        np.testing.assert_allclose(out, m.predict(x), atol=1e-2)
        sig = loaded.meta["saved_model_pb"]["meta_graphs"][0]["signature_def"]["serving_default"]
        assert sig["inputs"]["input_layer"]["shape"] == [None, *x.shape[1:]]


def _tf_saved_model_classes():
    """SavedModel / MetaGraphDef / SignatureDef / TensorInfo message classes built by google.protobuf
    from a descriptor with TensorFlow's field numbers (saved_model.proto, meta_graph.proto,
    tensor_shape.proto): an encoder-independent parser for saved_model.pb."""
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

    F = descriptor_pb2.FieldDescriptorProto
    fd = descriptor_pb2.FileDescriptorProto(name="ptg_tf_subset.proto", package="tfsub", syntax="proto3")

    def msg(name, fields, nested=()):
        m = fd.message_type.add(name=name)
        for n in nested:
            m.nested_type.add().CopyFrom(n)
        for num, fname, ftype, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=ftype, label=label)
            if tname:
                f.type_name = tname
        return m

    def entry(name, vtype):
        e = descriptor_pb2.DescriptorProto(name=name)
        e.options.map_entry = True
        e.field.add(name="key", number=1, type=F.TYPE_STRING, label=F.LABEL_OPTIONAL)
        e.field.add(name="value", number=2, type=F.TYPE_MESSAGE, label=F.LABEL_OPTIONAL, type_name=vtype)
        return e

    O, R = F.LABEL_OPTIONAL, F.LABEL_REPEATED
    dim = descriptor_pb2.DescriptorProto(name="Dim")
    dim.field.add(name="size", number=1, type=F.TYPE_INT64, label=O)
    msg("TensorShapeProto", [(2, "dim", F.TYPE_MESSAGE, R, ".tfsub.TensorShapeProto.Dim")], [dim])
    msg("TensorInfo", [(1, "name", F.TYPE_STRING, O, None), (2, "dtype", F.TYPE_INT32, O, None),
                       (3, "tensor_shape", F.TYPE_MESSAGE, O, ".tfsub.TensorShapeProto")])
    msg("SignatureDef", [(1, "inputs", F.TYPE_MESSAGE, R, ".tfsub.SignatureDef.InputsEntry"),
                         (2, "outputs", F.TYPE_MESSAGE, R, ".tfsub.SignatureDef.OutputsEntry"),
                         (3, "method_name", F.TYPE_STRING, O, None)],
        [entry("InputsEntry", ".tfsub.TensorInfo"), entry("OutputsEntry", ".tfsub.TensorInfo")])
    msg("MetaInfoDef", [(1, "meta_graph_version", F.TYPE_STRING, O, None), (4, "tags", F.TYPE_STRING, R, None),
                        (5, "tensorflow_version", F.TYPE_STRING, O, None)])
    msg("MetaGraphDef", [(1, "meta_info_def", F.TYPE_MESSAGE, O, ".tfsub.MetaInfoDef"),
                         (5, "signature_def", F.TYPE_MESSAGE, R, ".tfsub.MetaGraphDef.SignatureDefEntry")],
        [entry("SignatureDefEntry", ".tfsub.SignatureDef")])
    msg("SavedModel", [(1, "saved_model_schema_version", F.TYPE_INT64, O, None),
                       (2, "meta_graphs", F.TYPE_MESSAGE, R, ".tfsub.MetaGraphDef")])
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    return message_factory.GetMessageClass(pool.FindMessageTypeByName("tfsub.SavedModel"))


def test_saved_model_pb_parses_with_protobuf(tmp_path):
    from pyspark_tf_gke_amd.models import build_cnn_model

    m = build_cnn_model((32, 40, 3), flat=True, summary=False, device="cpu")
    d = str(tmp_path / "sm")
    m.export(d)
    SavedModel = _tf_saved_model_classes()
    sm = SavedModel()
    with open(os.path.join(d, "saved_model.pb"), "rb") as fh:
        sm.ParseFromString(fh.read())
    assert sm.saved_model_schema_version == 1 and len(sm.meta_graphs) == 1
    mg = sm.meta_graphs[0]
    assert list(mg.meta_info_def.tags) == ["serve"]
    sig = mg.signature_def["serving_default"]
    assert sig.method_name == "tensorflow/serving/predict"
    ti = sig.inputs["input_layer"]
    assert ti.dtype == 1 and ti.name == "serving_default_input_layer:0"
    assert [d.size for d in ti.tensor_shape.dim] == [-1, 32, 40, 3]
    assert [d.size for d in sig.outputs["output_0"].tensor_shape.dim] == [-1, 2]


def test_native_libraries_link_completely():
    """dlopen both HIP kernel libraries with immediate binding (no GPU needed): an unresolved
    symbol (e.g. a kernel whose host stub was dropped) fails here on the CPU box, not at round end."""
    import ctypes
    import os

    from pyspark_tf_gke_amd import _native

    _native.ensure_built()
    here = os.path.dirname(_native.__file__)
    for name in ("libptg_hip.so", "libptg_hip_checked.so"):
        path = os.path.join(here, name)
        if os.path.exists(path):
            ctypes.CDLL(path, mode=os.RTLD_NOW | os.RTLD_GLOBAL)
