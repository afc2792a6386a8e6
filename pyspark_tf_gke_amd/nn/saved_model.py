"""``tf.saved_model``-shaped export / load (BASELINE.json names SavedModel as an output format; the
reference itself only writes ``.keras`` files, train_tf_ps.py:675-676, :810-811).

Layout written by :func:`save` (mirrors a TF SavedModel directory)::

    <dir>/saved_model.pb                SavedModel proto: tags + serving_default SignatureDef (nn/tf_proto.py)
    <dir>/saved_model.json              graph (Keras layer configs + connectivity) and signatures
    <dir>/fingerprint.json              content hash of graph + variables
    <dir>/variables/variables.safetensors   every variable in Keras layout, keyed <layer>/<i>
    <dir>/variables/variables.index.json    name -> shape / dtype
    <dir>/assets/                           extra files (e.g. label_map.json)

``saved_model.pb`` is a real protobuf ``SavedModel`` (wire-encoded by ``nn/tf_proto.py`` with TF's field
numbers) holding the ``serve`` tag set and the ``serving_default`` signature, so TF tooling can read the
serving contract.  What is NOT reproduced: the GraphDef body and the TensorBundle
``variables.index``/``data`` shards — TensorFlow and its proto schemas are not available here, so the
graph is stored as the same Keras-config JSON the ``.keras`` zip uses and the tensors as safetensors.  :func:`load` restores a model whose ``signatures["serving_default"]`` runs inference on
the MI355X kernels, like ``tf.saved_model.load(...).signatures["serving_default"]``.
"""
from __future__ import annotations

import hashlib
import json
import os
import shutil

import numpy as np


class _Signature:
    def __init__(self, model, input_name: str, output_name: str):
        self.model = model
        self.input_name, self.output_name = input_name, output_name
        self.structured_input_signature = {input_name: {"shape": [None, *model.input_shape], "dtype": "float32"}}
        self.structured_outputs = {output_name: {"shape": [None, *model.output_shape], "dtype": "float32"}}

    def __call__(self, *args, **kwargs):
        x = kwargs.get(self.input_name, args[0] if args else None)
        return {self.output_name: self.model.predict(np.asarray(x) if not hasattr(x, "device") else x)}


class LoadedModel:
    """Result of :func:`load`: callable like the Keras model, with ``signatures``."""

    def __init__(self, model, meta: dict):
        self.model = model
        sig = meta["signatures"]["serving_default"]
        self.signatures = {"serving_default": _Signature(model, sig["inputs"][0], sig["outputs"][0])}
        self.meta = meta

    def __call__(self, x, training=False):
        return self.model(x, training=training)


def save(model, export_dir: str, signatures=None, assets: dict | None = None) -> str:
    """Export ``model`` (Sequential or functional) to ``export_dir``; returns the directory."""
    from safetensors.numpy import save_file

    st = model._strategy() if hasattr(model, "_strategy") else None
    if st is not None and not st.is_chief:
        return export_dir
    if hasattr(model, "_check_master"):
        model._check_master()
    tmp = export_dir.rstrip("/") + ".tmp"
    shutil.rmtree(tmp, ignore_errors=True)
    os.makedirs(os.path.join(tmp, "variables"))
    os.makedirs(os.path.join(tmp, "assets"))
    tensors, index = {}, {}
    for l in model.layers:
        for i, w in enumerate(l.keras_weights()):
            key = f"{l.name}/{i}"
            tensors[key] = np.ascontiguousarray(np.asarray(w, dtype=np.float32))
            index[key] = {"shape": list(tensors[key].shape), "dtype": "float32"}
    save_file(tensors, os.path.join(tmp, "variables", "variables.safetensors"))
    with open(os.path.join(tmp, "variables", "variables.index.json"), "w") as fh:
        json.dump(index, fh, indent=1)
    in_name = "input_layer"
    out_name = "output_0"
    graph = {"class_name": model._save_class_name(), "config": model.get_config(),
             "input_shape": list(model.input_shape), "output_shape": list(model.output_shape)}
    meta = {"saved_model_schema_version": 1, "format": "pyspark_tf_gke_amd.saved_model (TF SavedModel layout; "
            "JSON graph + safetensors variables)", "graph": graph,
            "signatures": {"serving_default": {"inputs": [in_name], "outputs": [out_name],
                                               "input_shape": [None, *model.input_shape],
                                               "output_shape": [None, *model.output_shape]}}}
    from . import tf_proto

    sig = tf_proto.signature_def({in_name: (f"serving_default_{in_name}:0", [None, *model.input_shape])},
                                 {out_name: ("StatefulPartitionedCall:0", [None, *model.output_shape])})
    with open(os.path.join(tmp, "saved_model.pb"), "wb") as fh:
        fh.write(tf_proto.saved_model({"serving_default": sig}))
    body = json.dumps(meta, sort_keys=True).encode()
    with open(os.path.join(tmp, "saved_model.json"), "wb") as fh:
        fh.write(json.dumps(meta, indent=1).encode())
    h = hashlib.sha256(body)
    for k in sorted(tensors):
        h.update(k.encode())
        h.update(tensors[k].tobytes())
    with open(os.path.join(tmp, "fingerprint.json"), "w") as fh:
        json.dump({"saved_model_checksum": h.hexdigest(), "num_variables": len(tensors)}, fh)
    for name, content in (assets or {}).items():
        with open(os.path.join(tmp, "assets", name), "w") as fh:
            fh.write(content if isinstance(content, str) else json.dumps(content))
    shutil.rmtree(export_dir, ignore_errors=True)
    os.replace(tmp, export_dir)
    return export_dir


def load(export_dir: str, device=None) -> LoadedModel:
    from safetensors.numpy import load_file

    from . import layers as L
    from .model import Sequential

    with open(os.path.join(export_dir, "saved_model.json")) as fh:
        meta = json.load(fh)
    pb = os.path.join(export_dir, "saved_model.pb")
    if os.path.exists(pb):  # the proto's serving contract must agree with the JSON graph
        from . import tf_proto

        with open(pb, "rb") as fh:
            proto = tf_proto.read(fh.read())
        sd = meta["signatures"]["serving_default"]
        got = proto["meta_graphs"][0]["signature_def"]["serving_default"]
        if (got["inputs"][sd["inputs"][0]]["shape"] != sd["input_shape"]
                or got["outputs"][sd["outputs"][0]]["shape"] != sd["output_shape"]):
            raise ValueError(f"{pb}: serving_default signature disagrees with saved_model.json")
        meta["saved_model_pb"] = proto
    g = meta["graph"]
    if g["class_name"] == "Functional":
        from .functional import model_from_config

        m = model_from_config(g["config"])
    else:
        L.reset_name_counters()
        m = Sequential(name=g["config"].get("name", "sequential"))
        for lc in g["config"]["layers"]:
            m.add(L.layer_from_config(lc["class_name"], lc["config"]))
    m.build(device=device)
    tensors = load_file(os.path.join(export_dir, "variables", "variables.safetensors"))
    for l in m.layers:
        ws, i = [], 0
        while f"{l.name}/{i}" in tensors:
            ws.append(tensors[f"{l.name}/{i}"])
            i += 1
        if ws:
            l.set_keras_weights(ws)
    m.store.refresh_bf16()
    return LoadedModel(m, meta)
