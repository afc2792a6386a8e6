"""Protobuf wire encoding of the ``saved_model.pb`` subset a SavedModel directory needs to be
inspected by TensorFlow tooling (``saved_model_cli show``: tags and the ``serving_default``
signature), written without TensorFlow or its generated proto classes.

The field numbers follow TensorFlow's public schemas (tensorflow/core/protobuf/saved_model.proto,
meta_graph.proto, tensor_shape.proto, types.proto, versions.proto):

    SavedModel      1: saved_model_schema_version (int64)   2: meta_graphs (MetaGraphDef, repeated)
    MetaGraphDef    1: meta_info_def   2: graph_def   5: signature_def (map<string, SignatureDef>)
    MetaInfoDef     1: meta_graph_version   4: tags (repeated string)   5: tensorflow_version
                    6: tensorflow_git_version   7: stripped_default_attrs (bool)
    GraphDef        4: versions (VersionDef: 1 producer, 2 min_consumer)
    SignatureDef    1: inputs / 2: outputs (map<string, TensorInfo>)   3: method_name
    TensorInfo      1: name   2: dtype (DataType enum; DT_FLOAT = 1)   3: tensor_shape
    TensorShapeProto 2: dim (Dim: 1 size int64, -1 = unknown)

The graph itself is not a TF GraphDef (the model is executed by the MI355X kernels from the
Keras-config JSON next to it), so ``tf.saved_model.load`` of this directory is not expected to work:
format parity of the graph body stays unpinned (no TensorFlow is importable here).  What the file
does pin is the signature contract: input/output names, dtypes and shapes, which :func:`read` decodes
back and ``nn.saved_model.load`` checks against the JSON graph.
"""
from __future__ import annotations

DT_FLOAT = 1
PREDICT_METHOD = "tensorflow/serving/predict"


# ---------------------------------------------------------------------------------------------- encode
def _varint(n: int) -> bytes:
    if n < 0:
        n += 1 << 64  # int64 two's complement, 10 bytes on the wire
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field: int, wt: int) -> bytes:
    return _varint(field << 3 | wt)


def _int(field: int, v: int) -> bytes:
    return _key(field, 0) + _varint(int(v))


def _bytes(field: int, b: bytes | str) -> bytes:
    if isinstance(b, str):
        b = b.encode()
    return _key(field, 2) + _varint(len(b)) + b


def _map_entry(field: int, k: str, v: bytes) -> bytes:
    return _bytes(field, _bytes(1, k) + _bytes(2, v))


def tensor_info(name: str, shape, dtype: int = DT_FLOAT) -> bytes:
    dims = b"".join(_bytes(2, _int(1, -1 if d is None else int(d))) for d in shape)
    return _bytes(1, name) + _int(2, dtype) + _bytes(3, dims)


def signature_def(inputs: dict, outputs: dict, method: str = PREDICT_METHOD) -> bytes:
    """``inputs``/``outputs``: key -> (tensor name, shape list with None for unknown dims)."""
    body = b"".join(_map_entry(1, k, tensor_info(n, s)) for k, (n, s) in inputs.items())
    body += b"".join(_map_entry(2, k, tensor_info(n, s)) for k, (n, s) in outputs.items())
    return body + _bytes(3, method)


def saved_model(signatures: dict, tags=("serve",), version: str = "pyspark_tf_gke_amd",
                producer: int = 1) -> bytes:
    """Serialized ``SavedModel`` with one MetaGraphDef carrying ``tags`` and ``signatures``
    (name -> SignatureDef bytes from :func:`signature_def`)."""
    info = _bytes(1, "") + b"".join(_bytes(4, t) for t in tags) + _bytes(5, version) + _bytes(6, version)
    info += _int(7, 1)
    graph = _bytes(4, _int(1, producer) + _int(2, 0))
    mg = _bytes(1, info) + _bytes(2, graph) + b"".join(_map_entry(5, k, v) for k, v in signatures.items())
    return _int(1, 1) + _bytes(2, mg)


# ---------------------------------------------------------------------------------------------- decode
def _read_varint(b: bytes, i: int) -> tuple[int, int]:
    n = shift = 0
    while True:
        c = b[i]
        i += 1
        n |= (c & 0x7F) << shift
        if not c & 0x80:
            return n, i
        shift += 7


def _fields(b: bytes) -> dict:
    """field number -> list of values (int for varints, bytes for length-delimited)."""
    out: dict = {}
    i = 0
    while i < len(b):
        k, i = _read_varint(b, i)
        f, wt = k >> 3, k & 7
        if wt == 0:
            v, i = _read_varint(b, i)
        elif wt == 2:
            n, i = _read_varint(b, i)
            v, i = b[i:i + n], i + n
        elif wt == 1:
            v, i = b[i:i + 8], i + 8
        elif wt == 5:
            v, i = b[i:i + 4], i + 4
        else:
            raise ValueError(f"unsupported wire type {wt} in saved_model.pb")
        out.setdefault(f, []).append(v)
    return out


def _s64(v: int) -> int:
    return v - (1 << 64) if v >= 1 << 63 else v


def _tensor_info(b: bytes) -> dict:
    f = _fields(b)
    dims = [_s64(_fields(d).get(1, [0])[0]) for d in _fields(f.get(3, [b""])[0]).get(2, [])]
    return {"name": f.get(1, [b""])[0].decode(), "dtype": f.get(2, [0])[0],
            "shape": [None if d < 0 else d for d in dims]}


def _map(entries: list, conv) -> dict:
    out = {}
    for e in entries:
        f = _fields(e)
        out[f[1][0].decode()] = conv(f.get(2, [b""])[0])
    return out


def read(data: bytes) -> dict:
    """Decode what :func:`saved_model` writes: schema version, tags and signatures."""
    top = _fields(data)
    mgs = []
    for mg in top.get(2, []):
        f = _fields(mg)
        info = _fields(f.get(1, [b""])[0])
        sigs = _map(f.get(5, []), lambda s: (lambda g: {
            "inputs": _map(g.get(1, []), _tensor_info), "outputs": _map(g.get(2, []), _tensor_info),
            "method_name": g.get(3, [b""])[0].decode()})(_fields(s)))
        mgs.append({"tags": [t.decode() for t in info.get(4, [])],
                    "tensorflow_version": info.get(5, [b""])[0].decode(), "signature_def": sigs})
    return {"saved_model_schema_version": top.get(1, [0])[0], "meta_graphs": mgs}
