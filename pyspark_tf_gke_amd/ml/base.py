"""Params / Estimator / Transformer / Model base classes and Spark-ML-style persistence.

Saved layout mirrors Spark ML's (spark_workload_to_cloud_k8s.py:149-154, k_means.py:120-136):
``<path>/metadata/part-00000`` (one JSON line: class, timestamp, sparkVersion, uid, paramMap,
defaultParamMap) and ``<path>/data/part-00000-<uuid>.snappy.parquet`` for model data, with pipeline
stages under ``<path>/stages/<idx>_<uid>/``.  Parquet is written with pyarrow (format only).
"""
from __future__ import annotations

import importlib
import json
import os
import shutil
import time
import uuid

from ..parallel import comm

SPARK_VERSION = "3.5.0-ptg"


class Params:
    _defaults: dict = {}

    def __init__(self, **kw):
        self.uid = f"{type(self).__name__}_{uuid.uuid4().hex[:12]}"
        self._params = dict(self._defaults)
        for k, v in kw.items():
            if v is not None:
                self._set(k, v)

    def _set(self, k, v):
        if k not in self._defaults:
            raise TypeError(f"{type(self).__name__} has no param {k!r}")
        self._params[k] = v
        return self

    def getOrDefault(self, k):  # noqa: N802
        return self._params.get(k, self._defaults.get(k))

    def __getattr__(self, item):
        # setX / getX accessors like pyspark (setK, setSeed, setMaxIter, getK, ...)
        if item.startswith(("set", "get")) and len(item) > 3:
            key = item[3].lower() + item[4:]
            cands = [k for k in self._defaults if k.lower() == key.lower()]
            if cands:
                k = cands[0]
                if item.startswith("set"):
                    return lambda v: self._set(k, v)
                return lambda: self.getOrDefault(k)
        raise AttributeError(item)

    def params_dict(self) -> dict:
        return {k: v for k, v in self._params.items() if v != self._defaults.get(k)}

    def explainParams(self) -> str:  # noqa: N802
        return "\n".join(f"{k}: {self.getOrDefault(k)!r} (default {v!r})" for k, v in self._defaults.items())

    def copy(self, extra=None):
        c = type(self).__new__(type(self))
        c.__dict__.update(self.__dict__)
        c._params = dict(self._params)
        for k, v in (extra or {}).items():
            c._params[k] = v
        return c


class Transformer(Params):
    def transform(self, dataset, params=None):
        return (self.copy(params) if params else self)._transform(dataset)

    def _transform(self, dataset):
        raise NotImplementedError


class Estimator(Params):
    def fit(self, dataset, params=None):
        return (self.copy(params) if params else self)._fit(dataset)

    def _fit(self, dataset):
        raise NotImplementedError


class Model(Transformer):
    pass


# ------------------------------------------------------------------------------------------------
# persistence
# ------------------------------------------------------------------------------------------------
def _class_path(obj) -> str:
    return f"{type(obj).__module__}.{type(obj).__name__}"


def write_metadata(obj, path: str, extra: dict | None = None) -> None:
    os.makedirs(os.path.join(path, "metadata"), exist_ok=True)
    meta = {"class": _class_path(obj), "timestamp": int(time.time() * 1000), "sparkVersion": SPARK_VERSION,
            "uid": obj.uid, "paramMap": _jsonable(obj.params_dict()), "defaultParamMap": _jsonable(obj._defaults)}
    if extra:
        meta.update(extra)
    with open(os.path.join(path, "metadata", "part-00000"), "w") as fh:
        fh.write(json.dumps(meta) + "\n")
    open(os.path.join(path, "metadata", "_SUCCESS"), "w").close()


def read_metadata(path: str) -> dict:
    with open(os.path.join(path, "metadata", "part-00000")) as fh:
        return json.loads(fh.readline())


def write_data(path: str, columns: dict) -> None:
    import pyarrow as pa
    import pyarrow.parquet as pq

    d = os.path.join(path, "data")
    os.makedirs(d, exist_ok=True)
    pq.write_table(pa.table(columns), os.path.join(d, f"part-00000-{uuid.uuid4().hex[:12]}.snappy.parquet"),
                   compression="snappy")
    open(os.path.join(d, "_SUCCESS"), "w").close()


def read_data(path: str) -> dict:
    import glob

    import pyarrow.parquet as pq

    files = sorted(glob.glob(os.path.join(path, "data", "*.parquet")))
    t = pq.read_table(files[0])
    return {n: t.column(n).to_pylist() for n in t.column_names}


def _jsonable(d):
    out = {}
    for k, v in d.items():
        if isinstance(v, tuple):
            v = list(v)
        out[k] = v
    return out


class MLWritable:
    def save(self, path: str) -> None:
        self.write().save(path)

    def write(self):
        return _Writer(self)


class _Writer:
    def __init__(self, obj):
        self.obj = obj
        self._overwrite = False

    def overwrite(self):
        self._overwrite = True
        return self

    def save(self, path: str) -> None:
        if comm.rank() == 0:
            if os.path.exists(path):
                if not self._overwrite:
                    raise FileExistsError(f"Path {path} already exists. Use write().overwrite().save(path).")
                shutil.rmtree(path)
            self.obj._save_impl(path)
        comm.barrier()


def load_any(path: str):
    meta = read_metadata(path)
    mod, cls = meta["class"].rsplit(".", 1)
    return getattr(importlib.import_module(mod), cls)._load_impl(path, meta)


class MLReadable:
    @classmethod
    def load(cls, path: str):
        return load_any(path)

    @classmethod
    def read(cls):
        class _R:
            @staticmethod
            def load(path):
                return load_any(path)

        return _R()
