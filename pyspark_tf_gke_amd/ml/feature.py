"""Feature transformers used by the KMeans workloads (k_means.py:33-68,
spark_workload_to_cloud_k8s.py:78-101): StringIndexer, OneHotEncoder, VectorAssembler.

* StringIndexer.fit: label counts = a device histogram of the dictionary codes, summed across
  ranks with one all-reduce; order = frequencyDesc with alphabetical tie-break (Spark 3 default).
  transform: a device gather through a code -> index lookup table.
* OneHotEncoder: (dropLast=True) category size from the indexer's label count (+1 for the
  ``handleInvalid="keep"`` bucket); its output column records (codes, size) and is materialised by
  the fused assembler kernel, so the 5x-repeated one-hot of k_means.py:56-64 never exists as
  separate [n, 31] matrices.
* VectorAssembler: one fused HIP kernel writes the [n, D] fp32 feature matrix from one-hot
  segments (with repeats) and numeric columns; general vector inputs are concatenated.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..ops import df as D
from ..parallel import comm
from ..sql import types as T
from ..sql.dataframe import DataFrame
from ..sql.table import ColumnVector, Table
from .base import Estimator, MLReadable, MLWritable, Model, Transformer, read_data, write_data, write_metadata


def _all_reduce_counts(counts: torch.Tensor) -> torch.Tensor:
    if not comm.distributed():
        return counts
    return comm.all_reduce_tensor_(counts.clone())


class StringIndexer(Estimator, MLWritable, MLReadable):
    _defaults = {"inputCol": None, "outputCol": None, "handleInvalid": "error", "stringOrderType": "frequencyDesc",
                 "inputCols": None, "outputCols": None}

    def __init__(self, inputCol=None, outputCol=None, handleInvalid="error", stringOrderType="frequencyDesc",  # noqa: N803
                 inputCols=None, outputCols=None):  # noqa: N803
        super().__init__(inputCol=inputCol, outputCol=outputCol, handleInvalid=handleInvalid,
                         stringOrderType=stringOrderType, inputCols=inputCols, outputCols=outputCols)

    def _fit(self, df: DataFrame):
        cv = df._t.column(self.getOrDefault("inputCol"))
        if not isinstance(cv.dtype, T.StringType):
            # numeric input: index the string form of the values (Spark casts to string)
            vals = [None if v is None else str(v) for v in cv.to_pylist()]
            from ..sql.table import column_from_python

            cv = column_from_python(vals, T.StringType(), cv.device)
        # ranks hold their own dictionaries: unify them (tensor control plane) before codes are
        # counted and the per-code histogram is all-reduced
        from ..sql.readwriter import unify_dictionary

        cv = unify_dictionary(cv)
        nd = len(cv.dictionary or [])
        counts = _all_reduce_counts(D.histogram(cv.data, nd).cpu())[:nd].numpy()
        labels = list(cv.dictionary or [])
        order = self.getOrDefault("stringOrderType")
        present = [i for i in range(nd) if counts[i] > 0]
        if order == "frequencyDesc":
            present.sort(key=lambda i: (-counts[i], labels[i]))
        elif order == "frequencyAsc":
            present.sort(key=lambda i: (counts[i], labels[i]))
        elif order == "alphabetDesc":
            present.sort(key=lambda i: labels[i], reverse=True)
        else:
            present.sort(key=lambda i: labels[i])
        m = StringIndexerModel(labels=[labels[i] for i in present])
        m._params.update(self._params)
        return m

    def _save_impl(self, path):
        write_metadata(self, path)

    @classmethod
    def _load_impl(cls, path, meta):
        o = cls()
        o._params.update(meta["paramMap"])
        o.uid = meta["uid"]
        return o


class StringIndexerModel(Model, MLWritable, MLReadable):
    _defaults = StringIndexer._defaults

    def __init__(self, labels=None, **kw):
        super().__init__(**kw)
        self.labels = list(labels or [])
        self.labelsArray = [self.labels]

    def _transform(self, df: DataFrame) -> DataFrame:
        t = df._t
        inc, outc = self.getOrDefault("inputCol"), self.getOrDefault("outputCol")
        cv = t.column(inc)
        if not isinstance(cv.dtype, T.StringType):
            from ..sql.table import column_from_python

            cv = column_from_python([None if v is None else str(v) for v in cv.to_pylist()], T.StringType(), cv.device)
        idx = {s: i for i, s in enumerate(self.labels)}
        nl = len(self.labels)
        hi = self.getOrDefault("handleInvalid")
        # lookup table: dictionary code -> label index; unseen -> nl (keep) / -1 (skip/error)
        unseen = float(nl) if hi == "keep" else -1.0
        lut = [float(idx[s]) if s in idx else unseen for s in (cv.dictionary or [])]
        lut_t = torch.tensor(lut + [unseen], dtype=torch.float64, device=cv.device)
        codes = cv.data.long()
        codes = torch.where(codes < 0, torch.full_like(codes, len(lut)), codes)
        out = D.gather_rows(lut_t, codes)
        if hi != "keep":
            bad = out < 0
            if hi == "error" and bool(bad.any()):
                raise RuntimeError(f"StringIndexer: unseen label or null in column {inc} (handleInvalid='error')")
            if hi == "skip":
                keep = D.compact((~bad).to(torch.uint8))
                t = t.take(keep)
                out = out[keep] if out.device.type == "cpu" else D.gather_rows(out, keep)
        res = ColumnVector(out, T.DoubleType())
        res.ml_attr = {"type": "nominal", "num_vals": nl + (1 if hi == "keep" else 0), "labels": self.labels}
        return df._new(t.with_column(outc, res))

    def _save_impl(self, path):
        write_metadata(self, path)
        import pyarrow as pa

        write_data(path, {"labelsArray": pa.array([[self.labels]])})

    @classmethod
    def _load_impl(cls, path, meta):
        data = read_data(path)
        o = cls(labels=data["labelsArray"][0][0])
        o._params.update(meta["paramMap"])
        o.uid = meta["uid"]
        return o


class OneHotEncoder(Estimator, MLWritable, MLReadable):
    _defaults = {"inputCol": None, "outputCol": None, "dropLast": True, "handleInvalid": "error",
                 "inputCols": None, "outputCols": None}

    def __init__(self, inputCol=None, outputCol=None, dropLast=True, handleInvalid="error", inputCols=None,  # noqa: N803
                 outputCols=None):  # noqa: N803
        super().__init__(inputCol=inputCol, outputCol=outputCol, dropLast=dropLast, handleInvalid=handleInvalid,
                         inputCols=inputCols, outputCols=outputCols)

    def _fit(self, df: DataFrame):
        cv = df._t.column(self.getOrDefault("inputCol"))
        attr = getattr(cv, "ml_attr", None)
        if attr is not None:
            size = attr["num_vals"]
        else:
            _, c, _, mx, _ = D.reduce_stats(cv.data, cv.valid_u8())
            mx = comm.all_reduce_float([mx], op=torch.distributed.ReduceOp.MAX)[0]
            size = int(mx) + 1 if c else 0
        m = OneHotEncoderModel(categorySizes=[size])
        m._params.update(self._params)
        return m

    def _save_impl(self, path):
        write_metadata(self, path)

    @classmethod
    def _load_impl(cls, path, meta):
        o = cls()
        o._params.update(meta["paramMap"])
        o.uid = meta["uid"]
        return o


class OneHotEncoderModel(Model, MLWritable, MLReadable):
    _defaults = OneHotEncoder._defaults

    def __init__(self, categorySizes=None, **kw):  # noqa: N803
        super().__init__(**kw)
        self.categorySizes = list(categorySizes or [])

    @property
    def vector_size(self) -> int:
        n = self.categorySizes[0]
        return n - 1 if self.getOrDefault("dropLast") else n

    def _transform(self, df: DataFrame) -> DataFrame:
        t = df._t
        cv = t.column(self.getOrDefault("inputCol"))
        V = self.vector_size
        codes = cv.data.to(torch.int32) if cv.data.dtype != torch.int32 else cv.data
        if cv.valid is not None:
            codes = torch.where(cv.valid.bool(), codes, torch.full_like(codes, -1))
        # codes >= V (the dropped last category / keep bucket) encode to the zero vector
        dense = D.assemble_features([("onehot", codes.contiguous(), 0, V, 1)], t.num_rows, V, t.device)
        out = ColumnVector(dense, T.VectorUDT())
        out.onehot = (codes.contiguous(), V)
        return df._new(t.with_column(self.getOrDefault("outputCol"), out))

    def _save_impl(self, path):
        write_metadata(self, path)
        write_data(path, {"categorySizes": [self.categorySizes]})

    @classmethod
    def _load_impl(cls, path, meta):
        data = read_data(path)
        o = cls(categorySizes=data["categorySizes"][0])
        o._params.update(meta["paramMap"])
        o.uid = meta["uid"]
        return o


class VectorAssembler(Transformer, MLWritable, MLReadable):
    _defaults = {"inputCols": None, "outputCol": None, "handleInvalid": "error"}

    def __init__(self, inputCols=None, outputCol=None, handleInvalid="error"):  # noqa: N803
        super().__init__(inputCols=inputCols, outputCol=outputCol, handleInvalid=handleInvalid)

    def _transform(self, df: DataFrame) -> DataFrame:
        t = df._t
        n = t.num_rows
        segs, blocks = [], []
        off = 0
        hi = self.getOrDefault("handleInvalid")
        bad = torch.zeros(n, dtype=torch.bool, device=t.device)
        names = list(self.getOrDefault("inputCols"))
        i = 0
        while i < len(names):
            cv = t.column(names[i])
            oh = getattr(cv, "onehot", None)
            if oh is not None:
                R = 1
                while i + R < len(names) and names[i + R] == names[i]:
                    R += 1
                segs.append(("onehot", oh[0], off, oh[1], R))
                off += oh[1] * R
                i += R
                continue
            if isinstance(cv.dtype, T.VectorUDT):
                blocks.append((off, cv.data))
                off += cv.data.shape[1]
            else:
                x = cv.data
                nulls = cv.null_mask()
                if x.dtype in (torch.float32, torch.float64):
                    nulls = nulls | torch.isnan(x)
                bad = bad | nulls
                if x.dtype == torch.float32:
                    segs.append(("f32", torch.where(cv.valid_bool(), x, torch.full_like(x, math.nan)).contiguous(), off, 0, 0))
                else:
                    xd = x.double()
                    segs.append(("f64", torch.where(cv.valid_bool(), xd, torch.full_like(xd, math.nan)).contiguous(),
                                 off, 0, 0))
                off += 1
            i += 1
        Dm = off
        out = None
        for s0 in range(0, len(segs), 8):
            part = D.assemble_features(segs[s0:s0 + 8], n, Dm, t.device)
            out = part if out is None else out + part  # disjoint segments (zeros elsewhere)
        if out is None:
            out = torch.zeros((n, Dm), dtype=torch.float32, device=t.device)
        for boff, blk in blocks:
            out[:, boff:boff + blk.shape[1]] = blk.float()
        if hi == "error" and bool(bad.any()):
            raise RuntimeError("VectorAssembler: null/NaN input value (handleInvalid='error')")
        if hi == "skip":
            keep = D.compact((~bad).to(torch.uint8))
            t = t.take(keep)
            out = D.gather_rows(out, keep)
        return df._new(t.with_column(self.getOrDefault("outputCol"), ColumnVector(out, T.VectorUDT())))

    def _save_impl(self, path):
        write_metadata(self, path)

    @classmethod
    def _load_impl(cls, path, meta):
        o = cls()
        o._params.update(meta["paramMap"])
        o.uid = meta["uid"]
        return o


_ = Table
