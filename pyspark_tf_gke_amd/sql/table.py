"""Columnar batches resident on the executor device.

A :class:`Table` is one partition of a DataFrame held by one rank (one executor = one GPU).
Columns are device tensors: numerics as-is, strings dictionary-encoded (int32 codes, -1 = null,
dictionary on the host), ML vectors as row-major [n, d] fp32.  Null masks are optional uint8
tensors (None = no nulls).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..ops import df as D
from . import types as T


class ColumnVector:
    def __init__(self, data: torch.Tensor, dtype: T.DataType, valid: torch.Tensor | None = None,
                 dictionary: list | None = None):
        self.data = data
        self.dtype = dtype
        self.valid = valid
        self.dictionary = dictionary
        self._dict_index = None

    def __len__(self):
        return int(self.data.shape[0])

    @property
    def device(self):
        return self.data.device

    def dict_index(self) -> dict:
        if self._dict_index is None:
            self._dict_index = {s: i for i, s in enumerate(self.dictionary or [])}
        return self._dict_index

    def valid_u8(self):
        if self.valid is None:
            return None
        return self.valid if self.valid.dtype == torch.uint8 else self.valid.to(torch.uint8)

    def valid_bool(self) -> torch.Tensor:
        if self.valid is None:
            return D.full(len(self), 1, torch.bool, self.device)
        if self.valid.dtype == torch.uint8 and self.valid.is_contiguous():
            return self.valid.view(torch.bool)  # (0 / 1 bytes: the same storage, no conversion kernel)
        return self.valid.bool()

    def null_mask(self) -> torch.Tensor:
        m = ~self.valid_bool()
        if isinstance(self.dtype, T.StringType):
            m = m | (self.data < 0)
        return m

    def take(self, idx: torch.Tensor) -> "ColumnVector":
        data = D.gather_rows(self.data, idx)
        valid = D.gather_rows(self.valid_u8(), idx) if self.valid is not None else None
        return ColumnVector(data, self.dtype, valid, self.dictionary)

    def to(self, device) -> "ColumnVector":
        return ColumnVector(self.data.to(device), self.dtype, None if self.valid is None else self.valid.to(device),
                            self.dictionary)

    def to_pylist(self) -> list:
        data = self.data.detach().cpu()
        valid = np.ones(len(self), dtype=bool) if self.valid is None else self.valid_bool().cpu().numpy()
        if isinstance(self.dtype, T.StringType):
            codes = data.numpy()
            d = self.dictionary or []
            return [d[c] if (v and c >= 0) else None for c, v in zip(codes, valid)]
        if isinstance(self.dtype, T.VectorUDT):
            from ..ml.linalg import DenseVector

            arr = data.numpy()
            return [DenseVector(arr[i]) for i in range(arr.shape[0])]
        arr = data.numpy()
        out = []
        if isinstance(self.dtype, T.BooleanType):
            return [bool(x) if v else None for x, v in zip(arr, valid)]
        if isinstance(self.dtype, T.TimestampType):
            return [T.micros_to_datetime(int(x)) if v else None for x, v in zip(arr, valid)]
        if isinstance(self.dtype, (T.IntegerType, T.LongType)):
            return [int(x) if v else None for x, v in zip(arr, valid)]
        for x, v in zip(arr, valid):
            out.append(float(x) if v else None)
        return out


def concat_columns(cvs: list) -> ColumnVector:
    base = cvs[0]
    if isinstance(base.dtype, T.StringType):
        # merge dictionaries
        merged, index = [], {}
        datas = []
        for cv in cvs:
            lut = []
            for s in cv.dictionary or []:
                if s not in index:
                    index[s] = len(merged)
                    merged.append(s)
                lut.append(index[s])
            lut_t = torch.tensor(lut + [-1], dtype=torch.int32, device=cv.device)
            codes = cv.data.long()
            codes = torch.where(codes < 0, torch.full_like(codes, len(lut)), codes)
            datas.append(lut_t[codes] if len(cv) else cv.data)
        data = torch.cat(datas)
        dictionary = merged
    else:
        data = torch.cat([cv.data for cv in cvs])
        dictionary = None
    if any(cv.valid is not None for cv in cvs):
        valid = torch.cat([cv.valid_u8() if cv.valid is not None else torch.ones(len(cv), dtype=torch.uint8,
                                                                                   device=cv.device) for cv in cvs])
    else:
        valid = None
    return ColumnVector(data, base.dtype, valid, dictionary)


class Table:
    def __init__(self, columns: dict, num_rows: int | None = None, device=None):
        self.columns = dict(columns)
        if num_rows is None:
            num_rows = len(next(iter(self.columns.values()))) if self.columns else 0
        self.num_rows = int(num_rows)
        self.device = torch.device(device) if device is not None else (
            next(iter(self.columns.values())).device if self.columns else torch.device("cpu"))

    @property
    def names(self):
        return list(self.columns)

    def column(self, name: str) -> ColumnVector:
        if name in self.columns:
            return self.columns[name]
        for k in self.columns:  # Spark column resolution is case-insensitive by default
            if k.lower() == name.lower():
                return self.columns[k]
        raise KeyError(f"Column '{name}' does not exist. Available: {', '.join(self.columns)}")

    def resolve(self, name: str) -> str:
        if name in self.columns:
            return name
        for k in self.columns:
            if k.lower() == name.lower():
                return k
        raise KeyError(f"Column '{name}' does not exist. Available: {', '.join(self.columns)}")

    def schema(self) -> T.StructType:
        return T.StructType([T.StructField(n, c.dtype, True) for n, c in self.columns.items()])

    def take(self, idx: torch.Tensor) -> "Table":
        return Table({n: c.take(idx) for n, c in self.columns.items()}, int(idx.numel()), self.device)

    def slice(self, start: int, stop: int) -> "Table":
        idx = D.arange(start, min(stop, self.num_rows), self.device)
        return self.take(idx)

    def with_column(self, name: str, cv: ColumnVector) -> "Table":
        cols = dict(self.columns)
        try:
            name = self.resolve(name)
        except KeyError:
            pass
        cols[name] = cv
        return Table(cols, self.num_rows, self.device)

    def select(self, names: list) -> "Table":
        return Table({self.resolve(n): self.column(n) for n in names}, self.num_rows, self.device)

    def to(self, device) -> "Table":
        return Table({n: c.to(device) for n, c in self.columns.items()}, self.num_rows, device)

    @staticmethod
    def concat(tables: list) -> "Table":
        tables = [t for t in tables if t is not None]
        if not tables:
            return Table({})
        if len(tables) == 1:
            return tables[0]
        names = tables[0].names
        return Table({n: concat_columns([t.column(n) for t in tables]) for n in names},
                     sum(t.num_rows for t in tables), tables[0].device)

    def rows(self, limit: int | None = None) -> list:
        t = self if limit is None or limit >= self.num_rows else self.slice(0, limit)
        cols = [t.column(n).to_pylist() for n in t.names]
        return list(zip(*cols)) if cols else [() for _ in range(t.num_rows)]


def column_from_python(values: list, dtype: T.DataType | None, device) -> ColumnVector:
    """Build a column from Python values (createDataFrame)."""
    if dtype is None:
        dtype = infer_python_type(values)
    n = len(values)
    valid = np.array([v is not None and not (isinstance(v, float) and math.isnan(v) and False) for v in values],
                     dtype=np.uint8)
    if isinstance(dtype, T.StringType):
        d, idx, codes = [], {}, np.empty(n, np.int32)
        for i, v in enumerate(values):
            if v is None:
                codes[i] = -1
                continue
            s = str(v)
            if s not in idx:
                idx[s] = len(d)
                d.append(s)
            codes[i] = idx[s]
        return ColumnVector(torch.from_numpy(codes).to(device), dtype, None, d)
    if isinstance(dtype, T.VectorUDT):
        arr = np.stack([np.asarray(getattr(v, "toArray", lambda: v)(), dtype=np.float32) for v in values])
        return ColumnVector(torch.from_numpy(arr).to(device), dtype)
    if isinstance(dtype, T.TimestampType):
        values = [T.to_micros(v) for v in values]
    npdt = {T.IntegerType: np.int32, T.LongType: np.int64, T.DoubleType: np.float64, T.FloatType: np.float32,
            T.BooleanType: np.bool_, T.TimestampType: np.int64}[type(dtype)]
    arr = np.array([(v if v is not None else 0) for v in values], dtype=npdt)
    v = torch.from_numpy(valid).to(device) if not valid.all() else None
    return ColumnVector(torch.from_numpy(arr).to(device), dtype, v)


def infer_python_type(values: list) -> T.DataType:
    t = None
    for v in values:
        if v is None:
            continue
        if isinstance(v, bool):
            c = T.BooleanType()
        elif isinstance(v, int):
            c = T.LongType()
        elif isinstance(v, float):
            c = T.DoubleType()
        elif isinstance(v, str):
            c = T.StringType()
        elif hasattr(v, "toArray") or isinstance(v, (list, np.ndarray)):
            c = T.VectorUDT()
        else:
            c = T.StringType()
        if t is None:
            t = c
        elif type(t) is not type(c):
            if isinstance(t, (T.LongType, T.DoubleType)) and isinstance(c, (T.LongType, T.DoubleType)):
                t = T.DoubleType()
            else:
                t = T.StringType()
    return t or T.StringType()
