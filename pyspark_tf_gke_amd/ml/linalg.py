"""``pyspark.ml.linalg`` vectors (host-side views of rows of a device feature matrix)."""
from __future__ import annotations

import numpy as np


class DenseVector:
    def __init__(self, values):
        self.array = np.asarray(values, dtype=np.float64).reshape(-1)

    def toArray(self):  # noqa: N802
        return self.array

    @property
    def size(self):
        return self.array.size

    def __len__(self):
        return self.array.size

    def __getitem__(self, i):
        return self.array[i]

    def __iter__(self):
        return iter(self.array)

    def __eq__(self, other):
        return np.array_equal(self.array, np.asarray(getattr(other, "array", other)))

    def dot(self, other):
        return float(self.array @ np.asarray(getattr(other, "array", other)))

    def squared_distance(self, other):
        d = self.array - np.asarray(getattr(other, "array", other))
        return float(d @ d)

    def __repr__(self):
        return "DenseVector([" + ", ".join(f"{x:.4g}" for x in self.array) + "])"

    __str__ = lambda self: "[" + ",".join(repr(float(x)) for x in self.array) + "]"  # noqa: E731


class SparseVector:
    def __init__(self, size, indices, values=None):
        if isinstance(indices, dict):
            items = sorted(indices.items())
            indices, values = [i for i, _ in items], [v for _, v in items]
        self.size = int(size)
        self.indices = np.asarray(indices, dtype=np.int32)
        self.values = np.asarray(values, dtype=np.float64)

    def toArray(self):  # noqa: N802
        a = np.zeros(self.size)
        a[self.indices] = self.values
        return a

    def __len__(self):
        return self.size

    def __repr__(self):
        return f"SparseVector({self.size}, {dict(zip(self.indices.tolist(), self.values.tolist()))})"


class Vectors:
    @staticmethod
    def dense(*values):
        if len(values) == 1 and hasattr(values[0], "__len__"):
            values = values[0]
        return DenseVector(values)

    @staticmethod
    def sparse(size, *args):
        return SparseVector(size, *args)

    @staticmethod
    def squared_distance(a, b):
        return DenseVector(getattr(a, "toArray", lambda: a)()).squared_distance(getattr(b, "toArray", lambda: b)())
