"""Minimal RDD API on the host executor (local[N]): what a classic PySpark wordcount uses
(textFile / flatMap / map / reduceByKey / collect).  Partitions are Python lists processed by a
thread pool of ``spark.default.parallelism`` workers; ``reduceByKey`` hash-shuffles into that
many partitions.  ``word_count_native`` is the fused native path (csrc/host word counter).
"""
from __future__ import annotations

import concurrent.futures as cf
import ctypes
import itertools

from .. import _native


class RDD:
    def __init__(self, sc, partitions_fn, nparts):
        self.ctx = sc
        self._fn = partitions_fn  # () -> list of lists
        self._n = nparts

    @staticmethod
    def from_list(sc, data, n):
        n = max(1, n)
        parts = [data[len(data) * i // n: len(data) * (i + 1) // n] for i in range(n)]
        return RDD(sc, lambda: parts, n)

    @staticmethod
    def from_rows(sc, rows):
        return RDD.from_list(sc, rows, sc.defaultParallelism)

    @staticmethod
    def text_file(sc, path, n):
        def load():
            with open(path, "r", encoding="utf-8", errors="replace") as fh:
                lines = fh.read().splitlines()
            return [lines[len(lines) * i // n: len(lines) * (i + 1) // n] for i in range(n)]

        r = RDD(sc, load, n)
        r._path = path
        return r

    def _pool_map(self, f):
        parts = self._fn()
        with cf.ThreadPoolExecutor(max(1, min(len(parts), self._n))) as ex:
            return list(ex.map(f, parts))

    def mapPartitions(self, f):  # noqa: N802
        src = self
        return RDD(self.ctx, lambda: src._pool_map(lambda p: list(f(iter(p)))), self._n)

    def map(self, f):
        return self.mapPartitions(lambda it: (f(x) for x in it))

    def flatMap(self, f):  # noqa: N802
        return self.mapPartitions(lambda it: (y for x in it for y in f(x)))

    def filter(self, f):
        return self.mapPartitions(lambda it: (x for x in it if f(x)))

    def mapValues(self, f):  # noqa: N802
        return self.map(lambda kv: (kv[0], f(kv[1])))

    def reduceByKey(self, f, numPartitions=None):  # noqa: N802, N803
        n = numPartitions or self._n
        src = self

        def run():
            def combine(p):
                d = {}
                for k, v in p:
                    d[k] = f(d[k], v) if k in d else v
                return d

            partials = src._pool_map(combine)
            buckets = [dict() for _ in range(n)]
            for d in partials:
                for k, v in d.items():
                    b = buckets[hash(k) % n]
                    b[k] = f(b[k], v) if k in b else v
            return [list(b.items()) for b in buckets]

        return RDD(self.ctx, run, n)

    def groupByKey(self):  # noqa: N802
        src = self

        def run():
            d = {}
            for p in src._fn_all():
                for k, v in p:
                    d.setdefault(k, []).append(v)
            items = list(d.items())
            return [items[len(items) * i // src._n: len(items) * (i + 1) // src._n] for i in range(src._n)]

        return RDD(self.ctx, run, self._n)

    def _fn_all(self):
        return self._fn()

    def sortBy(self, keyfunc, ascending=True):  # noqa: N802
        items = sorted(self.collect(), key=keyfunc, reverse=not ascending)
        return RDD.from_list(self.ctx, items, self._n)

    def collect(self):
        return list(itertools.chain.from_iterable(self._fn()))

    def count(self):
        return sum(len(p) for p in self._fn())

    def take(self, n):
        return self.collect()[:n]

    def first(self):
        return self.take(1)[0]

    def getNumPartitions(self):  # noqa: N802
        return self._n

    def foreach(self, f):
        for x in self.collect():
            f(x)

    def toDF(self, schema=None):  # noqa: N802
        from .session import SparkSession

        return SparkSession.getActiveSession().createDataFrame(self.collect(), schema)


def word_count_native(text: bytes, nthreads: int):
    """Fused native wordcount (split on whitespace, count, sort by count desc): [(word, count)]."""
    lib = _native.host_lib()
    buf = ctypes.create_string_buffer(text, len(text))
    nw, nb = ctypes.c_long(0), ctypes.c_long(0)
    lib.ptgh_word_count(buf, len(text), nthreads, None, 0, None, None, 0, ctypes.byref(nw), ctypes.byref(nb))
    out = ctypes.create_string_buffer(max(nb.value, 1))
    offs = (ctypes.c_long * (nw.value + 1))()
    cnts = (ctypes.c_longlong * max(nw.value, 1))()
    rc = lib.ptgh_word_count(buf, len(text), nthreads, out, nb.value, offs, cnts, nw.value, ctypes.byref(nw),
                             ctypes.byref(nb))
    if rc != 0:
        raise RuntimeError(f"word count failed ({rc})")
    raw = out.raw
    return [(raw[offs[i]:offs[i + 1]].decode("utf-8", "replace"), int(cnts[i])) for i in range(nw.value)]
