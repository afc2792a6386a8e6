"""``pyspark.sql.functions`` surface used by the reference workloads (col, isnan, when, count, avg,
...; k_means.py:6-7, spark_workload_to_cloud_k8s.py:17) plus the usual aggregate and math
helpers, ``split``/``explode`` (wordcount) and ``rand`` (synthetic data)."""
from __future__ import annotations

import builtins

from .column import Column, _wrap, col, lit  # noqa: F401

column = col


def when(cond, value) -> Column:
    return Column(("when", [(_wrap(cond).node, _wrap(value).node)], None))


def isnan(c) -> Column:
    return Column(("un", "ISNAN", _c(c).node))


def isnull(c) -> Column:
    return Column(("un", "ISNULL", _c(c).node))


def _c(c) -> Column:
    return col(c) if isinstance(c, str) else c


def _un(op):
    return lambda c: Column(("un", op, _c(c).node))


abs = _un("ABS")  # noqa: A001
sqrt = _un("SQRT")
log = _un("LOG")
exp = _un("EXP")
floor = _un("FLOOR")
ceil = _un("CEIL")


def round(c, scale: int = 0) -> Column:  # noqa: A001
    if scale == 0:
        return Column(("un", "ROUND", _c(c).node))
    f = 10.0 ** scale
    return Column(("un", "ROUND", (_c(c) * f).node)) / f


def pow(a, b) -> Column:  # noqa: A001
    return _c(a)._bin("pow", b)


def coalesce(*cols) -> Column:
    out = _c(cols[0])
    for c in cols[1:]:
        out = Column(("bin", "coalesce", out.node, _c(c).node))
    return out


def least(*cols) -> Column:
    out = _c(cols[0])
    for c in cols[1:]:
        out = Column(("bin", "least", out.node, _c(c).node))
    return out


def greatest(*cols) -> Column:
    out = _c(cols[0])
    for c in cols[1:]:
        out = Column(("bin", "greatest", out.node, _c(c).node))
    return out


# ---------------------------------------------------------------- aggregates
def _agg(fn):
    def f(c=None):
        if c is None or (isinstance(c, str) and c == "*"):
            return Column(("agg", fn, None))
        return Column(("agg", fn, _c(c).node))

    f.__name__ = fn
    return f


count = _agg("count")
sum = _agg("sum")  # noqa: A001
avg = _agg("avg")
mean = _agg("avg")
min = _agg("min")  # noqa: A001
max = _agg("max")  # noqa: A001
countDistinct = _agg("count_distinct")  # noqa: N816
count_distinct = countDistinct
first = _agg("first")
stddev = _agg("stddev")


# ---------------------------------------------------------------- strings / generators
def split(c, pattern: str, limit: int = -1) -> Column:
    return Column(("split", pattern, _c(c).node))


def explode(c) -> Column:
    return Column(("explode", _c(c).node))


def lower(c) -> Column:
    return Column(("strmap", "lower", _c(c).node))


def upper(c) -> Column:
    return Column(("strmap", "upper", _c(c).node))


def trim(c) -> Column:
    return Column(("strmap", "trim", _c(c).node))


def length(c) -> Column:
    return Column(("strlen", _c(c).node))


def rand(seed: int | None = None) -> Column:
    return Column(("rand", seed))


def monotonically_increasing_id() -> Column:
    return Column(("rowid",))


def desc(c) -> Column:
    return _c(c).desc()


def asc(c) -> Column:
    return _c(c).asc()


_ = builtins
