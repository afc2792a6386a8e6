"""DataFrame, GroupedData and Row — the PySpark DataFrame surface of the reference workloads
(k_means.py, spark_workload_to_cloud_k8s.py, spark_installation_check.py, google_health_SQL.py).

Execution model: SPMD, one rank per GPU = one Spark executor.  Each rank holds its partition as a
device-resident :class:`~.table.Table`.  Narrow transformations (filter, withColumn) are lazy: they
accumulate into a pending stage that is optimised (predicate pushdown, filter fusion) and run as
one retried task when the table is first needed (sql/plan.py); everything else runs on the
partition with the HIP kernels (expression VM, compaction, hash aggregation) and keeps its result resident
(the reference re-reads its JDBC source on every action because nothing is cached, SURVEY §3.3;
here nothing needs re-reading).  Actions combine ranks with RCCL (count/agg all-reduce, groupBy
partial-aggregate -> hash shuffle -> final aggregate) and gather small results to the driver view
(every rank, like a Spark driver) for ``collect``/``show``.
"""
from __future__ import annotations

import math
import re

import numpy as np
import torch
import torch.distributed as dist

from .. import config
from ..ops import df as D
from ..parallel import comm
from . import column as C
from . import types as T
from .column import Column, col, expr_name
from .table import ColumnVector, Table, column_from_python


class Row(tuple):
    def __new__(cls, *args, **kwargs):
        if kwargs:
            r = tuple.__new__(cls, tuple(kwargs.values()))
            r.__fields__ = list(kwargs.keys())
            return r
        r = tuple.__new__(cls, args)
        r.__fields__ = None
        return r

    @classmethod
    def _make(cls, fields, values):
        r = tuple.__new__(cls, tuple(values))
        r.__fields__ = list(fields)
        return r

    def asDict(self):  # noqa: N802
        return dict(zip(self.__fields__ or [], self))

    def __getattr__(self, item):
        f = self.__dict__.get("__fields__") if "__fields__" in self.__dict__ else None
        if f and item in f:
            return self[f.index(item)]
        raise AttributeError(item)

    def __getitem__(self, k):
        if isinstance(k, str):
            return tuple.__getitem__(self, self.__fields__.index(k))
        return tuple.__getitem__(self, k)

    def __repr__(self):
        if self.__fields__:
            return "Row(" + ", ".join(f"{k}={v!r}" for k, v in zip(self.__fields__, self)) + ")"
        return "<Row(" + ", ".join(repr(v) for v in self) + ")>"


_VM_OUT = {T.BooleanType: D.CT_U8, T.IntegerType: D.CT_I32, T.LongType: D.CT_I64, T.DoubleType: D.CT_F64,
           T.FloatType: D.CT_F32}
_TORCH_OF = {T.BooleanType: torch.uint8, T.IntegerType: torch.int32, T.LongType: torch.int64,
             T.DoubleType: torch.float64, T.FloatType: torch.float32}


def _to_col(c) -> Column:
    return col(c) if isinstance(c, str) else c


class DataFrame:
    def __init__(self, table: Table, session, replicated: bool = False, pending: list | None = None):
        self._src = table
        self._pending = list(pending or [])
        self._mat = None if self._pending else table
        self.sparkSession = session
        self._num_partitions = session.default_parallelism if session is not None else 1

    @property
    def _t(self) -> Table:
        """The materialised partition; runs the pending narrow stage (sql/plan.py) on first use."""
        if self._mat is None:
            from . import plan as P

            self._mat = P.run_task(self._src, self._pending, self.sparkSession)
        return self._mat

    def _visible_names(self) -> list:
        """Column names after the pending stage, without running it."""
        if self._mat is not None:
            return list(self._mat.names)
        names = list(self._src.names)
        for o in self._pending:
            if o[0] == "with":
                if o[1].lower() not in {n.lower() for n in names}:
                    names.append(o[1])
            elif o[0] == "select":
                names = [n for n, _ in o[1]]
        return names

    def _lazy(self, op) -> "DataFrame":
        from . import plan as P

        names = {n.lower() for n in self._visible_names()}
        nodes = [op[1].node] if op[0] == "filter" else [c.node for _, c in op[1]] if op[0] == "select" else [op[2].node]
        missing = set().union(*[P.referenced_columns(nd) for nd in nodes]) - names
        if missing:
            raise KeyError(f"Column '{sorted(missing)[0]}' does not exist. Available: {', '.join(sorted(names))}")
        base = self if self._mat is None else None
        d = DataFrame(self._src if base is not None else self._mat, self.sparkSession,
                      pending=(self._pending if base is not None else []) + [op])
        d._num_partitions = self._num_partitions
        return d

    def explain(self, extended: bool = False) -> None:
        from . import plan as P

        if comm.rank() == 0:
            text = getattr(self, "_plan_text", None)  # an aggregation computed by a fused scan
            print(text if text and self._mat is not None else P.describe(self._pending if self._mat is None else []),
                  flush=True)

    # ------------------------------------------------------------------ schema
    @property
    def columns(self):
        return self._visible_names()

    @property
    def schema(self) -> T.StructType:
        return self._t.schema()

    @property
    def dtypes(self):
        return [(f.name, f.dataType.simple) for f in self.schema]

    def printSchema(self):  # noqa: N802
        if comm.rank() == 0:
            print(self.schema.treeString(), end="", flush=True)

    def __getitem__(self, item):
        if isinstance(item, str):
            return col(self._t.resolve(item))
        if isinstance(item, Column):
            return self.filter(item)
        if isinstance(item, (list, tuple)):
            return self.select(*item)
        raise TypeError(item)

    def __getattr__(self, item):
        if item.startswith("_"):
            raise AttributeError(item)
        try:
            return col(self._t.resolve(item))
        except KeyError:
            raise AttributeError(item) from None

    # ------------------------------------------------------------------ expression evaluation
    def _new(self, table: Table) -> "DataFrame":
        d = DataFrame(table, self.sparkSession)
        d._num_partitions = self._num_partitions
        return d

    def _eval(self, c: Column, name_hint=None) -> tuple:
        node = c.node
        name = name_hint or expr_name(node)
        base = C.strip_alias(node)
        t = self._t
        if base[0] == "col":
            return name, t.column(base[1])
        if base[0] in ("split", "explode", "agg"):
            raise TypeError(f"{base[0]} is only valid as a top-level select() expression / in agg()")
        if base[0] == "strmap":
            src = self._eval(Column(base[2]))[1]
            f = {"lower": str.lower, "upper": str.upper, "trim": str.strip}[base[1]]
            mapped = [f(s) for s in src.dictionary or []]
            return name, _remap_dictionary(src, mapped)
        if base[0] == "strlen":
            src = self._eval(Column(base[1]))[1]
            lens = torch.tensor([len(s) for s in (src.dictionary or [])] + [0], dtype=torch.int32, device=t.device)
            codes = src.data.long()
            codes = torch.where(codes < 0, torch.full_like(codes, len(src.dictionary or [])), codes)
            return name, ColumnVector(D.gather_rows(lens, codes), T.IntegerType(), src.valid_u8() if src.valid is not None else (src.data >= 0).to(torch.uint8))
        if base[0] == "rand":
            g = torch.Generator(device=t.device)
            g.manual_seed((base[1] or 0) * 1000003 + comm.rank())
            return name, ColumnVector(torch.rand(t.num_rows, generator=g, dtype=torch.float64, device=t.device),
                                      T.DoubleType())
        if base[0] == "rowid":
            off = comm.rank() << 33
            return name, ColumnVector(torch.arange(t.num_rows, dtype=torch.int64, device=t.device) + off, T.LongType())
        if base[0] == "lit" and isinstance(base[1], str):
            return name, ColumnVector(torch.zeros(t.num_rows, dtype=torch.int32, device=t.device), T.StringType(),
                                      None, [base[1]])
        if base[0] == "bin" and base[1] == "coalesce":
            a, b = self._eval(Column(base[2]))[1], self._eval(Column(base[3]))[1]
            if isinstance(a.dtype, T.StringType) and isinstance(b.dtype, T.StringType):
                return name, _coalesce_strings(a, b)
        # rand()/monotonically_increasing_id() nested inside an expression: materialise them as
        # temporary columns so the device expression VM only sees column/literal leaves
        node, t = self._materialize_leaves(node, t)
        dtype = C.infer_type(node, t)
        if isinstance(dtype, T.StringType):
            raise TypeError(f"string-valued expression {name} is not supported")
        n = t.num_rows
        if t.device.type == "cuda":
            ins, r, consts, cols = C.compile_vm(node, t)
            out = torch.empty(n, dtype=_TORCH_OF[type(dtype)], device=t.device)
            valid = torch.empty(n, dtype=torch.uint8, device=t.device)
            if n:
                prog = D.pack_vm_prog(ins, r, _VM_OUT[type(dtype)], 0, consts, cols)
                D.expr_eval(prog, n, out, valid)
            if isinstance(dtype, T.BooleanType):
                out = out.bool()
            return name, ColumnVector(out, dtype, valid)
        v, ok = C.eval_host(node, t)
        tdt = _TORCH_OF[type(dtype)]
        if tdt == torch.uint8:
            out = (v != 0) & ok
            out = out.bool()
        elif tdt in (torch.int32, torch.int64):
            out = torch.where(ok, v, torch.zeros_like(v)).to(tdt)
        else:
            out = torch.where(ok, v, torch.full_like(v, math.nan)).to(tdt)
        return name, ColumnVector(out, dtype, ok.to(torch.uint8))

    def _materialize_leaves(self, node, t):
        tmp = {}

        def walk(nd):
            if isinstance(nd, tuple) and nd and nd[0] in ("rand", "rowid"):
                key = f"__leaf{len(tmp)}"
                tmp[key] = self._eval(Column(nd))[1]
                return ("col", key)
            if isinstance(nd, tuple):
                return tuple(walk(x) if isinstance(x, tuple) else (
                    [tuple(walk(y) for y in pair) if isinstance(pair, tuple) else pair for pair in x]
                    if isinstance(x, list) else x) for x in nd)
            return nd

        new = walk(node)
        if not tmp:
            return node, t
        for k, cv in tmp.items():
            t = t.with_column(k, cv)
        return new, t

    def _mask(self, cond) -> torch.Tensor:
        t = self._t
        n = t.num_rows
        if isinstance(cond, str):
            cond = _parse_sql_predicate(cond)
        if t.device.type == "cuda":
            ins, r, consts, cols = C.compile_vm(cond.node, t)
            mask = torch.empty(n, dtype=torch.uint8, device=t.device)
            if n:
                D.expr_eval(D.pack_vm_prog(ins, r, D.CT_U8, 1, consts, cols), n, mask)
            return mask
        v, ok = C.eval_host(cond.node, t)
        return ((v != 0) & ok).to(torch.uint8)

    # ------------------------------------------------------------------ transformations
    def filter(self, condition) -> "DataFrame":
        if isinstance(condition, str):
            condition = _parse_sql_predicate(condition)
        return self._lazy(("filter", condition))

    where = filter

    def select(self, *cols) -> "DataFrame":
        if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
            cols = tuple(cols[0])
        if any(isinstance(c, str) and c == "*" for c in cols):
            cols = tuple(x for c in cols for x in ([col(n) for n in self.columns] if c == "*" else [c]))
        cs = [_to_col(c) for c in cols]
        for c in cs:
            base = C.strip_alias(c.node)
            if base[0] == "explode":
                if len(cs) != 1:
                    raise NotImplementedError("explode() must be the only select expression")
                name = c.node[1] if c.node[0] == "alias" else "col"
                return self._explode(base, name)
            if base[0] == "agg":
                return self.agg(*cs)
        if self._mat is None:
            from . import plan as P

            named = [(expr_name(c.node), c) for c in cs]
            if all(P._inlinable(c.node) for _, c in named):
                # projection of a pending stage: stays lazy (fused into the next task / aggregation)
                return self._lazy(("select", named))
        out = {}
        for c in cs:
            name, cv = self._eval(c)
            out[name] = cv
        return self._new(Table(out, self._t.num_rows, self._t.device))

    def selectExpr(self, *exprs):  # noqa: N802
        return self.select(*[col(e) for e in exprs])

    def withColumn(self, colName: str, c: Column) -> "DataFrame":  # noqa: N802, N803
        base = C.strip_alias(c.node)
        if base[0] in ("split", "explode", "agg", "strmap", "strlen") or (base[0] == "lit" and isinstance(base[1], str)) \
                or (base[0] == "bin" and base[1] == "coalesce") or base[0] == "col":
            _, cv = self._eval(c, colName)  # dictionary-string / pass-through columns: eager
            return self._new(self._t.with_column(colName, cv))
        return self._lazy(("with", colName, c))

    def withColumnRenamed(self, existing: str, new: str) -> "DataFrame":  # noqa: N802
        cols = {}
        for n, cv in self._t.columns.items():
            cols[new if n.lower() == existing.lower() else n] = cv
        return self._new(Table(cols, self._t.num_rows, self._t.device))

    def toDF(self, *names) -> "DataFrame":  # noqa: N802
        return self._new(Table(dict(zip(names, self._t.columns.values())), self._t.num_rows, self._t.device))

    def drop(self, *names) -> "DataFrame":
        drop = {(n if isinstance(n, str) else expr_name(n.node)).lower() for n in names}
        return self._new(Table({n: c for n, c in self._t.columns.items() if n.lower() not in drop},
                               self._t.num_rows, self._t.device))

    def limit(self, num: int) -> "DataFrame":
        # global limit: ranks keep rows in rank order until `num` rows are taken
        counts = comm.all_gather_int(self._t.num_rows)
        before = sum(counts[: comm.rank()])
        keep = max(0, min(self._t.num_rows, num - before))
        return self._new(self._t.slice(0, keep))

    def _explode(self, node, name) -> "DataFrame":
        inner = node[1]
        if inner[0] != "split":
            raise NotImplementedError("explode() supports split(col, pattern)")
        pattern, src_node = inner[1], inner[2]
        _, src = self._eval(Column(src_node))
        rx = re.compile(pattern)
        toks = [[w for w in rx.split(s)] for s in (src.dictionary or [])]
        words, widx = [], {}
        tok_codes = []
        for ts in toks:
            cs = []
            for w in ts:
                if w not in widx:
                    widx[w] = len(words)
                    words.append(w)
                cs.append(widx[w])
            tok_codes.append(cs)
        codes = src.data.cpu().numpy()
        valid = codes >= 0
        lens = np.array([len(x) for x in tok_codes] + [0], dtype=np.int64)
        safe = np.where(valid, codes, len(tok_codes))
        per_row = lens[safe]
        flat = np.array([c for x in tok_codes for c in x] + [0], dtype=np.int32)
        starts = np.concatenate([[0], np.cumsum(lens[:-1])])
        row_rep = np.repeat(np.arange(len(codes)), per_row)
        within = np.arange(per_row.sum()) - np.repeat(np.cumsum(per_row) - per_row, per_row)
        out_codes = flat[starts[safe[row_rep]] + within] if len(row_rep) else np.zeros(0, np.int32)
        cv = ColumnVector(torch.from_numpy(out_codes.astype(np.int32)).to(self._t.device), T.StringType(), None, words)
        return self._new(Table({name: cv}, len(out_codes), self._t.device))

    # ------------------------------------------------------------------ actions
    def count(self) -> int:
        return int(comm.all_reduce_int([self._t.num_rows])[0])

    def collect(self) -> list:
        names = self.columns
        t = _gather_table_all(self._t) if comm.distributed() else self._t
        return [Row._make(names, r) for r in t.rows()]

    def take(self, num: int) -> list:
        return self.limit(num).collect()

    def head(self, n: int | None = None):
        if n is None:
            rows = self.take(1)
            return rows[0] if rows else None
        return self.take(n)

    def first(self):
        return self.head()

    def isEmpty(self) -> bool:  # noqa: N802
        return self.count() == 0

    def toPandas(self):  # noqa: N802
        import pandas as pd

        rows = self.collect()
        return pd.DataFrame([tuple(r) for r in rows], columns=self.columns)

    def show(self, n: int = 20, truncate=True, vertical: bool = False) -> None:
        rows = self.limit(n + 1).collect()
        more = len(rows) > n
        rows = rows[:n]
        if comm.rank() != 0:
            return
        width = 20 if truncate is True else (int(truncate) if truncate else 0)

        def fmt(v):
            if v is None:
                s = "NULL"
            elif isinstance(v, bool):
                s = str(v).lower()
            elif isinstance(v, float):
                s = "NaN" if math.isnan(v) else repr(v)
            else:
                s = str(v)
            if width and len(s) > width:
                s = s[: width - 3] + "..."
            return s

        cells = [[fmt(v) for v in r] for r in rows]
        names = self.columns
        w = [max([len(h)] + [len(c[i]) for c in cells]) for i, h in enumerate(names)]
        sep = "+" + "+".join("-" * x for x in w) + "+"
        out = [sep, "|" + "|".join(h.rjust(x) for h, x in zip(names, w)) + "|", sep]
        for c in cells:
            out.append("|" + "|".join(v.rjust(x) for v, x in zip(c, w)) + "|")
        out.append(sep)
        if more:
            out.append(f"only showing top {n} row{'s' if n != 1 else ''}")
        print("\n".join(out) + "\n", flush=True)

    # ------------------------------------------------------------------ aggregation
    def groupBy(self, *cols) -> "GroupedData":  # noqa: N802
        if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
            cols = tuple(cols[0])
        return GroupedData(self, [_to_col(c) for c in cols])

    groupby = groupBy

    def agg(self, *exprs) -> "DataFrame":
        return GroupedData(self, []).agg(*exprs)

    def describe(self, *cols) -> "DataFrame":
        names = list(cols) or [n for n, c in self._t.columns.items() if isinstance(c.dtype, T.NUMERIC)]
        stats = {}
        for n in names:
            s, c, mn, mx, _ = _global_stats(self._t.column(n))
            mean = s / c if c else None
            # second pass for stddev
            cv = self._t.column(n)
            x = cv.data.double()
            ok = cv.valid_bool() & ~torch.isnan(x)
            dev2 = float(((x - (mean or 0.0)) ** 2)[ok].sum()) if c else 0.0
            dev2 = comm.all_reduce_float([dev2])[0]
            sd = math.sqrt(dev2 / (c - 1)) if c > 1 else None
            stats[n] = [str(int(c)), str(mean), str(sd), str(mn if c else None), str(mx if c else None)]
        rows = [["count"], ["mean"], ["stddev"], ["min"], ["max"]]
        for i in range(5):
            rows[i] += [stats[n][i] for n in names]
        data = rows if comm.rank() == 0 else []
        return self.sparkSession.createDataFrame(data, ["summary"] + names, _local=True)

    # ------------------------------------------------------------------ misc
    def orderBy(self, *cols, ascending=True) -> "DataFrame":  # noqa: N802
        """Global sort.  World > 1: sample-based range partitioning on the first sort column (one
        tensor all-gather of samples, splitters picked on every rank identically), RCCL
        all-to-all-v of the rows, then a stable multi-column LSD radix sort (sort_scatter_k) on
        each rank; rank r holds the r-th key range, so rank-order concatenation is globally sorted."""
        if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
            cols = tuple(cols[0])
        asc = ascending if isinstance(ascending, (list, tuple)) else [ascending] * len(cols)
        specs = []
        for c, a in zip(cols, asc):
            c = _to_col(c)
            if c.node[0] == "sort":
                a = c.node[1]
                c = Column(c.node[2])
            specs.append((c, bool(a)))
        t = self._t
        world = comm.world_size()
        if comm.distributed():
            from . import shuffle as SH

            t = SH._unify_strings(t)
            data0, null0 = _sort_operand(DataFrame(t, self.sparkSession)._eval(specs[0][0])[1])
            k0, _, _ = D.sort_key(data0, desc=not specs[0][1])
            splitters = _range_splitters(k0 if null0 is None else k0[~null0], world)
            part, counts = D.range_partition(k0, splitters, world)
            if null0 is not None and bool(null0.any()):
                if part.is_cuda:
                    D.part_override(part, null0, 0 if specs[0][1] else world - 1)
                    counts = D.histogram(part, world)[:world]
                else:
                    part = torch.where(null0, torch.full_like(part, 0 if specs[0][1] else world - 1), part)
                    counts = torch.bincount(part.long(), minlength=world).to(torch.int64)
            t = SH.shuffle_table(t, D.partition_perm(part, counts), counts)
        if t.num_rows == 0 or not specs:
            return self._new(t)
        if len(specs) == 1 and specs[0][0].node[0] == "col":
            # one null-free integer sort column: the radix sort's own output keys ARE the sorted
            # column (decoded from the orderable form), so only the other columns are gathered
            name = t.resolve(specs[0][0].node[1])
            cv = t.column(name)
            if cv.valid is None and cv.data.dtype in (torch.int64, torch.int32) and not isinstance(cv.dtype, T.StringType):
                desc = not specs[0][1]
                # int64 on the GPU: the first radix pass reads the raw column and the last writes the
                # decoded values (XOR masks), so there is no key-prep write nor decode pass
                fused = cv.data.dtype == torch.int64 and cv.data.is_cuda and config.get("sort_fused_keys")
                if fused:  # one read of the column: key range + the first radix pass's counts
                    src = cv.data.contiguous()
                    lo, hi, h0 = D.sort_range_count(src, D.orderable_mask(desc))
                    rs = dict(xin=D.orderable_mask(desc), xout=D.orderable_mask(desc), hist0=h0)
                else:
                    k, lo, hi = D.sort_key(cv.data, desc=desc)
                    src, rs = k, {}
                others = [n for n in t.columns if n != name]
                oc = t.column(others[0]) if len(others) == 1 else None
                if (oc is not None and config.get("sort_value_payload") and oc.valid is None and oc.data.dim() == 1
                        and oc.data.element_size() == 8 and not isinstance(oc.dtype, T.StringType) and oc.data.is_cuda):
                    # exactly one other (8-byte, null-free) column: it rides through the radix passes as
                    # the payload (16 instead of 12 bytes per row per pass) instead of a row-id payload
                    # plus a random-access gather of the column by the permutation afterwards
                    sk, sv = D.radix_sort_u64(src, oc.data.contiguous().view(torch.int64), lo, hi, **rs)
                    kcol = sk if fused else D.decode_sort_key(sk, cv.data.dtype, desc)
                    cols = {n: (ColumnVector(kcol, cv.dtype, None, cv.dictionary) if n == name else
                                ColumnVector(sv.view(oc.data.dtype), oc.dtype, None, oc.dictionary))
                            for n in t.columns}
                    return self._new(Table(cols, t.num_rows, t.device))
                sk, perm = D.radix_sort_u64(src, None, lo, hi, row_payload=True, **rs)
                kcol = sk if fused else D.decode_sort_key(sk, cv.data.dtype, desc)
                cols = {n: (ColumnVector(kcol, cv.dtype, None, cv.dictionary) if n == name else c.take(perm))
                        for n, c in t.columns.items()}
                return self._new(Table(cols, t.num_rows, t.device))
        df_t = DataFrame(t, self.sparkSession)
        keys = []
        for c, a in specs:
            data, null = _sort_operand(df_t._eval(c)[1])
            keys.append((data, null, not a))
        return self._new(t.take(D.argsort_columns(keys)))
    sort = orderBy

    def distinct(self) -> "DataFrame":
        return self.dropDuplicates()

    def dropDuplicates(self, subset=None) -> "DataFrame":  # noqa: N802
        names = subset or self.columns
        g = GroupedData(self, [col(n) for n in names])
        return g.agg(*[]) if set(names) == set(self.columns) else g._first_rows()

    drop_duplicates = dropDuplicates

    def union(self, other: "DataFrame") -> "DataFrame":
        return self._new(Table.concat([self._t, other._t.select(self.columns) if other.columns != self.columns else other._t]))

    unionAll = union

    def unionByName(self, other: "DataFrame", allowMissingColumns=False) -> "DataFrame":  # noqa: N802, N803
        return self._new(Table.concat([self._t, other._t.select(self.columns)]))

    def repartition(self, numPartitions=None, *cols) -> "DataFrame":  # noqa: N803
        """``numPartitions`` partitions in total (default: spark.sql.shuffle.partitions with key
        columns, else the current count), partition p living on rank p % world as a contiguous row
        range of that rank's table (``_part_sizes``).  With columns: hash partitioning of the key
        (partition = hash % n) through the bucketed shuffle, one exchange round per partition round;
        without: rows spread round-robin over the ranks, then cut into that rank's share of equal
        contiguous partitions.  Each partition is a task of partition-wise operations (one file per
        partition on write)."""
        from .shuffle import bucket_exchange, round_robin_shuffle, shuffle_partitions

        if isinstance(numPartitions, (str, Column)):
            cols = (numPartitions,) + cols
            numPartitions = None
        world, rank = comm.world_size(), comm.rank()
        n = int(numPartitions) if numPartitions else (shuffle_partitions() if cols else self._num_partitions)
        n = max(1, n)
        t = self._t
        if cols:
            key = _group_keys(self, [_to_col(c) for c in cols])[0]
            if comm.distributed():
                pieces, sizes = [], []
                for _, pt in bucket_exchange(t, key, n, coalesce=False):
                    pieces.append(pt)
                    sizes.append(pt.num_rows)
                table = Table.concat(pieces) if pieces else t.take(torch.zeros(0, dtype=torch.int64, device=t.device))
            else:
                perm, counts = D.hash_partition(key, n)
                table = t.take(perm)
                sizes = [int(x) for x in counts.cpu().tolist()]
        else:
            table = round_robin_shuffle(t) if comm.distributed() else t
            mine = len(range(rank, n, world))
            sizes = [table.num_rows * (i + 1) // mine - table.num_rows * i // mine for i in range(mine)]
        d = self._new(table)
        d._num_partitions = n
        d._part_sizes = sizes
        return d

    def coalesce(self, numPartitions: int) -> "DataFrame":  # noqa: N803
        """Fewer partitions without a shuffle: adjacent local partitions are merged."""
        d = self._new(self._t)
        n = max(1, min(self._num_partitions, int(numPartitions)))
        d._num_partitions = n
        sizes = self.local_partition_sizes()
        mine = max(1, len(range(comm.rank(), n, comm.world_size())))
        if len(sizes) > mine:
            step = len(sizes) / mine
            d._part_sizes = [sum(sizes[int(i * step):int((i + 1) * step)]) for i in range(mine)]
        else:
            d._part_sizes = sizes
        return d

    def local_partition_sizes(self) -> list:
        """Row counts of this rank's partitions (contiguous ranges of its table, in order)."""
        sizes = getattr(self, "_part_sizes", None)
        n_rows = self._t.num_rows
        if sizes is not None and sum(sizes) == n_rows:
            return list(sizes)
        mine = max(1, len(range(comm.rank(), max(1, self._num_partitions), comm.world_size())))
        return [n_rows * (i + 1) // mine - n_rows * i // mine for i in range(mine)]

    def local_partitions(self) -> list:
        """This rank's partitions as Tables (views by row range, no copy of the data)."""
        t = self._t
        out, lo = [], 0
        for sz in self.local_partition_sizes():
            out.append(t.slice(lo, lo + sz))
            lo += sz
        return out

    def cache(self):
        """Materialise now (runs the pending narrow stage once) and keep the result resident."""
        _ = self._t
        return self

    persist = cache

    def unpersist(self, blocking=False):
        return self

    @property
    def rdd(self):
        from .rdd import RDD

        return RDD.from_list(self.sparkSession.sparkContext, self.collect(), max(1, self._num_partitions))

    @property
    def na(self):
        return _NaFunctions(self)

    def fillna(self, value, subset=None) -> "DataFrame":
        d = self
        items = value.items() if isinstance(value, dict) else [(n, value) for n in (subset or self.columns)]
        for n, v in items:
            cv = self._t.column(n)
            if isinstance(cv.dtype, T.StringType) != isinstance(v, str):
                continue
            if isinstance(v, str):
                d = d.withColumn(n, Column(("bin", "coalesce", col(n).node, ("lit", v))))
            else:
                d = d.withColumn(n, C.Column(("when", [((col(n).isNull() | C.Column(("un", "ISNAN", col(n).node))).node,
                                                        ("lit", v))], col(n).node)))
        return d

    def dropna(self, how="any", thresh=None, subset=None) -> "DataFrame":
        names = subset or self.columns
        conds = [col(n).isNotNull() for n in names]
        if how == "all" and thresh is None:
            out = conds[0]
            for c in conds[1:]:
                out = out | c
        else:
            out = conds[0]
            for c in conds[1:]:
                out = out & c
        return self.filter(out)

    def randomSplit(self, weights, seed=None):  # noqa: N802
        total = float(sum(weights))
        g = torch.Generator()
        g.manual_seed((seed or 0) + comm.rank())
        u = torch.rand(self._t.num_rows, generator=g).to(self._t.device)
        out, lo = [], 0.0
        for w in weights:
            hi = lo + w / total
            idx = D.compact(((u >= lo) & (u < hi)).to(torch.uint8))
            out.append(self._new(self._t.take(idx)))
            lo = hi
        return out

    def sample(self, withReplacement=False, fraction=0.1, seed=None):  # noqa: N803
        return self.randomSplit([fraction, 1 - fraction], seed)[0]

    def createOrReplaceTempView(self, name: str) -> None:  # noqa: N802
        self.sparkSession._views[name] = self

    createTempView = createOrReplaceTempView

    @property
    def write(self):
        from .readwriter import DataFrameWriter

        return DataFrameWriter(self)

    def __repr__(self):
        return "DataFrame[" + ", ".join(f"{n}: {t}" for n, t in self.dtypes) + "]"


class _NaFunctions:
    def __init__(self, df):
        self.df = df

    def fill(self, value, subset=None):
        return self.df.fillna(value, subset)

    def drop(self, how="any", thresh=None, subset=None):
        return self.df.dropna(how, thresh, subset)


def _remap_dictionary(src: ColumnVector, mapped: list) -> ColumnVector:
    new, idx, lut = [], {}, []
    for s in mapped:
        if s not in idx:
            idx[s] = len(new)
            new.append(s)
        lut.append(idx[s])
    lut_t = torch.tensor(lut + [-1], dtype=torch.int32, device=src.device)
    codes = src.data.long()
    codes = torch.where(codes < 0, torch.full_like(codes, len(lut)), codes)
    return ColumnVector(D.gather_rows(lut_t, codes), T.StringType(), src.valid, new)


def _coalesce_strings(a: ColumnVector, b: ColumnVector) -> ColumnVector:
    from .table import concat_columns

    merged = concat_columns([a, b])  # dictionary union + remap
    n = len(a)
    ca, cb = merged.data[:n], merged.data[n:]
    va = a.valid_bool() & (a.data >= 0)
    return ColumnVector(torch.where(va, ca, cb), T.StringType(), None, merged.dictionary)


def _parse_sql_predicate(s: str) -> Column:
    """Tiny SQL predicate parser for ``df.filter("Age > 30")``-style strings: <col> <op> <literal>
    joined by AND/OR."""
    parts = re.split(r"\s+(AND|OR)\s+", s.strip(), flags=re.I)
    out, pending = None, None
    for p in parts:
        if p.upper() in ("AND", "OR"):
            pending = p.upper()
            continue
        m = re.match(r"^\s*([A-Za-z_][\w]*)\s*(==|=|!=|<>|>=|<=|>|<)\s*(.+?)\s*$", p)
        if m:
            name, op, lit_s = m.groups()
            if lit_s.startswith(("'", '"')):
                lit_v = lit_s[1:-1]
            else:
                lit_v = float(lit_s) if any(ch in lit_s for ch in ".eE") else int(lit_s)
            op = {"=": "==", "<>": "!="}.get(op, op)
            c = col(name)._bin(op, lit_v)
        else:
            m = re.match(r"^\s*([A-Za-z_][\w]*)\s+IS\s+(NOT\s+)?NULL\s*$", p, flags=re.I)
            if not m:
                raise ValueError(f"unsupported predicate: {p!r}")
            c = col(m.group(1)).isNotNull() if m.group(2) else col(m.group(1)).isNull()
        out = c if out is None else (out & c if pending == "AND" else out | c)
    return out


def _global_stats(cv: ColumnVector):
    s, c, mn, mx, nul = D.reduce_stats(cv.data if cv.data.dtype != torch.bool else cv.data.to(torch.uint8),
                                       cv.valid_u8(), skip_nan=True)
    if comm.distributed():
        s, c, nul = comm.all_reduce_float([s, c, nul])
        mx, neg_mn = comm.all_reduce_float([mx, -mn], op=torch.distributed.ReduceOp.MAX)
        mn = -neg_mn
    return s, c, mn, mx, nul


def _gather_table_all(t: Table) -> Table:
    """Every rank's rows, in rank order, on every rank (collect): one tensor all-gather per column
    (+ validity), string columns after a dictionary union."""
    from .readwriter import unify_dictionary

    cols = {}
    for n, cv in t.columns.items():
        if isinstance(cv.dtype, T.StringType):
            cv = unify_dictionary(cv)
        data = torch.cat(comm.all_gather_v(cv.data.contiguous()))
        valid = None
        if comm.all_reduce_int([int(cv.valid is not None)])[0]:
            v = cv.valid_u8() if cv.valid is not None else torch.ones(len(cv), dtype=torch.uint8, device=cv.device)
            valid = torch.cat(comm.all_gather_v(v.contiguous()))
        cols[n] = ColumnVector(data, cv.dtype, valid, cv.dictionary)
    return Table(cols, sum(comm.all_gather_int(t.num_rows)), t.device)


def _sort_operand(cv: ColumnVector):
    """Column -> (tensor sort_key can order, null mask or None).  Strings sort by the rank of their
    dictionary entry (host sort of the distinct labels); NaN is a value (sorts above +inf)."""
    d = cv.data
    null = None
    if isinstance(cv.dtype, T.StringType):
        order = np.argsort(np.array(cv.dictionary or [], dtype=object), kind="stable")
        rank = np.empty(len(order) + 1, dtype=np.int64)
        rank[order] = np.arange(len(order))
        rank[-1] = 0
        lut = torch.from_numpy(rank).to(d.device)
        codes = d.long()
        null = codes < 0
        d = D.gather_rows(lut, torch.where(null, torch.full_like(codes, len(order)), codes))
    if cv.valid is not None:
        inv = ~cv.valid.bool()
        null = inv if null is None else (null | inv)
    if null is not None and not bool(null.any()):
        null = None
    return d, null


def _range_splitters(keys: torch.Tensor, world: int, per_rank: int = 4096) -> torch.Tensor:
    """world-1 splitters (u64 bit patterns in int64) from a strided sample of every rank's keys."""
    n = keys.numel()
    step = max(1, n // per_rank)
    sample = D.strided_sample(keys.contiguous(), step, min(per_rank, -(-n // step)))
    allk = comm.all_gather_v_host(sample).view(np.uint64)
    allk.sort()
    if allk.size == 0:
        return torch.zeros(world - 1, dtype=torch.int64)
    pos = [min(allk.size - 1, (i * allk.size) // world) for i in range(1, world)]
    return torch.from_numpy(allk[pos].view(np.int64).copy())


# ------------------------------------------------------------------------------------------------
# grouping
# ------------------------------------------------------------------------------------------------
def _key_of(cv: ColumnVector):
    """int64 grouping key of one column -> (key, null mask or None).  Null rows carry key 0; the
    mask keeps them in their own group, outside the key domain (no sentinel value can collide with
    a real key: every int64 and every double bit pattern is a legal key)."""
    d = cv.data
    if isinstance(cv.dtype, T.StringType):
        k = d.long()
        null = k < 0
    elif d.dtype in (torch.float64, torch.float32):
        x = d.double()
        x = torch.where(torch.isnan(x), torch.full_like(x, math.nan), x) + 0.0  # canonical NaN, -0 -> +0
        k = x.view(torch.int64)
        null = None
    else:
        k = d.long()
        null = None
    if cv.valid is not None:
        inv = ~cv.valid.bool()
        null = inv if null is None else (null | inv)
    if null is not None:
        if not bool(null.any()):
            return k, None
        k = torch.where(null, torch.zeros_like(k), k)
    return k, null


def _decode_key(k: torch.Tensor, src: ColumnVector, null: torch.Tensor | None = None) -> ColumnVector:
    """Inverse of :func:`_key_of`: group key (+ null flag) -> key column value (so grouped outputs
    need no representative-row lookup)."""
    valid = None if null is None or not bool(null.any()) else (~null).to(torch.uint8)
    if valid is None:  # no null group: the key is the value (no where / zeros kernels)
        if isinstance(src.dtype, T.StringType):
            return ColumnVector(k.to(torch.int32), src.dtype, None, src.dictionary)
        if src.data.dtype in (torch.float64, torch.float32):
            return ColumnVector(k.view(torch.float64).to(src.data.dtype), src.dtype, None)
        return ColumnVector(k.to(src.data.dtype), src.dtype, None)
    if isinstance(src.dtype, T.StringType):
        return ColumnVector(torch.where(null, torch.full_like(k, -1), k).to(torch.int32), src.dtype, None,
                            src.dictionary)
    if src.data.dtype in (torch.float64, torch.float32):
        v = torch.where(null, torch.zeros_like(k), k).view(torch.float64)
        return ColumnVector(v.to(src.data.dtype), src.dtype, valid)
    v = torch.where(null, torch.zeros_like(k), k)
    return ColumnVector(v.to(src.data.dtype), src.dtype, valid)


def _count_distinct(cv: ColumnVector) -> int:
    """countDistinct of one column (nulls ignored, NaN a value) across ranks.  GPU: orderable keys
    (key_prep), the valid rows compacted, distinct keys by hash aggregation without value columns,
    the ranks' distinct sets merged the same way - only our kernels."""
    world = comm.world_size()
    if cv.data.is_cuda:
        kt = _kt_of(cv)
        stats = torch.empty(3, dtype=torch.int64, device=cv.data.device)
        u, ok = D.key_prep(cv.data, kt, cv.valid, cv.valid is not None or kt == D.KT_CODE, stats, mode=D.KEY_RAW)
        if ok is not None:
            u = D.gather_rows(u, D.compact(ok))
        uk = D.distinct_raw(u)
        if comm.distributed():
            uk = D.distinct_raw(torch.cat(comm.all_gather_v(uk)))
        return int(uk.numel())
    k, null = _key_of(cv)
    ok = cv.valid_bool() if null is None else (cv.valid_bool() & ~null)
    loc = torch.unique(k[ok])
    return int(comm.all_gather_unique(loc).numel()) if comm.distributed() else int(loc.numel())


def _any_rank(flag: bool) -> bool:
    if not comm.distributed():
        return flag
    return bool(comm.all_reduce_int([int(flag)])[0])


def _kt_of(cv: ColumnVector) -> int:
    if isinstance(cv.dtype, T.StringType):
        return D.KT_CODE
    return D.TORCH_CT[cv.data.dtype]


def _group_keys_device(srcs: list):
    """Device path of :func:`_group_keys` (csrc/kernels/dfkey.hip): every key column becomes an
    orderable u64 key + valid flag + (min, max, nulls) in one kernel; the ranks agree on the ranges
    (three small all-reduces); each column gets a bit field of the combined int64 key holding
    (key - min), or its rank among the sorted distinct keys when the ranges do not fit 63 bits
    together, plus one code for null.  Exact (no hashing), and decoding the result groups is one
    kernel.  Returns None when even rank coding cannot fit (then the host-dictionary path runs)."""
    n = srcs[0][1].data.shape[0]
    dev = srcs[0][1].data.device
    nc = len(srcs)
    stats = torch.empty(3 * nc, dtype=torch.int64, device=dev)
    cols = []
    for j, (name, cv) in enumerate(srcs):
        kt = _kt_of(cv)
        maybe_null = cv.valid is not None or kt == D.KT_CODE
        u, ok = D.key_prep(cv.data, kt, cv.valid, maybe_null, stats[3 * j:3 * j + 3])
        cols.append({"name": name, "cv": cv, "u": u, "ok": ok, "lut": None, "type": kt})
    st = [x & ((1 << 64) - 1) for x in stats.cpu().tolist()]  # u64 bit patterns
    world = comm.world_size()
    if comm.distributed():  # orderable u64 -> signed order for the int64 collectives
        sg = lambda x: x - (1 << 63)  # noqa: E731
        mins = comm.all_reduce_int([sg(st[3 * j]) for j in range(nc)], op=dist.ReduceOp.MIN)
        maxs = comm.all_reduce_int([sg(st[3 * j + 1]) for j in range(nc)], op=dist.ReduceOp.MAX)
        nulls = comm.all_reduce_int([st[3 * j + 2] for j in range(nc)])
        for j in range(nc):
            st[3 * j], st[3 * j + 1], st[3 * j + 2] = mins[j] + (1 << 63), maxs[j] + (1 << 63), nulls[j]
    for j, c in enumerate(cols):
        lo, hi, nn = st[3 * j], st[3 * j + 1], st[3 * j + 2]
        empty = lo > hi  # every row null (or no rows)
        c["lo"] = 0 if empty else lo
        c["nvals"] = 0 if empty else hi - lo + 1
        c["has_null"] = nn > 0
        if not c["has_null"]:
            c["ok"] = None
    def bits_of(c):
        return max(1, (c["nvals"] + int(c["has_null"]) - 1).bit_length())
    # columns whose value range is too wide for the 63-bit budget switch to rank coding, widest first
    while sum(bits_of(c) for c in cols) > 63:
        wide = [c for c in cols if c["lut"] is None and c["nvals"] > 1]
        if not wide:
            return None
        c = max(wide, key=lambda q: q["nvals"])
        # distinct keys by hash aggregation over the RAW canonical keys (the orderable form of 0 is
        # the hash tables' empty marker), then orderable + radix-sorted for the pack kernel's search
        st1 = torch.empty(3, dtype=torch.int64, device=dev)
        raw, _ = D.key_prep(c["cv"].data, c["type"], c["cv"].valid, False, st1, mode=D.KEY_RAW)
        if c["ok"] is not None:
            raw = D.gather_rows(raw, D.compact(c["ok"]))
        raw = D.distinct_raw(raw)
        if comm.distributed():
            raw = D.distinct_raw(torch.cat(comm.all_gather_v(raw)))
        lut = D.sorted_orderable(raw, c["type"])
        c["lut"], c["lo"], c["nvals"] = lut, 0, int(lut.numel())
    shift = 0
    for c in cols:
        c["bits"] = bits_of(c)
        c["shift"] = shift
        c["nullcode"] = c["nvals"]
        shift += c["bits"]
    key, desc = D.key_pack(cols, n, dev)

    def decode(kk):
        m = kk.numel()
        outs, res = [], {}
        for c in cols:
            cv = c["cv"]
            data = torch.empty(m, dtype=torch.int32 if c["type"] == D.KT_CODE else cv.data.dtype, device=dev)
            valid = torch.empty(m, dtype=torch.uint8, device=dev) if c["has_null"] else None
            outs.append((data.view(torch.uint8) if data.dtype == torch.bool else data, valid))
            res[c["name"]] = ColumnVector(data, cv.dtype, valid, cv.dictionary)
        if m:
            D.key_unpack(kk.contiguous(), desc, outs)
        return res

    return key, decode


def _group_keys(df: "DataFrame", cols: list):
    """-> (int64 combined key per row, decode(keys) -> {name: ColumnVector}).  A single null-free
    int64 column is its own key.  On the GPU every other case packs the columns into one exact key
    on the device (:func:`_group_keys_device`); on the host every column is mapped to a dense code
    over the global set of its distinct values (+1 code for null), and the codes are combined
    mixed-radix (exact, no hash collisions)."""
    srcs = []
    for c in cols:
        name, cv = df._eval(c)
        srcs.append((name, cv))
    if not srcs:
        return torch.zeros(df._t.num_rows, dtype=torch.int64, device=df._t.device), lambda kk: {}
    cv0 = srcs[0][1]
    if cv0.data.is_cuda:
        plain = (len(srcs) == 1 and cv0.data.dtype == torch.int64 and not isinstance(cv0.dtype, T.StringType)
                 and not _any_rank(cv0.valid is not None))
        if not plain:
            r = _group_keys_device(srcs) if len(srcs) <= D.KMAX else None
            if r is not None:
                return r
    keyed = [(name, cv) + _key_of(cv) for name, cv in srcs]
    if len(keyed) == 1 and not _any_rank(keyed[0][3] is not None):
        name, cv, k, _ = keyed[0]
        return k, lambda kk: {name: _decode_key(kk, cv)}
    combined = None
    globs = []
    for _, cv, k, null in keyed:
        has_null = _any_rank(null is not None)
        kv = k if null is None else k[~null]
        if comm.distributed():
            # globally consistent dense codes: union of distinct keys across ranks
            glob = comm.all_gather_unique(torch.unique(kv))
        else:
            glob = torch.unique(kv)
        code = torch.searchsorted(glob, k) if glob.numel() else torch.zeros_like(k)
        if null is not None:
            code = torch.where(null, torch.full_like(code, glob.numel()), code)
        card = glob.numel() + int(has_null)
        globs.append((glob, card))
        combined = code.long() if combined is None else combined * card + code.long()

    def decode(kk):
        out = {}
        rem = kk.clone()
        codes = []
        for _, card in reversed(globs):
            codes.append(rem % card)
            rem = rem // card
        codes.reverse()
        for (name, cv, _, _), (g, card), c in zip(keyed, globs, codes):
            isnull = c >= g.numel()
            gv = g[c.clamp_max(max(g.numel() - 1, 0))] if g.numel() else torch.zeros_like(c)
            out[name] = _decode_key(gv, cv, isnull)
        return out

    return combined, decode


def _shuffle_by_key(t: Table, key: torch.Tensor) -> Table:
    """Hash-partition rows by key across ranks (bounded, chunked RCCL all-to-all-v; sql/shuffle.py)."""
    from .shuffle import hash_shuffle

    return hash_shuffle(t, key)


class GroupedData:
    def __init__(self, df: DataFrame, cols: list):
        self.df = df
        self.cols = cols

    def _aggs_from(self, exprs):
        aggs = []  # (out_name, fn, source column name or None)
        if len(exprs) == 1 and isinstance(exprs[0], dict):
            for cname, fn in exprs[0].items():
                fn = {"mean": "avg", "average": "avg"}.get(fn, fn)
                src = None if cname == "*" else cname
                label = f"{fn}({'1' if src is None and fn == 'count' else (cname if src else '*')})"
                aggs.append((label, fn, None if src is None else col(src)))
            return aggs
        for e in exprs:
            node = e.node
            name = node[1] if node[0] == "alias" else None
            base = C.strip_alias(node)
            if base[0] != "agg":
                raise TypeError(f"not an aggregate expression: {expr_name(node)}")
            fn, x = base[1], base[2]
            aggs.append((name or expr_name(base), fn, None if x is None else Column(x)))
        return aggs

    def count(self) -> DataFrame:
        return self.agg(Column(("alias", "count", ("agg", "count", None))))

    def _simple(self, fn, cols):
        df = self.df
        names = cols or [n for n, c in df._t.columns.items() if isinstance(c.dtype, T.NUMERIC)
                         and n not in {expr_name(c.node) for c in self.cols}]
        return self.agg(*[Column(("alias", f"{fn}({n})", ("agg", fn, col(n).node))) for n in names])

    def sum(self, *cols):
        return self._simple("sum", cols)

    def avg(self, *cols):
        return self._simple("avg", cols)

    mean = avg

    def min(self, *cols):
        return self._simple("min", cols)

    def max(self, *cols):
        return self._simple("max", cols)

    def agg(self, *exprs) -> DataFrame:
        df = self.df
        aggs = self._aggs_from(exprs)
        if df._mat is None and df._pending:
            from . import plan as P

            exprs_ok = all(P._inlinable(c.node) for c in self.cols) and all(
                src is None or P._inlinable(src.node) for _, fn, src in aggs) and all(
                fn not in ("first",) for _, fn, _ in aggs)
            if exprs_ok and P.fusable(df._pending):
                return self._agg_fused(aggs)
        return self._agg_table(df, aggs)

    def _agg_fused(self, aggs) -> DataFrame:
        """The aggregation consumes the pending stage in one fused scan (sql/plan.py): projections
        inlined, one predicate mask; a global aggregate reduces under the mask, a grouped one
        compacts once and gathers only the source columns its expressions read."""
        from . import plan as P

        df = self.df
        src = df._src
        inl = P.Inlined(df._pending)
        P.STATS["fused_aggs"] += 1
        base = DataFrame(src, df.sparkSession)
        mask = None
        if inl.cond is not None:
            mask = base._mask(Column(inl.cond))
            P.STATS["vm_passes"] += 1
        text = P.describe_fused_agg(df._pending, self.cols, aggs)
        if not self.cols:
            out = self._agg_global(aggs, lambda c: base._eval(Column(inl.expr(c.node)), expr_name(c.node)), mask,
                                   src)
            out._plan_text = text
            return out
        # grouped: compact once, gather only the source columns the key / value expressions read
        nodes = [inl.expr(c.node) for c in self.cols] + [inl.expr(s.node) for _, _, s in aggs if s is not None]
        leaves = set()
        for nd in nodes:
            leaves |= C.referenced_columns(nd)
        keep = [n for n in src.names if n in leaves or n.lower() in {x.lower() for x in leaves}]
        pruned = src.select(keep)
        if mask is not None:
            pruned = pruned.take(D.compact(mask))
            P.STATS["compactions"] += 1
            P.STATS["gathers"] += 1
        pdf = DataFrame(pruned, df.sparkSession)
        pdf._num_partitions = df._num_partitions
        keys = [Column(("alias", expr_name(c.node), inl.expr(c.node))) for c in self.cols]
        aggs2 = [(label, fn, None if s is None else Column(inl.expr(s.node))) for label, fn, s in aggs]
        out = GroupedData(pdf, keys)._agg_table(pdf, aggs2)
        out._plan_text = text
        return out

    def _agg_global(self, aggs, evalf, mask, t) -> DataFrame:
        """Global aggregates of value columns ``evalf(src)`` restricted to the rows of ``mask``."""
        df = self.df
        sess = df.sparkSession
        world = comm.world_size()
        vals = {}

        def masked(cv):
            if mask is None:
                return cv
            v = cv.valid_u8() if cv.valid is not None else None
            m = mask if v is None else (mask & v)
            return ColumnVector(cv.data, cv.dtype, m, cv.dictionary)

        nrows = None
        for label, fn, src in aggs:
            if src is None:
                if nrows is None:
                    local = int(mask.sum()) if mask is not None else t.num_rows
                    nrows = comm.all_reduce_int([local])[0]
                vals[label] = nrows
                continue
            _, cv = evalf(src)
            cv = masked(cv)
            if fn == "count_distinct":
                vals[label] = _count_distinct(cv)
                continue
            s_, c, mn, mx, nul = _global_stats(cv)
            if fn == "count":
                vals[label] = comm.all_reduce_int([int(cv.valid_bool().sum())])[0]
            elif fn == "sum":
                vals[label] = s_ if c else None
            elif fn == "avg":
                vals[label] = s_ / c if c else None
            elif fn == "min":
                vals[label] = mn if c else None
            elif fn == "max":
                vals[label] = mx if c else None
            elif fn == "stddev":
                mean = s_ / c if c else 0.0
                x = cv.data.double()
                ok = cv.valid_bool() & ~torch.isnan(x)
                d2 = comm.all_reduce_float([float(((x - mean) ** 2)[ok].sum())])[0]
                vals[label] = math.sqrt(d2 / (c - 1)) if c > 1 else None
            else:
                raise ValueError(f"unsupported aggregate {fn}")
        data = [tuple(vals.values())] if comm.rank() == 0 else []
        schema = []
        for (label, fn, src), v in zip(aggs, vals.values()):
            dt = T.LongType() if fn in ("count", "count_distinct") else T.DoubleType()
            if fn in ("min", "max", "sum") and src is not None:
                st = evalf(src)[1].dtype
                dt = st if fn != "sum" or isinstance(st, (T.DoubleType, T.FloatType)) else T.LongType()
            schema.append(T.StructField(label, dt))
        return sess.createDataFrame(data, T.StructType(schema), _local=True)

    def _agg_table(self, df, aggs) -> DataFrame:
        t = df._t
        sess = df.sparkSession
        world = comm.world_size()
        if not self.cols:  # global aggregation -> one row on rank 0
            vals = {}
            for label, fn, src in aggs:
                if src is None:
                    vals[label] = df.count()
                    continue
                _, cv = df._eval(src)
                if fn == "count_distinct":
                    vals[label] = _count_distinct(cv)
                    continue
                if fn == "first":
                    vals[label] = df.select(src).first()[0] if df.count() else None
                    continue
                s, c, mn, mx, nul = _global_stats(cv)
                if fn == "count":
                    vals[label] = int(c + (nul if cv.data.dtype in (torch.float32, torch.float64) and False else 0))
                    # Spark count(col) counts non-null values (NaN counts as a value)
                    x = cv.data
                    if x.dtype in (torch.float32, torch.float64):
                        vals[label] = comm.all_reduce_int([int((cv.valid_bool()).sum())])[0]
                elif fn == "sum":
                    vals[label] = s if c else None
                elif fn == "avg":
                    vals[label] = s / c if c else None
                elif fn == "min":
                    vals[label] = mn if c else None
                elif fn == "max":
                    vals[label] = mx if c else None
                elif fn == "stddev":
                    mean = s / c if c else 0.0
                    x = cv.data.double()
                    ok = cv.valid_bool() & ~torch.isnan(x)
                    d2 = comm.all_reduce_float([float(((x - mean) ** 2)[ok].sum())])[0]
                    vals[label] = math.sqrt(d2 / (c - 1)) if c > 1 else None
                else:
                    raise ValueError(f"unsupported aggregate {fn}")
            data = [tuple(vals.values())] if comm.rank() == 0 else []
            schema = []
            for (label, fn, src), v in zip(aggs, vals.values()):
                dt = T.LongType() if fn in ("count", "count_distinct") else T.DoubleType()
                if fn in ("min", "max", "sum") and src is not None:
                    st = C.infer_type(src.node, t)
                    dt = st if fn != "sum" or isinstance(st, (T.DoubleType, T.FloatType)) else T.LongType()
                schema.append(T.StructField(label, dt))
            return sess.createDataFrame(data, T.StructType(schema), _local=True)
        # ---- keyed aggregation
        key, decode = _group_keys(df, self.cols)
        value_cols = []
        for label, fn, src in aggs:
            if src is None:
                continue
            _, cv = df._eval(src)
            value_cols.append(cv)
        need_minmax = any(fn in ("min", "max") for _, fn, _ in aggs)
        # partial aggregation (rank-local)
        vdata = [_num(cv) for cv in value_cols]
        vvalid = [cv.valid_u8() for cv in value_cols]
        ukeys, rows, outs = _hash_agg_all(key, vdata, vvalid, need_minmax)
        if comm.distributed():
            # shuffle the partials to the key owners in spark.sql.shuffle.partitions hash buckets, one
            # reduce partition per round (RCCL all-to-all-v), and merge each received bucket as its
            # own reduce task: staging per round ~ 1/buckets of the partials
            from .shuffle import bucket_exchange, shuffle_partitions

            part_cols = {"__k": ColumnVector(ukeys, T.LongType()), "__rows": ColumnVector(rows, T.DoubleType())}
            for j, (s, c, mn, mx) in enumerate(outs):
                part_cols[f"__s{j}"] = ColumnVector(s, T.DoubleType())
                part_cols[f"__c{j}"] = ColumnVector(c, T.DoubleType())
                part_cols[f"__mn{j}"] = ColumnVector(mn, T.DoubleType())
                part_cols[f"__mx{j}"] = ColumnVector(mx, T.DoubleType())
            ks, rs, os_ = [], [], []
            for _, pt in bucket_exchange(Table(part_cols, ukeys.numel(), t.device), ukeys, shuffle_partitions()):
                if pt.num_rows == 0:
                    continue
                k2 = pt.column("__k").data
                vals2 = [pt.column("__rows").data]
                for j in range(len(outs)):
                    vals2 += [pt.column(f"__s{j}").data, pt.column(f"__c{j}").data, pt.column(f"__mn{j}").data,
                              pt.column(f"__mx{j}").data]
                uk2, _, o2 = _hash_agg_all(k2, vals2, [None] * len(vals2), need_minmax)
                ks.append(uk2)
                rs.append(o2[0][0])
                os_.append([(o2[1 + 4 * j][0], o2[2 + 4 * j][0], o2[3 + 4 * j][2], o2[4 + 4 * j][3])
                            for j in range(len(outs))])
            if len(ks) == 1:  # one reduce task (the usual case after adaptive coalescing): no copies
                ukeys, rows, outs = ks[0], rs[0], os_[0]
            elif ks:
                ukeys, rows = torch.cat(ks), torch.cat(rs)
                outs = [tuple(torch.cat([o[j][q] for o in os_]) for q in range(4)) for j in range(len(outs))]
            else:
                ukeys, rows = ukeys[:0], rows[:0]
                outs = [tuple(x[:0] for x in o) for o in outs]
        cols = dict(decode(ukeys))
        if ukeys.is_cuda:
            return df._new(Table(self._finalize_device(cols, aggs, value_cols, rows, outs), ukeys.numel(), t.device))
        j = 0
        for label, fn, src in aggs:
            if src is None:
                cols[label] = ColumnVector(rows.round().long(), T.LongType())
                continue
            s, c, mn, mx = outs[j]
            srct = value_cols[j].dtype
            j += 1
            has = c > 0
            if fn == "count":
                cols[label] = ColumnVector(c.round().long(), T.LongType())
            elif fn == "sum":
                integral = isinstance(srct, (T.IntegerType, T.LongType, T.BooleanType))
                cols[label] = ColumnVector(s.round().long() if integral else s, T.LongType() if integral else T.DoubleType(),
                                           has.to(torch.uint8))
            elif fn == "avg":
                cols[label] = ColumnVector(s / c.clamp_min(1.0), T.DoubleType(), has.to(torch.uint8))
            elif fn in ("min", "max"):
                v = mn if fn == "min" else mx
                if isinstance(srct, (T.IntegerType, T.LongType)):
                    cols[label] = ColumnVector(torch.where(has, v, torch.zeros_like(v)).to(_TORCH_OF[type(srct)]), srct,
                                               has.to(torch.uint8))
                else:
                    cols[label] = ColumnVector(v, T.DoubleType(), has.to(torch.uint8))
            else:
                raise ValueError(f"unsupported grouped aggregate {fn}")
        return df._new(Table(cols, ukeys.numel(), t.device))

    @staticmethod
    def _finalize_device(cols, aggs, value_cols, rows, outs) -> dict:
        """Result columns of a keyed aggregation in one kernel (dfkey.hip agg_finalize_k): counts,
        integral sums and min / max keep their integer types, null where a group had no value."""
        m = rows.numel()
        dev = rows.device
        specs = []
        j = 0
        for label, fn, src in aggs:
            if src is None:
                out = torch.empty(m, dtype=torch.int64, device=dev)
                specs.append(("rows", 3, None, None, None, None, out, None))
                cols[label] = ColumnVector(out, T.LongType())
                continue
            s_, c_, mn, mx = outs[j]
            srct = value_cols[j].dtype
            j += 1
            integral = isinstance(srct, (T.IntegerType, T.LongType, T.BooleanType))
            valid = torch.empty(m, dtype=torch.uint8, device=dev)
            if fn == "count":
                out = torch.empty(m, dtype=torch.int64, device=dev)
                specs.append(("count", 3, s_, c_, mn, mx, out, None))
                cols[label] = ColumnVector(out, T.LongType())
            elif fn == "sum":
                out = torch.empty(m, dtype=torch.int64 if integral else torch.float64, device=dev)
                specs.append(("sum_int" if integral else "sum", 3 if integral else 1, s_, c_, mn, mx, out, valid))
                cols[label] = ColumnVector(out, T.LongType() if integral else T.DoubleType(), valid)
            elif fn == "avg":
                out = torch.empty(m, dtype=torch.float64, device=dev)
                specs.append(("avg", 1, s_, c_, mn, mx, out, valid))
                cols[label] = ColumnVector(out, T.DoubleType(), valid)
            elif fn in ("min", "max"):
                if isinstance(srct, (T.IntegerType, T.LongType)):
                    tdt = _TORCH_OF[type(srct)]
                    out = torch.empty(m, dtype=tdt, device=dev)
                    specs.append((fn, D.TORCH_CT[tdt], s_, c_, mn, mx, out, valid))
                    cols[label] = ColumnVector(out, srct, valid)
                else:
                    out = torch.empty(m, dtype=torch.float64, device=dev)
                    specs.append((fn, 1, s_, c_, mn, mx, out, valid))
                    cols[label] = ColumnVector(out, T.DoubleType(), valid)
            else:
                raise ValueError(f"unsupported grouped aggregate {fn}")
        if m and specs:
            D.agg_finalize(rows, specs)
        return cols

    def _first_rows(self) -> DataFrame:
        df = self.df
        t = df._t
        key, _ = _group_keys(df, self.cols)
        if comm.distributed():
            t = _shuffle_by_key(t, key)
            df = df._new(t)
            key, _ = _group_keys(df, self.cols)
        if key.is_cuda:
            # first row of every group: min row id per key (hash aggregation), ids sorted by our
            # radix sort, rows gathered - dropDuplicates keeps the input order of the survivors
            ridx = D.iota_f64(t.num_rows, t.device)
            _, _, rep = _hash_agg_all(key, [ridx], [None], True)
            ids = D.f64_to_i64(rep[0][2])
            idx, _ = D.radix_sort_u64(ids, None, 0, max(t.num_rows - 1, 0))
            return df._new(t.take(idx))
        ridx = torch.arange(t.num_rows, dtype=torch.float64, device=t.device)
        _, _, rep = _hash_agg_all(key, [ridx], [None], True)
        idx = torch.sort(rep[0][2].long()).values
        return df._new(t.take(idx))


_PART_WS: dict = {}  # scratch buffers of the radix-partitioned aggregation, reused across queries
_RADIX_MIN_ROWS = 1 << 16
_RADIX_MIN_KEYS = 4096


def _num(cv: ColumnVector) -> torch.Tensor:
    d = cv.data
    if d.dtype == torch.bool:
        return d.to(torch.uint8)
    if isinstance(cv.dtype, T.StringType):
        raise TypeError("cannot aggregate a string column numerically")
    return d


def _hash_agg_all(key, vals, valids, want_minmax):
    """Rank-local groupBy aggregate of any number of value columns.  Few distinct keys: LDS
    tables + global table (hash_agg).  Many: recursive radix partitioning with one LDS table per
    partition (hash_agg_radix; exact at any cardinality).  Value columns go 4 per pass, the passes
    re-aligned by key order."""
    n = key.numel()
    fn = D.hash_agg
    est = None
    if key.is_cuda and n >= _RADIX_MIN_ROWS:
        est = D.estimate_distinct(key)
        if est > _RADIX_MIN_KEYS:
            def fn(k, v, vd, mm):
                return D.hash_agg_radix(k, v, vd, mm, ws=_PART_WS, est_keys=est)
        else:
            def fn(k, v, vd, mm):
                return D.hash_agg(k, v, vd, mm, est_keys=est)
    if len(vals) <= 4:
        return fn(key, vals, valids, want_minmax)
    uk = rows = None
    outs = []
    for i in range(0, len(vals), 4):
        k, r, o = fn(key, vals[i:i + 4], valids[i:i + 4], want_minmax)
        # every pass yields the same key set: one radix sort each (any consistent order aligns them)
        if k.is_cuda:
            k, order = D.radix_sort_u64(k, None, 0, D._U64, row_payload=True)
            r = D.gather_rows(r, order)
            o = [tuple(D.gather_rows(x, order) for x in q) for q in o]
        else:
            order = torch.argsort(k)
            k, r = k[order], r[order]
            o = [tuple(x[order] for x in q) for q in o]
        if uk is None:
            uk, rows = k, r
        outs += o
    return uk, rows, outs
