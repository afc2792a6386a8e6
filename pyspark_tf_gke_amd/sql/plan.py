"""Lazy narrow stages: the part of Spark's Catalyst planner + task scheduler the reference workloads
lean on (k_means.py:23-51 chains filter / withColumn(when(isnan ...)) / filter before every action;
spark_workload_to_cloud_k8s.py repeats the pattern on GCS CSVs).

``filter`` and ``withColumn`` do not run when called: they append to the DataFrame's pending
narrow stage, which runs when the table is first needed (an action, a wide transformation, or
``cache()``), then stays materialised in HBM.  Before it runs, the stage is optimised:

* predicate pushdown — a filter that reads only source columns (not a column produced earlier
  in the same stage) moves ahead of the projections, so they are computed on the surviving rows
  only;
* filter fusion — adjacent filters become ONE predicate: one expression-VM pass (df.hip
  expr_eval_k), one compaction and one row gather for all of them, instead of one of each per
  ``filter`` call;
* barriers — expressions with rand() / monotonically_increasing_id() depend on row positions, so
  nothing is reordered across them.

``select`` of plain expressions is lazy too (a projection that also prunes columns).  An
aggregation over a pending stage does not materialise it (``fused_aggregate``, the wide operation
joining the lazy plan the way Catalyst's whole-stage codegen feeds HashAggregate): the projections
are inlined into the filter and aggregate expressions (column references replaced by their defining
expressions over the source table), all filters become ONE predicate evaluated in one expression-VM
pass, and
* a global aggregate (``df.filter(...).select(c).agg({c: "avg"})``, k_means.py:45-51) reduces the
  source rows under the predicate mask - no compaction, no row gather;
* a grouped aggregate compacts the mask once and gathers only the source columns its key / value
  expressions read (column pruning), then partially aggregates.

The stage runs as a *task* with Spark's retry semantics (``spark.task.maxFailures``, default 4):
a narrow stage is rank-local (no collective inside), so a failed attempt is simply re-run from
its resident input.  Any ``RuntimeError`` of an attempt counts (a HIP launch error, an injected
fault); an out-of-memory attempt is re-planned: the retry runs the stage over 2, 4, ... row chunks
of its input (narrow operators are row-local; stages with position-dependent leaves - rand(),
monotonically_increasing_id() - are not chunked).  ``PTG_FAULT_TASK=k`` makes the first k task
attempts of the process fail, ``PTG_FAULT_TASK_OOM=k`` the first k with an out-of-memory error
(fault-injection for the retry tests).  ``DataFrame.explain()`` prints the optimised stage.
"""
from __future__ import annotations

import os

from .column import Column
from .table import Table

_BARRIER_LEAVES = ("rand", "rowid")
STATS = {"tasks": 0, "attempts": 0, "retries": 0, "vm_passes": 0, "gathers": 0, "replans": 0, "chunks": 0,
         "fused_aggs": 0, "compactions": 0}
_FAULTS = {"left": int(os.environ.get("PTG_FAULT_TASK", "0") or 0),
           "oom": int(os.environ.get("PTG_FAULT_TASK_OOM", "0") or 0)}


class TaskFailure(RuntimeError):
    """A task attempt failed (injected fault or a transient executor error)."""


def _walk(node):
    if isinstance(node, tuple):
        yield node
        for x in node:
            if isinstance(x, tuple):
                yield from _walk(x)
            elif isinstance(x, list):
                for pair in x:
                    if isinstance(pair, tuple):
                        for y in pair:
                            if isinstance(y, tuple):
                                yield from _walk(y)


def referenced_columns(node) -> set:
    return {n[1].lower() for n in _walk(node) if n and n[0] == "col" and isinstance(n[1], str)}


def is_barrier(node) -> bool:
    return any(n and n[0] in _BARRIER_LEAVES for n in _walk(node))


def optimize(ops: list) -> tuple[list, list]:
    """-> (pushed filters, remaining ops in order).  ops: ("filter", Column) | ("with", name, Column)."""
    produced: set = set()
    blocked = False
    pushed, rest = [], []
    for op in ops:
        if op[0] == "filter":
            node = op[1].node
            if not blocked and not (referenced_columns(node) & produced) and not is_barrier(node):
                pushed.append(op)
            else:
                rest.append(op)
                blocked = blocked or is_barrier(node)
        elif op[0] == "select":
            rest.append(op)
            blocked = True  # later filters see the projection's names only
        else:
            rest.append(op)
            produced.add(op[1].lower())
            blocked = blocked or is_barrier(op[2].node)
    return pushed, rest


def _groups(ops: list) -> list:
    """Adjacent filters fused into one ("filters", [Column, ...]) group."""
    out = []
    for op in ops:
        if op[0] == "filter" and out and out[-1][0] == "filters":
            out[-1][1].append(op[1])
        elif op[0] == "filter":
            out.append(("filters", [op[1]]))
        else:
            out.append(op)
    return out


def _and_all(conds: list) -> Column:
    c = conds[0]
    for x in conds[1:]:
        c = c & x
    return c


def _run_stage(src: Table, ops: list, session) -> Table:
    from .dataframe import DataFrame

    from ..ops import df as D

    pushed, rest = optimize(ops)
    groups = ([("filters", [op[1] for op in pushed])] if pushed else []) + _groups(rest)
    t = src
    for g in groups:
        view = DataFrame(t, session)
        if g[0] == "filters":
            idx = D.compact(view._mask(_and_all(g[1])))
            STATS["vm_passes"] += 1
            STATS["gathers"] += 1
            STATS["compactions"] += 1
            t = t.take(idx)
        elif g[0] == "select":
            cols = {}
            for name, c in g[1]:
                cols[name] = view._eval(c, name)[1]
                STATS["vm_passes"] += 1
            t = Table(cols, t.num_rows, t.device)
        else:
            _, cv = view._eval(g[2], g[1])
            STATS["vm_passes"] += 1
            t = t.with_column(g[1], cv)
    return t


def max_failures(session) -> int:
    try:
        return max(1, int(session.conf.get("spark.task.maxFailures", 4))) if session is not None else 4
    except (TypeError, ValueError):
        return 4


def _is_oom(e: BaseException) -> bool:
    import torch

    return isinstance(e, getattr(torch, "OutOfMemoryError", ())) or "out of memory" in str(e).lower()


def _chunked_stage(src: Table, ops: list, session, nchunks: int) -> Table:
    """The stage over ``nchunks`` contiguous row ranges of its input, concatenated (re-plan after
    an out-of-memory attempt: each chunk's intermediates are 1/nchunks of the whole)."""
    import torch

    n = src.num_rows
    parts = []
    for c in range(nchunks):
        lo, hi = n * c // nchunks, n * (c + 1) // nchunks
        idx = torch.arange(lo, hi, dtype=torch.int64, device=src.device)
        parts.append(_run_stage(src.take(idx), ops, session))
        STATS["chunks"] += 1
    return Table.concat(parts)


def run_task(src: Table, ops: list, session) -> Table:
    """Execute one pending narrow stage as a task with retries: any RuntimeError of an attempt is
    retried up to spark.task.maxFailures attempts; after an out-of-memory error the next attempt
    runs the stage in twice as many row chunks (not for position-dependent stages)."""
    STATS["tasks"] += 1
    limit = max_failures(session)
    chunks = 1
    chunkable = not any(is_barrier(op[1].node if op[0] == "filter" else op[2].node)
                        for op in ops if op[0] in ("filter", "with"))
    for attempt in range(1, limit + 1):
        STATS["attempts"] += 1
        try:
            if _FAULTS["left"] > 0:
                _FAULTS["left"] -= 1
                raise TaskFailure(f"injected task failure (attempt {attempt})")
            if _FAULTS["oom"] > 0:
                _FAULTS["oom"] -= 1
                import torch

                raise torch.OutOfMemoryError(f"injected out-of-memory (attempt {attempt})")
            if chunks > 1:
                return _chunked_stage(src, ops, session, chunks)
            return _run_stage(src, ops, session)
        except RuntimeError as e:
            if attempt == limit:
                raise
            STATS["retries"] += 1
            if _is_oom(e) and chunkable and src.num_rows > chunks:
                chunks *= 2
                STATS["replans"] += 1
                import gc

                gc.collect()
                try:
                    import torch

                    if torch.cuda.is_available():
                        torch.cuda.empty_cache()
                except Exception:  # noqa: BLE001
                    pass
    raise TaskFailure("unreachable")


# ---------------------------------------------------------------------------------------------
# aggregation over a pending stage (the wide operation joins the lazy plan)
# ---------------------------------------------------------------------------------------------
def substitute(node, env: dict):
    """Replace column references by their defining expressions (``env``: lower-case name -> node)."""
    if isinstance(node, tuple):
        if node and node[0] == "col" and isinstance(node[1], str) and node[1].lower() in env:
            return env[node[1].lower()]
        return tuple(substitute(x, env) if isinstance(x, (tuple, list)) else x for x in node)
    if isinstance(node, list):
        return [substitute(x, env) if isinstance(x, (tuple, list)) else x for x in node]
    return node


_INLINE_KINDS = {"col", "lit", "bin", "un", "when", "cast", "alias"}


def _inlinable(node) -> bool:
    return all(n[0] in _INLINE_KINDS for n in _walk(node) if n)


class Inlined:
    """A pending stage rewritten over its source table: one predicate (or None) + the visible
    columns as expressions over the source."""

    def __init__(self, ops: list):
        from .column import strip_alias

        self.env: dict = {}
        self.visible: list | None = None  # None: source columns + 'with' columns
        conds = []
        for op in ops:
            if op[0] == "filter":
                conds.append(substitute(op[1].node, self.env))
            elif op[0] == "with":
                self.env[op[1].lower()] = substitute(strip_alias(op[2].node), self.env)
                if self.visible is not None and op[1] not in self.visible:
                    self.visible.append(op[1])
            else:  # select
                new = {}
                for name, c in op[1]:
                    new[name.lower()] = substitute(strip_alias(c.node), self.env)
                self.env = new
                self.visible = [name for name, _ in op[1]]
        self.cond = None
        for c in conds:
            self.cond = c if self.cond is None else ("bin", "&", self.cond, c)
        self.ok = all(_inlinable(n) for n in list(self.env.values()) + ([self.cond] if self.cond else []))

    def expr(self, node):
        return substitute(node, self.env)


def fusable(ops: list) -> bool:
    return bool(ops) and Inlined(ops).ok


def describe_fused_agg(ops: list, keys: list, aggs: list) -> str:
    """explain() text of an aggregation computed by fused_aggregate."""
    from .column import expr_name

    inl = Inlined(ops)
    fns = ", ".join(f"{fn}({expr_name(inl.expr(src.node)) if src is not None else '1'})" for _, fn, src in aggs)
    if keys:
        ks = ", ".join(expr_name(inl.expr(c.node)) for c in keys)
        leaves = sorted(referenced_columns(("k", [(inl.expr(c.node), ("lit", 0)) for c in keys]
                                            + [(inl.expr(src.node), ("lit", 0)) for _, _, src in aggs if src is not None])))
        lines = ["== Physical Plan (one fused scan, one task per executor) ==",
                 f"HashAggregate(keys=[{ks}], functions=[{fns}])  [partial -> shuffle -> final]",
                 f"+- Project [pruned: {', '.join(leaves)}]  -> 1 row gather of the pruned columns only"]
    else:
        lines = ["== Physical Plan (one fused scan, one task per executor) ==",
                 f"HashAggregate(keys=[], functions=[{fns}])  [masked reduction: no compaction, no row gather]"]
    if inl.cond is not None:
        lines.append(f"+- Filter [fused, projections inlined]: {expr_name(inl.cond)}  -> 1 expression-VM pass")
    lines.append("+- Scan (materialised source table)")
    return "\n".join(lines)


def describe(ops: list) -> str:
    """Physical plan of a pending narrow stage (DataFrame.explain)."""
    from .column import expr_name

    pushed, rest = optimize(ops)
    lines = ["== Physical Plan (narrow stage, one task per executor) =="]
    if pushed:
        lines.append("Filter [fused, pushed down]: " + " AND ".join(expr_name(op[1].node) for op in pushed)
                     + "  -> 1 expression-VM pass, 1 compaction, 1 row gather")
    for g in _groups(rest):
        if g[0] == "filters":
            lines.append("Filter [fused]: " + " AND ".join(expr_name(c.node) for c in g[1]))
        elif g[0] == "select":
            lines.append("Project [" + ", ".join(f"{n} = {expr_name(c.node)}" for n, c in g[1]) + "]")
        else:
            lines.append(f"Project {g[1]} = {expr_name(g[2].node)}")
    if len(lines) == 1:
        lines.append("Scan (materialised table, nothing pending)")
    return "\n".join(lines)
