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

The stage runs as a *task* with Spark's retry semantics (``spark.task.maxFailures``, default 4):
a narrow stage is rank-local (no collective inside), so a failed attempt is simply re-run from
its resident input.  ``PTG_FAULT_TASK=k`` makes the first k task attempts of the process fail
(fault-injection for the retry tests).  ``DataFrame.explain()`` prints the optimised stage.
"""
from __future__ import annotations

import os

from .column import Column
from .table import Table

_BARRIER_LEAVES = ("rand", "rowid")
STATS = {"tasks": 0, "attempts": 0, "retries": 0, "vm_passes": 0, "gathers": 0}
_FAULTS = {"left": int(os.environ.get("PTG_FAULT_TASK", "0") or 0)}


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
            t = t.take(idx)
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


def run_task(src: Table, ops: list, session) -> Table:
    """Execute one pending narrow stage as a task with retries."""
    STATS["tasks"] += 1
    limit = max_failures(session)
    for attempt in range(1, limit + 1):
        STATS["attempts"] += 1
        try:
            if _FAULTS["left"] > 0:
                _FAULTS["left"] -= 1
                raise TaskFailure(f"injected task failure (attempt {attempt})")
            return _run_stage(src, ops, session)
        except TaskFailure:
            if attempt == limit:
                raise
            STATS["retries"] += 1
    raise TaskFailure("unreachable")


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
        else:
            lines.append(f"Project {g[1]} = {expr_name(g[2].node)}")
    if len(lines) == 1:
        lines.append("Scan (materialised table, nothing pending)")
    return "\n".join(lines)
