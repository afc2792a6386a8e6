"""Executor-to-executor shuffle: Spark's shuffle write / block manager / shuffle read collapsed onto
RCCL all-to-all-v between the GPUs of one node (the reference's Spark workers move
these blocks over the pod network, spark_session.py:80-83 sizes their memory).

* one device-side count exchange (a single int64 all_to_all), never pickled;
* rows are gathered per destination straight from the source columns (no permuted copy of the
  whole table), in as many rounds as the staging budget requires — ``spark.ptg.shuffle.buffer.gb``
  (deploy/node.yaml) bounds the bytes staged per direction per round, and every rank runs the same
  number of rounds (one all-reduce MAX of the round count);
* received chunks land directly in their final place of the output columns.

:data:`STATS` records the peak staging of the last shuffle (tests assert it stays under budget).
"""
from __future__ import annotations

import math

import torch

from ..ops import df as D
from ..parallel import comm
from . import types as T
from .table import ColumnVector, Table
from .. import config

DEFAULT_BUDGET_GB = 64.0  # deploy/node.yaml spark.ptg.shuffle.buffer.gb
STATS: dict = {"peak_staging_bytes": 0, "rounds": 0, "count_exchanges": 0}


def budget_bytes() -> int:
    from .session import SparkSession

    s = SparkSession.getActiveSession()
    gb = float(config.get("shuffle_buffer_gb"))  # env / submitted conf / default
    if s is not None and config.source("shuffle_buffer_gb") not in ("cli", "env"):
        gb = float(s.conf.get("spark.ptg.shuffle.buffer.gb", gb))  # the active session's conf
    return max(1, int(gb * (1 << 30)))


def exchange_counts(send_counts: torch.Tensor) -> list:
    """send_counts int64[world] (rows this rank sends to each rank) -> rows it receives from each."""
    world = comm.world_size()
    dev = comm._ctl_device()
    sc = send_counts.to(device=dev, dtype=torch.int64).contiguous()
    rc = torch.empty(world, dtype=torch.int64, device=dev)
    torch.distributed.all_to_all_single(rc, sc)
    STATS["count_exchanges"] += 1
    return [int(x) for x in rc.cpu().tolist()]


def _row_bytes(cv: ColumnVector) -> int:
    return int(math.prod(cv.data.shape[1:])) * cv.data.element_size() + (1 if cv.valid is not None else 0)


def _unify_strings(t: Table) -> Table:
    from .readwriter import unify_dictionary

    cols = {}
    for n, cv in t.columns.items():
        cols[n] = unify_dictionary(cv) if isinstance(cv.dtype, T.StringType) else cv
    return Table(cols, t.num_rows, t.device)


def shuffle_table(t: Table, perm: torch.Tensor, counts: torch.Tensor, budget: int | None = None) -> Table:
    """Send rows ``perm[start_d : start_d + counts[d]]`` to rank d (perm groups rows by destination)
    and return the rows this rank receives, ordered by source rank."""
    world = comm.world_size()
    if world == 1:
        return t.take(perm)
    budget = budget or budget_bytes()
    t = _unify_strings(t)
    sc = [int(x) for x in counts.cpu().tolist()]
    rc = exchange_counts(counts)
    row_bytes = sum(_row_bytes(cv) for cv in t.columns.values()) or 1
    need = max(sum(sc), sum(rc)) * row_bytes
    rounds = max(1, math.ceil(need / budget))
    rounds = comm.all_reduce_int([rounds], op=torch.distributed.ReduceOp.MAX)[0]
    dev = t.device
    send_start = [sum(sc[:d]) for d in range(world)]
    recv_start = [sum(rc[:s]) for s in range(world)]
    n_out = sum(rc)
    out = {}
    for n, cv in t.columns.items():
        data = torch.empty((n_out, *cv.data.shape[1:]), dtype=cv.data.dtype, device=dev)
        valid = torch.empty(n_out, dtype=torch.uint8, device=dev) if cv.valid is not None else None
        out[n] = (data, valid)
    peak = 0
    for r in range(rounds):
        c = [sc[d] * (r + 1) // rounds - sc[d] * r // rounds for d in range(world)]
        q = [rc[s] * (r + 1) // rounds - rc[s] * r // rounds for s in range(world)]
        parts = [perm[send_start[d] + sc[d] * r // rounds: send_start[d] + sc[d] * r // rounds + c[d]]
                 for d in range(world)]
        idx = torch.cat(parts) if parts else perm[:0]
        for n, cv in t.columns.items():
            for src_t, dst_t in ((cv.data, out[n][0]), (cv.valid_u8(), out[n][1])):
                if src_t is None:
                    continue
                send = D.gather_rows(src_t.contiguous(), idx)
                recv = comm.all_to_all_v(send, c, q)
                peak = max(peak, send.numel() * send.element_size() + recv.numel() * recv.element_size())
                off = 0
                for s in range(world):
                    if q[s]:
                        o = recv_start[s] + rc[s] * r // rounds
                        dst_t[o: o + q[s]].copy_(recv[off: off + q[s]])
                    off += q[s]
                del send, recv
    STATS["peak_staging_bytes"] = peak
    STATS["rounds"] = rounds
    cols = {n: ColumnVector(out[n][0], cv.dtype, out[n][1], cv.dictionary) for n, cv in t.columns.items()}
    return Table(cols, n_out, dev)


def hash_shuffle(t: Table, key: torch.Tensor, budget: int | None = None) -> Table:
    """Hash-partition rows by an int64 key across ranks (groupBy / repartition(cols) / distinct)."""
    perm, counts = D.hash_partition(key, comm.world_size())
    return shuffle_table(t, perm, counts, budget)


def round_robin_shuffle(t: Table, budget: int | None = None) -> Table:
    """repartition(n) without columns: spread this rank's rows evenly over all ranks."""
    world = comm.world_size()
    n = t.num_rows
    part = (torch.arange(n, dtype=torch.int64, device=t.device) + comm.rank()) % world
    part = part.to(torch.int32)
    counts = torch.bincount(part.long(), minlength=world).to(torch.int64)
    perm = D.partition_perm(part, counts)
    return shuffle_table(t, perm, counts, budget)
