"""Executor-to-executor shuffle: Spark's shuffle write / block manager / shuffle read collapsed onto
RCCL all-to-all-v between the GPUs of one node (the reference's Spark workers move
these blocks over the pod network, spark_session.py:80-83 sizes their memory).

* one device-side count exchange (a single int64 all_to_all), never pickled;
* rows are gathered per destination straight from the source columns (no permuted copy of the
  whole table), in as many rounds as the staging budget requires — ``spark.ptg.shuffle.buffer.gb``
  (deploy/node.yaml) bounds the bytes staged per direction per round, and every rank runs the same
  number of rounds (one all-reduce MAX of the round count);
* received chunks land directly in their final place of the output columns;
* ``spark.sql.shuffle.partitions`` (spark_installation_check.py:16) is the number of hash buckets of
  a keyed shuffle (:func:`bucket_exchange`): bucket b belongs to rank b % world and the exchange
  runs one reduce partition per round (round r moves bucket r * world + d to rank d), so each round
  stages ~1/buckets of the data and the consumer runs one reduce task per received bucket.

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
STATS: dict = {"peak_staging_bytes": 0, "rounds": 0, "count_exchanges": 0, "buckets": 0, "reduce_tasks": 0}


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
    if not comm.distributed():
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
    rank = comm.rank()
    # row i -> (i + rank) % world; the counts follow in closed form (no histogram pass)
    counts = torch.tensor([(n - ((p - rank) % world) + world - 1) // world for p in range(world)], dtype=torch.int64)
    if t.device.type == "cuda":
        part = D.rr_part(n, rank, world, t.device)
        counts = counts.to(t.device)
    else:
        part = ((torch.arange(n, dtype=torch.int64) + rank) % world).to(torch.int32)
    perm = D.partition_perm(part, counts)
    return shuffle_table(t, perm, counts, budget)


def shuffle_partitions(default: int = 200) -> int:
    """``spark.sql.shuffle.partitions`` of the active session (Spark's default 200)."""
    from .session import SparkSession

    sess = SparkSession.getActiveSession()
    try:
        return max(1, int(getattr(sess, "shuffle_partitions", default) if sess is not None else default))
    except (TypeError, ValueError):
        return default


def _aqe_advisory_bytes() -> int:
    """Adaptive coalescing of small shuffle partitions (Spark 3's ``spark.sql.adaptive.enabled``,
    default on, ``spark.sql.adaptive.advisoryPartitionSizeInBytes`` default 64 MB): 0 = off."""
    from .session import SparkSession

    sess = SparkSession.getActiveSession()
    conf = sess.conf if sess is not None else None
    get = (lambda k, d: conf.get(k, d)) if conf is not None else (lambda k, d: d)
    if str(get("spark.sql.adaptive.enabled", "true")).lower() in ("false", "0", "no"):
        return 0
    if str(get("spark.sql.adaptive.coalescePartitions.enabled", "true")).lower() in ("false", "0", "no"):
        return 0
    raw = str(get("spark.sql.adaptive.advisoryPartitionSizeInBytes", str(64 << 20))).strip().lower()
    mult = {"k": 1 << 10, "kb": 1 << 10, "m": 1 << 20, "mb": 1 << 20, "g": 1 << 30, "gb": 1 << 30}
    for suf in ("kb", "mb", "gb", "k", "m", "g"):
        if raw.endswith(suf):
            return int(float(raw[: -len(suf)]) * mult[suf])
    return int(float(raw))


def bucket_exchange(t: Table, key: torch.Tensor, nbuckets: int, budget: int | None = None, coalesce: bool = True):
    """Keyed shuffle in ``nbuckets`` hash buckets: bucket b belongs to rank b % world; yields
    ``(buckets, rows of those buckets from every rank)`` per reduce task of this rank, in bucket
    order.  A reduce round moves bucket-round rr (buckets rr * world + d to rank d); with adaptive
    coalescing on, consecutive bucket-rounds are merged until a round holds the advisory partition
    size (one reduce task then reads several buckets, as Spark's coalesced shuffle partitions do).
    Collective: every rank iterates the generator to the end."""
    world, rank = comm.world_size(), comm.rank()
    perm, counts = D.hash_partition(key, nbuckets)
    ch = [int(x) for x in counts.cpu().tolist()]
    starts = [0] * nbuckets
    for b in range(1, nbuckets):
        starts[b] = starts[b - 1] + ch[b - 1]
    nrr = -(-nbuckets // world)
    row_bytes = sum(_row_bytes(cv) for cv in t.columns.values()) or 1
    advisory = _aqe_advisory_bytes() if coalesce else 0
    if advisory > 0 and nrr > 1:
        glob = comm.all_reduce_int(ch)  # global rows per bucket (one collective, tensors)
        per_rr = [sum(glob[rr * world + d] for d in range(world) if rr * world + d < nbuckets) * row_bytes
                  for rr in range(nrr)]
        groups, cur, acc = [], [], 0
        for rr in range(nrr):
            cur.append(rr)
            acc += per_rr[rr]
            if acc >= advisory:
                groups.append(cur)
                cur, acc = [], 0
        if cur:
            groups.append(cur)
    else:
        groups = [[rr] for rr in range(nrr)]
    peak = 0
    for g in groups:
        sel, sc = [], []
        for d in range(world):
            n_d = 0
            for rr in g:
                b = rr * world + d
                if b < nbuckets and ch[b]:
                    sel.append(perm[starts[b]: starts[b] + ch[b]])
                    n_d += ch[b]
            sc.append(n_d)
        idx = torch.cat(sel) if sel else perm[:0]
        out = shuffle_table(t, idx, torch.tensor(sc, dtype=torch.int64), budget)
        peak = max(peak, STATS["peak_staging_bytes"])
        STATS["reduce_tasks"] += 1
        mine = [rr * world + rank for rr in g if rr * world + rank < nbuckets]
        if mine:
            yield mine, out
    STATS["peak_staging_bytes"] = peak
    STATS["buckets"] = nbuckets
    STATS["rounds"] = len(groups)
