"""Executor-to-executor shuffle: Spark's shuffle write / block manager / shuffle read collapsed onto
RCCL all-to-all-v between the GPUs of one node (the reference's Spark workers move
these blocks over the pod network, spark_session.py:80-83 sizes their memory).

* one device-side count exchange (a single int64 all-gather of every rank's count vector, so every
  rank knows the whole count matrix and the round count without another collective), never pickled;
* rows are gathered per destination straight from the source columns (no permuted copy of the
  whole table), in as many rounds as the staging budget requires — ``spark.ptg.shuffle.buffer.gb``
  (deploy/node.yaml) bounds the bytes staged per direction per round, and every rank runs the same
  number of rounds (one all-reduce MAX of the round count);
* every column and validity mask of a round goes out in one grouped point-to-point launch, and the
  backend writes each received chunk straight into its final slice of the output column (no
  receive staging, no copy after the collective); a rank's own rows are gathered into place;
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


def count_matrix(send_counts) -> list:
    """Every rank's send counts (int64[world], on the device or host) -> the full matrix
    M[src][dst] of rows, identical on every rank: ONE all-gather of the count vectors and ONE
    device-to-host copy.  Rank r receives column r; every rank derives the same round count."""
    world = comm.world_size()
    dev = comm._ctl_device()
    if isinstance(send_counts, torch.Tensor):
        sc = send_counts.to(device=dev, dtype=torch.int64).contiguous()
    else:
        sc = torch.tensor([int(x) for x in send_counts], dtype=torch.int64, device=dev)
    mat = torch.empty(world * world, dtype=torch.int64, device=dev)
    torch.distributed.all_gather_into_tensor(mat, sc)
    STATS["count_exchanges"] += 1
    flat = mat.cpu().tolist()
    return [flat[s * world:(s + 1) * world] for s in range(world)]


def exchange_counts(send_counts: torch.Tensor) -> list:
    """send_counts int64[world] (rows this rank sends to each rank) -> rows it receives from each."""
    m = count_matrix(send_counts)
    return [m[s][comm.rank()] for s in range(comm.world_size())]


def _row_bytes(cv: ColumnVector) -> int:
    return int(math.prod(cv.data.shape[1:])) * cv.data.element_size() + (1 if cv.valid is not None else 0)


def _unify_strings(t: Table) -> Table:
    from .readwriter import unify_dictionary

    cols = {}
    for n, cv in t.columns.items():
        cols[n] = unify_dictionary(cv) if isinstance(cv.dtype, T.StringType) else cv
    return Table(cols, t.num_rows, t.device)


def _seg_range(segs: list, lo: int, hi: int) -> list:
    """Views of the index segments ``segs`` (concatenated) covering positions [lo, hi)."""
    out, base = [], 0
    for sg in segs:
        n = sg.numel()
        a, b = max(lo, base), min(hi, base + n)
        if a < b:
            out.append(sg[a - base:b - base])
        base += n
        if base >= hi:
            break
    return out


def shuffle_table(t: Table, perm: torch.Tensor, counts, budget: int | None = None) -> Table:
    """Send rows ``perm[start_d : start_d + counts[d]]`` to rank d (perm groups rows by destination)
    and return the rows this rank receives, ordered by source rank."""
    if not comm.distributed():
        return t.take(perm)
    world = comm.world_size()
    mat = count_matrix(counts)
    sc = mat[comm.rank()]
    starts = [sum(sc[:d]) for d in range(world)]
    segs = [[perm[starts[d]:starts[d] + sc[d]]] for d in range(world)]
    return exchange(t, segs, mat, budget)


def exchange(t: Table, segs: list, mat: list, budget: int | None = None) -> Table:
    """The shuffle proper.  ``segs[d]``: index tensors (views) of the rows this rank sends to rank d,
    in order; ``mat``: the count matrix of :func:`count_matrix` (every rank's sends).

    Per round, every column and validity mask goes out in ONE grouped point-to-point launch
    (``batch_isend_irecv``: RCCL runs a round's sends and receives as one ncclGroup); each received
    chunk is written by the backend straight into its final slice of the output column (rows from
    source s at ``sum(rc[:s]) + rc[s] * r // rounds``), and this rank's own rows are gathered
    directly into theirs — no receive staging and no copy after the collective.  The only staging
    is the per-destination send gather, bounded by the budget per round."""
    world, rank = comm.world_size(), comm.rank()
    budget = budget or budget_bytes()
    t = _unify_strings(t)
    sc = mat[rank]
    rc = [mat[s][rank] for s in range(world)]
    row_bytes = sum(_row_bytes(cv) for cv in t.columns.values()) or 1
    # every rank computes the same round count from the same matrix (no extra collective)
    need = max(max(sum(mat[r]), sum(mat[s][r] for s in range(world))) for r in range(world)) * row_bytes
    rounds = max(1, math.ceil(need / budget))
    dev = t.device
    recv_start = [sum(rc[:s]) for s in range(world)]
    n_out = sum(rc)
    out, srcs = {}, []
    for n, cv in t.columns.items():
        data = torch.empty((n_out, *cv.data.shape[1:]), dtype=cv.data.dtype, device=dev)
        valid = torch.empty(n_out, dtype=torch.uint8, device=dev) if cv.valid is not None else None
        out[n] = (data, valid)
        srcs.append((cv.data.contiguous(), data))
        if valid is not None:
            srcs.append((cv.valid_u8().contiguous(), valid))
    peak = 0
    for r in range(rounds):
        ops, keep, staged = [], [], 0
        for d in range(world):
            lo, hi = sc[d] * r // rounds, sc[d] * (r + 1) // rounds
            s_lo, s_hi = rc[d] * r // rounds, rc[d] * (r + 1) // rounds
            parts = _seg_range(segs[d], lo, hi) if hi > lo else []
            for src, dst in srcs:
                if d == rank:
                    o = recv_start[d] + lo
                    for pt in parts:  # own rows: gathered straight into their output slice
                        D.gather_rows(src, pt, out=dst[o:o + pt.numel()])
                        o += pt.numel()
                    continue
                if hi > lo:
                    if len(parts) == 1:
                        buf = D.gather_rows(src, parts[0])
                    else:
                        buf = torch.empty((hi - lo, *src.shape[1:]), dtype=src.dtype, device=src.device)
                        o = 0
                        for pt in parts:
                            D.gather_rows(src, pt, out=buf[o:o + pt.numel()])
                            o += pt.numel()
                    keep.append(buf)
                    staged += buf.numel() * buf.element_size()
                    ops.append(torch.distributed.P2POp(torch.distributed.isend, buf, d))
                if s_hi > s_lo:
                    o = recv_start[d] + s_lo
                    ops.append(torch.distributed.P2POp(torch.distributed.irecv, dst[o:o + (s_hi - s_lo)], d))
        if ops:
            for req in torch.distributed.batch_isend_irecv(ops):
                req.wait()
        peak = max(peak, staged)
        del keep
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
            n_d, segs = 0, []
            for rr in g:
                b = rr * world + d
                if b < nbuckets and ch[b]:
                    segs.append(perm[starts[b]: starts[b] + ch[b]])
                    n_d += ch[b]
            sel.append(segs)
            sc.append(n_d)
        out = exchange(t, sel, count_matrix(sc), budget)
        peak = max(peak, STATS["peak_staging_bytes"])
        STATS["reduce_tasks"] += 1
        mine = [rr * world + rank for rr in g if rr * world + rank < nbuckets]
        if mine:
            yield mine, out
    STATS["peak_staging_bytes"] = peak
    STATS["buckets"] = nbuckets
    STATS["rounds"] = len(groups)
