"""BASELINE config "raw-spark DataFrame groupBy-aggregate over 1B synthetic rows on 1 MI355X".

The DataFrame is ``(key bigint, value double)`` with ``rows_per_gpu`` rows resident in HBM on every
rank (weak scaling: 1B rows per GPU, 16 GB); keys are hash(row) % num_keys.  One timed step is the
full ``df.groupBy("key").agg(sum("value"), count("*"))`` through the DataFrame API: rank-local
radix-partitioned LDS aggregation -> hash shuffle of the partial aggregates over RCCL ->
final merge.  rows/s = total rows aggregated per second over all GPUs.
"""
from __future__ import annotations

import time

import torch

from ..parallel import comm


def run(total_rows: int = 1_000_000_000, num_keys: int = 1_000_000, steps: int = 5, warmup: int = 1, device=None,
        rows_per_gpu: int | None = None, sparse: bool = False) -> dict:
    """``sparse``: the same number of distinct keys spread over the whole int64 range (the general
    hash-partitioned path), instead of the dense [0, num_keys) range."""
    from ..ops import df as D
    from . import functions as F
    from .dataframe import DataFrame
    from .session import SparkSession
    from .table import ColumnVector, Table
    from . import types as T

    world, rank = comm.world_size(), comm.rank()
    n = rows_per_gpu or total_rows
    spark = SparkSession.builder.master("mi355x").getOrCreate()
    dev = spark.device if device is None else torch.device(device)
    keys, vals = D.fill_synthetic_kv(n, num_keys, dev, offset=rank * n, seed=42, sparse=sparse)
    df = DataFrame(Table({"key": ColumnVector(keys, T.LongType()), "value": ColumnVector(vals, T.DoubleType())}, n, dev),
                   spark)

    def step():
        return df.groupBy("key").agg(F.sum("value").alias("s"), F.count("*").alias("c"))

    out = None
    for _ in range(warmup):
        out = step()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    comm.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = step()
    if dev.type == "cuda":
        torch.cuda.synchronize()
    comm.barrier()
    dt = comm.all_reduce_max_scalar(time.perf_counter() - t0)
    groups = out.count()
    total_c = int(out._t.column("c").data.sum().item())
    if comm.distributed():
        total_c = int(comm.all_reduce_int([total_c])[0])
    ok = total_c == n * world
    # value checksums against the input columns (reduced by a different kernel, in another order):
    # sum over the groups of sum(value) == sum of every value; for dense keys also
    # sum over the groups of key * count == sum of every key; and with >= 50 rows per key the
    # number of groups is the number of distinct keys (P(a key is never drawn) ~ e^-50)
    s_out = float(out._t.column("s").data.double().sum().item())
    s_in = D.reduce_stats(vals, None, skip_nan=False)[0]
    kw_out = 0.0 if sparse else float((out._t.column("key").data.double() * out._t.column("c").data.double()).sum().item())
    kw_in = 0.0 if sparse else D.reduce_stats(keys, None, skip_nan=False)[0]
    s_out, s_in, kw_out, kw_in = comm.all_reduce_float([s_out, s_in, kw_out, kw_in])
    sums_ok = abs(s_out - s_in) <= 1e-9 * max(1.0, abs(s_in)) and abs(kw_out - kw_in) <= 1e-12 * max(1.0, abs(kw_in))
    groups_ok = groups == num_keys if n * world >= 50 * num_keys else None
    return {"metric": "rows/sec Spark groupBy-aggregate", "value": round(n * world * steps / dt, 1), "unit": "rows/s",
            "ms_per_step": round(dt / steps * 1e3, 3),
            "config": {"model": "groupBy(key).agg(sum(value), count(*)) on (bigint key, double value)",
                       "rows_per_gpu": n, "global_rows": n * world, "distinct_keys": num_keys, "groups_out": groups,
                       "keys": "sparse (spread over int64)" if sparse else "dense [0, distinct_keys)",
                       "counts_check": ok, "sums_check": bool(sums_ok), "groups_check": groups_ok,
                       "parallelism": f"{world} executors (1 per GPU), RCCL all-to-all-v shuffle"}}


def run_sort(rows_per_gpu: int = 1_000_000_000, steps: int = 3, warmup: int = 1, device=None,
             key_range: int = (1 << 63) - 1) -> dict:
    """``df.orderBy("key")`` over (bigint key, double value) rows resident in HBM: orderable-key
    prep, stable LSD radix sort of the significant key bits (8 passes for full-range int64 keys),
    row gather of both columns; world > 1 adds the sample-based range shuffle over RCCL.
    rows/s = total rows sorted per second over all GPUs."""
    from ..ops import df as D
    from .dataframe import DataFrame
    from .session import SparkSession
    from .table import ColumnVector, Table
    from . import types as T

    world, rank = comm.world_size(), comm.rank()
    n = rows_per_gpu
    spark = SparkSession.builder.master("mi355x").getOrCreate()
    dev = spark.device if device is None else torch.device(device)
    keys, vals = D.fill_synthetic_kv(n, key_range, dev, offset=rank * n, seed=7)
    df = DataFrame(Table({"key": ColumnVector(keys, T.LongType()), "value": ColumnVector(vals, T.DoubleType())}, n, dev),
                   spark)
    out = None
    for _ in range(warmup):
        out = df.orderBy("key")
        del out
    if dev.type == "cuda":
        torch.cuda.synchronize()
    comm.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = df.orderBy("key")
    if dev.type == "cuda":
        torch.cuda.synchronize()
    comm.barrier()
    dt = comm.all_reduce_max_scalar(time.perf_counter() - t0)
    k = out._t.column("key").data
    ok = bool((k[1:] >= k[:-1]).all().item()) if k.numel() > 1 else True
    ok = bool(comm.all_reduce_int([int(not ok)])[0] == 0)
    total = comm.all_reduce_int([out._t.num_rows])[0]
    return {"metric": "rows/sec Spark orderBy (sort)", "value": round(n * world * steps / dt, 1), "unit": "rows/s",
            "ms_per_step": round(dt / steps * 1e3, 3),
            "config": {"model": "orderBy(key) on (bigint key, double value), full-range random int64 keys",
                       "rows_per_gpu": n, "global_rows": n * world, "sorted_check": ok and total == n * world,
                       "parallelism": f"{world} executors (1 per GPU), range shuffle over RCCL"}}
