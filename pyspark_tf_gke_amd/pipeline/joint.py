"""BASELINE.json config "Joint pipeline: Spark ETL -> Parquet -> TF train, 8 executors + 8 workers on
one 8xMI355X node".

Not in the reference as one program: the reference runs its Spark workloads (k_means.py, the JDBC
readers) and its TF trainer (train_tf_ps.py) as separate jobs on separate GKE node pools
(SURVEY.md §1, §7.1 Tier B).  Here every rank is BOTH a Spark executor and a TF worker on the same
GPU:

1. **ETL** (DataFrame API, device-resident columns): a synthetic health-records source shaped like
   the reference's ``health.csv`` rows (``measure_code``, ``value``, ``lower_ci``, ``upper_ci`` with
   missing values) is generated with ``spark.range`` + ``rand``; nulls are filtered / mean-imputed
   exactly like ``k_means.py:45-51``; a 15-class label (the reference MLP's ``subpopulation`` target,
   train_tf_ps.py:107-147) is derived; features are standardised with global (all-reduced)
   mean/stddev aggregates.
2. **Parquet**: ``df.write.parquet`` writes one rank-sharded part file per executor (``_SUCCESS``
   marker, snappy), the BASELINE-required hand-off format.
3. **Train**: every rank reads its Parquet shard (``spark.read.parquet`` assigns files to ranks),
   moves the columns to the GPU and trains the reference's CSV MLP (``build_deep_model``,
   train_tf_ps.py:328-343) with MultiWorkerMirroredStrategy (RCCL all-reduce) through the
   columnar ``Dataset`` fast path (shuffle/batch gathered on the device).  ``handoff="device"``
   additionally skips the Parquet read-back and trains straight from the ETL's device columns.
Artifacts: ``<out>/etl.parquet/``, ``<out>/model.keras``, ``<out>/saved_model/``, ``<out>/history.json``,
``<out>/label_map.json``, ``<out>/joint_report.json``.
"""
from __future__ import annotations

import json
import os
import time

import torch

from ..parallel import comm

NUM_CLASSES = 15
FEATURES = ("value", "lower_ci", "upper_ci")


def _sync(dev):
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


def etl(spark, rows_per_executor: int, seed: int = 7):
    """Synthetic source -> cleaned, standardised (f0, f1, f2, label) DataFrame (rank-local rows)."""
    from ..sql import functions as F

    world = comm.world_size()
    df = spark.range(rows_per_executor * world)
    df = (df.withColumn("measure_code", (F.col("id") % 30).cast("int"))
            .withColumn("value", F.rand(seed) * 100.0)
            .withColumn("lower_ci", F.col("value") - F.rand(seed + 1) * 10.0)
            .withColumn("upper_ci", F.col("value") + F.rand(seed + 2) * 10.0)
            .withColumn("value", F.when(F.rand(seed + 3) < 0.02, F.lit(None)).otherwise(F.col("value")))
            .withColumn("lower_ci", F.when(F.rand(seed + 4) < 0.05, F.lit(None)).otherwise(F.col("lower_ci"))))
    # k_means.py:23-28 style null filtering on the key measure, :45-51 mean imputation
    df = df.filter(F.col("value").isNotNull())
    for c in ("lower_ci", "upper_ci"):
        mean = df.select(c).agg(F.avg(c).alias("m")).collect()[0]["m"]
        df = df.withColumn(c, F.when(F.col(c).isNull() | F.isnan(F.col(c)), F.lit(float(mean))).otherwise(F.col(c)))
    # 15-class target: a deterministic band of the value (plus measure-dependent shift), learnable
    # from the three features like the reference's subpopulation labels
    df = df.withColumn("label", ((F.col("value") * 0.15 + (F.col("measure_code") % 3).cast("double") * 0.2)
                                 .cast("int") % NUM_CLASSES).cast("int"))
    stats = df.agg(*[F.avg(c).alias(f"{c}_mu") for c in FEATURES],
                   *[F.stddev(c).alias(f"{c}_sd") for c in FEATURES]).collect()[0]
    cols = []
    for i, c in enumerate(FEATURES):
        mu, sd = float(stats[f"{c}_mu"]), float(stats[f"{c}_sd"]) or 1.0
        cols.append(((F.col(c) - mu) / sd).cast("float").alias(f"f{i}"))
    return df.select(*cols, F.col("label"))


def _to_device_tensors(df, device):
    t = df._t
    x = torch.stack([t.column(f"f{i}").data.to(device, torch.float32) for i in range(len(FEATURES))], 1)
    y = t.column("label").data.to(device, torch.int32)
    return x.contiguous(), y.contiguous()


def run_joint(rows_per_executor: int = 1_000_000, out_dir: str = "./joint-out", epochs: int = 2,
              batch_size: int = 4096, handoff: str = "parquet", master: str = "mi355x", seed: int = 7,
              verbose: bool = True) -> dict:
    from .. import distribute as ds
    from ..data import Dataset
    from ..models import build_deep_model
    from ..sql import SparkSession

    spark = SparkSession.builder.appName("JointETLTrain").master(master).getOrCreate()
    dev = spark.device
    rank, world = comm.rank(), comm.world_size()
    t_all = time.perf_counter()

    # ---- 1+2. ETL and Parquet
    _sync(dev)
    comm.barrier()
    t0 = time.perf_counter()
    clean = etl(spark, rows_per_executor, seed)
    n_local = clean.count() if world == 1 else clean._t.num_rows
    pq_path = os.path.join(out_dir, "etl.parquet")
    clean.write.mode("overwrite").parquet(pq_path)
    _sync(dev)
    comm.barrier()
    etl_s = comm.all_reduce_max_scalar(time.perf_counter() - t0)
    n_total = int(comm.all_reduce_int([int(n_local)])[0]) if world > 1 else int(n_local)
    pq_bytes = sum(os.path.getsize(os.path.join(pq_path, f)) for f in os.listdir(pq_path) if f.endswith(".parquet"))

    # ---- 3. train
    if handoff == "parquet":
        train_df = spark.read.parquet(pq_path)
    elif handoff == "device":
        train_df = clean
    else:
        raise ValueError("handoff must be 'parquet' or 'device'")
    strategy = ds.MultiWorkerMirroredStrategy()
    x, y = _to_device_tensors(train_df, strategy.device)
    n_train = x.shape[0]
    steps = max(1, n_train // batch_size)
    steps = int(min(comm.all_gather_int(steps))) if world > 1 else steps  # lock-step collectives
    ds_train = Dataset.from_tensor_slices((x, y)).shuffle(n_train, seed=seed + rank).batch(
        batch_size, drop_remainder=True).repeat().prefetch(1)
    with strategy.scope():
        model = build_deep_model(len(FEATURES), NUM_CLASSES)
    _sync(strategy.device)
    comm.barrier()
    t1 = time.perf_counter()
    hist = model.fit(ds_train, epochs=epochs, steps_per_epoch=steps, verbose=1 if (verbose and rank == 0) else 0)
    _sync(strategy.device)
    comm.barrier()
    train_s = comm.all_reduce_max_scalar(time.perf_counter() - t1)
    samples = steps * epochs * batch_size * world

    report = {"rows_generated": rows_per_executor * world, "rows_after_etl": n_total, "etl_seconds": round(etl_s, 4),
              "etl_rows_per_s": round(rows_per_executor * world / etl_s, 1), "parquet_path": pq_path,
              "parquet_bytes_rank0_view": pq_bytes, "handoff": handoff, "train_samples": samples,
              "train_seconds": round(train_s, 4), "train_samples_per_s": round(samples / train_s, 1),
              "epochs": epochs, "batch_per_worker": batch_size, "executors": world, "workers": world,
              "final": {k: float(v[-1]) for k, v in hist.history.items()},
              "wall_seconds": round(time.perf_counter() - t_all, 3)}
    if rank == 0:
        model.save(os.path.join(out_dir, "model.keras"))
        model.export(os.path.join(out_dir, "saved_model"),
                     assets={"label_map.json": {f"class_{i}": i for i in range(NUM_CLASSES)}})
        with open(os.path.join(out_dir, "history.json"), "w") as fh:
            json.dump({k: [float(v) for v in vs] for k, vs in hist.history.items()}, fh)
        with open(os.path.join(out_dir, "label_map.json"), "w") as fh:
            json.dump({f"class_{i}": i for i in range(NUM_CLASSES)}, fh)
        with open(os.path.join(out_dir, "joint_report.json"), "w") as fh:
            json.dump(report, fh, indent=2)
    comm.barrier()
    return report
