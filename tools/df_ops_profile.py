"""The DataFrame operators of the verdict's "own kernels only" check, for a rocprofv3 kernel trace:

  * groupBy("measure_name", "subpopulation").agg(...) on the reference's health.csv (a nullable
    string key: 1,508 empty `subpopulation` values), countDistinct, dropDuplicates / distinct;
  * a two-column groupBy over --rows synthetic rows (key = hash(row) % --keys, second key column
    an expression of the value column), timed.

Run under ``rocprofv3 --kernel-trace --stats`` and list the kernels with tools/prof_summary.py; the
query sections are bracketed by torch.cuda.synchronize() so the setup kernels (CSV upload, the
synthetic data fill) are easy to tell apart.  Prints one JSON line per query."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=1_000_000_000)
ap.add_argument("--keys", type=int, default=1_000_000)
ap.add_argument("--reps", type=int, default=3)
a = ap.parse_args()

from pyspark_tf_gke_amd.ops import df as D  # noqa: E402
from pyspark_tf_gke_amd.sql import SparkSession  # noqa: E402
from pyspark_tf_gke_amd.sql.functions import avg, col, count, countDistinct, max as fmax, sum as fsum  # noqa: E402
from pyspark_tf_gke_amd.sql.table import ColumnVector, Table  # noqa: E402
from pyspark_tf_gke_amd.sql import types as T  # noqa: E402

spark = SparkSession.builder.master("local[1]").config("spark.ptg.device", "cuda").getOrCreate()
HEALTH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "data", "health.csv")
df = spark.read.csv(HEALTH, header=True, inferSchema=True)
df.count()
torch.cuda.synchronize()


def timed(name, fn):
    best = None
    out = None
    for _ in range(a.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    print(json.dumps({"query": name, "ms": round(best * 1e3, 3), "result": out}), flush=True)


timed("health groupBy(measure_name, subpopulation).agg(count, avg, sum, max)",
      lambda: len(df.groupBy("measure_name", "subpopulation").agg(
          count("*").alias("n"), avg("value").alias("m"), fsum("value").alias("s"),
          fmax("upper_ci").alias("hi")).collect()))
timed("health countDistinct(subpopulation, value, state_name)",
      lambda: list(df.agg(countDistinct("subpopulation"), countDistinct("value"),
                          countDistinct("state_name")).collect()[0]))
timed("health dropDuplicates(measure_name, subpopulation)",
      lambda: len(df.dropDuplicates(["measure_name", "subpopulation"]).collect()))
timed("health select(measure_name, state_name).distinct().count()",
      lambda: df.select("measure_name", "state_name").distinct().count())

if a.rows:
    k, v = D.fill_synthetic_kv(a.rows, a.keys, "cuda")
    from pyspark_tf_gke_amd.sql.dataframe import DataFrame

    big = DataFrame(Table({"k": ColumnVector(k, T.LongType()), "v": ColumnVector(v, T.DoubleType())}, a.rows,
                          k.device), spark)
    torch.cuda.synchronize()
    timed(f"{a.rows} rows groupBy(k, int(v * 4)).agg(count, sum)",
          lambda: big.groupBy(col("k"), (col("v") * 4).cast("int").alias("b")).agg(
              count("*").alias("n"), fsum("v").alias("s")).count())
