"""Time the DataFrame expression kernels over --rows synthetic rows: the specialised single-column
kernels (expr_affine_k) vs the expression VM (PTG_EXPR_SPECIALIZE=0), per expression, and the HBM
rate over the bytes each must move (input column + output column + validity bytes)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pyspark_tf_gke_amd.ops import df as D  # noqa: E402
from pyspark_tf_gke_amd.sql import SparkSession, types as T  # noqa: E402
from pyspark_tf_gke_amd.sql.dataframe import DataFrame  # noqa: E402
from pyspark_tf_gke_amd.sql.functions import col  # noqa: E402
from pyspark_tf_gke_amd.sql.table import ColumnVector, Table  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=200_000_000)
ap.add_argument("--reps", type=int, default=5)
a = ap.parse_args()
spark = SparkSession.builder.master("local[1]").config("spark.ptg.device", "cuda").getOrCreate()
k, v = D.fill_synthetic_kv(a.rows, 1000, "cuda")
df = DataFrame(Table({"k": ColumnVector(k, T.LongType()), "v": ColumnVector(v, T.DoubleType())}, a.rows,
                     k.device), spark)
exprs = {"(v*4).cast(int)": ((col("v") * 4).cast("int"), 8 + 4 + 1), "v + 1.5": (col("v") + 1.5, 8 + 8 + 1),
         "k * 3": (col("k") * 3, 8 + 8 + 1), "v > 0.5 (filter mask)": (col("v") > 0.5, 8 + 1 + 1)}
for name, (e, bpr) in exprs.items():
    res = {"expr": name, "rows": a.rows}
    for flag in ("1", "0"):
        os.environ["PTG_EXPR_SPECIALIZE"] = flag
        best = None
        for _ in range(a.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = df.select(e.alias("o"))
            out._t.column("o").data
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        tag = "specialised" if flag == "1" else "vm"
        res[f"{tag}_ms"] = round(best * 1e3, 3)
        res[f"{tag}_TBs"] = round(bpr * a.rows / best / 1e12, 2)
    print(json.dumps(res), flush=True)
