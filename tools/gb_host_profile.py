"""cProfile of one groupBy over synthetic keys (host-side time: syncs, allocations, Python):
python tools/gb_host_profile.py --keys 128000000 [--sparse]."""
import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pyspark_tf_gke_amd.ops import df as D  # noqa: E402
from pyspark_tf_gke_amd.sql import dataframe as DFM  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--keys", type=int, default=128_000_000)
ap.add_argument("--rows", type=int, default=1_000_000_000)
ap.add_argument("--sparse", action="store_true")
ap.add_argument("--full", action="store_true", help="profile the whole DataFrame groupBy().agg() step")
a = ap.parse_args()
k, v = D.fill_synthetic_kv(a.rows, a.keys, "cuda", sparse=a.sparse)
if a.full:
    from pyspark_tf_gke_amd.sql import functions as F
    from pyspark_tf_gke_amd.sql import types as T
    from pyspark_tf_gke_amd.sql.dataframe import DataFrame
    from pyspark_tf_gke_amd.sql.session import SparkSession
    from pyspark_tf_gke_amd.sql.table import ColumnVector, Table

    spark = SparkSession.builder.master("mi355x").getOrCreate()
    df = DataFrame(Table({"key": ColumnVector(k, T.LongType()), "value": ColumnVector(v, T.DoubleType())}, k.numel(),
                         k.device), spark)

    def step():
        return df.groupBy("key").agg(F.sum("value").alias("s"), F.count("*").alias("c"))
else:
    def step():
        return DFM._hash_agg_all(k, [v], [None], False)
step()  # warm-up
torch.cuda.synchronize()
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
out = step()
torch.cuda.synchronize()
pr.disable()
print(f"wall {1e3 * (time.perf_counter() - t0):.1f} ms", flush=True)
pstats.Stats(pr).sort_stats("cumulative").print_stats(40)
