"""One groupBy(key).agg(sum, count) case for profiling: python tools/groupby_case.py [--sparse] [--keys N]
[--rows N] [--steps K].  Prints the bench JSON line (sql/bench_groupby.run)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from pyspark_tf_gke_amd.sql import bench_groupby as bg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--sparse", action="store_true")
ap.add_argument("--keys", type=int, default=1_000_000)
ap.add_argument("--rows", type=int, default=1_000_000_000)
ap.add_argument("--steps", type=int, default=3)
a = ap.parse_args()
print(json.dumps(bg.run(rows_per_gpu=a.rows, num_keys=a.keys, steps=a.steps, warmup=1, sparse=a.sparse)), flush=True)
