"""BASELINE config "raw-spark DataFrame groupBy-aggregate over 1B synthetic rows on 1 MI355X".

Runs ``df.groupBy("key").agg(sum("value"), count("*"))`` over ``--rows`` synthetic (bigint, double)
rows per executor GPU (see pyspark_tf_gke_amd/sql/bench_groupby.py); launch N executors with
``python -m pyspark_tf_gke_amd.cli.spark_submit --num-executors N workloads/raw-spark/groupby_agg.py``.
"""
import argparse
import json

import _path  # noqa: F401

from pyspark_tf_gke_amd.parallel import comm
from pyspark_tf_gke_amd.sql.bench_groupby import run


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000_000, help="rows per executor")
    ap.add_argument("--keys", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--device", default=None)
    a = ap.parse_args(argv)
    res = run(rows_per_gpu=a.rows, num_keys=a.keys, steps=a.steps, warmup=a.warmup, device=a.device)
    if comm.rank() == 0:
        print(json.dumps(res))


if __name__ == "__main__":
    main()
