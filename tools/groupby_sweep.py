"""groupBy(key).agg(sum, count) over 1B rows by key cardinality, dense and sparse keys, one process:
python tools/groupby_sweep.py [--rows N] [--keys 1000,65536,...].  One JSON line per case
(sql/bench_groupby.run: counts checked against the row count, rows/s over the timed steps)."""
import argparse
import gc
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pyspark_tf_gke_amd.sql import bench_groupby as bg  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=1_000_000_000)
ap.add_argument("--keys", default="1000,65536,1000000,16000000,128000000")
ap.add_argument("--steps", type=int, default=3)
a = ap.parse_args()
for nk in [int(x) for x in a.keys.split(",")]:
    for sparse in (False, True):
        r = bg.run(rows_per_gpu=a.rows, num_keys=nk, steps=a.steps, warmup=1, sparse=sparse)
        print(json.dumps({"keys": nk, "kind": "sparse" if sparse else "dense", "G_rows_per_s": round(r["value"] / 1e9, 2),
                          "ms": r["ms_per_step"], "groups_out": r["config"].get("groups_out"),
                          "counts_check": r["config"].get("counts_check"), "sums_check": r["config"].get("sums_check"),
                          "groups_check": r["config"].get("groups_check")}), flush=True)
        gc.collect()
        torch.cuda.empty_cache()
