"""Executor loss (Spark standalone's lost-executor handling): a rank of a 3-executor
DataFrame job dies mid-job; the launcher (``--min-nproc``) drops that executor and restarts the job
on the 2 survivors.  The CSV source is split by (rank, world) at read time, so the lost executor's
partitions are re-assigned and recomputed from their lineage (read -> filter -> withColumn ->
groupBy/agg -> write).  The Parquet output equals a single-process pandas run of the same query."""
import json
import os
import subprocess
import sys
import textwrap

import numpy as np
import pandas as pd

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

JOB = """
import json, os, sys
from pyspark_tf_gke_amd.sql import SparkSession
from pyspark_tf_gke_amd.sql import functions as F
from pyspark_tf_gke_amd.parallel import comm
from pyspark_tf_gke_amd.runtime import fault
src, out = sys.argv[1], sys.argv[2]
spark = SparkSession.builder.master("mi355x").appName("loss").getOrCreate()
df = spark.read.csv(src, header=True, inferSchema=True)
df = df.filter(F.col("v") > 0.1).withColumn("w", F.col("v") * 2.0)
fault.maybe_fail()  # PTG_FAULT_RANK dies here on the first attempt, after its read
agg = df.groupBy("k").agg(F.sum("w").alias("s"), F.count("*").alias("c"))
agg.write.mode("overwrite").parquet(out)
if comm.rank() == 0:
    print("RESULT", json.dumps({"world": comm.world_size(), "lost": os.environ.get("PTG_LOST_EXECUTORS", "")}),
          flush=True)
"""


def test_lost_executor_partitions_recomputed_on_survivors(tmp_path):
    rng = np.random.default_rng(3)
    n = 3000
    pdf = pd.DataFrame({"k": rng.integers(0, 37, n), "v": rng.random(n)})
    src = tmp_path / "in.csv"
    pdf.to_csv(src, index=False)
    out = tmp_path / "out"
    env = dict(os.environ)
    env.update({"PYTHONPATH": ROOT + os.pathsep + env.get("PYTHONPATH", ""), "PTG_DEVICE": "cpu",
                "PTG_HOST_FP32": "1", "PTG_FAULT_RANK": "2", "PTG_FAULT_STEP": "1", "PTG_PG_TIMEOUT": "60"})
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-m", "pyspark_tf_gke_amd.runtime.launcher", "--nproc", "3", "--max-restarts", "1",
           "--min-nproc", "2", "--", sys.executable, "-c", textwrap.dedent(JOB), str(src), str(out)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "executor 2 lost" in r.stderr, r.stderr[-2000:]
    res = [json.loads(line.split("RESULT ", 1)[1]) for line in r.stdout.splitlines() if "RESULT " in line]
    assert res == [{"world": 2, "lost": "2"}], r.stdout[-2000:]
    got = pd.read_parquet(out).sort_values("k").reset_index(drop=True)
    ref = pdf[pdf.v > 0.1].assign(w=lambda d: d.v * 2.0).groupby("k").agg(s=("w", "sum"), c=("w", "size"))
    ref = ref.reset_index().sort_values("k").reset_index(drop=True)
    assert list(got.k) == list(ref.k)
    assert np.allclose(got.s.to_numpy(), ref.s.to_numpy(), rtol=1e-12)
    assert list(got.c) == list(ref.c)
