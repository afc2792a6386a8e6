"""BASELINE config "raw-spark wordcount on local[2] PySpark CPU (plumbing, no GPU)".

Classic RDD wordcount (textFile -> flatMap(split) -> map((w, 1)) -> reduceByKey(add) -> sortBy count)
on a ``local[2]`` session, cross-checked against the fused native C++ counter (csrc/host/csv.cpp,
``ptgh_word_count``).  Input: a text file, or ``--synthetic-mb`` of generated text.

    python workloads/raw-spark/wordcount.py [--input FILE] [--synthetic-mb 8] [--top 10]
"""
import argparse
import json
import operator
import os
import random
import tempfile
import time

import _path  # noqa: F401

from pyspark_tf_gke_amd.sql import SparkSession
from pyspark_tf_gke_amd.sql.rdd import word_count_native

WORDS = ("spark tensorflow kubernetes mi355x executor worker shuffle partition gradient parameter server "
         "cluster node pod driver dataframe column kernel wave lds hbm xgmi rccl").split()


def synthetic_text(mb: float, seed: int = 0) -> str:
    rng = random.Random(seed)
    n = int(mb * 1024 * 1024 / 8)
    lines, line = [], []
    for i in range(n):
        line.append(rng.choice(WORDS) if rng.random() < 0.9 else f"w{rng.randrange(5000)}")
        if len(line) == 12:
            lines.append(" ".join(line))
            line = []
    lines.append(" ".join(line))
    return "\n".join(lines) + "\n"


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--input")
    ap.add_argument("--synthetic-mb", type=float, default=8.0)
    ap.add_argument("--top", type=int, default=10)
    ap.add_argument("--master", default="local[2]")
    a = ap.parse_args(argv)
    path = a.input
    tmp = None
    if not path:
        tmp = tempfile.NamedTemporaryFile("w", suffix=".txt", delete=False)
        tmp.write(synthetic_text(a.synthetic_mb))
        tmp.close()
        path = tmp.name
    spark = (SparkSession.builder.appName("WordCount").master(a.master)
             .config("spark.sql.shuffle.partitions", "2").config("spark.default.parallelism", "2").getOrCreate())
    try:
        sc = spark.sparkContext
        t0 = time.perf_counter()
        counts = (sc.textFile(path).flatMap(lambda line: line.split()).map(lambda w: (w, 1))
                  .reduceByKey(operator.add).sortBy(lambda kv: (-kv[1], kv[0])).collect())
        t_rdd = time.perf_counter() - t0
        with open(path, "rb") as f:
            data = f.read()
        t0 = time.perf_counter()
        native = word_count_native(data, 2)
        t_native = time.perf_counter() - t0
        ok = dict(counts) == dict(native)
        words = sum(c for _, c in counts)
        for w, c in counts[: a.top]:
            print(f"{w}: {c}")
        print(json.dumps({"workload": "wordcount", "master": a.master, "bytes": len(data), "words": words,
                          "distinct": len(counts), "rdd_s": round(t_rdd, 3), "native_s": round(t_native, 4),
                          "words_per_s_rdd": round(words / t_rdd, 1), "words_per_s_native": round(words / t_native, 1),
                          "native_matches_rdd": ok}))
        if not ok:
            raise SystemExit("native and RDD word counts differ")
    finally:
        spark.stop()
        if tmp:
            os.unlink(tmp.name)


if __name__ == "__main__":
    main()
