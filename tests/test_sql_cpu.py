"""DataFrame API semantics on the host executor (local[N])."""
import math
import os

import numpy as np
import pandas as pd
import pytest

from pyspark_tf_gke_amd.sql import Row, SparkSession
from pyspark_tf_gke_amd.sql.functions import avg, col, count, isnan, lit, max as fmax, sum as fsum, when

HEALTH = os.path.join(os.path.dirname(__file__), "data", "health.csv")


@pytest.fixture(scope="module")
def spark():
    s = SparkSession.builder.appName("t").master("local[2]").config("spark.sql.shuffle.partitions", "2").getOrCreate()
    yield s
    s.stop()


def test_installation_check_flow(spark, capsys):
    """spark_installation_check.py:27-37 — createDataFrame, show, filter Age > 30."""
    df = spark.createDataFrame([("Alice", 34), ("Bob", 45), ("Charlie", 29)], ["Name", "Age"])
    df.show()
    out = capsys.readouterr().out
    assert "|  Alice| 34|" in out
    assert [r.Name for r in df.filter(df.Age > 30).collect()] == ["Alice", "Bob"]
    assert df.filter("Age > 30").count() == 2
    assert spark.sparkContext.applicationId.startswith("app-")


def test_csv_infer_schema_matches_pandas(spark):
    df = spark.read.csv(HEALTH, header=True, inferSchema=True)
    pdf = pd.read_csv(HEALTH)
    assert df.count() == len(pdf) == 18155
    assert df.columns == list(pdf.columns)
    types = dict(df.dtypes)
    assert types["measure_name"] == "string" and types["edition"] == "int"
    assert types["value"] in ("int", "double")
    # quoted commas in `source` survive tokenization
    src = [r["source"] for r in df.select("source").limit(50).collect()]
    assert src == list(pdf["source"].iloc[:50])
    v = df.select("value").filter(~isnan(col("value")) & col("value").isNotNull()).agg({"value": "avg"}).collect()[0][0]
    assert abs(v - pdf["value"].mean()) < 1e-6 * abs(v)


def test_null_handling_and_when(spark):
    df = spark.createDataFrame([(1, 2.0), (2, None), (3, float("nan")), (None, 4.0)], ["a", "b"])
    assert df.filter(col("b").isNull()).count() == 1
    assert df.filter(isnan(col("b"))).count() == 1
    f = df.withColumn("b", when(col("b").isNull() | isnan(col("b")), 9.0).otherwise(col("b")))
    assert [r.b for r in f.collect()] == [2.0, 9.0, 9.0, 4.0]
    g = df.withColumn("c", col("a") * 2 + 1)
    assert [r.c for r in g.collect()] == [3, 5, 7, None]
    h = df.withColumn("d", col("a") / lit(0))
    assert all(r.d is None for r in h.collect())


def test_groupby_agg_vs_pandas(spark):
    df = spark.read.csv(HEALTH, header=True, inferSchema=True)
    g = df.groupBy("measure_name").agg(count("*").alias("n"), avg("value").alias("m"), fmax("upper_ci").alias("mx"))
    got = {r["measure_name"]: (r["n"], r["m"], r["mx"]) for r in g.collect()}
    pdf = pd.read_csv(HEALTH)
    ref = pdf.groupby("measure_name").agg(n=("value", "size"), m=("value", "mean"), mx=("upper_ci", "max"))
    assert len(got) == len(ref) == 30
    for k, row in ref.iterrows():
        n, m, mx = got[k]
        assert n == row.n
        assert (m is None and math.isnan(row.m)) or abs(m - row.m) < 1e-6 * max(1, abs(row.m))
        assert (mx is None and math.isnan(row.mx)) or mx == row.mx


def test_multi_key_groupby_orderby_distinct(spark):
    df = spark.createDataFrame([("a", 1, 1.0), ("a", 1, 2.0), ("b", 2, 3.0), ("a", 2, 4.0)], ["k", "j", "v"])
    g = df.groupBy("k", "j").agg(fsum("v").alias("s")).orderBy("k", "j").collect()
    assert [(r.k, r.j, r.s) for r in g] == [("a", 1, 3.0), ("a", 2, 4.0), ("b", 2, 3.0)]
    assert df.select("k").distinct().count() == 2
    top = df.orderBy(col("v").desc()).first()
    assert top.v == 4.0
    assert df.groupBy("k").count().orderBy("k").collect()[0]["count"] == 3


def test_parquet_roundtrip(spark, tmp_path):
    df = spark.createDataFrame([("x", 1, 0.5), ("y", None, 1.5)], ["s", "i", "d"])
    p = str(tmp_path / "out.parquet")
    df.write.mode("overwrite").parquet(p)
    assert os.path.exists(os.path.join(p, "_SUCCESS"))
    back = spark.read.parquet(p)
    assert sorted(map(tuple, back.collect()), key=str) == sorted([("x", 1, 0.5), ("y", None, 1.5)], key=str)


def test_rdd_and_dataframe_wordcount(spark, tmp_path):
    p = tmp_path / "t.txt"
    p.write_text("a b a\nc a b\n\nd\n")
    sc = spark.sparkContext
    rdd = sc.textFile(str(p)).flatMap(lambda l: l.split()).map(lambda w: (w, 1)).reduceByKey(lambda a, b: a + b)
    assert dict(rdd.collect()) == {"a": 3, "b": 2, "c": 1, "d": 1}
    from pyspark_tf_gke_amd.sql.functions import explode, split

    words = spark.read.text(str(p)).select(explode(split(col("value"), r"\s+")).alias("word")).filter(col("word") != "")
    wc = {r.word: r["count"] for r in words.groupBy("word").count().collect()}
    assert wc == {"a": 3, "b": 2, "c": 1, "d": 1}
    from pyspark_tf_gke_amd.sql.rdd import word_count_native

    assert dict(word_count_native(p.read_bytes(), 2)) == {"a": 3, "b": 2, "c": 1, "d": 1}


def test_row_and_describe(spark):
    r = Row(name="x", v=1)
    assert r.name == "x" and r["v"] == 1 and r.asDict() == {"name": "x", "v": 1}
    df = spark.createDataFrame([(1.0,), (3.0,)], ["v"])
    d = {row["summary"]: row["v"] for row in df.describe().collect()}
    assert float(d["mean"]) == 2.0 and d["count"] == "2"
    _ = np


def test_groupby_null_key_is_its_own_group():
    """Nulls form one group outside the key domain: -2.0 (bit pattern 0xC000...) and -2**62 stay
    ordinary keys (a sentinel key value collided with them)."""
    from pyspark_tf_gke_amd.sql import SparkSession, functions as F

    spark = SparkSession.builder.master("local[1]").getOrCreate()
    df = spark.createDataFrame([(-2.0, 1), (-2.0, 2), (3.0, 5), (None, 7), (None, 1)], ["x", "y"])
    got = {r["x"]: r["s"] for r in df.groupBy("x").agg(F.sum("y").alias("s")).collect()}
    assert got == {-2.0: 3, 3.0: 5, None: 8}
    df = spark.createDataFrame([(-2.0, 1), (-2.0, 2), (3.0, 5)], ["x", "y"])
    got = {r["x"]: r["s"] for r in df.groupBy("x").agg(F.sum("y").alias("s")).collect()}
    assert got == {-2.0: 3, 3.0: 5}
    big = -(2 ** 62)
    df = spark.createDataFrame([(big, 1), (big, 2), (5, 5), (None, 4)], ["k", "y"])
    got = {r["k"]: r["c"] for r in df.groupBy("k").agg(F.count("*").alias("c")).collect()}
    assert got == {big: 2, 5: 1, None: 1}
    df = spark.createDataFrame([(1, None, 1.0), (1, "a", 2.0), (1, None, 3.0), (2, "a", 4.0)], ["a", "b", "v"])
    got = {(r["a"], r["b"]): r["s"] for r in df.groupBy("a", "b").agg(F.sum("v").alias("s")).collect()}
    assert got == {(1, None): 4.0, (1, "a"): 2.0, (2, "a"): 4.0}
    assert df.agg(F.countDistinct("b").alias("d")).collect()[0]["d"] == 1


def _py_sort_key(v, asc):
    """Spark order of one value: nulls first (asc) / last (desc); NaN above every number."""
    if v is None:
        return (0,) if asc else (2,)
    if isinstance(v, float) and math.isnan(v):
        return (1, 1, 0.0)
    return (1, 0, v)


@pytest.mark.parametrize("seed", [0, 1])
def test_orderby_matches_python_sort(spark, seed):
    """Multi-column orderBy (radix sort path; host executor) vs Python's stable sort with Spark's
    null/NaN ordering, ascending and descending."""
    rng = np.random.default_rng(seed)
    n = 3000
    rows = []
    for i in range(n):
        x = None if rng.random() < 0.05 else int(rng.integers(-50, 50))
        s = None if rng.random() < 0.05 else "k%02d" % rng.integers(0, 40)
        f = None if rng.random() < 0.05 else (float("nan") if rng.random() < 0.03 else float(rng.normal()))
        rows.append((x, s, f, i))
    df = spark.createDataFrame(rows, ["x", "s", "f", "i"])
    for spec in [(("x", True), ("f", False)), (("s", False), ("x", True)), (("f", True),), (("x", False), ("s", True), ("f", True))]:
        got = [tuple(r)[3] for r in df.orderBy(*[col(c).asc() if a else col(c).desc() for c, a in spec]).collect()]
        want = list(range(n))
        for c, a in reversed(spec):
            j = ["x", "s", "f"].index(c)
            nulls = [r for r in want if rows[r][j] is None]
            vals = [r for r in want if rows[r][j] is not None]
            vals.sort(key=lambda r: _py_sort_key(rows[r][j], True), reverse=not a)
            if not a:  # reverse=True breaks stability among equal keys: restore input order within ties
                groups = {}
                for r in vals:
                    groups.setdefault(_py_sort_key(rows[r][j], True), []).append(r)
                vals = [r for kk in sorted(groups, reverse=True) for r in sorted(groups[kk], key=want.index)]
            want = (nulls + vals) if a else (vals + nulls)
        assert got == want, spec


def test_shuffle_budget_and_tensor_control_plane(spark):
    """Single process: shuffles degenerate to a local take; count/describe/agg run without any
    pickled collective (the multi-rank variant is in test_distributed_cpu)."""
    from pyspark_tf_gke_amd.parallel import comm

    calls = []
    orig = comm.all_gather_object
    comm.all_gather_object = lambda o: calls.append(o) or orig(o)
    try:
        df = spark.createDataFrame([(i % 7, float(i)) for i in range(100)], ["k", "v"])
        assert df.count() == 100
        df.describe("v").collect()
        df.agg(fsum("v")).collect()
        df.orderBy("v").limit(3).collect()
    finally:
        comm.all_gather_object = orig
    assert calls == []


def test_lazy_stage_pushdown_fusion_and_retry(spark, capsys):
    """filter/withColumn chains run as one optimised narrow stage: filters on source columns are
    pushed ahead of the projections and fused into one predicate (one VM pass, one compaction, one
    gather); results equal the step-by-step evaluation; a failing task attempt is retried
    (spark.task.maxFailures) and explain() shows the plan."""
    from pyspark_tf_gke_amd.sql import plan as P

    rows = [(i, float(i) * 0.5 if i % 7 else None, "s%d" % (i % 5)) for i in range(1000)]
    df = spark.createDataFrame(rows, ["a", "b", "s"])
    q = (df.filter(col("a") > 10)
         .withColumn("c", col("a") * 2)
         .filter(col("b").isNotNull())
         .withColumn("d", when(col("c") > 100, col("c")).otherwise(lit(0)))
         .filter(col("d") > 0)
         .filter(col("a") < 900))
    q.explain()
    out = capsys.readouterr().out
    assert "pushed down" in out and "a > 10" in out.replace("(", "").replace(")", "") or "Filter" in out
    before = dict(P.STATS)
    got = sorted((r["a"], r["c"], r["d"]) for r in q.collect())
    # 3 source filters fused into 1 pass + 2 projections + 1 post filter = 4 VM passes, 2 gathers
    assert P.STATS["vm_passes"] - before["vm_passes"] == 4
    assert P.STATS["gathers"] - before["gathers"] == 2
    want = sorted((i, 2 * i, 2 * i) for i in range(1000) if 10 < i < 900 and i % 7 and 2 * i > 100)
    assert got == want
    # injected task failures are retried; beyond maxFailures the job fails
    P._FAULTS["left"] = 2
    r0 = P.STATS["retries"]
    assert df.filter(col("a") < 5).count() == 5
    assert P.STATS["retries"] - r0 == 2
    P._FAULTS["left"] = 10
    with pytest.raises(P.TaskFailure):
        df.filter(col("a") < 5).count()
    P._FAULTS["left"] = 0
    with pytest.raises(KeyError):
        df.filter(col("nope") > 1)


def test_range_window_plan():
    """Window planning of the dense-key groupBy path (ops/df.py): 256 << sh keys, centred on the
    sampled range so keys just past the sample's ends still fall inside; spans above 2^20 refuse."""
    from pyspark_tf_gke_amd.ops import df as D

    for lo, hi in ((0, 999_999), (15, 999_985), (-5_000_000_000, -5_000_000_000 + (1 << 20) - 1), (7, 7), (3, 300)):
        base, sh = D._range_window(lo, hi)
        assert sh <= 12 and (256 << sh) >= hi - lo + 1
        assert sh == 0 or (256 << (sh - 1)) < hi - lo + 1  # smallest window that fits
        assert base <= lo and hi < base + (256 << sh)
    base, sh = D._range_window(15, 999_985)  # a 64K-key sample of keys 0..999,999
    assert base <= 0 and 999_999 < base + (256 << sh)
    assert D._range_window(0, 1 << 20) is None


def test_config_precedence(monkeypatch):
    """Typed knob registry: CLI > env > active session conf > default; the stopped
    session's conf no longer applies; bool parsing of env strings."""
    from pyspark_tf_gke_amd import config
    from pyspark_tf_gke_amd.sql import SparkSession

    monkeypatch.delenv("PTG_RANGE_CHUNKS", raising=False)
    monkeypatch.delenv("PTG_SPARK_CONF", raising=False)
    assert config.get("groupby_range_chunks") == 8 and config.source("groupby_range_chunks") == "default"
    s = SparkSession.builder.master("local[1]").config("spark.ptg.groupby.rangeChunks", "4").getOrCreate()
    try:
        assert config.get("groupby_range_chunks") == 4 and config.source("groupby_range_chunks") == "conf"
        s.conf.set("spark.ptg.groupby.rangeChunks", 2)  # live
        assert config.get("groupby_range_chunks") == 2
        monkeypatch.setenv("PTG_RANGE_CHUNKS", "16")
        assert config.get("groupby_range_chunks") == 16 and config.source("groupby_range_chunks") == "env"
        config.set_cli("groupby_range_chunks", 3)
        assert config.get("groupby_range_chunks") == 3 and config.source("groupby_range_chunks") == "cli"
    finally:
        config._cli.pop("groupby_range_chunks", None)
        s.stop()
    monkeypatch.delenv("PTG_RANGE_CHUNKS")
    assert config.get("groupby_range_chunks") == 8
    for raw, want in (("0", False), ("false", False), ("1", True), ("yes", True)):
        monkeypatch.setenv("PTG_GROUPBY_RANGE", raw)
        assert config.get("groupby_range") is want
    assert {r["name"] for r in config.describe()} >= {"fused_adam", "shuffle_buffer_gb", "pg_timeout_s"}


def test_distinct_estimate_widens_at_most_to_the_cap(monkeypatch):
    """All-unique keys saturate every sample: the estimate widens once (bounded sample), then
    returns n instead of hashing ever larger samples (64K -> 1M -> 16M -> 256M)."""
    import torch

    from pyspark_tf_gke_amd.ops import df as D

    seen = []
    real = D.hash_agg

    def spy(keys, *a, **kw):
        seen.append(keys.numel())
        return real(keys, *a, **kw)

    monkeypatch.setattr(D, "hash_agg", spy)
    monkeypatch.setattr(D, "ESTIMATE_SAMPLE_MAX", 1 << 14)
    keys = torch.arange(1 << 20, dtype=torch.int64) * 7919
    assert D.estimate_distinct(keys, sample=1 << 10) == keys.numel()
    assert max(seen) <= 1 << 14 and len(seen) == 2, seen
    # a genuinely small key set is still estimated from the first sample
    seen.clear()
    small = torch.randint(0, 300, (1 << 20,), generator=torch.Generator().manual_seed(0))
    assert 250 <= D.estimate_distinct(small, sample=1 << 10) <= 400
    assert len(seen) == 1


def test_kmeans_chain_is_one_fused_scan(spark, capsys):
    """k_means.py:23-51 on health.csv: filter(measure_name not null) -> per column
    select(c).filter(~isnan & not null).agg(avg) -> withColumn(when(...)) imputation.  Every
    avg runs as ONE fused scan of the source (projections inlined, one predicate pass, masked
    reduction: no compaction or row gather), explain() shows it, and the numbers equal the
    materialise-everything evaluation."""
    from pyspark_tf_gke_amd.sql import plan as P

    src = spark.read.csv(HEALTH, header=True, inferSchema=True).cache()
    df = src.filter(col("measure_name").isNotNull())
    means, ref = {}, {}
    before = dict(P.STATS)
    for c in ["value", "lower_ci", "upper_ci"]:
        q = df.select(c).filter(~isnan(col(c)) & col(c).isNotNull()).agg({c: "avg"})
        means[c] = q.collect()[0][0]
        df = df.withColumn(c, when(col(c).isNull() | isnan(col(c)), means[c]).otherwise(col(c)))
    q.explain()
    out = capsys.readouterr().out
    assert "one fused scan" in out and "masked reduction" in out and "measure_name IS NOT NULL" in out, out
    assert P.STATS["fused_aggs"] - before["fused_aggs"] == 3
    assert P.STATS["compactions"] - before["compactions"] == 0 and P.STATS["gathers"] - before["gathers"] == 0
    assert P.STATS["tasks"] - before["tasks"] == 0  # nothing materialised
    # reference: pandas on the same rows
    pdf = pd.read_csv(HEALTH)
    pdf = pdf[pdf["measure_name"].notna()]
    for c in ["value", "lower_ci", "upper_ci"]:
        ref[c] = float(pdf[c].dropna().mean())
        pdf[c] = pdf[c].fillna(ref[c])
        assert abs(means[c] - ref[c]) <= 1e-9 * max(1.0, abs(ref[c])), (c, means[c], ref[c])
    # the imputed frame is still a pending stage: its aggregate inlines the CASE WHEN imputation
    fin = df.agg(avg("upper_ci"))
    fin.explain()
    assert "CASE WHEN" in capsys.readouterr().out
    got = fin.collect()[0][0]
    assert abs(got - float(pdf["upper_ci"].mean())) < 1e-9 * max(1.0, abs(got))


def test_grouped_agg_over_pending_stage_prunes_columns(spark, capsys):
    """filter -> withColumn -> groupBy.agg: one predicate pass, one compaction, and a gather of only
    the source columns the key / value expressions read (pruned), equal to the materialised path."""
    from pyspark_tf_gke_amd.sql import plan as P

    rows = [(i % 13, float(i), "x" * (i % 3), i * 2) for i in range(5000)]
    df = spark.createDataFrame(rows, ["k", "v", "s", "w"])
    before = dict(P.STATS)
    q = (df.filter(col("v") > 100).withColumn("v2", col("v") * 2 + col("k"))
         .filter(col("w") % 3 != 0).groupBy("k").agg(fsum("v2").alias("t"), count("*").alias("n")))
    got = sorted(tuple(r) for r in q.collect())
    assert P.STATS["fused_aggs"] - before["fused_aggs"] == 1 and P.STATS["compactions"] - before["compactions"] == 1
    assert P.STATS["tasks"] - before["tasks"] == 0
    q.explain()
    out = capsys.readouterr().out
    assert "pruned: k, v" in out and "w" not in out.split("pruned:")[1].split("]")[0].split(", ")
    pdf = pd.DataFrame(rows, columns=["k", "v", "s", "w"])
    pdf = pdf[(pdf.v > 100) & (pdf.w % 3 != 0)]
    pdf["v2"] = pdf.v * 2 + pdf.k
    want = sorted((int(k), float(g.v2.sum()), int(len(g))) for k, g in pdf.groupby("k"))
    assert [(a, pytest.approx(b), c) for a, b, c in want] == got


def test_stage_retry_on_genuine_runtime_error_and_oom_replan(spark, monkeypatch):
    """A RuntimeError raised inside a narrow stage (as a failed HIP launch would) is retried; an
    out-of-memory attempt re-plans the stage over 2 row chunks; the results are unchanged."""
    from pyspark_tf_gke_amd.ops import df as D
    from pyspark_tf_gke_amd.sql import plan as P

    df = spark.createDataFrame([(i, float(i % 17)) for i in range(4000)], ["a", "b"])
    q = df.filter(col("b") > 3).withColumn("c", col("a") + col("b"))
    want = sorted((r["a"], r["c"]) for r in q.cache().collect())
    real = D.compact
    state = {"n": 1}

    def flaky(mask):
        if state["n"] > 0:
            state["n"] -= 1
            raise RuntimeError("native kernel ptg_compact failed: hipError_t=719")
        return real(mask)

    monkeypatch.setattr(D, "compact", flaky)
    r0 = P.STATS["retries"]
    q2 = df.filter(col("b") > 3).withColumn("c", col("a") + col("b"))
    assert sorted((r["a"], r["c"]) for r in q2.collect()) == want
    assert P.STATS["retries"] - r0 == 1 and state["n"] == 0
    monkeypatch.setattr(D, "compact", real)
    # out of memory: re-planned in chunks
    p0, c0 = P.STATS["replans"], P.STATS["chunks"]
    P._FAULTS["oom"] = 1
    q3 = df.filter(col("b") > 3).withColumn("c", col("a") + col("b"))
    assert sorted((r["a"], r["c"]) for r in q3.collect()) == want
    assert P.STATS["replans"] - p0 == 1 and P.STATS["chunks"] - c0 == 2
    # a programming error is not retried
    with pytest.raises(KeyError):
        df.filter(col("zz") > 1)


def test_repartition_makes_local_partitions_and_write_tasks(spark, tmp_path):
    """repartition(n, col) on one executor: n hash partitions as contiguous row ranges, every key in
    exactly one partition; write() runs one task / file per non-empty partition; coalesce merges
    adjacent partitions without moving rows."""
    import pyarrow.parquet as pq

    df = spark.createDataFrame([(i % 50, float(i)) for i in range(3000)], ["k", "v"])
    r = df.repartition(8, "k")
    sizes = r.local_partition_sizes()
    assert len(sizes) == 8 and sum(sizes) == 3000 and r.rdd.getNumPartitions() == 8
    seen = {}
    for p, t in enumerate(r.local_partitions()):
        for k in set(int(x) for x in t.column("k").data.tolist()):
            assert seen.setdefault(k, p) == p
    assert len(seen) == 50
    out = str(tmp_path / "parts")
    r.write.parquet(out)
    files = [f for f in os.listdir(out) if f.endswith(".parquet")]
    assert len(files) == sum(1 for s in sizes if s)
    assert pq.read_table(out).num_rows == 3000
    c = r.coalesce(2)
    assert len(c.local_partition_sizes()) == 2 and sum(c.local_partition_sizes()) == 3000
    assert len(df.repartition(5).local_partition_sizes()) == 5


def test_hash9_table_sizing():
    """Planner side of the 512-way hash groupBy (ops/df.py): the LDS table holds the fullest of the
    512 partitions at load <= 0.7 within 150 KB, and declines key counts it cannot hold."""
    from pyspark_tf_gke_amd.ops import df as D

    assert D._h9_table_slots(1_000_000, 1) == 4096          # ~1953 keys / partition -> 4096 slots
    assert D._h9_table_slots(65_536, 1) == 1024              # minimum table
    assert D._h9_table_slots(1_000_000, 2) == 4096           # 36 B/slot -> 144 KB
    assert D._h9_table_slots(2_000_000, 1) is None           # 8192 x 24 B > 150 KB
    for k, nv in ((70_000, 0), (300_000, 1), (900_000, 2)):
        ts = D._h9_table_slots(k, nv)
        assert ts & (ts - 1) == 0 and k / D.H9_BINS * 1.15 <= 0.7 * ts and ts * (12 + 12 * nv) <= 150 * 1024
