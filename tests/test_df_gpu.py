"""DataFrame / ML kernels on the MI355X vs the host (CPU) executor path on identical data."""
import math
import os

import numpy as np
import pytest
import torch

from pyspark_tf_gke_amd.ops import df as D

pytestmark = pytest.mark.gpu

HEALTH = os.path.join(os.path.dirname(__file__), "data", "health.csv")


@pytest.fixture(scope="module")
def spark_gpu(hip_built):
    from pyspark_tf_gke_amd.sql import SparkSession

    s = SparkSession.builder.master("local[1]").config("spark.ptg.device", "cuda").getOrCreate()
    yield s
    s.stop()


def _host(fn):
    from pyspark_tf_gke_amd.sql.session import SparkSession

    s = SparkSession("host", "local[2]", {})
    return fn(s)


def test_compact_and_gather(hip_built):
    n = 1_000_003
    m = (torch.rand(n) < 0.3).to(torch.uint8)
    idx = D.compact(m.cuda())
    ref = torch.nonzero(m).view(-1)
    assert torch.equal(idx.cpu(), ref)
    x = torch.randn(n, 3)
    g = D.gather_rows(x.cuda(), idx)
    assert torch.equal(g.cpu(), x[ref])


def test_reduce_stats(hip_built):
    x = torch.randn(100_000, dtype=torch.float64)
    x[::7] = math.nan
    valid = (torch.rand(100_000) > 0.1).to(torch.uint8)
    g = D.reduce_stats(x.cuda(), valid.cuda())
    h = D.reduce_stats(x, valid)
    assert np.allclose(g, h, rtol=1e-9, equal_nan=True)


@pytest.mark.parametrize("nkeys", [7, 5000, 300_000])
def test_hash_agg_matches_host(hip_built, nkeys):
    n = 2_000_000
    k, v = D.fill_synthetic_kv(n, nkeys, "cpu")
    kg, rg, og = D.hash_agg(k.cuda(), [v.cuda()], [None], True)
    kh, rh, oh = D.hash_agg(k, [v], [None], True)
    order = torch.argsort(kg.cpu())
    assert torch.equal(kg.cpu()[order], kh)
    assert torch.allclose(rg.cpu()[order], rh)
    assert torch.allclose(og[0][0].cpu()[order], oh[0][0], rtol=1e-9)
    assert torch.allclose(og[0][2].cpu()[order], oh[0][2])
    assert torch.allclose(og[0][3].cpu()[order], oh[0][3])


@pytest.mark.parametrize("n,nkeys,pbits", [(4_000_000, 1_000_000, 9), (8_388_608, 1_000_000, 12),
                                           (5_000_000, 3_000, 12)])
def test_partitioned_agg(hip_built, n, nkeys, pbits):
    """pbits=12 with n >= 2^22 takes the two-level LDS-staged radix partitioning; 3,000 keys leave
    most of the 4,096 partitions (and some level-1 segments' tiles) empty."""
    k, v = D.fill_synthetic_kv(n, nkeys, "cuda")
    ok, osum, ocnt, m, _, overflow = D.hash_agg_partitioned(k, v, pbits=pbits)
    m = int(m.item())
    assert int(overflow.item()) == 0
    kh, rh, oh = D.hash_agg(k.cpu(), [v.cpu()], [None], False)
    assert m == kh.numel()
    order = torch.argsort(ok[:m].cpu())
    assert torch.equal(ok[:m].cpu()[order], kh)
    assert torch.allclose(osum[:m].cpu()[order], oh[0][0], rtol=1e-9)
    assert torch.allclose(ocnt[:m].cpu()[order], rh)


def test_synthetic_kv_device_matches_host(hip_built):
    kg, vg = D.fill_synthetic_kv(10_000, 1000, "cuda", offset=5, seed=3)
    kh, vh = D.fill_synthetic_kv(10_000, 1000, "cpu", offset=5, seed=3)
    assert torch.equal(kg.cpu(), kh) and torch.allclose(vg.cpu(), vh)


def test_dataframe_pipeline_gpu_vs_host(spark_gpu):
    from pyspark_tf_gke_amd.sql.functions import avg, col, count, isnan, when

    def run(spark):
        df = spark.read.csv(HEALTH, header=True, inferSchema=True)
        df = df.filter(col("measure_name").isNotNull())
        for c in ["value", "lower_ci", "upper_ci"]:
            mv = df.select(c).filter(~isnan(col(c)) & col(c).isNotNull()).agg({c: "avg"}).collect()[0][0]
            df = df.withColumn(c, when(col(c).isNull() | isnan(col(c)), mv).otherwise(col(c)))
        g = df.groupBy("measure_name").agg(count("*").alias("n"), avg("value").alias("m"))
        rows = sorted((r["measure_name"], r["n"], round(r["m"], 6)) for r in g.collect())
        f = df.filter((col("value") > 50) & (col("state_name") == "Texas")).count()
        return rows, f, df.count()

    g = run(spark_gpu)
    h = _host(run)
    assert g == h


def test_kmeans_and_silhouette_gpu_vs_host(spark_gpu):
    from pyspark_tf_gke_amd.ml import ClusteringEvaluator, KMeans, OneHotEncoder, Pipeline, StringIndexer, VectorAssembler
    from pyspark_tf_gke_amd.sql.functions import col

    def run(spark):
        df = spark.read.csv(HEALTH, header=True, inferSchema=True).na.fill(0)
        stages = [StringIndexer(inputCol="measure_name", outputCol="mi", handleInvalid="keep"),
                  OneHotEncoder(inputCol="mi", outputCol="mv"),
                  VectorAssembler(inputCols=["mv"] * 5 + ["value", "lower_ci", "upper_ci"], outputCol="features",
                                  handleInvalid="keep")]
        t = Pipeline(stages=stages).fit(df).transform(df)
        km = KMeans(k=5, seed=1, maxIter=50).fit(t)
        sil = ClusteringEvaluator().evaluate(km.transform(t))
        return km.summary.trainingCost, sil, t._t.column("features").data.float().cpu()

    cg, sg, fg = run(spark_gpu)
    ch, sh, fh = _host(run)
    assert torch.equal(fg, fh)
    assert abs(cg - ch) <= 1e-3 * abs(ch)
    assert abs(sg - sh) <= 1e-3
    _ = col
