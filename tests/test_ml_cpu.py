"""Spark-ML parity on the host path: StringIndexer ordering, OneHot sizing, assembler layout,
KMeans quality vs scikit-learn, silhouette vs scikit-learn, persistence."""
import os

import numpy as np
import pytest
from sklearn.cluster import KMeans as SKKMeans
from sklearn.metrics import silhouette_score

from pyspark_tf_gke_amd.ml import (ClusteringEvaluator, KMeans, KMeansModel, OneHotEncoder, Pipeline, PipelineModel,
                                   StringIndexer, VectorAssembler)
from pyspark_tf_gke_amd.sql import SparkSession

HEALTH = os.path.join(os.path.dirname(__file__), "data", "health.csv")


@pytest.fixture(scope="module")
def spark():
    return SparkSession.builder.master("local[2]").getOrCreate()


def test_string_indexer_frequency_desc_and_keep(spark):
    df = spark.createDataFrame([("b",), ("a",), ("b",), ("c",), ("a",), ("b",)], ["s"])
    m = StringIndexer(inputCol="s", outputCol="i", handleInvalid="keep").fit(df)
    assert m.labels == ["b", "a", "c"]
    test = spark.createDataFrame([("c",), ("zz",)], ["s"])
    assert [r.i for r in m.transform(test).collect()] == [2.0, 3.0]
    enc = OneHotEncoder(inputCol="i", outputCol="v").fit(m.transform(df))
    out = enc.transform(m.transform(test)).collect()
    assert list(out[0].v.toArray()) == [0, 0, 1] and list(out[1].v.toArray()) == [0, 0, 0]


def _health_features(spark, repeats=5):
    df = spark.read.csv(HEALTH, header=True, inferSchema=True).na.fill(0)
    stages = [StringIndexer(inputCol="measure_name", outputCol="mi", handleInvalid="keep"),
              OneHotEncoder(inputCol="mi", outputCol="mv"),
              VectorAssembler(inputCols=["mv"] * repeats + ["value", "lower_ci", "upper_ci"], outputCol="features",
                              handleInvalid="keep")]
    pm = Pipeline(stages=stages).fit(df)
    return pm, pm.transform(df)


def test_assembler_layout_matches_repeat_weighting(spark):
    pm, t = _health_features(spark)
    X = t._t.column("features").data.numpy()
    assert X.shape == (18155, 5 * 30 + 3)
    blocks = X[:, :150].reshape(-1, 5, 30)
    assert np.all(blocks == blocks[:, :1, :])  # five identical one-hot copies (k_means.py:56-64)
    assert np.all(blocks[:, 0, :].sum(1) <= 1)


def test_kmeans_cost_close_to_sklearn(spark):
    _, t = _health_features(spark)
    X = t._t.column("features").data.numpy().astype(np.float64)
    km = KMeans(k=5, seed=1, maxIter=100).fit(t)
    sk = SKKMeans(n_clusters=5, n_init=4, random_state=0).fit(X)
    assert km.summary.trainingCost <= 1.05 * sk.inertia_
    pred = km.transform(t)
    lab = pred._t.column("prediction").data.numpy()
    ours = ClusteringEvaluator().evaluate(pred)
    idx = np.random.default_rng(0).choice(len(X), 3000, replace=False)
    ref = silhouette_score(X[idx], lab[idx], metric="sqeuclidean")
    assert abs(ours - ref) < 0.02


def test_exact_silhouette_small(spark):
    rng = np.random.default_rng(0)
    X = np.concatenate([rng.normal(0, 1, (40, 3)), rng.normal(6, 1, (40, 3))]).astype(np.float32)
    lab = np.array([0] * 40 + [1] * 40)
    from pyspark_tf_gke_amd.ml.linalg import DenseVector

    df = spark.createDataFrame([(DenseVector(x), int(l)) for x, l in zip(X, lab)], ["features", "prediction"])
    ours = ClusteringEvaluator().evaluate(df)
    ref = silhouette_score(X, lab, metric="sqeuclidean")
    assert abs(ours - ref) < 1e-4


def test_pipeline_and_kmeans_save_load(spark, tmp_path):
    pm, t = _health_features(spark)
    km = KMeans(k=4, seed=1).fit(t)
    km.save(str(tmp_path / "km"))
    pm.save(str(tmp_path / "pm"))
    assert os.path.exists(tmp_path / "km" / "metadata" / "part-00000")
    assert any(f.endswith(".parquet") for f in os.listdir(tmp_path / "km" / "data"))
    km2 = KMeansModel.load(str(tmp_path / "km"))
    assert np.allclose(np.stack(km2.clusterCenters()), np.stack(km.clusterCenters()))
    pm2 = PipelineModel.load(str(tmp_path / "pm"))
    one = spark.createDataFrame([("Asthma", 10, 17, 15)], ["measure_name", "value", "lower_ci", "upper_ci"])
    p1 = km.transform(pm.transform(one)).first().prediction
    p2 = km2.transform(pm2.transform(one)).first().prediction
    assert p1 == p2
