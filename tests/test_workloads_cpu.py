"""The re-expressed reference workloads (workloads/raw-spark, workloads/raw-tf) run end to end on the
CPU executor path: SQLite-backed JDBC reads with Spark's partition predicates, the KMeans workload
with its 7-label inference, the GCS-style CSV -> KMeans -> silhouette -> save workload, the engine
install check, wordcount, the worker/PS server entry point and the model checker."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SPARK = os.path.join(ROOT, "workloads", "raw-spark")
TF = os.path.join(ROOT, "workloads", "raw-tf")
HEALTH = os.path.join(ROOT, "tests", "data", "health.csv")


def _run(script, *args, env=None, timeout=600, cwd=None):
    e = dict(os.environ)
    e["PYTHONPATH"] = ROOT + os.pathsep + e.get("PYTHONPATH", "")
    e.setdefault("SPARK_MASTER", "local[2]")
    e["PTG_DEVICE"] = "cpu"
    e.update(env or {})
    r = subprocess.run([sys.executable, script, *args], env=e, capture_output=True, text=True, timeout=timeout,
                       cwd=cwd or ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout + r.stderr


@pytest.fixture(scope="module")
def jdbc_root(tmp_path_factory):
    root = tmp_path_factory.mktemp("db")
    sys.path.insert(0, SPARK)
    try:
        import load_csv
    finally:
        sys.path.remove(SPARK)
    assert load_csv.load(HEALTH, str(root)) == 18155
    return str(root)


def test_jdbc_partition_predicates_follow_spark():
    from pyspark_tf_gke_amd.sql.readwriter import jdbc_partition_predicates as P

    w = P("id", 1, 1_000_000, 16)  # google_health_SQL.py:33-36
    assert len(w) == 16
    assert w[0] == '"id" < 62501 OR "id" IS NULL'
    assert w[1] == '"id" >= 62501 AND "id" < 125001'
    assert w[-1] == '"id" >= 937501'
    assert P("id", 0, 10, 1) == ["1=1"]
    assert len(P("id", 0, 3, 16)) == 3  # never more partitions than values in range


def test_jdbc_sqlite_partitioned_read(jdbc_root, monkeypatch):
    from pyspark_tf_gke_amd.sql import SparkSession
    from pyspark_tf_gke_amd.sql import types as T

    monkeypatch.setenv("PTG_JDBC_ROOT", jdbc_root)
    spark = SparkSession.builder.master("local[2]").getOrCreate()
    df = (spark.read.format("jdbc").option("url", "jdbc:mysql://db:3306/health_data")
          .option("dbtable", "health_disparities").option("partitionColumn", "id").option("lowerBound", "1")
          .option("upperBound", "1000000").option("numPartitions", "16").load())
    assert df.count() == 18155
    assert len(df.columns) == 12 and df.columns[0] == "id" and df.columns[-1] == "created_at"
    sch = {f.name: f.dataType for f in df.schema.fields}
    assert isinstance(sch["id"], T.IntegerType) and isinstance(sch["value"], T.FloatType)
    assert isinstance(sch["created_at"], T.TimestampType) and isinstance(sch["measure_name"], T.StringType)
    assert df.rdd.getNumPartitions() == 16
    ids = sorted(r["id"] for r in df.select("id").collect())
    assert ids[0] == 1 and ids[-1] == 18155
    # adaptive bounds: same rows
    df2 = (spark.read.format("jdbc").option("url", f"jdbc:sqlite:{jdbc_root}/health_data.sqlite")
           .option("dbtable", "health_disparities").option("partitionColumn", "id").option("lowerBound", "1")
           .option("upperBound", "1000000").option("numPartitions", "4").option("adaptiveBounds", "true").load())
    assert df2.count() == 18155


def test_kmeans_workload_with_inference(jdbc_root):
    out = _run(os.path.join(SPARK, "k_means.py"), env={"PTG_JDBC_ROOT": jdbc_root})
    assert "Rows after filtering out missing 'measure_name' values: 18155" in out
    assert "repeating measure_name_vec 5 time(s)" in out
    preds = [line for line in out.splitlines() if "Inference prediction:" in line]
    assert len(preds) == 7
    assert all(0 <= int(p.rsplit(":", 1)[1]) < 25 for p in preds)
    assert "Spark session stopped." in out


def test_cloud_kmeans_silhouette_and_save(tmp_path):
    out = _run(os.path.join(SPARK, "spark_checks", "python_checks", "spark_workload_to_cloud_k8s.py"),
               env={"HEALTH_CSV": HEALTH, "MODEL_OUTPUT_DIR": str(tmp_path)})
    sil = float(out.split("Silhouette with squared Euclidean distance = ", 1)[1].split()[0])
    assert 0.0 < sil <= 1.0
    assert out.count("Cluster Centers:") == 1
    from pyspark_tf_gke_amd.ml import KMeansModel, PipelineModel

    m = KMeansModel.load(str(tmp_path / "health_kmeans_model"))
    assert len(m.clusterCenters()) == 5
    p = PipelineModel.load(str(tmp_path / "health_kmeans_pipeline"))
    assert len(p.stages) == 3


def test_installation_check():
    out = _run(os.path.join(SPARK, "spark_checks", "python_checks", "spark_installation_check.py"))
    after = out.split("DataFrame with age > 30:", 1)[1]
    assert "Alice" in after and "Bob" in after and "Charlie" not in after
    assert "Spark version:" in out and "Stopping Spark session..." in out


def test_local_k8s_partitioned_check(jdbc_root):
    out = _run(os.path.join(SPARK, "spark_checks", "python_checks", "spark_workload_to_local_k8s.py"),
               env={"PTG_JDBC_ROOT": jdbc_root})
    assert "Rows read: 18155 in 16 JDBC partitions" in out


def test_wordcount_local2():
    out = _run(os.path.join(SPARK, "wordcount.py"), "--synthetic-mb", "0.5")
    res = json.loads([line for line in out.splitlines() if line.startswith("{")][-1])
    assert res["native_matches_rdd"] and res["master"] == "local[2]" and res["words"] > 0


def test_tf_server_roles():
    sys.path.insert(0, TF)
    try:
        import tf_server
    finally:
        sys.path.remove(TF)
    assert tf_server.parse_role("tf-trainer-1") == ("worker", 1)
    assert tf_server.parse_role("tf-trainer-ps-0") == ("ps", 0)
    out = _run(os.path.join(TF, "tf_server.py"), env={"HOSTNAME": "tf-trainer-ps-0"})
    assert "role=ps index=0 target=grpc://tf-trainer-ps-0.tf-trainer-ps-headless:2222" in out


def test_model_checker_writes_plots(tmp_path):
    from PIL import Image

    from pyspark_tf_gke_amd.models import tf_models

    m = tf_models.build_cnn_model((256, 320, 3), flat=False, device="cpu")
    mdir = tmp_path / "tf-model"
    mdir.mkdir()
    m.save(str(mdir / "150-320-by-256-B1-model.keras"))
    imgs = tmp_path / "images"
    imgs.mkdir()
    rng = np.random.default_rng(0)
    for i in range(2):
        Image.fromarray(rng.integers(0, 255, (300, 400, 3), dtype=np.uint8)).save(imgs / f"spot{i}.png")
    out = _run(os.path.join(TF, "test-model.py"), "--model-dir", str(mdir), "--images", str(imgs),
               "--device", "cpu")
    assert out.count("predicted (x=") == 2
    assert sorted(os.listdir(mdir / "plots")) == ["spot0.png", "spot1.png"]


def test_train_tf_ps_use_ps_async(tmp_path):
    """The reference driver's parameter-server path in asynchronous mode
    (`train_tf_ps.py --use-ps --ps-mode async`, train_tf_ps.py:505-510,612-645): one process, the
    coordinator loop trains two epochs and the chief saves the model."""
    out = _run(os.path.join(TF, "train_tf_ps.py"), "--use-ps", "--ps-mode", "async", "--worker-replicas", "1",
               "--ps-replicas", "1", "--data-path", HEALTH, "--epochs", "2", "--batch-size", "512", "--output-dir",
               str(tmp_path), "--chief-addr", "127.0.0.1", env={"PTG_PS_MODE": "sync"})  # the flag wins
    assert "Epoch 2" in out and "loss:" in out, out[-2000:]
    assert os.path.exists(os.path.join(str(tmp_path), "model.keras"))
