"""Joint Spark ETL -> Parquet -> TF train pipeline (BASELINE.json config 5) on the CPU host path:
one rank, and two ranks (gloo) where every rank is one executor + one worker."""
import json
import os

import pyarrow.parquet as pq
import pytest

from test_distributed_cpu import _results, _run_ranks


@pytest.mark.parametrize("handoff", ["parquet", "device"])
def test_joint_single_rank(tmp_path, handoff):
    from pyspark_tf_gke_amd.pipeline import run_joint

    out = str(tmp_path / "joint")
    rep = run_joint(rows_per_executor=6000, out_dir=out, epochs=4, batch_size=256, handoff=handoff,
                    master="local[2]", verbose=False)
    assert 5500 < rep["rows_after_etl"] <= 6000  # ~2% null values filtered
    files = [f for f in os.listdir(os.path.join(out, "etl.parquet")) if f.endswith(".parquet")]
    # local[2]: spark.default.parallelism = 2 partitions -> one write task and one file each
    assert len(files) == 2 and os.path.exists(os.path.join(out, "etl.parquet", "_SUCCESS"))
    t = pq.read_table(os.path.join(out, "etl.parquet"))
    assert t.column_names == ["f0", "f1", "f2", "label"] and t.num_rows == rep["rows_after_etl"]
    f0 = t.column("f0").to_numpy()
    assert abs(f0.mean()) < 0.05 and abs(f0.std() - 1) < 0.05  # standardised
    assert int(t.column("label").to_numpy().max()) < 15
    hist = json.load(open(os.path.join(out, "history.json")))
    assert hist["loss"][-1] < hist["loss"][0]
    assert os.path.exists(os.path.join(out, "model.keras"))
    assert os.path.exists(os.path.join(out, "saved_model", "saved_model.json"))


def test_joint_two_ranks(tmp_path):
    out = str(tmp_path / "joint2")
    r = _run_ranks(f"""
    import json
    from pyspark_tf_gke_amd.pipeline import run_joint
    from pyspark_tf_gke_amd.parallel import comm
    rep = run_joint(rows_per_executor=4000, out_dir={out!r}, epochs=2, batch_size=256, master="mi355x",
                    verbose=False)
    print(f"[rank{{comm.rank()}}] RESULT " + json.dumps(rep), flush=True)
    """)
    assert r.returncode == 0, r.stderr[-3000:]
    res = _results(r.stdout)
    assert set(res) == {0, 1}
    assert res[0]["executors"] == 2 and res[0]["rows_generated"] == 8000
    assert res[0]["rows_after_etl"] == res[1]["rows_after_etl"] > 7000
    parts = [f for f in os.listdir(os.path.join(out, "etl.parquet")) if f.endswith(".parquet")]
    assert len(parts) == 2  # one Parquet part per executor
    assert res[0]["final"]["loss"] == pytest.approx(res[1]["final"]["loss"], rel=1e-6)  # all-reduced metrics
