"""The reference's Spark workloads on the GPU executor path (SPARK_MASTER=mi355x: one executor per
GPU, feature assembly / KMeans / silhouette as HIP kernels), end to end, with wall times printed."""
import os
import subprocess
import sys
import time

import pytest

from test_workloads_cpu import HEALTH, ROOT, SPARK

pytestmark = pytest.mark.gpu


def _run_gpu(script, env=None, timeout=600):
    e = dict(os.environ)
    e["PYTHONPATH"] = ROOT + os.pathsep + e.get("PYTHONPATH", "")
    e["SPARK_MASTER"] = "mi355x"
    e.pop("PTG_DEVICE", None)
    e.update(env or {})
    t0 = time.time()
    r = subprocess.run([sys.executable, script], env=e, capture_output=True, text=True, timeout=timeout, cwd=ROOT)
    dt = time.time() - t0
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    print(f"{os.path.basename(script)}: {dt:.1f}s")
    return r.stdout + r.stderr


@pytest.fixture(scope="module")
def jdbc_root_gpu(tmp_path_factory):
    root = tmp_path_factory.mktemp("dbg")
    sys.path.insert(0, SPARK)
    try:
        import load_csv
    finally:
        sys.path.remove(SPARK)
    assert load_csv.load(HEALTH, str(root)) == 18155
    return str(root)


def test_kmeans_workload_gpu(jdbc_root_gpu):
    out = _run_gpu(os.path.join(SPARK, "k_means.py"), env={"PTG_JDBC_ROOT": jdbc_root_gpu})
    assert "Rows after filtering out missing 'measure_name' values: 18155" in out
    preds = [line for line in out.splitlines() if "Inference prediction:" in line]
    assert len(preds) == 7 and all(0 <= int(p.rsplit(":", 1)[1]) < 25 for p in preds)


def test_cloud_kmeans_gpu(tmp_path):
    out = _run_gpu(os.path.join(SPARK, "spark_checks", "python_checks", "spark_workload_to_cloud_k8s.py"),
                   env={"HEALTH_CSV": HEALTH, "MODEL_OUTPUT_DIR": str(tmp_path)})
    sil = float(out.split("Silhouette with squared Euclidean distance = ", 1)[1].split()[0])
    assert 0.0 < sil <= 1.0
