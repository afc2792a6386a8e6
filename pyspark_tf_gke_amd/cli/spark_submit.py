"""``spark-submit``-shaped launcher (README recipes: infra/local/local_spark/README.md:57-65,
infra/local/external_workloads/README.md:64-73).

  python -m pyspark_tf_gke_amd.cli.spark_submit [--master M] [--num-executors N] [--name APP]
         [--conf k=v ...] [--deploy-mode client] [--packages ...] [--py-files a.py,b.zip] script.py [args]

* ``--master local[N]``: the application runs in one process on the host executor (N threads).
* any other master (``spark://host:7077``, ``k8s://...``, ``mi355x``): one executor per GPU —
  ``--num-executors`` ranks (default: all GPUs) launched on this node; every rank runs the driver
  script SPMD and the session binds rank r to GPU r.  ``spark.driver.host/port`` and
  ``spark.blockManager.port`` confs are accepted for compatibility (RCCL carries the data).
Confs reach the application's ``SparkSession.builder`` through ``PTG_SPARK_CONF`` (JSON).
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys

from ..runtime.launcher import _gpu_count, launch


def parse(argv):
    ap = argparse.ArgumentParser(prog="spark-submit")
    ap.add_argument("--master", default=os.environ.get("SPARK_MASTER", "local[*]"))
    ap.add_argument("--deploy-mode", default="client")
    ap.add_argument("--name", default=None)
    ap.add_argument("--num-executors", type=int, default=0)
    ap.add_argument("--executor-cores", type=int, default=0)
    ap.add_argument("--conf", action="append", default=[])
    ap.add_argument("--packages", default=None)
    ap.add_argument("--jars", default=None)
    ap.add_argument("--py-files", default=None)
    ap.add_argument("--max-restarts", type=int, default=0)
    ap.add_argument("app")
    ap.add_argument("app_args", nargs=argparse.REMAINDER)
    return ap.parse_args(argv)


def main(argv=None) -> int:
    a = parse(sys.argv[1:] if argv is None else argv)
    conf = {}
    for kv in a.conf:
        k, _, v = kv.partition("=")
        conf[k.strip()] = v.strip()
    conf["spark.master"] = a.master
    if a.name:
        conf["spark.app.name"] = a.name
    env = {"SPARK_MASTER": a.master, "PTG_SPARK_CONF": json.dumps(conf)}
    if a.py_files:
        extra = [os.path.abspath(p) for p in a.py_files.split(",") if p]
        env["PYTHONPATH"] = os.pathsep.join(extra + [os.environ.get("PYTHONPATH", "")])
    cmd = [sys.executable, a.app, *a.app_args]
    if re.match(r"local(\[.*\])?$", a.master):
        full = dict(os.environ)
        full.update(env)
        return subprocess.call(cmd, env=full)
    n = a.num_executors or _gpu_count() or 1
    return launch(cmd, n, env_extra=env, max_restarts=a.max_restarts)


if __name__ == "__main__":
    sys.exit(main())
