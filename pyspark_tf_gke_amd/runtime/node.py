"""Single-node "cluster" front end: read ``deploy/node.yaml`` and launch a job with the configured
roles (the collapse of the reference's Kubernetes/Terraform layers, SURVEY.md §1 L5/L6 and §7.1
Tier C, onto one 8xMI355X node).

  python -m pyspark_tf_gke_amd.runtime.node deploy/node.yaml spark  <app.py> [args]
  python -m pyspark_tf_gke_amd.runtime.node deploy/node.yaml train  [train_tf_ps.py flags]
  python -m pyspark_tf_gke_amd.runtime.node deploy/node.yaml joint  [etl_to_train flags]
  python -m pyspark_tf_gke_amd.runtime.node deploy/node.yaml show

``spark`` goes through the spark-submit CLI (one executor per GPU), ``train`` launches one TF
worker per GPU running the reference trainer with ``--strategy`` from the config (``ps`` maps to the
sharded ParameterServerStrategy + ClusterCoordinator), ``joint`` runs the ETL -> Parquet -> train
pipeline with every rank both executor and worker.  Address/port settings become the rendezvous
endpoint and the ClusterSpec the trainer prints; nothing listens on 7077/7078/2222.
"""
from __future__ import annotations

import json
import os
import sys

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def load(path: str) -> dict:
    with open(path) as fh:
        cfg = yaml.safe_load(fh) or {}
    node = cfg.setdefault("node", {})
    node.setdefault("gpus", 8)
    node.setdefault("master_addr", "127.0.0.1")
    node.setdefault("master_port", 29500)
    cfg.setdefault("spark", {}).setdefault("executors", node["gpus"])
    cfg["spark"].setdefault("master", "mi355x")
    tf = cfg.setdefault("tensorflow", {})
    tf.setdefault("workers", node["gpus"])
    tf.setdefault("ps", node["gpus"])
    tf.setdefault("strategy", "mirrored")
    if cfg["spark"]["executors"] > node["gpus"] or tf["workers"] > node["gpus"]:
        raise ValueError("more executors/workers than GPUs on the node (one rank per GPU)")
    return cfg


def commands(cfg: dict, job: str, args: list) -> tuple[list, dict, int]:
    """(command, extra env, ranks) for ``job``."""
    node, sp, tf = cfg["node"], cfg["spark"], cfg["tensorflow"]
    env = {"MASTER_ADDR": str(node["master_addr"]), "MASTER_PORT": str(node["master_port"])}
    if job == "spark":
        cmd = [sys.executable, "-m", "pyspark_tf_gke_amd.cli.spark_submit", "--master", sp["master"],
               "--num-executors", str(sp["executors"])]
        for k, v in (sp.get("conf") or {}).items():
            cmd += ["--conf", f"{k}={v}"]
        return cmd + list(args), env, 1
    if job == "train":
        flags = ["--worker-replicas", str(tf["workers"]), "--ps-replicas", str(tf["ps"]),
                 "--port", str(tf.get("port", 2222)), "--chief-port", str(tf.get("chief_port", 2223)),
                 "--strategy", tf["strategy"]]
        if tf["strategy"] == "ps":
            flags.append("--use-ps")
        return [sys.executable, os.path.join(ROOT, "workloads", "raw-tf", "train_tf_ps.py"), *flags, *args], env, \
            tf["workers"]
    if job == "joint":
        return [sys.executable, os.path.join(ROOT, "workloads", "joint", "etl_to_train.py"), *args], env, \
            min(sp["executors"], tf["workers"])
    raise ValueError(f"unknown job {job!r} (spark | train | joint | show)")


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) < 2:
        print(__doc__)
        return 2
    cfg = load(argv[0])
    job, rest = argv[1], argv[2:]
    if rest[:1] == ["--"]:
        rest = rest[1:]
    if job == "show":
        print(json.dumps(cfg, indent=2))
        return 0
    cmd, env, ranks = commands(cfg, job, rest)
    if ranks == 1:
        import subprocess

        full = dict(os.environ)
        full.update(env)
        return subprocess.call(cmd, env=full)
    from .launcher import launch

    os.environ.update(env)
    return launch(cmd, ranks, master_addr=env["MASTER_ADDR"], master_port=int(env["MASTER_PORT"]))


if __name__ == "__main__":
    sys.exit(main())
