"""Worker / parameter-server "pod" entry point (reference: infra/local/raw-tf/tf-trainer-worker.yaml:43-68,
tf-trainer-ps.yaml:43-67).

Parses the ordinal from ``HOSTNAME`` (``tf-trainer-<i>`` or ``tf-trainer-ps-<i>``), takes the ``ps``
role when the name contains ``-ps-``, builds the same ClusterSpec as the trainer and starts a
:class:`~pyspark_tf_gke_amd.distribute.cluster.Server`.  In this runtime the servers' work is done by
the GPU ranks the launcher spawns, so ``--block`` (the reference's sleep-forever) is optional.
"""
import argparse
import os
import re

import _path  # noqa: F401

from pyspark_tf_gke_amd.distribute.cluster import Server, build_cluster_def


def parse_role(hostname: str):
    m = re.search(r"-(\d+)$", hostname or "")
    ordinal = int(m.group(1)) if m else 0
    return ("ps" if "-ps-" in (hostname or "") else "worker"), ordinal


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--block", action="store_true", help="park forever like the reference pods")
    a = ap.parse_args(argv)
    role, idx = parse_role(os.environ.get("HOSTNAME", ""))
    workers = int(os.environ.get("WORKER_REPLICAS", "1"))
    ps = int(os.environ.get("PS_REPLICAS", "1"))
    port = int(os.environ.get("TF_GRPC_PORT", "2222"))
    cluster = build_cluster_def(workers, ps, port, "", "", "", 2223)
    server = Server(cluster, job_name=role, task_index=idx, protocol="grpc")
    print(f"Starting tf.distribute.Server role={role} index={idx} target={server.target}", flush=True)
    server.join(block=a.block)


if __name__ == "__main__":
    main()
