"""Cluster description: ClusterSpec, TF_CONFIG, resolvers, partitioner, InputContext.

Keeps the reference's user-facing address/port surface (train_tf_ps.py:385-511,
tf-trainer-worker.yaml:43-68): ``build_cluster_def`` produces the same
``{"worker": [...], "ps": [...], "chief": [...]}`` dict (explicit addresses win, otherwise the
headless-service DNS names), chief addresses are validated as strict IPv4, and ``TF_CONFIG`` is
parsed/produced in the same JSON form.  On one 8xMI355X node these addresses are configuration
only: the roles map onto local ranks (rank r = worker r = PS shard r) and tensors move over RCCL.
"""
from __future__ import annotations

import math

import json
import os
from dataclasses import dataclass


def build_cluster_def(worker_replicas: int, ps_replicas: int, port: int, worker_addrs=None, ps_addrs=None,
                      chief_addr=None, chief_port: int = 2223) -> dict:
    """Same contract as the reference's ``build_cluster_def`` (train_tf_ps.py:385-437)."""
    if worker_addrs:
        workers = list(worker_addrs)
    else:
        workers = [f"tf-trainer-{i}.tf-trainer-worker-headless:{port}" for i in range(worker_replicas)]
    cluster = {"worker": workers}
    if ps_replicas > 0:
        cluster["ps"] = list(ps_addrs) if ps_addrs else [
            f"tf-trainer-ps-{i}.tf-trainer-ps-headless:{port}" for i in range(ps_replicas)]
    if chief_addr:
        cluster["chief"] = [f"{chief_addr}:{chief_port}"]
    return cluster


def validate_chief_addr(chief_addr: str) -> None:
    """Strict IPv4 validation of the coordinator address (train_tf_ps.py:474-490)."""
    if ":" in chief_addr and "." not in chief_addr:
        raise RuntimeError(f"chief_addr appears to be IPv6 ('{chief_addr}'). Please provide an IPv4 address.")
    if any(sym in chief_addr for sym in ["/", "[", "]", " "]):
        raise RuntimeError(f"chief_addr '{chief_addr}' is malformed. Provide a raw IPv4 like 192.168.1.10.")
    parts = chief_addr.split(".")
    if len(parts) != 4 or any(not p.isdigit() or not (0 <= int(p) <= 255) for p in parts):
        raise RuntimeError(f"chief_addr '{chief_addr}' is not a valid IPv4 address.")


class ClusterSpec:
    def __init__(self, cluster):
        if isinstance(cluster, ClusterSpec):
            cluster = cluster.as_dict()
        self._c = {k: list(v) for k, v in dict(cluster).items()}

    def as_dict(self) -> dict:
        return {k: list(v) for k, v in self._c.items()}

    @property
    def jobs(self):
        return list(self._c)

    def num_tasks(self, job: str) -> int:
        return len(self._c.get(job, []))

    def task_address(self, job: str, index: int) -> str:
        return self._c[job][index]

    def __repr__(self):
        return f"ClusterSpec({json.dumps(self._c)})"


class SimpleClusterResolver:
    def __init__(self, cluster_spec: ClusterSpec, task_type: str | None = None, task_id: int = 0,
                 rpc_layer: str = "grpc", num_accelerators=None):
        self._spec = ClusterSpec(cluster_spec)
        self.task_type = task_type
        self.task_id = task_id
        self.rpc_layer = rpc_layer

    def cluster_spec(self) -> ClusterSpec:
        return self._spec


class TFConfigClusterResolver(SimpleClusterResolver):
    """Reads ``TF_CONFIG`` (``{"cluster": ..., "task": {"type": ..., "index": ...}}``)."""

    def __init__(self, rpc_layer: str = "grpc"):
        cfg = json.loads(os.environ.get("TF_CONFIG", "{}") or "{}")
        task = cfg.get("task", {})
        super().__init__(ClusterSpec(cfg.get("cluster", {})), task.get("type"), int(task.get("index", 0)),
                         rpc_layer)


def make_tf_config(cluster: dict, task_type: str, index: int = 0) -> str:
    return json.dumps({"cluster": cluster, "task": {"type": task_type, "index": index}})


@dataclass
class InputContext:
    """``tf.distribute.InputContext``: which input pipeline this worker runs (train_tf_ps.py:596-600)."""

    num_input_pipelines: int = 1
    input_pipeline_id: int = 0
    num_replicas_in_sync: int = 1

    def get_per_replica_batch_size(self, global_batch_size: int) -> int:
        if global_batch_size % self.num_replicas_in_sync:
            raise ValueError("global batch size must divide evenly across replicas")
        return global_batch_size // self.num_replicas_in_sync


class MinSizePartitioner:
    """``tf.distribute.experimental.partitioners.MinSizePartitioner`` (train_tf_ps.py:505-507):
    a variable is cut along axis 0 into as many shards as keep every shard >= ``min_shard_bytes``
    (whole rows per shard), at most ``max_shards``.  TF's rule (min_max_variable_partitioner):
    slices_per_shard = max(1, ceil(min_shard_bytes / bytes_per_row)); shards = min(max_shards,
    ceil(rows / slices_per_shard)).  :class:`~.strategy.ParameterServerStrategy` places each shard
    on a PS task round-robin, the way TF's variable placement does."""

    def __init__(self, min_shard_bytes: int = 256 << 10, max_shards: int = 1, bytes_per_string: int = 16):
        self.min_shard_bytes = int(min_shard_bytes)
        self.max_shards = max(1, int(max_shards))

    def num_shards(self, shape, dtype_size: int = 4) -> int:
        shape = tuple(int(s) for s in shape) or (1,)
        rows = max(shape[0], 1)
        n = 1
        for s in shape:
            n *= s
        bytes_per_row = n * dtype_size / rows
        if bytes_per_row <= 0:
            return 1
        slices_per_shard = max(1, math.ceil(self.min_shard_bytes / bytes_per_row))
        return max(1, min(self.max_shards, math.ceil(rows / slices_per_shard)))

    def __call__(self, shape, dtype_size: int = 4):
        return [self.num_shards(shape, dtype_size)] + [1] * (len(tuple(shape)) - 1)


class Server:
    """``tf.distribute.Server`` stand-in (tf-trainer-worker.yaml:65): in this runtime worker and PS
    roles are GPU ranks spawned by the launcher, so a Server only records its role; ``join()``
    returns immediately unless ``block=True`` (then it parks like the reference pods)."""

    def __init__(self, cluster_spec, job_name: str, task_index: int = 0, protocol: str = "grpc", start=True):
        self.cluster_spec = ClusterSpec(cluster_spec)
        self.job_name = job_name
        self.task_index = task_index
        self.protocol = protocol
        self.target = f"{protocol}://{self.cluster_spec.task_address(job_name, task_index)}" \
            if self.cluster_spec.num_tasks(job_name) > task_index else ""

    def join(self, block: bool = False):
        if block:
            import time

            while True:
                time.sleep(3600)
