"""Typed runtime configuration: one registry for every framework knob.

The reference mixes argparse-with-env-defaults (train_tf_ps.py:822-840), raw env vars
(spark_session.py:44-50, k_means.py:57,186) and Spark ``--conf`` / builder ``.config()`` keys.  The
user-facing names of those stay where they are (the CLIs keep the reference's flags and env names).
Everything this framework adds is declared here once, with its type, default, env var and
``spark.ptg.*`` conf key, and resolved with a fixed precedence:

    CLI override (:func:`set_cli`)  >  environment variable  >  Spark conf (the active session's
    ``.config()`` / ``spark-submit --conf``, :func:`register_conf`; ``PTG_SPARK_CONF`` JSON)  >  default

``python -m pyspark_tf_gke_amd.config`` prints the table with the value each knob resolves to.
Knobs read at import time (the ``nn`` step switches) see the CLI, the environment and
``PTG_SPARK_CONF``; session confs set later apply to knobs read at call time (groupBy, shuffle).
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass
from typing import Any

_FALSE = ("0", "false", "no", "off", "")


@dataclass(frozen=True)
class Knob:
    name: str
    type: type
    default: Any
    env: str | None
    conf: str | None
    doc: str

    def parse(self, raw: Any) -> Any:
        if self.type is bool:
            return raw if isinstance(raw, bool) else str(raw).strip().lower() not in _FALSE
        if raw is None or (isinstance(raw, str) and raw == "" and self.type is not str):
            return self.default
        return self.type(raw)


_K = [
    # data engine
    Knob("groupby_range", bool, True, "PTG_GROUPBY_RANGE", "spark.ptg.groupby.range",
         "dense small-range integer keys take the one-pass range partition + direct LDS aggregation"),
    Knob("groupby_small_blocks", int, 1024, "PTG_GROUPBY_SMALL_BLOCKS", None,
         "workgroups of the tiny-key-range groupBy pass (small_range_agg_k; each writes one dense partial table)"),
    Knob("groupby_range2", bool, True, "PTG_GROUPBY_RANGE2", "spark.ptg.groupby.range2",
         "dense integer keys spanning 2^20..2^28 values: two 256-way range partitioning passes + direct LDS aggregation"),
    Knob("groupby_range_chunks", int, 8, "PTG_RANGE_CHUNKS", "spark.ptg.groupby.rangeChunks",
         "row chunks per range partition in the range aggregation (workgroups = 256 x chunks)"),
    Knob("groupby_hash9", bool, True, "PTG_GROUPBY_HASH9", "spark.ptg.groupby.hash9",
         "sparse keys at ~64K..1.3M groups: one 512-way hash partition + LDS hash tables (sum/count/avg, <= 2 columns)"),
    Knob("groupby_h9_chunks", int, 4, "PTG_H9_CHUNKS", "spark.ptg.groupby.h9Chunks",
         "row chunks per partition in the 512-way hash aggregation (workgroups = 512 x chunks)"),
    Knob("shuffle_buffer_gb", float, 64.0, "PTG_SHUFFLE_BUFFER_GB", "spark.ptg.shuffle.buffer.gb",
         "HBM staging budget of one all-to-all-v shuffle round"),
    Knob("device", str, "", "PTG_DEVICE", "spark.ptg.device", "executor device: cuda / cpu (default: cuda if present)"),
    Knob("jdbc_root", str, "", "PTG_JDBC_ROOT", None, "directory of the SQLite files behind jdbc: URLs"),
    Knob("fault_task", int, 0, "PTG_FAULT_TASK", None, "fault injection: fail this many stage-task attempts"),
    # training step
    Knob("fused_adam", bool, True, "PTG_FUSED_ADAM", None, "Adam inside the big Dense weight-gradient GEMM epilogue (1 GPU)"),
    Knob("flip_in_adam", bool, True, "PTG_FLIP_IN_ADAM", None,
         "the fused step's Adam pass writes the conv layers' flipped dgrad filters for the next backward "
         "(no flip kernel in the step); 0 = flip at the start of every backward"),
    Knob("mlp_fused", bool, True, "PTG_MLP_FUSED", None,
         "a model that is only a small Dense stack (the CSV MLP) runs each training step as ONE kernel (mlp.hip)"),
    Knob("fused_head", bool, True, "PTG_FUSED_HEAD", None, "CNN-B1 Dense(relu)->Dense->MSE head as two kernels"),
    Knob("device_feed", bool, True, "PTG_DEVICE_FEED", None, "fit(): pinned ring + side-stream H2D for host datasets"),
    Knob("side_stream", bool, True, "PTG_SIDE_STREAM", None, "weight gradients on a side HIP stream (1 replica)"),
    Knob("adam_stream", bool, True, "PTG_ADAM_STREAM", None,
         "the big Dense dW+Adam on a second side stream (the conv weight gradients do not queue behind it)"),
    Knob("sort_value_payload", bool, True, "PTG_SORT_VALUE_PAYLOAD", None,
         "orderBy of a (key, one 8-byte column) table carries the column through the radix passes"),
    Knob("sort_fused_keys", bool, True, "PTG_SORT_FUSED_KEYS", None,
         "orderBy on an int64 column: orderable-key transform inside the first / last radix pass"),
    Knob("fork_device_events", bool, True, "PTG_FORK_DEVICE_EVENTS", None,
         "side-stream fork/join through device-scope events (no system-scope cache flush per fork)"),
    Knob("tape_overlap", bool, True, "PTG_TAPE_OVERLAP", None,
         "GradientTape loops: big Dense Adam on an aux stream overlapping the rest of the backward"),
    Knob("tape_fused_head", bool, True, "PTG_TAPE_FUSED_HEAD", None,
         "GradientTape loops: an MSE loss on a [Dense(relu), Dense(<=4)] tail runs the fused head kernels"),
    Knob("tape_lazy_dw", bool, True, "PTG_TAPE_LAZY_DW", None,
         "GradientTape loops: big Dense dW deferred to apply_gradients and fused with Adam (computed on first read)"),
    Knob("raw_u8_input", bool, True, "PTG_RAW_U8_INPUT", None, "first conv reads the uint8 image batch directly"),
    Knob("sparse_first", bool, True, "PTG_SPARSE_FIRST", None, "first conv layer keeps a sparse pool record"),
    Knob("sparse_pool", bool, True, "PTG_SPARSE_POOL", None,
         "pooled 5x5 conv layers after the first (CNN-B1 layers 2-3) keep only the sparse pool record: the "
         "forward writes z at the window argmax + the argmax, the PReLU/pool backward writes dZ at the argmax, "
         "and the weight and data gradients expand it in their halo loaders (no full-resolution z or dZ). "
         "b256 A/B: 1.4044/1.4018 vs 1.4300/1.4257 ms (profiles/r6_ab_sparse_pool_record.txt)"),
    Knob("sparse_pool_min_batch", int, 128, "PTG_SPARSE_POOL_MIN_BATCH", None,
         "sparse_pool only from this batch size (b64: 0.6958/0.6841 vs 0.6848/0.6801 ms, b32 within noise)"),
    Knob("bn_relu_bits", bool, True, "PTG_BN_RELU_BITS", None,
         "residual BN + ReLU: the backward reads a 1-bit ReLU mask written by the forward instead of y"),
    Knob("bn_bwd_epi_stats", bool, True, "PTG_BN_BWD_EPI_STATS", None,
         "ResNet: the BN backward sums of a Conv->BN->ReLU block come from the epilogue of the dgrad that produces its gradient (no bn_bwd_reduce pass)"),
    Knob("bn_epi_stats", bool, True, "PTG_BN_EPI_STATS", None, "ResNet: BN batch statistics from the conv GEMM epilogue (A/B: 9.00k vs 8.78k img/s with the shuffle flush)"),
    Knob("conv32", bool, True, "PTG_CONV32", None,
         "5x5 convs with C, Cout in 16..64 (CNN-B1 layers 4-5 and their data gradients, see conv32_min_ch): the "
         "32x32x16-MFMA implicit GEMM of conv32.hip instead of the halo strip kernels (b256 A/B: 1.652/1.649 vs "
         "1.657/1.650 ms; on layer 3 as well: 1.80 ms)"),
    Knob("conv32_min_ch", int, 32, "PTG_CONV32_MINCH", None,
         "conv32 only where min(C, Cout) >= this (layer bench: it wins on CNN-B1 layers 4-5, loses the 32->16 dgrad)"),
    Knob("conv32_min_wg", int, 64, "PTG_CONV32_MINWG", None,
         "conv32 only when its grid (N x H / rows-per-tile workgroups) has at least this many workgroups "
         "(64 since the 160-px small-grid tiles: CNN-B1 b64 0.7057/0.7058 vs 0.7214/0.7106 ms at 128, which "
         "keeps layer 5 on the strip kernel; b32 at 0 loses, 0.562/0.559 vs 0.556/0.554 ms)"),
    Knob("conv1_rec", bool, True, "PTG_CONV1_REC", None, "first conv layer (conv1.hip): forward keeps the pool record, backward needs no recompute (0: recompute z in the backward)"),
    Knob("conv1_fused", bool, True, "PTG_CONV1_FUSED", None, "first conv layer: pooled-only forward + one recomputing backward kernel (conv1.hip)"),
    Knob("dense_fwd_splits", int, 0, "PTG_DENSE_FWD_SPLITS", None,
         "0: the big Dense forward streams its weight through dense.hip (split-K partial slices, plain stores); "
         ">0: the atomic split-K MFMA GEMM with this many splits (A/B)"),
    Knob("blaslt_dx", bool, False, "PTG_BLASLT_DX", None,
         "A/B only: big-Dense dX through hipBLASLt instead of dense.hip's weight-streaming kernel"),
    Knob("hip_graph", bool, False, "PTG_HIP_GRAPH", None, "capture the training step in a HIP graph (jit_compile)"),
    Knob("host_fp32", bool, False, "PTG_HOST_FP32", None, "CPU tensors: fp32 reference path everywhere"),
    Knob("seed", int, 1337, "PTG_SEED", None, "weight-initialisation seed when none is given"),
    # distribution
    Knob("dist_backend", str, "", "PTG_DIST_BACKEND", None, "torch.distributed backend override (default nccl=RCCL / gloo)"),
    Knob("force_pg", bool, False, "PTG_FORCE_PG", None,
         "create the process group even for one rank (a 1-rank RCCL group: the collective code paths run for real)"),
    Knob("collectives_world1", bool, False, "PTG_COLLECTIVES_WORLD1", None,
         "with a 1-rank process group (PTG_FORCE_PG): take the multi-rank code paths, so every collective "
         "(shuffles, range sort, PS rounds, KMeans sums, string unification) runs through the backend"),
    Knob("shard_world1", bool, False, "PTG_SHARD_WORLD1", None,
         "MWMS on one rank with a process group: build the sharded update anyway (RCCL reduce-scatter / all-gather "
         "of one rank through the side streams; a test of the N>1 path on one GPU)"),
    Knob("pg_timeout_s", float, 600.0, "PTG_PG_TIMEOUT", None, "process-group collective timeout (hang -> error -> restart)"),
    Knob("bucket_mb", float, 64.0, "PTG_BUCKET_MB", None, "MWMS gradient bucket size"),
    Knob("sharded_update", bool, True, "PTG_SHARDED_UPDATE", None, "MWMS: reduce-scatter + sharded optimizer + all-gather"),
    Knob("sim_world", int, 0, "PTG_SIM_WORLD", None,
         "1-rank MWMS runs rank 0's kernel sequence of an N-rank sharded update (collectives -> local kernels)"),
    Knob("sim_exact", bool, False, "PTG_SIM_EXACT", None,
         "sim_world: also apply the peers' shard updates (exact numerics of N identical-data ranks, N x the Adam work)"),
    Knob("persist_dynamic", bool, False, "PTG_PERSIST_DYNAMIC", None, "persistent conv kernels in work-queue mode for N > 1"),
    Knob("ps_mode", str, "sync", "PTG_PS_MODE", None, "ParameterServerStrategy: sync or async"),
    Knob("coord_dead_s", float, 60.0, "PTG_COORD_DEAD_S", None,
         "async ClusterCoordinator: a worker whose liveness beat is this old has its drawn-but-unfinished "
         "closures re-queued for the others"),
    Knob("coord_stall_s", float, 0.0, "PTG_COORD_STALL_S", None,
         "async ClusterCoordinator: fail every rank's join when no closure finished and no live worker ran "
         "one for this long (0: PTG_PG_TIMEOUT)"),
    Knob("ipc_allreduce", bool, False, "PTG_IPC_ALLREDUCE", None, "one-shot IPC all-reduce for small messages"),
    Knob("fault_rank", str, "", "PTG_FAULT_RANK", None, "fault injection: rank to kill"),
    Knob("fault_step", int, 1, "PTG_FAULT_STEP", None, "fault injection: step at which fault_rank dies"),
    Knob("heartbeat_dir", str, "", "PTG_HEARTBEAT_DIR", None, "progress heartbeat files for the launcher's hang detector"),
    # native code / observability
    Knob("checked", bool, False, "PTG_CHECKED", None, "load the bounds-checked kernel library"),
    Knob("hip_lib", str, "", "PTG_HIP_LIB", None, "in-tree kernel library variant to load (A/B runs)"),
    Knob("roctx", bool, True, "PTG_ROCTX", None, "roctx ranges around steps"),
    Knob("metrics_jsonl", str, "", "PTG_METRICS_JSONL", None, "per-step metrics JSONL path"),
    Knob("log_all_ranks", bool, False, "PTG_LOG_ALL_RANKS", None, "INFO logs from every rank, not only rank 0"),
]
KNOBS: dict[str, Knob] = {k.name: k for k in _K}

_cli: dict[str, Any] = {}
_confs: list[dict] = []


def set_cli(name: str, value: Any) -> None:
    """A command-line value: highest precedence."""
    _cli[KNOBS[name].name] = value


def register_conf(conf: dict | None) -> None:
    """Spark conf of the active session (``SparkSession.builder.config`` / ``spark.conf.set``, read
    live); ``None`` when the session stops."""
    _confs[:] = [conf] if conf is not None else []


def _submitted_conf() -> dict:
    raw = os.environ.get("PTG_SPARK_CONF")
    try:
        return json.loads(raw) if raw else {}
    except ValueError:
        return {}


def source(name: str) -> str:
    k = KNOBS[name]
    if k.name in _cli:
        return "cli"
    if k.env and os.environ.get(k.env) is not None:
        return "env"
    if k.conf and (any(k.conf in c for c in _confs) or k.conf in _submitted_conf()):
        return "conf"
    return "default"


def get(name: str) -> Any:
    k = KNOBS[name]
    if k.name in _cli:
        return k.parse(_cli[k.name])
    if k.env:
        raw = os.environ.get(k.env)
        if raw is not None:
            return k.parse(raw)
    if k.conf:
        for c in reversed(_confs):
            if k.conf in c:
                return k.parse(c[k.conf])
        sub = _submitted_conf()
        if k.conf in sub:
            return k.parse(sub[k.conf])
    return k.default


def describe() -> list[dict]:
    return [{"name": k.name, "type": k.type.__name__, "value": get(k.name), "source": source(k.name),
             "env": k.env, "conf": k.conf, "default": k.default, "doc": k.doc} for k in _K]


if __name__ == "__main__":
    for r in describe():
        print(f"{r['name']:22s} {r['type']:5s} {str(r['value']):10s} [{r['source']:7s}] "
              f"env={r['env'] or '-'} conf={r['conf'] or '-'}  {r['doc']}")
