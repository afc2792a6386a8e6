#!/usr/bin/env python
"""RCCL (backend "nccl") check on >= 2 GPUs, one rank per GPU — what the 8-GPU node runs:

* DataFrame groupBy of synthetic (key, value) rows: partial aggregate -> RCCL all-to-all-v shuffle
  -> final aggregate; every key lands on exactly one rank and count / sum match the totals;
* orderBy: sample-based range shuffle + local radix sort is globally ordered across ranks;
* MultiWorkerMirroredStrategy: sharded update (reduce-scatter / sharded Adam / all-gather) ==
  all-reduce update;
* ParameterServerStrategy (sync) on the same data keeps every rank's parameters identical.

Launch: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 tools/rccl_check.py
(writes $PTG_RCCL_OUT/rank<r>.json).
"""
import json
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    from pyspark_tf_gke_amd.distribute import MultiWorkerMirroredStrategy
    from pyspark_tf_gke_amd.models import build_cnn_model
    from pyspark_tf_gke_amd.ops import df as D
    from pyspark_tf_gke_amd.parallel import comm
    from pyspark_tf_gke_amd.sql import SparkSession
    from pyspark_tf_gke_amd.sql import functions as F
    from pyspark_tf_gke_amd.sql import types as T
    from pyspark_tf_gke_amd.sql.dataframe import DataFrame
    from pyspark_tf_gke_amd.sql.table import ColumnVector, Table

    st_s = MultiWorkerMirroredStrategy(sharded_update=True, bucket_mb=1.0)
    if os.environ.get("PTG_RCCL_ALLOW_GLOO") != "1":  # CPU rehearsal of this script: gloo
        assert torch.distributed.get_backend() == "nccl"
    rank, world = st_s.rank, st_s.world_size
    dev = st_s.device
    out = {"rank": rank, "world": world}
    # ---- groupBy over RCCL all-to-all-v
    spark = SparkSession.builder.master("mi355x").getOrCreate()
    n = int(os.environ.get("PTG_RCCL_ROWS", "4000000"))
    k, v = D.fill_synthetic_kv(n, 300_000, dev, offset=rank * n, seed=5)
    df = DataFrame(Table({"key": ColumnVector(k, T.LongType()), "value": ColumnVector(v, T.DoubleType())}, n, dev),
                   spark)
    g = df.groupBy("key").agg(F.sum("value").alias("s"), F.count("*").alias("c"))
    keys = g._t.column("key").data
    allk = torch.cat(comm.all_gather_v(keys))
    cnt = comm.all_reduce_int([int(g._t.column("c").data.sum().item())])[0]
    tot = comm.all_reduce_float([float(g._t.column("s").data.sum().item())])[0]
    want = comm.all_reduce_float([float(v.sum().item())])[0]
    out["groupby_ok"] = bool(allk.numel() == torch.unique(allk).numel() and cnt == n * world
                             and abs(tot - want) <= 1e-9 * n * world)
    # ---- orderBy
    o = df.orderBy(F.col("value").desc())
    col = o._t.column("value").data
    local_ok = bool((col[1:] <= col[:-1]).all().item()) if col.numel() > 1 else True
    ends = torch.tensor([col[0].item() if col.numel() else float("inf"), col[-1].item() if col.numel() else
                         float("-inf")], dtype=torch.float64, device=dev)
    allends = torch.cat(comm.all_gather_v(ends.view(1, 2))).cpu().tolist()
    chain = all(allends[r][1] >= allends[r + 1][0] for r in range(world - 1) if allends[r + 1][0] != float("inf"))
    out["orderby_ok"] = bool(comm.all_reduce_int([int(not local_ok)])[0] == 0 and chain
                             and comm.all_reduce_int([o._t.num_rows])[0] == n * world)
    del df, g, o, k, v
    # ---- MWMS sharded vs all-reduce
    st_p = MultiWorkerMirroredStrategy(sharded_update=False)
    gen = torch.Generator().manual_seed(100 + rank)
    X = torch.rand(3, 8, 64, 80, 3, generator=gen)
    Y = torch.rand(3, 8, 2, generator=gen) * 60
    models = {}
    for name, st in (("sharded", st_s), ("plain", st_p)):
        torch.manual_seed(0)
        with st.scope():
            models[name] = build_cnn_model((64, 80, 3), flat=True, summary=False, device=dev)
    ms, mp = models["sharded"], models["plain"]
    for i in range(3):
        for m in (ms, mp):
            xb, yb = m._prep_batch(X[i], Y[i])
            stats = m._stats_buf()
            stats.zero_()
            m.train_step_fast(xb, yb, stats)
    st_s.synchronize_master(ms)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    diff = max(float((p.data - mp.store.by_name(p.name).data).abs().max()) for p in ms.store.params)
    scale = max(float(p.data.abs().max()) for p in mp.store.params)
    out["mwms_diff"] = diff
    out["mwms_ok"] = diff <= 1e-4 * max(1.0, scale)
    # ---- parameter server (sync) keeps replicas identical
    from pyspark_tf_gke_amd import nn
    from pyspark_tf_gke_amd.cli.train import _ps_loop, make_parameter_server_strategy
    from pyspark_tf_gke_amd.data import Dataset
    from pyspark_tf_gke_amd.models import build_deep_model
    import numpy as np

    ps = make_parameter_server_strategy(world, 1, chief_addr="127.0.0.1")
    rng = np.random.default_rng(0)
    Xc = rng.normal(size=(512, 3)).astype(np.float32)
    yc = (Xc[:, 0] > 0).astype(np.int32)

    def ds_fn(ctx=None):
        ds = Dataset.from_tensor_slices((Xc, yc))
        if ctx is not None:
            ds = ds.shard(ctx.num_input_pipelines, ctx.input_pipeline_id)
        return ds.shuffle(100, seed=1).batch(16).repeat()

    with ps.scope():
        mm = build_deep_model(3, 2, device=dev)
        opt = nn.optimizers.Adam(1e-2)
        metrics = [nn.metrics.Mean("loss"), nn.metrics.SparseCategoricalAccuracy("accuracy")]
    h = _ps_loop(mm, ps, ds_fn, 5, 2, nn.losses.SparseCategoricalCrossentropy(), opt, metrics, lambda e, v: str(v))
    s = torch.tensor([float(mm.store.flat.double().sum())], dtype=torch.float64, device=dev)
    sums = torch.cat(comm.all_gather_v(s)).cpu().tolist()
    out["ps_ok"] = bool(len(set(sums)) == 1 and h["loss"][-1] == h["loss"][-1])
    out["ok"] = bool(out["groupby_ok"] and out["orderby_ok"] and out["mwms_ok"] and out["ps_ok"])
    od = os.environ.get("PTG_RCCL_OUT")
    if od:
        with open(os.path.join(od, f"rank{rank}.json"), "w") as fh:
            json.dump(out, fh)
    print("RCCL " + json.dumps(out), flush=True)
    comm.destroy()
    return 0 if out["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
