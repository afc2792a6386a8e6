#!/usr/bin/env python
"""Multi-rank rehearsal of the data-parallel training path on ONE GPU (every rank on cuda:0, gloo
collectives staged through the host): the sharded update (reduce-scatter / sharded Adam / bf16 +
fp32 all-gather waited per forward op) must give the same parameters as the all-reduce update, with
the real HIP kernels in the loop.  Launch:

    PTG_DIST_BACKEND=gloo python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        tools/rehearse_multirank.py
"""
import json
import os
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from pyspark_tf_gke_amd.distribute import MultiWorkerMirroredStrategy  # noqa: E402
from pyspark_tf_gke_amd.models import build_cnn_model  # noqa: E402


def main():
    st_s = MultiWorkerMirroredStrategy(sharded_update=True, bucket_mb=1.0)
    st_p = MultiWorkerMirroredStrategy(sharded_update=False)
    dev = st_s.device
    g = torch.Generator().manual_seed(100 + st_s.rank)
    X = torch.rand(3, 8, 64, 80, 3, generator=g)
    Y = torch.rand(3, 8, 2, generator=g) * 60
    models = {}
    for name, st in (("sharded", st_s), ("plain", st_p)):
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
    torch.cuda.synchronize()
    diff = max(float((p.data - mp.store.by_name(p.name).data).abs().max()) for p in ms.store.params)
    bdiff = max(float((p.bf16.float() - mp.store.by_name(p.name).bf16.float()).abs().max()) for p in ms.store.params)
    scale = max(float(p.data.abs().max()) for p in mp.store.params)
    out = {"rank": st_s.rank, "world": st_s.world_size, "buckets": len(ms._shard_plan.buckets), "diff": diff,
           "bf16_diff": bdiff, "scale": scale, "ok": diff <= 1e-4 * max(1.0, scale)}
    print("REHEARSAL " + json.dumps(out), flush=True)
    out_dir = os.environ.get("PTG_REHEARSE_OUT")
    if out_dir:  # ranks share stdout: lines can interleave, so the test reads one file per rank
        with open(os.path.join(out_dir, f"rank{st_s.rank}.json"), "w") as fh:
            json.dump(out, fh)
    return 0 if out["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
