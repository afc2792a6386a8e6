"""Repeat the sharded-vs-replicated 4-step comparison (tests/test_dist_gpu.py RCCL_BODY) many times in
one process to find a rare mismatch, and localise it: sharded vs sharded, fused vs fused, and
sharded vs fused, each pair over the same batches.  Prints one JSON line per repetition with the
max-abs parameter difference of each pair and, for any pair above 1e-4, the parameter, element and
values.  Same env as tools/diag_shard_grads.py (1-rank RCCL group)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pyspark_tf_gke_amd.distribute import MultiWorkerMirroredStrategy  # noqa: E402
from pyspark_tf_gke_amd.models import build_cnn_model  # noqa: E402

REPS = int(os.environ.get("DIAG_REPS", "12"))
STEPS = 4
st_s = MultiWorkerMirroredStrategy(sharded_update=True, bucket_mb=1.0)
st_p = MultiWorkerMirroredStrategy(sharded_update=False)
dev = st_s.device
g = torch.Generator().manual_seed(11)
X = torch.rand(STEPS, 16, 64, 80, 3, generator=g)
Y = torch.rand(STEPS, 16, 2, generator=g) * 60


def worst(ma, mb):
    best = (0.0, None, None, None, None)
    for p in ma.store.params:
        q = mb.store.by_name(p.name)
        d = (p.data.float() - q.data.float()).abs().reshape(-1)
        i = int(d.argmax())
        if float(d[i]) > best[0]:
            best = (float(d[i]), p.name, i, float(p.data.reshape(-1)[i]), float(q.data.reshape(-1)[i]))
    return best


for rep in range(REPS):
    models = {}
    for name, st in (("s1", st_s), ("s2", st_s), ("f1", st_p), ("f2", st_p)):
        with st.scope():
            models[name] = build_cnn_model((64, 80, 3), flat=True, summary=False, device=dev)
    for i in range(STEPS):
        for name, m in models.items():
            xb, yb = m._prep_batch(X[i], Y[i])
            stats = m._stats_buf()
            stats.zero_()
            m.train_step_fast(xb, yb, stats)
    for name in ("s1", "s2"):
        st_s.synchronize_master(models[name])
    torch.cuda.synchronize()
    out = {"rep": rep}
    for a, b in (("s1", "s2"), ("f1", "f2"), ("s1", "f1"), ("s2", "f2")):
        w = worst(models[a], models[b])
        out[a + b] = w[0]
        if w[0] > 1e-4:
            out[a + b + "_at"] = w[1:]
    print("REP", json.dumps(out), flush=True)
print("DONE", flush=True)
