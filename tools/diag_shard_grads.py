"""Diagnose sharded-vs-replicated MWMS update differences.

Runs four CNN-B1 (64x80) models side by side on one GPU through a real 1-rank RCCL group:
  sharded   - MultiWorkerMirroredStrategy(sharded_update=True): per-bucket reduce-scatter from the
              side stream, apply_shard, async all-gather;
  sharded2  - the same again (run-to-run noise of the sharded path);
  unfused   - replicated update with the big-Dense Adam NOT fused into its dW GEMM (flat_grad is
              materialised, so its gradients can be compared);
  unfused2  - the same again (run-to-run noise of the unfused path);
  fused     - the default replicated path (EpiAdam in the dW GEMM, adam_multi_k).
Per step it prints, per parameter, the relative L2 difference of the pre-optimizer gradients
(sharded vs unfused, unfused vs unfused2), and after every step the parameter max-abs differences
and how many elements differ by more than 1e-4.

Run: PTG_FORCE_PG=1 PTG_SHARD_WORLD1=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1
     MASTER_PORT=29661 python tools/diag_shard_grads.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pyspark_tf_gke_amd.distribute import MultiWorkerMirroredStrategy  # noqa: E402
from pyspark_tf_gke_amd.models import build_cnn_model  # noqa: E402
from pyspark_tf_gke_amd.nn import model as M  # noqa: E402

STEPS = int(os.environ.get("DIAG_STEPS", "4"))
st_s = MultiWorkerMirroredStrategy(sharded_update=True, bucket_mb=1.0)
st_s2 = MultiWorkerMirroredStrategy(sharded_update=True, bucket_mb=1.0)
st_p = MultiWorkerMirroredStrategy(sharded_update=False)
dev = st_s.device
g = torch.Generator().manual_seed(11)
X = torch.rand(STEPS, 16, 64, 80, 3, generator=g)
Y = torch.rand(STEPS, 16, 2, generator=g) * 60

names = ["sharded", "sharded2", "unfused", "unfused2", "fused"]
strat = {"sharded": st_s, "sharded2": st_s2, "unfused": st_p, "unfused2": st_p, "fused": st_p}
models = {}
for n in names:
    with strat[n].scope():
        models[n] = build_cnn_model((64, 80, 3), flat=True, summary=False, device=dev)
grads = {n: {} for n in names}


def hook_shard(name):
    m = models[name]
    opt = m.optimizer
    orig = opt.apply_shard

    def f(store, gsh, lo, hi, gscale=1.0, advance=True):
        grads[name][lo] = (hi, (gsh.float() * gscale).clone())
        return orig(store, gsh, lo, hi, gscale=gscale, advance=advance)

    opt.apply_shard = f


def hook_apply(name):
    m = models[name]
    opt = m.optimizer
    orig = opt.apply

    def f(store, gscale=1.0, lo=0, hi=None, advance=True):
        hi2 = store.total if hi is None else hi
        grads[name][lo] = (hi2, (store.flat_grad[lo:hi2].float() * gscale).clone())
        return orig(store, gscale=gscale, lo=lo, hi=hi, advance=advance)

    opt.apply = f


for n in ("sharded", "sharded2"):
    hook_shard(n)
for n in ("unfused", "unfused2"):
    hook_apply(n)


def param_grad(name, p):
    """p's gradient (flattened) from the captured ranges of model ``name``."""
    for lo, (hi, t) in grads[name].items():
        if lo <= p.offset and p.offset + p.numel <= hi:
            return t[p.offset - lo:p.offset - lo + p.numel]
    return None


def pdiff(a, b):
    out = {}
    for p in models[a].store.params:
        q = models[b].store.by_name(p.name)
        d = (p.data.float() - q.data.float()).abs()
        out[p.name] = (float(d.max()), int((d > 1e-4).sum()))
    return out


for i in range(STEPS):
    for n in names:
        m = models[n]
        grads[n].clear()
        old = M.FUSED_ADAM
        M.FUSED_ADAM = n == "fused"
        try:
            xb, yb = m._prep_batch(X[i], Y[i])
            stats = m._stats_buf()
            stats.zero_()
            m.train_step_fast(xb, yb, stats)
        finally:
            M.FUSED_ADAM = old
        torch.cuda.synchronize()
        m._diag_loss = float(stats[0] / stats[4])
    for n in ("sharded", "sharded2"):
        st = strat[n]
        st.wait_parameters(models[n])
    torch.cuda.synchronize()
    rep = {"step": i, "loss": {n: models[n]._diag_loss for n in names}, "grad_rel": {}}
    for p in models["unfused"].store.params:
        gu = param_grad("unfused", p)
        gu2 = param_grad("unfused2", models["unfused2"].store.by_name(p.name))
        gs = param_grad("sharded", models["sharded"].store.by_name(p.name))
        gs2 = param_grad("sharded2", models["sharded2"].store.by_name(p.name))
        nrm = float(gu.norm()) if gu is not None else float("nan")

        def rel(a, b):
            if a is None or b is None:
                return None
            return float((a - b).norm()) / max(nrm, 1e-30)

        def amax(a, b):
            if a is None or b is None:
                return None
            return float((a - b).abs().max())

        rep["grad_rel"][p.name] = {"norm": nrm, "s_vs_u": rel(gs, gu), "u_vs_u2": rel(gu, gu2),
                                   "s_vs_s2": rel(gs, gs2), "s_vs_u_max": amax(gs, gu), "u_vs_u2_max": amax(gu, gu2)}
    for a, b in (("sharded", "unfused"), ("unfused", "unfused2"), ("sharded", "sharded2"), ("fused", "unfused")):
        st = strat[a]
        if a.startswith("sharded"):
            st.synchronize_master(models[a])
        if b.startswith("sharded"):
            strat[b].synchronize_master(models[b])
        torch.cuda.synchronize()
        d = pdiff(a, b)
        worst = sorted(d.items(), key=lambda kv: -kv[1][0])[:4]
        rep[f"p_{a}_vs_{b}"] = worst
    print("DIAG", json.dumps(rep), flush=True)
print("DIAG_DONE", flush=True)
