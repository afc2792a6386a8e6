"""Fault tolerance and parameter-server fidelity on CPU ranks (gloo) — SURVEY §5.3, T14/T15:

* a coordinator closure that raises on one rank is retried as a whole round: final parameters are
  bit-identical to a fault-free run;
* rounds with fewer closures than ranks average over the contributors only and never advance the
  optimizer on zero pushes;
* ``MinSizePartitioner`` placement (per-variable shards round-robin over PS tasks) at 2/3/5 ranks,
  including world sizes that do not divide the parameter count;
* sync PS == single-process mean gradient; async PS == each worker's gradient applied as its own
  optimizer step, in worker order;
* process fault at step s -> launcher restart -> resume from the last checkpoint == uninterrupted;
* a rank that stops making progress (blocked in a collective) is detected and the group restarted.
"""
import json
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _launch(body: str, nproc: int, extra_env=None, launcher_args=(), timeout=300):
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env["PTG_DEVICE"] = "cpu"
    env["PTG_HOST_FP32"] = "1"
    env.pop("WORLD_SIZE", None)
    env.update(extra_env or {})
    cmd = [sys.executable, "-m", "pyspark_tf_gke_amd.runtime.launcher", "--nproc", str(nproc), *launcher_args, "--",
           sys.executable, "-c", textwrap.dedent(body)]
    return subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=timeout, cwd=ROOT)


def _results(out: str):
    res = {}
    for line in out.splitlines():
        if "RESULT " in line:
            rank = int(line.split("]")[0].replace("[rank", ""))
            res[rank] = json.loads(line.split("RESULT ", 1)[1])
    return res


COMMON = """
import json, os, torch, numpy as np
from pyspark_tf_gke_amd import nn
from pyspark_tf_gke_amd.distribute import ParameterServerStrategy, MultiWorkerMirroredStrategy, ClusterCoordinator
from pyspark_tf_gke_amd.distribute.cluster import MinSizePartitioner
from pyspark_tf_gke_amd.models import build_deep_model
from pyspark_tf_gke_amd.nn.tape import GradientTape
rng = np.random.default_rng(0)
X = rng.normal(size=(16, 32, 3)).astype(np.float32)
Y = rng.integers(0, 4, size=(16, 32)).astype(np.int32)
loss_fn = nn.losses.SparseCategoricalCrossentropy()

def make(st, lr=1e-2):
    with st.scope():
        m = build_deep_model(3, 4, device="cpu")
        opt = nn.optimizers.Adam(lr)
    return m, opt

def step_fn(m, opt, i, fail_box=None, rank=None):
    if fail_box is not None and fail_box.get(i, 0) > 0 and rank in fail_box.get("ranks", ()):
        fail_box[i] -= 1
        raise RuntimeError(f"injected closure failure {i}")
    with GradientTape() as tape:
        out = m(torch.from_numpy(X[i]), training=True)
        loss = loss_fn(torch.from_numpy(Y[i]), out)
    grads = tape.gradient(loss, m.trainable_variables)
    opt.apply_gradients(zip(grads, m.trainable_variables))
    return 1

def flat(m):
    return m.store.flat.clone()
"""


def test_coordinator_retry_is_bit_identical():
    body = COMMON + """
st = ParameterServerStrategy()
m_ok, o_ok = make(st)
m_ft, o_ft = make(st)
co = ClusterCoordinator(st)
for i in range(6):
    co.schedule(step_fn, args=(m_ok, o_ok, i))
co.join()
fail = {3: 1, 5: 2, "ranks": (1,)}   # closure 3 fails once, closure 5 twice, both on rank 1
co2 = ClusterCoordinator(st, max_retries=2)
rvs = [co2.schedule(step_fn, args=(m_ft, o_ft, i, fail, st.rank)) for i in range(6)]
co2.join()
same = bool(torch.equal(flat(m_ok), flat(m_ft)))
print("RESULT", json.dumps({"same": same, "retries": co2.retries, "it_ok": o_ok.iterations,
                            "it_ft": o_ft.iterations, "vals": [rv.fetch() for rv in rvs]}), flush=True)
"""
    r = _launch(body, 2)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = _results(r.stdout)
    assert len(res) == 2
    for v in res.values():
        assert v["same"], v
        assert v["retries"] == 3 and v["it_ok"] == v["it_ft"] == 3 and v["vals"] == [1] * 6, v


def test_coordinator_exhausted_retries_and_partial_rounds():
    """A closure failing more than max_retries is dropped (error on every rank) while the round's
    successful closure is committed without being re-run; a round with one closure on two ranks
    averages over that one worker; no optimizer step without contributors."""
    body = COMMON + """
st = ParameterServerStrategy()
m, o = make(st)
ref, ro = make(st)
co = ClusterCoordinator(st, max_retries=1)
fail = {1: 5, "ranks": (1,)}
rvs = [co.schedule(step_fn, args=(m, o, i, fail, st.rank)) for i in range(3)]
co.join()
errs = []
for rv in rvs:
    try:
        rv.fetch(); errs.append(None)
    except RuntimeError as e:
        errs.append("failed")
# round 1 = {rank 0: closure 0, rank 1: closure 1}: closure 1 fails twice (1 retry) and is dropped;
# rank 0's pending gradient is kept (not recomputed) and committed alone; round 2 = {rank 0: closure 2}
from pyspark_tf_gke_amd.nn import engine as E
def grad(model, i):
    model.store.grad_clean = False
    model.store.zero_grad()
    out = E.run_forward(model.ops, torch.from_numpy(X[i]), model.ws, True)
    d = model._loss_grad(out, torch.from_numpy(Y[i]), torch.zeros(8))
    E.run_backward(model.ops, d, model.ws)
    return model.store.flat_grad.clone()
g0 = grad(ref, 0)
ref.store.flat_grad.copy_(g0)
ro.apply(ref.store, gscale=1.0)
g2 = grad(ref, 2)
ref.store.flat_grad.copy_(g2)
ro.apply(ref.store, gscale=1.0)
diff = float((m.store.flat - ref.store.flat).abs().max())
# a 3-closure queue on 2 ranks with no failures: last round has one contributor
m2, o2 = make(st)
r2, ro2 = make(st)
co3 = ClusterCoordinator(st)
for i in range(3):
    co3.schedule(step_fn, args=(m2, o2, i))
co3.join()
ga, gb = grad(r2, 0), grad(r2, 1)
r2.store.flat_grad.copy_(ga + gb); ro2.apply(r2.store, gscale=0.5)
gc = grad(r2, 2)
r2.store.flat_grad.copy_(gc); ro2.apply(r2.store, gscale=1.0)
diff2 = float((m2.store.flat - r2.store.flat).abs().max())
print("RESULT", json.dumps({"errs": errs, "diff": diff, "it": o.iterations, "diff2": diff2, "it2": o2.iterations}),
      flush=True)
"""
    r = _launch(body, 2)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = _results(r.stdout)
    assert len(res) == 2
    for v in res.values():
        assert v["errs"] == [None, "failed", None], v
        assert v["it"] == 2 and v["diff"] < 1e-6, v
        assert v["it2"] == 2 and v["diff2"] < 1e-6, v


@pytest.mark.parametrize("nproc", [2, 3, 5])
def test_ps_partitioner_placement_and_sync_update(nproc):
    body = COMMON + """
st = ParameterServerStrategy(variable_partitioner=MinSizePartitioner(min_shard_bytes=256, max_shards=4))
m, o = make(st)
ref, ro = make(st)
W = st.world_size
for it in range(2):
    step_fn(m, o, st.rank + W * it)
from pyspark_tf_gke_amd.nn import engine as E
for it in range(2):
    acc = None
    for w in range(W):
        ref.store.zero_grad()
        out = E.run_forward(ref.ops, torch.from_numpy(X[w + W * it]), ref.ws, True)
        d = ref._loss_grad(out, torch.from_numpy(Y[w + W * it]), torch.zeros(8))
        E.run_backward(ref.ops, d, ref.ws)
        g = ref.store.flat_grad.clone()
        acc = g if acc is None else acc + g
    ref.store.flat_grad.copy_(acc)
    ro.apply(ref.store, gscale=1.0 / W)
diff = float((m.store.flat - ref.store.flat).abs().max())
pl = st.placement(m)
print("RESULT", json.dumps({"diff": diff, "placement": pl, "W": W}), flush=True)
"""
    r = _launch(body, nproc)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = _results(r.stdout)
    assert len(res) == nproc
    for v in res.values():
        assert v["diff"] < 1e-6, v
    pl = res[0]["placement"]
    # Dense kernels (rows x cols fp32): shards of whole rows, >= 256 B each unless the variable is
    # smaller, at most 4 per variable; PS tasks assigned round-robin in creation order
    by_var = {}
    for name, (r0, r1), task, owner in pl:
        by_var.setdefault(name, []).append((r0, r1, task, owner))
        assert owner == task % nproc
    assert [p[2] for p in pl] == [i % nproc for i in range(len(pl))]
    assert max(len(v) for v in by_var.values()) == 4
    for shards in by_var.values():
        assert shards[0][0] == 0 and all(a[1] == b[0] for a, b in zip(shards, shards[1:]))


def test_ps_single_ps_task_lives_on_rank0():
    """The reference's launcher config (1 PS): every variable unsplit, on PS task 0 = rank 0."""
    body = COMMON + """
from pyspark_tf_gke_amd.distribute.cluster import SimpleClusterResolver, ClusterSpec
spec = ClusterSpec({"worker": ["127.0.0.1:2222", "127.0.0.1:2223"], "ps": ["127.0.0.1:2224"]})
st = ParameterServerStrategy(SimpleClusterResolver(spec))
m, o = make(st)
step_fn(m, o, st.rank)
print("RESULT", json.dumps({"owners": sorted({p[3] for p in st.placement(m)}), "n": len(st.placement(m)),
                            "sum": float(m.store.flat.sum())}), flush=True)
"""
    r = _launch(body, 2)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = _results(r.stdout)
    assert res[0]["owners"] == [0] and res[0]["sum"] == res[1]["sum"]


def test_ps_async_single_active_worker_is_sequential_adam():
    """Async PS: rank 1 arrives late, so rank 0 draws every closure; each push is applied by the
    owners (both ranks' service threads) before apply_gradients returns and the next closure pulls,
    so the result is exactly 8 sequential Adam steps."""
    body = COMMON + """
import time
st = ParameterServerStrategy(mode="async", variable_partitioner=MinSizePartitioner(min_shard_bytes=256, max_shards=4))
m, o = make(st, lr=5e-3)
ref, ro = make(st, lr=5e-3)
co = ClusterCoordinator(st)
# rank 1 arrives late: it joins only after rank 0 has run every closure (a flag file written by the
# 8th closure, not a sleep, so a loaded machine cannot let it draw one); its service thread applies
# its shards meanwhile
flag = f"/tmp/ptg_ps_seq_{os.environ['MASTER_PORT']}.done"
ran = [0]
def fn(m, o, i):
    out = step_fn(m, o, i)
    ran[0] += 1
    if ran[0] == 8:
        open(flag, "w").close()
    return out
for i in range(8):
    co.schedule(fn, args=(m, o, i))
if st.rank == 1:
    t_end = time.time() + 120
    while not os.path.exists(flag) and time.time() < t_end:
        time.sleep(0.05)
co.join()
st.synchronize_master(m)
from pyspark_tf_gke_amd.nn import engine as E
for i in range(8):
    ref.store.grad_clean = False
    ref.store.zero_grad()
    out = E.run_forward(ref.ops, torch.from_numpy(X[i]), ref.ws, True)
    d = ref._loss_grad(out, torch.from_numpy(Y[i]), torch.zeros(8))
    E.run_backward(ref.ops, d, ref.ws)
    ro.apply(ref.store, gscale=1.0)
diff = float((m.store.flat - ref.store.flat).abs().max())
owners = sorted({p[3] for p in st.placement(m)})
print("RESULT", json.dumps({"diff": diff, "it": o.iterations, "ran": co.closures_run, "owners": owners}), flush=True)
st.shutdown()
"""
    r = _launch(body, 2)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = _results(r.stdout)
    assert len(res) == 2
    assert res[0]["ran"] == 8 and res[1]["ran"] == 0 and res[0]["owners"] == [0, 1], res
    for v in res.values():
        assert v["diff"] < 1e-6 and v["it"] == 8, v


SLOW_BODY = COMMON + """
import time
mode = os.environ["PS_MODE"]
st = ParameterServerStrategy(mode=mode)
m, o = make(st, lr=1e-3)
co = ClusterCoordinator(st)
def slow_step(i):
    if st.rank == 2:
        time.sleep(0.1)        # the straggler: 100 ms per step
    return step_fn(m, o, i % 16)
comm_t = torch.zeros(1)
from pyspark_tf_gke_amd.parallel import comm
comm.barrier()
t0 = time.time()
for i in range(30):
    co.schedule(slow_step, args=(i,))
co.join()
dt = time.time() - t0
print("RESULT", json.dumps({"dt": dt, "ran": co.closures_run, "it": o.iterations}), flush=True)
if mode == "async":
    st.shutdown()
"""


def test_ps_async_slow_worker_does_not_stall_the_others():
    """3 ranks, one sleeping 100 ms per step: the async coordinator hands the closures to the idle
    workers, so the job ends in about the straggler's few steps, not in 10 lock-step rounds of
    100 ms as the sync rounds do; every closure runs exactly once."""
    ra = _launch(SLOW_BODY, 3, extra_env={"PS_MODE": "async"})
    assert ra.returncode == 0, ra.stdout[-3000:] + ra.stderr[-3000:]
    a = _results(ra.stdout)
    rs = _launch(SLOW_BODY, 3, extra_env={"PS_MODE": "sync"})
    assert rs.returncode == 0, rs.stdout[-3000:] + rs.stderr[-3000:]
    s = _results(rs.stdout)
    assert sum(v["ran"] for v in a.values()) == 30 and all(v["it"] == 30 for v in a.values()), a
    assert a[2]["ran"] <= 4 < min(a[0]["ran"], a[1]["ran"]), a
    dt_async, dt_sync = max(v["dt"] for v in a.values()), max(v["dt"] for v in s.values())
    assert dt_sync >= 1.0, s
    assert dt_async < 0.6 * dt_sync, (dt_async, dt_sync)


def test_coordinator_retry_with_per_worker_iterators():
    """The reference's closure (train_tf_ps.py:616-631,642): ``next(per_worker_iterator)`` inside the
    scheduled step.  A closure that fails on rank 1 before drawing its batch is re-run there alone:
    the other ranks' closures are neither re-run nor their iterators advanced twice, so the result is
    bit-identical to the fault-free run and every rank consumed the same batches."""
    body = COMMON + """
from pyspark_tf_gke_amd.data.dataset import Dataset
XA = torch.from_numpy(rng.normal(size=(96, 3)).astype(np.float32))
YA = torch.from_numpy(rng.integers(0, 4, size=(96,)).astype(np.int32))
def run(fail_calls):
    st = ParameterServerStrategy()
    m, o = make(st)
    co = ClusterCoordinator(st, max_retries=2)
    ds = co.create_per_worker_dataset(
        lambda ctx: Dataset.from_tensor_slices((XA, YA)).shard(ctx.num_input_pipelines, ctx.input_pipeline_id).batch(8).repeat())
    it = iter(ds)
    calls, drawn = [0], []
    def per_worker_train_step(iterator):
        calls[0] += 1
        if st.rank == 1 and calls[0] in fail_calls:
            raise RuntimeError("injected worker failure")
        x, y = next(iterator)
        drawn.append(float(x.sum()))
        with GradientTape() as tape:
            loss = loss_fn(y, m(x, training=True))
        o.apply_gradients(zip(tape.gradient(loss, m.trainable_variables), m.trainable_variables))
        return 1
    for epoch in range(2):
        for _ in range(5):
            co.schedule(per_worker_train_step, args=(it,))
        co.join()
    return flat(m), drawn, co.retries, calls[0], o.iterations
a, da, _, ca, ia = run(set())
b, db, rb, cb, ib = run({2, 4})
print("RESULT", json.dumps({"same": bool(torch.equal(a, b)), "drawn_same": da == db, "retries": rb,
                            "calls": [ca, cb], "it": [ia, ib]}), flush=True)
"""
    r = _launch(body, 3)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = _results(r.stdout)
    assert len(res) == 3
    for rank, v in res.items():
        assert v["same"] and v["drawn_same"], v
        assert v["retries"] == 2 and v["it"] == [4, 4], v
        extra = 2 if rank == 1 else 0  # only the failed closures ran twice
        assert v["calls"][1] == v["calls"][0] + extra, v


RESUME_BODY = """
import json, os, sys, numpy as np, torch
from pyspark_tf_gke_amd.distribute import MultiWorkerMirroredStrategy
from pyspark_tf_gke_amd.models import build_deep_model
from pyspark_tf_gke_amd.utils.checkpoint import CheckpointCallback
st = MultiWorkerMirroredStrategy(device="cpu")
rng = np.random.default_rng(7)
X = rng.normal(size=(2, 96, 3)).astype(np.float32); y = rng.integers(0, 5, (2, 96)).astype(np.int32)
with st.scope():
    m = build_deep_model(3, 5, device="cpu")
cb = CheckpointCallback(os.environ["CKPT"], every=1, resume=True)
m.fit(X[st.rank], y[st.rank], batch_size=16, epochs=4, verbose=0, callbacks=[cb])
st.synchronize_master(m)
if st.rank == 0:
    np.save(os.environ["OUT"], m.store.flat.numpy())
print("RESULT", json.dumps({"restart": os.environ.get("PTG_RESTART_COUNT"), "start": cb.start_epoch}), flush=True)
"""


def test_fault_restart_resume_matches_uninterrupted(tmp_path):
    import numpy as np

    clean = _launch(RESUME_BODY, 2, extra_env={"CKPT": str(tmp_path / "ck_clean"), "OUT": str(tmp_path / "clean.npy")})
    assert clean.returncode == 0, clean.stdout[-2000:] + clean.stderr[-3000:]
    # rank 1 dies at its 15th train step (epoch 3 of 6 steps per epoch); the launcher restarts the
    # group, which resumes from the epoch-2 checkpoint
    faulty = _launch(RESUME_BODY, 2, extra_env={"CKPT": str(tmp_path / "ck_fault"), "OUT": str(tmp_path / "fault.npy"),
                                                "PTG_FAULT_RANK": "1", "PTG_FAULT_STEP": "15"},
                     launcher_args=("--max-restarts", "1"))
    assert faulty.returncode == 0, faulty.stdout[-2000:] + faulty.stderr[-3000:]
    assert "injected failure on rank 1" in faulty.stdout + faulty.stderr and "restarting all ranks" in faulty.stderr
    res = _results(faulty.stdout)
    assert any(v["restart"] == "1" and v["start"] == 2 for v in res.values()), res
    a, b = np.load(tmp_path / "clean.npy"), np.load(tmp_path / "fault.npy")
    assert np.array_equal(a, b)


def test_hang_detected_by_progress_counter():
    body = """
import os, time
from pyspark_tf_gke_amd.parallel import comm
from pyspark_tf_gke_amd.runtime import heartbeat
comm.init()
heartbeat.progress()
if os.environ.get("PTG_RESTART_COUNT") == "0":
    if comm.rank() == 1:
        time.sleep(120)        # stuck: makes no progress
    comm.barrier()             # rank 0 blocks in the collective; its heartbeat thread still runs
heartbeat.progress()
comm.barrier()
print("RESULT {\\"ok\\": 1}", flush=True)
"""
    r = _launch(body, 2, launcher_args=("--hang-timeout", "4", "--startup-timeout", "60", "--max-restarts", "1"),
                timeout=200)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    assert "made no progress" in r.stderr and "restarting all ranks" in r.stderr
    assert len(_results(r.stdout)) == 2


def test_ps_async_failed_closures_rescheduled_on_other_workers():
    """Async PS, 3 ranks, rank 1 raises in EVERY closure before its push: each failed closure goes
    back to the shared retry queue with rank 1 excluded, so ranks 0 and 2 run all of them; every
    RemoteValue resolves on every rank, join() returns, and every closure updated the model once."""
    body = COMMON + """
st = ParameterServerStrategy(mode="async")
m, o = make(st, lr=1e-3)
co = ClusterCoordinator(st, max_retries=2)
def closure(i):
    if st.rank == 1:
        raise RuntimeError("worker 1 is broken")
    step_fn(m, o, i % 16)
    return i * 10
rvs = [co.schedule(closure, args=(i,)) for i in range(12)]
co.join()
vals = [rv.fetch() for rv in rvs]
print("RESULT", json.dumps({"vals": vals, "ran": co.closures_run, "retries": co.retries, "it": o.iterations}),
      flush=True)
st.shutdown()
"""
    r = _launch(body, 3)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = _results(r.stdout)
    assert len(res) == 3
    for v in res.values():
        assert v["vals"] == [i * 10 for i in range(12)] and v["it"] == 12, v
    assert res[1]["ran"] == 0 and res[0]["ran"] + res[2]["ran"] == 12, res


def test_ps_async_failure_after_push_is_not_rerun():
    """A closure that raises after its gradient push (the PS already applied it) is recorded as
    failed rather than re-run: re-running would push the same batch twice."""
    body = COMMON + """
st = ParameterServerStrategy(mode="async")
m, o = make(st, lr=1e-3)
co = ClusterCoordinator(st, max_retries=3)
def closure(i):
    step_fn(m, o, i)
    if i == 2:
        raise RuntimeError("metric update failed after the push")
    return i
rvs = [co.schedule(closure, args=(i,)) for i in range(4)]
co.join()
out = []
for rv in rvs:
    try:
        out.append(rv.fetch())
    except RuntimeError as e:
        out.append("after its gradient push" in str(e))
print("RESULT", json.dumps({"out": out, "it": o.iterations, "retries": co.retries}), flush=True)
st.shutdown()
"""
    r = _launch(body, 2)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = _results(r.stdout)
    for v in res.values():
        assert v["out"] == [0, 1, True, 3] and v["it"] == 4, v
    assert sum(v["retries"] for v in res.values()) == 0, res


def test_ps_async_dead_worker_closures_requeued():
    """A worker process that dies holding a drawn closure stops its liveness beat; the idle workers
    re-queue that closure and run it, so every closure has a result on the survivors (the collective
    tail of join() then needs the launcher's group restart, so it is stubbed out here)."""
    body = COMMON + """
import sys, time
C = sys.modules["pyspark_tf_gke_amd.distribute.coordinator"]
st = ParameterServerStrategy(mode="async")
co = ClusterCoordinator(st)
def closure(i):
    if st.rank == 2:
        os._exit(0)                 # the worker dies mid-closure (no exception, no push)
    time.sleep(0.05)
    return i + 100
rvs = [co.schedule(closure, args=(i,)) for i in range(6)]
if st.rank != 2:
    time.sleep(1.0)                 # rank 2 draws first
    st.wait_all_applied = lambda: None
    C.comm.barrier = lambda: None
co.join()
print("RESULT", json.dumps({"vals": [rv.fetch() for rv in rvs], "ran": co.closures_run}), flush=True)
# rank 0 hosts the TCP store: it leaves only after rank 1 has read its results
from pyspark_tf_gke_amd.distribute.ps import _store
_store().set(f"test/done/{st.rank}", "1")
if st.rank == 0:
    _store().wait(["test/done/1"])
os._exit(0)
"""
    r = _launch(body, 3, extra_env={"PTG_COORD_DEAD_S": "2"})
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = _results(r.stdout)
    assert sorted(res) == [0, 1], res
    for v in res.values():
        assert v["vals"] == [i + 100 for i in range(6)], v
    assert res[0]["ran"] + res[1]["ran"] == 6, res


def test_coordinator_one_worker_rounds():
    """One worker (the reference's smallest PS cluster): the local round loop (coordinator.py
    _join_local) retries a failing closure bit-identically, drops one that keeps failing (no
    optimizer step, error on its RemoteValue), passes StopIteration through and returns values."""
    body = COMMON + """
st = ParameterServerStrategy()
assert st.world_size == 1
m_ok, o_ok = make(st)
m_ft, o_ft = make(st)
co = ClusterCoordinator(st)
for i in range(6):
    co.schedule(step_fn, args=(m_ok, o_ok, i))
co.join()
fail = {2: 1, 4: 5, "ranks": (0,)}   # closure 2 fails once, closure 4 always
co2 = ClusterCoordinator(st, max_retries=2)
rvs = [co2.schedule(step_fn, args=(m_ft, o_ft, i, fail, st.rank)) for i in range(6)]
def stop():
    raise StopIteration
rs = co2.schedule(stop)
co2.join()
errs = []
for rv in rvs + [rs]:
    try:
        errs.append(rv.fetch())
    except BaseException as e:
        errs.append(type(e).__name__)
m_ref, o_ref = make(st)
co3 = ClusterCoordinator(st)
for i in (0, 1, 2, 3, 5):
    co3.schedule(step_fn, args=(m_ref, o_ref, i))
co3.join()
print("RESULT", json.dumps({"retries": co2.retries, "it_ok": o_ok.iterations, "it_ft": o_ft.iterations,
                            "vals": errs, "same_as_skip4": bool(torch.equal(flat(m_ref), flat(m_ft))),
                            "ran": co2.closures_run}), flush=True)
"""
    r = _launch(body, 1)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    v = _results(r.stdout)[0]
    assert v["retries"] == 3 and v["it_ok"] == 6 and v["it_ft"] == 5, v
    assert v["vals"] == [1, 1, 1, 1, "RuntimeError", 1, "StopIteration"], v
    assert v["same_as_skip4"] and v["ran"] == 5, v


@pytest.mark.parametrize("mode", ["async", "sync"])
def test_train_tf_ps_cli_ps_mode(mode, tmp_path):
    """`train_tf_ps.py --use-ps --ps-mode {async,sync}` (the reference's CSV-MLP driver under
    ParameterServerStrategy + ClusterCoordinator, train_tf_ps.py:505-510,612-645) on 2 gloo ranks:
    the strategy runs in the requested mode, the loop trains and the chief saves the model."""
    script = os.path.join(ROOT, "workloads", "raw-tf", "train_tf_ps.py")
    body = f"""
    import runpy, sys, json
    sys.path.insert(0, {os.path.dirname(script)!r})
    from pyspark_tf_gke_amd.distribute import ParameterServerStrategy
    seen = {{}}
    _init = ParameterServerStrategy.__init__
    def _spy(self, *a, **k):
        _init(self, *a, **k)
        seen["mode"] = self.mode
    ParameterServerStrategy.__init__ = _spy
    sys.argv = ["train_tf_ps.py", "--use-ps", "--ps-mode", "{mode}", "--worker-replicas", "2", "--ps-replicas", "1",
                "--data-path", {os.path.join(ROOT, "tests", "data", "health.csv")!r}, "--epochs", "2",
                "--batch-size", "512", "--output-dir", {str(tmp_path)!r}, "--chief-addr", "127.0.0.1"]
    try:
        runpy.run_path({script!r}, run_name="__main__")
    except SystemExit as e:
        assert not e.code, e.code
    print("RESULT", json.dumps(seen), flush=True)
    """
    r = _launch(body, 2, timeout=400)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = _results(r.stdout)
    assert len(res) == 2 and all(v["mode"] == mode for v in res.values()), res
    assert "Epoch 2 - loss:" in r.stdout
    assert os.path.exists(os.path.join(str(tmp_path), "model.keras"))


def test_async_coordinator_long_closure_is_not_a_stall_and_stall_aborts_all():
    """a closure longer than the stall deadline on a live worker is progress (its busy
    mark and fresh liveness beat), not a stall; a real stall (here: the busy check stubbed out) is
    declared by the idle rank in the store, and the busy rank's join fails with the same message as
    soon as its closure returns, instead of walking into the collective tail."""
    body = COMMON + """
import sys, time
C = sys.modules["pyspark_tf_gke_amd.distribute.coordinator"]
st = ParameterServerStrategy(mode="async")
def run(stub):
    co = ClusterCoordinator(st)
    if stub:
        C.ClusterCoordinator._live_busy = staticmethod(lambda *a: False)
    def closure(i):
        if st.rank == 1:
            time.sleep(4.0)        # 2 x PTG_COORD_STALL_S
        return i
    if st.rank == 0:
        time.sleep(0.5)            # rank 1 draws closure 0 first
    rvs = [co.schedule(closure, args=(i,)) for i in range(2)]
    try:
        co.join()
        return [rv.fetch() for rv in rvs]
    except RuntimeError as e:
        return "ERR:" + str(e)[:60]
ok = run(False)
bad = run(True)
print("RESULT", json.dumps({"ok": ok, "bad": bad}), flush=True)
from pyspark_tf_gke_amd.distribute.ps import _store
_store().set(f"test/done/{st.rank}", "1")
if st.rank == 0:
    _store().wait(["test/done/1"])
os._exit(0)
"""
    r = _launch(body, 2, extra_env={"PTG_COORD_STALL_S": "2"})
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = _results(r.stdout)
    assert sorted(res) == [0, 1], r.stdout[-3000:] + r.stderr[-3000:]
    for v in res.values():
        assert v["ok"] == [0, 1], v
        assert v["bad"].startswith("ERR:ClusterCoordinator.join: no closure finished"), v
