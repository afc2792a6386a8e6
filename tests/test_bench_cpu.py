"""bench.py driver contract on the CPU: ``--gpus N`` self-launches N ranks (gloo) and the weak-scaled
N-rank run equals a 1-rank run at the global batch (same data, same initial weights)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = dict(os.environ)
    env["PTG_DEVICE"] = "cpu"
    env.pop("WORLD_SIZE", None)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    return json.loads(lines[0])


def test_bench_self_launch_matches_global_batch():
    two = _run("--gpus", "2", "--workload", "mlp", "--batch-size", "64", "--steps", "6", "--warmup", "2")
    one = _run("--gpus", "1", "--workload", "mlp", "--batch-size", "128", "--steps", "6", "--warmup", "2")
    assert two["n_gpus"] == 2 and one["n_gpus"] == 1
    assert two["config"]["global_batch"] == one["config"]["global_batch"] == 128
    assert abs(two["config"]["final_loss"] - one["config"]["final_loss"]) <= 1e-5 * abs(one["config"]["final_loss"])
    assert two["comm"]["buckets"] >= 1
    for k in ("metric", "value", "unit", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in two


def test_bench_three_ranks():
    three = _run("--gpus", "3", "--workload", "mlp", "--batch-size", "32", "--steps", "3", "--warmup", "1")
    one = _run("--gpus", "1", "--workload", "mlp", "--batch-size", "96", "--steps", "3", "--warmup", "1")
    assert three["n_gpus"] == 3
    assert abs(three["config"]["final_loss"] - one["config"]["final_loss"]) <= 1e-5 * abs(one["config"]["final_loss"])


def test_bench_eight_ranks_driver_launch():
    """The driver's own N=8 command line (torch.distributed.run, one rank per 'GPU', 127.0.0.1
    rendezvous) rehearsed on gloo: eight weak-scaled ranks give the 1-rank run at the global batch,
    rank 0 alone prints the one JSON line, and the gradient buckets were all-reduced."""
    env = dict(os.environ)
    env.update({"PTG_DEVICE": "cpu", "OMP_NUM_THREADS": "1"})
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8", "--master-addr",
           "127.0.0.1", "--master-port", "29741", "bench.py", "--gpus", "8", "--workload", "mlp", "--batch-size", "16",
           "--steps", "3", "--warmup", "1"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout
    eight = json.loads(lines[0])
    one = _run("--gpus", "1", "--workload", "mlp", "--batch-size", "128", "--steps", "3", "--warmup", "1")
    assert eight["n_gpus"] == 8 and eight["config"]["global_batch"] == 128 and eight["scaling"] == "weak"
    assert eight["config"]["parallelism"].startswith("dp8")
    assert eight["comm"]["buckets"] >= 1
    assert abs(eight["config"]["final_loss"] - one["config"]["final_loss"]) <= 1e-5 * abs(one["config"]["final_loss"])
