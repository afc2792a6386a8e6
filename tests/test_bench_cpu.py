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
