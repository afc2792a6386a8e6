"""RCCL over xGMI with one rank per GPU (skipped on boxes with fewer than 2 GPUs): all-to-all-v
groupBy, range-shuffled orderBy, sharded MWMS vs all-reduce, sync parameter server
(tools/rccl_check.py)."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs >= 2 GPUs (one RCCL rank per GPU)")
def test_rccl_two_gpus(hip_built, tmp_path):
    env = dict(os.environ, PYTHONPATH=ROOT, PTG_RCCL_OUT=str(tmp_path))
    env.pop("PTG_DIST_BACKEND", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29637", os.path.join(ROOT, "tools", "rccl_check.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=400, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = [json.loads((tmp_path / f"rank{k}.json").read_text()) for k in range(2)]
    assert all(v["ok"] for v in res), res
