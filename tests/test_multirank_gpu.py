"""Two ranks sharing the box's GPU (gloo collectives staged through the host, since RCCL refuses two
ranks on one device): the data-parallel path of the 8-GPU node with the real HIP kernels in the loop.
The sharded update (reduce-scatter during backward, per-rank Adam slice, bf16 / fp32 all-gathers
waited per forward op) must reproduce the all-reduce update's parameters."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_rank_sharded_update_on_gpu(hip_built, tmp_path):
    env = dict(os.environ, PTG_DIST_BACKEND="gloo", PYTHONPATH=ROOT, PTG_REHEARSE_OUT=str(tmp_path))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29617", os.path.join(ROOT, "tools", "rehearse_multirank.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    res = [json.loads((tmp_path / f"rank{k}.json").read_text()) for k in range(2)]
    assert len(res) == 2 and all(v["ok"] and v["buckets"] > 2 for v in res), res
