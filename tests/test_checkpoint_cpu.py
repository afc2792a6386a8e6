"""Checkpoint details: RNG state round-trips per rank, and the retired flat per-rank optimizer-shard
layout is refused with a clear error instead of loading scrambled."""
import json
import os

import pytest
import torch


def _model():
    from pyspark_tf_gke_amd.models import build_deep_model

    return build_deep_model(3, 5, device="cpu")


def test_rng_state_restored(tmp_path):
    from pyspark_tf_gke_amd.utils import checkpoint as C

    m = _model()
    d = str(tmp_path / "ck")
    torch.manual_seed(123)
    C.save_checkpoint(m, d, 0)
    want = torch.rand(4)
    torch.manual_seed(999)
    C.load_checkpoint(m, d)
    assert torch.equal(torch.rand(4), want)


def test_ps_flat_shards_refuse_other_layout(tmp_path):
    from pyspark_tf_gke_amd.utils import checkpoint as C

    m = _model()
    d = str(tmp_path / "ck")
    C.save_checkpoint(m, d, 0)
    mf = os.path.join(d, "manifest.json")
    with open(mf) as fh:
        man = json.load(fh)
    assert man["layout"] == "per-param" and man["total"] == m.store.total
    man.update(sharded=True, layout="ps-flat", world_size=2)
    with open(mf, "w") as fh:
        json.dump(man, fh)
    with pytest.raises(ValueError, match="no longer readable"):
        C.load_checkpoint(_model(), d)


def test_each_rank_restores_its_own_rng(tmp_path):
    """Two gloo ranks seed different RNG streams, checkpoint, scramble, resume: each gets its own
    stream back (rank 0's state used to be restored on every rank)."""
    import subprocess
    import sys
    import textwrap

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    body = f"""
    import json, torch
    from pyspark_tf_gke_amd.distribute import MultiWorkerMirroredStrategy
    from pyspark_tf_gke_amd.models import build_deep_model
    from pyspark_tf_gke_amd.utils import checkpoint as C
    st = MultiWorkerMirroredStrategy()
    with st.scope():
        m = build_deep_model(3, 5, device="cpu")
    torch.manual_seed(100 + st.rank)
    C.save_checkpoint(m, {str(tmp_path / "ck")!r}, 0)
    want = torch.rand(3).tolist()
    torch.manual_seed(7)
    C.load_checkpoint(m, {str(tmp_path / "ck")!r})
    print("RESULT", json.dumps({{"rank": st.rank, "want": want, "got": torch.rand(3).tolist()}}), flush=True)
    """
    env = dict(os.environ, PYTHONPATH=root, PTG_DEVICE="cpu", PTG_HOST_FP32="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, "-m", "pyspark_tf_gke_amd.runtime.launcher", "--nproc", "2", "--",
                        sys.executable, "-c", textwrap.dedent(body)], env=env, capture_output=True, text=True,
                       timeout=240, cwd=root)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    res = [json.loads(l.split("RESULT ", 1)[1]) for l in r.stdout.splitlines() if "RESULT " in l]
    assert len(res) == 2
    for v in res:
        assert v["got"] == v["want"], v
    assert res[0]["want"] != res[1]["want"]
