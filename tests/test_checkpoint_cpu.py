"""Single-process checkpoint details: RNG state round-trips, and parameter-server flat optimizer shards
refuse to load into a layout they were not written for (a silent scramble otherwise)."""
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
    with pytest.raises(ValueError, match="parameter-server optimizer shards"):
        C.load_checkpoint(_model(), d)
