"""Bounds-checked kernel build (``PTG_CHECKED=1`` -> libptg_hip_checked.so): a bad
index is clamped in range, reported with its source line and raised on the host - never a GPU
fault.  Runs in a child process because the library is chosen at import."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import torch
from pyspark_tf_gke_amd import _native
from pyspark_tf_gke_amd.ops import df as D
lib = _native.hip_lib()
# refuse to go on unless the checked build is the one loaded (its kernels clamp bad indices)
assert _native.HIP_LIB_PATH.name == "libptg_hip_checked.so", _native.HIP_LIB_PATH
assert hasattr(lib, "ptg_check_status_df")
src = torch.arange(64, dtype=torch.int32, device="cuda")
ok = D.gather_rows(src, torch.tensor([3, 5, 63], device="cuda"))
assert ok.cpu().tolist() == [3, 5, 63], ok
try:
    D.gather_rows(src, torch.tensor([1, 64], device="cuda"))  # one past the end
except RuntimeError as e:
    print("CAUGHT", e)
else:
    raise SystemExit("out-of-range gather index was not reported")
# the check word is cleared after reporting: later launches are clean
again = D.gather_rows(src, torch.tensor([7], device="cuda"))
assert again.cpu().tolist() == [7]
print("OK")
"""


def test_checked_build_reports_bad_index():
    if not os.path.exists(os.path.join(ROOT, "pyspark_tf_gke_amd", "_native", "libptg_hip_checked.so")):
        pytest.skip("checked kernel build not present (PTG_BUILD_CHECKED=0)")
    env = dict(os.environ, PTG_CHECKED="1", PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=180, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "CAUGHT native kernel index out of bounds at csrc/kernels/df.hip:" in r.stdout, r.stdout
    assert "OK" in r.stdout
