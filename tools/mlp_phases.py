"""Phase timeline of one fused CSV-MLP step inside mlp_train_k (wall_clock64 stamps of thread 0 at
each barrier of the first step).  Needs the PTG_MLP_PROF build:
  python -m pyspark_tf_gke_amd._native.build --variant mlpprof -D PTG_MLP_PROF=1
  PTG_HIP_LIB=libptg_hip_mlpprof.so python tools/mlp_phases.py [--batch 32]"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pyspark_tf_gke_amd import _native  # noqa: E402
from pyspark_tf_gke_amd.models import build_deep_model  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=32)
a = ap.parse_args()
B = a.batch
dev = torch.device("cuda")
m = build_deep_model(3, 15, device=dev)
x = torch.randn(B, 3, device=dev)
y = torch.randint(0, 15, (B,), device=dev).to(torch.int32)
st = m._stats_buf()
lib = _native.hip_lib()
names = {31: "kernel_start", 0: "prologue", 1: "input", 9: "loss", 30: "end"}
for l in range(4):
    names[2 + l] = f"fwd{l}"
    names[10 + 2 * l] = f"bwd{3 - l}_dx"
    names[11 + 2 * l] = f"bwd{3 - l}_dw_adam"
res = []
for it in range(20):
    m.train_step_fast(x, y, st)
    torch.cuda.synchronize()
    buf = (ctypes.c_longlong * 32)()
    lib.ptg_mlp_prof_read.argtypes = [ctypes.c_void_p]
    lib.ptg_mlp_prof_read(buf)
    res.append(list(buf))
last = res[-1]
t0 = last[0]
out = {names[i]: round((last[i] - t0) / 100.0, 2) for i in sorted(names) if last[i]}  # 100 MHz -> us
print(json.dumps({"batch": B, "us_since_prologue_end": out}))
