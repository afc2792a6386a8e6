"""conv2d_wgrad_halo (conv.hip conv_wgrad_strip_k) vs the fp32 torch weight gradient at the CNN-B1
layer shapes (a quick numerics check for tile-shape A/B builds: run with PTG_HIP_LIB=...)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from pyspark_tf_gke_amd.ops import nn as K  # noqa: E402

for (H, W, C, Co) in [(64, 80, 16, 32), (32, 40, 32, 64), (16, 20, 64, 64)]:
    g = torch.Generator(device="cuda").manual_seed(C)
    N = 8
    x = torch.randn((N, H, W, C), device="cuda", generator=g).bfloat16()
    dz = torch.randn((N, H, W, Co), device="cuda", generator=g).bfloat16()
    dw = torch.zeros((Co, 5, 5, C), device="cuda")
    K.conv2d_wgrad_halo(x, dz, 2, dw, zeroed=True)
    torch.cuda.synchronize()
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), (Co, C, 5, 5), dz.float().permute(0, 3, 1, 2),
                                      padding=2).permute(0, 2, 3, 1)
    err = float((dw - ref).abs().max() / ref.abs().max())
    print(json.dumps({"shape": [H, W, C, Co], "rel_err": err, "ok": err < 1e-3}), flush=True)
