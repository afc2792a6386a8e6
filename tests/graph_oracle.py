"""fp32 PyTorch-autograd oracle for functional models (test helper).

Evaluates a :class:`pyspark_tf_gke_amd.nn.Model` graph layer by layer with plain torch ops on the
model's own fp32 master weights, in training mode (batch-statistics BatchNormalization), and returns
the loss plus d(loss)/d(param) for every trainable parameter, keyed by parameter name.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from pyspark_tf_gke_amd.nn import layers as L


def oracle_grads(model, x: torch.Tensor, y: torch.Tensor):
    params = {}
    for p in model.store.params:
        params[p.name] = p.data.detach().float().cpu().clone().requires_grad_(True)
    vals = {}
    for t in model.nodes:
        l = t.layer
        if isinstance(l, L.Input):
            vals[id(t)] = x.float().permute(0, 3, 1, 2)  # NCHW
            continue
        ins = [vals[id(i)] for i in t.inputs]
        a = ins[0]
        if isinstance(l, L.ZeroPadding2D):
            v = F.pad(a, (l.pad,) * 4)
        elif isinstance(l, L.Conv2D):
            w = params[f"{l.name}/kernel"][..., : l.cin].permute(0, 3, 1, 2)
            b = params.get(f"{l.name}/bias")
            v = F.conv2d(a, w, b, stride=l.strides, padding=l.pad_amount())
        elif isinstance(l, L.BatchNormalization):
            mean = a.mean(dim=(0, 2, 3), keepdim=True)
            var = a.var(dim=(0, 2, 3), unbiased=False, keepdim=True)
            v = (a - mean) / torch.sqrt(var + l.epsilon)
            v = v * params[f"{l.name}/gamma"].view(1, -1, 1, 1) + params[f"{l.name}/beta"].view(1, -1, 1, 1)
        elif isinstance(l, (L.Activation, L.ReLU)):
            v = torch.relu(a) if getattr(l, "activation", "relu") == "relu" else a
        elif isinstance(l, L.Add):
            v = ins[0] + ins[1]
        elif isinstance(l, L.MaxPooling2D):
            v = F.max_pool2d(a, l.pool_size, l.strides)
        elif isinstance(l, L.GlobalAveragePooling2D):
            v = a.mean(dim=(2, 3))
        elif isinstance(l, L.Flatten):
            v = a.permute(0, 2, 3, 1).reshape(a.shape[0], -1)
        elif isinstance(l, L.Dense):
            v = a @ params[f"{l.name}/kernel"].t()
            if f"{l.name}/bias" in params:
                v = v + params[f"{l.name}/bias"]
            if l.activation == "relu":
                v = torch.relu(v)
            # softmax is folded into the loss below
        else:
            raise NotImplementedError(type(l).__name__)
        vals[id(t)] = v
    logits = vals[id(model.nodes[-1])]
    loss = F.cross_entropy(logits, y.long())
    loss.backward()
    return float(loss.detach()), {k: v.grad for k, v in params.items() if v.grad is not None}
