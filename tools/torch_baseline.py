"""Same-GPU library baseline: the bench.py training steps written in plain PyTorch-ROCm (MIOpen
convolutions, hipBLASLt GEMMs, PyTorch's own Adam/SGD kernels), bf16 autocast, channels_last.

The reference publishes no throughput numbers, so the yardstick for the HIP
engine is what the stock ROCm stack does with the same model, batch and optimizer on the same
MI355X.  Models mirror bench.py: CNN-B1 (train_tf_ps.py:346-378, flat=True: 5x [Conv2D 5x5 same ->
per-element PReLU -> MaxPool 2x2] 8/16/32/64/64, no pool after the 5th, Dense 2048 relu, Dense 2,
Adam 1e-3, MSE) and ResNet-50 v1 (keras.applications layout: stride on the first 1x1 conv of a
downsampling block; SGD 0.1 momentum 0.9, softmax cross-entropy).

usage: python tools/torch_baseline.py --workload cnn_b1|resnet50 [--batch-size B] [--steps K]
"""
import argparse
import json
import time

import torch
import torch.nn as nn
import torch.nn.functional as F


class PReLUElem(nn.Module):
    """Keras PReLU default: one alpha per (h, w, c) element, initialised to 0."""

    def __init__(self, c, h, w):
        super().__init__()
        self.alpha = nn.Parameter(torch.zeros(1, c, h, w))

    def forward(self, z):
        return torch.where(z > 0, z, self.alpha * z)


class CNNB1(nn.Module):
    def __init__(self, H=256, W=320):
        super().__init__()
        chans = [3, 8, 16, 32, 64, 64]
        self.convs, self.acts = nn.ModuleList(), nn.ModuleList()
        h, w = H, W
        for i in range(5):
            self.convs.append(nn.Conv2d(chans[i], chans[i + 1], 5, padding=2))
            self.acts.append(PReLUElem(chans[i + 1], h, w))
            if i < 4:
                h, w = h // 2, w // 2
        self.fc1 = nn.Linear(h * w * 64, 2048)
        self.fc2 = nn.Linear(2048, 2)

    def forward(self, x):
        for i in range(5):
            x = self.acts[i](self.convs[i](x))
            if i < 4:
                x = F.max_pool2d(x, 2)
        x = torch.flatten(x.permute(0, 2, 3, 1), 1)  # Keras Flatten order (NHWC)
        return self.fc2(F.relu(self.fc1(x)))


class Bottleneck(nn.Module):
    def __init__(self, cin, mid, stride, project):
        super().__init__()
        cout = mid * 4
        self.c1, self.b1 = nn.Conv2d(cin, mid, 1, stride, bias=True), nn.BatchNorm2d(mid, eps=1.001e-5)
        self.c2, self.b2 = nn.Conv2d(mid, mid, 3, 1, 1, bias=True), nn.BatchNorm2d(mid, eps=1.001e-5)
        self.c3, self.b3 = nn.Conv2d(mid, cout, 1, bias=True), nn.BatchNorm2d(cout, eps=1.001e-5)
        self.proj = None
        if project:
            self.proj = nn.Sequential(nn.Conv2d(cin, cout, 1, stride, bias=True), nn.BatchNorm2d(cout, eps=1.001e-5))

    def forward(self, x):
        y = F.relu(self.b1(self.c1(x)))
        y = F.relu(self.b2(self.c2(y)))
        y = self.b3(self.c3(y))
        return F.relu(y + (self.proj(x) if self.proj is not None else x))


class ResNet50(nn.Module):
    def __init__(self, classes=1000):
        super().__init__()
        self.stem = nn.Sequential(nn.Conv2d(3, 64, 7, 2, 3, bias=True), nn.BatchNorm2d(64, eps=1.001e-5), nn.ReLU(),
                                  nn.MaxPool2d(3, 2, 1))
        blocks, cin = [], 64
        for mid, n, stride in ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2)):
            for i in range(n):
                blocks.append(Bottleneck(cin, mid, stride if i == 0 else 1, i == 0))
                cin = mid * 4
        self.blocks = nn.Sequential(*blocks)
        self.fc = nn.Linear(2048, classes)

    def forward(self, x):
        x = self.blocks(self.stem(x))
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))


def groupby(a, dev):
    """groupBy(key).agg(sum, count) the stock way: sort-based unique + index_add / bincount."""
    n = a.rows
    keys = torch.randint(0, a.keys, (n,), device=dev, dtype=torch.int64)
    vals = torch.rand(n, device=dev, dtype=torch.float64)

    def step():
        uk, inv = torch.unique(keys, return_inverse=True)
        sums = torch.zeros(uk.numel(), device=dev, dtype=torch.float64).index_add_(0, inv, vals)
        cnts = torch.bincount(inv, minlength=uk.numel())
        return uk, sums, cnts

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        uk, sums, cnts = step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert int(cnts.sum()) == n
    print(json.dumps({"workload": "groupby", "framework": f"PyTorch {torch.__version__} (torch.unique + index_add_)",
                      "rows": n, "distinct_keys": int(uk.numel()), "rows_per_s": round(n * a.steps / dt, 1),
                      "ms_per_step": round(dt / a.steps * 1e3, 3)}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="cnn_b1", choices=["cnn_b1", "resnet50", "groupby"])
    ap.add_argument("--rows", type=int, default=1_000_000_000)
    ap.add_argument("--keys", type=int, default=1_000_000)
    ap.add_argument("--batch-size", type=int, default=0)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--find", type=int, default=1, help="MIOpen kernel search (cudnn.benchmark)")
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.backends.cudnn.benchmark = bool(a.find)
    torch.manual_seed(0)
    if a.workload == "groupby":
        return groupby(a, dev)
    if a.workload == "cnn_b1":
        B = a.batch_size or 256
        model = CNNB1().to(dev).to(memory_format=torch.channels_last)
        opt = torch.optim.Adam(model.parameters(), lr=1e-3, eps=1e-7, fused=True)
        x = torch.rand(B, 3, 256, 320, device=dev).to(memory_format=torch.channels_last)
        y = torch.rand(B, 2, device=dev) * 256
        loss_fn = F.mse_loss
    else:
        B = a.batch_size or 128
        model = ResNet50().to(dev).to(memory_format=torch.channels_last)
        opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9, fused=True)
        x = torch.rand(B, 3, 224, 224, device=dev).to(memory_format=torch.channels_last)
        y = torch.randint(0, 1000, (B,), device=dev)
        loss_fn = F.cross_entropy

    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = loss_fn(model(x).float(), y)
        loss.backward()
        opt.step()
        return loss

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"workload": a.workload, "framework": f"PyTorch {torch.__version__} eager (MIOpen/hipBLASLt), "
                      "bf16 autocast, channels_last", "miopen_find": bool(a.find), "batch": B, "samples_per_s": round(B * a.steps / dt, 1),
                      "ms_per_step": round(dt / a.steps * 1e3, 3), "loss": round(float(loss.detach()), 4)}))


if __name__ == "__main__":
    main()
