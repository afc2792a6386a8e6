"""Tracing / profiling (the reference has none).

* :class:`StepTimer` — HIP-event timing of named regions (no host sync inside the loop; one sync
  when results are read).
* :func:`range` — roctx range (``torch.cuda.nvtx`` maps to roctx on ROCm) so ``rocprofv3
  --marker-trace`` (or kernel-trace grouped by range) attributes kernels to stages.
* :class:`MetricsLogger` — structured per-step / per-stage JSONL (samples/s, rows/s, step time,
  comm time, HBM in use), one file per rank.
"""
from __future__ import annotations

import contextlib
import json
import os
import time

import torch


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors nvtx.range
    if torch.cuda.is_available() and os.environ.get("PTG_ROCTX", "1") == "1":
        try:
            torch.cuda.nvtx.range_push(name)
            yield
        finally:
            torch.cuda.nvtx.range_pop()
    else:
        yield


class StepTimer:
    def __init__(self):
        self.events: dict = {}
        self.host: dict = {}

    @contextlib.contextmanager
    def region(self, name: str):
        if torch.cuda.is_available():
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record()
            yield
            e.record()
            self.events.setdefault(name, []).append((s, e))
        else:
            t0 = time.perf_counter()
            yield
            self.host.setdefault(name, []).append((time.perf_counter() - t0) * 1e3)

    def summary(self) -> dict:
        out = {}
        if self.events:
            torch.cuda.synchronize()
        for k, lst in self.events.items():
            ms = [s.elapsed_time(e) for s, e in lst]
            out[k] = {"calls": len(ms), "total_ms": sum(ms), "mean_ms": sum(ms) / len(ms)}
        for k, ms in self.host.items():
            out[k] = {"calls": len(ms), "total_ms": sum(ms), "mean_ms": sum(ms) / len(ms)}
        return out


class MetricsLogger:
    def __init__(self, path: str | None = None):
        rank = int(os.environ.get("RANK", "0"))
        path = path or os.environ.get("PTG_METRICS_JSONL")
        self.fh = open(f"{path}.rank{rank}" if path and int(os.environ.get("WORLD_SIZE", "1")) > 1 else path, "a") \
            if path else None
        self.rank = rank

    def log(self, **kw):
        if self.fh is None:
            return
        rec = {"t": time.time(), "rank": self.rank, **kw}
        if torch.cuda.is_available():
            rec["hbm_gb"] = torch.cuda.memory_allocated() / 2 ** 30
        self.fh.write(json.dumps(rec) + "\n")
        self.fh.flush()
