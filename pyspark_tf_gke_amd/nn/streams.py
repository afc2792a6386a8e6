"""Side-stream overlap for single-replica training steps.

Weight gradients have no consumer inside the backward pass: only the optimizer reads them, after the
last layer's backward.  So on one replica (no per-op gradient collective to feed), each layer's
wgrad kernel — and the big Dense layer's fused dW+Adam GEMM — is forked onto a side HIP stream right
after its dZ is produced, and runs concurrently with the dgrad / activation-backward chain of the
layers below (those are latency- or MFMA-bound; the wgrads of the small-channel convs and the
HBM-bound Adam epilogue fill the idle CUs).  The step's stream joins the side stream before the
optimizer pass.  Both fork and join are stream-ordered events, so the step stays capturable in a
HIP graph.  Measured on CNN-B1 b256: 2.075 -> 1.91 ms per step (profiles/r2_side_stream_ab.txt).

``PTG_SIDE_STREAM=0`` turns it off (everything on the step's stream, as before).
"""
from __future__ import annotations

import os

import torch
from .. import config

ENABLED = config.get("side_stream")
SIDE_CU_QUARTERS = config.get("side_cu_quarters")
HEAVY_CU_QUARTERS = config.get("heavy_cu_quarters")
_STREAMS: dict = {}
_HEAVY: dict = {}


def _stream(dev) -> "torch.cuda.Stream":
    dev = torch.device(dev)
    s = _STREAMS.get(dev)
    if s is None:
        s = _STREAMS[dev] = _new_side_stream(dev)
    return s


def _heavy_stream(dev):
    """A third stream confined to PTG_HEAVY_CU_QUARTERS quarters of the CUs for the HBM-bound Dense
    dW+Adam GEMM, so it cannot take the CUs of the step's dgrad chain (the wgrads keep the side
    stream on every CU)."""
    dev = torch.device(dev)
    s = _HEAVY.get(dev)
    if s is None:
        s = _HEAVY[dev] = _new_side_stream(dev, int(HEAVY_CU_QUARTERS))
    return s


def _new_side_stream(dev, quarters=None):
    """The side stream; PTG_SIDE_CU_QUARTERS < 4 confines it to that many quarters of the CUs
    (csrc/kernels/comm.hip ptg_stream_cumask_create), so its kernels never occupy the CUs the
    step's own chain runs on."""
    q = int(SIDE_CU_QUARTERS if quarters is None else quarters)
    if q >= 4:
        return torch.cuda.Stream(device=dev)
    import ctypes

    from .. import _native

    with torch.cuda.device(dev):
        h = ctypes.c_void_p()
        _native.check(_native.hip_lib().ptg_stream_cumask_create(q, ctypes.byref(h)), "ptg_stream_cumask_create")
        return torch.cuda.ExternalStream(h.value, device=dev)


class SideStream:
    """Fork launches onto the per-device side stream; :meth:`join` makes the current stream wait."""

    def __init__(self):
        self._forks: list = []

    def fork(self, fn, dev, stream=None) -> None:
        """Run ``fn``'s launches after everything queued so far on the current stream.  The buffers
        they touch must stay untouched by the current stream until :meth:`join`."""
        side = stream if stream is not None else _stream(dev)
        side.wait_stream(torch.cuda.current_stream(side.device))
        with torch.cuda.stream(side):
            out = fn()
        if side not in self._forks:
            self._forks.append(side)
        return out

    def join(self) -> None:
        for side in self._forks:
            torch.cuda.current_stream(side.device).wait_stream(side)
        self._forks.clear()


def for_step(store, strategy) -> SideStream | None:
    """A SideStream for this training step, or None (CPU, disabled, or a strategy that did not opt
    in).  Data-parallel strategies launch their per-bucket gradient collectives through
    :func:`launch` too, so a collective is ordered after the side-stream wgrads of its bucket without
    making the step's stream wait for them."""
    if not ENABLED or not store.flat.is_cuda:
        return None
    if strategy is not None and strategy.dp_degree != 1 and not getattr(strategy, "side_stream_ok", False):
        return None
    return SideStream()


_CUR: list = [None]


def current() -> SideStream | None:
    """The SideStream of the backward pass in progress (None outside one, or when not overlapping)."""
    return _CUR[0]


def launch(fn, dev, heavy: bool = False):
    """Weight-gradient (or gradient-collective) launch: forked onto the side stream when a step has
    one, else inline.  ``heavy`` (the Dense dW+Adam GEMM): onto the CU-fenced stream when
    PTG_HEAVY_CU_QUARTERS is 1..3.  Returns ``fn()``'s result (e.g. an async collective's handle)."""
    side = _CUR[0]
    if side is not None and torch.device(dev).type == "cuda":
        if heavy and 1 <= int(HEAVY_CU_QUARTERS) <= 3:
            return side.fork(fn, dev, _heavy_stream(dev))
        return side.fork(fn, dev)
    return fn()


class active:
    """``with streams.active(side): backward...`` — then ``side.join()`` before the update."""

    def __init__(self, side: SideStream | None):
        self.side = side

    def __enter__(self):
        self.prev = _CUR[0]
        _CUR[0] = self.side
        return self.side

    def __exit__(self, *exc):
        _CUR[0] = self.prev
        if self.side is not None:
            self.side.join()
        return False
