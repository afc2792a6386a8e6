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

import torch
from .. import config

ENABLED = config.get("side_stream")
_STREAMS: dict = {}


def _stream(dev) -> "torch.cuda.Stream":
    dev = torch.device(dev)
    s = _STREAMS.get(dev)
    if s is None:
        s = _STREAMS[dev] = torch.cuda.Stream(device=dev)
    return s


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


def launch(fn, dev):
    """Weight-gradient (or gradient-collective) launch: forked onto the side stream when a step has
    one, else inline.  Returns ``fn()``'s result (e.g. an async collective's handle)."""
    side = _CUR[0]
    if side is not None and torch.device(dev).type == "cuda":
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
