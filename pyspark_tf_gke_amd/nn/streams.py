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
DEVICE_EVENTS = config.get("fork_device_events")
_STREAMS: dict = {}
_EVENTS: list = []  # free device-scope events (native handles), reused across steps


class _DevEvent:
    """A HIP event recorded with a device-scope release only (comm.hip ptg_event_create_device).
    torch's events end their record with a system-scope release - a cache writeback and invalidate
    that stalled the step's stream ~6.5 us at every fork; two streams of one device need only
    device-scope ordering."""

    def __init__(self):
        import ctypes

        from .. import _native

        h = ctypes.c_void_p()
        _native.check(_native.hip_lib().ptg_event_create_device(ctypes.byref(h)), "ptg_event_create_device")
        self.h = h.value

    @staticmethod
    def get() -> "_DevEvent":
        return _EVENTS.pop() if _EVENTS else _DevEvent()

    def record(self, handle: int) -> None:
        from .. import _native

        _native.call("ptg_event_record", self.h, handle)

    def wait(self, handle: int) -> None:
        from .. import _native

        _native.call("ptg_stream_wait_event", self.h, handle)


def _cur_handle() -> int:
    from ..ops._util import stream_handle

    return stream_handle()


def _wait(waiter, producer, used: list) -> None:
    """``waiter`` runs its later work after everything queued on ``producer`` so far (both
    torch.cuda.Stream objects)."""
    if DEVICE_EVENTS:
        e = _DevEvent.get()
        e.record(producer.cuda_stream)
        e.wait(waiter.cuda_stream)
        used.append(e)
    else:
        waiter.wait_stream(producer)


def _stream(dev, k: int = 0) -> "torch.cuda.Stream":
    """Side stream ``k`` of ``dev`` (0: weight gradients; 1: the big Dense dW+Adam, see launch())."""
    dev = torch.device(dev)
    s = _STREAMS.get((dev, k))
    if s is None:
        s = _STREAMS[(dev, k)] = torch.cuda.Stream(device=dev)
    return s


class SideStream:
    """Fork launches onto the per-device side stream; :meth:`join` makes the current stream wait."""

    def __init__(self):
        self._forks: list = []
        self._events: list = []  # device events recorded this step (back to the pool at the join)
        self._main = None  # the step's stream (looked up once: current_stream() costs ~5 us)

    def fork(self, fn, dev, stream=None) -> None:
        """Run ``fn``'s launches after everything queued so far on the current stream.  The buffers
        they touch must stay untouched by the current stream until :meth:`join`."""
        side = stream if stream is not None else _stream(dev)
        main = self._main
        if main is None or main.device != side.device or main.cuda_stream != _cur_handle():
            main = self._main = torch.cuda.current_stream(side.device)
        _wait(side, main, self._events)
        torch.cuda.set_stream(side)
        try:
            out = fn()
        finally:
            torch.cuda.set_stream(main)
        if side not in self._forks:
            self._forks.append(side)
        return out

    def join(self) -> None:
        for side in self._forks:
            _wait(torch.cuda.current_stream(side.device), side, self._events)
        self._forks.clear()
        # an event may be re-recorded once its waits are enqueued: each wait captured its record
        _EVENTS.extend(self._events)
        self._events.clear()


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


# PTG_ADAM_STREAM: the big Dense dW+Adam GEMM forks onto a second side stream.  On the shared side
# stream it ran first (the largest side kernel, ~0.25-0.36 ms) and every conv weight gradient queued
# behind it, so the last one (layer 2) still ran after the main stream's backward had finished.
ADAM_STREAM = config.get("adam_stream")


def launch(fn, dev, aux: bool = False):
    """Weight-gradient (or gradient-collective) launch: forked onto the side stream when a step has
    one, else inline.  ``aux``: the second side stream (PTG_ADAM_STREAM).  Returns ``fn()``'s result
    (e.g. an async collective's handle)."""
    side = _CUR[0]
    if side is not None and torch.device(dev).type == "cuda":
        return side.fork(fn, dev, stream=_stream(dev, 1) if aux and ADAM_STREAM else None)
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
