"""Host -> HBM input feed: the device half of ``tf.data``'s ``prefetch`` (train_tf_ps.py:301-321
prefetches decoded batches; TF's ``tf.data.experimental.prefetch_to_device`` is the API this
mirrors).

A background thread pulls host batches (numpy / CPU tensors: decoded uint8 images + targets) from
the upstream iterator, copies them into a ring of PINNED staging buffers that are allocated once
and reused, and issues the host->device copies on a dedicated HIP stream.  Each ring slot carries
two events:

* ``ready``  recorded on the copy stream after the H2D copy — the consumer's compute stream waits
  on it (a GPU-side wait: the host never blocks on the copy);
* ``free``   recorded on the compute stream after the step that used the slot — the copy stream
  waits on it before overwriting the slot's device buffers, so a slot is recycled only after the
  kernels that read it have finished.

With ``depth`` slots the copy of batch i+1.. overlaps the train step of batch i; raw uint8 images
cross PCIe at 1 byte/pixel and are normalised / channel-padded to bf16 by the model's first op on
the GPU.  :data:`STATS` counts batches and host-side wait time (a host-decode-bound pipeline shows
up as ``wait_s`` growing).
"""
from __future__ import annotations

import queue
import threading
import time

import numpy as np
import torch

STATS = {"batches": 0, "wait_s": 0.0, "h2d_bytes": 0}


def _host_tensor(a) -> torch.Tensor:
    if isinstance(a, torch.Tensor):
        return a.contiguous()
    return torch.from_numpy(np.ascontiguousarray(a))


class _Slot:
    def __init__(self):
        self.host: list = []
        self.dev: list = []
        self.ready = torch.cuda.Event()
        self.free = torch.cuda.Event()
        self.used = False

    def fit(self, parts, device) -> bool:
        if len(parts) != len(self.host):
            return False
        return all(h.shape == p.shape and h.dtype == p.dtype for h, p in zip(self.host, parts))

    def alloc(self, parts, device):
        self.host = [torch.empty(p.shape, dtype=p.dtype, pin_memory=True) for p in parts]
        self.dev = [torch.empty(p.shape, dtype=p.dtype, device=device) for p in parts]


class DeviceFeeder:
    """Iterator of device batches (tuples of tensors on ``device``) fed from host batches."""

    def __init__(self, source, device, depth: int = 3):
        self.src = iter(source)
        self.device = torch.device(device)
        self.depth = max(2, int(depth))
        self.copy_stream = torch.cuda.Stream(device=self.device)
        self.slots = [_Slot() for _ in range(self.depth)]
        self.free_q: queue.Queue = queue.Queue()
        for i in range(self.depth):
            self.free_q.put(i)
        self.ready_q: queue.Queue = queue.Queue()
        self._last = None
        self._stop = threading.Event()
        self._done = object()
        self._thread = threading.Thread(target=self._worker, daemon=True)
        self._thread.start()

    def _worker(self):
        try:
            torch.cuda.set_device(self.device)
            for batch in self.src:
                if self._stop.is_set():
                    return
                tup = batch if isinstance(batch, (tuple, list)) else (batch,)
                parts = [_host_tensor(a) for a in tup]
                i = self.free_q.get()
                if i is None:
                    return
                s = self.slots[i]
                if not s.fit(parts, self.device):
                    if s.used:
                        s.free.synchronize()  # old device buffers may still be read
                    s.alloc(parts, self.device)
                for h, p in zip(s.host, parts):
                    h.copy_(p)  # host memcpy into pinned staging (no GIL-held per-element work)
                with torch.cuda.stream(self.copy_stream):
                    if s.used:
                        self.copy_stream.wait_event(s.free)
                    for d, h in zip(s.dev, s.host):
                        d.copy_(h, non_blocking=True)
                    s.ready.record(self.copy_stream)
                # the pinned buffer is re-filled only after its copy ran: wait here (copy thread)
                s.ready.synchronize()
                STATS["h2d_bytes"] += sum(h.numel() * h.element_size() for h in s.host)
                self.ready_q.put((i, isinstance(batch, (tuple, list))))
        except BaseException as e:  # noqa: BLE001 - surface in the consumer
            self.ready_q.put(e)
            return
        self.ready_q.put(self._done)

    def __iter__(self):
        return self

    def __next__(self):
        self._release_last()
        t0 = time.perf_counter()
        item = self.ready_q.get()
        STATS["wait_s"] += time.perf_counter() - t0
        if item is self._done:
            self.ready_q.put(self._done)
            raise StopIteration
        if isinstance(item, BaseException):
            raise item
        i, was_tuple = item
        s = self.slots[i]
        torch.cuda.current_stream(self.device).wait_event(s.ready)
        self._last = i
        STATS["batches"] += 1
        out = tuple(s.dev)
        return out if was_tuple else out[0]

    def _release_last(self):
        """The previous batch's kernels are queued on the compute stream: mark its slot free."""
        if self._last is None:
            return
        s = self.slots[self._last]
        s.free.record(torch.cuda.current_stream(self.device))
        s.used = True
        self.free_q.put(self._last)
        self._last = None

    def close(self):
        self._stop.set()
        self.free_q.put(None)

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


def prefetch_to_device(device, buffer_size=None):
    """``tf.data.experimental.prefetch_to_device`` : ``ds.apply(prefetch_to_device("cuda:0"))``."""
    from .dataset import Dataset

    def apply(ds):
        depth = 3 if buffer_size in (None, -1) else max(2, int(buffer_size))
        dev = torch.device(device)
        if dev.type != "cuda" or not torch.cuda.is_available():
            return ds.prefetch(depth)
        out = Dataset(lambda: DeviceFeeder(ds, dev, depth), ds.cardinality())
        out._on_device = True
        return out

    return apply
