"""One-shot all-reduce of small GPU tensors over peer-mapped HBM (csrc/kernels/comm.hip).

RCCL's ring all-reduce is link-bandwidth-optimal for big buckets, but a few-KB message — the KMeans
partial sums of every Lloyd iteration (k_means.py:83-87: k x D sums + counts + cost, ~31 KB at k=100,
D=153), the DataFrame control plane's counts — pays 2*(world-1) dependent hops of latency.  On one
node every GPU maps every other GPU's memory over its xGMI links, so :class:`IpcAllReduce` does it
in ONE kernel: copy in, one epoch-flag round trip per 2048-element block, read the world's slots and
sum (see comm.hip for the slot / flag protocol and memory ordering).

Setup is collective: each rank hipMallocs a registered buffer (2 data slots of ``cap_bytes`` plus a
flag region), exports it with hipIpcGetMemHandle, all-gathers the 64-byte handles as a uint8 tensor
and opens the peers' buffers.  Ranks must share a node (LOCAL_WORLD_SIZE == WORLD_SIZE) and issue
their calls in the same order on one stream each.  A flag wait that exceeds its poll budget marks an
error word instead of hanging; :meth:`check` (and every ``check_every``-th call) raises on it, and
consumers call :func:`check_all` (via ``comm.check_fast_paths``) before they read a result.

Off by default: ``PTG_IPC_ALLREDUCE=1`` routes :func:`comm.all_reduce_tensor_` calls on CUDA tensors
of up to ``cap_bytes`` (fp32 / fp64 / int64, SUM) through it; RCCL handles everything else.
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.distributed as dist

from .. import _native
from .. import config

ENABLED = config.get("ipc_allreduce")
DEFAULT_CAP = 1 << 20
_DT = {torch.float32: 0, torch.float64: 1, torch.int64: 2}
_INSTANCES: dict = {}


def supported(world: int | None = None) -> bool:
    """One node, a GPU per rank, at most 16 ranks, and the native library present."""
    if not dist.is_initialized() or not torch.cuda.is_available():
        return False
    world = dist.get_world_size() if world is None else world
    if world < 2 or world > 16:
        return False
    if int(os.environ.get("LOCAL_WORLD_SIZE", world)) != world:
        return False
    try:
        _native.hip_lib()
    except _native.NativeUnavailable:
        return False
    return True


class IpcAllReduce:
    def __init__(self, device=None, cap_bytes: int = DEFAULT_CAP, spin_limit: int = 4_000_000, check_every: int = 64):
        self.world = dist.get_world_size()
        self.rank = dist.get_rank()
        self.dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self.cap = int(cap_bytes + 255) // 256 * 256
        self.spin_limit = int(spin_limit)
        self.check_every = max(1, int(check_every))
        lib = _native.hip_lib()
        if self.world > lib.ptg_ipc_max_world():
            raise ValueError(f"IpcAllReduce supports at most {lib.ptg_ipc_max_world()} ranks")
        hbytes = lib.ptg_ipc_handle_bytes()
        total = lib.ptg_ipc_flag_bytes() + 2 * self.cap
        with torch.cuda.device(self.dev):
            base = ctypes.c_void_p()
            handle = ctypes.create_string_buffer(hbytes)
            _native.check(lib.ptg_ipc_alloc(total, ctypes.byref(base), handle), "ptg_ipc_alloc")
            self._own = base.value
            # exchange the handles as a uint8 tensor (control device of the process group)
            ctl = self.dev if dist.get_backend() == "nccl" else torch.device("cpu")
            mine = torch.frombuffer(bytearray(handle.raw), dtype=torch.uint8).to(ctl)
            allh = torch.empty(self.world * hbytes, dtype=torch.uint8, device=ctl)
            dist.all_gather_into_tensor(allh, mine)
            allh = allh.cpu().numpy().tobytes()
            ptrs, self._opened = [], []
            for r in range(self.world):
                if r == self.rank:
                    ptrs.append(self._own)
                    continue
                hb = ctypes.create_string_buffer(allh[r * hbytes:(r + 1) * hbytes], hbytes)
                p = ctypes.c_void_p()
                _native.check(lib.ptg_ipc_open(hb, ctypes.byref(p)), "ptg_ipc_open")
                ptrs.append(p.value)
                self._opened.append(p.value)
        self._peers = (ctypes.c_uint64 * 16)(*ptrs, *([0] * (16 - self.world)))
        self.err = torch.zeros(1, dtype=torch.int32, device=self.dev)
        self.epoch = 0
        dist.barrier()  # every rank has opened every buffer before the first signal

    def fits(self, t: torch.Tensor) -> bool:
        return (t.is_cuda and t.device == self.dev and t.dtype in _DT and t.is_contiguous()
                and t.numel() * t.element_size() <= self.cap)

    def all_reduce_(self, t: torch.Tensor) -> torch.Tensor:
        """In-place SUM over all ranks (stream-ordered on the current stream)."""
        if not self.fits(t):
            raise ValueError("IpcAllReduce: tensor must be a contiguous fp32/fp64/int64 CUDA tensor on "
                             f"{self.dev} of at most {self.cap} bytes")
        self.epoch += 1
        if self.epoch >= (1 << 31) - 1:
            raise RuntimeError("IpcAllReduce epoch space exhausted; create a new instance")
        stream = torch.cuda.current_stream(self.dev).cuda_stream
        _native.check(_native.hip_lib().ptg_ipc_allreduce(
            t.data_ptr(), t.data_ptr(), t.numel(), _DT[t.dtype], ctypes.addressof(self._peers), self.world,
            self.rank, self.cap, self.epoch, self.err.data_ptr(), self.spin_limit, stream), "ptg_ipc_allreduce")
        if self.epoch % self.check_every == 0:
            self.check()
        return t

    def check(self) -> None:
        """Raise if any flag wait so far ran out of polls (a peer never arrived)."""
        if int(self.err.item()):
            raise RuntimeError("IpcAllReduce: a peer did not signal within the poll budget (ranks out of "
                               "step, or not all ranks issued the same all-reduces)")

    def close(self) -> None:
        if getattr(self, "_own", None) is None:
            return
        torch.cuda.synchronize(self.dev)
        dist.barrier()  # no peer still reads our buffer
        lib = _native.hip_lib()
        for p in self._opened:
            lib.ptg_ipc_close(ctypes.c_void_p(p))
        lib.ptg_ipc_free(ctypes.c_void_p(self._own))
        self._own = None


def check_all() -> None:
    """Raise if any live instance's flag wait timed out.  Call before reading results that went
    through the one-shot path (the per-call check runs only every ``check_every`` calls)."""
    for inst in list(_INSTANCES.values()):
        if getattr(inst, "_own", None) is not None:
            inst.check()


def get(device=None) -> IpcAllReduce | None:
    """The process-wide instance for the current process group (created collectively on first use)."""
    if not ENABLED or not supported():
        return None
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    key = (id(dist.group.WORLD), dev)
    inst = _INSTANCES.get(key)
    if inst is None:
        inst = _INSTANCES[key] = IpcAllReduce(dev)
    return inst
