"""Process-group bootstrap and the collectives the runtime uses (RCCL over xGMI on MI355X).

One OS process per GPU.  Ranks are launched by ``torch.distributed.run`` or by our own launcher
(:mod:`pyspark_tf_gke_amd.runtime.launcher`) and read RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT.  On GPUs the backend is ``nccl`` (= RCCL on ROCm); on CPU it is ``gloo``
(the multi-process CPU tests).

This replaces the reference's transports: Spark Netty shuffle/RPC (ports 7077/7078/7079,
spark_session.py:44-50) and TF gRPC between chief, workers and PS (train_tf_ps.py:501-504) —
SURVEY §2.4.  Tensor payloads go through RCCL; control goes through the TCP store torch creates.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist
from .. import config


def env_rank() -> tuple[int, int, int]:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return rank, local, world


def device_index() -> int:
    """This rank's GPU: LOCAL_RANK, or the launcher's PTG_DEVICE_ORDINAL after an executor was lost."""
    rank, local, _ = env_rank()
    return int(os.environ.get("PTG_DEVICE_ORDINAL", local)) % max(torch.cuda.device_count(), 1)


def is_initialized() -> bool:
    return dist.is_available() and dist.is_initialized()


def init(backend: str | None = None, device_type: str | None = None, timeout_s: int | None = None) -> tuple[int, int]:
    """Initialise the default process group from the environment (idempotent).
    Returns (rank, world_size).  ``timeout_s`` (default ``PTG_PG_TIMEOUT`` or 600 s) bounds every
    collective: a rank whose peer died or hung gets an error (gloo) or is aborted by the RCCL
    watchdog instead of blocking forever, exits non-zero, and the launcher restarts the group."""
    if timeout_s is None:
        timeout_s = int(config.get("pg_timeout_s"))
    rank, local, world = env_rank()
    if is_initialized():
        return dist.get_rank(), dist.get_world_size()
    if world <= 1 and not config.get("force_pg"):
        return 0, 1
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    if backend is None:
        # PTG_DIST_BACKEND=gloo: host-staged collectives even for GPU tensors (lets several ranks share
        # one GPU, e.g. a multi-rank rehearsal on a 1-GPU box; RCCL refuses duplicate devices)
        backend = config.get("dist_backend") or ("nccl" if device_type == "cuda" else "gloo")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29500")
    kw = {}
    if device_type == "cuda":
        dev = device_index()
        torch.cuda.set_device(dev)
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", dev)
    dist.init_process_group(backend=backend, rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=timeout_s), **kw)
    import atexit

    from ..runtime import heartbeat

    atexit.register(destroy)  # orderly teardown: no backend threads left running at interpreter exit
    heartbeat.start()
    return rank, world


def rank() -> int:
    return dist.get_rank() if is_initialized() else 0


def world_size() -> int:
    return dist.get_world_size() if is_initialized() else 1


def distributed() -> bool:
    """Whether the multi-rank code paths run: a process group of >1 ranks, or a 1-rank group with
    PTG_COLLECTIVES_WORLD1=1 (every collective site then runs through the real backend - RCCL on
    the GPU - against itself: the test of the N > 1 paths on one GPU)."""
    if not is_initialized():
        return False
    return dist.get_world_size() > 1 or bool(config.get("collectives_world1"))


def barrier() -> None:
    if is_initialized():
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def all_reduce_(t: torch.Tensor, op=dist.ReduceOp.SUM, async_op: bool = False):
    if not distributed():
        return None
    return dist.all_reduce(t, op=op, async_op=async_op)


def all_reduce_max_scalar(x: float) -> float:
    if not is_initialized():
        return x
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def broadcast_(t: torch.Tensor, src: int = 0):
    if distributed():
        dist.broadcast(t, src)
    return t


def reduce_scatter_flat(out_shard: torch.Tensor, full: torch.Tensor, async_op=False):
    return dist.reduce_scatter_tensor(out_shard, full, op=dist.ReduceOp.SUM, async_op=async_op)


def all_gather_flat(full: torch.Tensor, shard: torch.Tensor, async_op=False):
    return dist.all_gather_into_tensor(full, shard, async_op=async_op)


def all_to_all_v(send: torch.Tensor, send_counts: list[int], recv_counts: list[int] | None = None) -> torch.Tensor:
    """Variable all-to-all of rows (dim 0).  Size exchange first (one int64 all_to_all), then the
    payload with split sizes: the two-phase shuffle of SURVEY §5.8 / M12."""
    if not distributed():
        return send
    world = dist.get_world_size()
    dev = send.device
    if recv_counts is None:
        sc = torch.tensor(send_counts, dtype=torch.int64, device=dev)
        rc = torch.empty(world, dtype=torch.int64, device=dev)
        dist.all_to_all_single(rc, sc)
        recv_counts = rc.cpu().tolist()
    row = send.shape[1:]
    out = torch.empty((int(sum(recv_counts)), *row), dtype=send.dtype, device=dev)
    dist.all_to_all_single(out, send, output_split_sizes=[int(c) for c in recv_counts],
                           input_split_sizes=[int(c) for c in send_counts])
    return out


# ---- tensor control plane: small scalars / vectors travel as tensors (one collective each), never as
# pickled Python objects (no host serialisation, no extra all_gather of byte sizes)
def _ctl_device() -> torch.device:
    if is_initialized() and dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def all_reduce_int(values, op=dist.ReduceOp.SUM) -> list:
    """All-reduce a short list of Python ints (int64) -> list of ints."""
    vals = [int(v) for v in values]
    if not distributed():
        return vals
    t = torch.tensor(vals, dtype=torch.int64, device=_ctl_device())
    dist.all_reduce(t, op=op)
    return [int(x) for x in t.cpu().tolist()]


def all_reduce_float(values, op=dist.ReduceOp.SUM) -> list:
    """All-reduce a short list of Python floats (fp64) -> list of floats."""
    vals = [float(v) for v in values]
    if not distributed():
        return vals
    t = torch.tensor(vals, dtype=torch.float64, device=_ctl_device())
    dist.all_reduce(t, op=op)
    return [float(x) for x in t.cpu().tolist()]


def all_gather_int(value: int) -> list:
    """Every rank's int (one int64 all-gather) -> list in rank order."""
    if not distributed():
        return [int(value)]
    dev = _ctl_device()
    t = torch.tensor([int(value)], dtype=torch.int64, device=dev)
    out = torch.empty(dist.get_world_size(), dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(out, t)
    return [int(x) for x in out.cpu().tolist()]


def all_reduce_tensor_(t: torch.Tensor, op=dist.ReduceOp.SUM) -> torch.Tensor:
    """In-place all-reduce of a tensor on whatever device it lives (staged through the control
    device when the backend cannot reach it, e.g. CPU tensors under RCCL)."""
    if not distributed():
        return t
    if op == dist.ReduceOp.SUM and t.is_cuda:
        from . import ipc

        fast = ipc.get(t.device)  # PTG_IPC_ALLREDUCE=1: one-shot kernel over peer-mapped HBM
        if fast is not None and fast.fits(t):
            return fast.all_reduce_(t)
    dev = _ctl_device()
    if t.device == dev or (dev.type == "cuda" and t.is_cuda):
        dist.all_reduce(t, op=op)
        return t
    s = t.to(dev)
    dist.all_reduce(s, op=op)
    t.copy_(s.to(t.device))
    return t


def check_fast_paths() -> None:
    """Fail loudly if a one-shot IPC all-reduce issued so far timed out (its error word is only read
    every few calls, so a consumer calls this before it trusts the reduced values)."""
    if not distributed():
        return
    from . import ipc

    ipc.check_all()


def all_gather_v(t: torch.Tensor) -> list:
    """Variable-length all-gather along dim 0 -> list of per-rank tensors (on ``t``'s device).
    One int64 all-gather of the lengths, then one all_gather_into_tensor of the padded rows."""
    if not distributed():
        return [t]
    world = dist.get_world_size()
    dev = _ctl_device()
    n = torch.tensor([t.shape[0]], dtype=torch.int64, device=dev)
    ns = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(ns, n)
    lens = [int(x) for x in ns.cpu().tolist()]
    out, mx = _all_gather_padded(t, lens, dev)
    return [out[r * mx: r * mx + lens[r]].to(t.device) for r in range(world)]


def _all_gather_padded(t: torch.Tensor, lens: list, dev) -> tuple:
    """All-gather of every rank's rows padded to the longest (the pad rows are never read, so they
    are not initialised): -> (out [world * mx, ...] on ``dev``, mx)."""
    world = len(lens)
    mx = max(lens)
    row = t.shape[1:]
    if t.shape[0] == mx and t.device == torch.device(dev) and t.is_contiguous():
        src = t
    else:
        src = torch.empty((mx, *row), dtype=t.dtype, device=dev)
        if t.shape[0]:
            src[: t.shape[0]].copy_(t)
    out = torch.empty((world * mx, *row), dtype=t.dtype, device=dev)
    dist.all_gather_into_tensor(out, src)
    return out, mx


def all_gather_v_host(t: torch.Tensor):
    """:func:`all_gather_v` concatenated in rank order as ONE host numpy array (one device-to-host
    copy of the padded gather, the concatenation done on the host)."""
    import numpy as np

    if not distributed():
        return t.cpu().numpy()
    world = dist.get_world_size()
    dev = _ctl_device()
    n = torch.tensor([t.shape[0]], dtype=torch.int64, device=dev)
    ns = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(ns, n)
    lens = [int(x) for x in ns.cpu().tolist()]
    if max(lens) == 0:
        return t.cpu().numpy()[:0]
    out, mx = _all_gather_padded(t, lens, dev)
    h = out.cpu().numpy()
    return np.concatenate([h[r * mx: r * mx + lens[r]] for r in range(world)])


def all_gather_unique(t: torch.Tensor) -> torch.Tensor:
    """Sorted union of the per-rank distinct values of a 1-D tensor."""
    parts = all_gather_v(t)
    allv = torch.cat(parts)
    if allv.is_cuda and allv.dtype == torch.int64:
        from ..ops import df as D

        # our kernels: distinct by hash aggregation, orderable form radix-sorted, decoded back
        kt = D.TORCH_CT[torch.int64]
        return D.decode_sort_key(D.sorted_orderable(D.distinct_raw(allv), kt), torch.int64, False)
    return torch.unique(allv)


def all_gather_bytes(blobs: list) -> list:
    """Every rank's list of byte strings, in rank order: one all_gather_v of the int64 lengths and
    one of the concatenated uint8 payload (tensors only, nothing pickled)."""
    if not distributed():
        return [list(blobs)]
    lens = torch.tensor([len(b) for b in blobs], dtype=torch.int64)
    raw = b"".join(blobs)
    data = torch.frombuffer(bytearray(raw), dtype=torch.uint8) if raw else torch.zeros(0, dtype=torch.uint8)
    all_lens = all_gather_v(lens.to(_ctl_device()))
    all_data = all_gather_v(data.to(_ctl_device()))
    out = []
    for ln, dt in zip(all_lens, all_data):
        buf = dt.cpu().numpy().tobytes()
        parts, o = [], 0
        for n in ln.cpu().tolist():
            parts.append(buf[o:o + n])
            o += n
        out.append(parts)
    return out


def _str_hash64(s: str) -> int:
    import hashlib

    return int.from_bytes(hashlib.blake2b(s.encode("utf-8"), digest_size=8).digest(), "little", signed=True)


def union_strings(strings: list) -> list:
    """Union of every rank's string list, first occurrence in rank order (identical on every rank).
    Tensor control plane: one all_gather_v of 64-bit string hashes decides which rank first holds
    each distinct string, then only those strings' UTF-8 bytes travel (all_gather_bytes)."""
    strings = list(strings)
    if not distributed():
        seen, out = set(), []
        for x in strings:
            if x not in seen:
                seen.add(x)
                out.append(x)
        return out
    rank = dist.get_rank()
    h = torch.tensor([_str_hash64(x) for x in strings], dtype=torch.int64)
    per_rank = [t.cpu().tolist() for t in all_gather_v(h.to(_ctl_device()))]
    seen: set = set()
    first: list = []  # (rank, index) of every first occurrence, in merge order
    for r, hs in enumerate(per_rank):
        for i, x in enumerate(hs):
            if x not in seen:
                seen.add(x)
                first.append((r, i))
    mine = [strings[i].encode("utf-8") for r, i in first if r == rank]
    got = all_gather_bytes(mine)
    cursor = [0] * len(got)
    out = []
    for r, _ in first:
        out.append(got[r][cursor[r]].decode("utf-8"))
        cursor[r] += 1
    return out


def all_gather_object(obj):
    if not distributed():
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def destroy() -> None:
    if is_initialized():
        dist.destroy_process_group()
