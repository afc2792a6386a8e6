"""ParameterServerStrategy on GPU ranks (the reference's strategy, train_tf_ps.py:440-511, 612-645).

Every rank is a worker and hosts PS tasks.  Variables are cut by ``variable_partitioner`` (default
``MinSizePartitioner(256 KiB, max_shards=#ps)``, :505-507) along axis 0 and the shards are placed
round-robin over the PS tasks; PS task t lives on rank ``t % world``.  An owner keeps its shards
packed in one segment: the forward-bf16 pieces (matmul / conv weights) first, then the pieces the
forward reads in fp32 (biases, PReLU alphas).

Data movement is ONE kernel per direction and step (``ptg_piece_copy``, csrc/kernels/comm.hip): the
pieces are pre-split into <= 64K-element chunks in a device table, and every chunk is copied between
the flat parameter store and the owners' segments with the fp32 <-> bf16 conversion on the way.

``mode="sync"`` (default, TF's ``ClusterCoordinator`` rounds made collective): push = the packed
gradients reduce-scattered to the owners (one collective), each owner applies the optimizer to its
shards with the gradient averaged over the workers that contributed, pull = ONE bf16 all-gather of
the forward-bf16 pieces + one fp32 all-gather of the (small) fp32 pieces, unpacked by one kernel
each.  Workers never hold a current fp32 copy of the bf16 pieces between steps
(``store.master_stale``; ``synchronize_master`` pulls it).

``mode="async"`` (TF's asynchronous PS): no collective per step.  Each rank exposes a one-sided
*window* - [owned fp32 values][owned bf16 values][NSLOT gradient inbox slots] - in HBM exported
with HIP IPC (peers map it over xGMI; on CPU ranks a shared-memory file).  A worker's push claims a
ticket per owner (an atomic fetch-add in a /dev/shm control block, :class:`_Mailbox`, signalled
with shared futexes by csrc/host/shmsync.cpp instead of TCP-store round trips), writes its gradient
pieces straight into the owners' inbox slots (one kernel for all owners), publishes the tickets and
waits until the owners applied them
(``apply_gradients`` returns after the PS update, as in TF); each owner runs a service thread that
applies every push as its own optimizer step, in ticket order, on its own HIP stream - while its
main thread is busy with its own closure.  Pulls read the owners' bf16 / fp32 values directly from
their windows (system-scope loads, no owner involvement).  With :class:`~.coordinator.
ClusterCoordinator` closures are handed to whichever worker is idle (a store ticket per closure), so
a slow worker runs fewer steps instead of stalling the others.
"""
from __future__ import annotations

import ctypes
import datetime
import math
import mmap
import os
import threading
import uuid

import torch
import torch.distributed as dist

from .. import config
from ..parallel import comm
from .cluster import ClusterSpec, MinSizePartitioner, TFConfigClusterResolver
from .strategy import Strategy

_CHUNK = 1 << 16  # elements per device-table chunk (one workgroup each)
NSLOT = 4  # gradient inbox slots per owner (pushes in flight to one owner)
_MAX_WINDOWS = 16  # base addresses one ptg_piece_copy launch takes (comm.hip IPC_MAXW)


_TLS = threading.local()


def _store():
    """This thread's own client of the job's TCP store (MASTER_ADDR:MASTER_PORT).  A TCPStore client
    serialises its requests, so the owner service thread (blocked in ``wait`` most of the time) and
    the main thread must not share one."""
    st = getattr(_TLS, "store", None)
    if st is None:
        host = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ.get("MASTER_PORT", "29500"))
        st = _TLS.store = dist.TCPStore(host, port, is_master=False, wait_for_workers=False,
                                        timeout=datetime.timedelta(seconds=int(config.get("pg_timeout_s"))))
    return st


class _Piece:
    __slots__ = ("param", "lo", "n", "owner", "task", "xlo", "bf")

    def __init__(self, param, lo, n, owner, task, bf):
        self.param, self.lo, self.n, self.owner, self.task, self.bf = param, lo, n, owner, task, bf
        self.xlo = -1


class _PieceTable:
    """Rows (src base index, src element offset, dst base index, dst element offset, n).  The host
    rows drive the CPU path; on the GPU the rows are split into chunks in a device int64 table and
    the copy is one ``ptg_piece_copy`` launch."""

    def __init__(self, rows, device):
        self.rows = [r for r in rows if r[4] > 0]
        self.dev = None
        self.nch = 0
        if device.type == "cuda" and self.rows:
            ch = []
            for ss, so, ds, do, n in self.rows:
                for o in range(0, n, _CHUNK):
                    ch.append((ss, so + o, ds, do + o, min(_CHUNK, n - o)))
            self.dev = torch.tensor(ch, dtype=torch.int64, device=device).reshape(-1)
            self.nch = len(ch)

    def copy(self, srcs, src_bf16: bool, dsts, dst_bf16: bool, sys: bool = False) -> None:
        """``srcs`` / ``dsts``: per base index a 1-D tensor, or (GPU) a raw device address of a peer's
        window.  ``sys``: system-scope loads (a source another rank writes)."""
        if not self.rows:
            return
        if self.dev is None:
            for ss, so, ds, do, n in self.rows:
                dsts[ds][do:do + n].copy_(srcs[ss][so:so + n])
            return
        from .. import _native
        from ..ops._util import stream_handle

        if len(srcs) > _MAX_WINDOWS or len(dsts) > _MAX_WINDOWS:
            raise ValueError(f"ptg_piece_copy takes at most {_MAX_WINDOWS} base addresses per side")

        def bases(xs):
            arr = (ctypes.c_uint64 * _MAX_WINDOWS)()
            for i, x in enumerate(xs):
                arr[i] = x if isinstance(x, int) else x.data_ptr()
            return arr

        sb, db = bases(srcs), bases(dsts)
        _native.check(_native.hip_lib().ptg_piece_copy(
            ctypes.addressof(sb), len(srcs), int(src_bf16), ctypes.addressof(db), len(dsts), int(dst_bf16),
            self.dev.data_ptr(), self.nch, int(sys), stream_handle()), "ptg_piece_copy")


class _PSPlan:
    """Variable placement of one model (see the module docstring): per owner a packed segment of
    ``seg = seg_b + seg_f`` elements, forward-bf16 pieces in [0, seg_b), fp32 pieces in
    [seg_b, seg); the owner keeps its shards' fp32 values (``master``), their bf16 copy
    (``master_bf``) and optimizer moments in that layout: the variables live on the PS."""

    def __init__(self, model, partitioner, num_ps: int, world: int, rank: int, windows: bool = False):
        from ..nn.params import ALIGN

        st = model.store
        self.pieces: list[_Piece] = []
        task = 0
        for p in sorted(st.params, key=lambda q: q.order):  # variable creation order
            k = partitioner.num_shards(p.shape, 4) if partitioner is not None else 1
            rows = p.shape[0] if p.shape else 1
            row_elems = p.numel // max(rows, 1)
            k = max(1, min(k, rows))
            base, rem = divmod(rows, k)
            r0 = 0
            for j in range(k):
                nr = base + (1 if j < rem else 0)
                t = task % num_ps
                self.pieces.append(_Piece(p, p.offset + r0 * row_elems, nr * row_elems, t % world, t,
                                          bool(p.fwd_bf16)))
                r0 += nr
                task += 1
        nb, nf = [0] * world, [0] * world
        for pc in self.pieces:
            if pc.bf:
                pc.xlo = nb[pc.owner]
                nb[pc.owner] += pc.n
        self.seg_b = int(math.ceil(max(nb) / ALIGN) * ALIGN) if max(nb) else 0
        for pc in self.pieces:
            if not pc.bf:
                pc.xlo = self.seg_b + nf[pc.owner]
                nf[pc.owner] += pc.n
        self.seg_f = int(math.ceil(max(nf) / ALIGN) * ALIGN) if max(nf) else 0
        self.seg = max(ALIGN, self.seg_b + self.seg_f)
        self.owner_elems = [nb[r] + nf[r] for r in range(world)]
        self.world, self.rank = world, rank
        self.mine = [pc for pc in self.pieces if pc.owner == rank]
        dev = st.flat.device
        self.device = dev
        T = lambda rows: _PieceTable(rows, dev)  # noqa: E731
        # push: fp32 gradient pieces -> owner segments; pulls: owner segments -> flat store.
        # windows (async): one base address per owner (its IPC / shm window, <= 16 of them);
        # otherwise the owners' segments are consecutive slices of ONE collective buffer, so every
        # row names base 0 at the owner's slice offset and the world size is not capped.
        self.windows = windows

        def own(pc, size, off):  # (base index, element offset) of a piece in an owner layout
            return (pc.owner, off) if windows else (0, pc.owner * size + off)

        self.t_push = T([(0, pc.lo) + own(pc, self.seg, pc.xlo) + (pc.n,) for pc in self.pieces])
        self.t_pull_b = T([own(pc, self.seg_b, pc.xlo) + (0, pc.lo, pc.n) for pc in self.pieces if pc.bf])
        self.t_pull_f = T([own(pc, self.seg_f, pc.xlo - self.seg_b) + (0, pc.lo, pc.n)
                           for pc in self.pieces if not pc.bf])
        self.t_pull_all = T([own(pc, self.seg, pc.xlo) + (0, pc.lo, pc.n) for pc in self.pieces])
        self.t_own = T([(0, pc.lo, 0, pc.xlo, pc.n) for pc in self.mine])
        self.xbuf = None  # sync push buffer (world * seg fp32), allocated on first use
        self.gshard = torch.zeros(self.seg, dtype=torch.float32, device=dev)
        self.master = torch.zeros(self.seg, dtype=torch.float32, device=dev)  # owned values
        self.master_bf = torch.zeros(self.seg, dtype=st.flat_bf16.dtype, device=dev)
        self.slots: dict[str, torch.Tensor] = {}  # packed optimizer moments of the owned shards
        self.window = None
        self.pack_params(st)

    def placement(self) -> list:
        """[(param name, row range, ps task, owner rank)] — the variable-to-PS map."""
        out = []
        for pc in self.pieces:
            rows = pc.param.shape[0] if pc.param.shape else 1
            re = pc.param.numel // max(rows, 1)
            r0 = (pc.lo - pc.param.offset) // max(re, 1)
            out.append((pc.param.name, (r0, r0 + pc.n // max(re, 1)), pc.task, pc.owner))
        return out

    def segs(self, t: torch.Tensor) -> list:
        return [t[r * self.seg:(r + 1) * self.seg] for r in range(self.world)]

    def pack_params(self, st) -> None:
        """Owned shards' values from the full layout (registration / checkpoint load)."""
        self.t_own.copy([st.flat], False, [self.master], False)
        from ..ops import nn as K

        K.cast_f32_bf16(self.master, self.master_bf)
        if self.window is not None:
            self.window.publish_values(self.master, self.master_bf)

    def slot(self, name: str) -> torch.Tensor:
        t = self.slots.get(name)
        if t is None:
            t = self.slots[name] = torch.zeros(self.seg, dtype=torch.float32, device=self.master.device)
        return t


def _apply_packed(opt, master, grad, slot, master_bf, step: int, gscale: float) -> None:
    """One optimizer step of an owner's packed shards (Adam or SGD, the fused flat kernels)."""
    from ..nn import optimizers as OPT
    from ..ops import nn as K

    n = master.numel()
    if isinstance(opt, OPT.Adam):
        K.adam(master, grad[:n], slot("m"), slot("v"), master_bf, opt.lr_t(step), opt.beta_1, opt.beta_2,
               opt.epsilon, gscale)
    elif isinstance(opt, OPT.SGD):
        vel = slot("velocity") if opt.momentum > 0 else None
        K.sgd(master, grad[:n], vel, master_bf, opt.learning_rate, opt.momentum, opt.nesterov, gscale)
    else:
        raise TypeError(f"unsupported optimizer {type(opt).__name__}")


class _PSWindow:
    """One-sided PS memory of every rank (async mode).  Layout per rank (bytes):
    [values fp32: seg][values bf16: seg][inbox: NSLOT x seg fp32].  GPU: a device buffer exported
    with HIP IPC (handle + offset all-gathered as tensors, peers map it with hipIpcOpenMemHandle);
    CPU: a /dev/shm file every rank maps."""

    def __init__(self, plan: _PSPlan, prefix: str):
        self.plan, self.prefix = plan, prefix
        seg = plan.seg
        self.bf_dtype = plan.master_bf.dtype  # bf16 (fp32 in the host fp32 mode)
        self.o_vals = 0
        self.o_bf = seg * 4
        self.o_inbox = self.o_bf + ((seg * plan.master_bf.element_size() + 255) // 256) * 256
        self.nbytes = self.o_inbox + NSLOT * seg * 4
        self.world, self.rank = plan.world, plan.rank
        dev = plan.device
        self.cuda = dev.type == "cuda"
        self._opened: list = []
        self._files: list = []
        if self.cuda:
            from .. import _native

            lib = _native.hip_lib()
            self.buf = torch.zeros(self.nbytes, dtype=torch.uint8, device=dev)
            hb = lib.ptg_ipc_handle_bytes()
            handle = ctypes.create_string_buffer(hb)
            off = ctypes.c_long()
            _native.check(lib.ptg_ipc_export(self.buf.data_ptr(), handle, ctypes.byref(off)), "ptg_ipc_export")
            ctl = dev if dist.get_backend() == "nccl" else torch.device("cpu")
            mine = torch.frombuffer(bytearray(handle.raw + int(off.value).to_bytes(8, "little")),
                                    dtype=torch.uint8).to(ctl)
            allh = torch.empty(self.world * (hb + 8), dtype=torch.uint8, device=ctl)
            dist.all_gather_into_tensor(allh, mine)
            raw = allh.cpu().numpy().tobytes()
            self.bases = []
            for r in range(self.world):
                if r == self.rank:
                    self.bases.append(self.buf.data_ptr())
                    continue
                rec = raw[r * (hb + 8):(r + 1) * (hb + 8)]
                p = ctypes.c_void_p()
                _native.check(lib.ptg_ipc_open(ctypes.create_string_buffer(rec[:hb], hb), ctypes.byref(p)),
                              "ptg_ipc_open")
                self._opened.append(p.value)
                self.bases.append(p.value + int.from_bytes(rec[hb:], "little"))
            self.peer_bufs = None
        else:
            token = prefix.replace("/", "_")
            path = f"/dev/shm/ptg_ps_{token}_{self.rank}"
            with open(path, "wb") as fh:
                fh.truncate(self.nbytes)
            self._files.append(path)
            self.buf = torch.from_file(path, shared=True, size=self.nbytes, dtype=torch.uint8)
            comm.barrier()
            self.peer_bufs = [self.buf if r == self.rank else
                              torch.from_file(f"/dev/shm/ptg_ps_{token}_{r}", shared=True, size=self.nbytes,
                                              dtype=torch.uint8) for r in range(self.world)]
            self.bases = None
        comm.barrier()  # every rank has mapped every window

    # ---- views / addresses
    def _view(self, r: int, off: int, n: int, dtype):
        esz = torch.tensor([], dtype=dtype).element_size()
        if self.cuda:
            if r == self.rank:
                return self.buf[off:off + n * esz].view(dtype)
            return self.bases[r] + off  # raw peer address (element offsets are added by the kernel)
        return self.peer_bufs[r][off:off + n * esz].view(dtype)

    def vals(self, r: int):
        return self._view(r, self.o_vals, self.plan.seg, torch.float32)

    def vals_f(self, r: int):
        v = self.vals(r)
        off = self.plan.seg_b
        return v[off:] if isinstance(v, torch.Tensor) else v + off * 4

    def vals_bf(self, r: int):
        return self._view(r, self.o_bf, self.plan.seg, self.bf_dtype)

    def inbox(self, r: int, slot: int):
        return self._view(r, self.o_inbox + slot * self.plan.seg * 4, self.plan.seg, torch.float32)

    def publish_values(self, master, master_bf) -> None:
        """The owner's current values into its own window (registration / checkpoint load)."""
        self.vals(self.rank).copy_(master)
        self.vals_bf(self.rank).copy_(master_bf)

    def close(self) -> None:
        if self.cuda and self._opened:
            from .. import _native

            torch.cuda.synchronize(self.plan.device)
            lib = _native.hip_lib()
            for p in self._opened:
                lib.ptg_ipc_close(ctypes.c_void_p(p))
            self._opened = []
        for f in self._files:
            try:
                os.unlink(f)
            except OSError:
                pass
        self._files = []


class _Mailbox:
    """Push signalling of one async-PS model between the ranks of a node: per owner one 64-byte line
    each for the ticket counter, the applied counter and a stop word, then NSLOT slot lines
    (sequence, optimizer index, gradient scale).  Rank 0 creates the /dev/shm file, every rank maps
    it; the atomics and futex waits are csrc/host/shmsync.cpp."""

    LINE = 64
    PER = 3 + NSLOT

    def __init__(self, path: str, world: int, rank: int):
        from .. import _native

        self.lib = _native.host_lib()
        self.path, self.world, self.owner_file = path, world, rank == 0
        size = world * self.PER * self.LINE
        if rank == 0:
            with open(path, "wb") as fh:
                fh.truncate(size)
        comm.barrier()
        fd = os.open(path, os.O_RDWR)
        try:
            self.mm = mmap.mmap(fd, size)
        finally:
            os.close(fd)
        self._anchor = ctypes.c_char.from_buffer(self.mm)
        self.base = ctypes.addressof(self._anchor)
        self.timeout_s = float(config.get("pg_timeout_s"))

    def _line(self, r: int, k: int) -> ctypes.c_void_p:
        return ctypes.c_void_p(self.base + (r * self.PER + k) * self.LINE)

    def ticket(self, r: int) -> int:
        old = ctypes.c_int()
        self.lib.ptgh_shm_add(self._line(r, 0), 1, ctypes.byref(old))
        return old.value

    def tickets_issued(self, r: int) -> int:
        v = ctypes.c_int()
        self.lib.ptgh_shm_load(self._line(r, 0), ctypes.byref(v))
        return v.value

    def wait_applied(self, r: int, n: int, alive=None) -> None:
        """Block until owner r applied n pushes; ``alive()`` raises if this rank's own service died."""
        waited = 0.0
        while self.lib.ptgh_shm_wait_ge(self._line(r, 1), int(n), 1_000_000):
            waited += 1.0
            if alive is not None:
                alive()
            if waited >= self.timeout_s:
                raise RuntimeError(f"parameter server {r} did not apply push {n - 1} within {self.timeout_s:.0f} s")

    def set_applied(self, r: int, n: int) -> None:
        self.lib.ptgh_shm_store(self._line(r, 1), int(n))

    def publish(self, r: int, t: int, gscale: float, oi: int) -> None:
        self.lib.ptgh_mbox_publish(self._line(r, 3 + t % NSLOT), t + 1, float(gscale), int(oi))

    def take(self, r: int, t: int, timeout_us: int):
        """(gscale, optimizer index) of push t to owner r, or None on timeout."""
        g, oi = ctypes.c_double(), ctypes.c_int()
        if self.lib.ptgh_mbox_take(self._line(r, 3 + t % NSLOT), t + 1, int(timeout_us), ctypes.byref(g),
                                   ctypes.byref(oi)):
            return None
        return g.value, oi.value

    def wake(self, r: int, t: int) -> None:
        self.lib.ptgh_shm_wake(self._line(r, 3 + t % NSLOT))

    def close(self) -> None:
        if self.mm is None:
            return
        del self._anchor
        self.mm.close()
        self.mm = None
        if self.owner_file:
            try:
                os.unlink(self.path)
            except OSError:
                pass


class _OwnerService(threading.Thread):
    """Applies the pushes addressed to this rank's shards, one optimizer step each, in ticket order,
    on its own stream, while the rank's main thread runs closures (async mode)."""

    def __init__(self, strategy, model, plan: _PSPlan, win: _PSWindow, prefix: str):
        super().__init__(daemon=True, name=f"ptg-ps-owner-{prefix}")
        self.st, self.model, self.plan, self.win, self.prefix = strategy, model, plan, win, prefix
        self.applied = 0
        # optimizer steps applied before this service's first push (a restored checkpoint): Adam's
        # bias correction continues from there (on_state_loaded sets it)
        self.step_offset = 0
        self.last_opt = None
        self.stop_flag = False
        self.error: BaseException | None = None
        self.grad = torch.zeros(plan.seg, dtype=torch.float32, device=plan.device)
        self._one = _PieceTable([(0, 0, 0, 0, plan.seg)], plan.device)

    def run(self):  # noqa: D401 - thread body
        rank = self.plan.rank
        mbox = self.plan.mbox
        if self.plan.device.type == "cuda":
            torch.cuda.set_device(self.plan.device)  # a new thread starts on device 0
        stream = torch.cuda.Stream(self.plan.device) if self.plan.device.type == "cuda" else None
        try:
            while not self.stop_flag:
                got = mbox.take(rank, self.applied, 500_000)
                if got is None:  # timeout: look at the stop flag, wait again
                    continue
                gscale, oi = got
                t = self.applied
                opt = self.st.optimizers[oi] if oi >= 0 else self.model.optimizer
                self.last_opt = opt
                ctx = torch.cuda.stream(stream) if stream is not None else _nullctx()
                with ctx:
                    # the inbox slot is written by peers: read it with system-scope loads
                    self._one.copy([self.win.inbox(rank, t % NSLOT)], False, [self.grad], False, sys=True)
                    master = self.win.vals(rank)
                    _apply_packed(opt, master, self.grad, self.plan.slot, self.win.vals_bf(rank),
                                  self.step_offset + t + 1, gscale)
                if stream is not None:
                    stream.synchronize()
                self.applied = t + 1
                mbox.set_applied(rank, t + 1)
        except BaseException as e:  # noqa: BLE001 - surfaced to the main thread on its next push
            self.error = e


class _nullctx:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


class ParameterServerStrategy(Strategy):
    """See the module docstring.  ``mode`` defaults to ``PTG_PS_MODE`` (``sync``)."""

    _instances = 0

    def __init__(self, cluster_resolver=None, variable_partitioner=None, device=None, mode: str | None = None):
        super().__init__(device)
        self.cluster_resolver = cluster_resolver or TFConfigClusterResolver()
        spec = self.cluster_resolver.cluster_spec() if hasattr(self.cluster_resolver, "cluster_spec") else ClusterSpec({})
        self.cluster_spec = ClusterSpec(spec)
        self.num_workers = max(self.cluster_spec.num_tasks("worker"), self.world_size)
        self.num_ps = self.cluster_spec.num_tasks("ps") or self.world_size
        self.variable_partitioner = variable_partitioner or MinSizePartitioner(256 << 10, max(self.num_ps, 1))
        self.mode = (mode or config.get("ps_mode")).lower()
        if self.mode not in ("sync", "async"):
            raise ValueError(f"ParameterServerStrategy mode must be 'sync' or 'async', not {self.mode!r}")
        ParameterServerStrategy._instances += 1
        self._sid = ParameterServerStrategy._instances
        self._services: list = []
        self._token = None

    @property
    def is_async(self) -> bool:
        return self.mode == "async" and self.world_size > 1

    def register_model(self, model) -> None:
        super().register_model(model)  # broadcast rank 0's initial values first
        if self.is_async and self.world_size > _MAX_WINDOWS:
            raise ValueError(f"asynchronous ParameterServerStrategy maps every rank's window into one copy kernel: "
                             f"at most {_MAX_WINDOWS} ranks (world size {self.world_size}); use mode='sync'")
        lws = os.environ.get("LOCAL_WORLD_SIZE")
        if self.is_async and lws is not None and int(lws) != self.world_size:
            raise ValueError("asynchronous ParameterServerStrategy signals gradient pushes through a /dev/shm "
                             "control block and maps its peers' windows by HIP IPC: every rank must run on one node "
                             f"(LOCAL_WORLD_SIZE {lws} != WORLD_SIZE {self.world_size}); use mode='sync' across nodes")
        plan = model._ps_plan = _PSPlan(model, self.variable_partitioner, self.num_ps, self.world_size, self.rank,
                                        windows=self.is_async)
        if self.is_async:
            if self._token is None:  # one job-unique token for the store keys and shm files
                store = _store()
                key = f"ptg/ps/{self._sid}/token"
                if self.rank == 0:
                    store.set(key, uuid.uuid4().hex[:12])
                self._token = store.get(key).decode()
            prefix = f"ptg/ps/{self._token}/{len(self.models) - 1}"
            plan.window = _PSWindow(plan, prefix)
            plan.window.publish_values(plan.master, plan.master_bf)
            plan.prefix = prefix
            plan.mbox = _Mailbox("/dev/shm/" + prefix.replace("/", "_") + "_ctl", self.world_size, self.rank)
            plan.tickets = [0] * self.world_size
            svc = _OwnerService(self, model, plan, plan.window, prefix)
            plan.service = svc
            self._services.append(svc)
            comm.barrier()
            svc.start()

    def placement(self, model) -> list:
        return model._ps_plan.placement()

    # ---- sync mode -------------------------------------------------------------------------------
    def _pull(self, model) -> None:
        """bf16 values of the forward-bf16 pieces + fp32 values of the rest, from every owner."""
        plan = model._ps_plan
        st = model.store
        if self.is_async:
            win = plan.window
            plan.t_pull_b.copy([win.vals_bf(r) for r in range(self.world_size)], True, [st.flat_bf16], True, sys=True)
            plan.t_pull_f.copy([win.vals_f(r) for r in range(self.world_size)], False, [st.flat], False, sys=True)
        else:
            if plan.seg_b:
                xb = torch.empty(self.world_size * plan.seg_b, dtype=plan.master_bf.dtype, device=plan.device)
                comm.all_gather_flat(xb, plan.master_bf[:plan.seg_b].contiguous())
                plan.t_pull_b.copy([xb], True, [st.flat_bf16], True)
            if plan.seg_f:
                xf = torch.empty(self.world_size * plan.seg_f, dtype=torch.float32, device=plan.device)
                comm.all_gather_flat(xf, plan.master[plan.seg_b:plan.seg_b + plan.seg_f].contiguous())
                plan.t_pull_f.copy([xf], False, [st.flat], False)
        st.master_stale = plan.seg_b > 0 and st.flat_bf16.data_ptr() != st.flat.data_ptr()

    def _push_apply_sync(self, model, opt, contributed: list) -> None:
        plan = model._ps_plan
        st = model.store
        n_ok = sum(bool(c) for c in contributed)
        if plan.xbuf is None:
            plan.xbuf = torch.zeros(self.world_size * plan.seg, dtype=torch.float32, device=plan.device)
        if contributed[self.rank]:
            plan.t_push.copy([st.flat_grad], False, [plan.xbuf], False)
        else:
            plan.xbuf.zero_()
        comm.reduce_scatter_flat(plan.gshard, plan.xbuf)
        _apply_packed(opt, plan.master, plan.gshard, plan.slot, plan.master_bf, opt.iterations + 1, 1.0 / n_ok)
        opt.iterations += 1
        self._pull(model)

    # ---- async mode ------------------------------------------------------------------------------
    def _push_async(self, model, opt) -> None:
        """Send this worker's gradient to every owner and wait until each applied it (TF:
        ``apply_gradients`` on PS variables returns after the PS update); then pull."""
        plan = model._ps_plan
        st = model.store
        svc = plan.service
        if svc.error is not None:
            raise RuntimeError("parameter-server service thread failed") from svc.error
        # the owners name the optimizer by its index in strategy.optimizers, which is the same on
        # every rank only for optimizers created under strategy.scope(); the model's compiled
        # optimizer is addressed as "" (every owner has its own copy of that model)
        if any(o is opt for o in self.optimizers):
            oi = next(i for i, o in enumerate(self.optimizers) if o is opt)
        elif opt is model.optimizer:
            oi = -1
        else:
            raise RuntimeError("asynchronous ParameterServerStrategy: create the optimizer under strategy.scope() "
                               "(or compile it into the model) so every parameter server knows it")
        owners = [r for r in range(self.world_size) if plan.owner_elems[r] > 0]
        mbox = plan.mbox
        tick = {}
        for r in owners:
            t = mbox.ticket(r)
            if t >= NSLOT:  # the slot's previous push must have been consumed
                mbox.wait_applied(r, t - NSLOT + 1, self._check_service(svc))
            tick[r] = t
        win = plan.window
        dsts = [win.inbox(r, tick[r] % NSLOT) if r in tick else win.inbox(self.rank, 0)
                for r in range(self.world_size)]
        plan.t_push.copy([st.flat_grad], False, dsts, False)
        if st.flat_grad.is_cuda:
            torch.cuda.current_stream(st.flat_grad.device).synchronize()
        for r, t in tick.items():
            mbox.publish(r, t, self._commit_scale, oi)
        self._closure_pushed = True  # from here on the update is applied whatever the closure does next
        for r, t in tick.items():
            mbox.wait_applied(r, t + 1, self._check_service(svc))
        opt.iterations += 1
        self._pull(model)

    @staticmethod
    def _check_service(svc):
        def alive():
            if svc.error is not None:
                raise RuntimeError("parameter-server service thread failed") from svc.error
        return alive

    def wait_all_applied(self) -> None:
        """Collective: every push issued so far has been applied by its owner (end of ``join``)."""
        comm.barrier()
        for model in self.models:
            plan = getattr(model, "_ps_plan", None)
            if plan is None or plan.window is None:
                continue
            n = plan.mbox.tickets_issued(self.rank)
            if n:
                plan.mbox.wait_applied(self.rank, n, self._check_service(plan.service))
        comm.barrier()
        for model in self.models:
            if getattr(model, "_ps_plan", None) is not None and model._ps_plan.window is not None:
                self._pull(model)
                # the host step counter of the optimizer that pushed = the updates the owners applied
                # (every push goes to every owner: each owner's count is the job's step count)
                svc = model._ps_plan.service
                n_applied = comm.all_reduce_int([svc.step_offset + svc.applied], op=dist.ReduceOp.MAX)[0]
                for opt in {id(o): o for o in [model.optimizer, model._ps_plan.service.last_opt] if o}.values():
                    if opt is model._ps_plan.service.last_opt or opt.iterations:
                        opt.iterations = max(opt.iterations, n_applied)

    def shutdown(self) -> None:
        """Stop the owner threads and unmap the windows (collective)."""
        if not self._services:
            return
        comm.barrier()
        for model in self.models:
            plan = getattr(model, "_ps_plan", None)
            if plan is None or plan.window is None:
                continue
            plan.service.stop_flag = True
            plan.mbox.wake(self.rank, plan.service.applied)
        for svc in self._services:
            svc.join(timeout=10)
        comm.barrier()
        for model in self.models:
            plan = getattr(model, "_ps_plan", None)
            if plan is not None and plan.window is not None:
                plan.window.close()
                plan.window = None
                plan.mbox.close()
        self._services = []

    # ---- engine hooks -----------------------------------------------------------------------------
    def finish_gradients(self, model) -> None:
        pass  # the push happens in apply_update (after the whole backward)

    def apply_update(self, model, optimizer=None) -> None:
        if self.in_round():
            self._defer(model, optimizer)
            return
        opt = optimizer or model.optimizer
        if not comm.distributed():
            self._apply_local(model, opt)
        elif self.is_async:
            self._push_async(model, opt)
        else:
            self._push_apply_sync(model, opt, [True] * self.world_size)

    def commit_round(self, model, optimizer, contributed: list) -> None:
        opt = optimizer or model.optimizer
        if sum(bool(c) for c in contributed) == 0:
            self._pending = None
            return
        if not comm.distributed():
            self._apply_local(model, opt)
        else:
            self._push_apply_sync(model, opt, contributed)
        self._pending = None

    @staticmethod
    def _apply_local(model, opt) -> None:
        """One worker: the update is local.  After a GradientTape step whose gradients went straight
        to apply_gradients, the big Dense ranges update on an aux stream as soon as their dW is
        ready (nn/tape.py _apply_overlapped); otherwise one flat pass."""
        ready = getattr(model, "_tape_overlap", None)
        model._tape_overlap = None
        if ready:
            from ..nn.tape import _apply_overlapped

            _apply_overlapped(opt, model.store, ready, model)
        else:
            opt.apply(model.store)

    # ---- full-precision state (saving, checkpoints) -------------------------------------------------
    def _gather_full(self, model, src_local: torch.Tensor, src_window, dst: torch.Tensor) -> None:
        plan = model._ps_plan
        if plan.window is not None:
            plan.t_pull_all.copy([src_window(r) for r in range(self.world_size)], False, [dst], False, sys=True)
        else:
            xb = torch.empty(self.world_size * plan.seg, dtype=torch.float32, device=plan.device)
            comm.all_gather_flat(xb, src_local.contiguous())
            plan.t_pull_all.copy([xb], False, [dst], False)

    def synchronize_master(self, model) -> None:
        """Collective: the full fp32 values on every rank (after bf16 pulls only the fp32 pieces are)."""
        plan = getattr(model, "_ps_plan", None)
        st = model.store
        if plan is None or not comm.distributed() or not getattr(st, "master_stale", False):
            return
        if plan.window is not None:
            self.wait_all_applied()
        self._gather_full(model, plan.master, plan.window.vals if plan.window is not None else None, st.flat)
        st.refresh_bf16()
        st.master_stale = False

    def synchronize_state(self, model) -> None:
        """Collective: every owner's values AND optimizer moments unpacked into the full layout on
        every rank, so checkpoints are stored per parameter name."""
        plan = getattr(model, "_ps_plan", None)
        opt = model.optimizer
        if plan is None or not comm.distributed():
            return
        model.store.master_stale = True
        self.synchronize_master(model)
        if opt is None:
            return
        opt.build(model.store)
        for name, full in opt.state_tensors().items():
            if full is None or full.numel() != model.store.total:
                continue
            xb = torch.empty(self.world_size * plan.seg, dtype=torch.float32, device=plan.device)
            comm.all_gather_flat(xb, plan.slot(name))
            if plan.windows:
                plan.t_pull_all.copy(plan.segs(xb), False, [full], False)
            else:
                plan.t_pull_all.copy([xb], False, [full], False)

    def on_state_loaded(self, model) -> None:
        """After a checkpoint load into the full layout: re-pack the owned shards."""
        plan = getattr(model, "_ps_plan", None)
        if plan is None:
            return
        if plan.window is not None:
            self.wait_all_applied()
        plan.pack_params(model.store)
        opt = model.optimizer
        if opt is None:
            return
        if plan.window is not None:
            plan.service.step_offset = opt.iterations - plan.service.applied
        for name, full in opt.state_tensors().items():
            if full is not None and full.numel() == model.store.total:
                plan.t_own.copy([full], False, [plan.slot(name)], False)
        comm.barrier()
