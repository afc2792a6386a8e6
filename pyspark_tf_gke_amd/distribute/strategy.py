"""Distribution strategies over RCCL (one process per MI355X GPU).

* :class:`MultiWorkerMirroredStrategy` (BASELINE.json's ResNet-50 / scaling config):
  replicated parameters, gradients all-reduced in buckets that are launched *during* backward as
  soon as a contiguous prefix of the flat gradient buffer is complete (the flat store is laid out
  in backward-completion order), so the large Dense/last-layer gradients travel over xGMI while
  the convolution backward is still running.  Gradient averaging (1/world) is folded into the
  fused Adam kernel.
* :class:`ParameterServerStrategy` (the reference's strategy, train_tf_ps.py:440-511): variables
  are sharded across the GPUs that act as PS shards; each step reduce-scatters the flat gradient
  to the shard owners, every rank applies Adam to the shard it owns, and the updated parameters
  are all-gathered back ("pull" = all-gather, "push + apply" = reduce-scatter + sharded Adam; M1/M2
  of SURVEY §2.2.c).  Combined with :class:`~.coordinator.ClusterCoordinator` for the
  ``schedule()/join()`` driver API.
* :class:`OneDeviceStrategy` / :class:`MirroredStrategy` for single-process use.
"""
from __future__ import annotations

import contextlib
import math
import os

import torch

from ..parallel import comm
from .cluster import ClusterSpec, InputContext, MinSizePartitioner, TFConfigClusterResolver
from .. import config

_STACK: list = []


def current_strategy():
    return _STACK[-1] if _STACK else None


class Strategy:
    def __init__(self, device=None):
        self.rank, self.world_size = comm.init()
        _, local, _ = comm.env_rank()
        if device is not None:
            self.device = torch.device(device)
        elif torch.cuda.is_available():
            self.device = torch.device("cuda", local % max(torch.cuda.device_count(), 1))
            torch.cuda.set_device(self.device)
        else:
            self.device = torch.device("cpu")
        self.models: list = []
        self.optimizers: list = []
        self._in_round = False
        self._pending = None
        self._commit_scale = 1.0

    @property
    def num_replicas_in_sync(self) -> int:
        return self.world_size

    @property
    def is_chief(self) -> bool:
        return self.rank == 0

    @contextlib.contextmanager
    def scope(self):
        _STACK.append(self)
        try:
            yield self
        finally:
            _STACK.remove(self)

    def register_model(self, model) -> None:
        self.models.append(model)
        model.strategy = self
        if self.world_size > 1:
            comm.broadcast_(model.store.flat, 0)
            model.store.refresh_bf16()

    # ---- tf.distribute surface
    def run(self, fn, args=(), kwargs=None):
        return fn(*args, **(kwargs or {}))

    def input_context(self) -> InputContext:
        return InputContext(self.world_size, self.rank, self.world_size)

    def distribute_datasets_from_function(self, dataset_fn):
        return dataset_fn(self.input_context())

    def experimental_distribute_dataset(self, dataset):
        return dataset.shard(self.world_size, self.rank) if self.world_size > 1 else dataset

    def all_reduce_sum(self, t: torch.Tensor) -> torch.Tensor:
        if self.world_size == 1:
            return t
        dev_t = t.to(self.device) if comm.is_initialized() and torch.distributed.get_backend() == "nccl" else t.cpu()
        dev_t = dev_t.clone()
        comm.all_reduce_(dev_t)
        return dev_t.to(t.device)

    def reduce(self, reduce_op, value, axis=None):
        v = torch.as_tensor(value)
        s = self.all_reduce_sum(v.clone().float())
        if str(reduce_op).upper().endswith("MEAN"):
            s = s / self.world_size
        return s

    # ---- training hooks (called by the engine)
    def on_op_grads_ready(self, model, op) -> None:
        pass

    def finish_gradients(self, model) -> None:
        pass

    def apply_update(self, model, optimizer=None) -> None:
        if self.in_round():
            self._defer(model, optimizer)
            return
        (optimizer or model.optimizer).apply(model.store, gscale=self._commit_scale)

    # ---- ClusterCoordinator rounds (see coordinator.py): inside a round the gradient sync and the
    # update are deferred; after every rank ran (or failed, or had no) closure, the ranks agree on
    # who contributed and commit the round together, so every rank issues the same collectives.
    def begin_round(self) -> None:
        self._in_round = True
        self._pending = None

    def end_round_local(self) -> None:
        self._in_round = False

    def in_round(self) -> bool:
        return getattr(self, "_in_round", False)

    def _defer(self, model, optimizer) -> None:
        opt = optimizer or model.optimizer
        if getattr(self, "_pending", None) not in (None, (model, opt)):
            raise RuntimeError("a coordinator closure may update only one (model, optimizer) pair")
        self._pending = (model, opt)

    def pending_ids(self) -> tuple[int, int]:
        """(model index, optimizer index) of this rank's deferred update, or (-1, -1)."""
        pend = getattr(self, "_pending", None)
        if pend is None:
            return -1, -1
        model, opt = pend
        if opt not in self.optimizers:
            self.optimizers.append(opt)
        return self.models.index(model), self.optimizers.index(opt)

    def abort_round(self) -> None:
        pend = getattr(self, "_pending", None)
        if pend is not None:
            pend[0].store.flat_grad.zero_()
        self._pending = None

    def commit_round(self, model, optimizer, contributed: list) -> None:
        """Collective.  Apply one round: ``contributed[r]`` says whether rank r holds a gradient.
        Default (mirrored): average over the contributors; a rank without one pushes zeros; no
        update at all when nobody contributed (the optimizer does not advance)."""
        n_ok = sum(bool(c) for c in contributed)
        if not contributed[self.rank]:
            model.store.flat_grad.zero_()
        if n_ok == 0:
            return
        self._commit_scale = float(self.world_size) / n_ok
        try:
            self.finish_gradients(model)
            self.apply_update(model, optimizer)
        finally:
            self._commit_scale = 1.0
        self._pending = None


class OneDeviceStrategy(Strategy):
    def __init__(self, device=None):
        super().__init__(device)


class _Bucket:
    """One contiguous, world-divisible range of the flat buffers: reduce-scattered as soon as its
    gradients are complete, updated shard-wise, all-gathered before its parameters are next read."""

    __slots__ = ("idx", "lo", "hi", "fp32", "slo", "shi", "gshard", "nparams")

    def __init__(self, idx, lo, hi, fp32, world, rank):
        self.idx, self.lo, self.hi, self.fp32 = idx, lo, hi, fp32
        cnt = (hi - lo) // world
        self.slo, self.shi = lo + rank * cnt, lo + (rank + 1) * cnt
        self.gshard = None
        self.nparams = 0


class _ShardPlan:
    """Per-model state of the sharded data-parallel update (ZeRO-1 style).

    The flat store is re-laid out as [weights read as bf16 in forward][everything else], each part
    in backward-completion order, grouped into buckets (closed at ``bucket_elems`` or after any
    weight of >= ``BIG`` elements), every bucket padded to ``world * 64`` elements and split
    further when larger than ``bucket_elems``.  Rank r owns slice r of every bucket: it keeps the optimizer moments and
    the fp32 master for that slice current, the rest of its fp32 copy of a bf16-group bucket goes
    stale between :meth:`MultiWorkerMirroredStrategy.synchronize_master` calls (``store.master_stale``)."""

    BIG = 4 << 20  # elements

    def __init__(self, model, world, rank, bucket_elems):
        from ..nn.params import ALIGN

        st = model.store
        ps = sorted(st.params, key=lambda p: p.offset)  # backward-completion order
        groups = []
        for fp32 in (False, True):
            cur, size = [], 0
            for p in ps:
                if p.fwd_bf16 == fp32:
                    continue
                if cur and size >= bucket_elems:
                    groups.append((cur, fp32))
                    cur, size = [], 0
                cur.append(p)
                size += p.numel
                if p.numel >= self.BIG:
                    # a large weight closes its bucket: its reduce-scatter starts as soon as its own
                    # gradient exists instead of waiting for the (later) gradients of the layers below
                    groups.append((cur, fp32))
                    cur, size = [], 0
            if cur:
                groups.append((cur, fp32))
        q = world * ALIGN
        ranges = st.relayout([g for g, _ in groups], q)
        self.buckets: list[_Bucket] = []
        for (lo, hi), (_, fp32) in zip(ranges, groups):
            n = hi - lo
            nb = max(1, math.ceil(n / max(bucket_elems, q)))
            step = math.ceil(n / nb / q) * q
            b = lo
            while b < hi:
                e = min(hi, b + step)
                self.buckets.append(_Bucket(len(self.buckets), b, e, fp32, world, rank))
                b = e
        self.param_buckets: dict[int, list[_Bucket]] = {}
        for p in st.params:
            lo, hi = p.offset, p.offset + p.numel
            bs = [b for b in self.buckets if b.lo < hi and lo < b.hi]
            self.param_buckets[id(p)] = bs
            for b in bs:
                b.nparams += 1
        self.pending = [b.nparams for b in self.buckets]
        self.launched = [False] * len(self.buckets)
        self.rs_works: list = []
        self.ag_works: dict[int, tuple] = {}
        st.master_stale = False


class MultiWorkerMirroredStrategy(Strategy):
    """Synchronous data parallelism over RCCL.

    ``sharded_update`` (default on for more than one rank; ``PTG_SHARDED_UPDATE=0`` turns it off)
    replaces the gradient all-reduce + replicated optimizer by reduce-scatter + sharded optimizer +
    all-gather: each bucket's gradient is reduce-scattered during backward as soon as it completes,
    each rank runs Adam/SGD on its 1/world slice only (the optimizer pass is HBM-bound: 30 B per
    parameter for Adam), and the updated slices are all-gathered asynchronously — in bf16 for the
    matmul/conv weights — and waited for only right before the forward op that reads them, so the
    large Dense weight's gather overlaps the next step's convolution forward.  Per step and GPU
    this moves (w-1)/w * (4 + 2) bytes per bf16-forward parameter instead of the all-reduce's
    (w-1)/w * 8 over xGMI.  Without it: bucketed fp32 all-reduce launched during backward."""

    side_stream_ok = True  # gradient collectives go through streams.launch (see _rs / _launch)

    def __init__(self, cluster_resolver=None, communication_options=None, bucket_mb: float | None = None,
                 device=None, sharded_update: bool | None = None):
        super().__init__(device)
        self.cluster_resolver = cluster_resolver or TFConfigClusterResolver()
        mb = bucket_mb if bucket_mb is not None else float(config.get("bucket_mb"))
        self.bucket_elems = max(1, int(mb * (1 << 20) / 4))
        if sharded_update is None:
            sharded_update = config.get("sharded_update")
        self.sharded_update = bool(sharded_update) and self.world_size > 1
        self._works: list = []
        self._launched = 0
        if self.world_size > 1 and self.device.type == "cuda" and config.get("persist_dynamic"):
            # opt-in: work-queue conv kernels (absorb CUs taken by the concurrent RCCL kernels).  The
            # default stays the static-grid kernels, the faster ones in the only A/B measured so far
            # (1 GPU, 119.5k vs 114.3k samples/s, README); re-measure on 8 GPUs before flipping it.
            from ..ops import nn as K

            K.set_persist_mode(True)

    def register_model(self, model) -> None:
        if self.sharded_update:
            model._shard_plan = _ShardPlan(model, self.world_size, self.rank, self.bucket_elems)
        super().register_model(model)

    # ---- replicated update: bucketed all-reduce
    def _launch(self, model, hi: int) -> None:
        from ..nn import streams as S

        g = model.store.flat_grad
        while self._launched < hi:
            end = min(hi, self._launched + 4 * self.bucket_elems)
            seg = g[self._launched:end]
            self._works.append(S.launch(lambda: comm.all_reduce_(seg, async_op=True), seg.device))
            self._launched = end

    # ---- sharded update
    def _rs(self, model, plan, b) -> None:
        st = model.store
        if b.gshard is None or b.gshard.device != st.flat_grad.device:
            b.gshard = torch.empty(b.shi - b.slo, dtype=torch.float32, device=st.flat_grad.device)
        # through the step's side stream (nn/streams.py): after this bucket's side-stream wgrads and
        # everything the compute stream queued so far, without making the compute stream wait
        from ..nn import streams as S

        g = st.flat_grad[b.lo:b.hi]
        plan.rs_works.append(S.launch(lambda: comm.reduce_scatter_flat(b.gshard, g, async_op=True), g.device))
        plan.launched[b.idx] = True

    def _wait_gather(self, model, plan, b) -> None:
        ent = plan.ag_works.pop(b.idx, None)
        if ent is None:
            return
        work, _src = ent
        if work is not None:
            work.wait()
        if b.fp32:
            from ..ops import nn as K

            st = model.store
            K.cast_f32_bf16(st.flat[b.lo:b.hi], st.flat_bf16[b.lo:b.hi])

    def before_forward_op(self, model, op) -> None:
        plan = getattr(model, "_shard_plan", None)
        if plan is None or not plan.ag_works:
            return
        for p in op.params:
            for b in plan.param_buckets.get(id(p), ()):
                self._wait_gather(model, plan, b)

    def wait_parameters(self, model) -> None:
        """Block the compute stream on every outstanding parameter all-gather."""
        plan = getattr(model, "_shard_plan", None)
        if plan is None:
            return
        for b in plan.buckets:
            self._wait_gather(model, plan, b)

    def synchronize_master(self, model) -> None:
        """Collective (every rank calls it): make the full fp32 master copy current on every rank
        (after sharded updates only each rank's own slices of the bf16-forward weights are)."""
        plan = getattr(model, "_shard_plan", None)
        st = model.store
        if plan is None or not getattr(st, "master_stale", False):
            return
        self.wait_parameters(model)
        for b in plan.buckets:
            if not b.fp32:
                comm.all_gather_flat(st.flat[b.lo:b.hi], st.flat[b.slo:b.shi].clone())
        st.master_stale = False

    def synchronize_state(self, model) -> None:
        """Collective: full fp32 master AND optimizer moments on every rank (checkpointing)."""
        plan = getattr(model, "_shard_plan", None)
        if plan is None:
            return
        self.synchronize_master(model)
        opt = model.optimizer
        if opt is None:
            return
        for t in opt.state_tensors().values():
            if t is None or t.numel() != model.store.total:
                continue
            for b in plan.buckets:
                comm.all_gather_flat(t[b.lo:b.hi], t[b.slo:b.shi].clone())

    # ---- engine hooks
    def on_op_grads_ready(self, model, op) -> None:
        if self.world_size == 1 or not op.params or self.in_round():
            return
        plan = getattr(model, "_shard_plan", None)
        if plan is not None:
            for p in op.params:
                for b in plan.param_buckets.get(id(p), ()):
                    plan.pending[b.idx] -= 1
            # launch in bucket order only (every rank must issue the same collective sequence)
            for b in plan.buckets:
                if plan.launched[b.idx]:
                    continue
                if plan.pending[b.idx] > 0:
                    break
                self._rs(model, plan, b)
            return
        hi = max(p.offset + p.numel for p in op.params)
        if hi - self._launched >= self.bucket_elems:
            self._launch(model, hi)

    def finish_gradients(self, model) -> None:
        if self.world_size == 1 or self.in_round():
            return
        plan = getattr(model, "_shard_plan", None)
        if plan is not None:
            for b in plan.buckets:
                if not plan.launched[b.idx]:
                    self._rs(model, plan, b)
            for w in plan.rs_works:
                if w is not None:
                    w.wait()
            plan.rs_works.clear()
            plan.pending = [b.nparams for b in plan.buckets]
            plan.launched = [False] * len(plan.buckets)
            return
        self._launch(model, model.store.total)
        for w in self._works:
            if w is not None:
                w.wait()
        self._works.clear()
        self._launched = 0

    def apply_update(self, model, optimizer=None) -> None:
        if self.in_round():
            self._defer(model, optimizer)
            return
        opt = optimizer or model.optimizer
        plan = getattr(model, "_shard_plan", None)
        gs = self._commit_scale / self.world_size
        if plan is None:
            opt.apply(model.store, gscale=gs)
            return
        st = model.store
        self.wait_parameters(model)  # (no-op in steady state: the forward waited for every bucket)
        for b in plan.buckets:
            opt.apply_shard(st, b.gshard, b.slo, b.shi, gscale=gs, advance=False)
        opt.iterations += 1
        for b in plan.buckets:
            buf = st.flat if b.fp32 else st.flat_bf16
            src = buf[b.slo:b.shi].clone()  # out-of-place gather: the source never aliases the output
            plan.ag_works[b.idx] = (comm.all_gather_flat(buf[b.lo:b.hi], src, async_op=True), src)
        st.master_stale = any(not b.fp32 for b in plan.buckets)


MirroredStrategy = MultiWorkerMirroredStrategy


class _Piece:
    __slots__ = ("param", "lo", "n", "owner", "xlo", "task")

    def __init__(self, param, lo, n, owner, task):
        self.param, self.lo, self.n, self.owner, self.task = param, lo, n, owner, task
        self.xlo = -1


class _PSPlan:
    """Variable placement of one model: every parameter is cut by the partitioner along axis 0
    (whole rows per shard, TF's MinSizePartitioner rule) and shard i of the running count goes to
    PS task ``i % num_ps`` (TF's round-robin variable placement); PS task t lives on rank
    ``t % world``.  An owner's shards are packed into its segment of an exchange buffer of
    ``world * seg`` elements, so "push" is ONE reduce-scatter (sync) or one send per owner (async)
    and "pull" is ONE all-gather, whatever the placement.  The owner keeps its shards' fp32 values
    and optimizer moments in packed form: the variables live on the PS."""

    def __init__(self, model, partitioner, num_ps: int, world: int, rank: int):
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
                self.pieces.append(_Piece(p, p.offset + r0 * row_elems, nr * row_elems, t % world, t))
                r0 += nr
                task += 1
        per_owner = [0] * world
        for pc in self.pieces:
            pc.xlo = per_owner[pc.owner]
            per_owner[pc.owner] += pc.n
        self.owner_elems = per_owner
        self.seg = max(ALIGN, int(math.ceil(max(per_owner) / ALIGN) * ALIGN))
        for pc in self.pieces:
            pc.xlo += pc.owner * self.seg
        self.world, self.rank = world, rank
        self.mine = [pc for pc in self.pieces if pc.owner == rank]
        dev = st.flat.device
        self.xbuf = torch.zeros(world * self.seg, dtype=torch.float32, device=dev)  # exchange buffer
        self.gshard = torch.zeros(self.seg, dtype=torch.float32, device=dev)
        self.master = torch.zeros(self.seg, dtype=torch.float32, device=dev)  # owned values
        self.master_bf = torch.zeros(self.seg, dtype=st.flat_bf16.dtype, device=dev)
        self.slots: dict[str, torch.Tensor] = {}  # packed optimizer moments of the owned shards
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

    def pack(self, src: torch.Tensor, dst: torch.Tensor, only_mine: bool = False) -> None:
        for pc in (self.mine if only_mine else self.pieces):
            x0 = pc.xlo - (self.rank * self.seg if only_mine else 0)
            dst[x0:x0 + pc.n].copy_(src[pc.lo:pc.lo + pc.n])

    def unpack(self, src: torch.Tensor, dst: torch.Tensor) -> None:
        for pc in self.pieces:
            dst[pc.lo:pc.lo + pc.n].copy_(src[pc.xlo:pc.xlo + pc.n])

    def pack_params(self, st) -> None:
        self.pack(st.flat, self.master, only_mine=True)

    def slot(self, name: str) -> torch.Tensor:
        t = self.slots.get(name)
        if t is None:
            t = self.slots[name] = torch.zeros(self.seg, dtype=torch.float32, device=self.master.device)
        return t


class ParameterServerStrategy(Strategy):
    """The reference's strategy (train_tf_ps.py:440-511) on GPU ranks: every rank is a worker and
    hosts PS tasks.  Variables are placed per shard by ``variable_partitioner`` (default
    ``MinSizePartitioner(256 KiB, max_shards=#ps)``, :505-507) round-robin over the PS tasks; PS
    task t lives on rank ``t % world`` (``num_ps`` from the cluster spec, or one per rank).

    ``mode="sync"`` (default): a step pushes gradients with one reduce-scatter of the packed
    exchange buffer (owners receive the sum), owners apply the optimizer to the shards they host
    with the gradient averaged over the workers that contributed, and every worker pulls the new
    values with one all-gather (M1/M2 of SURVEY §2.2.c).

    ``mode="async"`` (TF's asynchronous PS semantics): each worker's gradient is sent point-to-point
    to the owner of every shard (``batch_isend_irecv``; RCCL runs it on its own stream) and the
    owner applies it as its own optimizer step, in worker order, without averaging; workers pull the
    values after all pushes of the round were applied, so a worker's gradient is up to
    ``workers - 1`` updates stale, as under TF's asynchronous PS with that many concurrent workers.

    Under :class:`~.coordinator.ClusterCoordinator` the push/apply is committed per round after the
    ranks agree who contributed: no zero-gradient pushes, no optimizer step when nobody did."""

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

    def register_model(self, model) -> None:
        super().register_model(model)  # broadcast rank 0's initial values first
        model._ps_plan = _PSPlan(model, self.variable_partitioner, self.num_ps, self.world_size, self.rank)

    def placement(self, model) -> list:
        return model._ps_plan.placement()

    # ---- optimizer on the owned (packed) shards
    def _apply_owned(self, model, opt, grad: torch.Tensor, gscale: float) -> None:
        from ..nn import optimizers as OPT
        from ..ops import nn as K

        plan = model._ps_plan
        n = plan.seg
        if isinstance(opt, OPT.Adam):
            step = opt.iterations + 1
            K.adam(plan.master[:n], grad[:n], plan.slot("m"), plan.slot("v"), plan.master_bf[:n], opt.lr_t(step),
                   opt.beta_1, opt.beta_2, opt.epsilon, gscale)
        elif isinstance(opt, OPT.SGD):
            vel = plan.slot("velocity") if opt.momentum > 0 else None
            K.sgd(plan.master[:n], grad[:n], vel, plan.master_bf[:n], opt.learning_rate, opt.momentum, opt.nesterov,
                  gscale)
        else:
            raise TypeError(f"unsupported optimizer {type(opt).__name__}")
        opt.iterations += 1

    def _pull(self, model) -> None:
        from ..ops import nn as K

        plan = model._ps_plan
        st = model.store
        comm.all_gather_flat(plan.xbuf, plan.master)
        plan.unpack(plan.xbuf, st.flat)
        K.cast_f32_bf16(st.flat, st.flat_bf16)

    def _push_apply(self, model, opt, contributed: list) -> None:
        plan = model._ps_plan
        st = model.store
        n_ok = sum(bool(c) for c in contributed)
        if n_ok == 0:
            return
        if self.world_size == 1:
            opt.apply(st)
            return
        if self.mode == "sync":
            if contributed[self.rank]:
                plan.pack(st.flat_grad, plan.xbuf)
            else:
                plan.xbuf.zero_()
            comm.reduce_scatter_flat(plan.gshard, plan.xbuf)
            self._apply_owned(model, opt, plan.gshard, 1.0 / n_ok)
        else:
            import torch.distributed as dist

            if contributed[self.rank]:
                plan.pack(st.flat_grad, plan.xbuf)
            ops, recv = [], {}
            for w in range(self.world_size):
                if w == self.rank or not contributed[w]:
                    continue
                recv[w] = torch.empty(plan.seg, dtype=torch.float32, device=plan.xbuf.device)
                ops.append(dist.P2POp(dist.irecv, recv[w], w))
            if contributed[self.rank]:
                for r in range(self.world_size):
                    if r != self.rank:
                        ops.append(dist.P2POp(dist.isend, plan.xbuf[r * plan.seg:(r + 1) * plan.seg], r))
            if ops:
                for req in dist.batch_isend_irecv(ops):
                    req.wait()
            for w in range(self.world_size):  # apply each worker's push as its own step, in order
                if not contributed[w]:
                    continue
                g = plan.xbuf[self.rank * plan.seg:(self.rank + 1) * plan.seg] if w == self.rank else recv[w]
                self._apply_owned(model, opt, g, 1.0)
        self._pull(model)

    # ---- engine hooks
    def finish_gradients(self, model) -> None:
        pass  # the push happens in apply_update (after the whole backward)

    def apply_update(self, model, optimizer=None) -> None:
        if self.in_round():
            self._defer(model, optimizer)
            return
        self._push_apply(model, optimizer or model.optimizer, [True] * self.world_size)

    def commit_round(self, model, optimizer, contributed: list) -> None:
        self._push_apply(model, optimizer or model.optimizer, contributed)
        self._pending = None

    # ---- checkpoint support: the canonical optimizer state is per parameter (full layout)
    def synchronize_state(self, model) -> None:
        """Collective: unpack every owner's moments into the optimizer's full-layout slots (and the
        values into the store) on every rank, so checkpoints are stored per parameter name."""
        plan = getattr(model, "_ps_plan", None)
        opt = model.optimizer
        if plan is None or self.world_size == 1:
            return
        self._pull(model)
        if opt is None:
            return
        opt.build(model.store)
        for name, full in opt.state_tensors().items():
            if full is None or full.numel() != model.store.total:
                continue
            comm.all_gather_flat(plan.xbuf, plan.slot(name))
            plan.unpack(plan.xbuf, full)

    def on_state_loaded(self, model) -> None:
        """After a checkpoint load into the full layout: re-pack the owned shards."""
        plan = getattr(model, "_ps_plan", None)
        if plan is None:
            return
        plan.pack_params(model.store)
        opt = model.optimizer
        if opt is None:
            return
        for name, full in opt.state_tensors().items():
            if full is not None and full.numel() == model.store.total:
                plan.pack(full, plan.slot(name), only_mine=True)
