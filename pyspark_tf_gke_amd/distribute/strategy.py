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
        (optimizer or model.optimizer).apply(model.store)

    def null_step(self, model, optimizer=None) -> None:
        """Take part in a step's collectives with a zero gradient (coordinator rounds)."""
        model.store.flat_grad.zero_()
        self.finish_gradients(model)
        self.apply_update(model, optimizer)


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

    def __init__(self, cluster_resolver=None, communication_options=None, bucket_mb: float | None = None,
                 device=None, sharded_update: bool | None = None):
        super().__init__(device)
        self.cluster_resolver = cluster_resolver or TFConfigClusterResolver()
        mb = bucket_mb if bucket_mb is not None else float(os.environ.get("PTG_BUCKET_MB", "64"))
        self.bucket_elems = max(1, int(mb * (1 << 20) / 4))
        if sharded_update is None:
            sharded_update = os.environ.get("PTG_SHARDED_UPDATE", "1") != "0"
        self.sharded_update = bool(sharded_update) and self.world_size > 1
        self._works: list = []
        self._launched = 0
        if self.world_size > 1 and self.device.type == "cuda" and os.environ.get("PTG_PERSIST_DYNAMIC") is None:
            # reduce-scatter / all-gather kernels run beside the backward: work-queue conv kernels
            from ..ops import nn as K

            K.set_persist_mode(True)

    def register_model(self, model) -> None:
        if self.sharded_update:
            model._shard_plan = _ShardPlan(model, self.world_size, self.rank, self.bucket_elems)
        super().register_model(model)

    # ---- replicated update: bucketed all-reduce
    def _launch(self, model, hi: int) -> None:
        g = model.store.flat_grad
        while self._launched < hi:
            end = min(hi, self._launched + 4 * self.bucket_elems)
            self._works.append(comm.all_reduce_(g[self._launched:end], async_op=True))
            self._launched = end

    # ---- sharded update
    def _rs(self, model, plan, b) -> None:
        st = model.store
        if b.gshard is None or b.gshard.device != st.flat_grad.device:
            b.gshard = torch.empty(b.shi - b.slo, dtype=torch.float32, device=st.flat_grad.device)
        plan.rs_works.append(comm.reduce_scatter_flat(b.gshard, st.flat_grad[b.lo:b.hi], async_op=True))
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
        if self.world_size == 1 or not op.params:
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
        if self.world_size == 1:
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
        opt = optimizer or model.optimizer
        plan = getattr(model, "_shard_plan", None)
        if plan is None:
            opt.apply(model.store, gscale=1.0 / self.world_size)
            return
        st = model.store
        self.wait_parameters(model)  # (no-op in steady state: the forward waited for every bucket)
        for b in plan.buckets:
            opt.apply_shard(st, b.gshard, b.slo, b.shi, gscale=1.0 / self.world_size, advance=False)
        opt.iterations += 1
        for b in plan.buckets:
            buf = st.flat if b.fp32 else st.flat_bf16
            src = buf[b.slo:b.shi].clone()  # out-of-place gather: the source never aliases the output
            plan.ag_works[b.idx] = (comm.all_gather_flat(buf[b.lo:b.hi], src, async_op=True), src)
        st.master_stale = any(not b.fp32 for b in plan.buckets)


MirroredStrategy = MultiWorkerMirroredStrategy


class ParameterServerStrategy(Strategy):
    """Synchronous sharded parameter server.  ``mode='sync'`` is the only mode: the reference's
    asynchronous PS has every worker apply updates to PS variables independently; on one xGMI node
    the sharded synchronous form moves the same bytes per step as collectives (reduce-scatter +
    all-gather of the flat buffer) without a central bottleneck."""

    def __init__(self, cluster_resolver=None, variable_partitioner=None, device=None):
        super().__init__(device)
        self.cluster_resolver = cluster_resolver or TFConfigClusterResolver()
        spec = self.cluster_resolver.cluster_spec() if hasattr(self.cluster_resolver, "cluster_spec") else ClusterSpec({})
        self.cluster_spec = ClusterSpec(spec)
        self.num_workers = max(self.cluster_spec.num_tasks("worker"), self.world_size)
        self.num_ps = self.cluster_spec.num_tasks("ps")
        self.variable_partitioner = variable_partitioner or MinSizePartitioner(256 << 10, max(self.num_ps, 1))
        self._gshard = None

    def shard_range(self, model) -> tuple[int, int]:
        total = model.store.total
        per = total // self.world_size
        return self.rank * per, (self.rank + 1) * per

    def register_model(self, model) -> None:
        st = model.store
        pad = 1024
        if st.total % pad:
            # pad the flat buffers so the byte range splits evenly over the PS shards
            new_total = int(math.ceil(st.total / pad) * pad)
            for name in ("flat", "flat_grad", "flat_bf16"):
                t = getattr(st, name)
                nt = torch.zeros(new_total, dtype=t.dtype, device=t.device)
                nt[: st.total] = t
                setattr(st, name, nt)
            st.total = new_total
            st._bind_views()
        super().register_model(model)

    def finish_gradients(self, model) -> None:
        if self.world_size == 1:
            return
        lo, hi = self.shard_range(model)
        if self._gshard is None or self._gshard.numel() != hi - lo or self._gshard.device != model.store.flat.device:
            self._gshard = torch.empty(hi - lo, dtype=torch.float32, device=model.store.flat.device)
        comm.reduce_scatter_flat(self._gshard, model.store.flat_grad)

    def apply_update(self, model, optimizer=None) -> None:
        opt = optimizer or model.optimizer
        st = model.store
        if self.world_size == 1:
            opt.apply(st)
            return
        from ..ops import nn as K

        lo, hi = self.shard_range(model)
        opt.apply_shard(st, self._gshard, lo, hi, 1.0 / self.world_size)
        comm.all_gather_flat(st.flat, st.flat[lo:hi].clone())
        K.cast_f32_bf16(st.flat, st.flat_bf16)

    def null_step(self, model, optimizer=None) -> None:
        """Participate in a step's collectives with zero gradient (ranks without a scheduled closure
        in the last round of ``ClusterCoordinator.join``)."""
        model.store.flat_grad.zero_()
        self.finish_gradients(model)
        self.apply_update(model, optimizer)
