"""Distribution strategies over RCCL (one process per MI355X GPU).

* :class:`MultiWorkerMirroredStrategy` (BASELINE.json's ResNet-50 / scaling config):
  replicated parameters, gradients all-reduced in buckets that are launched *during* backward as
  soon as a contiguous prefix of the flat gradient buffer is complete (the flat store is laid out
  in backward-completion order), so the large Dense/last-layer gradients travel over xGMI while
  the convolution backward is still running.  Gradient averaging (1/world) is folded into the
  fused Adam kernel.
* :class:`~.ps.ParameterServerStrategy` (the reference's strategy, train_tf_ps.py:440-511), in
  ps.py: variables sharded over the ranks acting as PS tasks, sync (collective push/pull) or async
  (one-sided windows + owner service threads) - with :class:`~.coordinator.ClusterCoordinator` for
  the ``schedule()/join()`` driver API.
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
            self.device = torch.device("cuda", comm.device_index())
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
    def dp_degree(self) -> int:
        """Data-parallel degree the step's kernel sequence is built for (the world size, or the
        simulated world of MultiWorkerMirroredStrategy's PTG_SIM_WORLD mode on one rank)."""
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
        if comm.distributed():
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
        if not comm.distributed():
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

    def begin_round_retry(self) -> None:
        """A failed closure runs again inside the same round (its rank's pending update was aborted)."""
        self._in_round = True
        self._pending = None

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
        """Discard this rank's gradients of the round (a failed closure may have stopped anywhere in
        its backward, before or after its deferred update was recorded)."""
        pend = getattr(self, "_pending", None)
        models = list(self.models) + ([pend[0]] if pend is not None and pend[0] not in self.models else [])
        for m in models:
            m._lazy_dw = None  # deferred tape weight gradients of the aborted attempt (nn/tape.py)
            m._tape_overlap = None
            if hasattr(m, "_drop_pending_head"):
                m._drop_pending_head()  # a closure that failed between its forward and its loss
            m.store.flat_grad.zero_()
            m.store.grad_clean = True
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
        # simulated world (PTG_SIM_WORLD=N on ONE rank): build the shard plan of an N-rank job and run
        # rank 0's exact kernel sequence of the sharded update - weight gradients into flat_grad, per-
        # bucket reduce-scatter, shard optimizer, all-gather + bf16 re-cast - with each collective
        # replaced by a local kernel moving the same local HBM bytes (ops.nn.sim_reduce_scatter /
        # sim_all_gather).  The peers are N-1 ranks with identical data: the reduced shard is N x ours.
        # PTG_SIM_EXACT=1 also applies the peers' shard updates, so parameters equal a real N-rank run
        # with identical per-rank batches (at N x the optimizer work); without it the peers' chunks keep
        # their values (cost model only).
        self.sim_world = 0
        self.sim_exact = False
        if self.world_size == 1 and int(config.get("sim_world")) > 1:
            self.sim_world = int(config.get("sim_world"))
            self.sim_exact = bool(config.get("sim_exact"))
        if sharded_update is None:
            sharded_update = config.get("sharded_update")
        # PTG_SHARD_WORLD1 (with PTG_FORCE_PG): a 1-rank process group still takes the sharded path, so
        # the RCCL reduce-scatter / all-gather calls of an N-rank step run for real on one GPU
        force1 = self.world_size == 1 and not self.sim_world and comm.is_initialized() and bool(
            config.get("shard_world1"))
        self.sharded_update = bool(sharded_update) and (self.dp_degree > 1 or force1)
        if self.sim_world and not self.sharded_update:
            raise ValueError("PTG_SIM_WORLD simulates the sharded update only (PTG_SHARDED_UPDATE=1)")
        self._works: list = []
        self._launched = 0
        if self.world_size > 1 and self.device.type == "cuda" and config.get("persist_dynamic"):
            # opt-in: work-queue conv kernels (absorb CUs taken by the concurrent RCCL kernels).  The
            # default stays the static-grid kernels, the faster ones in the only A/B measured so far
            # (1 GPU, 119.5k vs 114.3k samples/s, README); re-measure on 8 GPUs before flipping it.
            from ..ops import nn as K

            K.set_persist_mode(True)

    @property
    def dp_degree(self) -> int:
        return self.sim_world or self.world_size

    def register_model(self, model) -> None:
        if self.sharded_update:
            model._shard_plan = _ShardPlan(model, self.dp_degree, self.rank, self.bucket_elems)
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
        if self.sim_world:
            from ..ops import nn as K

            n = self.sim_world
            S.launch(lambda: K.sim_reduce_scatter(g, b.gshard, n, float(n), 0.0), g.device)
        else:
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
        if self.sim_world:  # no peers to gather from (exact mode keeps every chunk's master current)
            st.master_stale = False
            return
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
        if opt is None or self.sim_world:
            return
        for t in opt.state_tensors().values():
            if t is None or t.numel() != model.store.total:
                continue
            for b in plan.buckets:
                comm.all_gather_flat(t[b.lo:b.hi], t[b.slo:b.shi].clone())

    # ---- engine hooks
    def on_op_grads_ready(self, model, op) -> None:
        if (self.dp_degree == 1 and not self.sharded_update) or not op.params or self.in_round():
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
        if (self.dp_degree == 1 and not self.sharded_update) or self.in_round():
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
        gs = self._commit_scale / self.dp_degree
        if plan is None:
            opt.apply(model.store, gscale=gs)
            return
        st = model.store
        self.wait_parameters(model)  # (no-op in steady state: the forward waited for every bucket)
        for b in plan.buckets:
            opt.apply_shard(st, b.gshard, b.slo, b.shi, gscale=gs, advance=False)
        if self.sim_world:
            self._sim_peers_update(model, plan, opt, gs)
            opt.iterations += 1
            return
        opt.iterations += 1
        for b in plan.buckets:
            buf = st.flat if b.fp32 else st.flat_bf16
            src = buf[b.slo:b.shi].clone()  # out-of-place gather: the source never aliases the output
            plan.ag_works[b.idx] = (comm.all_gather_flat(buf[b.lo:b.hi], src, async_op=True), src)
        st.master_stale = any(not b.fp32 for b in plan.buckets)

    def _sim_peers_update(self, model, plan, opt, gs) -> None:
        """Simulated world: the all-gather of every bucket.  Exact mode computes what each identical
        peer applied to its own chunk (N x our gradient chunk, the same optimizer step); otherwise the
        peers' chunks are rewritten in place (the bytes the gather writes, values unchanged).  fp32
        buckets are re-cast to bf16 before their forward use, as after a real gather."""
        from ..ops import nn as K

        st = model.store
        n = self.sim_world
        for b in plan.buckets:
            cnt = b.shi - b.slo
            if self.sim_exact:
                for r in range(1, n):
                    lo = b.lo + r * cnt
                    tmp = torch.empty(cnt, dtype=torch.float32, device=st.flat_grad.device)
                    K.sim_reduce_scatter(st.flat_grad[lo:lo + cnt], tmp, 1, float(n), 0.0)
                    opt.apply_shard(st, tmp, lo, lo + cnt, gscale=gs, advance=False)
            else:
                buf = st.flat if b.fp32 else st.flat_bf16
                K.sim_all_gather(buf[b.lo:b.hi], cnt)
            plan.ag_works[b.idx] = (None, None)
        st.master_stale = False


MirroredStrategy = MultiWorkerMirroredStrategy


def __getattr__(name):  # ParameterServerStrategy lives in ps.py (it builds on Strategy above)
    if name == "ParameterServerStrategy":
        from .ps import ParameterServerStrategy

        return ParameterServerStrategy
    raise AttributeError(name)
