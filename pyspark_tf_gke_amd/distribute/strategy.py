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


class MultiWorkerMirroredStrategy(Strategy):
    def __init__(self, cluster_resolver=None, communication_options=None, bucket_mb: float | None = None,
                 device=None):
        super().__init__(device)
        self.cluster_resolver = cluster_resolver or TFConfigClusterResolver()
        mb = bucket_mb if bucket_mb is not None else float(os.environ.get("PTG_BUCKET_MB", "64"))
        self.bucket_elems = max(1, int(mb * (1 << 20) / 4))
        self._works: list = []
        self._launched = 0

    def _launch(self, model, hi: int) -> None:
        g = model.store.flat_grad
        while self._launched < hi:
            end = min(hi, self._launched + 4 * self.bucket_elems)
            self._works.append(comm.all_reduce_(g[self._launched:end], async_op=True))
            self._launched = end

    def on_op_grads_ready(self, model, op) -> None:
        if self.world_size == 1 or not op.params:
            return
        hi = max(p.offset + p.numel for p in op.params)
        if hi - self._launched >= self.bucket_elems:
            self._launch(model, hi)

    def finish_gradients(self, model) -> None:
        if self.world_size == 1:
            return
        self._launch(model, model.store.total)
        for w in self._works:
            if w is not None:
                w.wait()
        self._works.clear()
        self._launched = 0

    def apply_update(self, model, optimizer=None) -> None:
        (optimizer or model.optimizer).apply(model.store, gscale=1.0 / self.world_size)


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
