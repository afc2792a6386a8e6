"""``ClusterCoordinator``: the reference's schedule/join driver (train_tf_ps.py:612-614, :634-647,
:734-736, :755-769) on SPMD ranks.

Every rank runs the same driver script.  ``schedule(fn, args)`` queues a closure and returns a
:class:`RemoteValue`; ``join()`` executes the queue in rounds of ``world_size`` closures, closure i
running on rank ``i % world`` (so ``steps_per_epoch`` scheduled steps are spread over the workers,
each worker consuming its own per-worker dataset iterator).  Inside a closure,
``strategy.run(step_fn, ...)`` executes locally and ``optimizer.apply_gradients`` performs the
PS strategy's reduce-scatter / sharded Adam / all-gather — so every round is one synchronous
collective step.  A rank without a closure in the last round takes a zero-gradient step so the
collectives stay matched.  ``join()`` is the epoch barrier of the reference.

Fault handling: a closure that raises is re-queued (retried) up to ``max_retries`` times on the
next round, mirroring TF's coordinator re-scheduling of failed closures.
"""
from __future__ import annotations

from ..parallel import comm


class RemoteValue:
    def __init__(self):
        self._value = None
        self._done = False
        self._error = None
        self._local = False

    def _set(self, v, local=True):
        self._value, self._done, self._local = v, True, local

    def fetch(self):
        if self._error is not None:
            raise self._error
        return self._value

    def get(self):
        return self.fetch()


class PerWorkerIterator:
    def __init__(self, it):
        self._it = it

    def __next__(self):
        return next(self._it)

    def __iter__(self):
        return self


class PerWorkerDataset:
    def __init__(self, ds):
        self._ds = ds

    def __iter__(self):
        return PerWorkerIterator(iter(self._ds))


class ClusterCoordinator:
    def __init__(self, strategy, max_retries: int = 2):
        self.strategy = strategy
        self._queue: list = []
        self.max_retries = max_retries
        self.closures_run = 0

    def create_per_worker_dataset(self, dataset_fn):
        ctx = self.strategy.input_context()
        ds = dataset_fn(ctx) if callable(dataset_fn) else dataset_fn
        return PerWorkerDataset(ds)

    def schedule(self, fn, args=(), kwargs=None) -> RemoteValue:
        rv = RemoteValue()
        self._queue.append((fn, tuple(args), dict(kwargs or {}), rv, 0))
        return rv

    def join(self) -> None:
        world, rank = self.strategy.world_size, self.strategy.rank
        while self._queue:
            batch, self._queue = self._queue[:world], self._queue[world:]
            mine = batch[rank] if rank < len(batch) else None
            if mine is not None:
                fn, args, kwargs, rv, tries = mine
                try:
                    rv._set(fn(*args, **kwargs))
                    self.closures_run += 1
                except StopIteration as e:
                    rv._error = e
                    for m in self.strategy.models:
                        self.strategy.null_step(m)
                except Exception as e:  # noqa: BLE001 - retry like TF's coordinator
                    if tries < self.max_retries:
                        self._queue.append((fn, args, kwargs, rv, tries + 1))
                    else:
                        rv._error = e
                    for m in self.strategy.models:
                        self.strategy.null_step(m)
            else:
                for m in self.strategy.models:
                    self.strategy.null_step(m)
            for rv_ in (b[3] for b in batch):
                if not rv_._done and rv_._error is None:
                    rv_._done = True  # executed on another rank
        comm.barrier()

    def done(self) -> bool:
        return not self._queue

    def fetch(self, values):
        if isinstance(values, (list, tuple)):
            return [v.fetch() for v in values]
        return values.fetch()
