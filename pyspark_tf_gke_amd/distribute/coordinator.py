"""``ClusterCoordinator``: the reference's schedule/join driver (train_tf_ps.py:612-614, :634-647,
:734-736, :755-769) on SPMD ranks.

Every rank runs the same driver script.  ``schedule(fn, args)`` queues a closure and returns a
:class:`RemoteValue`; ``join()`` executes the queue in rounds of ``world_size`` closures, closure i
of a round running on rank ``i % world`` (so ``steps_per_epoch`` scheduled steps are spread over the
workers, each worker consuming its own per-worker dataset iterator).  ``join()`` is the epoch
barrier of the reference.

A round is a transaction:
  1. every rank runs its closure (if any) with the strategy in *deferred* mode: gradient pushes and
     optimizer updates inside the closure (``optimizer.apply_gradients``, ``model.train_step``) are
     recorded, not executed, so a closure that raises leaves no collective half-issued;
  2. the ranks exchange one small status tensor (all-reduce, no pickles): per rank ok / no closure /
     failed, plus which (model, optimizer) the update belongs to;
  3. if some closure failed and may be retried, EVERY rank discards the round's gradients and the
     whole round is queued again with the same closure-to-rank assignment (TF's coordinator
     re-schedules failed closures; re-running the round keeps every rank's step sequence
     identical, and a deterministic closure reproduces the fault-free result bit for bit);
     a closure that exhausted ``max_retries`` is dropped with its error recorded on every rank;
  4. otherwise the round is committed collectively: the strategy pushes the contributors'
     gradients (ranks without a closure push nothing and the average is over the contributors;
     nobody contributing means no optimizer step).

Closures must not call collectives themselves (every rank would have to reach them).
"""
from __future__ import annotations

from ..parallel import comm


def _encode_value(v) -> tuple[int, float]:
    """Scalar closure results (Python numbers, one-element tensors) are shared with every rank."""
    import torch

    if isinstance(v, bool):
        return 4, float(v)
    if isinstance(v, int):
        return 1, float(v)
    if isinstance(v, float):
        return 2, v
    if isinstance(v, torch.Tensor) and v.numel() == 1:
        return 3, float(v.detach().double().cpu().item())
    return 0, 0.0


def _decode_value(vtype: int, x: float):
    import torch

    return {0: None, 1: int(round(x)), 2: x, 3: torch.tensor(x), 4: bool(x)}.get(vtype)


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
        self.retries = 0

    def create_per_worker_dataset(self, dataset_fn):
        ctx = self.strategy.input_context()
        ds = dataset_fn(ctx) if callable(dataset_fn) else dataset_fn
        return PerWorkerDataset(ds)

    def schedule(self, fn, args=(), kwargs=None) -> RemoteValue:
        rv = RemoteValue()
        self._queue.append((fn, tuple(args), dict(kwargs or {}), rv, 0))
        return rv

    def join(self) -> None:
        import torch

        from ..runtime import heartbeat

        st = self.strategy
        world, rank = st.world_size, st.rank
        while self._queue:
            batch = self._queue[:world]
            rest = self._queue[world:]
            mine = batch[rank] if rank < len(batch) else None
            status, err = 0, None  # 0 = no closure / StopIteration, 1 = gradient pending, 2 = failed
            st.begin_round()
            try:
                if mine is not None:
                    fn, args, kwargs, rv, tries = mine
                    try:
                        value = fn(*args, **kwargs)
                        status = 1
                    except StopIteration as e:
                        err = e
                    except Exception as e:  # noqa: BLE001 - reported to every rank below
                        status, err = 2, e
            finally:
                st.end_round_local()
            mi, oi = st.pending_ids() if status == 1 else (-1, -1)
            if status == 1 and mi < 0:
                status = 3  # ran fine but produced no update (e.g. an evaluation closure)
            vtype, vnum = _encode_value(value) if status == 1 or status == 3 else (0, 0.0)
            vec = torch.zeros(4 * world, dtype=torch.int64)
            vec[4 * rank: 4 * rank + 4] = torch.tensor([status, mi + 1, oi + 1, vtype])
            vec = torch.tensor(comm.all_reduce_int(vec.tolist()), dtype=torch.int64).view(world, 4)
            fvec = [0.0] * world
            fvec[rank] = vnum
            fvec = comm.all_reduce_float(fvec) if any(vec[:, 3].tolist()) else fvec
            statuses = vec[:, 0].tolist()
            failed = [r for r, s_ in enumerate(statuses) if s_ == 2]
            if failed:
                st.abort_round()
                requeue = []
                for r, item in enumerate(batch):
                    fn, args, kwargs, rv, tries = item
                    if r in failed:
                        if tries >= self.max_retries:
                            rv._error = err if r == rank else RuntimeError(
                                f"closure failed on worker {r} after {tries + 1} attempts")
                            rv._done = True
                            continue
                        tries += 1
                    requeue.append((fn, args, kwargs, rv, tries))
                self.retries += sum(1 for r in failed if r < len(batch))
                self._queue = requeue + rest
                continue
            if mine is not None:
                rv = mine[3]
                if status in (1, 3):
                    rv._set(value)
                    self.closures_run += 1
                elif err is not None:
                    rv._error = err
            contributed = [s_ == 1 for s_ in statuses]
            ids = [(int(m) - 1, int(o) - 1) for m, o in vec[:, 1:3].tolist() if m > 0]
            if ids:
                if len(set(ids)) != 1:
                    raise RuntimeError(f"closures of one round updated different (model, optimizer) pairs: {ids}")
                mi, oi = ids[0]
                model = st.models[mi]
                opt = st.optimizers[oi] if oi < len(st.optimizers) else model.optimizer
                st.commit_round(model, opt, contributed)
            for r, item in enumerate(batch):
                rv_ = item[3]
                if not rv_._done and rv_._error is None:
                    # executed on another rank: scalar results travel in the status exchange
                    rv_._set(_decode_value(int(vec[r, 3]), fvec[r]), local=False)
            self._queue = rest
            heartbeat.progress()
        comm.barrier()

    def done(self) -> bool:
        return not self._queue

    def fetch(self, values):
        if isinstance(values, (list, tuple)):
            return [v.fetch() for v in values]
        return values.fetch()
