"""``tf.data``-shaped input pipeline (train_tf_ps.py:297-321, :597-601, :664-668).

Supported: ``from_tensor_slices``, ``from_generator``, ``range``, ``zip``, ``map`` (optionally
parallel on a thread pool, ``num_parallel_calls=AUTOTUNE``), ``filter``, ``shard``, ``shuffle``
(buffer semantics: a sliding buffer of ``buffer_size`` elements, reshuffled each iteration),
``batch`` (numpy stacking; ``drop_remainder``), ``unbatch``, ``repeat``, ``take``, ``skip``,
``prefetch`` (background thread), ``cache``, ``cardinality``, ``as_numpy_iterator``.

Elements are tuples of numpy arrays (or a single array).  Batches stay on the host until the
trainer's device feed (data/device_feed.py: pinned staging ring, H2D on a side stream, event
handoff to the compute stream) moves them to HBM; raw uint8 images are resized / normalised on the
GPU by the first conv op.

Columnar fast path: a ``from_tensor_slices`` source followed only by ``shard`` / ``shuffle`` /
``batch`` / ``repeat`` / ``prefetch`` never iterates elements in Python: it builds index
permutations and gathers whole batches (``index_select`` on device tensors, fancy indexing on host
arrays).  Device tensors stay on the device, so a DataFrame column handed over by the ETL stage
(the joint Spark -> TF pipeline) feeds the trainer without a host round trip.  ``shuffle`` with
``buffer_size >= cardinality`` is an exact uniform shuffle; a smaller buffer is emulated by
shuffling within consecutive windows of ``buffer_size`` elements and then shuffling window order.
"""
from __future__ import annotations

import concurrent.futures as cf
import itertools
import queue
import threading

import numpy as np

AUTOTUNE = -1
INFINITE = -1
UNKNOWN = -2


def _np(x):
    try:
        import torch

        if isinstance(x, torch.Tensor):
            return x.detach().cpu().numpy()
    except ImportError:  # pragma: no cover
        pass
    return np.asarray(x)


class _ColPlan:
    """Vectorised plan of an array-backed dataset (see module docstring)."""

    def __init__(self, arrays, kind, keys=None):
        self.arrays, self.kind, self.keys = arrays, kind, keys
        self.n = len(arrays[0])
        self.ops: list = []  # ("shard", n, i) | ("shuffle", buf, seed, reshuffle) | ("batch", bs, drop) | ("repeat", c)
        self.epoch = 0

    def extend(self, op) -> "_ColPlan":
        p = _ColPlan(self.arrays, self.kind, self.keys)
        p.ops = self.ops + [op]
        return p

    def names(self):
        return [o[0] for o in self.ops]

    def _is_torch(self, a):
        return type(a).__module__.startswith("torch")

    def _device(self):
        """Device of the GPU-resident columns (index math then stays on the GPU), else None."""
        for a in self.arrays:
            if self._is_torch(a):
                return a.device
        return None

    def _gather(self, sel):
        out = []
        for a in self.arrays:
            if self._is_torch(a):
                import torch

                idx = sel if isinstance(sel, torch.Tensor) else torch.as_tensor(sel, device=a.device)
                out.append(a.index_select(0, idx))
            else:
                out.append(a[sel.cpu().numpy() if hasattr(sel, "cpu") else sel])
        return self._pack(out)

    def _pack(self, cols):
        if self.kind == "tuple":
            return tuple(cols)
        if self.kind == "dict":
            return dict(zip(self.keys, cols))
        return cols[0]

    def _order(self, base, shuffle, epoch):
        if shuffle is None:
            return base
        _, buf, seed, reshuffle = shuffle
        s = seed if seed is not None else 0x5EED
        dev = self._device()
        if dev is not None and buf >= len(base):
            import torch

            g = torch.Generator(device=dev)
            g.manual_seed(int(s) * 1000003 + (epoch if reshuffle else 0))
            return base[torch.randperm(len(base), generator=g, device=dev)]
        if dev is not None:
            base = base.cpu().numpy()
        rng = np.random.default_rng((s, epoch) if reshuffle else s)
        if buf >= len(base):
            return base[rng.permutation(len(base))]
        w = max(1, int(buf))
        chunks = [base[i:i + w] for i in range(0, len(base), w)]
        chunks = [c[rng.permutation(len(c))] for c in chunks]
        return np.concatenate([chunks[i] for i in rng.permutation(len(chunks))]) if chunks else base

    def on_device(self, dev) -> "_ColPlan":
        """The same plan over copies of the columns resident on ``dev`` (uploaded once): batches are
        then gathered on the device, no per-step host gather or host->device copy."""
        import torch

        arrs = [a if (self._is_torch(a) and a.device == dev) else torch.as_tensor(np.ascontiguousarray(_np(a))).to(dev)
                for a in self.arrays]
        p = _ColPlan(arrs, self.kind, self.keys)
        p.ops = list(self.ops)
        return p

    def __iter__(self):
        return self.iter_groups(1)

    def iter_groups(self, group: int = 1, with_count: bool = False):
        """Batches as the plan defines them; ``group`` > 1 yields up to ``group`` consecutive FULL
        batches as one gather (``with_count``: (batch, number of batches)); a partial batch always
        comes alone.  Same order and contents as ``group`` = 1."""
        for b, k in self._iter(max(1, int(group))):
            yield (b, k) if with_count else b

    def _iter(self, group):
        dev = self._device()
        if dev is not None:
            import torch

            base = torch.arange(self.n, device=dev)
        else:
            base = np.arange(self.n)
        shuffle, batch, repeat, batch_before_repeat = None, None, None, True
        for op in self.ops:
            if op[0] == "shard":
                base = base[op[2]::op[1]]
            elif op[0] == "shuffle":
                shuffle = op
            elif op[0] == "batch":
                batch = op
            elif op[0] == "repeat":
                repeat = op[1]
                batch_before_repeat = batch is not None
        epochs = itertools.count() if (repeat is not None and repeat < 0) else range(1 if repeat is None else repeat)

        def epoch_orders():
            for _ in epochs:
                e = self.epoch
                self.epoch += 1
                yield self._order(base, shuffle, e)

        if batch is None:
            for order in epoch_orders():
                for i in order:
                    yield self._pack([a[int(i)] for a in self.arrays]), 1
            return
        bs, drop = batch[1], batch[2]
        if batch_before_repeat:
            for order in epoch_orders():
                st = 0
                while st < len(order):
                    k = max(1, min(group, (len(order) - st) // bs))
                    sel = order[st:st + k * bs]
                    if drop and len(sel) < bs:
                        break
                    yield self._gather(sel), (k if len(sel) == k * bs else 1)
                    st += len(sel)
            return
        pending = None
        for order in epoch_orders():
            if pending is None:
                pending = order
            elif dev is not None:
                import torch

                pending = torch.cat([pending, order])
            else:
                pending = np.concatenate([pending, order])
            while len(pending) >= bs:
                k = max(1, min(group, len(pending) // bs))
                yield self._gather(pending[:k * bs]), k
                pending = pending[k * bs:]
        if pending is not None and len(pending) and not drop:
            yield self._gather(pending), 1


def _keep(a):
    """Array-like for the columnar path: GPU tensors stay on the device, the rest become numpy."""
    if type(a).__module__.startswith("torch") and a.is_cuda:
        return a
    return _np(a)


class Dataset:
    def __init__(self, gen_fn, card: int = UNKNOWN, plan: _ColPlan | None = None):
        self._gen_fn = gen_fn
        self._card = card
        self._plan = plan

    @staticmethod
    def _from_plan(plan: _ColPlan, card: int) -> "Dataset":
        return Dataset(lambda: iter(plan), card, plan)

    # ------------------------------------------------------------------ sources
    @staticmethod
    def from_tensor_slices(tensors) -> "Dataset":
        if isinstance(tensors, dict):
            keys = list(tensors)
            arrs = [_keep(tensors[k]) for k in keys]
            plan = _ColPlan(arrs, "dict", keys)
        elif isinstance(tensors, (tuple, list)):
            arrs = [_keep(t) for t in tensors]
            if any(len(a) != len(arrs[0]) for a in arrs):
                raise ValueError("from_tensor_slices: components differ in length")
            plan = _ColPlan(arrs, "tuple")
        else:
            plan = _ColPlan([_keep(tensors)], "single")
        return Dataset._from_plan(plan, plan.n)

    @staticmethod
    def from_generator(generator, output_signature=None, output_types=None) -> "Dataset":
        return Dataset(lambda: iter(generator()), UNKNOWN)

    @staticmethod
    def range(*args) -> "Dataset":
        r = range(*args)
        return Dataset(lambda: (np.int64(i) for i in r), len(r))

    @staticmethod
    def zip(datasets) -> "Dataset":
        ds = tuple(datasets)
        card = min((d._card for d in ds if d._card >= 0), default=UNKNOWN)
        if any(d._card == INFINITE for d in ds) and all(d._card == INFINITE for d in ds):
            card = INFINITE
        return Dataset(lambda: zip(*(iter(d) for d in ds)), card)

    # ------------------------------------------------------------------ transforms
    def map(self, fn, num_parallel_calls=None, deterministic=True) -> "Dataset":
        src = self

        def call(e):
            return fn(*e) if isinstance(e, tuple) else fn(e)

        if not num_parallel_calls or num_parallel_calls == 1:
            return Dataset(lambda: (call(e) for e in src), self._card)
        workers = 8 if num_parallel_calls == AUTOTUNE else int(num_parallel_calls)

        def gen():
            with cf.ThreadPoolExecutor(workers) as ex:
                pending = []
                for e in src:
                    pending.append(ex.submit(call, e))
                    if len(pending) >= 2 * workers:
                        yield pending.pop(0).result()
                for f in pending:
                    yield f.result()

        return Dataset(gen, self._card)

    def filter(self, pred) -> "Dataset":
        src = self
        return Dataset(lambda: (e for e in src if (pred(*e) if isinstance(e, tuple) else pred(e))), UNKNOWN)

    def shard(self, num_shards: int, index: int) -> "Dataset":
        src = self
        card = UNKNOWN if self._card < 0 else (self._card - index + num_shards - 1) // num_shards
        if self._plan is not None and self._plan.ops == []:
            return Dataset._from_plan(self._plan.extend(("shard", num_shards, index)), card)
        return Dataset(lambda: itertools.islice(iter(src), index, None, num_shards), card)

    def shuffle(self, buffer_size: int, seed=None, reshuffle_each_iteration: bool = True) -> "Dataset":
        src = self
        if self._plan is not None and set(self._plan.names()) <= {"shard"}:
            return Dataset._from_plan(self._plan.extend(("shuffle", int(buffer_size), seed, reshuffle_each_iteration)),
                                      self._card)
        state = {"epoch": 0}

        def gen():
            s = seed if seed is not None else np.random.SeedSequence().entropy
            rng = np.random.default_rng((s, state["epoch"]) if reshuffle_each_iteration else s)
            state["epoch"] += 1
            buf = []
            for e in src:
                if len(buf) < buffer_size:
                    buf.append(e)
                    continue
                j = int(rng.integers(len(buf)))
                yield buf[j]
                buf[j] = e
            rng.shuffle(buf)
            yield from buf

        ds = Dataset(gen, self._card)
        return ds

    def batch(self, batch_size: int, drop_remainder: bool = False) -> "Dataset":
        src = self
        if self._plan is not None and "batch" not in self._plan.names():
            if self._card >= 0:
                card = self._card // batch_size if drop_remainder else -(-self._card // batch_size)
            else:
                card = self._card
            return Dataset._from_plan(self._plan.extend(("batch", int(batch_size), bool(drop_remainder))), card)

        def stack(items):
            if isinstance(items[0], tuple):
                return tuple(np.stack([it[k] for it in items]) for k in range(len(items[0])))
            if isinstance(items[0], dict):
                return {k: np.stack([it[k] for it in items]) for k in items[0]}
            return np.stack(items)

        def gen():
            it = iter(src)
            while True:
                items = list(itertools.islice(it, batch_size))
                if not items or (drop_remainder and len(items) < batch_size):
                    return
                yield stack(items)

        if self._card >= 0:
            card = self._card // batch_size if drop_remainder else -(-self._card // batch_size)
        else:
            card = self._card
        return Dataset(gen, card)

    def unbatch(self) -> "Dataset":
        src = self

        def gen():
            for b in src:
                if isinstance(b, tuple):
                    for i in range(len(b[0])):
                        yield tuple(x[i] for x in b)
                else:
                    yield from b

        return Dataset(gen, UNKNOWN)

    def repeat(self, count=None) -> "Dataset":
        src = self
        if self._plan is not None and "repeat" not in self._plan.names():
            c = -1 if count is None else int(count)
            card = INFINITE if c < 0 else (self._card * c if self._card >= 0 else UNKNOWN)
            return Dataset._from_plan(self._plan.extend(("repeat", c)), card)

        def gen():
            n = 0
            while count is None or count < 0 or n < count:
                got = False
                for e in src:
                    got = True
                    yield e
                if not got:
                    return
                n += 1

        card = INFINITE if (count is None or count < 0) else (self._card * count if self._card >= 0 else UNKNOWN)
        return Dataset(gen, card)

    def take(self, count: int) -> "Dataset":
        src = self
        return Dataset(lambda: itertools.islice(iter(src), count),
                       count if self._card < 0 and self._card != UNKNOWN else min(count, self._card) if self._card >= 0 else count)

    def skip(self, count: int) -> "Dataset":
        src = self
        return Dataset(lambda: itertools.islice(iter(src), count, None),
                       max(self._card - count, 0) if self._card >= 0 else self._card)

    def prefetch(self, buffer_size=1) -> "Dataset":
        src = self
        if self._plan is not None:
            return self  # batches are gathered on demand (device-side for device tensors)
        depth = 2 if buffer_size in (None, AUTOTUNE) else max(1, int(buffer_size))

        def gen():
            q: queue.Queue = queue.Queue(maxsize=depth)
            done = object()
            stop = threading.Event()

            def worker():
                try:
                    for e in src:
                        if stop.is_set():
                            return
                        q.put(e)
                finally:
                    q.put(done)

            t = threading.Thread(target=worker, daemon=True)
            t.start()
            try:
                while True:
                    e = q.get()
                    if e is done:
                        return
                    yield e
            finally:
                stop.set()

        return Dataset(gen, self._card)

    def cache(self, filename: str = "") -> "Dataset":
        src = self
        store: list = []
        state = {"full": False}

        def gen():
            if state["full"]:
                yield from store
                return
            for e in src:
                store.append(e)
                yield e
            state["full"] = True

        return Dataset(gen, self._card)

    # ------------------------------------------------------------------ iteration
    def __iter__(self):
        return iter(self._gen_fn())

    def apply(self, transformation_func) -> "Dataset":
        return transformation_func(self)

    def as_numpy_iterator(self):
        return iter(self)

    def cardinality(self) -> int:
        return self._card

    def __len__(self):
        if self._card < 0:
            raise TypeError("dataset length is unknown or infinite")
        return self._card


class experimental:  # noqa: N801
    AUTOTUNE = AUTOTUNE

    @staticmethod
    def prefetch_to_device(device, buffer_size=None):
        from .device_feed import prefetch_to_device

        return prefetch_to_device(device, buffer_size)

    INFINITE_CARDINALITY = INFINITE
    UNKNOWN_CARDINALITY = UNKNOWN
