"""``tf.data``-shaped input pipeline (train_tf_ps.py:297-321, :597-601, :664-668).

Supported: ``from_tensor_slices``, ``from_generator``, ``range``, ``zip``, ``map`` (optionally
parallel on a thread pool, ``num_parallel_calls=AUTOTUNE``), ``filter``, ``shard``, ``shuffle``
(buffer semantics: a sliding buffer of ``buffer_size`` elements, reshuffled each iteration),
``batch`` (numpy stacking; ``drop_remainder``), ``unbatch``, ``repeat``, ``take``, ``skip``,
``prefetch`` (background thread), ``cache``, ``cardinality``, ``as_numpy_iterator``.

Elements are tuples of numpy arrays (or a single array).  Batches stay on the host; the trainer
uploads them with pinned, non-blocking copies (and raw uint8 images are resized/normalised on the
GPU by the first conv op).
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


class Dataset:
    def __init__(self, gen_fn, card: int = UNKNOWN):
        self._gen_fn = gen_fn
        self._card = card

    # ------------------------------------------------------------------ sources
    @staticmethod
    def from_tensor_slices(tensors) -> "Dataset":
        if isinstance(tensors, dict):
            keys = list(tensors)
            arrs = [_np(tensors[k]) for k in keys]
            n = len(arrs[0])

            def gen():
                for i in range(n):
                    yield {k: a[i] for k, a in zip(keys, arrs)}

            return Dataset(gen, n)
        if isinstance(tensors, (tuple, list)):
            arrs = [_np(t) for t in tensors]
            n = len(arrs[0])
            if any(len(a) != n for a in arrs):
                raise ValueError("from_tensor_slices: components differ in length")

            def gen():
                for i in range(n):
                    yield tuple(a[i] for a in arrs)

            ds = Dataset(gen, n)
            ds._arrays = arrs  # fast path for index-based batching
            return ds
        arr = _np(tensors)

        def gen1():
            for i in range(len(arr)):
                yield arr[i]

        return Dataset(gen1, len(arr))

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
        ds = Dataset(lambda: itertools.islice(iter(src), index, None, num_shards), card)
        if hasattr(self, "_arrays"):
            ds._arrays = [a[index::num_shards] for a in self._arrays]
        return ds

    def shuffle(self, buffer_size: int, seed=None, reshuffle_each_iteration: bool = True) -> "Dataset":
        src = self
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
    INFINITE_CARDINALITY = INFINITE
    UNKNOWN_CARDINALITY = UNKNOWN
