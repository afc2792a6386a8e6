"""``ClusterCoordinator``: the reference's schedule/join driver (train_tf_ps.py:612-614, :634-647,
:734-736, :755-769) on SPMD ranks.

Every rank runs the same driver script, so every rank holds the same closure queue;
``schedule(fn, args)`` queues a closure and returns a :class:`RemoteValue`; ``join()`` is the epoch
barrier of the reference.  A closure runs on exactly one rank, with that rank's per-worker dataset
iterator (``create_per_worker_dataset``), and its scalar result is visible on every rank.

Asynchronous parameter server (``ParameterServerStrategy(mode="async")``, N > 1): closures are
handed to whichever worker is idle - each rank draws the next closure index from a counter in the
TCP store until the queue is exhausted - and a closure's ``apply_gradients`` pushes straight to the
PS owners (one-sided, ps.py) without any collective, so a slow worker simply runs fewer closures
(TF's ``ClusterCoordinator.schedule`` dispatch).  A closure that raises before its push goes back to
a shared retry queue for a DIFFERENT idle worker, up to ``max_retries`` times; the closures of a
worker whose process stops beating are re-queued for the others.  Results travel through the
store.

Synchronous strategies (sync PS, MWMS): ``join()`` runs the queue in rounds of ``world_size``
closures, closure i of a round on rank ``i % world``; a round is a transaction:
  1. every rank runs its closure (if any) with the strategy in *deferred* mode: gradient pushes and
     optimizer updates inside the closure (``optimizer.apply_gradients``, ``model.train_step``) are
     recorded, not executed, so a closure that raises leaves no collective half-issued;
  2. the ranks exchange one small status tensor (all-reduce, no pickles): per rank ok / no closure /
     failed, plus which (model, optimizer) the update belongs to;
  3. if some closure failed and may be retried, ONLY the failed closures run again, on the ranks
     that failed them, with their partial gradients discarded; the ranks whose closures succeeded
     keep their pending gradients and results (their iterators are not advanced twice, their forward
     side effects are not repeated); a closure that exhausted ``max_retries`` is dropped with its
     error recorded on every rank;
  4. then the round is committed collectively: the strategy pushes the contributors' gradients
     (ranks without a closure push nothing and the average is over the contributors; nobody
     contributing means no optimizer step).

Closures must not call collectives themselves (every rank would have to reach them).
"""
from __future__ import annotations

from ..parallel import comm

_COORDINATORS = [0]


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
        self._remote_key = None  # async dispatch: where the executing rank published the result

    def _set(self, v, local=True):
        self._value, self._done, self._local = v, True, local

    def _resolve(self):
        if self._done or self._error is not None or self._remote_key is None:
            return
        from .ps import _store

        msg = _store().get(self._remote_key).decode()
        kind, _, rest = msg.partition(":")
        if kind == "E":
            self._error = RuntimeError(rest)
        else:
            vt, _, x = rest.partition(":")
            self._set(_decode_value(int(vt), float(x)), local=False)

    def fetch(self):
        self._resolve()
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
        _COORDINATORS[0] += 1
        self._cid = _COORDINATORS[0]  # same on every rank: coordinators are created in the same order
        self._gen = 0

    def create_per_worker_dataset(self, dataset_fn):
        ctx = self.strategy.input_context()
        ds = dataset_fn(ctx) if callable(dataset_fn) else dataset_fn
        return PerWorkerDataset(ds)

    def schedule(self, fn, args=(), kwargs=None) -> RemoteValue:
        rv = RemoteValue()
        self._queue.append((fn, tuple(args), dict(kwargs or {}), rv, 0))
        return rv

    def join(self) -> None:
        if getattr(self.strategy, "is_async", False):
            self._join_async()
        else:
            self._join_rounds()

    # ---- asynchronous dispatch ------------------------------------------------------------------
    def _join_async(self) -> None:
        """Closures go to whichever worker asks first (a store counter).  A closure that raises
        before its gradient push goes back to a shared retry queue with the failing worker excluded,
        so a different idle worker runs it (TF's ClusterCoordinator reschedules a failed closure on
        another worker, train_tf_ps.py:612,642-645); a worker excluded by every rank may take it
        again.  A closure that fails after its push (the update is already applied) or after
        ``max_retries`` retries is recorded as failed.  Closures drawn by a worker whose liveness
        beat stops (its process died) are re-queued for the others.  Every outcome is published in
        the store, so each rank's RemoteValue resolves to it."""
        import threading
        import time

        from .. import config
        from ..runtime import heartbeat
        from .ps import _store

        st = self.strategy
        store = _store()
        self._gen += 1
        pre = f"ptg/coord/{st._token if getattr(st, '_token', None) else 'x'}/{self._cid}/{self._gen}"
        queue, self._queue = self._queue, []
        n = len(queue)
        world, rank = st.world_size, st.rank
        every = (1 << world) - 1
        dead_s = float(config.get("coord_dead_s"))
        stop = threading.Event()

        def beat():  # liveness (not progress): stops only when this process does
            bs = _store()
            while not stop.is_set():
                bs.set(f"{pre}/hb/{rank}", repr(time.time()))
                stop.wait(min(1.0, dead_s / 4))

        store.set(f"{pre}/hb/{rank}", repr(time.time()))  # nobody reads this rank as dead before its thread runs
        hb = threading.Thread(target=beat, daemon=True, name="ptg-coord-beat")
        hb.start()

        def finalize(i, msg) -> bool:
            # exactly one outcome per closure (a re-queued closure of a worker presumed dead may
            # still complete there)
            if store.add(f"{pre}/fin/{i}", 1) != 1:
                return False
            store.set(f"{pre}/rv/{i}", msg)
            store.add(pre + "/nfin", 1)
            return True

        def requeue(i, tries, excl):
            # the owner mark says "queued" from now on, so a dead-worker scan cannot queue it twice
            store.set(f"{pre}/own/{i}", "q")
            j = store.add(pre + "/rq/alloc", 1) - 1
            store.set(f"{pre}/rq/{j}", f"{i}:{tries}:{excl}")

        dead_mask = [0]  # ranks found dead by this rank's scans
        seen_nfin = [-1]
        skipped: list = []  # retry entries this rank was excluded from (claimable once the others die)
        deadline_s = float(config.get("coord_stall_s")) or float(config.get("pg_timeout_s"))
        cursor, fresh_done, last_scan, last_progress = 0, False, time.time(), time.time()
        try:
            while True:
                job = None
                nq = store.add(pre + "/rq/alloc", 0)
                while job is None and cursor < nq:
                    store.wait([f"{pre}/rq/{cursor}"])
                    i, tries, excl = (int(x) for x in store.get(f"{pre}/rq/{cursor}").decode().split(":"))
                    j, cursor = cursor, cursor + 1
                    if excl & (1 << rank) and (excl | dead_mask[0]) != every:
                        skipped.append((j, i, tries, excl))
                        continue  # a worker that failed it leaves it to the others (while one is alive)
                    if store.add(f"{pre}/rq/{j}/claim", 1) == 1:
                        job = (i, tries, excl & every if excl != every else 0)
                if job is None and not fresh_done:
                    i = store.add(pre + "/next", 1) - 1
                    if i < n:
                        job = (i, 0, 0)
                    else:
                        fresh_done = True
                if job is None:
                    nfin = store.add(pre + "/nfin", 0)
                    if nfin >= n:
                        break
                    now = time.time()
                    if now - last_scan > min(1.0, dead_s / 4):
                        last_scan = now
                        dead_mask[0] |= self._rescue_dead(store, pre, n, world, rank, dead_s, requeue)
                        self._check_abort(store, pre)
                        if nfin != seen_nfin[0] or self._live_busy(store, pre, world, rank, dead_mask[0], now, dead_s):
                            # progress, or a live worker is inside a closure (a first-call native build
                            # or an epoch-sized closure is not a stall)
                            seen_nfin[0], last_progress = nfin, now
                        elif now - last_progress > deadline_s:
                            msg = (f"ClusterCoordinator.join: no closure finished for {deadline_s:.0f} s and no "
                                   f"live worker is running one ({nfin}/{n} done; PTG_COORD_STALL_S), seen by "
                                   f"worker {rank}")
                            store.set(pre + "/abort", msg)  # every rank's loop fails with it, not just ours
                            raise RuntimeError(msg)
                    for k, (j, i, tries, excl) in enumerate(skipped):
                        if (excl | dead_mask[0]) == every:
                            del skipped[k]
                            if store.add(f"{pre}/rq/{j}/claim", 1) == 1:
                                job = (i, tries, 0)
                            break
                    if job is None:
                        time.sleep(0.002)
                        continue
                last_progress = time.time()
                i, tries, excl = job
                store.set(f"{pre}/own/{i}", str(rank))
                store.set(f"{pre}/busy/{rank}", "1")
                fn, args, kwargs, rv, _ = queue[i]
                st._closure_pushed = False
                try:
                    value = fn(*args, **kwargs)
                except StopIteration as e:
                    if finalize(i, f"E:StopIteration on worker {rank}"):
                        rv._error = e
                except Exception as e:  # noqa: BLE001 - rescheduled on another idle worker
                    if getattr(st, "_closure_pushed", False) or tries >= self.max_retries:
                        why = "after its gradient push" if getattr(st, "_closure_pushed", False) else \
                            f"after {tries + 1} attempts"
                        msg = f"closure failed on worker {rank} {why}: {e!r}"[:2000]
                        if finalize(i, "E:" + msg):
                            rv._error = RuntimeError(msg)
                            rv._error.__cause__ = e
                    else:
                        self.retries += 1
                        requeue(i, tries + 1, excl | (1 << rank))
                else:
                    vt, x = _encode_value(value)
                    if finalize(i, f"V:{vt}:{x!r}"):
                        rv._set(value)
                        self.closures_run += 1
                store.set(f"{pre}/busy/{rank}", "0")
                heartbeat.progress()
                self._check_abort(store, pre)
        finally:
            stop.set()
            hb.join(timeout=5)
        st.wait_all_applied()  # collective: every push applied, every rank pulled the final values
        for i, (_, _, _, rv, _) in enumerate(queue):
            if not rv._done and rv._error is None:
                rv._remote_key = f"{pre}/rv/{i}"  # ran elsewhere: resolved on fetch()
        comm.barrier()

    @staticmethod
    def _check_abort(store, pre) -> None:
        """Fail this rank's join too once any rank declared the round stalled."""
        if store.check([pre + "/abort"]):
            raise RuntimeError(store.get(pre + "/abort").decode())

    @staticmethod
    def _live_busy(store, pre, world, rank, dead_mask, now, dead_s) -> bool:
        """Whether another worker whose liveness beat is fresh is running a closure right now."""
        for r in range(world):
            if r == rank or dead_mask & (1 << r):
                continue
            bk, hk = f"{pre}/busy/{r}", f"{pre}/hb/{r}"
            if store.check([bk, hk]) and store.get(bk) == b"1" and now - float(store.get(hk).decode()) <= dead_s:
                return True
        return False

    @staticmethod
    def _rescue_dead(store, pre, n, world, rank, dead_s, requeue) -> None:
        """Re-queue the unfinished closures of workers whose liveness beat is older than dead_s."""
        import time

        now = time.time()
        dead = []
        for r in range(world):
            if r == rank:
                continue
            key = f"{pre}/hb/{r}"
            if store.check([key]) and now - float(store.get(key).decode()) > dead_s:
                dead.append(r)
        if not dead:
            return 0
        for i in range(n):
            own = f"{pre}/own/{i}"
            if not store.check([own]) or store.check([f"{pre}/rv/{i}"]):
                continue
            o = store.get(own).decode()
            if not o.isdigit():
                continue  # already back in the retry queue (its failed attempt re-queued it)
            r = int(o)
            if r in dead and store.add(f"{pre}/rescue/{i}/{r}", 1) == 1:
                requeue(i, 0, 1 << r)
        return sum(1 << r for r in dead)

    # ---- transactional rounds (sync) ---------------------------------------------------------------
    def _join_rounds(self) -> None:
        import torch

        from ..runtime import heartbeat

        st = self.strategy
        world, rank = st.world_size, st.rank
        if not comm.distributed():
            self._join_local()
            return
        while self._queue:
            batch = self._queue[:world]
            rest = self._queue[world:]
            mine = batch[rank] if rank < len(batch) else None
            tries = mine[4] if mine is not None else 0
            # 0 = no closure / StopIteration, 1 = gradient pending, 2 = failed (retry), 3 = ran, no
            # update, 4 = failed for good (dropped)
            status, err, value = None, None, None
            st.begin_round()
            while True:
                if status is None or status == 2:
                    status, err, value = self._run_mine(st, mine)
                    if status == 2 and tries >= self.max_retries:
                        status = 4
                        st.abort_round()  # dropped: its partial gradient goes nowhere
                mi, oi = st.pending_ids() if status == 1 else (-1, -1)
                if status == 1 and mi < 0:
                    status = 3  # ran fine but produced no update (e.g. an evaluation closure)
                # a tensor result is shared through the status exchange only when another rank
                # needs it: encoding reads it on the host, which drained the stream every closure
                # (one worker: 2.08 -> see profiles/r3_tape_overlap_ps_vs_fit.txt)
                share = status in (1, 3) and (world > 1 or not isinstance(value, torch.Tensor))
                vtype, vnum = _encode_value(value) if share else (0, 0.0)
                vec = torch.zeros(4 * world, dtype=torch.int64)
                vec[4 * rank: 4 * rank + 4] = torch.tensor([status, mi + 1, oi + 1, vtype])
                vec = torch.tensor(comm.all_reduce_int(vec.tolist()), dtype=torch.int64).view(world, 4)
                statuses = vec[:, 0].tolist()
                failed = [r for r, s_ in enumerate(statuses) if s_ == 2]
                if not failed:
                    break
                # only the failed closures run again; the others keep their pending gradients
                self.retries += len(failed)
                if status == 2:
                    st.abort_round()  # this rank's partial gradient of the failed attempt
                    tries += 1
                    st.begin_round_retry()
            fvec = [0.0] * world
            fvec[rank] = vnum
            fvec = comm.all_reduce_float(fvec) if any(vec[:, 3].tolist()) else fvec
            for r, item in enumerate(batch):
                rv_ = item[3]
                if r == rank:
                    if status in (1, 3):
                        rv_._set(value)
                        self.closures_run += 1
                    elif err is not None:
                        rv_._error = err
                elif statuses[r] == 4:
                    rv_._error = RuntimeError(f"closure failed on worker {r} after {self.max_retries + 1} attempts")
                elif statuses[r] in (1, 3):
                    # executed on another rank: scalar results travel in the status exchange
                    rv_._set(_decode_value(int(vec[r, 3]), fvec[r]), local=False)
                elif statuses[r] == 0:
                    rv_._set(None, local=False)
            contributed = [s_ == 1 for s_ in statuses]
            ids = [(int(m) - 1, int(o) - 1) for m, o in vec[:, 1:3].tolist() if m > 0]
            if ids:
                if len(set(ids)) != 1:
                    raise RuntimeError(f"closures of one round updated different (model, optimizer) pairs: {ids}")
                mi, oi = ids[0]
                model = st.models[mi]
                opt = st.optimizers[oi] if oi < len(st.optimizers) else model.optimizer
                st.commit_round(model, opt, contributed)
            else:
                st.abort_round()
            self._queue = rest
            heartbeat.progress()
        comm.barrier()

    def _join_local(self) -> None:
        """One worker: the same transactional rounds (retry, drop after max_retries, commit) with no
        status exchange and no per-round host tensors."""
        from ..runtime import heartbeat

        st = self.strategy
        while self._queue:
            q, self._queue = self._queue, []
            for k, item in enumerate(q):
                tries = item[4]
                st.begin_round()
                while True:
                    status, err, value = self._run_mine(st, item)
                    if status != 2:
                        break
                    st.abort_round()  # the failed attempt's partial gradient
                    if tries >= self.max_retries:
                        status = 4
                        break
                    self.retries += 1
                    tries += 1
                    st.begin_round_retry()
                mi, oi = st.pending_ids() if status == 1 else (-1, -1)
                rv = item[3]
                if status in (1, 3):
                    rv._set(value)
                    self.closures_run += 1
                elif err is not None:
                    rv._error = err
                if status == 1 and mi >= 0:
                    model = st.models[mi]
                    opt = st.optimizers[oi] if oi < len(st.optimizers) else model.optimizer
                    try:
                        st.commit_round(model, opt, [True])
                    except BaseException:
                        self._queue = list(q[k + 1:]) + self._queue
                        raise
                elif status != 4:
                    st.abort_round()
                heartbeat.progress()

    def _run_mine(self, st, mine):
        if mine is None:
            return 0, None, None
        fn, args, kwargs, _, _ = mine
        try:
            return 1, None, fn(*args, **kwargs)
        except StopIteration as e:
            return 0, e, None
        except Exception as e:  # noqa: BLE001 - reported to every rank
            return 2, e, None
        finally:
            st.end_round_local()

    def done(self) -> bool:
        return not self._queue

    def fetch(self, values):
        if isinstance(values, (list, tuple)):
            return [v.fetch() for v in values]
        return values.fetch()
