"""The async parameter server's shared-memory mailbox (csrc/host/shmsync.cpp, distribute/ps.py
_Mailbox): unique tickets under contention, publish -> take of the slot payload across threads,
applied-counter waits, the ring's slot reuse, and the timeout path."""
import os
import threading
import time

import pytest

from pyspark_tf_gke_amd import _native
from pyspark_tf_gke_amd.distribute import ps as PS

pytestmark = pytest.mark.skipif(not _native.host_available(), reason="host runtime not built")


@pytest.fixture
def mbox(monkeypatch, tmp_path):
    monkeypatch.setattr(PS.comm, "barrier", lambda *a, **k: None)
    path = f"/dev/shm/ptg_test_mbox_{os.getpid()}"
    m = PS._Mailbox(path, world=2, rank=0)
    yield m
    m.close()
    assert not os.path.exists(path)


def test_tickets_unique_under_contention(mbox):
    got = []
    lock = threading.Lock()

    def worker():
        mine = [mbox.ticket(1) for _ in range(500)]
        with lock:
            got.extend(mine)

    ths = [threading.Thread(target=worker) for _ in range(4)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    assert sorted(got) == list(range(2000))
    assert mbox.tickets_issued(1) == 2000 and mbox.tickets_issued(0) == 0


def test_publish_take_and_applied_ring(mbox):
    """An owner thread consumes 3 x NSLOT pushes in ticket order through the slot ring while the
    pusher waits for each slot's previous push before reusing it."""
    n = 3 * PS.NSLOT
    seen = []

    def owner():
        for t in range(n):
            got = None
            while got is None:
                got = mbox.take(0, t, 200_000)
            seen.append((t,) + got)
            mbox.set_applied(0, t + 1)

    th = threading.Thread(target=owner)
    th.start()
    for i in range(n):
        t = mbox.ticket(0)
        if t >= PS.NSLOT:
            mbox.wait_applied(0, t - PS.NSLOT + 1)
        mbox.publish(0, t, 0.5 * t, t % 3 - 1)
    mbox.wait_applied(0, n)
    th.join(timeout=10)
    assert [s[0] for s in seen] == list(range(n))
    assert all(g == 0.5 * t and oi == t % 3 - 1 for t, g, oi in seen)


def test_take_timeout_and_wait_error(mbox):
    t0 = time.perf_counter()
    assert mbox.take(1, 0, 20_000) is None
    assert time.perf_counter() - t0 >= 0.015
    mbox.timeout_s = 1.0
    with pytest.raises(RuntimeError, match="did not apply"):
        mbox.wait_applied(1, 1)

    def dead():
        raise RuntimeError("service thread failed")

    mbox.timeout_s = 30.0
    with pytest.raises(RuntimeError, match="service thread failed"):
        mbox.wait_applied(1, 1, dead)
