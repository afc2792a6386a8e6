"""Rank progress heartbeats for hang detection.

A liveness beat cannot see a hang: a rank blocked inside a collective still has a running
heartbeat thread.  So the beat carries a *progress counter* that only the training loop advances
(:func:`progress` is called once per train step / coordinator round).  A daemon thread writes
``"<counter> <time of the last counter change>"`` to ``$PTG_HEARTBEAT_DIR/rank<r>`` every
``interval`` seconds; the launcher declares a rank hung when its counter has not moved for
``hang_timeout`` seconds (before the first step: ``startup`` seconds), kills the group and restarts
it from the latest checkpoint.
"""
from __future__ import annotations

import os
import threading
import time

_started = False
_count = 0
_changed = time.time()


def progress(n: int = 1) -> None:
    """Advance this rank's progress counter (cheap: two Python assignments)."""
    global _count, _changed
    _count += n
    _changed = time.time()


def count() -> int:
    return _count


def start(interval: float = 2.0) -> None:
    global _started
    d = os.environ.get("PTG_HEARTBEAT_DIR")
    if _started or not d:
        return
    _started = True
    path = os.path.join(d, f"rank{os.environ.get('RANK', '0')}")
    born = time.time()

    def beat():
        while True:
            try:
                tmp = path + ".tmp"
                with open(tmp, "w") as fh:
                    fh.write(f"{_count} {_changed if _count else born}")
                os.replace(tmp, path)
            except OSError:
                pass
            time.sleep(interval)

    threading.Thread(target=beat, daemon=True, name="ptg-heartbeat").start()


def read(d: str, rank: int):
    """-> (counter, time of its last change) or None if the rank has not reported yet."""
    try:
        with open(os.path.join(d, f"rank{rank}")) as fh:
            c, t = fh.read().split()
        return int(c), float(t)
    except (OSError, ValueError):
        return None


def stale_ranks(d: str, nprocs: int, timeout: float, startup: float | None = None) -> list:
    """Ranks whose progress counter has not moved for ``timeout`` seconds (``startup`` seconds while
    it is still 0: imports, rendezvous and kernel warm-up come before the first step)."""
    now = time.time()
    startup = max(timeout, startup if startup is not None else 10 * timeout)
    out = []
    for r in range(nprocs):
        ent = read(d, r)
        if ent is None:
            continue  # not started yet
        c, t = ent
        if now - t > (timeout if c > 0 else startup):
            out.append(r)
    return out
