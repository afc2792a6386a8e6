"""Rank heartbeats for hang detection: a daemon thread touches ``$PTG_HEARTBEAT_DIR/rank<r>``
every ``interval`` seconds; the launcher declares a rank hung when its file goes stale."""
from __future__ import annotations

import os
import threading
import time

_started = False


def start(interval: float = 2.0) -> None:
    global _started
    d = os.environ.get("PTG_HEARTBEAT_DIR")
    if _started or not d:
        return
    _started = True
    path = os.path.join(d, f"rank{os.environ.get('RANK', '0')}")

    def beat():
        while True:
            try:
                with open(path, "w") as fh:
                    fh.write(str(time.time()))
            except OSError:
                pass
            time.sleep(interval)

    threading.Thread(target=beat, daemon=True, name="ptg-heartbeat").start()


def stale_ranks(d: str, nprocs: int, timeout: float) -> list:
    now = time.time()
    out = []
    for r in range(nprocs):
        p = os.path.join(d, f"rank{r}")
        try:
            if now - os.path.getmtime(p) > timeout:
                out.append(r)
        except FileNotFoundError:
            continue  # not started yet
    return out
