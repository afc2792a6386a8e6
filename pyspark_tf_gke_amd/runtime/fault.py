"""Fault injection for recovery tests: ``PTG_FAULT_RANK=r PTG_FAULT_STEP=s`` makes rank r exit with
code 17 at training step s (only on the first launch attempt unless PTG_FAULT_EVERY_ATTEMPT=1)."""
from __future__ import annotations

import os
import sys

_step = 0


def maybe_fail() -> None:
    global _step
    _step += 1
    fr = os.environ.get("PTG_FAULT_RANK")
    if fr is None:
        return
    if os.environ.get("PTG_RESTART_COUNT", "0") != "0" and not os.environ.get("PTG_FAULT_EVERY_ATTEMPT"):
        return
    if int(os.environ.get("RANK", "0")) == int(fr) and _step == int(os.environ.get("PTG_FAULT_STEP", "1")):
        sys.stderr.write(f"[fault] injected failure on rank {fr} at step {_step}\n")
        sys.stderr.flush()
        os._exit(17)
