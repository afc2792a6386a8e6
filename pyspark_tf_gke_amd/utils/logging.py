"""Logging in the reference's format (spark_session.py:8-26): module logger at INFO with
``%(asctime)s - %(name)s - %(levelname)s - %(message)s``, root at ERROR; rank-aware (only rank 0
logs INFO unless PTG_LOG_ALL_RANKS=1)."""
from __future__ import annotations

import logging
import os

FORMAT = "%(asctime)s - %(name)s - %(levelname)s - %(message)s"


class _RankFilter(logging.Filter):
    def filter(self, record):
        rank = int(os.environ.get("RANK", "0"))
        if rank != 0 and not os.environ.get("PTG_LOG_ALL_RANKS") and record.levelno < logging.WARNING:
            return False
        record.msg = f"[rank {rank}] {record.msg}" if int(os.environ.get("WORLD_SIZE", "1")) > 1 else record.msg
        return True


def configure(root_level=logging.ERROR) -> None:
    logging.basicConfig(level=root_level, format=FORMAT)
    for noisy in ("urllib3", "botocore"):
        logging.getLogger(noisy).setLevel(logging.ERROR)


def get_logger(name: str, level=logging.INFO) -> logging.Logger:
    configure()
    lg = logging.getLogger(name)
    lg.setLevel(level)
    lg.propagate = False
    if not lg.handlers:
        h = logging.StreamHandler()
        h.setLevel(level)
        h.setFormatter(logging.Formatter(FORMAT))
        h.addFilter(_RankFilter())
        lg.addHandler(h)
    return lg
