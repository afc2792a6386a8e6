"""Single-node rank launcher — replaces the reference's Kubernetes control plane (Spark master/worker
Deployments, TF worker/PS StatefulSets, MetalLB/headless-service discovery) on one
8xMI355X node: one OS process per GPU, rank r = Spark executor r = TF worker r.

Failure detection / elastic recovery:
  * a rank that exits non-zero makes the launcher stop the others (SIGTERM, then SIGKILL after a
    grace period) — no rank is left blocked in a collective;
  * ranks report a progress counter through files in ``PTG_HEARTBEAT_DIR`` (:mod:`.heartbeat`); a
    rank whose counter has not moved for ``hang_timeout`` seconds (e.g. blocked in a collective) is
    treated as hung (before its first step the limit is ``startup_timeout``);
  * ``max_restarts`` relaunches the whole group (applications resume from their checkpoint, e.g.
    ``train --checkpoint-every 1 --resume``);
  * ``min_nprocs`` (executor loss, Spark standalone's lost-executor handling): instead of relaunching
    the failed rank, the group restarts WITHOUT it on the remaining devices (``PTG_DEVICE_ORDINAL``
    keeps every survivor on its own GPU).  Sources are split by (rank, world) at read time, so the
    lost executor's partitions are re-assigned to the survivors and recomputed from their lineage
    (the source read + the narrow / wide stages after it) - down to ``min_nprocs`` executors;
  * fault injection for tests: ``PTG_FAULT_RANK`` / ``PTG_FAULT_STEP`` (:mod:`.fault`).
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import tempfile
import threading
import time


def free_port(addr: str = "127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((addr, 0))
        return s.getsockname()[1]


def _pump(stream, rank: int, out):
    for line in iter(stream.readline, b""):
        try:
            out.write(f"[rank{rank}] " + line.decode("utf-8", "replace"))
            out.flush()
        except ValueError:
            break
    stream.close()


def _die_with_parent():
    """preexec: SIGKILL this rank if the launcher dies (no orphaned ranks blocked in collectives)."""
    try:
        import ctypes

        ctypes.CDLL("libc.so.6").prctl(1, signal.SIGKILL)  # PR_SET_PDEATHSIG
    except OSError:
        pass


def _spawn(cmd, nprocs, master_addr, master_port, env_extra, hb_dir, prefix, devices=None):
    procs, pumps = [], []
    for r in range(nprocs):
        env = dict(os.environ)
        env.update(env_extra or {})
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(nprocs), "LOCAL_WORLD_SIZE": str(nprocs),
                    "MASTER_ADDR": master_addr, "MASTER_PORT": str(master_port), "PTG_HEARTBEAT_DIR": hb_dir})
        if devices is not None:
            env["PTG_DEVICE_ORDINAL"] = str(devices[r])
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if prefix:
            p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, start_new_session=True,
                                 preexec_fn=_die_with_parent)
            t = threading.Thread(target=_pump, args=(p.stdout, r, sys.stdout), daemon=True)
            t.start()
            pumps.append(t)
        else:
            p = subprocess.Popen(cmd, env=env, start_new_session=True, preexec_fn=_die_with_parent)
        procs.append(p)
    return procs, pumps


def _terminate(procs, grace: float = 10.0):
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass
    t0 = time.time()
    while time.time() - t0 < grace and any(p.poll() is None for p in procs):
        time.sleep(0.1)
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGKILL)
            except ProcessLookupError:
                pass
            p.wait()


def launch(cmd: list, nprocs: int, master_addr: str = "127.0.0.1", master_port: int | None = None,
           env_extra: dict | None = None, max_restarts: int = 0, hang_timeout: float = 0.0, prefix_output: bool = True,
           poll: float = 0.2, startup_timeout: float | None = None, min_nprocs: int = 0) -> int:
    """Run ``cmd`` on ``nprocs`` ranks; return 0 or the first failing rank's exit code.
    ``min_nprocs`` > 0: a failed rank's executor is dropped and the group restarts on the survivors
    (while at least ``min_nprocs`` remain) instead of relaunching it."""
    attempt = 0
    devices = list(range(nprocs))
    lost: list = []
    while True:
        port = master_port or free_port(master_addr)
        hb_dir = tempfile.mkdtemp(prefix="ptg_hb_")
        env = dict(env_extra or {})
        env["PTG_RESTART_COUNT"] = str(attempt)
        if lost:
            env["PTG_LOST_EXECUTORS"] = ",".join(str(d) for d in lost)
        procs, pumps = _spawn(cmd, nprocs, master_addr, port, env, hb_dir, prefix_output,
                              devices if min_nprocs > 0 else None)
        rc, failed = 0, None
        try:
            while True:
                codes = [p.poll() for p in procs]
                bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
                if bad:
                    failed, rc = bad[0]
                    break
                if all(c == 0 for c in codes):
                    break
                if hang_timeout > 0:
                    from .heartbeat import stale_ranks

                    stale = stale_ranks(hb_dir, nprocs, hang_timeout, startup_timeout)
                    if stale:
                        failed, rc = stale[0], 124
                        sys.stderr.write(f"[launcher] rank {failed} made no progress for > {hang_timeout}s: treating as hung\n")
                        break
                time.sleep(poll)
        except KeyboardInterrupt:
            _terminate(procs)
            return 130
        if failed is not None:
            sys.stderr.write(f"[launcher] rank {failed} exited with {rc}; stopping the other ranks\n")
            _terminate(procs)
        for t in pumps:
            t.join(timeout=2)
        if rc == 0 or attempt >= max_restarts:
            return rc
        attempt += 1
        if min_nprocs > 0 and failed is not None and nprocs - 1 >= min_nprocs:
            lost.append(devices.pop(failed))
            nprocs -= 1
            sys.stderr.write(f"[launcher] executor {lost[-1]} lost: its partitions are re-planned onto the {nprocs} "
                             f"remaining executors (attempt {attempt}/{max_restarts})\n")
            continue
        sys.stderr.write(f"[launcher] restarting all ranks (attempt {attempt}/{max_restarts})\n")


def main(argv=None) -> int:
    import argparse

    ap = argparse.ArgumentParser(description="Launch one process per GPU (RANK/LOCAL_RANK/WORLD_SIZE env)")
    ap.add_argument("--nproc", type=int, default=0, help="ranks (default: number of GPUs, or 1)")
    ap.add_argument("--master-addr", default="127.0.0.1")
    ap.add_argument("--master-port", type=int, default=0)
    ap.add_argument("--max-restarts", type=int, default=0)
    ap.add_argument("--hang-timeout", type=float, default=0.0)
    ap.add_argument("--startup-timeout", type=float, default=None)
    ap.add_argument("--min-nproc", type=int, default=0,
                    help="on a rank failure drop its executor and restart on the survivors (down to this many)")
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    if not cmd:
        ap.error("missing command")
    n = a.nproc or _gpu_count() or 1
    return launch(cmd, n, a.master_addr, a.master_port or None, max_restarts=a.max_restarts,
                  hang_timeout=a.hang_timeout, startup_timeout=a.startup_timeout, min_nprocs=a.min_nproc)


def _gpu_count() -> int:
    try:
        import torch

        return torch.cuda.device_count()  # does not initialise HIP on this image
    except Exception:  # noqa: BLE001
        return 0


if __name__ == "__main__":
    sys.exit(main())
