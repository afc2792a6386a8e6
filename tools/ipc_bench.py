"""Latency of the one-shot IPC all-reduce (parallel/ipc.py) per message size.

    python -m pyspark_tf_gke_amd.runtime.launcher --nproc 2 -- python tools/ipc_bench.py

Each rank issues ``reps`` back-to-back in-place all-reduces (no host sync between them) and reports
microseconds per call.  With several ranks on ONE GPU (the 1-GPU box) this measures the kernel +
flag round-trip protocol with every "link" being local HBM; on an 8-GPU node the same script
measures it over xGMI, and ``--rccl`` adds torch.distributed all_reduce (RCCL) for comparison.
"""
import argparse
import json
import time

import torch
import torch.distributed as dist

from pyspark_tf_gke_amd.parallel import comm, ipc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--rccl", action="store_true")
    a = ap.parse_args()
    comm.init(backend="nccl" if a.rccl else "gloo", device_type="cuda")
    dev = torch.device("cuda", torch.cuda.current_device())
    ar = ipc.IpcAllReduce(dev, cap_bytes=1 << 20)
    out = {}
    for nbytes in (256, 4096, 31 * 1024, 256 * 1024, 1 << 20):
        x = torch.ones(nbytes // 4, device=dev)
        for _ in range(10):
            ar.all_reduce_(x)
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            ar.all_reduce_(x)
        torch.cuda.synchronize()
        us = (time.perf_counter() - t0) / a.reps * 1e6
        rec = {"ipc_us": round(us, 2)}
        if a.rccl:
            for _ in range(10):
                dist.all_reduce(x)
            torch.cuda.synchronize()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(a.reps):
                dist.all_reduce(x)
            torch.cuda.synchronize()
            rec["rccl_us"] = round((time.perf_counter() - t0) / a.reps * 1e6, 2)
        out[nbytes] = rec
    ar.check()
    ar.close()
    if comm.rank() == 0:
        print(json.dumps({"world": comm.world_size(), "per_call": out}), flush=True)


if __name__ == "__main__":
    main()
