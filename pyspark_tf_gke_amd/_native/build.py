"""In-tree build of the native libraries.

* ``libptg_hip.so``  — every HIP kernel under ``csrc/kernels`` compiled for gfx950 with hipcc
  (``--offload-arch=gfx950``), one object per translation unit, linked into one shared object.
* ``libptg_host.so`` — the host C++ runtime under ``csrc/host`` (CSV tokenizer / type inference,
  hash aggregation for the CPU ``local[N]`` path, word tokenizer, image batch assembly).

Both land next to this file so they travel with a ``gpurun`` snapshot and are what the Python
process dlopens (no site-packages install, no JIT cache). Objects are rebuilt only when a source
or header is newer than the object.

Usage: ``python -m pyspark_tf_gke_amd._native.build [--force] [-j N]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
ROOT = HERE.parent.parent
CSRC = ROOT / "csrc"
BUILD = ROOT / "build" / "native"
ARCH = os.environ.get("PTG_OFFLOAD_ARCH", "gfx950")

HIP_LIB = HERE / "libptg_hip.so"
HIP_LIB_CHECKED = HERE / "libptg_hip_checked.so"  # -DPTG_CHECKED: index-checked kernels (PTG_CHECKED=1)
HOST_LIB = HERE / "libptg_host.so"


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (need ROCm at /opt/rocm)")


def _newest_dep(src: Path, headers: list[Path]) -> float:
    t = src.stat().st_mtime
    for h in headers:
        t = max(t, h.stat().st_mtime)
    return t


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def build_hip(force: bool = False, jobs: int = 8, verbose: bool = True, checked: bool = False,
              variant: str | None = None, defines: tuple = ()) -> Path:
    """``checked``: the bounds-checked variant - every PTG_CHECKED_IDX site verifies its
    index, clamps it in range and reports the source line instead of faulting.
    ``variant``/``defines``: an A/B build ``libptg_hip_<variant>.so`` with extra -D macros, loaded by
    setting ``PTG_HIP_LIB=libptg_hip_<variant>.so`` (not part of the default tree)."""
    srcs = sorted((CSRC / "kernels").glob("*.hip"))
    headers = sorted((CSRC / "kernels").glob("*.h"))
    bdir = BUILD / ("checked" if checked else f"var_{variant}" if variant else "")
    out_lib = HIP_LIB_CHECKED if checked else (HERE / f"libptg_hip_{variant}.so" if variant else HIP_LIB)
    bdir.mkdir(parents=True, exist_ok=True)
    hipcc = _hipcc()
    flags = ["--offload-arch=" + ARCH, "-O3", "-fPIC", "-std=c++17", "-munsafe-fp-atomics",
             "-Wno-unused-result", "-I", str(CSRC / "kernels")] + (["-DPTG_CHECKED"] if checked else [])
    flags += [f"-D{d}" for d in defines]
    if not force and out_lib.exists() and srcs and \
            out_lib.stat().st_mtime >= max(_newest_dep(s, headers) for s in srcs):
        return out_lib  # up to date (objects need not exist: a snapshot ships only the library)
    objs, todo = [], []
    for s in srcs:
        o = bdir / (s.stem + ".o")
        objs.append(o)
        if force or not o.exists() or o.stat().st_mtime < _newest_dep(s, headers):
            todo.append((s, o))

    def compile_one(so):
        s, o = so
        if verbose:
            print(f"[build] hipcc {s.name}" + (" (checked)" if checked else ""), flush=True)
        _run([hipcc, *flags, "-c", str(s), "-o", str(o)])
        return o

    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        list(ex.map(compile_one, todo))
    if force or todo or not out_lib.exists() or any(out_lib.stat().st_mtime < o.stat().st_mtime for o in objs):
        tmp = out_lib.with_suffix(".so.tmp")
        _run([hipcc, "--offload-arch=" + ARCH, "-shared", "-fPIC", *map(str, objs), "-o", str(tmp)])
        os.replace(tmp, out_lib)
        if verbose:
            print(f"[build] linked {out_lib}", flush=True)
    return out_lib


def build_host(force: bool = False, verbose: bool = True) -> Path:
    srcs = sorted((CSRC / "host").glob("*.cpp"))
    headers = sorted((CSRC / "host").glob("*.h"))
    if not srcs:
        return HOST_LIB
    newest = max(_newest_dep(s, headers) for s in srcs)
    if not force and HOST_LIB.exists() and HOST_LIB.stat().st_mtime >= newest:
        return HOST_LIB
    cxx = shutil.which("g++") or "g++"
    tmp = HOST_LIB.with_suffix(".so.tmp")
    cmd = [cxx, "-O3", "-march=x86-64-v2", "-std=c++17", "-shared", "-fPIC", "-pthread",
           "-I", str(CSRC / "host"), *map(str, srcs), "-o", str(tmp)]
    if os.environ.get("PTG_HOST_ASAN"):  # sanitizer build of the host runtime
        cmd[1:1] = ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-g"]
    if verbose:
        print(f"[build] g++ {' '.join(s.name for s in srcs)}", flush=True)
    _run(cmd)
    os.replace(tmp, HOST_LIB)
    return HOST_LIB


def build_all(force: bool = False, jobs: int = 8, verbose: bool = True) -> None:
    build_host(force=force, verbose=verbose)
    build_hip(force=force, jobs=jobs, verbose=verbose)
    if os.environ.get("PTG_BUILD_CHECKED", "1") != "0":
        build_hip(force=force, jobs=jobs, verbose=verbose, checked=True)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=min(8, os.cpu_count() or 4))
    ap.add_argument("--host-only", action="store_true")
    ap.add_argument("--variant", help="A/B build name (libptg_hip_<variant>.so)")
    ap.add_argument("-D", dest="defines", action="append", default=[], help="extra macro for --variant")
    a = ap.parse_args(argv)
    if a.variant:
        build_hip(force=a.force, jobs=a.jobs, variant=a.variant, defines=tuple(a.defines))
    elif a.host_only:
        build_host(force=a.force)
    else:
        build_all(force=a.force, jobs=a.jobs)
    return 0


if __name__ == "__main__":
    sys.exit(main())
