"""Loader for the in-tree native libraries (HIP kernels + host C++ runtime).

The HIP library is dlopened *after* ``import torch`` so that its ``libamdhip64.so.7`` dependency
resolves (by soname) to the HIP runtime torch already loaded: our kernels and torch's allocator,
streams and RCCL then share one runtime, and a torch stream handle can be passed straight to
``hipLaunchKernelGGL``.  Every entry point returns a ``hipError_t``; :func:`check` raises on
non-zero so a failed launch is never silent.
"""
from __future__ import annotations

import ctypes
import os
import re
import threading
from pathlib import Path

HERE = Path(__file__).resolve().parent
# PTG_CHECKED=1 loads the bounds-checked kernel build (build.py ``checked``): every launch is
# followed by a poll of the per-source-file check words, and a bad index raises with its line
CHECKED = os.environ.get("PTG_CHECKED") == "1"
HIP_LIB_PATH = HERE / ("libptg_hip_checked.so" if CHECKED else "libptg_hip.so")
if os.environ.get("PTG_HIP_LIB"):  # A/B runs: an in-tree variant build (tools/build_variant.sh)
    HIP_LIB_PATH = HERE / os.environ["PTG_HIP_LIB"]
_CHECK_TUS = ("conv", "gemm", "nn_eltwise", "bn", "df", "ml")
HOST_LIB_PATH = HERE / "libptg_host.so"

_lock = threading.Lock()
_hip = None
_host = None
_hip_err: str | None = None

P, I, L, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_float
_T = {"p": P, "i": I, "l": L, "f": F, "d": ctypes.c_double}

# Signatures are parsed from the extern "C" definitions in csrc/ (single source of truth):
# pointer / hipStream_t -> c_void_p, long -> c_long, float -> c_float, int -> c_int.
_SIG_RE = re.compile(r"^\s*int\s+(ptgh?_\w+)\s*\(([^)]*)\)\s*\{", re.M)


def _param_code(decl: str) -> str:
    d = decl.strip()
    if "*" in d or "hipStream_t" in d:
        return "p"
    if d.startswith("long") or d.startswith("int64_t") or d.startswith("size_t"):
        return "l"
    if d.startswith("float"):
        return "f"
    if d.startswith("double"):
        return "d"
    return "i"


def parse_sigs(paths) -> dict:
    sigs = {}
    for path in paths:
        text = Path(path).read_text()
        for m in _SIG_RE.finditer(text):
            params = [x for x in m.group(2).split(",") if x.strip() and x.strip() != "void"]
            sigs[m.group(1)] = "".join(_param_code(x) for x in params)
    return sigs


_CSRC = HERE.parent.parent / "csrc"


def _hip_sigs() -> dict:
    return parse_sigs(sorted((_CSRC / "kernels").glob("*.hip")))


def _host_sigs() -> dict:
    return parse_sigs(sorted((_CSRC / "host").glob("*.cpp")))


class NativeUnavailable(RuntimeError):
    pass


def _bind(lib, sigs):
    for name, codes in sigs.items():
        fn = getattr(lib, name, None)
        if fn is None:
            continue
        fn.argtypes = [_T[c] for c in codes]
        fn.restype = ctypes.c_int


def hip_lib():
    """Return the HIP kernel library, loading it on first use. Raises NativeUnavailable."""
    global _hip, _hip_err
    if _hip is not None:
        return _hip
    with _lock:
        if _hip is not None:
            return _hip
        import torch  # noqa: F401  (HIP runtime must come from torch)

        if not HIP_LIB_PATH.exists():
            _hip_err = f"{HIP_LIB_PATH} not built (run python -m pyspark_tf_gke_amd._native.build)"
            raise NativeUnavailable(_hip_err)
        lib = ctypes.CDLL(str(HIP_LIB_PATH), mode=ctypes.RTLD_GLOBAL)
        _bind(lib, _hip_sigs())
        _hip = lib
        return _hip


def host_lib():
    global _host
    if _host is not None:
        return _host
    with _lock:
        if _host is None:
            if not HOST_LIB_PATH.exists():
                raise NativeUnavailable(f"{HOST_LIB_PATH} not built")
            lib = ctypes.CDLL(str(HOST_LIB_PATH))
            _bind(lib, _host_sigs())
            _host = lib
    return _host


def host_available() -> bool:
    try:
        host_lib()
        return True
    except (NativeUnavailable, OSError):
        return False


def check(rc: int, name: str) -> None:
    if rc != 0:
        raise RuntimeError(f"native kernel {name} failed: hipError_t={rc}")


_FNS: dict = {}  # bound entry points by name (a ctypes attribute lookup per launch was measurable)


def call(name: str, *args) -> None:
    """Invoke a HIP entry point and raise on error."""
    fn = _FNS.get(name)
    if fn is None:
        fn = _FNS[name] = getattr(hip_lib(), name)
    rc = fn(*args)
    if rc:
        check(rc, name)
    if CHECKED:
        check_kernels(name)


def check_kernels(after: str = "") -> None:
    """Checked builds: raise if any kernel clamped an out-of-range index (file and line)."""
    lib = hip_lib()
    for tu in _CHECK_TUS:
        f = getattr(lib, "ptg_check_status_" + tu, None)
        if f is None:
            continue
        line = f()
        if line:
            raise RuntimeError(f"native kernel index out of bounds at csrc/kernels/{tu}.hip:{line}"
                               + (f" (detected after {after})" if after else ""))


def loaded_paths() -> list[str]:
    out = []
    if _hip is not None:
        out.append(str(HIP_LIB_PATH))
    if _host is not None:
        out.append(str(HOST_LIB_PATH))
    return out


def ensure_built(verbose: bool = False) -> None:
    """Build missing libraries in-tree (used by build()/tests on the CPU box)."""
    if os.environ.get("PTG_NO_AUTOBUILD"):
        return
    from . import build

    build.build_all(verbose=verbose)
