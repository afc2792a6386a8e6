"""Small helpers shared by the op wrappers: pointers, current stream, dtype checks."""
from __future__ import annotations

import torch

from .. import _native


def ptr(t: torch.Tensor | None) -> int | None:
    if t is None:
        return None
    return t.data_ptr()


# The current stream's raw handle straight from the C++ stream state (torch.cuda.current_stream()
# builds a Stream object through several Python device-index lookups: ~5 us per kernel launch, which
# made the CNN-B1 b32 step host-bound, tools/host_profile.py).  Same answer: torch.cuda.stream()
# contexts set that C++ state.
_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_CUR_DEVICE = getattr(torch._C, "_cuda_getDevice", None)


def stream_handle() -> int:
    if _RAW_STREAM is not None and _CUR_DEVICE is not None:
        return _RAW_STREAM(_CUR_DEVICE())
    return torch.cuda.current_stream().cuda_stream


def on_device(*ts) -> bool:
    """True when the op must run through the HIP kernels (any tensor on the GPU)."""
    return any(t is not None and t.is_cuda for t in ts)


def hip(name: str, *args) -> None:
    """Launch a HIP entry point on the current stream. Fails loudly if the library is missing."""
    _native.call(name, *args, stream_handle())


def need(t: torch.Tensor, dtype: torch.dtype, name: str) -> None:
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: tensor must be contiguous")
