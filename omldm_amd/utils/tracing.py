"""Tracing / profiling hooks (the reference has println only).

* ``range(name)`` — a roctx range (visible in ``rocprofv3 --marker-trace`` timelines)
  when the ROCm roctx library is loadable, plus a host wall-clock accumulator per stage
  that ``report()`` returns (exported in the job statistics).
* Enabled by default; ``OMLDM_TRACE=0`` disables both.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import time
from collections import defaultdict

_ENABLED = os.environ.get("OMLDM_TRACE", "1") != "0"
_roctx = None
_stats = defaultdict(lambda: [0, 0.0])


def _load_roctx():
    global _roctx
    if _roctx is not None:
        return _roctx
    _roctx = False
    for name in ("librocprofiler-sdk-roctx.so", "libroctx64.so",
                 "/opt/rocm/lib/librocprofiler-sdk-roctx.so", "/opt/rocm/lib/libroctx64.so"):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            _roctx = lib
            break
        except (OSError, AttributeError):
            continue
    return _roctx


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors the roctx API name
    if not _ENABLED:
        yield
        return
    lib = _load_roctx()
    if lib:
        lib.roctxRangePushA(name.encode())
    t = time.perf_counter()
    try:
        yield
    finally:
        dt = time.perf_counter() - t
        if lib:
            lib.roctxRangePop()
        s = _stats[name.split(":")[0]]
        s[0] += 1
        s[1] += dt


def report() -> dict:
    return {k: {"calls": v[0], "host_ms": round(v[1] * 1e3, 3)} for k, v in _stats.items()}


def reset() -> None:
    _stats.clear()
