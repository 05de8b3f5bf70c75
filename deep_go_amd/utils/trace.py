"""roctx ranges around the phases of a training step.

The reference only had wall-clock timers (train.lua:94,113,126).  Here each phase (loader
wait, H2D / input copy, forward+backward, gradient all-reduce wait, optimizer, validation,
checkpoint) can be bracketed by a roctx range, visible in
``rocprofv3 --marker-trace --kernel-trace`` timelines next to the HIP kernels.

Enabled with ``DG_ROCTX=1`` (or ``enable()``); otherwise ``range`` is a no-op context manager
with no library load and no per-call cost beyond a flag test.  The roctx library is the
rocprofiler-sdk one (``librocprofiler-sdk-roctx.so``), with the legacy ``libroctx64.so`` as
fallback; if neither loads, tracing silently stays off.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import time
from typing import Dict, Optional

_lib = None
_enabled = os.environ.get("DG_ROCTX", "0") == "1"
_totals: Dict[str, float] = {}
_timing = False


def _load():
    global _lib
    if _lib is not None:
        return _lib
    for name in ("/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", "/opt/rocm/lib/libroctx64.so",
                 "librocprofiler-sdk-roctx.so.1", "libroctx64.so"):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _lib = lib
            return lib
        except OSError:
            continue
    _lib = False
    return _lib


def enable(on: bool = True, host_timing: bool = False):
    """Turn roctx ranges on; host_timing also accumulates wall time per range name
    (``totals()``), for a quick phase breakdown without a profiler."""
    global _enabled, _timing
    _enabled = on
    _timing = host_timing


def enabled() -> bool:
    return _enabled


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors roctxRange naming
    if not _enabled:
        yield
        return
    lib = _load()
    t0 = time.perf_counter() if _timing else 0.0
    if lib:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib:
            lib.roctxRangePop()
        if _timing:
            _totals[name] = _totals.get(name, 0.0) + time.perf_counter() - t0


def mark(name: str):
    if _enabled:
        lib = _load()
        if lib:
            lib.roctxMarkA(name.encode())


def totals(reset: bool = False) -> Dict[str, float]:
    out = dict(_totals)
    if reset:
        _totals.clear()
    return out


def available() -> Optional[bool]:
    return bool(_load())
