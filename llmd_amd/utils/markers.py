"""roctx ranges around engine phases and kvx transfers (SURVEY §5.1 "Ours":
roctx ranges next to the kernels in rocprofv3 timelines; the reference has no
in-tree GPU profiler hooks).

Off unless ``LLMD_ROCTX=1`` (each range is two ctypes calls, ~1 µs). Then
``rocprofv3 --marker-trace --kernel-trace -- python ...`` shows
``llmd.schedule / llmd.plan / llmd.forward / llmd.sample / llmd.update`` per
engine step and ``llmd.kvx.pull <request>`` per KV transfer (rocprofiler-sdk roctx, the library rocprofv3 intercepts) (transfer threads
use start/stop ranges, which are not tied to a thread's push/pop stack).
"""
from __future__ import annotations

import contextlib
import ctypes
import os

_lib = None
_enabled = os.environ.get("LLMD_ROCTX", "0") == "1"


def _roctx():
    global _lib, _enabled
    if _lib is None:
        for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so.4"):
            for d in ("", "/opt/rocm/lib/"):
                try:
                    _lib = ctypes.CDLL(d + name)
                    break
                except OSError:
                    continue
            if _lib is not None:
                break
        if _lib is None:
            _enabled = False
            return None
        _lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
        _lib.roctxRangeStartA.argtypes = [ctypes.c_char_p]
        _lib.roctxRangeStartA.restype = ctypes.c_uint64
        _lib.roctxRangeStop.argtypes = [ctypes.c_uint64]
    return _lib


def enabled() -> bool:
    return _enabled


def set_enabled(on: bool):
    global _enabled
    _enabled = bool(on)


@contextlib.contextmanager
def range(name: str):  # noqa: A001 - mirrors roctx naming
    """Nested push/pop range on the calling thread."""
    lib = _roctx() if _enabled else None
    if lib is None:
        yield
        return
    lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        lib.roctxRangePop()


def start(name: str) -> int:
    """Process-wide range (any thread may stop it); 0 when disabled."""
    lib = _roctx() if _enabled else None
    return int(lib.roctxRangeStartA(name.encode())) if lib is not None else 0


def stop(rid: int):
    if rid and _lib is not None:
        _lib.roctxRangeStop(rid)
