"""Pipeline tracing.

The reference times its stages ad hoc: ``completed in {N}ms`` activity messages
(worker/tasks.py:1090, :1268, :1679, :1723), stage ``*_elapsed`` fields and ffmpeg
``-progress`` parsing.  Here every pipeline stage is a :func:`span`:

* with ``TV_ROCTX=1`` (or under ``rocprofv3 --marker-trace``) each span is also a ROCTx
  range (``librocprofiler-sdk-roctx``), so host stages line up with the HIP kernels of the
  same process in the rocprofv3 timeline; the native engine emits its own per-frame
  ranges (csrc/gpu/engine.hip);
* every span is accumulated in a per-process registry (:func:`summary`: count / total /
  max ms per name) that the worker publishes into the job hash and the agent exposes;
* ``TV_TRACE_FILE=path.json`` additionally writes Chrome trace events (chrome://tracing /
  Perfetto) at exit, one track per thread.
"""
from __future__ import annotations

import atexit
import contextlib
import ctypes
import json
import os
import threading
import time

_lock = threading.Lock()
_stats: dict[str, list] = {}  # name -> [count, total_ms, max_ms]
_events: list = []
_roctx = None
_roctx_tried = False


def _roctx_lib():
    global _roctx, _roctx_tried
    if _roctx_tried:
        return _roctx
    _roctx_tried = True
    if os.environ.get("TV_ROCTX", "0") != "1":
        return None
    for name in ("librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so", "libroctx64.so"):
        for d in ("", "/opt/rocm/lib/"):
            try:
                lib = ctypes.CDLL(d + name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                lib.roctxMarkA.argtypes = [ctypes.c_char_p]
                _roctx = lib
                return lib
            except OSError:
                continue
    return None


@contextlib.contextmanager
def span(name: str, **args):
    """Time a stage; also a ROCTx range when enabled."""
    lib = _roctx_lib()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    t0 = time.perf_counter()
    try:
        yield
    finally:
        dt = (time.perf_counter() - t0) * 1000.0
        if lib is not None:
            lib.roctxRangePop()
        with _lock:
            s = _stats.setdefault(name, [0, 0.0, 0.0])
            s[0] += 1
            s[1] += dt
            s[2] = max(s[2], dt)
            if _trace_file():
                _events.append({"name": name, "ph": "X", "ts": t0 * 1e6, "dur": dt * 1000.0, "pid": os.getpid(),
                                "tid": threading.get_ident() % 100000, "args": args})


def mark(name: str) -> None:
    lib = _roctx_lib()
    if lib is not None:
        lib.roctxMarkA(name.encode())
    if _trace_file():
        with _lock:
            _events.append({"name": name, "ph": "i", "ts": time.perf_counter() * 1e6, "pid": os.getpid(),
                            "tid": threading.get_ident() % 100000, "s": "t"})


def summary(reset: bool = False) -> dict:
    """{name: {"count", "total_ms", "max_ms", "avg_ms"}} of the spans so far."""
    with _lock:
        out = {k: {"count": c, "total_ms": round(t, 3), "max_ms": round(m, 3), "avg_ms": round(t / max(c, 1), 3)}
               for k, (c, t, m) in _stats.items()}
        if reset:
            _stats.clear()
    return out


def since(before: dict) -> dict:
    """The spans recorded after the :func:`summary` snapshot `before` (count / total per
    name; max_ms is over the whole process)."""
    out = {}
    for k, v in summary().items():
        b = before.get(k, {"count": 0, "total_ms": 0.0})
        c, t = v["count"] - b["count"], round(v["total_ms"] - b["total_ms"], 3)
        if c > 0:
            out[k] = {"count": c, "total_ms": t, "max_ms": v["max_ms"], "avg_ms": round(t / c, 3)}
    return out


def _trace_file() -> str | None:
    return os.environ.get("TV_TRACE_FILE")


def flush(path: str | None = None) -> str | None:
    path = path or _trace_file()
    if not path:
        return None
    with _lock:
        ev = list(_events)
    tmp = f"{path}.{os.getpid()}.tmp"
    with open(tmp, "w") as f:
        json.dump({"traceEvents": ev, "displayTimeUnit": "ms"}, f)
    os.replace(tmp, path)
    return path


atexit.register(lambda: flush() if _trace_file() else None)
