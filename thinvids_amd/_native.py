"""ctypes bindings to the in-tree native libraries (``_lib/libtvcore.so``, ``_lib/libtvgpu.so``).

The libraries are built by :mod:`thinvids_amd._build` (``__graft_entry__.build()``).  On a
GPU box the GPU library is REQUIRED by the GPU engine: :func:`gpu_lib` raises instead of
falling back to anything else, so a missing build fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os
import threading
from pathlib import Path

import numpy as np

LIBDIR = Path(__file__).resolve().parent / "_lib"
_lock = threading.Lock()
_core = None
_gpu = None

u8p = C.POINTER(C.c_uint8)
i16p = C.POINTER(C.c_int16)
vp = C.c_void_p


def _which(name: str) -> str:
    return "core" if name == "libtvcore.so" else "gpu"


def _embedded_ok(path: Path, digest: str) -> bool:
    """The library's exported build hash (a string literal in .rodata) equals `digest`."""
    try:
        return digest.encode() in path.read_bytes()
    except OSError:
        return False


def _ensure_built(name: str) -> Path:
    """Return the library path, guaranteeing it was built from the CURRENT sources: the
    content hash embedded at link time must match the hash of csrc/ now.  A missing or
    stale library is rebuilt (TV_NO_AUTOBUILD=1: refused loudly instead)."""
    from . import _build

    path = LIBDIR / name
    have_src = (_build.CSRC / "core").is_dir()
    want = _build.expected_hash(_which(name)) if have_src else None
    if want is not None and not _embedded_ok(path, want):
        if os.environ.get("TV_NO_AUTOBUILD") == "1":
            state = "stale (built from other sources)" if path.exists() else "missing"
            raise RuntimeError(f"native library {path} is {state}; run `python -m thinvids_amd._build`")
        if name == "libtvcore.so":
            _build.build_core()
        else:
            _build.build_gpu()
        if not _embedded_ok(path, want):
            raise RuntimeError(f"native library {path} does not match the sources after a rebuild")
    if not path.exists():
        raise RuntimeError(f"native library {path} is missing; run `python -m thinvids_amd._build`")
    return path


def build_hash(lib, which: str) -> str:
    f = getattr(lib, f"tv_{which}_build_hash")
    f.restype = C.c_char_p
    return f().decode()


def _sig(lib, name, res, args):
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = args
    return f


def core_lib():
    global _core
    with _lock:
        if _core is None:
            lib = C.CDLL(str(_ensure_built("libtvcore.so")), mode=C.RTLD_GLOBAL)
            _sig(lib, "tv_last_error", C.c_char_p, [])
            _sig(lib, "tv_bytes_new", vp, [])
            _sig(lib, "tv_bytes_free", None, [vp])
            _sig(lib, "tv_bytes_size", C.c_size_t, [vp])
            _sig(lib, "tv_bytes_data", vp, [vp])
            _sig(lib, "tv_bytes_clear", None, [vp])
            _sig(lib, "tv_synth_frame", None, [C.c_uint32, C.c_int, C.c_int, C.c_int, u8p, u8p, u8p])
            _sig(lib, "tv_cpu_encoder_new", vp, [C.c_int] * 6)
            _sig(lib, "tv_cpu_encoder_free", None, [vp])
            _sig(lib, "tv_cpu_encoder_encode", C.c_int,
                 [vp, u8p, u8p, u8p, C.c_int, C.c_int, C.c_int, C.c_int, vp])
            _sig(lib, "tv_cpu_encoder_recon", None, [vp, u8p, u8p, u8p])
            _sig(lib, "tv_cpu_encoder_decisions", None, [vp, u8p, u8p, u8p, i16p, u8p])
            _sig(lib, "tv_reconstruct_frame", C.c_int,
                 [C.c_int] * 4 + [u8p] * 6 + [u8p, u8p, u8p, i16p, u8p, i16p, i16p, i16p, u8p, u8p, u8p])
            _sig(lib, "tv_write_frame", C.c_int,
                 [C.c_int] * 7 + [u8p, u8p, u8p, i16p, u8p, i16p, i16p, i16p, vp])
            _sig(lib, "tv_decoder_new", vp, [])
            _sig(lib, "tv_decoder_free", None, [vp])
            _sig(lib, "tv_decoder_decode", C.c_int, [vp, u8p, C.c_size_t])
            _sig(lib, "tv_decoder_info", None, [vp] + [C.POINTER(C.c_int)] * 5)
            _sig(lib, "tv_decoder_frame", C.c_int, [vp, C.c_int, C.c_int, u8p, u8p, u8p])
            _sig(lib, "tv_mux_mp4", C.c_int, [u8p, C.c_size_t, C.c_int, C.c_int, C.c_int, C.c_int, vp])
            _sig(lib, "tv_demux_mp4", C.c_int,
                 [u8p, C.c_size_t] + [C.POINTER(C.c_int)] * 5 + [vp])
            _core = lib
    return _core


def check(rc: int) -> None:
    if rc != 0:
        raise RuntimeError(core_lib().tv_last_error().decode())


def ptr(a: np.ndarray, t=u8p):
    assert a.flags["C_CONTIGUOUS"], "array must be C-contiguous"
    return a.ctypes.data_as(t)


class Bytes:
    """Owning handle around a native byte vector."""

    def __init__(self):
        self.lib = core_lib()
        self.h = self.lib.tv_bytes_new()

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.tv_bytes_free(self.h)
            self.h = None

    def tobytes(self) -> bytes:
        n = self.lib.tv_bytes_size(self.h)
        if n == 0:
            return b""
        return C.string_at(self.lib.tv_bytes_data(self.h), n)

    def clear(self) -> None:
        self.lib.tv_bytes_clear(self.h)


def gpu_lib():
    """Load libtvgpu.so (HIP kernels + GPU engine).  Raises if it cannot be loaded."""
    global _gpu
    core_lib()
    with _lock:
        if _gpu is None:
            _gpu = C.CDLL(str(_ensure_built("libtvgpu.so")), mode=C.RTLD_GLOBAL)
    return _gpu
