"""Native build driver: compiles the C++ core (g++) and the HIP/CDNA4 kernels (hipcc,
gfx950) into in-tree shared libraries under ``thinvids_amd/_lib``.

* ``libtvcore.so`` — CABAC/HEVC syntax writer, decoder oracle, CPU reference encoder,
  MP4 muxer, synthetic source (host C++17).
* ``libtvgpu.so``  — HIP kernels for gfx950 + the native GPU encode engine (streams,
  pinned ring buffers, entropy-coding thread pool); links ``libtvcore.so``.

Staleness is decided by CONTENT, not mtime: every object is keyed by the sha256 of its
source, every header it may include, the compiler flags and the target arch; each library
embeds the combined hash of its inputs (``tv_core_build_hash`` / ``tv_gpu_build_hash``)
and :mod:`thinvids_amd._native` refuses (or rebuilds) a library whose embedded hash does
not match the current sources, so a stale ``.so`` pushed with the tree can never stand in
for new kernels.  ``python -m thinvids_amd._build [--force]``.
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
CSRC = ROOT / "csrc"
INC = CSRC / "include"
LIBDIR = Path(__file__).resolve().parent / "_lib"
OBJDIR = ROOT / "build" / "obj"
GENDIR = ROOT / "build" / "gen"
ARCH = os.environ.get("TV_OFFLOAD_ARCH", "gfx950")

CXXFLAGS = ["-O2", "-std=c++17", "-fPIC", "-pthread", "-Wall", "-Wno-unused-function", f"-I{INC}"]
HIPFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", f"-I{INC}",
            "-Wno-unused-result", "-munsafe-fp-atomics", *os.environ.get("TV_HIPFLAGS_EXTRA", "").split()]
GPU_LINK = ["-L/opt/rocm/lib", "-lrocprofiler-sdk-roctx", "-lhsa-runtime64", "-Wl,-rpath,/opt/rocm/lib", "-lpthread"]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm required to build the gfx950 kernels)")


def _headers() -> list[Path]:
    return sorted(INC.rglob("*.h")) + sorted((CSRC / "core").glob("*.h")) + sorted((CSRC / "gpu").glob("*.h"))


def core_sources() -> list[Path]:
    return sorted((CSRC / "core").glob("*.cpp"))


def gpu_sources() -> list[Path]:
    return sorted((CSRC / "gpu").glob("*.hip")) + sorted((CSRC / "gpu").glob("*.cpp"))


def _digest(parts) -> str:
    h = hashlib.sha256()
    for p in parts:
        h.update(p if isinstance(p, bytes) else str(p).encode())
        h.update(b"\0")
    return h.hexdigest()


def _headers_digest() -> str:
    return _digest([p.relative_to(ROOT).as_posix().encode() + b":" + p.read_bytes() for p in _headers()])


def _obj_key(src: Path, flags: list[str], hdr: str) -> str:
    return _digest([src.read_bytes(), " ".join(flags).replace(str(ROOT), "<root>"), hdr])


def expected_hash(which: str) -> str:
    """Content hash the library `which` ('core' | 'gpu') must embed to be current."""
    hdr = _headers_digest()
    core = _digest([_obj_key(s, CXXFLAGS, hdr) for s in core_sources()])
    if which == "core":
        return core
    return _digest([core] + [_obj_key(s, HIPFLAGS, hdr) for s in gpu_sources()] + [ARCH])


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def _compile(src: Path, obj: Path, compiler: str, flags: list[str], key: str, force: bool) -> tuple[Path, bool]:
    stamp = obj.with_suffix(".key")
    if not force and obj.exists() and stamp.exists() and stamp.read_text() == key:
        return obj, False
    obj.parent.mkdir(parents=True, exist_ok=True)
    _run([compiler, *flags, "-c", str(src), "-o", str(obj)])
    stamp.write_text(key)
    return obj, True


def _stamp_obj(which: str, digest: str, compiler: str) -> Path:
    """A tiny object exporting the library's content hash."""
    GENDIR.mkdir(parents=True, exist_ok=True)
    src = GENDIR / f"stamp_{which}.cpp"
    src.write_text(f'extern "C" const char* tv_{which}_build_hash() {{ return "{digest}"; }}\n')
    obj = GENDIR / f"stamp_{which}.o"
    _run([compiler if which == "core" else "g++", "-O0", "-fPIC", "-c", str(src), "-o", str(obj)])
    return obj


def _lib_current(out: Path, digest: str) -> bool:
    stamp = out.with_suffix(".so.key")
    return out.exists() and stamp.exists() and stamp.read_text() == digest


def build_core(force: bool = False, jobs: int = 8) -> Path:
    hdr = _headers_digest()
    srcs = core_sources()
    out = LIBDIR / "libtvcore.so"
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, OBJDIR / "core" / (s.stem + ".o"), "g++", CXXFLAGS,
                                              _obj_key(s, CXXFLAGS, hdr), force), srcs))
    digest = expected_hash("core")
    if force or not _lib_current(out, digest):
        LIBDIR.mkdir(parents=True, exist_ok=True)
        stamp = _stamp_obj("core", digest, "g++")
        tmp = out.with_suffix(".so.tmp")
        _run(["g++", "-shared", "-pthread", "-o", str(tmp), *[str(o) for o, _ in objs], str(stamp)])
        os.replace(tmp, out)
        out.with_suffix(".so.key").write_text(digest)
    return out


def build_gpu(force: bool = False, jobs: int = 8) -> Path:
    hipcc = _hipcc()
    core = build_core(force, jobs)
    hdr = _headers_digest()
    srcs = gpu_sources()
    out = LIBDIR / "libtvgpu.so"
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, OBJDIR / "gpu" / (s.stem + ".o"), hipcc, HIPFLAGS,
                                              _obj_key(s, HIPFLAGS, hdr), force), srcs))
    digest = expected_hash("gpu")
    if force or not _lib_current(out, digest):
        stamp = _stamp_obj("gpu", digest, "g++")
        tmp = out.with_suffix(".so.tmp")
        _run([hipcc, "-shared", f"--offload-arch={ARCH}", "-fPIC", "-o", str(tmp), *[str(o) for o, _ in objs],
              str(stamp), f"-L{LIBDIR}", "-ltvcore", "-Wl,-rpath,$ORIGIN", *GPU_LINK])
        os.replace(tmp, out)
        out.with_suffix(".so.key").write_text(digest)
    del core
    return out


def build_all(force: bool = False) -> None:
    build_core(force)
    if gpu_sources():
        build_gpu(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
    print("built:", *sorted(p.name for p in LIBDIR.glob("*.so")))
