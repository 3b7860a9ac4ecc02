"""Native build driver: compiles the C++ core (g++) and the HIP/CDNA4 kernels (hipcc,
gfx950) into in-tree shared libraries under ``thinvids_amd/_lib``.

* ``libtvcore.so`` — CABAC/HEVC syntax writer, decoder oracle, CPU reference encoder,
  MP4 muxer, synthetic source (host C++17).
* ``libtvgpu.so``  — HIP kernels for gfx950 + the native GPU encode engine (streams,
  pinned ring buffers, entropy-coding thread pool); links ``libtvcore.so``.

Incremental (mtime based) and parallel.  ``python -m thinvids_amd._build [--force]``.
"""
from __future__ import annotations

import concurrent.futures as cf
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
ARCH = os.environ.get("TV_OFFLOAD_ARCH", "gfx950")

CXXFLAGS = ["-O2", "-std=c++17", "-fPIC", "-pthread", "-Wall", "-Wno-unused-function", f"-I{INC}"]
HIPFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", f"-I{INC}",
            "-Wno-unused-result", "-munsafe-fp-atomics", *os.environ.get("TV_HIPFLAGS_EXTRA", "").split()]


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm required to build the gfx950 kernels)")


def _headers() -> list[Path]:
    return sorted(INC.rglob("*.h")) + sorted((CSRC / "gpu").glob("*.h"))


def _stale(target: Path, deps: list[Path]) -> bool:
    if not target.exists():
        return True
    t = target.stat().st_mtime
    return any(d.stat().st_mtime > t for d in deps)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"build failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")


def _compile(src: Path, obj: Path, compiler: str, flags: list[str], force: bool) -> Path:
    if force or _stale(obj, [src] + _headers()):
        obj.parent.mkdir(parents=True, exist_ok=True)
        _run([compiler, *flags, "-c", str(src), "-o", str(obj)])
    return obj


def build_core(force: bool = False, jobs: int = 8) -> Path:
    srcs = sorted((CSRC / "core").glob("*.cpp"))
    out = LIBDIR / "libtvcore.so"
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, OBJDIR / "core" / (s.stem + ".o"), "g++", CXXFLAGS, force), srcs))
    if force or _stale(out, objs):
        LIBDIR.mkdir(parents=True, exist_ok=True)
        _run(["g++", "-shared", "-pthread", "-o", str(out), *map(str, objs)])
    return out


def build_gpu(force: bool = False, jobs: int = 8) -> Path:
    hipcc = _hipcc()
    core = build_core(force, jobs)
    srcs = sorted((CSRC / "gpu").glob("*.hip")) + sorted((CSRC / "gpu").glob("*.cpp"))
    out = LIBDIR / "libtvgpu.so"
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, OBJDIR / "gpu" / (s.stem + ".o"), hipcc, HIPFLAGS, force), srcs))
    if force or _stale(out, objs + [core]):
        _run([hipcc, "-shared", f"--offload-arch={ARCH}", "-fPIC", "-o", str(out), *map(str, objs),
              f"-L{LIBDIR}", "-ltvcore", "-Wl,-rpath,$ORIGIN", "-L/opt/rocm/lib", "-lrocprofiler-sdk-roctx",
              "-Wl,-rpath,/opt/rocm/lib", "-lpthread"])
    return out


def build_all(force: bool = False) -> None:
    build_core(force)
    if list((CSRC / "gpu").glob("*.hip")):
        build_gpu(force)


if __name__ == "__main__":
    build_all(force="--force" in sys.argv)
    print("built:", *sorted(p.name for p in LIBDIR.glob("*.so")))
