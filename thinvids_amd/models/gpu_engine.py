"""GPU encode engine (libtvgpu.so): batched HEVC encoding of GOP-aligned segments on one
MI355X.  One instance per process/GPU; see csrc/gpu/engine.hip.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

from .._native import gpu_lib, ptr
from .hevc import coded_size

_sigs_done = False


def _lib():
    global _sigs_done
    lib = gpu_lib()
    if not _sigs_done:
        vp = C.c_void_p
        lib.tv_gpu_last_error.restype = C.c_char_p
        lib.tv_gpu_device_count.restype = C.c_int
        lib.tv_engine_new.restype = vp
        lib.tv_engine_new.argtypes = [C.c_int] * 7 + [C.c_uint32, C.c_int, C.c_int, C.c_int, C.c_int]
        lib.tv_engine_new_b.restype = vp
        lib.tv_engine_new_b.argtypes = [C.c_int] * 7 + [C.c_uint32, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int]
        lib.tv_engine_free.argtypes = [vp]
        lib.tv_engine_encode_synth.restype = C.c_int
        lib.tv_engine_encode_synth.argtypes = [vp, C.POINTER(C.c_int), C.c_int, C.c_int, vp]
        lib.tv_engine_encode_host.restype = C.c_int
        lib.tv_engine_encode_host.argtypes = [vp, C.POINTER(C.c_uint8), C.c_int, C.c_int, vp]
        lib.tv_engine_encode_device.restype = C.c_int
        lib.tv_engine_encode_device.argtypes = [vp, vp, C.c_int, C.c_int, vp]
        lib.tv_engine_segment_size.restype = C.c_size_t
        lib.tv_engine_segment_size.argtypes = [vp, C.c_int]
        lib.tv_engine_segment_copy.argtypes = [vp, C.c_int, C.POINTER(C.c_uint8)]
        lib.tv_engine_sse.argtypes = [vp, C.c_int, C.POINTER(C.c_double)]
        lib.tv_engine_timing.argtypes = [vp] + [C.POINTER(C.c_double)] * 4
        lib.tv_engine_last_recon.restype = C.c_int
        lib.tv_engine_last_recon.argtypes = [vp, C.c_int] + [C.POINTER(C.c_uint8)] * 3
        _sigs_done = True
    return lib


def device_count() -> int:
    return _lib().tv_gpu_device_count()


def cgroup_cpu_quota() -> float | None:
    """CPUs this process may use per the cgroup (v2 cpu.max, v1 cfs quota), or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def default_threads() -> int:
    """CABAC pool size: 1.5 x the CPUs this rank may use (affinity, capped by the cgroup
    quota), at most 32.  Slices block briefly on the slot ring and the D2H fetch, so a pool
    the size of the quota leaves it idle (measured on a 16-CPU-quota MI355X box: 8 threads
    3880 frames/s, 16 threads ~6050, 24 threads 6250-6660 with all 16 CPUs busy)."""
    env = os.environ.get("TV_THREADS")
    if env:
        return max(1, int(env))
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        n = os.cpu_count() or 4
    q = cgroup_cpu_quota()
    cpus = min(n, q) if q else n
    return max(2, min(32, int(cpus * 1.5)))


class GpuEngine:
    def __init__(self, width: int, height: int, qp: int = 27, batch: int = 8, gop: int = 16,
                 search_range: int = 64, deblock: bool = True, sao: bool = False, seed: int = 1,
                 threads: int | None = None,
                 device: int = 0, max_merge: int = 5, crf: int = 0, bframes: int = 1, wpp: bool = True,
                 rqt: bool = True, pintra: bool = True, entropy: str | None = None, cascade: bool = True,
                 rdoq: bool = True):
        """`bframes` > 1: hierarchical-B mini-GOPs of that size (power of 2, tv/gop.h); the
        segments' streams are then in coding order (the decoder reorders by POC) and
        :meth:`last_recon` returns the last DISPLAY frame.

        `wpp` (default): one CABAC substream per CTB row.  `entropy` (same bytes either way):
        "gpu" codes them ON THE GPU (csrc/gpu/k_entropy.hip; the host only writes slice
        headers and entry points), "host" with the C++ CABAC writer on the thread pool, "auto"
        (default; env TV_ENTROPY) picks by the host CPU budget (:func:`auto_entropy`).
        wpp=False always codes on the host."""
        self.lib = _lib()
        self.width, self.height, self.qp = width, height, qp
        self.batch, self.gop = batch, gop
        self.cw, self.ch = coded_size(width, height)
        self.threads = threads or default_threads()
        self.sao = sao
        self.device = device
        self.bframes = int(bframes)
        from .hevc import codec_flags

        self.entropy = resolve_entropy(entropy) if wpp else "host"
        self.flags = codec_flags(deblock, sao, wpp, rqt, pintra, cascade, rdoq) | (32 if self.entropy == "host" else 0)
        self.h = self.lib.tv_engine_new_b(width, height, qp, batch, gop, search_range, self.flags,
                                          seed & 0xFFFFFFFF, self.threads, device, max_merge, int(crf), self.bframes)
        if not self.h:
            raise RuntimeError("GPU engine init failed: " + self.lib.tv_gpu_last_error().decode())

    def close(self):
        if getattr(self, "h", None):
            self.lib.tv_engine_free(self.h)
            self.h = None

    __del__ = close

    def _qmap(self, qp, nseg: int, nframes: int):
        """None -> sequence QP; int -> that QP everywhere; array -> [nseg][nframes] slice QPs."""
        if qp is None:
            self._qbuf = None
            return None
        q = np.asarray(qp)
        q = np.broadcast_to(q, (nseg, nframes)) if q.ndim < 2 else q
        if q.shape != (nseg, nframes) or (q < 0).any() or (q > 51).any():
            raise ValueError(f"qp map must be [{nseg}][{nframes}] in 0..51")
        self._qbuf = np.ascontiguousarray(q, dtype=np.int8)
        self.last_qp = self._qbuf
        return C.c_void_p(self._qbuf.ctypes.data)

    def _check(self, rc):
        if rc != 0:
            raise RuntimeError(self.lib.tv_gpu_last_error().decode())

    def encode_synthetic(self, starts, nframes: int | None = None, qp=None) -> list[bytes]:
        """Encode len(starts) segments generated on the GPU; segment b = synthetic frames
        [starts[b], starts[b] + nframes) (nframes defaults to the GOP).  `qp`: rate-control
        slice QPs (int or [nseg][nframes])."""
        n = self.gop if nframes is None else int(nframes)
        if not 1 <= n <= self.gop or not 1 <= len(starts) <= self.batch:
            raise ValueError(f"need 1..{self.batch} segments of 1..{self.gop} frames")
        arr = (C.c_int * len(starts))(*[int(s) for s in starts])
        self._check(self.lib.tv_engine_encode_synth(self.h, arr, len(starts), n, self._qmap(qp, len(starts), n)))
        self.last_frames = n
        return [self.segment(b) for b in range(len(starts))]

    def encode_frames(self, segments, qp=None) -> list[bytes]:
        """segments: list (<= batch) of equally long lists (1..gop) of display-size (Y, U, V)
        frames; each segment becomes one closed GOP (IDR + P frames)."""
        n = len(segments[0]) if segments else 0
        if not segments or len(segments) > self.batch:
            raise ValueError(f"need 1..{self.batch} segments")
        if not 1 <= n <= self.gop or any(len(s) != n for s in segments):
            raise ValueError(f"segments must all have the same length in 1..{self.gop}")
        # one pinned upload per segment, edge padding to the coded size on the GPU
        import torch

        from ..ops import stage

        dev = torch.device("cuda", self.device)
        fsz = self.cw * self.ch * 3 // 2
        staging = torch.empty(len(segments) * n * fsz, dtype=torch.uint8, device=dev)
        for b, seg in enumerate(segments):
            stage.to_staging(stage.upload_frames(seg, dev), self.width, self.height, staging, b * n)
        torch.cuda.current_stream(dev).synchronize()
        return self.encode_device(staging, len(segments), n, qp=qp)

    def encode_device(self, frames, nseg: int, nframes: int, qp=None) -> list[bytes]:
        """frames: a contiguous uint8 CUDA tensor on this engine's GPU laid out
        [segment][frame][Y | U | V] at the coded size (edge-padded), already written (the
        producing stream synchronised).  Copied device-to-device into the engine."""
        fsz = self.cw * self.ch * 3 // 2
        if not 1 <= nseg <= self.batch or not 1 <= nframes <= self.gop:
            raise ValueError(f"need 1..{self.batch} segments of 1..{self.gop} frames")
        if not frames.is_cuda or not frames.is_contiguous() or frames.numel() * frames.element_size() < nseg * nframes * fsz:
            raise ValueError("frames must be a contiguous CUDA tensor of nseg*nframes coded-size I420 frames")
        self._check(self.lib.tv_engine_encode_device(self.h, C.c_void_p(frames.data_ptr()), nseg, nframes,
                                                     self._qmap(qp, nseg, nframes)))
        self.last_frames = nframes
        return [self.segment(b) for b in range(nseg)]

    def segment(self, b: int) -> bytes:
        n = self.lib.tv_engine_segment_size(self.h, b)
        out = np.empty(n, np.uint8)
        self.lib.tv_engine_segment_copy(self.h, b, ptr(out))
        return out.tobytes()

    def footprint(self) -> dict:
        """HBM and pinned-host bytes this engine allocated (the native allocation ledger)."""
        d, h = C.c_ulonglong(), C.c_ulonglong()
        self.lib.tv_engine_footprint.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong), C.POINTER(C.c_ulonglong)]
        self.lib.tv_engine_footprint(self.h, C.byref(d), C.byref(h))
        return {"dev": int(d.value), "host": int(h.value)}

    def sse(self, b: int) -> tuple[float, float, float]:
        a = (C.c_double * 3)()
        self.lib.tv_engine_sse(self.h, b, a)
        return a[0], a[1], a[2]

    def psnr(self, b: int) -> dict:
        y, u, v = self.sse(b)
        npx = self.width * self.height * getattr(self, "last_frames", self.gop)
        f = lambda s, n: float("inf") if s == 0 else 10 * np.log10(255.0 ** 2 * n / s)
        py, pu, pv = f(y, npx), f(u, npx / 4), f(v, npx / 4)
        return {"y": py, "u": pu, "v": pv, "yuv": (6 * py + pu + pv) / 8}

    def timing(self) -> dict:
        """Last encode call: GPU stream time, engine wall time, summed CPU entropy-coding
        time (all threads), and compact level bytes transferred device->host."""
        g, w, e, m = C.c_double(), C.c_double(), C.c_double(), C.c_double()
        self.lib.tv_engine_timing(self.h, C.byref(g), C.byref(w), C.byref(e), C.byref(m))
        return {"gpu_ms": g.value, "wall_ms": w.value, "entropy_cpu_ms": e.value, "coef_mb": m.value}

    def entropy_stats(self) -> dict:
        """GPU entropy coding: whether it is on, pictures the host writer coded instead since
        construction (device capacity), and the OR of their device status words."""
        on, fb, st = C.c_int(), C.c_longlong(), C.c_int()
        f = self.lib.tv_engine_entropy_stats
        f.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_longlong), C.POINTER(C.c_int)]
        f(self.h, C.byref(on), C.byref(fb), C.byref(st))
        hp = self.lib.tv_engine_entropy_host_pictures
        hp.argtypes, hp.restype = [C.c_void_p], C.c_longlong
        lp = self.lib.tv_engine_entropy_lane_pictures
        lp.argtypes, lp.restype = [C.c_void_p, C.c_int], C.c_longlong
        return {"gpu": bool(on.value), "fallbacks": int(fb.value), "status": int(st.value),
                "host_pictures": int(hp(self.h)), "lane_pictures": [int(lp(self.h, l)) for l in range(2)]}

    def last_recon(self, b: int):
        y = np.empty((self.ch, self.cw), np.uint8)
        u = np.empty((self.ch // 2, self.cw // 2), np.uint8)
        v = np.empty_like(u)
        self._check(self.lib.tv_engine_last_recon(self.h, b, ptr(y), ptr(u), ptr(v)))
        return y, u, v


def pad_frame(y, u, v, cw, ch) -> np.ndarray:
    """Edge-replicate a display-size I420 frame to the coded size; returns flat Y|U|V."""
    h, w = y.shape
    Y = np.pad(y, ((0, ch - h), (0, cw - w)), mode="edge")
    U = np.pad(u, ((0, ch // 2 - h // 2), (0, cw // 2 - w // 2)), mode="edge")
    V = np.pad(v, ((0, ch // 2 - h // 2), (0, cw // 2 - w // 2)), mode="edge")
    return np.concatenate([Y.ravel(), U.ravel(), V.ravel()])


def auto_entropy(cpus: int | None = None) -> str:
    """Where WPP substreams are CABAC-coded when nobody asked: the host writer costs ~1 core
    per 1000 frames/s of 1080p (8.4 busy cores at the 1080p bench rate, ~15 on grainy
    content) and leaves the GPU at its full analysis rate; the GPU coder frees the host (1.4
    busy cores) for a ~12 % longer GPU step (profiles/README.md, round 5).  A process with at
    least TV_ENT_AUTO_CPUS (12) CPUs in its affinity set -- one rank's share of an 8-GPU,
    128-CPU node is 16 -- codes on the host, a smaller share on the GPU."""
    n = cpus if cpus is not None else len(os.sched_getaffinity(0))
    return "host" if n >= int(os.environ.get("TV_ENT_AUTO_CPUS", "12")) else "gpu"


def resolve_entropy(entropy: str | None = None) -> str:
    e = entropy or os.environ.get("TV_ENTROPY", "auto")
    if e == "auto":
        e = auto_entropy()
    if e not in ("gpu", "host"):
        raise ValueError("entropy must be 'gpu', 'host' or 'auto'")
    return e


def estimate_footprint(width: int, height: int, batch: int, gop: int, sao: bool = False, bframes: int = 1,
                       wpp: bool = True, rqt: bool = True, pintra: bool = True, entropy: str | None = None,
                       cascade: bool = True, rdoq: bool = True) -> dict:
    """HBM / pinned-host bytes an engine of this geometry would allocate, computed by the
    native constructor's own size formulas without allocating (tv_engine_estimate)."""
    from .hevc import codec_flags

    lib = _lib()
    ent = resolve_entropy(entropy) if wpp else "host"
    flags = codec_flags(True, sao, wpp, rqt, pintra, cascade, rdoq) | (32 if ent == "host" else 0)
    d, h = C.c_ulonglong(), C.c_ulonglong()
    f = lib.tv_engine_estimate
    f.argtypes = [C.c_int] * 6 + [C.POINTER(C.c_ulonglong)] * 2
    if f(width, height, batch, gop, flags, int(bframes), C.byref(d), C.byref(h)) != 0:
        raise ValueError(lib.tv_gpu_last_error().decode())
    return {"dev": int(d.value), "host": int(h.value)}
