"""Device staging: job sources -> encode-engine input without host bounces.

A segment's frames reach the GPU exactly once — uploaded from a pinned buffer (file
sources), received over RCCL (node scatter), or generated on the device (synthetic
sources, SURVEY §2.2 P5 direct source) — and every further step runs on the device:

    DevFrames (display size, 8-bit I420 or 10-bit planar PQ)
      -> [tone-map PQ -> SDR]      (HDR10 sources, k_tonemap_pq)
      -> Lanczos resize / edge pad (k_resize2d / k_pad_plane)
      -> engine staging            coded-size [segment][frame][Y | U | V]
      -> GpuEngine.encode_device   D2D into the engine

Reference analogue: the ffmpeg filter chain `bwdif,scale=-2:H,format=nv12,hwupload` in
front of h264_vaapi (reference worker/tasks.py:436-461, :1573-1586).
"""
from __future__ import annotations

import ctypes as C
import threading
from dataclasses import dataclass, field

import numpy as np

from ..models.hevc import coded_size


def _lib():
    from .._native import gpu_lib

    lib = gpu_lib()
    if not getattr(lib, "_stage_sigs", False):
        vp, ci, cl = C.c_void_p, C.c_int, C.c_long
        lib.tv_pad_batch.argtypes = [vp, ci, ci, ci, cl, vp, ci, ci, ci, cl, ci, vp]
        lib.tv_synth_batch.argtypes = [vp, ci, ci, ci, C.POINTER(C.c_int), C.c_uint32, vp]
        lib.tv_stage_last_error.restype = C.c_char_p
        lib.tv_resize_batch.argtypes = [vp, ci, ci, ci, cl, vp, ci, ci, ci, cl, ci, ci, ci,
                                        vp, vp, ci, vp, vp, ci, vp, ci, ci, ci, vp]
        lib.tv_tonemap_pq_batch.argtypes = [vp, vp, ci, ci, ci, vp, C.c_float, C.c_float, vp]
        lib.tv_ops_last_error.restype = C.c_char_p
        lib.tv_thumbs8_batch.argtypes = [vp, ci, ci, ci, ci, cl, ci, vp, vp]
        lib._stage_sigs = True
    return lib


def _ok(rc: int, which: str = "stage") -> None:
    if rc != 0:
        lib = _lib()
        msg = lib.tv_stage_last_error() if which == "stage" else lib.tv_ops_last_error()
        raise RuntimeError(msg.decode())


@dataclass
class DevFrames:
    """n frames resident on one GPU.  `planes[c]` = (element offset, width, height, row
    stride, frame stride) of plane c inside `buf` (uint8, or int16 holding 0..1023 when
    bits == 10)."""
    buf: object
    n: int
    w: int
    h: int
    planes: list
    bits: int = 8
    keep: list = field(default_factory=list)  # tensors that must outlive the async work

    def ptr(self, c: int) -> int:
        return self.buf.data_ptr() + self.planes[c][0] * self.buf.element_size()

    def select(self, f0: int, n: int) -> "DevFrames":
        """Frames [f0, f0 + n) as a view (no copy)."""
        pl = [(off + f0 * fs, pw, ph, st, fs) for off, pw, ph, st, fs in self.planes]
        return DevFrames(self.buf, n, self.w, self.h, pl, self.bits, self.keep)


def flat_layout(w: int, h: int) -> list:
    """[frame][Y | U | V] display-size planar frames (y4m order)."""
    ysz, csz = w * h, (w // 2) * (h // 2)
    fsz = ysz + 2 * csz
    return [(0, w, h, w, fsz), (ysz, w // 2, h // 2, w // 2, fsz), (ysz + csz, w // 2, h // 2, w // 2, fsz)]


_STATS_LOCK = threading.Lock()


class _Pinned:
    """Grow-only pinned host buffer per thread (H2D uploads without pageable staging)."""

    _tls = threading.local()

    @classmethod
    def get(cls, nbytes: int):
        import torch

        b = getattr(cls._tls, "buf", None)
        if b is None or b.numel() < nbytes:
            b = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8).pin_memory()
            cls._tls.buf = b
        return b


def from_flat(t, w: int, h: int, n: int | None = None, bits: int = 8) -> DevFrames:
    """Wrap a device tensor holding [frame][Y | U | V] planar frames (e.g. an RCCL-received
    segment) — no copy."""
    n = n if n is not None else t.shape[0]
    return DevFrames(t, n, w, h, flat_layout(w, h), bits)


def thumbs8(ptr: int, bits: int, w: int, h: int, stride: int, fs: int, n: int, out) -> None:
    """8x8 block means of n luma planes at device address `ptr` (element strides) into the
    float32 CUDA tensor `out` [n][h // 8][w // 8], on the current stream."""
    import torch

    st = C.c_void_p(torch.cuda.current_stream(out.device).cuda_stream)
    _ok(_lib().tv_thumbs8_batch(C.c_void_p(ptr), bits, w, h, stride, fs, n, C.c_void_p(out.data_ptr()), st))


def upload_frames(frames, device) -> DevFrames:
    """Host (Y, U, V) numpy frames (uint8, or uint16 for 10-bit) -> one device tensor,
    through a reusable pinned buffer (one H2D copy per segment)."""
    import torch

    n = len(frames)
    h, w = frames[0][0].shape
    dt = frames[0][0].dtype
    bits = 10 if dt == np.uint16 else 8
    lay = flat_layout(w, h)
    fsz = lay[0][4]
    esz = 2 if bits == 10 else 1
    pin = _Pinned.get(n * fsz * esz)
    host = pin[: n * fsz * esz].numpy().view(np.int16 if bits == 10 else np.uint8).reshape(n, fsz)
    ysz, csz = w * h, (w // 2) * (h // 2)
    for k, (y, u, v) in enumerate(frames):
        host[k, :ysz] = y.reshape(-1)
        host[k, ysz:ysz + csz] = u.reshape(-1)
        host[k, ysz + csz:] = v.reshape(-1)
    tdt = torch.int16 if bits == 10 else torch.uint8
    dev = torch.empty((n, fsz), dtype=tdt, device=device)
    dev.copy_(pin[: n * fsz * esz].view(tdt).view(n, fsz), non_blocking=True)
    # the pinned buffer is reused by the next upload on this thread: wait for this copy
    torch.cuda.current_stream(device).synchronize()
    return DevFrames(dev, n, w, h, lay, bits)


def synth_frames(seed: int, w: int, h: int, starts, device) -> DevFrames:
    """Synthetic source frames t in `starts` generated on the device (tv/synth.h), exactly
    the frames the engine's own generator and the CPU golden model produce."""
    import torch

    n = len(starts)
    cw, ch = coded_size(w, h)
    ysz, csz = cw * ch, (cw // 2) * (ch // 2)
    buf = torch.empty(n * (ysz + 2 * csz), dtype=torch.uint8, device=device)
    ts = (C.c_int * n)(*[int(t) for t in starts])
    st = C.c_void_p(torch.cuda.current_stream(device).cuda_stream)
    _ok(_lib().tv_synth_batch(C.c_void_p(buf.data_ptr()), w, h, n, ts, seed & 0xFFFFFFFF, st))
    planes = [(0, w, h, cw, ysz), (n * ysz, w // 2, h // 2, cw // 2, csz),
              (n * ysz + n * csz, w // 2, h // 2, cw // 2, csz)]
    return DevFrames(buf, n, w, h, planes, 8)


def tone_map(src: DevFrames, src_peak: float = 1000.0, dst_peak: float = 100.0) -> DevFrames:
    """10-bit planar PQ (BT.2020) -> 8-bit SDR BT.709 I420 on the device (k_tonemap_pq)."""
    import torch

    if src.bits != 10:
        return src
    n, w, h = src.n, src.w, src.h
    dev = src.buf.device
    (yo, _, _, ys, yfs), (uo, _, _, us, ufs), (vo, _, _, vs, vfs) = src.planes
    flat = src.buf.reshape(-1)

    def plane(off, pw, ph, stride, fs):
        return torch.as_strided(flat, (n, ph, pw), (fs, stride, 1), off).to(torch.int32)

    # P010 layout the tone-map kernel reads: MSB-aligned 16-bit samples (int16 bit patterns
    # of the uint16 values), UV interleaved
    y16 = (plane(yo, w, h, ys, yfs) << 6).to(torch.int16).contiguous()
    u = plane(uo, w // 2, h // 2, us, ufs) << 6
    v = plane(vo, w // 2, h // 2, vs, vfs) << 6
    uv16 = torch.stack([u, v], -1).reshape(n, h // 2, w).to(torch.int16).contiguous()
    fsz = w * h * 3 // 2
    out = torch.empty((n, fsz), dtype=torch.uint8, device=dev)
    st = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    _ok(_lib().tv_tonemap_pq_batch(y16.data_ptr(), uv16.data_ptr(), w, h, n, out.data_ptr(), C.c_float(src_peak),
                                   C.c_float(dst_peak), st), "ops")
    res = DevFrames(out, n, w, h, flat_layout(w, h), 8)
    res.keep = [y16, uv16]
    return res


def staging_planes(w: int, h: int, coded: tuple | None = None) -> tuple[int, list]:
    """(coded frame size, [(offset, display w, h, row stride, coded w, coded h)]) of the
    engine staging layout (`coded` overrides the HEVC CTB-aligned coded size, e.g. the AV1
    engine's 16-aligned one)."""
    cw, ch = coded or coded_size(w, h)
    ysz, csz = cw * ch, (cw // 2) * (ch // 2)
    return ysz + 2 * csz, [(0, w, h, cw, cw, ch), (ysz, w // 2, h // 2, cw // 2, cw // 2, ch // 2),
                           (ysz + csz, w // 2, h // 2, cw // 2, cw // 2, ch // 2)]


def to_staging(src: DevFrames, out_w: int, out_h: int, dst, frame0: int = 0, coded: tuple | None = None) -> None:
    """Write src's frames (tone-mapped if 10-bit) into the engine staging tensor `dst`
    (coded-size [frame][Y|U|V] of out_w x out_h) starting at frame slot `frame0`: edge pad
    when the size is unchanged, fused Lanczos otherwise.  Runs on the current stream."""
    import torch

    from ..models.abr import _tables, resize2d_plan

    src = tone_map(src)
    lib = _lib()
    dev = dst.device
    st = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    fsz, planes = staging_planes(out_w, out_h, coded)
    base = dst.data_ptr() + frame0 * fsz
    for c, (doff, dw, dh, dstride, pw, ph) in enumerate(planes):
        _, sw, sh, sstride, sfs = src.planes[c]
        sp = src.ptr(c)
        if (sw, sh) == (dw, dh):
            _ok(lib.tv_pad_batch(sp, sw, sh, sstride, sfs, base + doff, pw, ph, dstride, fsz, src.n, st))
            continue
        ix, wx, tx = _tables(sw, dw, 3, dev.index)
        iy, wy, ty = _tables(sh, dh, 3, dev.index)
        th, wp, smem = resize2d_plan(sw, sh, dw, dh, pw, ph)
        tmp = torch.empty(1 if th else src.n * sh * dw, dtype=torch.int16, device=dev)
        _ok(lib.tv_resize_batch(sp, sw, sh, sstride, sfs, base + doff, dw, dh, dstride, fsz, pw, ph, src.n,
                                ix.data_ptr(), wx.data_ptr(), tx, iy.data_ptr(), wy.data_ptr(), ty, tmp.data_ptr(),
                                th, wp, smem, st), "ops")


INGEST_CHUNK = 32 << 20  # bytes per ring slot (2 slots per reader thread)


def read_y4m_device(src, start: int, n: int, device, threads: int | None = None, stats: dict | None = None) -> DevFrames:
    """Frames [start, start + n) of a Y4M source (models.media.Y4MSource) -> device, the
    file-ingest path of a node job (reference GET part,
    worker/tasks.py:1497-1525): csrc/gpu/ingest.hip reads the segment's byte range with
    `threads` pread threads into a pinned ring and streams each 32 MiB chunk to HBM with
    hipMemcpyAsync while the next chunks are read (read and DMA overlapped, no host
    repacking).  The FRAME headers stay in the buffer: the plane descriptors step over them.
    `stats` accumulates the bytes, the wall seconds and the summed per-thread read seconds."""
    import os

    import torch

    info = src.info
    n = max(0, min(n, src.nframes - start))
    nbytes = n * info.frame_bytes
    lib = _lib()
    if not getattr(lib, "_ingest_sigs", False):
        lib.tv_ingest_h2d.argtypes = [C.c_char_p, C.c_longlong, C.c_longlong, C.c_void_p, C.c_void_p, C.c_longlong,
                                      C.c_int, C.c_void_p, C.POINTER(C.c_double)]
        lib.tv_ingest_last_error.restype = C.c_char_p
        lib._ingest_sigs = True
    if threads is None:
        threads = max(1, min(12, len(os.sched_getaffinity(0))))
    ring = _Pinned.get(2 * threads * INGEST_CHUNK)
    esz = 2 if info.bits > 8 else 1
    buf = torch.empty(nbytes // esz, dtype=torch.int16 if esz == 2 else torch.uint8, device=device)
    tm = (C.c_double * 2)()
    st = C.c_void_p(torch.cuda.current_stream(device).cuda_stream)
    if lib.tv_ingest_h2d(src.path.encode(), info.header_len + start * info.frame_bytes, nbytes,
                         C.c_void_p(buf.data_ptr()), C.c_void_p(ring.data_ptr()), ring.numel(), threads, st, tm) != 0:
        raise RuntimeError(f"{src.path}: ingest of frames {start}..{start + n} failed: "
                           f"{lib.tv_ingest_last_error().decode()}")
    w, h = info.width, info.height
    hdr = (info.frame_bytes - w * h * 3 // 2 * esz) // esz  # FRAME header, in elements
    fs = info.frame_bytes // esz
    ysz, csz = w * h, (w // 2) * (h // 2)
    planes = [(hdr, w, h, w, fs), (hdr + ysz, w // 2, h // 2, w // 2, fs), (hdr + ysz + csz, w // 2, h // 2, w // 2, fs)]
    if stats is not None:  # the node job's prefetch thread and its main thread share `stats`
        with _STATS_LOCK:
            stats["read_bytes"] = stats.get("read_bytes", 0) + nbytes
            stats["ingest_s"] = stats.get("ingest_s", 0.0) + tm[1]
            stats["read_thread_s"] = stats.get("read_thread_s", 0.0) + tm[0]
            stats["read_threads"] = threads
    return DevFrames(buf, n, w, h, planes, 8 if esz == 1 else 10)


def write_synth_y4m(path: str, w: int, h: int, n: int, seed: int = 1, device=0, chunk: int = 64) -> int:
    """A y4m file of n frames of the seeded synthetic source, generated on the GPU
    (tv/synth.h) `chunk` frames at a time and written as they come back — the file source
    of the ingest bench (bench.py --job --source y4m).  Returns the file size."""
    import os

    import torch

    dev = torch.device("cuda", device) if isinstance(device, int) else device
    fsz = w * h * 3 // 2
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(f"YUV4MPEG2 W{w} H{h} F30:1 Ip A1:1 C420jpeg\n".encode())
        for t0 in range(0, n, chunk):
            k = min(chunk, n - t0)
            src = synth_frames(seed, w, h, list(range(t0, t0 + k)), dev)
            flat = src.buf.reshape(-1)
            out = torch.empty((k, 6 + fsz), dtype=torch.uint8, device=dev)
            out[:, :6] = torch.tensor(list(b"FRAME\n"), dtype=torch.uint8, device=dev)
            o = 6
            for off, pw, ph, stride, fs in src.planes:
                out[:, o:o + pw * ph] = torch.as_strided(flat, (k, ph, pw), (fs, stride, 1), off).reshape(k, -1)
                o += pw * ph
            f.write(memoryview(out.cpu().numpy()).cast("B"))
    os.replace(tmp, path)
    return os.path.getsize(path)
