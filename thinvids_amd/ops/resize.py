"""Lanczos plane resampling (reference `scale=-2:H`,
worker/tasks.py:62-65 / :436-449, Lanczos in tools/upscale_benchmark.py:163,183).

Filter tables are built here (numpy) and consumed by the HIP kernels `k_resize_h/v`
(csrc/gpu/k_ops.hip).  `resize_plane` dispatches on the tensor's device: a CUDA (HIP)
tensor runs the HIP kernels (the native library is required — no fallback), a numpy
array / CPU tensor runs the float64 reference of the same separable filter.
"""
from __future__ import annotations

import ctypes as C
from functools import lru_cache

import numpy as np

Q = 14


def _lanczos(x: np.ndarray, a: int) -> np.ndarray:
    x = np.asarray(x, np.float64)
    out = np.sinc(x) * np.sinc(x / a)
    out[np.abs(x) >= a] = 0.0
    return out


@lru_cache(maxsize=64)
def filter_table(n_in: int, n_out: int, a: int = 3) -> tuple[np.ndarray, np.ndarray, np.ndarray]:
    """(start index int32 [n_out], float64 weights [n_out, taps], Q14 int16 weights).

    Pixel-centre aligned mapping; when down-scaling the kernel is stretched by the ratio
    (anti-aliasing), exactly like a swscale Lanczos filter of parameter `a`."""
    scale = n_in / n_out
    support = a * max(1.0, scale)
    taps = int(np.ceil(2 * support))
    centers = (np.arange(n_out) + 0.5) * scale - 0.5
    start = np.floor(centers - support + 1).astype(np.int64)
    k = np.arange(taps)
    pos = start[:, None] + k[None, :]
    w = _lanczos((pos - centers[:, None]) / max(1.0, scale), a)
    w /= w.sum(1, keepdims=True)
    wq = np.round(w * (1 << Q)).astype(np.int64)
    # make every row sum exactly 1<<Q (fix the rounding residue on the largest tap)
    resid = (1 << Q) - wq.sum(1)
    wq[np.arange(n_out), np.argmax(w, 1)] += resid
    return start.astype(np.int32), w, wq.astype(np.int16)


def resize_plane_ref(src: np.ndarray, out_h: int, out_w: int, a: int = 3) -> np.ndarray:
    """float64 reference (same taps, edge clamp), rounded to uint8."""
    src = np.asarray(src, np.float64)
    h, w = src.shape
    sx, wx, _ = filter_table(w, out_w, a)
    sy, wy, _ = filter_table(h, out_h, a)
    cols = np.clip(sx[:, None] + np.arange(wx.shape[1])[None, :], 0, w - 1)
    tmp = np.einsum("yxk,xk->yx", src[:, cols], wx)
    rows = np.clip(sy[:, None] + np.arange(wy.shape[1])[None, :], 0, h - 1)
    out = np.einsum("ykx,yk->yx", tmp[rows, :], wy)
    return np.clip(np.rint(out), 0, 255).astype(np.uint8)


def _dev_tables(n_in, n_out, a, device):
    import torch

    s, _, wq = filter_table(n_in, n_out, a)
    return (torch.from_numpy(s.copy()).to(device), torch.from_numpy(wq.copy()).to(device), wq.shape[1])


def resize_plane(src, out_h: int, out_w: int, a: int = 3, out=None):
    """Resample one 8-bit plane.  `src` may be a numpy array (reference path) or a torch
    uint8 tensor; on a GPU tensor the HIP kernels run on the current stream."""
    if isinstance(src, np.ndarray):
        return resize_plane_ref(src, out_h, out_w, a)
    import torch

    if not src.is_cuda:
        return torch.from_numpy(resize_plane_ref(src.numpy(), out_h, out_w, a))
    from .._native import gpu_lib

    lib = gpu_lib()
    h, w = src.shape
    src = src.contiguous()
    dev = src.device
    ix, wx, tx = _dev_tables(w, out_w, a, dev)
    iy, wy, ty = _dev_tables(h, out_h, a, dev)
    tmp = torch.empty((h, out_w), dtype=torch.int16, device=dev)
    if out is None:
        out = torch.empty((out_h, out_w), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    vp = C.c_void_p
    rc = lib.tv_resize_plane(vp(src.data_ptr()), w, h, w, vp(out.data_ptr()), out_w, out_h, out.stride(0),
                             vp(ix.data_ptr()), vp(wx.data_ptr()), tx, vp(iy.data_ptr()), vp(wy.data_ptr()), ty,
                             vp(tmp.data_ptr()), vp(stream))
    if rc != 0:
        lib.tv_ops_last_error.restype = C.c_char_p
        raise RuntimeError(lib.tv_ops_last_error().decode())
    return out


def resize_frame(frame, out_w: int, out_h: int, a: int = 3):
    """Resize an I420 frame (Y, U, V) to out_w x out_h (even)."""
    y, u, v = frame
    return (resize_plane(y, out_h, out_w, a), resize_plane(u, out_h // 2, out_w // 2, a),
            resize_plane(v, out_h // 2, out_w // 2, a))
