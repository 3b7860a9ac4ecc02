"""Colour-space conversion and HDR10 tone mapping (SURVEY.md §2.3 K2 `format=nv12`, K15
tone-map for the 8K HDR10 ABR config).  HIP kernels in csrc/gpu/k_ops.hip; numpy float64
references of the same math for tests and CPU-only hosts (chosen by the input's type,
never as a silent substitute for a GPU tensor).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

_MAT = {
    True: (0.2126, 0.7152, 0.0722, -0.1146, -0.3854, 0.5, 0.5, -0.4542, -0.0458),
    False: (0.299, 0.587, 0.114, -0.168736, -0.331264, 0.5, 0.5, -0.418688, -0.081312),
}


def _sat(x):
    return np.clip(np.rint(x), 0, 255).astype(np.uint8)


def _to_yuv420(r, g, b, bt709=True):
    ry, gy, by, ru, gu, bu, rv, gv, bv = _MAT[bool(bt709)]
    Y = _sat(16 + 219 * (ry * r + gy * g + by * b))
    cu = ru * r + gu * g + bu * b
    cv = rv * r + gv * g + bv * b
    pool = lambda c: (c[0::2, 0::2] + c[0::2, 1::2] + c[1::2, 0::2] + c[1::2, 1::2]) / 4
    return Y, _sat(128 + 224 * pool(cu)), _sat(128 + 224 * pool(cv))


def rgb_to_i420_ref(rgb: np.ndarray, bt709: bool = True):
    f = np.asarray(rgb, np.float64) / 255.0
    return _to_yuv420(f[..., 0], f[..., 1], f[..., 2], bt709)


def p010_to_i420_ref(y16: np.ndarray, uv16: np.ndarray):
    y8 = np.minimum(255, ((y16.astype(np.int32) >> 6) + 2) >> 2).astype(np.uint8)
    c = np.minimum(255, ((uv16.astype(np.int32) >> 6) + 2) >> 2).astype(np.uint8)
    return y8, np.ascontiguousarray(c[:, 0::2]), np.ascontiguousarray(c[:, 1::2])


# ------------------------------------------------------------------ PQ tone map
_M1, _M2, _C1, _C2, _C3 = 0.1593017578125, 78.84375, 0.8359375, 18.8515625, 18.6875


def pq_eotf(e):
    p = np.power(np.clip(e, 0.0, 1.0), 1.0 / _M2)
    return np.power(np.maximum(p - _C1, 0.0) / (_C2 - _C3 * p), 1.0 / _M1)


def pq_oetf(l):
    p = np.power(np.maximum(l, 0.0), _M1)
    return np.power((_C1 + _C2 * p) / (1.0 + _C3 * p), _M2)


def _eetf(e, src_pq, dst_pq):
    en, maxl = e / src_pq, dst_pq / src_pq
    ks = 1.5 * maxl - 0.5
    t = np.clip((en - ks) / (1.0 - ks), 0.0, None)
    t2, t3 = t * t, t * t * t
    knee = (2 * t3 - 3 * t2 + 1) * ks + (t3 - 2 * t2 + t) * (1 - ks) + (-2 * t3 + 3 * t2) * maxl
    return np.where(en > ks, knee, en) * src_pq


def _bt709_oetf(l):
    l = np.clip(l, 0.0, 1.0)
    return np.where(l < 0.018, 4.5 * l, 1.099 * np.power(l, 0.45) - 0.099)


def tonemap_pq_ref(y16: np.ndarray, uv16: np.ndarray, src_peak: float = 1000.0, dst_peak: float = 100.0):
    """HDR10 P010 (BT.2020 PQ, limited range) -> SDR I420 BT.709 (same steps as the kernel)."""
    h, w = y16.shape
    yp = ((y16.astype(np.int64) >> 6) - 64) / 876.0
    uv = (uv16.astype(np.int64) >> 6).astype(np.float64)
    cb = np.repeat(np.repeat((uv[:, 0::2] - 512) / 896.0, 2, 0), 2, 1)[:h, :w]
    cr = np.repeat(np.repeat((uv[:, 1::2] - 512) / 896.0, 2, 0), 2, 1)[:h, :w]
    r, g, b = yp + 1.4746 * cr, yp - 0.16455 * cb - 0.57135 * cr, yp + 1.8814 * cb
    src_pq, dst_pq = pq_oetf(src_peak / 10000.0), pq_oetf(dst_peak / 10000.0)
    mx = np.maximum(np.maximum(r, g), np.maximum(b, 1e-6))
    lm, lt = pq_eotf(mx), pq_eotf(_eetf(mx, src_pq, dst_pq))
    sc = np.where(lm > 1e-6, lt / np.where(lm > 1e-6, lm, 1), 0.0) * (10000.0 / dst_peak)
    R, G, B = pq_eotf(r) * sc, pq_eotf(g) * sc, pq_eotf(b) * sc
    r7 = 1.6605 * R - 0.5876 * G - 0.0728 * B
    g7 = -0.1246 * R + 1.1329 * G - 0.0083 * B
    b7 = -0.0182 * R - 0.1006 * G + 1.1187 * B
    return _to_yuv420(_bt709_oetf(r7), _bt709_oetf(g7), _bt709_oetf(b7), True)


# ------------------------------------------------------------------ GPU wrappers
def _call(name, *args):
    import torch  # noqa: F401

    from .._native import gpu_lib

    lib = gpu_lib()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        lib.tv_ops_last_error.restype = C.c_char_p
        raise RuntimeError(lib.tv_ops_last_error().decode())


def _p(t):
    return C.c_void_p(t.data_ptr())


def _stream(t):
    import torch

    return C.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _planes(h, w, dev):
    import torch

    return (torch.empty((h, w), dtype=torch.uint8, device=dev),
            torch.empty((h // 2, w // 2), dtype=torch.uint8, device=dev),
            torch.empty((h // 2, w // 2), dtype=torch.uint8, device=dev))


def rgb_to_i420(rgb, bt709: bool = True):
    if isinstance(rgb, np.ndarray):
        return rgb_to_i420_ref(rgb, bt709)
    rgb = rgb.contiguous()
    h, w, _ = rgb.shape
    y, u, v = _planes(h, w, rgb.device)
    _call("tv_rgb_to_i420", _p(rgb), w, h, w * 3, _p(y), _p(u), _p(v), int(bt709), _stream(rgb))
    return y, u, v


def p010_to_i420(y16, uv16):
    """y16: (h, w) uint16; uv16: (h/2, w) interleaved uint16 (P010 layout)."""
    if isinstance(y16, np.ndarray):
        return p010_to_i420_ref(y16, uv16)
    h, w = y16.shape
    y, u, v = _planes(h, w, y16.device)
    _call("tv_p010_to_i420", _p(y16.contiguous()), _p(uv16.contiguous()), w, h, _p(y), _p(u), _p(v), _stream(y16))
    return y, u, v


def tonemap_pq(y16, uv16, src_peak: float = 1000.0, dst_peak: float = 100.0):
    if isinstance(y16, np.ndarray):
        return tonemap_pq_ref(y16, uv16, src_peak, dst_peak)
    h, w = y16.shape
    y, u, v = _planes(h, w, y16.device)
    _call("tv_tonemap_pq", _p(y16.contiguous()), _p(uv16.contiguous()), w, h, _p(y), _p(u), _p(v),
          C.c_float(src_peak), C.c_float(dst_peak), _stream(y16))
    return y, u, v
