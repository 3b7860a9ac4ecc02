"""Quality metrics: PSNR and SSIM.  SSIM is the mean over 8x8 windows
on a 4-sample grid (x264/libvpx convention); HIP kernel `k_ssim` for GPU tensors, float64
numpy reference for numpy inputs."""
from __future__ import annotations

import ctypes as C

import numpy as np

C1, C2 = (0.01 * 255) ** 2, (0.03 * 255) ** 2


def psnr(a, b) -> float:
    mse = np.mean((np.asarray(a, np.float64) - np.asarray(b, np.float64)) ** 2)
    return float("inf") if mse == 0 else float(10 * np.log10(255.0 ** 2 / mse))


def ssim_ref(a: np.ndarray, b: np.ndarray) -> float:
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    h, w = a.shape
    vals = []
    for y0 in range(0, h - 7, 4):
        for x0 in range(0, w - 7, 4):
            p, q = a[y0:y0 + 8, x0:x0 + 8], b[y0:y0 + 8, x0:x0 + 8]
            ma, mb = p.mean(), q.mean()
            va, vb = (p * p).mean() - ma * ma, (q * q).mean() - mb * mb
            cov = (p * q).mean() - ma * mb
            vals.append(((2 * ma * mb + C1) * (2 * cov + C2)) / ((ma * ma + mb * mb + C1) * (va + vb + C2)))
    return float(np.mean(vals))


def ssim(a, b) -> float:
    if isinstance(a, np.ndarray):
        return ssim_ref(a, b)
    import torch

    from .._native import gpu_lib

    h, w = a.shape
    acc = torch.zeros(1, dtype=torch.float64, device=a.device)
    lib = gpu_lib()
    rc = lib.tv_ssim_plane(C.c_void_p(a.data_ptr()), C.c_void_p(b.data_ptr()), w, h, a.stride(0), b.stride(0),
                           C.c_void_p(acc.data_ptr()), C.c_void_p(torch.cuda.current_stream(a.device).cuda_stream))
    if rc != 0:
        lib.tv_ops_last_error.restype = C.c_char_p
        raise RuntimeError(lib.tv_ops_last_error().decode())
    n = ((w - 8) // 4 + 1) * ((h - 8) // 4 + 1)
    return float(acc.item()) / n


def ssim_yuv(ref, dist) -> dict:
    y, u, v = (ssim(r, d) for r, d in zip(ref, dist))
    return {"y": y, "u": u, "v": v, "all": (6 * y + u + v) / 8}
