"""Frame-number stamping (reference `drawtext text=%{n}` centred, font
size 72, border 5 — worker/tasks.py:2377-2395).

The label is rasterised on the host from an embedded 5x7 digit font into a small mask
(0 keep / 1 border / 2 glyph); the HIP kernel `k_overlay_mask` burns the masks of a whole
batch of frames in one launch.  numpy frames take the reference path.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

_FONT = {
    "0": ["01110", "10001", "10011", "10101", "11001", "10001", "01110"],
    "1": ["00100", "01100", "00100", "00100", "00100", "00100", "01110"],
    "2": ["01110", "10001", "00001", "00010", "00100", "01000", "11111"],
    "3": ["11111", "00010", "00100", "00010", "00001", "10001", "01110"],
    "4": ["00010", "00110", "01010", "10010", "11111", "00010", "00010"],
    "5": ["11111", "10000", "11110", "00001", "00001", "10001", "01110"],
    "6": ["00110", "01000", "10000", "11110", "10001", "10001", "01110"],
    "7": ["11111", "00001", "00010", "00100", "01000", "01000", "01000"],
    "8": ["01110", "10001", "10001", "01110", "10001", "10001", "01110"],
    "9": ["01110", "10001", "10001", "01111", "00001", "00010", "01100"],
}


def _dilate(m: np.ndarray, r: int) -> np.ndarray:
    out = m.copy()
    for dy in range(-r, r + 1):
        for dx in range(-r, r + 1):
            out |= np.roll(np.roll(m, dy, 0), dx, 1)
    return out


def label_mask(text: str, size: int = 72, border: int = 5) -> np.ndarray:
    """uint8 mask of `text` (digits) with glyph height ~`size` px and a `border` px outline."""
    s = max(1, size // 7)
    glyphs = []
    for ch in text:
        g = np.array([[c == "1" for c in row] for row in _FONT[ch]], bool)
        glyphs.append(np.kron(g, np.ones((s, s), bool)))
        glyphs.append(np.zeros((7 * s, s), bool))
    core = np.concatenate(glyphs[:-1], 1) if glyphs else np.zeros((7 * s, 1), bool)
    pad = border + 1
    core = np.pad(core, pad)
    halo = _dilate(core, border)
    mask = np.where(core, 2, np.where(halo, 1, 0)).astype(np.uint8)
    if mask.shape[1] & 1:
        mask = np.pad(mask, ((0, 0), (0, 1)))
    if mask.shape[0] & 1:
        mask = np.pad(mask, ((0, 1), (0, 0)))
    return mask


def placement(w: int, h: int, mw: int, mh: int) -> tuple[int, int]:
    return ((w - mw) // 2) & ~1, ((h - mh) // 2) & ~1


def stamp_ref(frame, text: str, size: int = 72, border: int = 5):
    """numpy reference: returns a stamped copy of (Y, U, V)."""
    y, u, v = (np.array(p, np.uint8, copy=True) for p in frame)
    m = label_mask(text, size, border)
    h, w = y.shape
    x0, y0 = placement(w, h, m.shape[1], m.shape[0])
    ys, xs = np.nonzero(m)
    gy, gx = ys + y0, xs + x0
    ok = (gy >= 0) & (gy < h) & (gx >= 0) & (gx < w)
    ys, xs, gy, gx = ys[ok], xs[ok], gy[ok], gx[ok]
    y[gy, gx] = np.where(m[ys, xs] == 2, 235, 16)
    c = ((gy & 1) == 0) & ((gx & 1) == 0)
    u[gy[c] // 2, gx[c] // 2] = 128
    v[gy[c] // 2, gx[c] // 2] = 128
    return y, u, v


def stamp_frames_gpu(frames_dev, w: int, h: int, numbers, size: int = 72, border: int = 5):
    """Stamp `numbers[i]` into frame i of a contiguous uint8 CUDA tensor laid out
    [n, Y|U|V] (I420, w x h), in place, with one kernel launch."""
    import torch

    from .._native import gpu_lib

    texts = [str(int(n)) for n in numbers]
    masks = [label_mask(t, size, border) for t in texts]
    mh = max(m.shape[0] for m in masks)
    mw = max(m.shape[1] for m in masks)
    stack = np.zeros((len(masks), mh, mw), np.uint8)
    for i, m in enumerate(masks):  # centre every label in the common box
        oy, ox = ((mh - m.shape[0]) // 2) & ~1, ((mw - m.shape[1]) // 2) & ~1
        stack[i, oy:oy + m.shape[0], ox:ox + m.shape[1]] = m
    x0, y0 = placement(w, h, mw, mh)
    dm = torch.from_numpy(stack).to(frames_dev.device)
    lib = gpu_lib()
    stream = torch.cuda.current_stream(frames_dev.device).cuda_stream
    rc = lib.tv_overlay_mask(C.c_void_p(frames_dev.data_ptr()), len(texts), w, h, C.c_void_p(dm.data_ptr()), mw, mh,
                             x0, y0, C.c_void_p(stream))
    if rc != 0:
        lib.tv_ops_last_error.restype = C.c_char_p
        raise RuntimeError(lib.tv_ops_last_error().decode())
    return frames_dev
