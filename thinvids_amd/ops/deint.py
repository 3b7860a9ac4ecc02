"""Bob-Weaver deinterlacing (reference `bwdif=mode=send_frame:
parity=auto:deint=all` for DVD-native 480/576 material, worker/tasks.py:62-63, :475-500).

HIP kernel `k_bwdif` (csrc/gpu/k_ops.hip) on GPU tensors; an integer numpy reference of the
same filter for numpy inputs (tests, CPU-only hosts).
"""
from __future__ import annotations

import ctypes as C

import numpy as np


def bwdif_plane_ref(prev: np.ndarray, cur: np.ndarray, nxt: np.ndarray, tff: bool = True) -> np.ndarray:
    h, w = cur.shape
    P, Cu, N = (np.asarray(a, np.int64) for a in (prev, cur, nxt))
    out = Cu.copy()
    keep = 0 if tff else 1

    def at(f, y, dy):
        return f[np.clip(y + dy, 0, h - 1)]

    for y in range(h):
        if (y & 1) == keep:
            continue
        if y < 2 or y >= h - 2:
            up = Cu[y - 1] if y > 0 else Cu[y + 1]
            dn = Cu[y + 1] if y < h - 1 else Cu[y - 1]
            out[y] = (up + dn + 1) >> 1
            continue
        p2, n2 = P, Cu
        c, e = at(Cu, y, -1), at(Cu, y, 1)
        d = (at(p2, y, 0) + at(n2, y, 0)) >> 1
        td0 = np.abs(at(p2, y, 0) - at(n2, y, 0))
        td1 = (np.abs(at(P, y, -1) - c) + np.abs(at(P, y, 1) - e)) >> 1
        td2 = (np.abs(at(N, y, -1) - c) + np.abs(at(N, y, 1) - e)) >> 1
        diff = np.maximum(td0 >> 1, np.maximum(td1, td2))
        b = ((at(p2, y, -2) + at(n2, y, -2)) >> 1) - c
        f = ((at(p2, y, 2) + at(n2, y, 2)) >> 1) - e
        dc, de = d - c, d - e
        mx = np.maximum(np.maximum(de, dc), np.minimum(b, f))
        mn = np.minimum(np.minimum(de, dc), np.maximum(b, f))
        diff2 = np.maximum(np.maximum(diff, mn), -mx)
        hf = ((5570 * (at(p2, y, 0) + at(n2, y, 0)) - 3801 * (at(p2, y, -2) + at(n2, y, -2) + at(p2, y, 2)
                                                            + at(n2, y, 2))
               + 1016 * (at(p2, y, -4) + at(n2, y, -4) + at(p2, y, 4) + at(n2, y, 4))) >> 2) \
            + 4309 * (c + e) - 213 * (at(Cu, y, -3) + at(Cu, y, 3))
        sp = 5077 * (c + e) - 981 * (at(Cu, y, -3) + at(Cu, y, 3))
        interp = np.where(np.abs(c - e) > td0, hf, sp) >> 13
        v = np.clip(interp, d - diff2, d + diff2)
        out[y] = np.where(diff == 0, d, v)
    return np.clip(out, 0, 255).astype(np.uint8)


def bwdif_frame(prev, cur, nxt, tff: bool = True):
    """Deinterlace an I420 frame (tuples of planes) given its neighbours."""
    return tuple(bwdif_plane(p, c, n, tff) for p, c, n in zip(prev, cur, nxt))


def bwdif_plane(prev, cur, nxt, tff: bool = True):
    if isinstance(cur, np.ndarray):
        return bwdif_plane_ref(prev, cur, nxt, tff)
    import torch

    from .._native import gpu_lib

    h, w = cur.shape
    out = torch.empty_like(cur)
    lib = gpu_lib()
    p = lambda t: C.c_void_p(t.contiguous().data_ptr())
    rc = lib.tv_bwdif_plane(p(prev), p(cur), p(nxt), C.c_void_p(out.data_ptr()), w, h, int(tff),
                            C.c_void_p(torch.cuda.current_stream(cur.device).cuda_stream))
    if rc != 0:
        lib.tv_ops_last_error.restype = C.c_char_p
        raise RuntimeError(lib.tv_ops_last_error().decode())
    return out


def deinterlace_device(df, tff: bool = True):
    """bwdif (send_frame) over a segment of 8-bit device frames (ops.stage.DevFrames) with
    ``k_bwdif_seg``: one launch for every frame and plane, frame i from (i-1, i, i+1), the
    segment's edges repeat (the split pipeline's per-part rule).  Returns new DevFrames in the
    same layout."""
    import torch

    from .._native import gpu_lib
    from .stage import DevFrames

    if df.bits != 8:
        raise ValueError("bwdif: 8-bit frames only")
    out = torch.empty_like(df.buf)
    lib = gpu_lib()
    stream = C.c_void_p(torch.cuda.current_stream(df.buf.device).cuda_stream)
    esz = df.buf.element_size()
    if any(st != pw for _, pw, _, st, _ in df.planes):
        raise ValueError("bwdif: planes must be packed")
    fs = df.planes[0][4]
    base = min(off for off, *_ in df.planes)
    rel = [off - base for off, *_ in df.planes]
    if any(p[4] != fs for p in df.planes) or any(r + pw * ph > fs for r, (_, pw, ph, _, _) in zip(rel, df.planes)):
        raise ValueError("bwdif: planes of one frame must share the frame stride")
    npl = len(df.planes)
    f = lib.tv_bwdif_segment
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_long, C.c_int, C.c_int, C.POINTER(C.c_long), C.POINTER(C.c_int),
                  C.POINTER(C.c_int), C.c_int, C.c_void_p]
    rc = f(C.c_void_p(df.buf.data_ptr() + base * esz), C.c_void_p(out.data_ptr() + base * esz), fs * esz, df.n, npl,
           (C.c_long * npl)(*[r * esz for r in rel]), (C.c_int * npl)(*[p[1] for p in df.planes]),
           (C.c_int * npl)(*[p[2] for p in df.planes]), int(tff), stream)
    if rc != 0:
        lib.tv_ops_last_error.restype = C.c_char_p
        raise RuntimeError(lib.tv_ops_last_error().decode())
    return DevFrames(out, df.n, df.w, df.h, df.planes, df.bits, [df.buf, *df.keep])


def deinterlace_frames(frames: list, tff: bool = True) -> list:
    """send_frame mode over a sequence: frame i uses (i-1, i, i+1), edges repeat."""
    n = len(frames)
    return [bwdif_frame(frames[max(0, i - 1)], frames[i], frames[min(n - 1, i + 1)], tff) for i in range(n)]
