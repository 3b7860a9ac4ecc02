"""AV1 in-loop filter tools (BASELINE config #4 "AV1 with CDEF +
loop-restoration HIP kernels"): CDEF direction search / strength search / filter, Wiener
and self-guided loop restoration with their encoder-side parameter searches.

Every op has two implementations with identical integer results:

* numpy planes   -> the C++ golden model (``libtvcore.so``, csrc/core/av1_tools.cpp);
* torch (cuda)   -> the gfx950 kernels (``libtvgpu.so``, csrc/gpu/k_av1.hip); a GPU tensor
  always runs the HIP kernel and raises if the native library is missing.

GPU entry points take a batch of planes ``(B, h, w)`` uint8 (one launch per batch).  The
parameter *decisions* (which CDEF preset per 64x64 block, which Wiener taps / self-guided
set per 64x64 restoration unit) are small least-squares / argmin problems solved here on
the host from the kernels' statistics.

Scope: the filters follow the AV1 arithmetic (8-bit: Cdef_Directions, primary/secondary
taps and constrain(), variance-adjusted luma strength, 7-tap symmetric Wiener with
InterRound0/1 = 3/11, SGR parameter sets and A/B guide); loop restoration works on 64x64
units with edge-replicated context instead of AV1's 64-row stripes.  There is no AV1
bitstream writer: a conformant one needs the spec's default CDF tables, which are not
available offline (the range coder itself is in csrc/core/av1_tools.cpp).  Parity with
libaom/dav1d is therefore unpinned; tests pin GPU == C++ golden and the filters' gains.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

RU = 64  # restoration unit
PRESETS = 64  # CDEF (primary 0..15) x (secondary {0,1,2,4})
WIENER_MIN = np.array([-5, -23, -17])
WIENER_MAX = np.array([10, 8, 46])
SGR_XQD_MIN = np.array([-96, -32])
SGR_XQD_MAX = np.array([31, 95])

_vp = C.c_void_p


def _core():
    from .._native import core_lib

    lib = core_lib()
    if not getattr(lib, "_av1_sigs", False):
        i, u8, i32, i64 = C.c_int, C.POINTER(C.c_uint8), C.POINTER(C.c_int32), C.POINTER(C.c_int64)
        lib.tv_av1_cdef_find_dirs.argtypes = [u8, i, i, u8, i32]
        lib.tv_av1_cdef_search.argtypes = [u8, u8, i, i, i, u8, i32, i, i, C.POINTER(C.c_uint64)]
        lib.tv_av1_cdef_apply.argtypes = [u8, i, i, i, u8, i32, i, i, C.POINTER(C.c_int8), u8]
        lib.tv_av1_wiener_apply.argtypes = [u8, i, i, i32, u8]
        lib.tv_av1_wiener_stats.argtypes = [u8, u8, i, i, i, i32, i64]
        lib.tv_av1_sgr_apply.argtypes = [u8, i, i, i32, u8]
        lib.tv_av1_sgr_stats.argtypes = [u8, u8, i, i, i, i64]
        lib.tv_av1_sgr_filter_planes.argtypes = [u8, i, i, i, i32, i32]
        lib.tv_av1_deblock.argtypes = [u8, i, i, i, C.POINTER(C.c_uint32), i, u8]
        lib.tv_av1_deblock.restype = C.c_int
        lib.tv_av1_last_error.restype = C.c_char_p
        lib.tv_av1_rc_roundtrip.argtypes = [_vp, _vp, _vp, i, i, i, _vp, _vp]
        lib.tv_av1_rc_roundtrip.restype = C.c_int
        lib._av1_sigs = True
    return lib


def _gpu():
    from .._native import gpu_lib

    lib = gpu_lib()
    if not getattr(lib, "_av1_sigs", False):
        for name in ("tv_gpu_cdef_dirs", "tv_gpu_cdef_search", "tv_gpu_cdef_apply", "tv_gpu_wiener_apply",
                     "tv_gpu_wiener_stats", "tv_gpu_sgr_stats", "tv_gpu_sgr_apply", "tv_gpu_av1_deblock",
                     "tv_gpu_sgr_search", "tv_gpu_sgr_select", "tv_gpu_av1_deblock_step"):
            getattr(lib, name).restype = C.c_int
        lib.tv_av1_gpu_last_error.restype = C.c_char_p
        lib._av1_sigs = True
    return lib


def _p(a: np.ndarray, t=C.c_uint8):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(C.POINTER(t))


def _t(x):
    return _vp(x.data_ptr())


def _stream(x):
    import torch

    return _vp(torch.cuda.current_stream(x.device).cuda_stream)


def _check(rc: int):
    if rc != 0:
        raise RuntimeError(_gpu().tv_av1_gpu_last_error().decode())


def _is_np(x) -> bool:
    return isinstance(x, np.ndarray)


def n_fb(w: int, h: int, chroma: bool) -> int:
    f = 32 if chroma else 64
    return -(-w // f) * -(-h // f)


def n_units(w: int, h: int) -> int:
    return -(-w // RU) * -(-h // RU)


# --------------------------------------------------------------------------- CDEF ----
def cdef_dirs(Y):
    """Direction (0..7) and variance of every 8x8 block.  numpy (h, w) -> (dir, var) of
    shape (h/8, w/8); torch (B, h, w) cuda -> tensors (B, h/8 * w/8)."""
    if _is_np(Y):
        h, w = Y.shape
        d = np.zeros((h // 8, w // 8), np.uint8)
        v = np.zeros((h // 8, w // 8), np.int32)
        _core().tv_av1_cdef_find_dirs(_p(np.ascontiguousarray(Y)), w, h, _p(d), _p(v, C.c_int32))
        return d, v
    import torch

    B, h, w = Y.shape
    n8 = (h // 8) * (w // 8)
    d = torch.empty((B, n8), dtype=torch.uint8, device=Y.device)
    v = torch.empty((B, n8), dtype=torch.int32, device=Y.device)
    _check(_gpu().tv_gpu_cdef_dirs(_t(Y.contiguous()), w, h, B, _t(d), _t(v), _stream(Y)))
    return d, v


def cdef_search(src, rec, dirs, var, chroma: bool, damping: int = 5, luma_w8: int | None = None,
                pmask: int = (1 << 64) - 1, checker: bool = False):
    """SSE of every (64x64 filter block, preset) after CDEF: numpy -> (nfb, 64) uint64;
    torch (B, h, w) -> (B, nfb, 64) int64.  `pmask` (GPU path) restricts the evaluated
    presets (bit p); the others report 2^40.  `checker`: only the 8x8 (chroma 4x4) blocks
    with (bx + by) even are measured (the AV1 encoder's search)."""
    if _is_np(rec):
        h, w = rec.shape
        lw8 = luma_w8 or (w * (2 if chroma else 1)) // 8
        out = np.zeros((n_fb(w, h, chroma), PRESETS), np.uint64)
        _core().tv_av1_cdef_search(_p(np.ascontiguousarray(src)), _p(np.ascontiguousarray(rec)), w, h, int(chroma),
                                   _p(np.ascontiguousarray(dirs)), _p(np.ascontiguousarray(var), C.c_int32), lw8,
                                   damping, _p(out, C.c_uint64))
        return out
    import torch

    B, h, w = rec.shape
    lw8 = luma_w8 or (w * (2 if chroma else 1)) // 8
    out = torch.empty((B, n_fb(w, h, chroma), PRESETS), dtype=torch.int64, device=rec.device)
    _check(_gpu().tv_gpu_cdef_search(_t(src.contiguous()), _t(rec.contiguous()), w, h, B, int(chroma),
                                     _t(dirs), _t(var), lw8, dirs.shape[-1], damping, _t(out), _stream(rec),
                                     C.c_ulonglong(pmask), int(checker)))
    return out


def cdef_apply(rec, dirs, var, fb_preset, chroma: bool, damping: int = 5, luma_w8: int | None = None):
    """Filter with one preset index per filter block (-1 = off)."""
    if _is_np(rec):
        h, w = rec.shape
        lw8 = luma_w8 or (w * (2 if chroma else 1)) // 8
        out = np.empty_like(rec)
        _core().tv_av1_cdef_apply(_p(np.ascontiguousarray(rec)), w, h, int(chroma), _p(np.ascontiguousarray(dirs)),
                                  _p(np.ascontiguousarray(var), C.c_int32), lw8, damping,
                                  _p(np.ascontiguousarray(fb_preset, np.int8), C.c_int8), _p(out))
        return out
    import torch

    B, h, w = rec.shape
    lw8 = luma_w8 or (w * (2 if chroma else 1)) // 8
    out = torch.empty_like(rec)
    fbp = fb_preset.to(device=rec.device, dtype=torch.int8).contiguous()
    _check(_gpu().tv_gpu_cdef_apply(_t(rec.contiguous()), w, h, B, int(chroma), _t(dirs), _t(var), lw8,
                                    dirs.shape[-1], damping, _t(fbp), _t(out), _stream(rec)))
    return out


def cdef_select(sse_y: np.ndarray, sse_uv: np.ndarray, max_presets: int = 8, lam_bits: float = 0.0):
    """Encoder decision: a frame table of up to `max_presets` (luma preset, chroma preset)
    pairs (AV1 cdef_bits <= 3) and one table index per filter block, greedily minimising
    the total SSE (+ lam_bits * index bits).  Inputs (nfb, 64).  Returns (table [(py, puv)],
    per-block index, total SSE)."""
    sy = np.asarray(sse_y, np.float64)
    su = np.asarray(sse_uv, np.float64)
    pair = sy[:, :, None] + su[:, None, :]  # (nfb, 64, 64)
    nfb = pair.shape[0]
    flat = pair.reshape(nfb, -1)
    best = np.full(nfb, np.inf)
    table: list = []
    prev_total = np.inf
    for k in range(max_presets):
        bits = np.log2(max(2, len(table) + 1)) if k else 0.0
        cand = np.minimum(best[:, None], flat).sum(0) + lam_bits * bits * nfb
        j = int(np.argmin(cand))
        if cand[j] >= prev_total:
            break
        prev_total = cand[j]
        table.append((j // PRESETS, j % PRESETS))
        best = np.minimum(best, flat[:, j])
    cols = np.array([py * PRESETS + pu for py, pu in table])
    idx = np.argmin(flat[:, cols], axis=1)
    return table, idx.astype(np.int32), float(flat[np.arange(nfb), cols[idx]].sum())


# ------------------------------------------------------------------ loop restoration ----
def wiener_apply(rec, coef):
    """Per-unit taps coef (units, 6) = (h0,h1,h2,v0,v1,v2); all-zero = unit off."""
    if _is_np(rec):
        h, w = rec.shape
        out = np.empty_like(rec)
        _core().tv_av1_wiener_apply(_p(np.ascontiguousarray(rec)), w, h,
                                    _p(np.ascontiguousarray(coef, np.int32), C.c_int32), _p(out))
        return out
    import torch

    B, h, w = rec.shape
    out = torch.empty_like(rec)
    cf = torch.as_tensor(np.asarray(coef, np.int32)).to(rec.device).reshape(B, -1, 6).contiguous()
    _check(_gpu().tv_gpu_wiener_apply(_t(rec.contiguous()), w, h, B, _t(cf), _t(out), _stream(rec)))
    return out


def wiener_stats(src, rec, direction: int, other):
    """Normal equations of one separable pass (see av1.h): (units, 9) int64."""
    if _is_np(rec):
        h, w = rec.shape
        st = np.zeros((n_units(w, h), 9), np.int64)
        _core().tv_av1_wiener_stats(_p(np.ascontiguousarray(src)), _p(np.ascontiguousarray(rec)), w, h, direction,
                                    _p(np.ascontiguousarray(other, np.int32), C.c_int32), _p(st, C.c_int64))
        return st
    import torch

    B, h, w = rec.shape
    st = torch.empty((B, n_units(w, h), 9), dtype=torch.int64, device=rec.device)
    oth = torch.as_tensor(np.asarray(other, np.int32)).to(rec.device).reshape(B, -1, 3).contiguous()
    _check(_gpu().tv_gpu_wiener_stats(_t(src.contiguous()), _t(rec.contiguous()), w, h, B, direction, _t(oth),
                                      _t(st), _stream(rec)))
    return st


def _solve_wiener(st: np.ndarray) -> np.ndarray:
    """(..., 9) normal equations -> quantised, range-clipped (c0, c1, c2) taps."""
    st = np.asarray(st, np.float64)
    A = np.stack([st[..., [0, 1, 2]], st[..., [1, 3, 4]], st[..., [2, 4, 5]]], -2)
    b = st[..., 6:9]
    A = A + np.eye(3) * (1e-3 * np.trace(A, axis1=-2, axis2=-1)[..., None, None] + 1.0)
    x = np.linalg.solve(A, b[..., None])[..., 0]
    return np.clip(np.rint(x), WIENER_MIN, WIENER_MAX).astype(np.int32)


def sgr_stats(src, rec, sgr_set: int):
    if _is_np(rec):
        h, w = rec.shape
        st = np.zeros((n_units(w, h), 5), np.int64)
        _core().tv_av1_sgr_stats(_p(np.ascontiguousarray(src)), _p(np.ascontiguousarray(rec)), w, h, sgr_set,
                                 _p(st, C.c_int64))
        return st
    import torch

    B, h, w = rec.shape
    st = torch.empty((B, n_units(w, h), 5), dtype=torch.int64, device=rec.device)
    _check(_gpu().tv_gpu_sgr_stats(_t(src.contiguous()), _t(rec.contiguous()), w, h, B, sgr_set, _t(st),
                                   _stream(rec)))
    return st


def sgr_apply(rec, params):
    """Per-unit (set, w0, w1); set < 0 = unit off."""
    if _is_np(rec):
        h, w = rec.shape
        out = np.empty_like(rec)
        _core().tv_av1_sgr_apply(_p(np.ascontiguousarray(rec)), w, h,
                                 _p(np.ascontiguousarray(params, np.int32), C.c_int32), _p(out))
        return out
    import torch

    B, h, w = rec.shape
    out = torch.empty_like(rec)
    if isinstance(params, torch.Tensor):
        pr = params.to(device=rec.device, dtype=torch.int32).reshape(B, -1, 3).contiguous()
    else:
        pr = torch.as_tensor(np.asarray(params, np.int32)).to(rec.device).reshape(B, -1, 3).contiguous()
    _check(_gpu().tv_gpu_sgr_apply(_t(rec.contiguous()), w, h, B, _t(pr), _t(out), _stream(rec)))
    return out


def _solve_sgr(st: np.ndarray) -> np.ndarray:
    st = np.asarray(st, np.float64)
    H = np.stack([st[..., [0, 1]], st[..., [1, 2]]], -2) + np.eye(2) * 1.0
    x = np.linalg.solve(H, st[..., 3:5, None])[..., 0]
    return np.clip(np.rint(x), SGR_XQD_MIN, SGR_XQD_MAX).astype(np.int32)


def _unit_sse(a, b, w: int, h: int) -> np.ndarray:
    """Per-unit SSE of two (B, h, w) stacks -> (B, units)."""
    if not _is_np(a):
        import torch

        d = (a.to(torch.int32) - b.to(torch.int32)) ** 2
        B = d.shape[0]
        ph, pw = -(-h // RU) * RU, -(-w // RU) * RU
        d = torch.nn.functional.pad(d, (0, pw - w, 0, ph - h))
        return d.reshape(B, ph // RU, RU, pw // RU, RU).sum((2, 4)).reshape(B, -1).cpu().numpy()
    d = (a.astype(np.int64) - b.astype(np.int64)) ** 2
    B = d.shape[0]
    ph, pw = -(-h // RU) * RU, -(-w // RU) * RU
    d = np.pad(d, ((0, 0), (0, ph - h), (0, pw - w)))
    return d.reshape(B, ph // RU, RU, pw // RU, RU).sum((2, 4)).reshape(B, -1)


@dataclass
class LrDecision:
    kind: np.ndarray     # (B, units): 0 off, 1 Wiener, 2 self-guided
    wiener: np.ndarray   # (B, units, 6)
    sgr: np.ndarray      # (B, units, 3)
    sse_off: np.ndarray
    sse_best: np.ndarray


def loop_restoration_search(src, rec, sgr_sets=range(16), iters: int = 2) -> LrDecision:
    """Per-unit restoration decision for planes (numpy (h, w) or torch (B, h, w)): Wiener
    taps by alternating separable least squares (horizontal taps given the vertical ones
    and back, starting from identity), every SGR set with its least-squares projection
    weights; the unit SSE decides off / Wiener / SGR."""
    if _is_np(rec):
        h, w = rec.shape
        B, S, R = 1, src[None], rec[None]
        ws = lambda d, oth: wiener_stats(src, rec, d, oth[0])[None]
        wa = lambda coef: wiener_apply(rec, coef[0])[None]
        ss = lambda st: sgr_stats(src, rec, st)[None]
        sa = lambda prm: sgr_apply(rec, prm[0])[None]
    else:
        B, h, w = rec.shape
        S, R = src, rec
        ws = lambda d, oth: wiener_stats(src, rec, d, oth).cpu().numpy()
        wa = lambda coef: wiener_apply(rec, coef)
        ss = lambda st: sgr_stats(src, rec, st).cpu().numpy()
        sa = lambda prm: sgr_apply(rec, prm)
    nu = n_units(w, h)
    v = np.zeros((B, nu, 3), np.int32)
    hc = v
    for _ in range(iters):
        hc = _solve_wiener(ws(0, v))
        v = _solve_wiener(ws(1, hc))
    coef = np.ascontiguousarray(np.concatenate([hc, v], -1).astype(np.int32))
    sse_off = _unit_sse(S, R, w, h).astype(np.float64)
    sse_w = _unit_sse(S, wa(coef), w, h).astype(np.float64)
    best_s = np.full((B, nu), np.inf)
    best_p = np.full((B, nu, 3), -1, np.int32)
    for st in sgr_sets:
        xq = _solve_sgr(ss(st))
        prm = np.ascontiguousarray(np.concatenate([np.full((B, nu, 1), st, np.int32), xq], -1))
        e = _unit_sse(S, sa(prm), w, h).astype(np.float64)
        better = e < best_s
        best_s = np.where(better, e, best_s)
        best_p[better] = prm[better]
    kind = np.zeros((B, nu), np.int8)
    best = sse_off.copy()
    kind[sse_w < best] = 1
    best = np.minimum(best, sse_w)
    kind[best_s < best] = 2
    best = np.minimum(best, best_s)
    coef[kind != 1] = 0
    best_p[kind != 2] = -1
    return LrDecision(kind, coef, best_p, sse_off, best)


def loop_restoration_apply(rec, dec: LrDecision):
    """Apply the per-unit decision (Wiener units, then SGR units; the kinds are disjoint)."""
    if _is_np(rec):
        out = wiener_apply(rec, dec.wiener[0])
        sg = sgr_apply(rec, dec.sgr[0])
        m = np.repeat(np.repeat((dec.kind[0] == 2).reshape(-(-rec.shape[0] // RU), -1), RU, 0), RU, 1)
        m = m[:rec.shape[0], :rec.shape[1]]
        return np.where(m, sg, out)
    import torch

    B, h, w = rec.shape
    out = wiener_apply(rec, dec.wiener)
    sg = sgr_apply(rec, dec.sgr)
    m = torch.as_tensor(dec.kind == 2, device=rec.device).reshape(B, -(-h // RU), -(-w // RU))
    m = m.repeat_interleave(RU, 1).repeat_interleave(RU, 2)[:, :h, :w]
    return torch.where(m, sg, out)


# ------------------------------------------------------------------ whole-frame tool ----
# ------------------------------------------------------------------ deblocking ----
def lf_info(tx_w, tx_h, bs_w, bs_h, lvl_v, lvl_h, skip_inter=None) -> np.ndarray:
    """Pack per-4x4 loop-filter info words (layout: csrc/include/tv/av1_defs.h).  Sizes are
    in pixels (4..64), levels 0..63; all arrays share one (h/4, w/4) shape."""
    lg = lambda a: (np.log2(np.asarray(a)).astype(np.uint32) - 2) & 7  # noqa: E731
    word = (lg(tx_w) | lg(tx_h) << 3 | lg(bs_w) << 6 | lg(bs_h) << 9
            | (np.asarray(lvl_v, np.uint32) & 63) << 12 | (np.asarray(lvl_h, np.uint32) & 63) << 18)
    if skip_inter is not None:
        word |= (np.asarray(skip_inter, np.uint32) & 1) << 24
    return np.ascontiguousarray(word, np.uint32)


def random_lf_info(w: int, h: int, rng: np.random.Generator, chroma: bool = False, lvl_max: int = 63,
                   skip_p: float = 0.3) -> np.ndarray:
    """A random but valid partition of a plane for tests / benches: superblocks (64, or 32 in
    a 4:2:0 chroma plane) split recursively into square / half blocks, each block carrying a
    uniform tx grid of a size <= the block, one level pair and a skip && inter flag."""
    h4, w4 = h // 4, w // 4
    f = {k: np.zeros((h4, w4), np.int64) for k in ("txw", "txh", "bw", "bh", "lv", "lh", "sk")}

    def block(x, y, bw, bh):
        if x >= w or y >= h:
            return
        r = rng.random()
        if bw > 8 and bh > 8 and r < 0.35:
            hw, hh = bw // 2, bh // 2
            for dy in (0, hh):
                for dx in (0, hw):
                    block(x + dx, y + dy, hw, hh)
            return
        if bw == bh and bw > 4 and r < 0.5:
            if rng.random() < 0.5:
                block(x, y, bw, bh // 2), block(x, y + bh // 2, bw, bh // 2)
            else:
                block(x, y, bw // 2, bh), block(x + bw // 2, y, bw // 2, bh)
            return
        tw = min(bw, 64) >> int(rng.integers(0, 3))
        th = min(bh, 64) >> int(rng.integers(0, 3))
        tw, th = max(tw, 4), max(th, 4)
        if tw > 4 * th or th > 4 * tw:  # AV1 tx aspect <= 4:1
            tw = th = min(tw, th)
        sl = np.s_[y // 4:(y + bh) // 4, x // 4:(x + bw) // 4]
        f["txw"][sl], f["txh"][sl], f["bw"][sl], f["bh"][sl] = tw, th, bw, bh
        f["lv"][sl], f["lh"][sl] = rng.integers(0, lvl_max + 1), rng.integers(0, lvl_max + 1)
        f["sk"][sl] = rng.random() < skip_p

    sb = 32 if chroma else 64
    for y in range(0, h, sb):
        for x in range(0, w, sb):
            block(x, y, sb, sb)
    return lf_info(f["txw"], f["txh"], f["bw"], f["bh"], f["lv"], f["lh"], f["sk"])


def deblock(rec, info, chroma: bool = False, sharpness: int = 0, estep: int = 4):
    """AV1 deblocking loop filter (7.14) of a plane: numpy (h, w) + info (h/4, w/4) -> the
    C++ golden model; torch (B, h, w) cuda + info (B, h/4, w/4) -> one fused HIP launch
    (k_deblock, both passes per 64x64 LDS tile).  estep (GPU): edge grid in samples, 8 / 16
    only when every transform and block edge lies on it (the AV1 encoder's planes)."""
    if _is_np(rec):
        h, w = rec.shape
        out = np.empty_like(rec)
        rc = _core().tv_av1_deblock(_p(np.ascontiguousarray(rec)), w, h, int(chroma),
                                    _p(np.ascontiguousarray(info, np.uint32), C.c_uint32), sharpness, _p(out))
        if rc != 0:
            raise RuntimeError(_core().tv_av1_last_error().decode())
        return out
    import torch

    B, h, w = rec.shape
    if _is_np(info):
        info = torch.from_numpy(np.ascontiguousarray(info, np.uint32).view(np.int32))
    inf = info.to(device=rec.device, dtype=torch.int32).reshape(B, h // 4, w // 4).contiguous()
    out = torch.empty_like(rec)
    _check(_gpu().tv_gpu_av1_deblock_step(_t(rec.contiguous()), _t(out), w, h, B, int(chroma), _t(inf), sharpness,
                                          estep, _stream(rec)))
    return out


def psnr(a, b) -> float:
    if not _is_np(a):
        a, b = a.cpu().numpy(), b.cpu().numpy()
    mse = np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2)
    return float("inf") if mse == 0 else float(10 * np.log10(255.0 ** 2 / mse))


def postfilter_frames(src: tuple, rec: tuple, damping: int = 5, restore: bool = True, sgr_sets=(0, 4, 8, 10, 14),
                      lf: tuple | None = None, sharpness: int = 0):
    """AV1 in-loop filter chain on a batch of decoded I420 frames: deblocking (when `lf` =
    per-plane info maps is given), CDEF (strength search + filter), then loop restoration.
    src/rec = (Y, U, V) torch uint8 stacks (B, h, w) on the GPU (or numpy (h, w) planes on
    the CPU golden path).  Returns (filtered planes, report dict)."""
    psnr_rec = None
    if lf is not None:
        psnr_rec = [psnr(s, r) for s, r in zip(src, rec)]
        rec = tuple(deblock(r, i, c > 0, sharpness) for c, (r, i) in enumerate(zip(rec, lf)))
    Ys, Us, Vs = src
    Yr, Ur, Vr = rec
    dirs, var = cdef_dirs(Yr)
    sy = cdef_search(Ys, Yr, dirs, var, False, damping)
    su = cdef_search(Us, Ur, dirs, var, True, damping)
    sv = cdef_search(Vs, Vr, dirs, var, True, damping)
    np_in = _is_np(Yr)
    to_np = (lambda x: x) if np_in else (lambda x: x.cpu().numpy())
    sy, suv = to_np(sy).astype(np.float64), (to_np(su) + to_np(sv)).astype(np.float64)
    if np_in:
        sy, suv = sy[None], suv[None]
    tables, py, puv = [], [], []
    for b in range(sy.shape[0]):
        table, idx, _ = cdef_select(sy[b], suv[b])
        tables.append(table)
        py.append(np.array([table[i][0] for i in idx], np.int8))
        puv.append(np.array([table[i][1] for i in idx], np.int8))
    if np_in:
        out = [cdef_apply(Yr, dirs, var, py[0], False, damping), cdef_apply(Ur, dirs, var, puv[0], True, damping),
               cdef_apply(Vr, dirs, var, puv[0], True, damping)]
    else:
        import torch

        PY, PUV = torch.as_tensor(np.stack(py)), torch.as_tensor(np.stack(puv))
        out = [cdef_apply(Yr, dirs, var, PY, False, damping), cdef_apply(Ur, dirs, var, PUV, True, damping),
               cdef_apply(Vr, dirs, var, PUV, True, damping)]
    rep = {"psnr_in": [psnr(s, r) for s, r in zip(src, rec)], "cdef_tables": tables}
    if psnr_rec is not None:
        rep["psnr_in"], rep["psnr_deblock"] = psnr_rec, rep["psnr_in"]
    rep["psnr_cdef"] = [psnr(s, o) for s, o in zip(src, out)]
    if restore:
        lr = [loop_restoration_search(s, o, sgr_sets=sgr_sets) for s, o in zip(src, out)]
        out = [loop_restoration_apply(o, d) for o, d in zip(out, lr)]
        rep["lr_units"] = [{k: int((d.kind == i).sum()) for i, k in enumerate(("off", "wiener", "sgr"))} for d in lr]
        rep["psnr_lr"] = [psnr(s, o) for s, o in zip(src, out)]
    return tuple(out), rep


def range_coder_roundtrip(symbols, alphabet, contexts, adapt: bool = True):
    """Encode a symbol sequence with the AV1 range coder (adaptive CDFs per context) and
    decode it back.  Returns (bytes, decoded symbols)."""
    from .._native import Bytes

    sym = np.ascontiguousarray(symbols, np.int32)
    alp = np.ascontiguousarray(alphabet, np.int32)
    ctx = np.ascontiguousarray(contexts, np.int32)
    if not (len(sym) == len(alp) == len(ctx)):
        raise ValueError("length mismatch")
    if ((alp < 2) | (alp > 16)).any() or (sym < 0).any() or (sym >= alp).any():
        raise ValueError("symbols must be in [0, alphabet), alphabet in 2..16")
    dec = np.zeros_like(sym)
    buf = Bytes()
    lib = _core()
    rc = lib.tv_av1_rc_roundtrip(sym.ctypes.data_as(_vp), alp.ctypes.data_as(_vp), ctx.ctypes.data_as(_vp), len(sym),
                                 int(ctx.max()) + 1 if len(ctx) else 1, int(adapt), _vp(buf.h), dec.ctypes.data_as(_vp))
    if rc != 0:
        raise RuntimeError(lib.tv_av1_last_error().decode())
    return buf.tobytes(), dec


# ------------------------------------------------------------------- transforms ----
TX_TYPES = {"dct": 0, "adst": 1, "flipadst": 2, "idtx": 3}
_basis_cache: dict = {}


def txfm_basis(kind: str | int, n: int) -> np.ndarray:
    """(n, n) int32 basis of a 1-D AV1 transform (row k = basis function k)."""
    t = TX_TYPES.get(kind, kind)
    out = np.zeros((n, n), np.int32)
    lib = _core()
    lib.tv_av1_txfm_basis.argtypes = [C.c_int, C.c_int, C.POINTER(C.c_int32)]
    if lib.tv_av1_txfm_basis(int(t), n, _p(out, C.c_int32)) != 0:
        raise ValueError(f"unsupported transform {kind} x {n}")
    return out


def txfm2d(blocks, col: str = "dct", row: str = "dct", inverse: bool = False):
    """Forward (columns then rows) or inverse AV1 2-D transform of N x N int16 blocks:
    numpy (nblk, N, N) -> C++ golden model; torch cuda -> MFMA kernels (bit-identical)."""
    tc, tr = TX_TYPES.get(col, col), TX_TYPES.get(row, row)
    nblk, n, n2 = blocks.shape
    if n != n2 or n not in (4, 8, 16, 32, 64):
        raise ValueError("blocks must be (nblk, N, N) with N in 4..64")
    log2n = n.bit_length() - 1
    if _is_np(blocks):
        x = np.ascontiguousarray(blocks, np.int16)
        out = np.empty_like(x)
        lib = _core()
        lib.tv_av1_txfm_ref.argtypes = [C.POINTER(C.c_int16), C.POINTER(C.c_int16)] + [C.c_int] * 5
        lib.tv_av1_txfm_ref.restype = C.c_int
        if lib.tv_av1_txfm_ref(_p(x, C.c_int16), _p(out, C.c_int16), nblk, log2n, tc, tr, int(inverse)) != 0:
            raise ValueError(lib.tv_av1_last_error().decode())
        return out
    import torch

    key = (tc, tr, n, blocks.device)
    if key not in _basis_cache:
        _basis_cache[key] = (torch.from_numpy(txfm_basis(tc, n)).to(blocks.device),
                             torch.from_numpy(txfm_basis(tr, n)).to(blocks.device))
    bc, br = _basis_cache[key]
    x = blocks.to(torch.int16).contiguous()
    out = torch.empty_like(x)
    lib = _gpu()
    lib.tv_gpu_av1_txfm.restype = C.c_int
    lib.tv_av1_txfm_last_error.restype = C.c_char_p
    rc = lib.tv_gpu_av1_txfm(_t(x), _t(out), nblk, log2n, int(inverse), _t(bc), _t(br), _stream(x))
    if rc != 0:
        raise RuntimeError(lib.tv_av1_txfm_last_error().decode())
    return out
