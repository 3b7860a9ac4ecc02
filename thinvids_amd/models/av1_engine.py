"""GPU AV1 encode engine (BASELINE config #4) for one MI355X.

Encodes a BATCH of B independent GOP-aligned segments in lock-step: frame t of every
segment is one launch of each kernel (grid = blocks x segments).  Per frame, on the
current HIP stream:

    key frame   k_av1e_intra (anti-diagonal wavefront of 16x16 blocks)
    P frame     k_av1e_inter (full-pel +-16 LDS search, quarter-pel refine, recon)
    both        k_av1e_lfinfo -> k_deblock (Y, U, V) -> k_cdef_dir -> k_av1e_cdef_skip ->
                k_cdef_search (Y, U, V) -> k_av1e_cdef_choose -> k_cdef_apply -> next reference

Decisions (mode / MV words, quantised levels, CDEF tables and indices) of the whole GOP
stay resident in HBM; at the end of the GOP the nonzero transform blocks are compacted on
the device and copied to the host once, and a CPU thread pool writes every segment's OBU
temporal units (range coder) while the GPU moves on to the next GOP.

Bit-exact with the C++ golden encoder (``av1.golden_encode``), whose streams decode
bit-exactly with dav1d (tests/test_av1_conformance.py), and with the decoder oracle
(``av1.decode``): tests/test_av1_codec.py.
"""
from __future__ import annotations

import concurrent.futures as cf
import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

from . import av1 as av1m

_vp = C.c_void_p


def _cdef_mask(pri, sec) -> int:
    return sum(1 << (p * 4 + s) for p in pri for s in sec)


# evaluated CDEF presets: av1_enc.h kCdefMaskY / kCdefMaskUV
CDEF_MASK_Y = _cdef_mask((0, 1, 2, 3, 5, 7, 10, 13), (0, 2))
CDEF_MASK_UV = _cdef_mask((0, 2, 4, 7), (0, 2))


def _gpu():
    from .._native import gpu_lib

    lib = gpu_lib()
    if not getattr(lib, "_av1e_sigs", False):
        for n in ("tv_av1e_inter", "tv_av1e_intra", "tv_av1e_lfinfo", "tv_av1e_cdef_choose", "tv_av1e_lr_solve",
                  "tv_av1e_unit_sse", "tv_av1e_merge", "tv_av1e_tb_len", "tv_av1e_tb_pack", "tv_av1e_cdef_skip"):
            getattr(lib, n).restype = C.c_int
        lib.tv_av1e_last_error.restype = C.c_char_p
        lib._av1e_sigs = True
    return lib


def _ok(rc: int):
    if rc != 0:
        raise RuntimeError(_gpu().tv_av1e_last_error().decode())


def _p(t):
    return _vp(t.data_ptr())


LR_SETS = (4, 10)  # av1_enc.h lr_set()


def lr_grid(size: int) -> int:
    """Restoration units along a plane dimension (av1_defs.h lr_count_units, 64-px units)."""
    return max(1, (size + 32) // 64)


def lr_rate_cost(q: int) -> int:
    """Rate of a restored unit in SSE units (av1_enc.h lr_rate_cost)."""
    a = av1m.ac_q(q)
    return ((a * a * 9) >> 10) * 16


def lf_level(q: int) -> int:
    """Frame loop-filter level of a q-index (av1_enc.h lf_level_for_q)."""
    return min(63, max(0, (av1m.ac_q(q) * 20723 + 1015158) >> 18))


@dataclass
class GopHost:
    """Host copy of one GOP's decisions for the entropy stage."""
    nframes: int
    mode: np.ndarray     # (F, B, nb) uint32
    mv: np.ndarray
    tabs: np.ndarray     # (F, B, 16) uint8
    fbidx: np.ndarray    # (F, B, nfb) int8
    packed: list         # per plane: (eob-truncated scan-order TBs int16, start offsets (F, B) int64)
    sse: np.ndarray      # (F, B, 3) int64
    key: list            # per frame
    qm: np.ndarray = None  # (F, B) q-index per frame and segment
    lr: np.ndarray = None  # (F, B, 3, nu, 3) restoration units (set | -1, xqd0, xqd1)


class Av1GpuEngine:
    """B segments x one GOP per call on one GPU; see module docstring."""

    def __init__(self, width: int, height: int, batch: int, qindex: int = 100, device: int = 0,
                 threads: int | None = None, cascade: bool = True):
        import torch

        self.cascade = bool(cascade)  # constant q: the low-delay q cascade (av1.cascade_qmap)
        self.torch = torch
        self.w, self.h, self.B, self.q = width, height, batch, int(qindex)
        self.W, self.H = av1m.coded_size(width, height)
        self.dev = torch.device("cuda", device)
        self.nb = (self.W // 16) * (self.H // 16)
        self.nfb = ((self.W + 63) // 64) * ((self.H + 63) // 64)
        self.nu = av1m.lr_units(self.W, self.H)
        self.lr_enabled = True
        self.lvl = self._lf_level()
        self.damping = 3 + (self.q >> 6)
        B, H, W = batch, self.H, self.W
        u8 = dict(dtype=torch.uint8, device=self.dev)
        mk = lambda: (torch.zeros((B, H, W), **u8), torch.zeros((B, H // 2, W // 2), **u8),
                      torch.zeros((B, H // 2, W // 2), **u8))
        self.src, self.rec, self.fin = mk(), mk(), mk()
        self.pool = cf.ThreadPoolExecutor(max_workers=threads or min(32, os.cpu_count() or 8))
        self._gop_cap = 0
        self.lock = None  # set by the worker's engine cache
        self.staging = None
        self._copy_stream = torch.cuda.Stream(self.dev)
        self._copy_pool = cf.ThreadPoolExecutor(max_workers=1)

    def _lf_level(self, q: int | None = None) -> int:
        return lf_level(self.q if q is None else q)

    _NAMES = ("mode", "mv", "ly", "lu", "lv", "tabs", "fbidx", "sse", "lr")

    def _alloc_gop(self, F: int):
        """Two GOP decision buffers (slots): the GPU fills one while the previous GOP's is
        compacted and copied to the host on the copy stream (encode_gop(async_host=True))."""
        torch = self.torch
        if F <= self._gop_cap:
            return
        B, nb, nfb = self.B, self.nb, self.nfb
        d = self.dev
        self._slots = []
        for _ in range(2):
            self._slots.append({
                "mode": torch.zeros((F, B, nb), dtype=torch.int32, device=d),
                "mv": torch.zeros((F, B, nb), dtype=torch.int32, device=d),
                "ly": torch.zeros((F, B, nb, 256), dtype=torch.int16, device=d),
                "lu": torch.zeros((F, B, nb, 64), dtype=torch.int16, device=d),
                "lv": torch.zeros((F, B, nb, 64), dtype=torch.int16, device=d),
                "tabs": torch.zeros((F, B, 16), dtype=torch.uint8, device=d),
                "fbidx": torch.zeros((F, B, nfb), dtype=torch.int8, device=d),
                "sse": torch.zeros((F, B, 3), dtype=torch.int64, device=d),
                "lr": torch.zeros((F, B, 3, self.nu, 3), dtype=torch.int32, device=d),
            })
        self._slot_busy = [None, None]
        self._slot = 0
        self._gop_cap = F

    def _use_slot(self):
        s = self._slot
        self._slot ^= 1
        if self._slot_busy[s] is not None:  # the previous GOP in this slot is still being collected
            self._slot_busy[s].result()
            self._slot_busy[s] = None
        for n in self._NAMES:
            setattr(self, "g_" + n, self._slots[s][n])
        return s

    # ------------------------------------------------------------------ one frame ----
    def _frame(self, t: int, key: bool, nseg: int, qarr, lvl, q_rate):
        from ..ops import av1 as ops

        torch = self.torch
        lib = _gpu()
        st = _vp(torch.cuda.current_stream(self.dev).cuda_stream)
        W, H, B, q = self.W, self.H, nseg, self.q
        sy, su, sv = (x[:B] for x in self.src)
        ry, ru, rv = (x[:B] for x in self.rec)
        fy, fu, fv = (x[:B] for x in self.fin)
        mode, mv = self.g_mode[t, :B], self.g_mv[t, :B]
        ly, lu, lv = self.g_ly[t, :B], self.g_lu[t, :B], self.g_lv[t, :B]
        if key:
            _ok(lib.tv_av1e_intra(_p(sy), _p(su), _p(sv), _p(ry), _p(ru), _p(rv), _p(mode), _p(mv), _p(ly), _p(lu),
                                  _p(lv), W, H, B, _p(qarr), st))
        else:
            if getattr(self, "_mvtmp", None) is None:
                self._mvtmp = torch.empty(self.B * self.nb, dtype=torch.int32, device=self.dev)
                self._satd = torch.empty(self.B, dtype=torch.int64, device=self.dev)  # per-segment frame SATD
                # refinement memo: 2 x [B][nb] x (11 MV words + 11 SATDs + a count)
                self._memo = torch.empty(2 * self.B * self.nb * (11 * 8 + 1), dtype=torch.uint8, device=self.dev)
            _ok(lib.tv_av1e_inter(_p(sy), _p(su), _p(sv), _p(fy), _p(fu), _p(fv), _p(ry), _p(ru), _p(rv), _p(mode),
                                  _p(mv), _p(self._mvtmp), _p(self._satd), _p(self._memo), _p(ly), _p(lu), _p(lv), W, H,
                                  B, _p(qarr), st))
            _ok(lib.tv_av1e_merge(_p(mode), _p(mv), W, H, B, st))
        iy = torch.empty((B, H // 4, W // 4), dtype=torch.int32, device=self.dev)
        iu = torch.empty((B, H // 8, W // 8), dtype=torch.int32, device=self.dev)
        iv = torch.empty_like(iu)
        _ok(lib.tv_av1e_lfinfo(_p(mode), W, H, B, _p(lvl), _p(iy), _p(iu), _p(iv), st))
        # every transform / block edge of the encoder's planes is on the 16 (luma) / 8
        # (chroma) grid: blocks are 16x16 or merged 32 / 64 with one TX per plane
        dy = ops.deblock(ry, iy, False, 0, estep=16)
        du = ops.deblock(ru, iu, True, 0, estep=8)
        dv = ops.deblock(rv, iv, True, 0, estep=8)
        dirs, var = ops.cdef_dirs(dy)
        _ok(lib.tv_av1e_cdef_skip(_p(mode), _p(dirs), W, H, B, st))  # skip blocks are not filtered
        se_y = ops.cdef_search(sy, dy, dirs, var, False, self.damping, pmask=CDEF_MASK_Y, checker=True)
        se_u = ops.cdef_search(su, du, dirs, var, True, self.damping, luma_w8=W // 8, pmask=CDEF_MASK_UV, checker=True)
        se_v = ops.cdef_search(sv, dv, dirs, var, True, self.damping, luma_w8=W // 8, pmask=CDEF_MASK_UV, checker=True)
        py = torch.empty((B, self.nfb), dtype=torch.int8, device=self.dev)
        puv = torch.empty_like(py)
        _ok(lib.tv_av1e_cdef_choose(_p(se_y), _p(se_u), _p(se_v), _p(mode), W, H, B, _p(self.g_tabs[t, :B]),
                                    _p(self.g_fbidx[t, :B]), _p(py), _p(puv), st))
        self.fin = (ops.cdef_apply(dy, dirs, var, py, False, self.damping),
                    ops.cdef_apply(du, dirs, var, puv, True, self.damping, luma_w8=W // 8),
                    ops.cdef_apply(dv, dirs, var, puv, True, self.damping, luma_w8=W // 8))
        if self.lr_enabled:
            self.fin = self._restore(t, B, q_rate, (dy, du, dv))
        w, h = self.w, self.h
        if B < self.B:  # keep full-batch planes: the slice's final frames become the reference
            fin = [torch.empty_like(x) for x in self.src]
            for full, part in zip(fin, self.fin):
                full[:B].copy_(part)
            self.fin = tuple(fin)
        for c, (s, f) in enumerate(zip(self.src, self.fin)):
            self.g_sse[t, :B, c] = self._unit_sse(s[:B], f[:B], w >> (c > 0), h >> (c > 0)).sum(dim=1)

    def _unit_sse(self, a, b, vw: int | None = None, vh: int | None = None):
        """(B, h, w) uint8 pair -> per-64x64-unit SSE (B, units) int64 (ceil layout) over
        the valid region vw x vh (default: the whole plane); one fused kernel."""
        torch = self.torch
        B, h, w = a.shape
        out = torch.empty((B, (-(-h // 64)) * (-(-w // 64))), dtype=torch.int64, device=self.dev)
        _ok(_gpu().tv_av1e_unit_sse(_p(a), _p(b), w, h, w if vw is None else vw, h if vh is None else vh, B, _p(out),
                                    _vp(torch.cuda.current_stream(self.dev).cuda_stream)))
        return out

    def _restore(self, t: int, B: int, rate, dbk):
        """Normative self-guided restoration search + apply on the CDEF output (7.17 unit
        grid and stripes; `dbk` = the deblocked pre-CDEF planes the stripe edges read): the
        golden encoder's per-unit off / set-4 / set-10 choice (SSE + rate, first minimum), one
        fused k_sgr_select launch per plane."""
        from ..ops import av1 as ops

        torch = self.torch
        st = _vp(torch.cuda.current_stream(self.dev).cuda_stream)
        rate = rate.to(torch.int64).contiguous()
        out = []
        for p, (S, X, D) in enumerate(zip((x[:B] for x in self.src), self.fin, dbk)):
            h, w = X.shape[1], X.shape[2]
            nu = lr_grid(w) * lr_grid(h)
            prm = torch.empty((B, nu, 3), dtype=torch.int32, device=self.dev)
            o = torch.empty_like(X)
            rc = ops._gpu().tv_gpu_sgr_select(_p(S), _p(X), _p(D), w, h, 1 if p else 0, B, _p(rate), _p(prm),
                                              _p(o), st)
            if rc != 0:
                raise RuntimeError(ops._gpu().tv_av1_gpu_last_error().decode())
            self.g_lr[t, :B, p, :nu] = prm
            out.append(o)
        return tuple(out)

    def encode_gop(self, nframes: int, load_frame, nseg: int | None = None, qmap=None, async_host: bool = False):
        """Run the GPU part of one GOP for all B segments.  load_frame(t, (Y, U, V)) fills
        the coded-size source planes [B, H, W] of frame t (device tensors).  `qmap`
        (optional (nframes, nseg) ints): per-frame, per-segment q-index from rate control
        (2-pass / CRF plans); None = the engine's constant q-index.  Returns the host copy
        of the decisions (one device->host transfer of compacted levels).  async_host=True
        returns a Future of it instead: the copy runs on a copy stream / thread behind the next
        GOP's kernels (double-buffered decision slots)."""
        torch = self.torch
        nseg = nseg or self.B
        if not 1 <= nseg <= self.B:
            raise ValueError(f"nseg {nseg} outside 1..{self.B}")
        self._alloc_gop(nframes)
        slot = self._use_slot()
        if qmap is None:
            col = av1m.cascade_qmap(self.q, nframes) if self.cascade else [self.q] * nframes
            qm = np.repeat(np.asarray(col, np.int32)[:, None], nseg, axis=1)
        else:
            qm = np.clip(np.asarray(qmap, np.int32).reshape(nframes, nseg), 1, 255)
        lv = np.array([[[lf_level(int(x))] * 4 for x in row] for row in qm], np.int32)
        # pinned + non_blocking: a pageable upload would block the host on the previous
        # GOP's kernels (the stream drains before this GOP's first launch)
        up = lambda a: torch.from_numpy(np.ascontiguousarray(a)).pin_memory().to(self.dev, non_blocking=True)
        qd = up(qm)
        ld = up(lv)
        rd = up(np.array([[lr_rate_cost(int(x)) for x in row] for row in qm], np.int64))
        self._keep = (qd, ld, rd)
        if not self.lr_enabled:
            self.g_lr[:nframes, :nseg, :, :, 0] = -1
        for t in range(nframes):
            load_frame(t, self.src)
            self._frame(t, t == 0, nseg, qd[t], ld[t], rd[t])
        self.nseg = nseg
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.dev))
        S = self._slots[slot]
        if not async_host:
            return self._collect(S, ev, nframes, nseg, qm)
        fut = self._copy_pool.submit(self._collect, S, ev, nframes, nseg, qm)
        self._slot_busy[slot] = fut
        return fut

    def _collect(self, S: dict, ev, F: int, nseg: int, qm) -> GopHost:
        """Pack the nonzero TBs of a GOP slot eob-truncated in scan order on the copy stream
        (after `ev`: k_av1e_tb_len -> cumsum -> k_av1e_tb_pack) and copy every decision
        array to the host."""
        torch = self.torch
        torch.cuda.set_device(self.dev)
        cs = self._copy_stream
        lib = _gpu()
        Bmax, nb = S["mode"].shape[1], S["mode"].shape[2]
        ntb = F * nseg * nb
        with torch.cuda.stream(cs):
            cs.wait_event(ev)
            st = _vp(cs.cuda_stream)
            lens, ends = [], []
            for p, k in enumerate(("ly", "lu", "lv")):
                ln = torch.empty(ntb, dtype=torch.int32, device=self.dev)
                _ok(lib.tv_av1e_tb_len(_p(S[k]), _p(S["mode"]), C.c_long(ntb), nb, nseg, Bmax, p, _p(ln), st))
                lens.append(ln)
                ends.append(torch.cumsum(ln, 0, dtype=torch.int64))
            totals = torch.stack([e[-1] for e in ends]).cpu().tolist()
            outs = []
            for p, k in enumerate(("ly", "lu", "lv")):
                o = torch.empty(max(1, totals[p]), dtype=torch.int16, device=self.dev)
                _ok(lib.tv_av1e_tb_pack(_p(S[k]), _p(lens[p]), _p(ends[p]), C.c_long(ntb), nb, nseg, Bmax, p, _p(o),
                                        st))
                outs.append((o, (ends[p] - lens[p]).view(F, nseg, nb)[:, :, 0]))
            host = GopHost(
                nframes=F,
                mode=S["mode"][:F, :nseg].cpu().numpy().view(np.uint32),
                mv=S["mv"][:F, :nseg].cpu().numpy().view(np.uint32),
                tabs=S["tabs"][:F, :nseg].cpu().numpy(),
                fbidx=S["fbidx"][:F, :nseg].cpu().numpy(),
                packed=[(o[:max(1, t)].cpu().numpy(), off.cpu().numpy().astype(np.int64))
                        for (o, off), t in zip(outs, totals)],
                sse=S["sse"][:F, :nseg].cpu().numpy(),
                key=[t == 0 for t in range(F)],
                qm=qm,
                lr=S["lr"][:F, :nseg].cpu().numpy(),
            )
        return host

    # ------------------------------------------------------------------ entropy ------
    def write_segment(self, g: GopHost, b: int) -> list:
        """Temporal units of segment b of a GOP (runs on a pool thread; the native writer
        releases the GIL)."""
        tus = []
        wr = av1m.StreamWriter(self.w, self.h)
        for t in range(g.nframes):
            tabs = g.tabs[t, b]
            q = int(g.qm[t, b])
            fp = av1m.frame_params(g.key[t], q, [lf_level(q)] * 4, 0, self.damping, tabs[:8], tabs[8:])
            lev = [pk[0][pk[1][t, b]:] for pk in g.packed]  # eob-truncated scan-order TBs
            tus.append(wr.write(fp, np.ascontiguousarray(g.mode[t, b]), np.ascontiguousarray(g.mv[t, b]), lev[0],
                                lev[1], lev[2], np.ascontiguousarray(g.fbidx[t, b]), packed=2, seq_header=g.key[t],
                                lr=np.ascontiguousarray(g.lr[t, b])))
        return tus

    def submit_entropy(self, g: GopHost) -> list:
        return [self.pool.submit(self.write_segment, g, b) for b in range(g.mode.shape[1])]

    def psnr(self, g: GopHost) -> dict:
        n = g.sse.shape[0] * g.sse.shape[1]
        px = [self.w * self.h, (self.w // 2) * (self.h // 2), (self.w // 2) * (self.h // 2)]
        out = {}
        for c, k in enumerate("yuv"):
            mse = g.sse[:, :, c].sum() / (n * px[c])
            out[k] = float("inf") if mse == 0 else float(10 * np.log10(255.0 ** 2 / mse))
        mse = g.sse.sum() / (n * sum(px))
        out["yuv"] = float("inf") if mse == 0 else float(10 * np.log10(255.0 ** 2 / mse))
        return out

    def close(self):
        self._copy_pool.shutdown(wait=True)
        self.pool.shutdown(wait=True)
