"""ABR ladder on one MI355X: HDR10 source -> tone-map -> N Lanczos rungs -> N HEVC engines,
with every intermediate resident in HBM (BASELINE.json config #5: "8K HDR10 -> 5-rung ABR
ladder (tone-map + Lanczos downscale)"; SURVEY.md P10 ABR-ladder fan-out, K2 scale, K15
tone-map).

The reference encodes one target height per job (reference worker/tasks.py:57,
:426-441, ``scale=-2:H`` at :475-500) and re-reads the source for every rendition.  Here one
pass over the source feeds every rung:

    k_synth_p010 (or caller P010)      n x 8K P010, one launch per segment chunk
      -> k_tonemap_pq (batched)        PQ -> SDR BT.709 I420, once per source frame
      -> k_resize_h/v (batched)        per rung and plane, written straight into the rung
                                       engine's staging buffer at its coded size with the
                                       edge padding folded into the V pass
      -> GpuEngine.encode_device       D2D into the engine, rungs encoded concurrently
                                       (one host thread each; ctypes drops the GIL)

so a source frame crosses PCIe zero times and only compact coefficients come back for
CABAC.  Multi-GPU: every rank runs its own ladder on its own segment range (direct-source
range parallelism) and bitstreams are gathered over RCCL (``bench.py --ladder``,
``parallel/node_job.py --ladder`` for file inputs).
"""
from __future__ import annotations

import ctypes as C
import threading
from functools import lru_cache

from ..worker.helpers import output_geometry
from .gpu_engine import GpuEngine, default_threads
from .hevc import coded_size

LADDER = (2160, 1440, 1080, 720, 480)
SRC_8K = (7680, 4320)


def plan_rungs(src_w: int, src_h: int, heights=LADDER) -> list[tuple[int, int]]:
    """Rung display sizes (``scale=-2:H`` semantics, never upscaling); duplicates dropped."""
    out = []
    for h in heights:
        g = output_geometry(src_w, src_h, h)
        if g not in out:
            out.append(g)
    return out


def split_threads(rungs, total: int) -> list[int]:
    """CABAC threads per rung engine, proportional to its pixel count (entropy work scales
    with coded area), at least 2 each."""
    px = [w * h for w, h in rungs]
    s = float(sum(px))
    return [max(2, int(round(total * p / s))) for p in px]


def staging_layout(w: int, h: int) -> dict:
    """Byte offsets / strides of one coded-size I420 frame in an engine staging buffer."""
    cw, ch = coded_size(w, h)
    ysz, csz = cw * ch, (cw // 2) * (ch // 2)
    return {"cw": cw, "ch": ch, "fsz": ysz + 2 * csz,
            "planes": [(0, w, h, cw, cw, ch), (ysz, w // 2, h // 2, cw // 2, cw // 2, ch // 2),
                       (ysz + csz, w // 2, h // 2, cw // 2, cw // 2, ch // 2)]}


@lru_cache(maxsize=64)
def _tables(n_in: int, n_out: int, a: int, dev_index: int):
    import torch

    from ..ops.resize import filter_table

    s, _, wq = filter_table(n_in, n_out, a)
    dev = torch.device("cuda", dev_index)
    return torch.from_numpy(s.copy()).to(dev), torch.from_numpy(wq.copy()).to(dev), int(wq.shape[1])


@lru_cache(maxsize=64)
def resize2d_plan(sw: int, sh: int, dw: int, dh: int, pw: int, ph: int, a: int = 3,
                  budget: int = 40 * 1024) -> tuple[int, int, int]:
    """(th, wp, smem) for the fused k_resize2d: the tallest output tile (64 wide, th rows)
    whose staged source window (R rows x wp bytes) + int16 intermediate (R x 64) fits the
    LDS budget, over every tile of the plane (exact, from the filter tables).  40 KB keeps 4
    workgroups (16 waves) per CU.  (0, 0, 0) -> the two-pass kernels."""
    import numpy as np

    from ..ops.resize import filter_table

    ix, _, wxq = filter_table(sw, dw, a)
    iy, _, wyq = filter_table(sh, dh, a)
    tx, ty = wxq.shape[1], wyq.shape[1]
    x0 = np.arange(0, pw, 64)
    wmax = int((ix[np.minimum(x0 + 63, dw - 1)] + tx - ix[np.minimum(x0, dw - 1)]).max())
    wp = (wmax + 3) & ~3
    for th in (64, 48, 32, 24, 16, 12, 8, 4, 2, 1):
        y0 = np.arange(0, ph, th)
        rmax = int((iy[np.minimum(y0 + th - 1, dh - 1)] + ty - iy[np.minimum(y0, dh - 1)]).max())
        smem = ((rmax * wp + 15) & ~15) + rmax * 64 * 2
        if smem <= budget:
            return th, wp, smem
    return 0, 0, 0


def _ops():
    from .._native import gpu_lib

    lib = gpu_lib()
    if not getattr(lib, "_abr_sigs", False):
        vp, ci, cl = C.c_void_p, C.c_int, C.c_long
        lib.tv_synth_p010.argtypes = [vp, vp, ci, ci, ci, ci, C.c_uint32, vp]
        lib.tv_tonemap_pq_batch.argtypes = [vp, vp, ci, ci, ci, vp, C.c_float, C.c_float, vp]
        lib.tv_resize_batch.argtypes = [vp, ci, ci, ci, cl, vp, ci, ci, ci, cl, ci, ci, ci,
                                        vp, vp, ci, vp, vp, ci, vp, ci, ci, ci, vp]
        lib.tv_ops_last_error.restype = C.c_char_p
        lib._abr_sigs = True
    return lib


def _ok(lib, rc: int) -> None:
    if rc != 0:
        raise RuntimeError(lib.tv_ops_last_error().decode())


class AbrLadder:
    """One source resolution, N rungs, `segments` GOP-aligned segments of `gop` frames per
    call.  HBM: chunk P010 (2 B/px x 1.5) + chunk SDR I420 + resize scratch + per-rung
    staging (segments x gop coded frames) — ~11 GB at 8K, 16 x 16 frames."""

    def __init__(self, src_w: int = SRC_8K[0], src_h: int = SRC_8K[1], heights=LADDER, qp: int = 27,
                 segments: int = 16, gop: int = 16, device: int = 0, threads: int | None = None, seed: int = 1,
                 src_peak: float = 1000.0, dst_peak: float = 100.0, search_range: int = 64,
                 concurrent: bool = True, sao: bool = False, cascade: bool = True, slots: int = 2,
                 fused: bool = True):
        import torch

        if (src_w | src_h) & 1:
            raise ValueError("source must have even dimensions")
        self.src_w, self.src_h = src_w, src_h
        self.segments, self.gop, self.seed = segments, gop, seed
        self.src_peak, self.dst_peak = src_peak, dst_peak
        self.concurrent, self.cascade, self.fused = concurrent, cascade, fused
        self.dev = torch.device("cuda", device)
        self.rungs = plan_rungs(src_w, src_h, heights)
        self.layouts = [staging_layout(w, h) for w, h in self.rungs]
        total = threads or default_threads()
        self.engines = [GpuEngine(width=w, height=h, qp=qp, batch=segments, gop=gop, search_range=search_range,
                                  seed=seed, threads=t, device=device, sao=sao)
                        for (w, h), t in zip(self.rungs, split_threads(self.rungs, total))]
        u8, i16, u16 = torch.uint8, torch.int16, torch.uint16
        # slots: staging sets, so the pre-processing of call k+1 can fill one while the
        # engines read the other (prepare_synthetic(..., slot) / encode_prepared(n, slot))
        self.staging_slots = [[torch.empty((segments * gop, L["fsz"]), dtype=u8, device=self.dev)
                               for L in self.layouts] for _ in range(max(1, slots))]
        self.staging = self.staging_slots[0]
        self.src_fsz = src_w * src_h * 3 // 2
        self.y16 = torch.empty((gop, src_h, src_w), dtype=u16, device=self.dev)
        self.uv16 = torch.empty((gop, src_h // 2, src_w), dtype=u16, device=self.dev)
        self.sdr = torch.empty((gop, self.src_fsz), dtype=u8, device=self.dev)
        self.tmp = torch.empty(gop * src_h * max(w for w, _ in self.rungs) if not fused else 1, dtype=i16,
                               device=self.dev)
        self.lib = _ops()

    def close(self) -> None:
        for e in self.engines:
            e.close()
        self.engines = []

    # ------------------------------------------------------------ pre-processing
    def _stream(self):
        import torch

        return C.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)

    def synth_p010(self, t0: int, n: int) -> None:
        """Seeded synthetic HDR10 frames t0..t0+n-1 into the chunk buffers."""
        _ok(self.lib, self.lib.tv_synth_p010(self.y16.data_ptr(), self.uv16.data_ptr(), self.src_w, self.src_h, n,
                                             t0, self.seed & 0xFFFFFFFF, self._stream()))

    def ladder_chunk(self, slot0: int, n: int, slot: int = 0) -> None:
        """Tone-map the n chunk frames (in y16/uv16) and resample them into every rung's
        staging frames slot0..slot0+n-1 of staging set `slot`.  With `cascade` the lower
        rungs are resampled from the first (largest) rung instead of the full source: the
        first rung is already band-limited above every lower rung's Nyquist, and the H pass
        then reads a 4x smaller picture (8K -> 4K -> 1440p/1080p/720p/480p)."""
        lib, st = self.lib, self._stream()
        staging = self.staging_slots[slot]
        _ok(lib, lib.tv_tonemap_pq_batch(self.y16.data_ptr(), self.uv16.data_ptr(), self.src_w, self.src_h, n,
                                         self.sdr.data_ptr(), C.c_float(self.src_peak), C.c_float(self.dst_peak), st))
        sw, sh = self.src_w, self.src_h
        full = (self.sdr.data_ptr(), self.src_fsz,
                [(0, sw, sh, sw), (sw * sh, sw // 2, sh // 2, sw // 2), (sw * sh * 5 // 4, sw // 2, sh // 2, sw // 2)])
        L0 = self.layouts[0]
        first = (staging[0].data_ptr() + slot0 * L0["fsz"], L0["fsz"],
                 [(off, w, h, stride) for off, w, h, stride, _, _ in L0["planes"]])
        for r, (L, buf) in enumerate(zip(self.layouts, staging)):
            src_ptr, sfs, src_planes = first if (self.cascade and r > 0) else full
            base = buf.data_ptr() + slot0 * L["fsz"]
            for (soff, pw_, ph_, sstride), (doff, dw, dh, dstride, pw, ph) in zip(src_planes, L["planes"]):
                ix, wx, tx = _tables(pw_, dw, 3, self.dev.index)
                iy, wy, ty = _tables(ph_, dh, 3, self.dev.index)
                th, wp, smem = resize2d_plan(pw_, ph_, dw, dh, pw, ph) if self.fused else (0, 0, 0)
                _ok(lib, lib.tv_resize_batch(src_ptr + soff, pw_, ph_, sstride, sfs, base + doff, dw, dh, dstride,
                                             L["fsz"], pw, ph, n, ix.data_ptr(), wx.data_ptr(), tx, iy.data_ptr(),
                                             wy.data_ptr(), ty, self.tmp.data_ptr(), th, wp, smem, st))

    def prepare_synthetic(self, starts, slot: int = 0) -> None:
        """Segment b = synthetic frames [starts[b], starts[b] + gop)."""
        if not 1 <= len(starts) <= self.segments:
            raise ValueError(f"need 1..{self.segments} segments")
        for b, t0 in enumerate(starts):
            self.synth_p010(int(t0), self.gop)
            self.ladder_chunk(b * self.gop, self.gop, slot)

    def prepare_p010(self, segments, slot: int = 0) -> None:
        """segments: list of (y16, uv16) CUDA uint16 tensors shaped (gop, h, w) / (gop, h/2, w)."""
        for b, (y16, uv16) in enumerate(segments):
            self.y16.copy_(y16)
            self.uv16.copy_(uv16)
            self.ladder_chunk(b * self.gop, self.gop, slot)

    # -------------------------------------------------------------------- encode
    def encode_prepared(self, nseg: int, slot: int = 0, synced: bool = False) -> list[list[bytes]]:
        """Encode the staged segments of staging set `slot` on every rung; returns
        bitstreams [rung][segment].  `synced`: the caller already synchronised the
        pre-processing stream (e.g. it runs this on another thread while it prepares the
        next slot on the same stream)."""
        import torch

        if not synced:
            torch.cuda.current_stream(self.dev).synchronize()
        staging = self.staging_slots[slot]
        self._nseg = nseg
        out: list = [None] * len(self.engines)
        errs: list = []

        def run(r):
            try:
                out[r] = self.engines[r].encode_device(staging[r], nseg, self.gop)
            except Exception as e:  # surfaced after the join
                errs.append(e)

        if self.concurrent and len(self.engines) > 1:
            ths = [threading.Thread(target=run, args=(r,), daemon=True) for r in range(len(self.engines))]
            for t in ths:
                t.start()
            for t in ths:
                t.join()
        else:
            for r in range(len(self.engines)):
                run(r)
        if errs:
            raise errs[0]
        return out

    def encode_synthetic(self, starts) -> list[list[bytes]]:
        self.prepare_synthetic(starts)
        return self.encode_prepared(len(starts))

    def encode_overlapped(self, nseg: int, slot: int, prepare_next=None) -> list[list[bytes]]:
        """Encode staging set `slot` (already prepared and synchronised) on a helper thread
        while this thread runs `prepare_next()` (which should fill the other slot and end
        with a stream synchronise): the next call's tone-map / Lanczos kernels overlap this
        call's encode kernels and CABAC."""
        res: dict = {}

        def enc():
            try:
                res["out"] = self.encode_prepared(nseg, slot, synced=True)
            except Exception as e:  # re-raised on the caller's thread
                res["err"] = e

        t = threading.Thread(target=enc, daemon=True)
        t.start()
        try:
            if prepare_next is not None:
                prepare_next()
        finally:
            t.join()
        if "err" in res:
            raise res["err"]
        return res["out"]

    def psnr(self) -> list[dict]:
        """Per rung: PSNR of the last call's reconstruction vs the rung's own (tone-mapped,
        scaled) input, summed over its segments."""
        import numpy as np

        res = []
        for (w, h), e in zip(self.rungs, self.engines):
            n = getattr(self, "_nseg", None) or e.batch
            sse = np.array([e.sse(b) for b in range(n)]).sum(0)
            npx = w * h * e.last_frames * n
            f = lambda s, k: float("inf") if s == 0 else float(10 * np.log10(255.0 ** 2 * k / s))
            py, pu, pv = f(sse[0], npx), f(sse[1], npx / 4), f(sse[2], npx / 4)
            res.append({"w": w, "h": h, "y": py, "yuv": (6 * py + pu + pv) / 8})
        return res
