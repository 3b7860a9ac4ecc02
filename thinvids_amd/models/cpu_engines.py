"""CPU stand-ins of the GPU engines with the interfaces bench.py drives — the golden C++
encoders (HEVC: csrc/core/cpu_encoder.cpp, AV1: csrc/core/av1_codec.cpp) behind the
methods of GpuEngine, Av1GpuEngine and AbrLadder.

They exist so that ``bench.py --cpu`` runs the benchmark's whole N-rank logic — the step
pipelines, the post-thread collective ordering, the 2-pass plan all-reduce, the bitstream
gather — on the gloo backend with N processes on a machine without GPUs
(tests/test_launch.py), before the driver's multi-GPU run ever meets it.  The bitstreams
are the golden encoders' (the GPU engines are bit-exact with them), so a CPU run also
produces decodable output.  Not a performance path: numbers from ``--cpu`` are not
MI355X numbers and bench.py labels them so.
"""
from __future__ import annotations

import concurrent.futures as cf
import time
from dataclasses import dataclass

import numpy as np

from . import av1 as av1m
from . import hevc


def _sse(a: np.ndarray, b: np.ndarray) -> float:
    d = a.astype(np.int64) - b.astype(np.int64)
    return float((d * d).sum())


def _frame_sse(src, rec, w: int, h: int) -> np.ndarray:
    return np.array([_sse(src[c], rec[c][:(h if c == 0 else h // 2), :(w if c == 0 else w // 2)]) for c in range(3)])


class CpuHevcEngine:
    """GpuEngine's synthetic-source interface on the golden HEVC encoder: batch segments
    per call, encoded concurrently on a thread pool (the native encoder releases the GIL)."""

    def __init__(self, width: int, height: int, qp: int = 27, batch: int = 2, gop: int = 8, search_range: int = 16,
                 sao: bool = False, seed: int = 1, threads: int | None = None, bframes: int = 1, wpp: bool = True,
                 rqt: bool = True, pintra: bool = True, cascade: bool = True, rdoq: bool = True, **_):
        self.width, self.height, self.qp, self.batch, self.gop = width, height, qp, batch, gop
        self.tools = {"wpp": wpp, "rqt": rqt, "pintra": pintra, "cascade": cascade, "rdoq": rdoq}
        self.search_range, self.sao, self.seed, self.bframes = search_range, sao, seed, int(bframes)
        self.threads = threads or 2
        self.pool = cf.ThreadPoolExecutor(self.threads)
        self._sse = [np.zeros(3)] * batch
        self._t = {"gpu_ms": 0.0, "wall_ms": 0.0, "entropy_cpu_ms": 0.0, "coef_mb": 0.0}

    def _one(self, start: int, n: int, fq):
        frames = [hevc.synth_frame(self.seed, start + t, self.width, self.height) for t in range(n)]
        data, recons = hevc.encode_sequence_cpu(frames, qp=self.qp, gop=n, sao=self.sao, search_range=self.search_range,
                                                bframes=self.bframes, frame_qps=fq, **self.tools)
        return data, sum(_frame_sse(f, r, self.width, self.height) for f, r in zip(frames, recons))

    def encode_synthetic(self, starts, nframes: int | None = None, qp=None) -> list[bytes]:
        n = self.gop if nframes is None else int(nframes)
        t0 = time.perf_counter()
        qps = [None] * len(starts)
        if qp is not None:
            q = np.asarray(qp)
            qps = [np.full(n, int(q)) if q.ndim == 0 else q[b] for b in range(len(starts))]
        got = list(self.pool.map(lambda a: self._one(a[0], n, a[1]), zip(starts, qps)))
        self._sse = [s for _, s in got]
        self.last_frames = n
        self._t["wall_ms"] = 1000 * (time.perf_counter() - t0)
        return [d for d, _ in got]

    def sse(self, b: int):
        return tuple(float(x) for x in self._sse[b])

    def psnr(self, b: int) -> dict:
        y, u, v = self.sse(b)
        npx = self.width * self.height * getattr(self, "last_frames", self.gop)
        f = lambda s, n: float("inf") if s == 0 else 10 * np.log10(255.0 ** 2 * n / s)  # noqa: E731
        py, pu, pv = f(y, npx), f(u, npx / 4), f(v, npx / 4)
        return {"y": py, "u": pu, "v": pv, "yuv": (6 * py + pu + pv) / 8}

    def timing(self) -> dict:
        return dict(self._t)

    def close(self) -> None:
        self.pool.shutdown(wait=True)


@dataclass
class CpuGop:
    """Av1GpuEngine.GopHost's role: one GOP of `B` segments, already entropy-coded."""
    tus: list          # per segment: list of temporal units
    sse: np.ndarray    # (F, B, 3)
    mode: np.ndarray   # (F, B, 1) — only its shape is read (segment count)


class CpuAv1Engine:
    """Av1GpuEngine's encode_gop / submit_entropy interface on the golden AV1 encoder.  The
    loader argument is the list of segment start frames (the GPU engine takes a device
    loader callback instead)."""

    def __init__(self, width: int, height: int, batch: int, qindex: int = 100, threads: int | None = None, seed: int = 1,
                 cascade: bool = True, **_):
        self.w, self.h, self.B, self.q, self.seed = width, height, batch, int(qindex), seed
        self.cascade = cascade
        self.W, self.H = av1m.coded_size(width, height)
        self.pool = cf.ThreadPoolExecutor(threads or 2)
        self.lr_enabled = True

    def _one(self, start: int, n: int, qm):
        frames = [hevc.synth_frame(self.seed, start + t, self.w, self.h) for t in range(n)]
        r = av1m.golden_encode(frames, self.w, self.h, self.q, qmap=qm, cascade=self.cascade)
        tus = av1m.split_temporal_units(r.stream, r.tu_sizes)
        W, H = self.W, self.H
        sse = []
        for f, rec in zip(frames, r.recon):
            planes = (rec[:W * H].reshape(H, W), rec[W * H:W * H * 5 // 4].reshape(H // 2, W // 2),
                      rec[W * H * 5 // 4:].reshape(H // 2, W // 2))
            sse.append(_frame_sse(f, planes, self.w, self.h))
        return tus, np.array(sse)

    def encode_gop(self, nframes: int, starts, nseg: int | None = None, qmap=None, async_host: bool = False):
        nseg = nseg or len(starts)
        qm = None if qmap is None else np.asarray(qmap, np.int32).reshape(nframes, nseg)

        def run():
            got = list(self.pool.map(lambda b: self._one(starts[b], nframes, None if qm is None else qm[:, b]),
                                     range(nseg)))
            return CpuGop([t for t, _ in got], np.stack([s for _, s in got], 1), np.zeros((nframes, nseg, 1)))

        if not async_host:
            return run()
        fut: cf.Future = cf.Future()
        fut.set_result(run())
        return fut

    def submit_entropy(self, g: CpuGop) -> list:
        out = []
        for tus in g.tus:
            f: cf.Future = cf.Future()
            f.set_result(tus)
            out.append(f)
        return out

    def close(self) -> None:
        self.pool.shutdown(wait=True)


class CpuAbrLadder:
    """AbrLadder's call pattern (prepare a staging slot, encode every rung's segments while
    the next slot is prepared) on the CPU: SDR synthetic source frames -> numpy Lanczos
    (ops.resize reference) per rung -> golden HEVC encoder.  The HDR10 tone-map stage is
    GPU-only and skipped here."""

    def __init__(self, src_w: int, src_h: int, heights, qp: int = 27, segments: int = 2, gop: int = 4,
                 threads: int | None = None, seed: int = 1, search_range: int = 16, sao: bool = False, **_):
        from .abr import plan_rungs

        self.src_w, self.src_h, self.segments, self.gop, self.seed = src_w, src_h, segments, gop, seed
        self.rungs = plan_rungs(src_w, src_h, heights)
        self.engines = [CpuHevcEngine(w, h, qp=qp, batch=segments, gop=gop, search_range=search_range, sao=sao,
                                      seed=seed, threads=threads) for w, h in self.rungs]
        self.slots: dict = {}
        self._sse = [np.zeros(3) for _ in self.rungs]
        self._frames = [0 for _ in self.rungs]

    def prepare_synthetic(self, starts, slot: int = 0) -> None:
        from ..ops.resize import resize_plane_ref

        per_rung = []
        for w, h in self.rungs:
            segs = []
            for s in starts:
                frames = []
                for t in range(self.gop):
                    src = hevc.synth_frame(self.seed, s + t, self.src_w, self.src_h)
                    if (w, h) == (self.src_w, self.src_h):
                        frames.append(src)
                        continue
                    frames.append(tuple(np.clip(np.rint(resize_plane_ref(p, oh, ow)), 0, 255).astype(np.uint8)
                                        for p, (ow, oh) in zip(src, ((w, h), (w // 2, h // 2), (w // 2, h // 2)))))
                segs.append(frames)
            per_rung.append(segs)
        self.slots[slot] = per_rung

    def encode_overlapped(self, nseg: int, slot: int, prepare_next=None) -> list[list[bytes]]:
        if prepare_next is not None:
            prepare_next()
        out = []
        for r, (eng, segs) in enumerate(zip(self.engines, self.slots.pop(slot))):
            rung = []
            for frames in segs[:nseg]:
                data, recons = hevc.encode_sequence_cpu(frames, qp=eng.qp, gop=len(frames), sao=eng.sao,
                                                        search_range=eng.search_range)
                rung.append(data)
                self._sse[r] = self._sse[r] + sum(_frame_sse(f, x, eng.width, eng.height)
                                                  for f, x in zip(frames, recons))
                self._frames[r] += len(frames)
            out.append(rung)
        return out

    def psnr(self) -> list[dict]:
        out = []
        for (w, h), s, n in zip(self.rungs, self._sse, self._frames):
            mse = s[0] / max(1, n * w * h)
            out.append({"y": float("inf") if mse == 0 else float(10 * np.log10(255.0 ** 2 / mse))})
        return out

    def close(self) -> None:
        for e in self.engines:
            e.close()
