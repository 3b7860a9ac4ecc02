"""Segment encoder used by the worker's ``encode`` task (replaces the reference's ffmpeg
VA-API / libx264 invocation, worker/tasks.py:1532-1651).

MI355X-first shape: a *part* (a run of frames, possibly many GOPs) is cut into closed GOP
chunks; the chunks of every part handed to one call — typically several parts pulled as
one batch by the per-GPU encode consumer — are packed into batched engine launches of up
to ``engine_batch`` chunks of equal length, so the GPU always sees B segments at once.
Every chunk starts with an IDR + parameter sets, so a part's bitstream is the plain
concatenation of its chunks.

``software=True`` selects the C++ reference encoder on the CPU (the reference's per-job
``software_encode`` path, libx264 there).
"""
from __future__ import annotations

import logging
import os
import threading
from dataclasses import dataclass

import numpy as np

from ..models import hevc

log = logging.getLogger("thinvids.worker.encoder")


@dataclass(frozen=True)
class EncodeSpec:
    width: int
    height: int
    qp: int = 27
    gop: int = 64
    search_range: int = 64
    deblock: bool = True
    sao: bool = False
    software: bool = False

    def engine_key(self):
        return (self.width, self.height, self.qp, self.gop, self.search_range, self.deblock, self.sao)


class EngineCache:
    """Per-process GPU engines keyed by stream geometry/QP (allocation is HBM-heavy, so an
    engine lives for the life of the consumer).  Thread-safe; one engine serialises its
    own calls."""

    def __init__(self, device: int = 0, batch: int = 8, max_engines: int = 4):
        self.device, self.batch, self.max_engines = device, batch, max_engines
        self._engines: dict = {}
        self._order: list = []
        self._lock = threading.Lock()

    def get(self, spec: EncodeSpec):
        from ..models.gpu_engine import GpuEngine

        key = spec.engine_key()
        with self._lock:
            eng = self._engines.get(key)
            if eng is None:
                while len(self._order) >= self.max_engines:
                    old = self._order.pop(0)
                    self._engines.pop(old).close()
                eng = GpuEngine(spec.width, spec.height, qp=spec.qp, batch=self.batch, gop=spec.gop,
                                search_range=spec.search_range, deblock=spec.deblock, sao=spec.sao,
                                device=self.device)
                eng.lock = threading.Lock()
                self._engines[key] = eng
                self._order.append(key)
            return eng

    def close(self):
        with self._lock:
            for e in self._engines.values():
                e.close()
            self._engines.clear()
            self._order.clear()


_default_cache: EngineCache | None = None


def default_cache() -> EngineCache:
    global _default_cache
    if _default_cache is None:
        from .config import get_config

        dev = int(os.environ.get("LOCAL_RANK", os.environ.get("TV_DEVICE", "0")))
        _default_cache = EngineCache(device=dev, batch=get_config().engine_batch)
    return _default_cache


def gpu_available() -> bool:
    if os.environ.get("TV_FORCE_CPU") == "1":
        return False
    try:
        from ..models.gpu_engine import device_count

        return device_count() > 0
    except Exception:
        return False


def chunk_plan(nframes: int, gop: int) -> list[tuple[int, int]]:
    """Closed-GOP chunks [(start, n)] covering a part."""
    return [(s, min(gop, nframes - s)) for s in range(0, nframes, gop)]


def encode_parts(parts: list[list], spec: EncodeSpec, cache: EngineCache | None = None) -> list[bytes]:
    """Encode several parts (lists of (Y, U, V) frames at spec size); returns one Annex-B
    bitstream per part."""
    if spec.software or not gpu_available():
        if not spec.software:
            raise RuntimeError("no GPU available for a hardware encode (set software_encode for the CPU path)")
        return [hevc.encode_sequence_cpu(frames, qp=spec.qp, gop=spec.gop, deblock=spec.deblock,
                                           sao=spec.sao)[0]
                for frames in parts]
    eng = (cache or default_cache()).get(spec)
    # (part, chunk index, frames) grouped by chunk length
    chunks: dict[int, list] = {}
    out: list[list] = []
    for p, frames in enumerate(parts):
        plan = chunk_plan(len(frames), spec.gop)
        out.append([b""] * len(plan))
        for c, (s, n) in enumerate(plan):
            chunks.setdefault(n, []).append((p, c, frames[s:s + n]))
    with eng.lock:
        for n, items in chunks.items():
            for i in range(0, len(items), eng.batch):
                grp = items[i:i + eng.batch]
                bits = eng.encode_frames([fr for _, _, fr in grp])
                for (p, c, _), b in zip(grp, bits):
                    out[p][c] = b
    return [b"".join(x) for x in out]


def prepare_frames(frames: list, out_w: int, out_h: int, device: str | None = None,
                   deinterlace: bool = False) -> list:
    """Optional bwdif deinterlace, then Lanczos resize of a list of I420 frames to
    out_w x out_h (identity when already there).  On a GPU host both HIP kernels run on the
    device and each frame crosses PCIe once each way."""
    if not frames:
        return frames
    h, w = frames[0][0].shape
    if (w, h) == (out_w, out_h) and not deinterlace:
        return frames
    from ..ops.deint import bwdif_frame
    from ..ops.resize import resize_frame

    n = len(frames)
    if device is None and gpu_available():
        import torch

        dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", os.environ.get("TV_DEVICE", "0"))))
        # np.require(W) copies read-only views (y4m frombuffer) so torch gets a writable array
        up = [tuple(torch.from_numpy(np.require(p, np.uint8, ["C", "W"])).to(dev, non_blocking=True) for p in f)
              for f in frames]
        out = []
        for i in range(n):
            f = up[i]
            if deinterlace:
                f = bwdif_frame(up[max(0, i - 1)], f, up[min(n - 1, i + 1)])
            if (w, h) != (out_w, out_h):
                f = resize_frame(f, out_w, out_h)
            out.append(tuple(p.cpu().numpy() for p in f))
        return out
    frames = [tuple(np.asarray(p) for p in f) for f in frames]
    if deinterlace:
        frames = [bwdif_frame(frames[max(0, i - 1)], frames[i], frames[min(n - 1, i + 1)]) for i in range(n)]
    if (w, h) == (out_w, out_h):
        return frames
    return [resize_frame(f, out_w, out_h) for f in frames]
