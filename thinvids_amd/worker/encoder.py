"""Segment encoder used by the worker's ``encode`` task and the node executor (replaces the
reference's ffmpeg VA-API / libx264 invocation, worker/tasks.py:1532-1651).

MI355X-first shape: a *part* (a run of frames, possibly many GOPs) is cut into closed GOP
chunks; the chunks of every part handed to one call — several parts pulled as one batch
by the per-GPU encode consumer, or a node rank's claimed segments — are packed into
batched engine launches of up to ``engine_batch`` chunks of equal length, so the GPU
always sees B segments at once.  Every chunk starts with an IDR + parameter sets, so a
part's bitstream is the plain concatenation of its chunks.

GPU path (no host bounce): a part's frames reach the device once (pinned upload, an RCCL
receive or on-device synthesis) and are tone-mapped / resized / edge-padded by HIP kernels
straight into the engine's staging buffer (:mod:`thinvids_amd.ops.stage`), then encoded
with ``GpuEngine.encode_device``.  A synthetic part at the engine's own size is generated
inside the engine (``encode_synthetic``: zero copies).

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
    seed: int = 1  # synthetic sources generated inside the engine
    crf: int = 0  # > 0: in-engine CRF (per-frame QP from the lookahead)
    scenecut: bool = False  # restart the closed GOP (IDR) at detected scene cuts
    codec: str = "hevc"  # "av1": the AV1 engine (models/av1_engine.py), BASELINE config #4
    qindex: int = 0  # AV1 q-index (0: matched to qp)
    bframes: int = 1  # HEVC hierarchical-B mini-GOP (1: I P P P; tv/gop.h)
    # HEVC bitstream identity beyond the rate point (explicit, never from the environment):
    # WPP substreams (entropy-coded on the GPU), residual quadtree, intra CUs in P pictures
    wpp: bool = True
    rqt: bool = True
    pintra: bool = True
    cascade: bool = True  # constant-QP I P P P: the low-delay QP cascade (tv/gop.h)
    rdoq: bool = True  # inter TBs drop trailing lone-+-1 coefficient groups (tv/hevc_defs.h)
    # where the WPP substreams are CABAC-coded ("auto" / "gpu" / "host"): the same bytes, so
    # not a coding tool (not in tools() / the checkpoint fingerprint), but its own engine
    entropy: str = "auto"

    def engine_key(self):
        if self.codec == "av1":
            return ("av1", self.width, self.height, self.av1_qindex(), self.cascade)
        return (self.width, self.height, self.qp, self.gop, self.search_range, self.deblock, self.sao, self.seed,
                self.crf, self.hevc_bframes(), self.wpp, self.rqt, self.pintra, self.cascade, self.rdoq, self.entropy)

    def tools(self) -> dict:
        """The coding-tool switches as GpuEngine / CpuEncoder keyword arguments."""
        return {"wpp": self.wpp, "rqt": self.rqt, "pintra": self.pintra, "cascade": self.cascade, "rdoq": self.rdoq}

    def hevc_bframes(self) -> int:
        """Mini-GOP actually used: in-engine CRF keeps I P P P (its lookahead QP is per
        frame in coding order)."""
        return 1 if self.crf > 0 else max(1, int(self.bframes))

    def av1_qindex(self) -> int:
        from ..models.av1 import qindex_for_hevc_qp

        return self.qindex or qindex_for_hevc_qp(self.qp)


@dataclass(frozen=True)
class SynthRange:
    """Frames [t0, t0 + n) of the seeded synthetic source (w x h): generated on the GPU
    where they are encoded (no scatter, no I/O)."""
    seed: int
    width: int
    height: int
    t0: int
    n: int

    def __len__(self):
        return self.n

    def host_frames(self) -> list:
        return [hevc.synth_frame(self.seed, self.t0 + k, self.width, self.height) for k in range(self.n)]


@dataclass
class PartStats:
    """Per part: frames encoded and summed SSE (Y, U, V) of the reconstruction vs the
    encoder input (the job's per-part PSNR)."""
    frames: int = 0
    sse: tuple = (0.0, 0.0, 0.0)

    def add(self, frames: int, sse) -> None:
        self.frames += frames
        self.sse = tuple(a + float(b) for a, b in zip(self.sse, sse))


def psnr_from_sse(sse, npx_luma: float) -> dict:
    f = lambda s, n: float("inf") if s <= 0 else float(10 * np.log10(255.0 ** 2 * n / s))
    y, u, v = f(sse[0], npx_luma), f(sse[1], npx_luma / 4), f(sse[2], npx_luma / 4)
    return {"y": y, "u": u, "v": v, "yuv": (6 * y + u + v) / 8}


HBM_FRACTION = 0.8  # share of the GPU's HBM the engine cache may hold (TV_HBM_FRACTION)


def device_budget(device: int = 0) -> int:
    """Bytes of HBM the engines of this process may use: ``TV_HBM_BUDGET_GB`` when set, else
    TV_HBM_FRACTION (0.8) of the device's total memory (hipMemGetInfo via torch)."""
    gb = os.environ.get("TV_HBM_BUDGET_GB")
    if gb:
        return int(float(gb) * (1 << 30))
    import torch

    _, total = torch.cuda.mem_get_info(device)
    return int(float(os.environ.get("TV_HBM_FRACTION", HBM_FRACTION)) * total)


def _staging_bytes(spec: "EncodeSpec", batch: int) -> int:
    from ..ops.stage import staging_planes

    if spec.codec == "av1":
        from ..models.av1 import coded_size

        fsz, _ = staging_planes(spec.width, spec.height, coded_size(spec.width, spec.height))
    else:
        fsz, _ = staging_planes(spec.width, spec.height)
    return batch * spec.gop * fsz


def engine_bytes(spec: "EncodeSpec", batch: int) -> int:
    """Device bytes of an engine for `spec` at `batch` segments, including the staging
    buffer the cache attaches to it (batch x GOP coded frames).  HEVC: the native
    constructor's own size formulas (gpu_engine.estimate_footprint); AV1: its per-segment
    GOP decision slots and frame sets (models/av1_engine.py allocations)."""
    if spec.codec == "av1":
        from ..models.av1 import coded_size

        W, H = coded_size(spec.width, spec.height)
        # two GOP decision slots of (mode, mv, 256 + 2 x 64 int16 levels) per 16x16 block
        # and frame (~384 B per pixel of a GOP-64 segment), plus the source / recon /
        # filtered frame sets and the filters' scratch (~11 coded frames)
        eng = batch * (2 * spec.gop * (W // 16) * (H // 16) * 776 + 11 * W * H * 3 // 2)
    else:
        from ..models.gpu_engine import estimate_footprint

        eng = estimate_footprint(spec.width, spec.height, batch, spec.gop, spec.sao, spec.hevc_bframes(),
                                 **spec.tools())["dev"]
    return eng + _staging_bytes(spec, batch)


class EngineCache:
    """Per-process GPU engines keyed by stream geometry/QP (allocation is HBM-heavy, so an
    engine lives for the life of the consumer).  Thread-safe; one engine serialises its
    own calls.  Each engine owns a device staging buffer (batch x GOP coded frames).

    Sized in BYTES, not engine counts (the reference sizes work by bytes too: its 10 MiB
    segment target, common.py:184): every engine's footprint (native allocation ledger +
    staging) is charged against ``budget`` (default: device_budget(), 0.8 of HBM), and the
    least recently used engines are evicted until a new one fits.  ``max_engines`` stays
    an upper bound on the count.  ``batch=0`` sizes each engine with auto_batch(spec,
    budget): the CU-fill heuristic capped by the byte budget."""

    def __init__(self, device: int = 0, batch: int = 8, max_engines: int = 8, budget: int | None = None):
        self.device, self.batch, self.max_engines = device, batch, max_engines
        self._budget = budget
        self._engines: dict = {}
        self._bytes: dict = {}
        self._order: list = []
        self._lock = threading.Lock()
        self.constructed = 0
        self.evicted = 0

    @property
    def budget(self) -> int:
        if self._budget is None:
            self._budget = device_budget(self.device)
        return self._budget

    def used_bytes(self) -> int:
        return sum(self._bytes.values())

    def _build(self, spec: "EncodeSpec", batch: int):
        from ..models.gpu_engine import GpuEngine

        if spec.codec == "av1":
            from ..models.av1_engine import Av1GpuEngine

            eng = Av1GpuEngine(spec.width, spec.height, batch=batch, qindex=spec.av1_qindex(), device=self.device,
                               cascade=spec.cascade)
            eng.batch = eng.B
            return eng
        return GpuEngine(spec.width, spec.height, qp=spec.qp, batch=batch, gop=spec.gop, search_range=spec.search_range,
                         deblock=spec.deblock, sao=spec.sao, seed=spec.seed, device=self.device, crf=spec.crf,
                         bframes=spec.hevc_bframes(), entropy=spec.entropy, **spec.tools())

    def get(self, spec: EncodeSpec):
        key = spec.engine_key()
        with self._lock:
            eng = self._engines.get(key)
            if eng is not None:  # LRU: most recently used last
                self._order.remove(key)
                self._order.append(key)
                return eng
            batch = self.batch or auto_batch(spec, self.budget)
            if spec.codec == "av1":
                batch = min(32, batch)
            batch = max(1, min(64, batch))
            need = engine_bytes(spec, batch)
            if need > self.budget:
                raise MemoryError(f"an engine for {spec.width}x{spec.height} x{batch} needs {need / 2**30:.1f} GiB, "
                                  f"over the HBM budget of {self.budget / 2**30:.1f} GiB")
            while self._order and (len(self._order) >= self.max_engines or self.used_bytes() + need > self.budget):
                old = self._order.pop(0)
                self._engines.pop(old).close()
                self._bytes.pop(old)
                self.evicted += 1
            eng = self._build(spec, batch)
            eng.lock = threading.Lock()
            eng.staging = None
            fp = eng.footprint()["dev"] if hasattr(eng, "footprint") else None
            self._bytes[key] = (fp + _staging_bytes(spec, batch)) if fp is not None else need
            self._engines[key] = eng
            self._order.append(key)
            self.constructed += 1
            return eng

    def close(self):
        with self._lock:
            for e in self._engines.values():
                e.close()
            self._engines.clear()
            self._bytes.clear()
            self._order.clear()


def auto_batch(spec: EncodeSpec, budget: int | None = None) -> int:
    """Segments per engine call: enough CTBs in flight to fill 256 CUs (measured on MI355X:
    48 at <= 1080p, 24 at 4K, 8 above; profiles/README.md), capped so that the engine plus
    its staging buffer take at most half of the HBM budget (the rest holds the claims'
    source frames, the ABR rungs and a second engine)."""
    px = spec.width * spec.height
    if spec.codec == "av1":  # measured: 32 at <= 1080p, 16 at 4K (bench.py --codec av1)
        want = 32 if px <= 1920 * 1088 else (16 if px <= 3840 * 2176 else 4)
    else:
        want = 48 if px <= 1920 * 1088 else (24 if px <= 3840 * 2176 else 8)
    if budget is None:
        return want
    b = want
    while b > 1 and engine_bytes(spec, b) > budget // 2:
        b = max(1, b * 3 // 4)
    return b


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


def chunk_plan(nframes: int, gop: int, cuts=()) -> list[tuple[int, int]]:
    """Closed-GOP chunks [(start, n)] covering a part: every `gop` frames, and a new GOP
    at each scene cut (the cadence restarts there)."""
    out, s, cuts = [], 0, sorted(c for c in cuts if 0 < c < nframes)
    while s < nframes:
        e = min(s + gop, nframes)
        nxt = next((c for c in cuts if s < c < e), None)
        e = nxt if nxt is not None else e
        out.append((s, e - s))
        s = e
    return out


def _cuts(part, spec: EncodeSpec) -> list[int]:
    if not spec.scenecut or isinstance(part, SynthRange):
        return []
    from ..models.scenecut import part_cuts

    return part_cuts(part)


def _nframes(part) -> int:
    return part.n if hasattr(part, "n") else len(part)


def _slice(part, s: int, n: int):
    if isinstance(part, SynthRange):
        return SynthRange(part.seed, part.width, part.height, part.t0 + s, n)
    if hasattr(part, "select"):  # DevFrames
        return part.select(s, n)
    return part[s:s + n]


def _host_frames(part) -> list:
    if isinstance(part, SynthRange):
        return part.host_frames()
    if hasattr(part, "select"):  # DevFrames -> host (software path only)
        flat = part.buf.reshape(-1).cpu().numpy()
        out = []
        for k in range(part.n):
            pl = []
            for off, pw, ph, st, fs in part.planes:
                o = off + k * fs
                pl.append(np.lib.stride_tricks.as_strided(flat[o:], (ph, pw), (st * flat.itemsize, flat.itemsize)).copy())
            out.append(tuple(pl))
        return out
    return part


def encode_parts(parts: list, spec: EncodeSpec, cache: EngineCache | None = None,
                 stats: list | None = None, qps: list | None = None) -> list[bytes]:
    """Encode several parts into one Annex-B bitstream each.  A part is a list of host
    (Y, U, V) frames (any size: resized to the spec), a :class:`~thinvids_amd.ops.stage.DevFrames`
    already on this GPU, or a :class:`SynthRange`.  `stats` (optional list of
    :class:`PartStats`, one per part) receives frames and reconstruction SSE.  `qps`
    (optional, one per part): per-frame slice QPs from rate control (None = spec.qp)."""
    qps = qps or [None] * len(parts)
    if spec.software or not gpu_available():
        if not spec.software:
            raise RuntimeError("no GPU available for a hardware encode (set software_encode for the CPU path)")
        out = []
        for i, p in enumerate(parts):
            frames = _host_frames(p)
            plan = chunk_plan(len(frames), max(len(frames), 1), _cuts(frames, spec))  # split at cuts only
            out.append(b"".join(_encode_cpu(frames[a:a + n], spec, stats[i] if stats else None,
                                            None if qps[i] is None else qps[i][a:a + n]) for a, n in plan))
        return out
    return _encode_gpu(parts, spec, cache or default_cache(), stats, qps)


def _encode_cpu(frames, spec: EncodeSpec, st: PartStats | None, fq=None) -> bytes:
    h, w = frames[0][0].shape
    if (w, h) != (spec.width, spec.height) or frames[0][0].dtype != np.uint8:
        frames = prepare_frames(frames, spec.width, spec.height)
    if spec.codec == "av1":  # C++ golden AV1 encoder, one closed GOP per `gop` frames
        from ..models import av1

        bs, recons = b"", []
        W, H = av1.coded_size(spec.width, spec.height)
        for a in range(0, len(frames), spec.gop):
            qm = None if fq is None else [av1.qindex_for_hevc_qp(int(x)) for x in fq[a:a + spec.gop]]
            r = av1.golden_encode(frames[a:a + spec.gop], spec.width, spec.height, spec.av1_qindex(), qmap=qm,
                                  cascade=spec.cascade)
            bs += r.stream
            for f in r.recon:
                recons.append((f[:W * H].reshape(H, W), f[W * H:W * H * 5 // 4].reshape(H // 2, W // 2),
                               f[W * H * 5 // 4:].reshape(H // 2, W // 2)))
    else:
        bs, recons = hevc.encode_sequence_cpu(frames, qp=spec.qp, gop=spec.gop, deblock=spec.deblock, sao=spec.sao,
                                              search_range=spec.search_range, frame_qps=fq, crf=spec.crf,
                                              bframes=spec.hevc_bframes(), **spec.tools())
    if st is not None:
        sse = np.zeros(3)
        for f, r in zip(frames, recons):
            for c in range(3):
                hh, ww = f[c].shape
                d = f[c].astype(np.int64) - r[c][:hh, :ww].astype(np.int64)
                sse[c] += float((d * d).sum())
        st.add(len(frames), sse)
    return bs


def _encode_gpu(parts, spec: EncodeSpec, cache: EngineCache, stats, qps) -> list[bytes]:
    import torch

    from ..ops import stage

    eng = cache.get(spec)
    dev = torch.device("cuda", cache.device)
    # host parts go to the device once (one pinned H2D each)
    dparts = [p if (isinstance(p, SynthRange) or hasattr(p, "select")) else stage.upload_frames(p, dev)
              for p in parts]
    chunks: dict[int, list] = {}
    out: list[list] = []
    for pi, p in enumerate(dparts):
        plan = chunk_plan(_nframes(p), spec.gop, _cuts(p, spec))
        out.append([b""] * len(plan))
        for c, (s, n) in enumerate(plan):
            q = None if qps[pi] is None else np.asarray(qps[pi][s:s + n], np.int64)
            chunks.setdefault(n, []).append((pi, c, _slice(p, s, n), q))
    if spec.codec == "av1":
        return _encode_gpu_av1(eng, chunks, out, spec, dev, stats)
    fsz, _ = stage.staging_planes(spec.width, spec.height)
    own_size = (spec.width, spec.height)
    with eng.lock:
        for n, items in chunks.items():
            for i in range(0, len(items), eng.batch):
                grp = items[i:i + eng.batch]
                srcs = [x[2] for x in grp]
                # segments without a plan keep the engine's constant-QP default (its I P P P cascade)
                dflt = (np.asarray(hevc.ippp_cascade_qps(spec.qp, n)) if spec.cascade and spec.hevc_bframes() == 1
                        and not spec.crf else np.full(n, spec.qp))
                qmap = None if all(x[3] is None for x in grp) else \
                    np.stack([x[3] if x[3] is not None else dflt for x in grp])
                if all(isinstance(s, SynthRange) and s.seed == spec.seed and (s.width, s.height) == own_size
                       for s in srcs):
                    bits = eng.encode_synthetic([s.t0 for s in srcs], nframes=n, qp=qmap)
                else:
                    need = eng.batch * spec.gop * fsz
                    if eng.staging is None or eng.staging.numel() < need:
                        eng.staging = torch.empty(need, dtype=torch.uint8, device=dev)
                    for j, s in enumerate(srcs):
                        if isinstance(s, SynthRange):
                            s = stage.synth_frames(s.seed, s.width, s.height, range(s.t0, s.t0 + s.n), dev)
                        stage.to_staging(s, spec.width, spec.height, eng.staging, j * n)
                    torch.cuda.current_stream(dev).synchronize()
                    bits = eng.encode_device(eng.staging, len(grp), n, qp=qmap)
                for j, ((pi, c, _, _), b) in enumerate(zip(grp, bits)):
                    out[pi][c] = b
                    if stats is not None:
                        stats[pi].add(n, eng.sse(j))
    return [b"".join(x) for x in out]


def _encode_gpu_av1(eng, chunks: dict, out: list, spec: EncodeSpec, dev, stats) -> list[bytes]:
    """AV1 engine: equal-length chunks in groups of up to eng.B segments; sources are
    staged (tone-map / resize / edge pad) straight into the engine's coded-size planes.

    The groups are software-pipelined: group k + 1 is staged and its GPU part issued
    (encode_gop async_host: decisions collected on the copy stream) before group k's
    decisions go to the OBU writers, so entropy coding overlaps the next group's kernels.  The
    chunks are cut into equal groups, at least two (>= 8 segments) to get that overlap.  Staging
    and the per-frame source copies are ordered on the current stream, so reusing the staging
    buffer for the next group never races the previous group's copies."""
    import torch

    from ..models import av1
    from ..ops import stage

    cw, ch = av1.coded_size(spec.width, spec.height)
    fsz = cw * ch * 3 // 2
    ysz, csz = cw * ch, cw * ch // 4
    groups = []
    for n, items in chunks.items():
        ng = max(-(-len(items) // eng.B), 2 if len(items) >= 8 else 1)  # equal groups, >= 2 to overlap
        step = -(-len(items) // ng)
        groups += [(n, items[i:i + step]) for i in range(0, len(items), step)]
    writers = []  # (part index, chunk index, writer future)

    def to_writers(n, grp, fut):
        g = fut.result()
        for j, ((pi, c, _, _), fu) in enumerate(zip(grp, eng.submit_entropy(g))):
            writers.append((pi, c, fu))
            if stats is not None:
                stats[pi].add(n, g.sse[:, j].sum(axis=0))

    with eng.lock:
        pending = None
        for n, grp in groups:
            need = len(grp) * n * fsz
            if eng.staging is None or eng.staging.numel() < need:
                if pending is not None:  # the previous group's copies still read the old buffer
                    to_writers(*pending)
                    pending = None
                eng.staging = torch.empty(need, dtype=torch.uint8, device=dev)
            for j, (_, _, s, _) in enumerate(grp):
                if isinstance(s, SynthRange):
                    s = stage.synth_frames(s.seed, s.width, s.height, range(s.t0, s.t0 + s.n), dev)
                stage.to_staging(s, spec.width, spec.height, eng.staging, j * n, coded=(cw, ch))
            frames = eng.staging[:need].view(len(grp), n, fsz)

            def load(t, planes, frames=frames, k=len(grp)):
                f = frames[:, t]
                planes[0][:k].copy_(f[:, :ysz].view(-1, ch, cw))
                planes[1][:k].copy_(f[:, ysz:ysz + csz].view(-1, ch // 2, cw // 2))
                planes[2][:k].copy_(f[:, ysz + csz:].view(-1, ch // 2, cw // 2))

            qmap = None
            if any(x[3] is not None for x in grp):  # rate-control plan: per-frame HEVC QP -> q-index
                # segments without a plan keep the engine's constant-q default (its cascade)
                base = (av1.cascade_qmap(spec.av1_qindex(), n) if spec.cascade else [spec.av1_qindex()] * n)
                qmap = np.array([[av1.qindex_for_hevc_qp(int(x[3][t])) if x[3] is not None
                                  else base[t] for x in grp] for t in range(n)], np.int32)
            fut = eng.encode_gop(n, load, nseg=len(grp), qmap=qmap, async_host=True)
            if pending is not None:
                to_writers(*pending)
            pending = (n, grp, fut)
        if pending is not None:
            to_writers(*pending)
        for pi, c, fu in writers:
            out[pi][c] = b"".join(fu.result())
    return [b"".join(x) for x in out]


def _tonemap_planar_ref(y, u, v):
    """Host tone-map of a 10-bit planar PQ frame (values 0..1023) via the P010 reference."""
    from ..ops.color import tonemap_pq_ref

    y16 = (y.astype(np.uint16) << 6)
    uv16 = np.stack([u.astype(np.uint16) << 6, v.astype(np.uint16) << 6], -1).reshape(u.shape[0], -1)
    return tonemap_pq_ref(y16, uv16)


def prepare_frames(frames: list, out_w: int, out_h: int, device: str | None = None,
                   deinterlace: bool = False) -> list:
    """Optional bwdif deinterlace, then Lanczos resize of a list of I420 frames to
    out_w x out_h (identity when already there); 10-bit PQ frames are tone-mapped first.
    The worker's deinterlace path and the software encoder use this; the GPU job path
    stages on the device instead (:mod:`thinvids_amd.ops.stage`)."""
    if not frames:
        return frames
    h, w = frames[0][0].shape
    if frames[0][0].dtype == np.uint16:
        frames = [_tonemap_planar_ref(*f) for f in frames]
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
