"""Single-node SPMD transcode: one process per GPU, RCCL over xGMI for the data plane
(BASELINE configs #3-#5).

    torchrun --standalone --nproc-per-node 8 -m thinvids_amd.parallel.node_job \\
        --input movie.y4m --output movie.mp4 [--height 1080] [--qp 27 | --bitrate-kbps 4000]
        [--gop 64] [--segment-frames 256] [--mode direct|scatter] [--ladder 2160,1440,1080,720,480]

Flow (the reference's split -> encode -> stitch, without HTTP or disk in between):

1. rank 0 probes the source and plans GOP-aligned segments (closed GOPs, IDR first);
2. segments are handed out **dynamically** through an atomic counter in the rendezvous
   store (the Huey pull model: a fast GPU takes more), or, in ``scatter`` mode, rank 0
   reads frames and sends every rank its segment over RCCL point-to-point (one xGMI hop);
   in ``direct`` mode each rank reads its own range (no scatter traffic, P5);
3. each rank resizes (HIP Lanczos) and encodes its segments in batched engine launches;
4. with ``--bitrate-kbps`` a first pass measures bits per segment at the base QP; the
   per-segment sizes are **all-reduced** and every rank derives the same per-segment QP
   plan (complexity^0.6 allocation), then encodes pass 2;
5. single-pass jobs with a plain MP4 output are **stitched while they encode**: every
   finished claim goes to rank 0 (its own in memory, the peers' as part files, or with
   ``TV_STITCH_TRANSPORT=rccl`` point-to-point in per-claim gather rounds on a comm thread,
   comm.SegmentStream), whose stitch thread appends each rung's segments in order to a
   streaming faststart MP4 writer; otherwise bitstreams are gathered to rank 0 after the last pass (all_gather
   of sizes + grouped send/recv) and muxed in segment order.  ``--ladder`` fans rungs x
   segments out over all ranks and writes one MP4 per rung.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import json
import math
import os
import sys
import threading
import time

import numpy as np

from ..models.ratecontrol import (AV1_SLOPE, QCOMP, QCOMP_BFRAMES, SLOPE, AbrController, RateFeedback, frame_sizes,
                                  plan_frame_qps, predict_bits, round_qps, vbv_ok, vbv_repair_offset, vbv_scale)
from ..utils import fault, trace

RC_TOLERANCE = 0.04  # a pass within +-4 % of the target bitrate is final (the contract is +-5 %)


def _dist():
    import torch.distributed as dist

    return dist if dist.is_available() and dist.is_initialized() else None


def _device():
    import torch

    if torch.cuda.is_available() and os.environ.get("TV_FORCE_CPU") != "1":
        return torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0")))
    return torch.device("cpu")


def plan_segments(nframes: int, segment_frames: int, gop: int) -> list[tuple[int, int]]:
    """GOP-aligned [start, n) ranges: segment length is rounded up to a GOP multiple."""
    seg = max(gop, int(math.ceil(max(1, segment_frames) / gop)) * gop)
    return [(s, min(seg, nframes - s)) for s in range(0, nframes, seg)]


def qp_plan_two_pass(bits: np.ndarray, frames: np.ndarray, base_qp: int, target_bits: float,
                     qcomp: float = 0.6, qp_min: int = 10, qp_max: int = 51) -> np.ndarray:
    """Per-segment QP from first-pass sizes.  Rate model: bits(QP) = b0 * 2^(-(QP-QP0)/6).
    Segment i gets target t_i proportional to frames_i * (b_i/frames_i)^qcomp (complexity
    compression as in x264's qcomp), scaled so sum(t) = target_bits."""
    bits = np.maximum(np.asarray(bits, np.float64), 1.0)
    frames = np.maximum(np.asarray(frames, np.float64), 1.0)
    w = frames * (bits / frames) ** qcomp
    t = target_bits * w / w.sum()
    qp = base_qp + 6.0 * np.log2(bits / t)
    return np.clip(np.rint(qp), qp_min, qp_max).astype(np.int64)


class _Counter:
    """Atomic work counter in the torch.distributed rendezvous store (dynamic stealing)."""

    def __init__(self, key: str):
        dist = _dist()
        self.store = dist.distributed_c10d._get_default_store() if dist else None
        self.key, self.local = _ns(key), 0

    def next(self) -> int:
        if self.store is None:
            self.local += 1
            return self.local - 1
        return int(self.store.add(self.key, 1)) - 1

    def peek(self) -> int:
        """Items handed out so far (no claim)."""
        return self.local if self.store is None else int(self.store.add(self.key, 0))


def _ns(key: str) -> str:
    """Store keys are namespaced by the elastic restart count, so a torchrun restart of the
    process group (``--max-restarts``) starts with fresh counters."""
    return f"tv{os.environ.get('TORCHELASTIC_RESTART_COUNT', '0')}_{key}"


class _LocalStore:
    """Single-process stand-in for the c10d store (add/set/get)."""

    def __init__(self):
        self.kv: dict = {}

    def add(self, k, n):
        self.kv[k] = int(self.kv.get(k, 0)) + n
        return self.kv[k]

    def set(self, k, v):
        self.kv[k] = v if isinstance(v, bytes) else str(v).encode()

    def get(self, k):
        return self.kv[k]


class WorkQueue:
    """Segment work queue shared by all ranks through the rendezvous store — the reference's
    Huey pull model (any encoder takes the next part, worker/tasks.py:1276, :1322) plus its
    failure path (a failed part is re-enqueued for *any* node, :1385-1464):

    * ``claim(n)``: up to n fresh items from an atomic counter (a fast GPU takes more);
    * ``fail(item)``: count the failure; re-publish the item on the retry list, or raise
      the job-wide abort flag when it has failed ``max_retries`` + 1 times;
    * ``claim_retry()``: claim one unclaimed retry item (one ``add`` per item: exactly one
      rank wins it);
    * ``finished()``: True once every rank has drained the fresh items, no retry is in
      flight and every retry item is claimed — the termination check re-reads the retry
      count around the in-flight read so an item published meanwhile keeps ranks looping.
    """

    def __init__(self, name: str, items: list, world: int, max_retries: int = 3):
        dist = _dist()
        self.store = dist.distributed_c10d._get_default_store() if dist else _LocalStore()
        self.name, self.items, self.world, self.max_retries = name, items, world, max_retries
        self.ctr = _Counter(f"{name}_next") if dist else None
        self._local_next = 0
        self._scan = 0

    def _k(self, s: str) -> str:
        return _ns(f"{self.name}_{s}")

    def _add(self, s: str, n: int = 1) -> int:
        return int(self.store.add(self._k(s), n))

    def claim(self, n: int) -> list:
        out = []
        for _ in range(max(1, n)):
            if self.ctr is not None:
                k = self.ctr.next()
            else:
                k, self._local_next = self._local_next, self._local_next + 1
            if k >= len(self.items):
                break
            out.append(self.items[k])
        return out

    def unclaimed(self) -> int:
        """Fresh items nobody has claimed yet (a snapshot: other ranks keep claiming)."""
        taken = self.ctr.peek() if self.ctr is not None else self._local_next
        return max(0, len(self.items) - taken)

    def fresh_done(self) -> None:
        self._add("done")

    def aborted(self) -> str | None:
        if self._add("abort", 0):
            return self.store.get(self._k("abort_msg")).decode()
        return None

    def fail(self, item, why: str) -> None:
        key = json.dumps(list(item))
        n = self._add(f"fail_{key}")
        if n > self.max_retries:
            self.store.set(self._k("abort_msg"), f"segment {item} failed {n} times: {why}")
            self._add("abort")
            return
        idx = self._add("rq_n") - 1
        self.store.set(self._k(f"rq_{idx}"), key)

    def claim_retry(self):
        n = self._add("rq_n", 0)
        while self._scan < n:
            i = self._scan
            self._scan += 1
            if self._add(f"rq_c_{i}") == 1:
                self._add("inflight")
                return tuple(json.loads(self.store.get(self._k(f"rq_{i}")).decode()))
        return None

    def retry_done(self) -> None:
        self._add("inflight", -1)

    def fail_all(self, why: str) -> None:
        """Raise the job-wide abort flag (cooperative halt: every rank stops claiming)."""
        self.store.set(self._k("abort_msg"), why)
        self._add("abort")

    def finished(self) -> bool:
        if self._add("done", 0) < self.world:
            return False
        n1 = self._add("rq_n", 0)
        busy = self._add("inflight", 0)
        n2 = self._add("rq_n", 0)
        if busy or n1 != n2:
            return False
        return all(self._add(f"rq_c_{i}", 0) >= 1 for i in range(n2))


# bumped whenever the encoders' output for identical settings changes (a checkpoint written
# by an older build must not be mixed into a newer job's output)
BITSTREAM_VERSION = 11  # 11: RDOQ-lite trailing coefficient-group trimming (inter); 10: the constant-QP I P P P QP cascade by default (9: WPP substreams)


class Checkpoint:
    """Segment-level resume: every encoded segment is published atomically
    as ``<dir>/<fingerprint>/r<rung>_s<idx>_q<qp>.hevc`` with a ``.sha256`` sidecar written
    last; a rerun (or an elastic restart) reuses every segment whose checksum verifies.
    Keyed by QP, so first-pass segments double as the 2-pass statistics checkpoint.  The
    fingerprint covers everything that changes a segment's bytes (source identity, ladder
    geometry, GOP, segmentation, search range, codec, q-index, CRF, rate-control mode and
    the bitstream version), so a reused directory never mixes jobs or codecs."""

    def __init__(self, root: str | None, fingerprint: str = ""):
        self.root = os.path.join(root, fingerprint) if root and fingerprint else root
        if self.root:
            os.makedirs(self.root, exist_ok=True)

    @staticmethod
    def fingerprint(**fields) -> str:
        return hashlib.sha256(json.dumps(fields, sort_keys=True, default=str).encode()).hexdigest()[:20]

    def _path(self, r: int, i: int, qp: int) -> str:
        return os.path.join(self.root, f"r{r}_s{i}_q{qp}.hevc")

    def load(self, r: int, i: int, qp: int) -> bytes | None:
        if not self.root:
            return None
        p = self._path(r, i, qp)
        try:
            with open(p, "rb") as f:
                data = f.read()
            with open(p + ".sha256") as f:
                want = f.read().strip()
        except OSError:
            return None
        return data if hashlib.sha256(data).hexdigest() == want else None

    def save(self, r: int, i: int, qp: int, data: bytes) -> None:
        if not self.root:
            return
        p = self._path(r, i, qp)
        for path, payload, mode in ((p, data, "wb"), (p + ".sha256", hashlib.sha256(data).hexdigest(), "w")):
            tmp = f"{path}.{os.getpid()}.tmp"
            with open(tmp, mode) as f:
                f.write(payload)
            os.replace(tmp, path)


_job_seq = [0]  # run_job calls in this process (identical on every rank: SPMD)


class JobHooks:
    """Callbacks a node job reports through (the node executor binds them to the job hash:
    progress counters, heartbeat, cooperative halt — reference worker/tasks.py:1694-1733,
    :392-394).  The default does nothing."""

    def segment_done(self, frames: int) -> None:
        pass

    def new_pass(self, index: int) -> None:
        """A rate-control pass starts (0 = the first): per-pass progress restarts."""

    def halted(self) -> bool:
        return False


def _part_path(parts_dir: str, r: int, i: int) -> str:
    return os.path.join(parts_dir, f"r{r}_s{i}.part")


def _attempt_parts_dir(output: str, job_tag: str, rank: int) -> str:
    """Part-file directory of THIS attempt of the job (file transport only): rank 0 empties
    ``{output}.parts`` and publishes a fresh token through the rendezvous store before any
    peer can write, so parts left by a killed earlier attempt (same output name, possibly
    other settings) are never read into this one."""
    import shutil
    import uuid

    root = f"{output}.parts"
    dist = _dist()
    store = dist.distributed_c10d._get_default_store() if dist else None
    key = _ns(f"{job_tag}_parts_token")
    if rank == 0:
        shutil.rmtree(root, ignore_errors=True)
        token = uuid.uuid4().hex[:16]
        os.makedirs(os.path.join(root, token))
        if store is not None:
            store.set(key, token)
    else:
        token = store.get(key).decode()  # blocks until rank 0 has cleaned up and published
    return os.path.join(root, token)


def publish_part(parts_dir: str, r: int, i: int, data: bytes) -> None:
    """A peer rank's finished segment for the stitch rank: written to a temporary name and
    renamed, so the stitcher never sees a partial part."""
    p = _part_path(parts_dir, r, i)
    tmp = f"{p}.{os.getpid()}.tmp"
    with open(tmp, "wb") as f:
        f.write(data)
    os.replace(tmp, p)


class StreamStitcher:
    """Rank 0's stitch thread (reference overlap: the stitcher ingests parts while encoders
    run, worker/tasks.py:1805-1822, :1898-2029): segment i of every rung is appended, in
    segment order, to that rung's streaming faststart MP4 (models.hevc.Mp4StreamWriter) as
    soon as it exists.  Segments arrive through put(): rank 0's own directly, the peers'
    from the RCCL segment stream (comm.SegmentStream).  With ``parts_dir`` set (the
    ``TV_STITCH_TRANSPORT=files`` fallback) peers' segments are part files (publish_part)
    that are read once and deleted.  Nothing is joined or copied at the end: close() only
    writes each file's head."""

    def __init__(self, parts_dir: str | None, paths: list, geoms: list, nseg: int, frames: int, fps_num: int, fps_den: int):
        from ..models.hevc import Mp4StreamWriter

        self.parts_dir, self.paths, self.nseg = parts_dir, paths, nseg
        self.own: dict = {}
        self.cv = threading.Condition()
        self.err: BaseException | None = None
        self.stop = False
        self.bytes = [0] * len(paths)
        self.sizes: list = []
        self.writers = [Mp4StreamWriter(p, w, h, fps_num, fps_den, frames) for p, (w, h) in zip(paths, geoms)]
        self.th = threading.Thread(target=self._run, name="stitch", daemon=True)
        self.th.start()

    def put(self, r: int, i: int, data: bytes) -> None:
        with self.cv:
            self.own[(r, i)] = data
            self.cv.notify()

    def _get(self, r: int, i: int) -> bytes:
        path = _part_path(self.parts_dir, r, i) if self.parts_dir else None
        while True:
            with self.cv:
                if (r, i) in self.own:
                    return self.own.pop((r, i))
                if self.stop:
                    raise RuntimeError("stitch cancelled")
            if path and os.path.exists(path):
                with open(path, "rb") as f:
                    data = f.read()
                os.remove(path)
                return data
            with self.cv:  # put() notifies; only the file fallback needs the short poll
                if (r, i) not in self.own and not self.stop:
                    self.cv.wait(0.005 if path else 1.0)

    def _run(self) -> None:
        try:
            for i in range(self.nseg):  # rung-interleaved: every rung's file grows together
                for r, w in enumerate(self.writers):
                    b = self._get(r, i)
                    with trace.span("node_job.stitch_append"):
                        w.append(b)
                    self.bytes[r] += len(b)
            with trace.span("node_job.stitch_close"):
                self.sizes = [w.close() for w in self.writers]
        except BaseException as e:  # noqa: BLE001 - surfaced by finish()
            self.err = e
            for w in self.writers:
                w.abort()

    def finish(self) -> list:
        """Wait for the last segment; returns the file sizes (raises the thread's error)."""
        self.th.join()
        if self.err is not None:
            raise RuntimeError(f"streaming stitch failed: {self.err}") from self.err
        return self.sizes

    def cancel(self) -> None:
        """Stop the stitch thread; it aborts its own writers on the way out (all writer
        calls stay on that thread).  If it does not exit in time (stuck inside a native
        append), the writers and files are left alone and only the error is reported."""
        with self.cv:
            self.stop = True
            self.cv.notify_all()
        self.th.join(timeout=30)
        if self.th.is_alive():
            print("[node_job] stitch thread did not stop within 30 s; its files are left in place",
                  file=sys.stderr, flush=True)
            return
        for p in self.paths:
            if os.path.exists(p):
                os.remove(p)


def _encode_many(items: list, cache) -> tuple[dict, dict]:
    """items: [(key, part, spec, per-frame QPs or None)] -> ({key: annexb}, {key: PartStats});
    batched per spec on the engine (a part may be host frames, device frames or a synthetic
    range)."""
    from ..worker.encoder import PartStats, encode_parts

    out, st, groups = {}, {}, {}
    for key, part, spec, q in items:
        groups.setdefault(spec, []).append((key, part, q))
    for spec, grp in groups.items():
        stats = [PartStats() for _ in grp]
        bits = encode_parts([g[1] for g in grp], spec, cache, stats, [g[2] for g in grp])
        for (k, _, _), b, ps in zip(grp, bits, stats):
            out[k] = b
            st[k] = ps
    return out, st


def _side_plan(input_path: str, audio_stream: int = 0):
    """Audio / English-subtitle streams of the source for the output container (None when
    the source cannot be indexed: the video output is kept, as the reference keeps its MP4
    when the subtitle remux fails, worker/tasks.py:2202-2219)."""
    from ..models.streams import plan_output

    try:
        return plan_output(input_path, audio_stream)
    except Exception as e:  # noqa: BLE001
        print(f"[node_job] side streams skipped: {e}", file=sys.stderr, flush=True)
        return None


def job_entropy(src, width: int, height: int) -> str:
    """Where a node job's WPP substreams are CABAC-coded (TV_ENTROPY overrides).  Decoded
    sources (MPEG-2 / HEVC / AV1 files) spend the host on decoding: from 720p up they use the
    GPU coder; smaller pictures (DVD 480i / 576i), synthetic and y4m sources follow the CPU
    budget ("auto").  A y4m job with the GPU coder measured 4559 vs 4949 frames/s with the
    host writer; at 480p the GPU coder's short per-picture row chain (15 rows, ~3.4 ms per
    picture batch) bounded the DVD job at 955 frames/s against 1633 with the host writer
    (profiles/README.md, round 5)."""
    from ..models import media

    env = os.environ.get("TV_ENTROPY")
    if env:
        return env
    decoded = not isinstance(src, (media.SynthSource, media.Y4MSource))
    return "gpu" if decoded and width * height >= 1280 * 720 else "auto"


def run_job(input_path: str, output: str, height: int | None = None, qp: int = 27, gop: int = 64,
            segment_frames: int = 256, mode: str = "direct", bitrate_kbps: float = 0.0, ladder=None,
            search_range: int = 64, software: bool = False, batch_segments: int = 8,
            resume_dir: str | None = None, max_retries: int = 3, hooks: JobHooks | None = None,
            deblock: bool = True, sao: bool = False, cache=None, crf: int = 0, scenecut: bool = False,
            audio_stream: int = 0, codec: str = "hevc", qindex: int = 0, rc_mode: str = "",
            vbv_maxrate_kbps: float = 0.0, vbv_bufsize_kbit: float = 0.0, bframes: int = 1,
            tools: dict | None = None, deinterlace: bool = False) -> dict:
    """One job over the node's ranks (SPMD).  Rate control: ``bitrate_kbps`` > 0 selects
    frame-level 2-pass, or single-pass ABR when ``rc_mode == "abr"`` (optionally under a VBV:
    ``vbv_maxrate_kbps`` / ``vbv_bufsize_kbit``, checked and repaired per segment, see
    models/ratecontrol.py); else ``crf`` > 0 in-engine CRF; else constant ``qp``.  ``tools``:
    HEVC coding-tool switches (EncodeSpec wpp / rqt / pintra; default all on) -- part of the
    checkpoint fingerprint, so a resume with other tools re-encodes.  ``deinterlace``: bwdif
    (K3, the DVD-native rule of worker/helpers.effective_target_height) on every segment
    before the resize, in the source's field order."""
    import torch

    from ..models import hevc, media
    from ..models.streams import write_output
    from ..worker.encoder import EncodeSpec, EngineCache, PartStats, SynthRange, gpu_available, psnr_from_sse
    from ..worker.helpers import output_geometry

    tool_kw = dict(EncodeSpec(1, 1).tools(), **(tools or {}))
    from .comm import (SegmentStream, allreduce_stats, gather_bytes_to_root, scatter_frames_from_root, scatter_root,
                       stage_segment_frames)

    hooks = hooks or JobHooks()
    trace0 = trace.summary()
    _job_seq[0] += 1
    job_tag = f"j{_job_seq[0]}"  # rendezvous-store keys of this job (a long-lived executor runs many)
    dist = _dist()
    world = dist.get_world_size() if dist else 1
    rank = dist.get_rank() if dist else 0
    dev = _device()
    t0 = time.time()
    src = media.open_source(input_path)
    w0, h0, nfr = src.width, src.height, src.nframes
    heights = [int(x) for x in ladder] if ladder else [int(height or h0)]
    rungs = [output_geometry(w0, h0, th) for th in heights]
    segs = plan_segments(nfr, segment_frames, gop)
    software = software or not gpu_available()
    synthetic = isinstance(src, media.SynthSource)
    deinterlace = bool(deinterlace) and not synthetic
    entropy = job_entropy(src, w0, h0)
    tff = bool(getattr(src, "top_field_first", True))
    fps = src.fps_num / src.fps_den
    abr = rc_mode == "abr" and bitrate_kbps > 0
    vbv = abr and vbv_maxrate_kbps > 0 and vbv_bufsize_kbit > 0
    rc_name = "abr" if abr else ("2pass" if bitrate_kbps > 0 else ("crf" if crf else "cqp"))
    if getattr(src, "bits", 8) != 8 and mode == "scatter":
        mode = "direct"  # 10-bit sources: every rank reads its own range
    # one engine per rung stays resident (a 5-rung ladder thrashed the default 4-engine cache:
    # every eviction re-allocates an engine's HBM and streams)
    own_cache = cache is None and not software
    if own_cache:
        cache = EngineCache(device=dev.index or 0, batch=min(64, batch_segments * max(1, -(-segment_frames // gop))),
                            max_engines=max(4, len(rungs)))
    jobs = [(r, i) for r in range(len(rungs)) for i in range(len(segs))]  # ladder fan-out (P10)
    st = os.stat(input_path) if os.path.exists(input_path) else None
    ckpt = Checkpoint(resume_dir, Checkpoint.fingerprint(
        src=os.path.abspath(input_path), size=st.st_size if st else 0, mtime=st.st_mtime_ns if st else 0,
        rungs=rungs, gop=gop, segment_frames=segment_frames, search_range=search_range, software=software,
        deblock=deblock, sao=sao, scenecut=scenecut, codec=codec, qindex=qindex, crf=crf, bframes=bframes,
        rc=rc_name, bitstream_version=BITSTREAM_VERSION, tools=tool_kw, deinterlace=bool(deinterlace),
        **({"kbps": bitrate_kbps, "vbv": [vbv_maxrate_kbps, vbv_bufsize_kbit] if vbv else None} if abr else {})))
    stats = {"encoded": 0, "resumed": 0, "retried": 0, "reads": 0}
    quality: dict = {}  # (r, i) -> PartStats of segments encoded here
    # streaming stitch (single pass, plain MP4 output): decided identically on every rank
    side = _side_plan(input_path, audio_stream)
    streaming = ((bitrate_kbps <= 0 or abr) and os.environ.get("TV_STREAM_STITCH", "1") != "0"
                 and (side is None or (not side.tracks and side.ext == ".mp4")))
    out_paths = [output if len(rungs) == 1 else f"{os.path.splitext(output)[0]}_{oh}p.mp4" for _, oh in rungs]
    if side is not None:
        out_paths = [os.path.splitext(p)[0] + side.ext for p in out_paths]
    # peers' finished segments reach the stitch rank as part files through the node-local job
    # directory, or with TV_STITCH_TRANSPORT=rccl over the collective backend
    # (comm.SegmentStream).  The stream is proven byte-identical on gloo at world 4 and 8
    # (tests/test_parallel.py) but has not yet run on RCCL at world > 1 (1-GPU test boxes), so
    # the part files stay the default until it has
    transport = os.environ.get("TV_STITCH_TRANSPORT", "files") if world > 1 else "local"
    parts_dir = None
    stitcher = None
    if streaming and transport == "files":
        parts_dir = _attempt_parts_dir(output, job_tag, rank)
    if streaming and rank == 0:
        stitcher = StreamStitcher(parts_dir, [p + ".tmp" for p in out_paths], rungs, len(segs), nfr,
                                  src.fps_num, src.fps_den)
    gather = {"stream": None, "stats": {}}
    # checkpoint (hash + write) and peer part files are written off the critical path
    io_pool = cf.ThreadPoolExecutor(1)
    io_futs: list = []

    def drain_io():
        for f in io_futs:
            f.result()
        io_futs.clear()

    def spec(r):  # the QP is a per-frame input now: one resident engine per rung, whatever the plan
        return EncodeSpec(rungs[r][0], rungs[r][1], qp=qp, gop=gop, search_range=search_range,
                          software=software, deblock=deblock, sao=sao, seed=getattr(src, "seed", 1),
                          crf=0 if bitrate_kbps > 0 else crf, scenecut=scenecut, codec=codec, qindex=qindex,
                          bframes=bframes, entropy=entropy, **tool_kw)

    rc = {"plan": None, "fb": RateFeedback(), "bits": {}}  # pass-2 plan, feedback, per-frame bits
    rung_scale = [(rw * rh) / (rungs[0][0] * rungs[0][1]) for rw, rh in rungs]  # per-rung budget ~ pixels
    if abr:  # one rank-local controller per rung; this batch's plans
        rc.update(abr=[AbrController(qp) for _ in rungs], abr_q={})
    vstat = {"checked": 0, "repaired": 0, "reencodes": 0, "violations": 0}

    def seg_qps(r, i, offset):
        """(integer per-frame QPs or None, checkpoint key) of segment i on rung r."""
        if abr:  # an ABR segment on disk is reused whatever plan produced it (same target)
            return rc["abr_q"][(r, i)], "abr"
        if rc["plan"] is None:
            return None, qp
        q = round_qps(rc["plan"][r][i], offset)
        return q, "p" + hashlib.sha1(q.astype(np.int8).tobytes()).hexdigest()[:12]

    prefetched: dict = {}  # segment -> device frames loaded ahead by the prefetch thread
    stats_lock = threading.Lock()  # stats["reads"]: main thread and prefetch thread

    def load(i):
        """Segment i's source: a synthetic range (generated where it is encoded), a Y4M byte
        range read in parallel into pinned memory and copied to this GPU once for all rungs
        (stage.read_y4m_device), or decoded host frames uploaded once."""
        if i in prefetched:
            fr = prefetched.pop(i)
            buf = getattr(fr, "buf", None)
            if buf is not None and buf.is_cuda:  # allocated on the prefetch stream, used on this one
                buf.record_stream(torch.cuda.current_stream(buf.device))
            return fr
        s, n = segs[i]
        with stats_lock:  # load() also runs on the prefetch thread
            stats["reads"] += 1
        if synthetic:
            return SynthRange(src.seed, w0, h0, src.start + s, n)
        if isinstance(src, media.Y4MSource) and not software:
            from ..ops import stage

            return finish(stage.read_y4m_device(src, s, n, dev, stats=stats))
        return finish(src.read(s, n))

    def finish(fr):
        """Decoded host frames (or Y4M device frames) -> this rank's encoder input: bwdif when
        asked, on the device for GPU encodes."""
        from ..ops import deint

        if software:
            return deint.deinterlace_frames(fr, tff) if deinterlace else fr
        if isinstance(fr, list):
            from ..ops import stage

            fr = stage.upload_frames(fr, dev)
        return deint.deinterlace_device(fr, tff) if deinterlace else fr

    # decoded sources (MPEG-2 / HEVC / AV1 files): a claim's segments are decoded on parallel
    # host threads (each decode is one GOP range; the native decoders release the GIL)
    decoded = not synthetic and not isinstance(src, media.Y4MSource)
    ndec = int(os.environ.get("TV_DECODE_THREADS", "0") or 0) or min(16, len(os.sched_getaffinity(0)))
    dec_pool = cf.ThreadPoolExecutor(ndec) if decoded and ndec > 1 else None

    def preload(ids):
        ids = [i for i in ids if i not in prefetched]
        if dec_pool is None or len(ids) < 2:
            return {}
        with trace.span("node_job.decode", segments=len(ids)):
            hosts = list(dec_pool.map(lambda i: src.read(*segs[i]), ids))
        with stats_lock:
            stats["reads"] += len(ids)
        return {i: finish(fr) for i, fr in zip(ids, hosts)}

    # file sources on the GPU: the next claim is read + uploaded on a side thread / HIP
    # stream while this claim encodes (the reference overlaps GET part with the previous
    # encode only across nodes; here ingest hides behind the engine on every rank)
    # Y4M sources: their reads are pread threads + DMA, so the side thread costs the engine
    # nothing.  Decoded sources (HEVC / AV1 / MPEG-2) prefetch too when the decode pool exists:
    # the next claim's segments decode on the pool's threads (the native decoders release the
    # GIL) and upload on the prefetch stream while this claim encodes.
    prefetch = (not synthetic and not software and dev.type == "cuda"
                and (isinstance(src, media.Y4MSource) or dec_pool is not None)
                and os.environ.get("TV_PREFETCH", "1") != "0")
    prefetcher = None
    if prefetch:
        def _prefetch_init():
            torch.cuda.set_device(dev)
            _prefetch_init.stream = torch.cuda.Stream(dev)

        prefetcher = cf.ThreadPoolExecutor(1, initializer=_prefetch_init)

        def load_ahead(ids):
            with torch.cuda.stream(_prefetch_init.stream), trace.span("node_job.prefetch"):
                got = preload(ids)
                return {i: got[i] if i in got else load(i) for i in ids}

    def encode_segments(seg_ids, source_of, on_loaded=None) -> dict:
        """Work item = one segment with ALL its rungs: the source range is read (or received)
        once, every rung is staged from it on the device, and each rung engine then encodes
        the claimed segments in one batched launch.  In pass 2 the per-frame QP plan of
        every segment is offset by this rank's rate feedback so far."""
        out, todo, keep, plans = {}, [], [], {}
        offset = rc["fb"].offset()
        if abr:
            frames = [segs[i][1] for i in seg_ids]
            for r, ctl in enumerate(rc["abr"]):
                nominal = bitrate_kbps * 1000 * sum(frames) / fps * rung_scale[r]
                for i, q in zip(seg_ids, ctl.plan(nominal, frames)):
                    rc["abr_q"][(r, i)] = q
        for i in seg_ids:
            need = []
            for r in range(len(rungs)):
                q, key = seg_qps(r, i, offset)
                plans[(r, i)] = (q, key)
                b = ckpt.load(r, i, key)
                if b is not None:
                    out[(r, i)] = b
                    stats["resumed"] += 1
                else:
                    need.append(r)
            if need:
                with trace.span("node_job.load"):
                    part = source_of(i)
                todo.extend(((r, i), part, spec(r), plans[(r, i)][0]) for r in need)
                keep.append(part)
        if on_loaded is not None:
            on_loaded()
        if todo:
            with trace.span("node_job.encode", segments=len(todo)):
                got, qual = _encode_many(todo, cache)
            if vbv:
                with trace.span("node_job.vbv", segments=len(todo)):
                    vbv_repair(todo, got, qual, plans)
            for (r, i), b in got.items():
                io_futs.append(io_pool.submit(ckpt.save, r, i, plans[(r, i)][1], b))
                out[(r, i)] = b
                quality[(r, i)] = qual[(r, i)]
                stats["encoded"] += 1
        del keep  # device / host source copies of this claim are released here
        for (r, i), b in out.items():
            fb = frame_sizes(b)
            rc["bits"][(r, i)] = fb
            q = plans[(r, i)][0]
            if q is not None and not abr:  # rate feedback: actual vs the model's prediction at these QPs
                rc["fb"].record(8.0 * sum(fb), float(predict_bits(rc["b1"][(r, i)], qp, q).sum()))
        if abr:
            for r, ctl in enumerate(rc["abr"]):
                ctl.record(sum(8.0 * sum(rc["bits"][(r, i)]) for i in seg_ids))
        if streaming:  # the stitch rank takes them now; this rank keeps no bitstream
            for (r, i), b in out.items():
                if gather["stream"] is not None:
                    gather["stream"].put((r, i), b)
                elif stitcher is not None:
                    stitcher.put(r, i, b)
                else:
                    io_futs.append(io_pool.submit(publish_part, parts_dir, r, i, b))
            out = {k: b"" for k in out}
        with trace.span("node_job.hooks"):
            for i in seg_ids:
                hooks.segment_done(segs[i][1])
        return out

    def vbv_repair(todo, got, qual, plans):
        """Per-segment VBV (see models/ratecontrol.py): a segment that underflows the decoder
        buffer or ends emptier than it started is re-encoded at a coarser QP (the model's
        offset for its compliant scale, +1 per failed attempt), batched with the other
        violators of this claim; after 3 attempts it is kept and counted as a violation."""
        maxrate, buf = vbv_maxrate_kbps * 1000 * 1.0, vbv_bufsize_kbit * 1000.0
        items = {k: (part, sp) for k, part, sp, _ in todo}
        bad = {}
        for k, b in got.items():
            vstat["checked"] += 1
            fb = 8.0 * np.asarray(frame_sizes(b, decode_order=True), np.float64)  # VBV: decoding order
            if not vbv_ok(fb, fps * 1.0, maxrate * rung_scale[k[0]], buf * rung_scale[k[0]]):
                bad[k] = fb
        fixed = set()
        for attempt in range(3):
            if not bad:
                break
            redo = []
            for k, fb in bad.items():
                sc = vbv_scale(fb, fps, maxrate * rung_scale[k[0]], buf * rung_scale[k[0]])
                q0 = plans[k][0] if plans[k][0] is not None else np.full(len(fb), qp)
                q = np.clip(np.asarray(q0) + vbv_repair_offset(sc, attempt), 0, 51)
                plans[k] = (q, plans[k][1])
                rc["abr_q"][k] = q  # the reported plan is the one encoded
                redo.append((k, items[k][0], items[k][1], q))
            vstat["reencodes"] += len(redo)
            g2, q2 = _encode_many(redo, cache)
            bad = {}
            for k, b in g2.items():
                got[k], qual[k] = b, q2[k]
                fb = 8.0 * np.asarray(frame_sizes(b, decode_order=True), np.float64)  # VBV: decoding order
                if vbv_ok(fb, fps, maxrate * rung_scale[k[0]], buf * rung_scale[k[0]]):
                    fixed.add(k)
                else:
                    bad[k] = fb
        vstat["repaired"] += len(fixed)
        vstat["violations"] += len(bad)

    def encode_pass() -> dict:
        mine = {}
        if mode == "scatter" and world > 1:
            # rounds of `world` segments; the round's root (rotating, comm.scatter_root) reads
            # them, stages each one straight into a device buffer and sends each peer its
            # segment over one xGMI hop; the received tensor stays on the device
            fsz = w0 * h0 * 3 // 2
            for rd, base in enumerate(range(0, len(segs), world)):
                if hooks.halted():
                    raise RuntimeError("job halted")
                rnd = list(range(base, min(len(segs), base + world)))
                n_max = max(segs[i][1] for i in rnd)
                shape = (n_max, fsz)
                root = scatter_root(rd, world)
                payload = None
                if rank == root:
                    payload = []
                    for k in range(world):
                        fr = src.read(*segs[rnd[k]]) if k < len(rnd) else []
                        stats["reads"] += k < len(rnd)
                        stats["roots"] = stats.get("roots", 0) + (k == 0)
                        payload.append(stage_segment_frames(fr, shape, dev))
                got = scatter_frames_from_root(payload, shape, dev, root=root)
                if rank < len(rnd):
                    i = rnd[rank]
                    n = segs[i][1]
                    if got.is_cuda and not software:
                        from ..ops import stage

                        part = stage.from_flat(got, w0, h0, n)
                    else:
                        g = got.cpu().numpy()
                        ysz, csz = w0 * h0, w0 * h0 // 4
                        part = [(x[:ysz].reshape(h0, w0), x[ysz:ysz + csz].reshape(h0 // 2, w0 // 2),
                                 x[ysz + csz:].reshape(h0 // 2, w0 // 2)) for x in g[:n]]
                    mine.update(encode_segments([i], lambda _i, p=part: p))
        else:
            wq = WorkQueue(f"{job_tag}_pass{encode_pass.calls}", list(range(len(segs))), world, max_retries)
            fault.check("rank", rank)  # TV_FAULT=rank:<r>:hang|die|fail (tests)

            def run(batch, on_loaded=None):
                todo = []
                for i in batch:
                    try:
                        fault.check("segment", i)
                        todo.append(i)
                    except fault.InjectedFault as e:
                        wq.fail((i,), str(e))
                if not todo:
                    return
                try:
                    prefetched.update(preload(todo))
                    mine.update(encode_segments(todo, load, on_loaded))
                except Exception as e:  # a real engine/IO failure: every item goes back
                    for i in todo:
                        wq.fail((i,), repr(e))

            ahead = None  # (next claim, future of its loaded segments)
            try:
                while True:
                    msg = wq.aborted()
                    if msg:
                        raise RuntimeError(msg)
                    if hooks.halted():
                        wq.fail_all("job halted")
                        raise RuntimeError("job halted")
                    if ahead is not None:
                        claimed, fut = ahead
                        ahead = None
                        with trace.span("node_job.prefetch_wait"):
                            try:
                                prefetched.update(fut.result())
                            except Exception:  # noqa: BLE001 - run() reloads and takes the failure path
                                pass
                    else:
                        with trace.span("node_job.claim"):
                            claimed = wq.claim(batch_segments)  # a batch -> one batched launch per rung
                    if not claimed:
                        break
                    # claim ahead only while enough work remains for every rank: at the tail of a
                    # job a prefetched batch would sit idle on this rank while others starve
                    pend = None  # [next claim, its prefetch future once submitted]
                    if (prefetcher is not None and len(claimed) == batch_segments
                            and wq.unclaimed() >= world * batch_segments):
                        with trace.span("node_job.claim"):
                            nxt = wq.claim(batch_segments)
                        if nxt:
                            pend = [nxt, None]
                    cold = pend is not None and not all(i in prefetched for i in claimed)

                    def start_ahead(p=pend):
                        if p is not None and p[1] is None:
                            p[1] = prefetcher.submit(load_ahead, p[0])

                    if not cold:
                        start_ahead()
                    # a claim not prefetched (a job's first) loads on this thread first: its
                    # successor's prefetch starts once those reads are done instead of halving
                    # their host-memory / DMA bandwidth while the engine waits on them
                    run(claimed, start_ahead if cold else None)
                    start_ahead()  # run() failed before its loads finished
                    if pend is not None:
                        ahead = (pend[0], pend[1])
                    if len(claimed) < batch_segments and ahead is None:
                        break
            finally:
                if ahead is not None:
                    ahead[1].cancel()
                prefetched.clear()
            wq.fresh_done()
            while not wq.finished():  # failed segments, re-published for any rank
                msg = wq.aborted()
                if msg:
                    raise RuntimeError(msg)
                it = wq.claim_retry()
                if it is None:
                    time.sleep(0.01)
                    continue
                try:
                    stats["retried"] += 1
                    run([it[0]])
                finally:
                    wq.retry_done()
            msg = wq.aborted()
            if msg:
                raise RuntimeError(msg)
        encode_pass.calls += 1
        return mine

    try:
        encode_pass.calls = 0
        cdev = dev if dev.type == "cuda" else torch.device("cpu")

        def agreed_pass():
            """encode_pass + a collective verdict: a rank that failed (halt, abort, engine
            error) never strands its peers inside the next collective."""
            err, got = None, {}
            hooks.new_pass(agreed_pass.n)
            agreed_pass.n += 1
            if streaming and transport == "rccl":
                gather["stream"] = SegmentStream(cdev, lambda k, b: stitcher.put(*k, b), root=0)
            try:
                got = encode_pass()
                with trace.span("node_job.io_drain"):
                    drain_io()  # checkpoints and part files of this pass are on disk
            except Exception as e:  # noqa: BLE001 - re-raised below on every rank
                err = e
            if gather["stream"] is not None:  # this rank is done: leave the gather rounds
                with trace.span("node_job.stream_close"):
                    try:
                        gather["stats"] = gather["stream"].close()
                    except Exception as e:  # noqa: BLE001
                        err = err or e
                gather["stream"] = None
            with trace.span("node_job.verdict"):
                failed = allreduce_stats([1.0 if err else 0.0], cdev, op="max")[0]
            if failed:
                raise err if err is not None else RuntimeError("a peer rank failed this job")
            return got

        agreed_pass.n = 0
        passes = 1
        rc_errors: list = []  # per pass after pass 1: achieved / target - 1, per rung
        if bitrate_kbps > 0 and not abr:
            # pass 1 at the base QP -> every frame's bits, all-reduced over the node (RCCL) ->
            # one global per-frame QP plan -> pass 2 with rank-local rate feedback
            agreed_pass()
            starts = np.cumsum([0] + [n for _, n in segs])
            flat = np.zeros(len(rungs) * nfr)
            for (r, i), fb in rc["bits"].items():
                flat[r * nfr + starts[i]:r * nfr + starts[i] + len(fb)] = 8.0 * np.asarray(fb, np.float64)
            flat = allreduce_stats(flat, cdev)  # RC statistics all-reduce
            rc["b1"] = {(r, i): flat[r * nfr + starts[i]:r * nfr + starts[i] + n] for r in range(len(rungs))
                        for i, (_, n) in enumerate(segs)}
            plan = []
            for r in range(len(rungs)):
                target = bitrate_kbps * 1000 * nfr / fps * rung_scale[r]
                per_seg, _ = plan_frame_qps([rc["b1"][(r, i)] for i in range(len(segs))], qp, target,
                                            key_offset=-2.0 if codec == "av1" else None,
                                            qcomp=QCOMP_BFRAMES if bframes > 1 and codec != "av1" else QCOMP,
                                            slope=AV1_SLOPE if codec == "av1" else SLOPE)
                plan.append(per_seg)
            rc["plan"] = plan
            targets = [bitrate_kbps * 1000 * nfr / fps * (rw * rh) / (rungs[0][0] * rungs[0][1]) for rw, rh in rungs]
            passes = 1
            for _ in range(2):  # pass 2, plus a corrected pass 3 only when pass 2 misses by > RC_TOLERANCE
                rc["bits"] = {}
                rc["fb"] = RateFeedback()
                quality.clear()
                mine = agreed_pass()
                passes += 1
                got = np.zeros(len(rungs))
                for (r, i), fb in rc["bits"].items():
                    if (r, i) in mine:
                        got[r] += 8.0 * sum(fb)
                got = allreduce_stats(got, cdev)
                err = got / np.asarray(targets) - 1.0
                rc_errors.append([round(float(e), 4) for e in err])
                if np.all(np.abs(err) <= RC_TOLERANCE):
                    break
                # the response to a uniform QP shift around the pass-2 operating point: move
                # every frame's plan by the rung's residual (the model slope only scales it)
                for r in range(len(rungs)):
                    d = SLOPE * math.log2(max(got[r], 1.0) / targets[r])
                    plan[r] = [q + d for q in plan[r]]
                    for i in range(len(segs)):  # feedback baseline = pass-2 bits at the pass-2 QPs
                        rc["b1"][(r, i)] = predict_bits(rc["b1"][(r, i)], 0, -d)
        else:
            mine = agreed_pass()
            if abr:  # one pass: the achieved rate per rung over the node, and the VBV record
                got = np.zeros(len(rungs))
                for (r, i), fb in rc["bits"].items():
                    if (r, i) in mine:
                        got[r] += 8.0 * sum(fb)
                vv = allreduce_stats(np.concatenate([got, [vstat[k] for k in sorted(vstat)]]), cdev)
                targets = [bitrate_kbps * 1000 * nfr / fps * sc for sc in rung_scale]
                rc_errors.append([round(float(e), 4) for e in vv[:len(rungs)] / np.asarray(targets) - 1.0])
                for j, k in enumerate(sorted(vstat)):
                    vstat[k] = int(vv[len(rungs) + j])
        t_enc = time.time() - t0
        # quality: per-rung frames + SSE of the segments encoded on this rank, all-reduced
        qv = np.zeros((len(rungs), 4))
        for (r, i), ps in quality.items():
            qv[r] += [ps.frames, *ps.sse]
        qv = allreduce_stats(qv.reshape(-1), cdev).reshape(len(rungs), 4)
        # gather bitstreams to rank 0 (one message per rank: json index + concatenated bytes)
        keys = sorted(mine)
        header = json.dumps({"seg": [[r, i, len(mine[(r, i)])] for r, i in keys], "stats": stats}).encode()
        blob = len(header).to_bytes(8, "little") + header + b"".join(mine[k] for k in keys)
        with trace.span("node_job.gather"):
            parts = gather_bytes_to_root(blob, cdev) if world > 1 else [blob]
        result = {"world": world, "segments": len(segs), "rungs": [list(x) for x in rungs], "passes": passes,
                  "rc": rc_name, "rc_errors": rc_errors,
                  "stitch": {"streaming": streaming, "transport": transport if streaming else "gather",
                             **{k: round(v, 4) if isinstance(v, float) else v for k, v in gather["stats"].items()}}}
        if abr:
            result["abr_steps_rank0"] = [c.log for c in rc["abr"]]  # [actual, want, offset] / nominal
        if vbv:
            result["vbv"] = dict(vstat, maxrate_kbps=vbv_maxrate_kbps, bufsize_kbit=vbv_bufsize_kbit)
        if rank == 0:
            streams: dict = {}
            per_rank = []
            for p in parts:  # (empty bitstream lists when the stitch streamed)
                p = memoryview(p)
                hl = int.from_bytes(p[:8], "little")
                hdr = json.loads(bytes(p[8:8 + hl]))
                idx = hdr["seg"]
                per_rank.append(hdr["stats"])
                off = 8 + hl
                for r, i, n in idx:
                    streams[(r, i)] = p[off:off + n]
                    off += n
            outs = []
            if stitcher is not None:  # every segment is already in the streaming files
                with trace.span("node_job.stitch_wait"):
                    sizes = stitcher.finish()
                for r, (ow, oh) in enumerate(rungs):
                    os.replace(out_paths[r] + ".tmp", out_paths[r])
                    outs.append({"path": out_paths[r], "bytes": sizes[r], "width": ow, "height": oh,
                                 "seg_bytes": stitcher.bytes[r]})
            else:
                missing = [k for k in jobs if k not in streams]
                if missing:
                    raise RuntimeError(f"segments missing at stitch: {missing}")
                for r, (ow, oh) in enumerate(rungs):
                    seg_bits = [streams[(r, i)] for i in range(len(segs))]
                    with trace.span("node_job.mux"):  # streamed from the gathered buffers, no joined copy
                        path, nbytes = write_output(seg_bits, ow, oh, src.fps_num, src.fps_den, out_paths[r], side)
                    outs.append({"path": path, "bytes": nbytes, "width": ow, "height": oh,
                                 "seg_bytes": sum(len(b) for b in seg_bits)})
            for r, o in enumerate(outs):
                q = psnr_from_sse(qv[r, 1:], o["width"] * o["height"] * qv[r, 0]) if qv[r, 0] else {}
                o.update(frames=nfr, fps_num=src.fps_num, fps_den=src.fps_den,
                         kbps=o.pop("seg_bytes") * 8 / (nfr * src.fps_den / src.fps_num) / 1000,
                         psnr_y=round(q["y"], 3) if q else None, psnr_yuv=round(q["yuv"], 3) if q else None,
                         quality_frames=int(qv[r, 0]))
            el = time.time() - t0
            result.update(side_fields=side.fields if side else {}, side_warnings=side.warnings if side else [])
            result.update(trace=trace.since(trace0), per_rank=per_rank, outputs=outs, qp_plan=[[round(float(np.mean(q)), 2) for q in row] for row in rc["plan"]] if rc["plan"] else
                          [[round(float(np.mean(rc["abr_q"][(r, i)])), 2) if (r, i) in rc["abr_q"] else None
                            for i in range(len(segs))] for r in range(len(rungs))] if abr else
                          [[qp] * len(segs) for _ in rungs], rc_offset=round(rc["fb"].offset(), 3),
                          seconds=round(el, 3), encode_seconds=round(t_enc, 3),
                          fps=round(nfr * len(rungs) / el, 2), encode_fps=round(nfr * len(rungs) * passes / max(t_enc, 1e-9), 2))
    except BaseException:
        if stitcher is not None:
            stitcher.cancel()
        raise
    finally:
        io_pool.shutdown(wait=True)
        if prefetcher is not None:
            prefetcher.shutdown(wait=True)
        if dec_pool is not None:
            dec_pool.shutdown(wait=True)
        if parts_dir and rank == 0:
            import shutil

            shutil.rmtree(os.path.dirname(parts_dir), ignore_errors=True)
    if own_cache:
        cache.close()
    return result


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--input", required=True)
    ap.add_argument("--output", required=True)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--qp", type=int, default=27)
    ap.add_argument("--gop", type=int, default=64)
    ap.add_argument("--segment-frames", type=int, default=256)
    ap.add_argument("--mode", choices=("direct", "scatter"), default="direct")
    ap.add_argument("--bitrate-kbps", type=float, default=0.0)
    ap.add_argument("--ladder", default="")
    ap.add_argument("--software", action="store_true")
    ap.add_argument("--bframes", type=int, default=1, help="HEVC hierarchical-B mini-GOP (1 = I P P P)")
    ap.add_argument("--backend", default=None)
    ap.add_argument("--resume-dir", default=None, help="segment checkpoint directory (resume / elastic restart)")
    ap.add_argument("--max-retries", type=int, default=3, help="per-segment retry budget before the job aborts")
    ap.add_argument("--timeout-sec", type=float, default=600.0, help="collective timeout (a hung rank surfaces)")
    ap.add_argument("--no-wpp", dest="wpp", action="store_false", help="HEVC: one CABAC substream per slice (host)")
    ap.add_argument("--no-rqt", dest="rqt", action="store_false", help="HEVC: no residual quadtree")
    ap.add_argument("--no-cascade", dest="cascade", action="store_false", help="HEVC: flat QP (no I P P P QP cascade)")
    ap.add_argument("--no-pintra", dest="pintra", action="store_false", help="HEVC: no intra CUs in P pictures")
    ap.add_argument("--no-rdoq", dest="rdoq", action="store_false", help="HEVC: no RDOQ-lite coefficient-group trimming")
    ap.add_argument("--deinterlace", action="store_true", help="bwdif every segment (DVD-native interlaced sources)")
    a = ap.parse_args(argv)
    import torch
    import torch.distributed as dist

    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        backend = a.backend or ("nccl" if torch.cuda.is_available() and not a.software else "gloo")
        import datetime

        kw = {}
        if backend == "nccl":  # eager communicator on this rank's GPU (not lazily on a first p2p)
            local = int(os.environ.get("LOCAL_RANK", "0"))
            torch.cuda.set_device(local)
            kw["device_id"] = torch.device("cuda", local)
        dist.init_process_group(backend, timeout=datetime.timedelta(seconds=a.timeout_sec), **kw)
    ladder = [int(x) for x in a.ladder.split(",") if x.strip()] or None
    res = run_job(a.input, a.output, a.height, a.qp, a.gop, a.segment_frames, a.mode, a.bitrate_kbps, ladder,
                  software=a.software, resume_dir=a.resume_dir, max_retries=a.max_retries, bframes=a.bframes,
                  tools={"wpp": a.wpp, "rqt": a.rqt, "pintra": a.pintra, "cascade": a.cascade, "rdoq": a.rdoq},
                  deinterlace=a.deinterlace)
    if int(os.environ.get("RANK", "0")) == 0:
        print(json.dumps(res), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
