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
5. bitstreams are gathered to rank 0 (all_gather of sizes + grouped send/recv) and muxed
   in segment order into one faststart MP4; ``--ladder`` fans rungs x segments out over
   all ranks and writes one MP4 per rung.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np


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
        self.key, self.local = key, 0

    def next(self) -> int:
        if self.store is None:
            self.local += 1
            return self.local - 1
        return int(self.store.add(self.key, 1)) - 1


def _encode_many(items: list, spec_for, cache) -> dict:
    """items: [(key, frames, spec)] -> {key: annexb}; batched per spec on the engine."""
    from ..worker.encoder import encode_parts

    out, groups = {}, {}
    for key, frames, spec in items:
        groups.setdefault(spec, []).append((key, frames))
    for spec, grp in groups.items():
        for k, b in zip([g[0] for g in grp], encode_parts([g[1] for g in grp], spec, cache)):
            out[k] = b
    return out


def run_job(input_path: str, output: str, height: int | None = None, qp: int = 27, gop: int = 64,
            segment_frames: int = 256, mode: str = "direct", bitrate_kbps: float = 0.0, ladder=None,
            search_range: int = 16, software: bool = False, batch_segments: int = 8) -> dict:
    import torch

    from ..models import hevc, media
    from ..worker.encoder import EncodeSpec, EngineCache, gpu_available, prepare_frames
    from ..worker.helpers import output_geometry
    from .comm import allreduce_stats, gather_bytes_to_root, scatter_frames_from_root

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
    cache = None if software else EngineCache(device=dev.index or 0, batch=batch_segments)
    jobs = [(r, i) for r in range(len(rungs)) for i in range(len(segs))]  # ladder fan-out (P10)

    def spec(r, q):
        return EncodeSpec(rungs[r][0], rungs[r][1], qp=int(q), gop=gop, search_range=search_range,
                          software=software)

    def load(i):
        s, n = segs[i]
        return src.read(s, n)

    def encode_pass(qps) -> dict:
        mine = {}
        if mode == "scatter" and world > 1:
            # round-robin rounds: rank 0 reads `world` segments and sends one to each rank
            fsz = w0 * h0 * 3 // 2
            for base in range(0, len(jobs), world):
                rnd = jobs[base:base + world]
                n_max = max(segs[i][1] for _, i in rnd)
                shape = (n_max, fsz)
                payload = None
                if rank == 0:
                    payload = []
                    for k in range(world):
                        buf = np.zeros(shape, np.uint8)
                        if k < len(rnd):
                            for f, (y, u, v) in enumerate(load(rnd[k][1])):
                                buf[f] = np.concatenate([y.ravel(), u.ravel(), v.ravel()])
                        payload.append(buf)
                got = scatter_frames_from_root(payload, shape, dev).cpu().numpy()
                if rank < len(rnd):
                    r, i = rnd[rank]
                    ysz, csz = w0 * h0, w0 * h0 // 4
                    frames = [(x[:ysz].reshape(h0, w0), x[ysz:ysz + csz].reshape(h0 // 2, w0 // 2),
                               x[ysz + csz:].reshape(h0 // 2, w0 // 2)) for x in got[:segs[i][1]]]
                    fr = prepare_frames(frames, *rungs[r])
                    mine.update(_encode_many([((r, i), fr, spec(r, qps[r][i]))], None, cache))
        else:
            ctr = _Counter(f"tv_seg_pass{encode_pass.calls}")  # same key on every rank
            while True:
                claimed = []
                for _ in range(max(1, batch_segments)):  # claim a batch -> one batched launch
                    k = ctr.next()
                    if k >= len(jobs):
                        break
                    claimed.append(jobs[k])
                if not claimed:
                    break
                items = [((r, i), prepare_frames(load(i), *rungs[r]), spec(r, qps[r][i])) for r, i in claimed]
                mine.update(_encode_many(items, None, cache))
                if len(claimed) < batch_segments:
                    break
        encode_pass.calls += 1
        return mine

    encode_pass.calls = 0
    base = [[qp] * len(segs) for _ in rungs]
    passes = 1
    if bitrate_kbps > 0:
        first = encode_pass(base)
        sizes = np.zeros(len(jobs))
        for (r, i), b in first.items():
            sizes[jobs.index((r, i))] = len(b) * 8
        sizes = allreduce_stats(sizes, dev if dev.type == "cuda" else torch.device("cpu"))  # RC stats all-reduce
        fps = src.fps_num / src.fps_den
        qps = []
        for r in range(len(rungs)):
            idx = [jobs.index((r, i)) for i in range(len(segs))]
            scale = (rungs[r][0] * rungs[r][1]) / (rungs[0][0] * rungs[0][1])  # per-rung budget ~ pixels
            target = bitrate_kbps * 1000 * nfr / fps * scale
            qps.append(list(qp_plan_two_pass(sizes[idx], [n for _, n in segs], qp, target)))
        passes = 2
    else:
        qps = base
    mine = encode_pass(qps)
    # gather bitstreams to rank 0 (one message per rank: json index + concatenated bytes)
    keys = sorted(mine)
    header = json.dumps([[r, i, len(mine[(r, i)])] for r, i in keys]).encode()
    blob = len(header).to_bytes(8, "little") + header + b"".join(mine[k] for k in keys)
    parts = gather_bytes_to_root(blob, dev) if world > 1 else [blob]
    result = {"world": world, "segments": len(segs), "rungs": [list(x) for x in rungs], "passes": passes}
    if rank == 0:
        streams: dict = {}
        for p in parts:
            hl = int.from_bytes(p[:8], "little")
            idx = json.loads(p[8:8 + hl])
            off = 8 + hl
            for r, i, n in idx:
                streams[(r, i)] = p[off:off + n]
                off += n
        outs = []
        for r, (ow, oh) in enumerate(rungs):
            annexb = b"".join(streams[(r, i)] for i in range(len(segs)))
            path = output if len(rungs) == 1 else f"{os.path.splitext(output)[0]}_{oh}p.mp4"
            data = hevc.mux_mp4(annexb, ow, oh, src.fps_num, src.fps_den)
            tmp = path + ".tmp"
            with open(tmp, "wb") as f:
                f.write(data)
            os.replace(tmp, path)
            outs.append({"path": path, "bytes": len(data), "width": ow, "height": oh,
                         "kbps": len(annexb) * 8 / (nfr * src.fps_den / src.fps_num) / 1000})
        result.update(outputs=outs, qp_plan=[[int(q) for q in row] for row in qps],
                      seconds=round(time.time() - t0, 3), fps=round(nfr * len(rungs) / (time.time() - t0), 2))
    if cache:
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
    ap.add_argument("--backend", default=None)
    a = ap.parse_args(argv)
    import torch
    import torch.distributed as dist

    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        backend = a.backend or ("nccl" if torch.cuda.is_available() and not a.software else "gloo")
        if backend == "nccl":
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_process_group(backend)
    ladder = [int(x) for x in a.ladder.split(",") if x.strip()] or None
    res = run_job(a.input, a.output, a.height, a.qp, a.gop, a.segment_frames, a.mode, a.bitrate_kbps, ladder,
                  software=a.software)
    if int(os.environ.get("RANK", "0")) == 0:
        print(json.dumps(res), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
