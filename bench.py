#!/usr/bin/env python3
"""Flagship benchmark: encoded frames/s (whole node) of the MI355X HEVC engine at fixed QP,
reporting the resulting PSNR — BASELINE.json metric, configs #2 (1080p30 HEVC on one
MI355X) and #3 (4K30 HEVC GOP-aligned segments data-parallel across GPUs).

One step = every rank encodes `batch` GOP-aligned segments of `gop` synthetic frames
(weak scaling: per-GPU work is fixed as N grows), then the encoded bitstreams are gathered
to the stitch rank (rank 0) with RCCL point-to-point over xGMI and the rate/quality
statistics are all-reduced — the intra-node data plane that replaces the reference's HTTP
part upload to the stitcher (reference worker/tasks.py:1655-1674).

    python bench.py --gpus N --steps K --warmup W [--res 1080p|4k] [--batch B] [--gop G]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "encoded frames/sec (whole node) at fixed PSNR, 1080p & 4K HEVC, 1/2/4/8 MI355X"
RES = {"1080p": (1920, 1080), "4k": (3840, 2160), "720p": (1280, 720), "360p": (640, 360)}
SRC = {"8k": (7680, 4320), "4k": (3840, 2160), "1080p": (1920, 1080)}
LADDER_METRIC = "HDR10 source frames/sec (whole node) through a tone-map + Lanczos + HEVC ABR ladder"


def _dist_setup(args):
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    return world, rank, local, dev


def ladder_main(args) -> None:
    """BASELINE config #5 on N GPUs: each rank pushes `batch` segments x `gop` frames of a
    seeded synthetic HDR10 (P010, PQ) source through tone-map -> every rung's Lanczos
    downscale -> every rung's HEVC engine (all HBM-resident, rungs encoded concurrently);
    bitstreams gathered to rank 0 over RCCL.  value = source frames/s (each one produces
    one frame on every rung)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from thinvids_amd.models.abr import AbrLadder
    from thinvids_amd.parallel.comm import gather_bytes_to_root

    world, rank, local, dev = _dist_setup(args)
    sw, sh = SRC[args.src]
    heights = [int(x) for x in args.ladder.split(",") if x.strip()]
    batch = args.batch or 24  # measured 8K ladder: b8 183, b16 360, b24 373, b32 365 source frames/s
    lad = AbrLadder(sw, sh, heights, qp=args.qp, segments=batch, gop=args.gop, device=local,
                    threads=args.threads or None, seed=args.seed, search_range=args.range, sao=args.sao)

    def prep(i: int):  # step i's source -> tone-map -> rungs into staging slot i % 2
        base = (i * world + rank) * batch
        lad.prepare_synthetic([(base + b) * args.gop for b in range(batch)], slot=i % 2)
        torch.cuda.current_stream(dev).synchronize()

    # step i encodes staging slot i % 2 while this thread prepares step i + 1 into the other
    # slot (every step = one full prep + one full encode; prep(0) runs before warm-up)
    prep(0)
    counter = [0]

    def step(_s: int):
        i = counter[0]
        counter[0] += 1
        segs = lad.encode_overlapped(batch, i % 2, prepare_next=lambda: prep(i + 1))
        nbytes = sum(len(x) for r in segs for x in r)
        stats = np.array([batch * args.gop, nbytes], dtype=np.float64)
        if world > 1:
            t = torch.from_numpy(stats).to(dev)
            dist.all_reduce(t)
            stats = t.cpu().numpy()
            gather_bytes_to_root(b"".join(x for r in segs for x in r), dev)
        return stats

    for s in range(args.warmup):
        step(-1 - s)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tot = None
    step_ms = []
    for s in range(args.steps):
        ts = time.perf_counter()
        st = step(s)
        step_ms.append(round(1000 * (time.perf_counter() - ts), 2))
        tot = st if tot is None else tot + st
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el_t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
    el = float(el_t.item())
    q = lad.psnr()
    if rank == 0:
        tm = [e.timing() for e in lad.engines]
        print(json.dumps({
            "metric": LADDER_METRIC,
            "value": round(tot[0] / el, 2),
            "unit": "source frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000 * el / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "P010 in / uint8 video / int32 integer transforms (bit-exact HEVC)",
            "data": "synthetic (seeded procedural HDR10 P010 source generated on GPU)",
            "config": {
                "model": f"HDR10 {args.src} -> {len(lad.rungs)}-rung HEVC Main CQP{args.qp} ladder",
                "global_batch": world * batch,
                "seq_len": args.gop,
                "parallelism": f"dp{world}",
                "source": f"{sw}x{sh}",
                "rungs": [f"{w}x{h}" for w, h in lad.rungs],
                "output_frames_per_s": round(tot[0] * len(lad.rungs) / el, 2),
                "psnr_y_db_per_rung": [round(x["y"], 3) for x in q],
                "mbit_per_step": round(tot[1] * 8 / 1e6 / args.steps, 2),
                "last_step_gpu_ms_per_rung": [round(t["gpu_ms"], 2) for t in tm],
                "last_step_entropy_cpu_ms_per_rung": [round(t["entropy_cpu_ms"], 2) for t in tm],
                "step_ms": step_ms,
            },
        }), flush=True)
    lad.close()
    if world > 1:
        dist.destroy_process_group()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--res", default="1080p", choices=sorted(RES))
    ap.add_argument("--batch", type=int, default=0, help="segments per GPU per step (0 = auto)")
    ap.add_argument("--gop", type=int, default=16, help="frames per GOP-aligned segment")
    ap.add_argument("--qp", type=int, default=27)
    ap.add_argument("--sao", action="store_true", help="enable SAO (in-loop sample adaptive offset)")
    ap.add_argument("--range", type=int, default=16)
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--ladder", default="", help="ABR mode (config #5): rung heights, e.g. 2160,1440,1080,720,480")
    ap.add_argument("--src", default="8k", choices=sorted(SRC), help="ABR mode: HDR10 source resolution")
    args = ap.parse_args()
    if args.ladder:
        return ladder_main(args)

    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    from thinvids_amd.models.gpu_engine import GpuEngine
    from thinvids_amd.parallel.comm import gather_bytes_to_root

    w, h = RES[args.res]
    # segments per GPU: enough CTBs per wavefront diagonal of the I-frame recon and per
    # motion-search launch to fill 256 CUs (measured: 1080p 8 -> 32 segments = +47 %); the
    # engine splits them into two stream groups one frame apart (measured on MI355X:
    # 1080p 32 -> 48 segments +3 %, 4K 16 -> 24 segments +9 %; profiles/README.md)
    batch = args.batch or (48 if args.res in ("1080p", "720p", "360p") else 24)
    eng = GpuEngine(width=w, height=h, qp=args.qp, batch=batch, gop=args.gop, search_range=args.range, sao=args.sao,
                    seed=args.seed, threads=args.threads or None, device=local)

    prof = {"encode": 0.0, "post": 0.0}

    def step(s: int):
        base = (s * world + rank) * batch
        t_a = time.perf_counter()
        segs = eng.encode_synthetic([(base + b) * args.gop for b in range(batch)])
        t_b = time.perf_counter()
        prof["encode"] += t_b - t_a
        sse = np.array([eng.sse(b) for b in range(batch)]).sum(0)
        nbytes = sum(len(x) for x in segs)
        stats = np.array([batch * args.gop, nbytes, *sse], dtype=np.float64)
        gathered = None
        if world > 1:
            t = torch.from_numpy(stats).to(dev)
            dist.all_reduce(t)  # rate-control / quality statistics
            stats = t.cpu().numpy()
            gathered = gather_bytes_to_root(b"".join(segs), dev)  # bitstreams -> stitch rank
        prof["post"] += time.perf_counter() - t_b
        return stats, gathered

    for s in range(args.warmup):
        step(-1 - s)
    prof["encode"] = prof["post"] = 0.0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tot = None
    step_ms = []
    for s in range(args.steps):
        ts = time.perf_counter()
        stats, _ = step(s)
        step_ms.append(round(1000 * (time.perf_counter() - ts), 2))
        tot = stats if tot is None else tot + stats
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    el_t = torch.tensor([el], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
    el = float(el_t.item())
    frames = tot[0]
    npx = frames * w * h
    psnr = lambda s, n: float(10 * np.log10(255.0 ** 2 * n / s)) if s > 0 else float("inf")
    py, pu, pv = psnr(tot[2], npx), psnr(tot[3], npx / 4), psnr(tot[4], npx / 4)
    fps = frames / el
    kbps = tot[1] * 8 / (frames / 30.0) / 1000.0 / world  # per 30 fps stream
    if rank == 0:
        tm = eng.timing()
        print(json.dumps({
            "metric": METRIC,
            "value": round(fps, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000 * el / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "uint8 video / int32 integer transforms (bit-exact HEVC)",
            "data": "synthetic (seeded procedural YUV 4:2:0 source generated on GPU)",
            "config": {
                "model": f"HEVC Main CQP{args.qp} CTB32 {args.res} synthetic" + (" +SAO" if args.sao else ""),
                "global_batch": world * batch,
                "seq_len": args.gop,
                "parallelism": f"dp{world}",
                "resolution": f"{w}x{h}",
                "segments_per_gpu": batch,
                "frames_per_segment": args.gop,
                "psnr_y_db": round(py, 3),
                "psnr_yuv_db": round((6 * py + pu + pv) / 8, 3),
                "kbps_per_30fps_stream": round(kbps, 1),
                "last_step_gpu_ms": round(tm["gpu_ms"], 2),
                "last_step_engine_wall_ms": round(tm["wall_ms"], 2),
                "last_step_entropy_cpu_ms": round(tm["entropy_cpu_ms"], 2),
                "last_step_coef_mb_d2h": round(tm["coef_mb"], 2),
                "encode_s": round(prof["encode"], 3),
                "post_s": round(prof["post"], 3),
                "cpu_threads": eng.threads,
                "step_ms": step_ms,
            },
        }), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
