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
RES = {"1080p": (1920, 1080), "4k": (3840, 2160), "720p": (1280, 720), "360p": (640, 360), "tiny": (160, 96)}
SRC = {"8k": (7680, 4320), "4k": (3840, 2160), "1080p": (1920, 1080), "360p": (640, 360), "tiny": (320, 192)}
LADDER_METRIC = "HDR10 source frames/sec (whole node) through a tone-map + Lanczos + HEVC ABR ladder"
AV1_KEY_QP_OFFSET = -2.0  # 2-pass: key frame QP relative to its segment's inter frames
AV1_METRIC = "encoded frames/sec (whole node) at fixed PSNR, AV1 (CDEF in loop), 1/2/4/8 MI355X"


def _dist_setup(args):
    """One rank per GPU, always inside a live RCCL (`nccl`) process group — also at N=1, so
    the same all_reduce / all_gather code runs on the GPU whatever N is.  The rank's CPU set
    (CABAC pool) is pinned NUMA-local before the engine spawns its threads.  ``--cpu``: a
    gloo group of N CPU processes driving the golden encoders (models/cpu_engines.py) — the
    rehearsal of this file's N-rank logic on a machine without GPUs."""
    import torch
    import torch.distributed as dist

    from thinvids_amd.parallel.launch import free_port, pin_rank

    if "WORLD_SIZE" not in os.environ:  # N=1 without a launcher: a one-rank group
        os.environ.update(RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", LOCAL_WORLD_SIZE="1",
                          MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()))
    world = int(os.environ["WORLD_SIZE"])
    rank = int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    cpus = pin_rank(local, int(os.environ.get("LOCAL_WORLD_SIZE", world)))
    import datetime

    # a stuck rank fails the collectives in minutes, not at the driver's time limit
    timeout = datetime.timedelta(seconds=float(os.environ.get("TV_COLL_TIMEOUT", "240")))
    if args.cpu:
        dist.init_process_group("gloo", timeout=timeout)
        assert dist.get_world_size() == args.gpus, "live group size != --gpus"
        return dist.get_world_size(), dist.get_rank(), local, torch.device("cpu"), cpus
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("nccl", device_id=dev, timeout=timeout)
    assert dist.get_world_size() == args.gpus, "live group size != --gpus"
    return dist.get_world_size(), dist.get_rank(), local, dev, cpus


def _batch_for(args, local: int, codec: str, w: int, h: int):
    """Segments per GPU per step: --batch, else worker.encoder.auto_batch — the CU-fill
    heuristic (enough CTBs per wavefront diagonal and per motion-search launch to fill 256
    CUs; measured 1080p 8 -> 32 segments +47 %, 32 -> 48 +3 %, 4K 16 -> 24 +9 %,
    profiles/README.md) capped by this GPU's HBM budget (hipMemGetInfo).  Returns (batch,
    JSON description)."""
    from thinvids_amd.worker.encoder import EncodeSpec, auto_batch, device_budget, engine_bytes

    spec = EncodeSpec(w, h, qp=args.qp, gop=args.gop, sao=args.sao, codec=codec,
                      bframes=args.bframes if codec == "hevc" else 1, wpp=args.wpp, rqt=args.rqt, pintra=args.pintra,
                      cascade=args.cascade, rdoq=args.rdoq)
    if args.batch:
        return args.batch, {"batch": args.batch, "source": "--batch"}
    if args.cpu:
        return auto_batch(spec), {"batch": auto_batch(spec), "source": "auto (cpu rehearsal)"}
    budget = device_budget(local)
    b = auto_batch(spec, budget)
    return b, {"batch": b, "source": "auto: CU-fill heuristic capped by the HBM budget",
               "hbm_budget_gib": round(budget / 2**30, 1), "engine_plus_staging_gib": round(engine_bytes(spec, b) / 2**30, 2)}


def _sync(dev) -> None:
    import torch

    if dev.type == "cuda":
        torch.cuda.synchronize(dev)


class _CpuMeter:
    """Process CPU seconds (all threads: CABAC pool + Python) over the timed region."""

    def start(self):
        import resource

        r = resource.getrusage(resource.RUSAGE_SELF)
        self.c0, self.t0 = r.ru_utime + r.ru_stime, time.perf_counter()

    def cores(self) -> float:
        import resource

        r = resource.getrusage(resource.RUSAGE_SELF)
        return (r.ru_utime + r.ru_stime - self.c0) / max(1e-9, time.perf_counter() - self.t0)


def _per_rank(values, dev):
    """all_gather a small float vector from every rank -> list of lists (rank order)."""
    import torch
    import torch.distributed as dist

    t = torch.tensor(values, dtype=torch.float64, device=dev)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [[round(float(x), 3) for x in o.cpu()] for o in out]


class _PostQueue:
    """Per-step communication (RC/quality stats all-reduce + bitstream gather to the stitch
    rank) on one background thread, so step s's collectives overlap step s+1's encode.  Only
    this thread issues collectives between start and drain, so every rank issues them in the
    same order."""

    def __init__(self, local: int, cpu: bool = False):
        import concurrent.futures as cf

        import torch

        self.ex = cf.ThreadPoolExecutor(1, initializer=None if cpu else (lambda: torch.cuda.set_device(local)))
        self.futs = []

    def submit(self, fn, *a):
        self.futs.append(self.ex.submit(fn, *a))

    def drain(self):
        out = [f.result() for f in self.futs]
        self.futs = []
        return out

    def close(self):
        self.ex.shutdown(wait=True)


def _timed(args, step, dev, world, post, extra_ranks=None):
    """W untimed warm-up steps, then exactly K timed steps bracketed by barrier + device
    synchronise on both sides; returns (elapsed = MAX over ranks, per-step ms, post results,
    per-rank [cpu cores busy, cpus pinned])."""
    import torch
    import torch.distributed as dist

    for s in range(args.warmup):
        step(-1 - s)
    post.drain()
    dist.barrier()
    _sync(dev)
    meter = _CpuMeter()
    meter.start()
    t0 = time.perf_counter()
    step_ms = []
    for s in range(args.steps):
        ts = time.perf_counter()
        step(s)
        step_ms.append(round(1000 * (time.perf_counter() - ts), 2))
    res = post.drain()  # the last step's collectives complete inside the timed region
    dist.barrier()
    _sync(dev)
    el_t = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    cores = meter.cores()
    dist.all_reduce(el_t, op=dist.ReduceOp.MAX)
    # extra per-rank values; callables are read after the timed region (e.g. byte counters)
    ranks = _per_rank([cores] + [v() if callable(v) else v for v in (extra_ranks or [])], dev)
    return float(el_t.item()), step_ms, res, ranks


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

    world, rank, local, dev, cpus = _dist_setup(args)
    sw, sh = SRC[args.src]
    heights = [int(x) for x in args.ladder.split(",") if x.strip()]
    batch = args.batch or 24  # measured 8K ladder: b8 183, b16 360, b24 373, b32 365 source frames/s
    if args.cpu:
        from thinvids_amd.models.cpu_engines import CpuAbrLadder as AbrLadder  # noqa: F811
    lad = AbrLadder(sw, sh, heights, qp=args.qp, segments=batch, gop=args.gop, device=local,
                    threads=args.threads or None, seed=args.seed, search_range=args.range, sao=args.sao)
    post = _PostQueue(local, args.cpu)

    def prep(i: int):  # step i's source -> tone-map -> rungs into staging slot i % 2
        base = (i * world + rank) * batch
        lad.prepare_synthetic([(base + b) * args.gop for b in range(batch)], slot=i % 2)
        if dev.type == "cuda":
            torch.cuda.current_stream(dev).synchronize()

    def comm(segs):
        nbytes = sum(len(x) for r in segs for x in r)
        t = torch.tensor([batch * args.gop, nbytes], dtype=torch.float64, device=dev)
        dist.all_reduce(t)
        gathered = gather_bytes_to_root(b"".join(x for r in segs for x in r), dev)
        return np.concatenate([t.cpu().numpy(), [sum(len(x) for x in gathered) if gathered else 0]])

    # step i encodes staging slot i % 2 while this thread prepares step i + 1 into the other
    # slot (every step = one full prep + one full encode; prep(0) runs before warm-up)
    prep(0)
    counter = [0]

    def step(_s: int):
        i = counter[0]
        counter[0] += 1
        segs = lad.encode_overlapped(batch, i % 2, prepare_next=lambda: prep(i + 1))
        post.submit(comm, segs)

    el, step_ms, res, ranks = _timed(args, step, dev, world, post, [len(cpus), lad.engines[0].threads])
    tot = np.sum(res, axis=0)
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
            "data": CPU_DATA if args.cpu else "synthetic (seeded procedural HDR10 P010 source generated on GPU)",
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
                "bytes_all_reduced_mb": round(tot[1] / 1e6, 6),
                "gathered_mb_at_root": round(tot[2] / 1e6, 6),
                "last_step_gpu_ms_per_rung": [round(t["gpu_ms"], 2) for t in tm],
                "last_step_entropy_cpu_ms_per_rung": [round(t["entropy_cpu_ms"], 2) for t in tm],
                "per_rank_cpu": [{"busy_cores": r[0], "pinned_cpus": int(r[1]), "cabac_threads": int(r[2])}
                                 for r in ranks],
                "step_ms": step_ms,
            },
        }), flush=True)
    post.close()
    lad.close()
    dist.destroy_process_group()


JOB_METRIC = "end-to-end job frames/sec (add_job -> DONE, node executor, whole node)"
CPU_DATA = ("CPU REHEARSAL (--cpu: gloo ranks + golden C++ encoders at a tiny geometry) of the N-rank bench logic; "
            "not an MI355X measurement")


def job_main(args) -> None:
    """End-to-end job throughput (verdict r1 item 2): a node executor with N ranks (one per
    GPU, RCCL group) takes a transcode job from the queue — segment claims through the
    store, ingest, batched HIP encode, per-claim bitstream stream to rank 0 over RCCL, the
    streaming MP4 stitch and library publish — and the wall time from submission to DONE is
    measured.  One untimed warm-up job first (engines stay resident across jobs).

    ``--source synth`` (default): the seeded synthetic stream (.synth: generated on each
    GPU, P5).  ``--source y4m``: a raw y4m file written to local scratch BEFORE the timed
    region (GPU-generated frames, a child process), then read by the job: native parallel
    pread into pinned memory + one H2D per segment (``--job-mode direct``, every rank reads
    its own range) or the rotating-root xGMI scatter (``--job-mode scatter``); the JSON
    reports read / H2D GB/s per rank (verdict r3 item 3)."""
    import subprocess
    import tempfile
    import uuid

    from thinvids_amd.models import media
    from thinvids_amd.parallel.launch import spawn_ranks
    from thinvids_amd.store import RemoteStore, set_store
    from thinvids_amd.store.server import StoreServer

    w, h = RES[args.res]
    tmp = tempfile.mkdtemp(prefix="tvjob_", dir=os.environ.get("TV_BENCH_SCRATCH") or None)
    y4m = args.source == "y4m"
    dvd = args.source == "mpeg2"
    seg_frames = args.gop * 16
    frames = args.job_frames or (args.gop * 16 * 3 * 4 * args.gpus if y4m else args.gop * 16 * 2 * 48 * args.gpus)
    # y4m: two claims per rank, so the warm-up also runs the next-claim prefetch (its thread,
    # stream and that stream's device buffers) -- a resident executor's steady state; with one
    # claim the timed job's first prefetch allocated ~10 GB beside the first encode (+250 ms)
    warm_frames = args.gop * 16 * (6 if y4m else 1) * args.gpus
    if dvd:  # DVD-native: 720x480 kept (never upscaled), bwdif, segments of 2 GOPs
        w, h = 720, 480
        seg_frames = args.gop * 2
        frames = args.job_frames or 3000 * args.gpus
        warm_frames = 300 * args.gpus
        os.makedirs(f"{tmp}/watch/dvd", exist_ok=True)
        t0 = time.perf_counter()
        code = ("import sys, json; sys.path.insert(0, %r); from thinvids_amd.models.mpeg2 import write_dvd_title; "
                "write_dvd_title(%r, %d, seed=%d); print(json.dumps(write_dvd_title(%r, %d, seed=%d)))"
                % (ROOT, f"{tmp}/watch/dvd/warmup.mkv", warm_frames, args.seed + 7,
                   f"{tmp}/watch/dvd/timed.mkv", frames, args.seed))
        dvd_info = json.loads(subprocess.run([sys.executable, "-c", code], check=True, capture_output=True,
                                             text=True).stdout.strip().splitlines()[-1])
        frames = dvd_info["frames"]
        gen_s = time.perf_counter() - t0
    if y4m:  # source files first, in a child process (this parent never touches the GPU)
        os.makedirs(f"{tmp}/watch", exist_ok=True)
        t0 = time.perf_counter()
        code = ("import sys; sys.path.insert(0, %r); from thinvids_amd.ops.stage import write_synth_y4m; "
                "write_synth_y4m(%r, %d, %d, %d, %d); write_synth_y4m(%r, %d, %d, %d, %d)"
                % (ROOT, f"{tmp}/watch/warmup.y4m", w, h, warm_frames, args.seed + 7,
                   f"{tmp}/watch/timed.y4m", w, h, frames, args.seed))
        subprocess.run([sys.executable, "-c", code], check=True)
        gen_s = time.perf_counter() - t0
    srv = StoreServer("127.0.0.1", 0)
    srv.start_background()
    port = srv.server_address[1]
    env = {"TV_STORE": f"tcp://127.0.0.1:{port}", "PROJECT_ROOT": f"{tmp}/projects", "LIBRARY_ROOT": f"{tmp}/library",
           "WATCH_ROOT": f"{tmp}/watch", "TV_NODE_HOST": "bench-node", "HOSTNAME": "bench-node"}
    os.environ.update(env)
    os.makedirs(f"{tmp}/watch", exist_ok=True)
    store = RemoteStore("127.0.0.1", port)
    set_store(store)
    from thinvids_amd.common import save_settings
    from thinvids_amd.worker.node_executor import live_executor, submit

    save_settings({"tv_codec": args.codec, "tv_gop": str(args.gop), "tv_qp": str(args.qp), "tv_sao": "1" if args.sao else "0",
                   "tv_search_range": str(args.range), "tv_node_segment_frames": str(seg_frames),
                   "tv_node_mode": args.job_mode,
                   "tv_node_batch": str(16 if dvd else max(1, (args.batch or (48 if w * h <= 1920 * 1088 else 24)) // 16))},
                  store)
    import threading

    res = {}
    th = threading.Thread(target=lambda: res.update(rc=spawn_ranks(
        args.gpus, ["-m", "thinvids_amd.worker.node_executor", "--max-jobs", "2", "--idle-exit", "600"])), daemon=True)
    th.start()
    t0 = time.time()
    while live_executor(store) is None:
        if time.time() - t0 > 300 or not th.is_alive():
            raise SystemExit("node executor did not come up")
        time.sleep(0.1)

    def run(name, n):
        if dvd:
            spec, fname = f"{tmp}/watch/dvd/{name}.mkv", f"dvd/{name}.mkv"
        elif y4m:
            spec, fname = f"{tmp}/watch/{name}.y4m", f"{name}.y4m"
        else:
            spec, fname = f"{tmp}/watch/{name}.synth", f"{name}.synth"
            media.write_synth_spec(spec, w, h, n, 30, args.seed)
        job_id, tok = str(uuid.uuid4()), uuid.uuid4().hex
        store.hset(f"job:{job_id}", mapping={"job_id": job_id, "filename": fname, "input_path": spec,
                                             "status": "STARTING", "pipeline_run_token": tok, "target_height": str(h)})
        ts = time.perf_counter()
        submit(job_id, tok, "bench-node")
        while store.hget(f"job:{job_id}", "status") not in ("DONE", "FAILED"):
            time.sleep(0.02)
        el = time.perf_counter() - ts
        job = store.hgetall(f"job:{job_id}")
        if job["status"] != "DONE":
            raise SystemExit(f"job failed: {job.get('error')}")
        return el, job

    run("warmup", warm_frames)
    el, job = run("timed", frames)
    th.join(120)
    ingest = json.loads(job.get("ingest_json") or "[]")
    gb = lambda b, s: round(b / 1e9 / s, 2) if s else None  # noqa: E731
    cfg_src = {}
    if dvd:
        cfg_src = {"source_file": f"DVD title: MPEG-2 MP@ML 720x480 interlaced (tff) in Matroska V_MPEG2, {frames} frames, "
                                  f"{dvd_info['kbps']} kbps ({dvd_info['unique']} unique frames repeated; written before the "
                                  "timed region); decoded on host threads, bwdif (k_bwdif) + HEVC on the GPU",
                   "source_gen_s": round(gen_s, 2), "job_mode": args.job_mode,
                   "decode_threads_per_rank": os.environ.get("TV_DECODE_THREADS") or "auto (min(16, cpus))"}
    if y4m:
        fb = w * h * 3 // 2
        cfg_src = {"source_file": f"y4m {w}x{h} 8-bit 4:2:0, {frames} frames, {round(frames * (fb + 6) / 1e9, 2)} GB "
                                  "(written before the timed region; page-cache resident when read)",
                   "source_gen_s": round(gen_s, 2), "job_mode": args.job_mode,
                   "raw_gb_per_s_consumed": round(frames * fb / 1e9 / el, 2),
                   "per_rank_ingest": [{"reads": p.get("reads"), "read_gb": round((p.get("read_bytes") or 0) / 1e9, 2),
                                        "ingest_gb_per_s": gb(p.get("read_bytes") or 0, p.get("ingest_s")),
                                        "ingest_s": round(p.get("ingest_s") or 0, 3),
                                        "read_threads": p.get("read_threads"),
                                        "per_thread_read_gb_per_s": gb((p.get("read_bytes") or 0) / max(1, p.get("read_threads") or 1),
                                                                       p.get("read_thread_s") and p["read_thread_s"] / max(1, p.get("read_threads") or 1))}
                                       for p in ingest]}
    print(json.dumps({
        "metric": JOB_METRIC, "value": round(frames / el, 2), "unit": "frames/s", "n_gpus": args.gpus,
        "steps": 1, "warmup": 1, "ms_per_step": round(1000 * el, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "uint8 video / int32 integer transforms (bit-exact "
        + ("AV1 subset)" if args.codec == "av1" else "HEVC)"),
        "data": ("synthetic frames in a raw y4m FILE read by the job (native pread threads -> pinned ring -> overlapped H2D DMA)" if y4m
                 else "synthetic interlaced frames in an MPEG-2 DVD title read and decoded by the job" if dvd
                 else "synthetic (seeded procedural YUV 4:2:0 .synth source generated on each GPU)"),
        "config": {"model": (f"AV1 subset (tv) q-index for QP{args.qp} {args.res} synthetic" if args.codec == "av1" else
                             f"HEVC Main CQP{args.qp} CTB32 {'480p DVD' if dvd else args.res} synthetic"
                             + (" +SAO" if args.sao else "")),
                   "codec": job.get("dest_codec"), "source": args.source, **cfg_src,
                   "job_frames": frames, "resolution": f"{w}x{h}", "parallelism": f"dp{args.gpus} node executor",
                   "job_wall_s": round(el, 3), "job_fps_reported": float(job.get("job_fps") or 0),
                   "encode_fps_reported": float(job.get("encode_fps") or 0), "psnr_y_db": float(job.get("psnr_y") or 0),
                   "kbps": float(job.get("bitrate_kbps") or 0), "segments": int(job.get("parts_total") or 0),
                   "output_bytes": int(job.get("dest_file_size") or 0),
                   "stitch": json.loads(job.get("stitch_json") or "{}"),
                   "encode_elapsed_s": float(job.get("encode_elapsed") or 0), "run_job_s": float(job.get("job_seconds") or 0),
                   "rank0_spans_ms": {k: v for k, v in json.loads(job.get("trace_json") or "{}").items()}},
    }), flush=True)
    srv.shutdown()
    import shutil

    shutil.rmtree(tmp, ignore_errors=True)


def av1_main(args) -> None:
    """BASELINE config #4 (AV1 with in-loop CDEF on the GPU): each rank encodes `batch`
    GOP-aligned segments x `gop` synthetic frames per step on the AV1 engine
    (thinvids_amd/models/av1_engine.py), the OBU writer pool entropy-codes them behind the
    GPU, and the bitstreams are gathered to rank 0 over RCCL with the quality statistics
    all-reduced — the same data plane as the HEVC bench."""
    import ctypes as C

    import numpy as np
    import torch
    import torch.distributed as dist

    world, rank, local, dev, cpus = _dist_setup(args)

    from thinvids_amd.models import av1 as av1m
    from thinvids_amd.models.av1_engine import Av1GpuEngine
    from thinvids_amd.ops import stage
    from thinvids_amd.parallel.comm import gather_bytes_to_root

    w, h = RES[args.res]
    q = args.qindex or av1m.qindex_for_hevc_qp(args.qp)
    batch, sizing = _batch_for(args, local, "av1", w, h)
    if args.cpu:
        from thinvids_amd.models.cpu_engines import CpuAv1Engine as Av1GpuEngine  # noqa: F811
    eng = Av1GpuEngine(w, h, batch=batch, qindex=q, device=local, threads=args.threads or None, cascade=args.cascade,
                       **({"seed": args.seed} if args.cpu else {}))
    post = _PostQueue(local, args.cpu)
    W, H = eng.W, eng.H
    lib = stage._lib()

    def comm(gfut):
        g = gfut.result()  # decisions on the host (copy stream, behind the next GOP's kernels)
        sse = g.sse.sum(axis=(0, 1)).astype(np.float64)
        segs = [b"".join(f.result()) for f in eng.submit_entropy(g)]
        stats = torch.tensor([batch * args.gop, sum(len(x) for x in segs), *sse], dtype=torch.float64, device=dev)
        dist.all_reduce(stats)
        gathered = gather_bytes_to_root(b"".join(segs), dev)
        return stats.cpu().numpy(), (sum(len(x) for x in gathered) if gathered else 0)

    pass1_bits = []
    gathered_mb = lambda res: round(sum(r[1] for r in res) / 1e6, 6)  # noqa: E731
    from thinvids_amd.models.ratecontrol import BatchRateController

    ctl = BatchRateController()
    nominal = args.kbps * 1000.0 * (world * batch * args.gop) / 30.0  # bits per step, whole node
    predicted = {}

    def comm_rc(i, gfut):
        out = comm(gfut)
        if args.kbps > 0:  # the post thread: every rank records the same all-reduced totals
            want, u = predicted.pop(i)
            ctl.record(nominal, want, u, 8.0 * float(out[0][1]))
        return out

    def plan_pass2(i, g1fut):
        """Config #4's 2-pass, post thread (the only thread issuing collectives): pass-1
        per-frame bits of every rank's segments all-reduced over RCCL -> one global
        per-frame plan for this step's share of the target, corrected by the finished steps'
        bias and debt (ratecontrol.BatchRateController) -> this rank's per-frame q-index
        maps for pass 2."""
        from thinvids_amd.models.ratecontrol import AV1_SLOPE, frame_sizes, plan_frame_qps, round_qps

        g1 = g1fut.result()
        seg1 = [b"".join(f.result()) for f in eng.submit_entropy(g1)]
        flat = torch.zeros(world * batch * args.gop, dtype=torch.float64, device=dev)
        mine = np.concatenate([8.0 * np.asarray(frame_sizes(x), np.float64) for x in seg1])
        flat[rank * batch * args.gop:(rank + 1) * batch * args.gop] = torch.from_numpy(mine).to(dev)
        dist.all_reduce(flat)  # RC statistics all-reduce over the node
        allb = flat.cpu().numpy().reshape(world * batch, args.gop)
        ask, want, u = ctl.request(nominal)
        plan, _ = plan_frame_qps(list(allb), args.qp, ask, key_offset=AV1_KEY_QP_OFFSET, slope=AV1_SLOPE)
        qall = np.stack([round_qps(p, u) for p in plan])
        predicted[i] = (want, u)
        pass1_bits.append(float(mine.sum()))
        return np.array([[av1m.qindex_for_hevc_qp(int(v)) for v in qall[rank * batch + b]]
                         for b in range(batch)], np.int32).T

    def loader(i: int):
        base = (i * world + rank) * batch
        if args.cpu:  # the CPU engine generates its own frames from the segment starts
            return [(base + b) * args.gop for b in range(batch)]

        def load(t, planes):
            st = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
            src = stage.synth_frames(args.seed, w, h, [(base + b) * args.gop + t for b in range(batch)], dev)
            for c, dst in enumerate(planes):
                off, pw, ph, stride, fs = src.planes[c]
                cw, chh = (W, H) if c == 0 else (W // 2, H // 2)
                stage._ok(lib.tv_pad_batch(C.c_void_p(src.ptr(c)), pw, ph, stride, fs, C.c_void_p(dst.data_ptr()),
                                           cw, chh, cw, cw * chh, batch, st))
        return load

    plans = {}
    counter = [0]

    def pass1(i: int):
        """Pass 1 of step i on the GPU, a fast first pass (x264-style): no restoration
        search, whose ~28 % of the GPU step only fine-tunes the reconstruction; the measured
        QP-offset response absorbs the small pass-1 / pass-2 difference.  Its plan queues on the
        post thread."""
        eng.lr_enabled = False
        try:
            g1 = eng.encode_gop(args.gop, loader(i), async_host=True)
        finally:
            eng.lr_enabled = True
        plans[i] = post.ex.submit(plan_pass2, i, g1)

    def step(_s: int):
        i = counter[0]
        counter[0] += 1
        if args.kbps > 0:
            # software pipeline: step i runs pass 1 of step i + 1 on the GPU, then pass 2 of
            # step i, whose plan (pass-1 entropy + all-reduce, post thread) was computed
            # behind the previous step's GPU work -- the GPU never waits for the host plan
            if i == 0:
                pass1(0)
            pass1(i + 1)
            qm = plans.pop(i).result()
            post.submit(comm_rc, i, eng.encode_gop(args.gop, loader(i), qmap=qm, async_host=True))
        else:
            post.submit(comm, eng.encode_gop(args.gop, loader(i), async_host=True))

    from thinvids_amd.parallel.comm import COMM_STATS

    c0 = dict(COMM_STATS)
    el, step_ms, res, ranks = _timed(args, step, dev, world, post,
                                     [len(cpus), eng.pool._max_workers,
                                      lambda: COMM_STATS["p2p_sent_bytes"] - c0["p2p_sent_bytes"],
                                      lambda: COMM_STATS["p2p_recv_bytes"] - c0["p2p_recv_bytes"]])
    for f in plans.values():  # the look-ahead pass 1 of the step after the last one
        f.result()
    tot = np.sum([r[0] for r in res], axis=0)
    frames = tot[0]
    npx = frames * w * h
    psnr = lambda s, n: float(10 * np.log10(255.0 ** 2 * n / s)) if s > 0 else float("inf")
    py, pu, pv = psnr(tot[2], npx), psnr(tot[3], npx / 4), psnr(tot[4], npx / 4)
    if rank == 0:
        print(json.dumps({
            "metric": AV1_METRIC,
            "value": round(frames / el, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000 * el / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "uint8 video / int32 integer transforms (bit-exact AV1 subset)",
            "data": CPU_DATA if args.cpu else f"synthetic ({args.content} seeded procedural YUV 4:2:0 source generated on GPU)",
            "config": {
                "model": f"AV1 subset (tv) qindex {q} 16x16 blocks, refined + unified MV field, 32/64 merged skip blocks, "
                         f"+deblock +CDEF +LR {args.res} synthetic"
                + (f" 2-pass {args.kbps:g} kbps" if args.kbps > 0 else ""),
                "rate_control": (f"2-pass: pass-1 per-frame bits all-reduced, per-frame q-index plan, target "
                                 f"{args.kbps:g} kbps per 30 fps stream, fast first pass (no LR search), batch "
                                 "feedback (measured QP offset response + bounded debt)" if args.kbps > 0 else "constant q-index"),
                "kbps_error_pct": round(100 * (tot[1] * 8 / (frames / 30.0) / 1000.0 / args.kbps - 1), 2)
                if args.kbps > 0 else None,
                "rc_steps_actual_wanted_offset": ctl.log if args.kbps > 0 else None,
                "global_batch": world * batch,
                "seq_len": args.gop,
                "parallelism": f"dp{world}",
                "comm": f"{dist.get_backend()} world={world}: stats all_reduce + bitstream gather to rank 0 (overlapped)",
                "per_rank_comm": [{"transport": "rccl p2p" if dist.get_backend() == "nccl" else dist.get_backend(),
                                   "p2p_sent_mb_incl_warmup": round(r[3] / 1e6, 3), "p2p_recv_mb_incl_warmup": round(r[4] / 1e6, 3)}
                                  for r in ranks],
                "resolution": f"{w}x{h}",
                "segments_per_gpu": batch,
                "batch_sizing": sizing,
                "frames_per_segment": args.gop,
                "psnr_y_db": round(py, 3),
                "psnr_yuv_db": round((6 * py + pu + pv) / 8, 3),
                "kbps_per_30fps_stream": round(tot[1] * 8 / (frames / 30.0) / 1000.0, 1),
                "pass1_kbps_rank0": round(sum(pass1_bits[-args.steps:]) / (batch * args.gop * args.steps / 30.0)
                                          / 1000.0, 1) if pass1_bits else None,
                "gathered_mb_at_root": gathered_mb(res),
                "bytes_all_reduced_mb": round(tot[1] / 1e6, 6),
                "per_rank_cpu": [{"busy_cores": r[0], "pinned_cpus": int(r[1]), "writer_threads": int(r[2])}
                                 for r in ranks],
                "step_ms": step_ms,
            },
        }), flush=True)
    post.close()
    eng.close()
    dist.destroy_process_group()


# the benchmarked configuration is the shipped worker configuration (common/settings.py)
from thinvids_amd.common.settings import DEFAULT_SETTINGS as _DEFAULTS  # noqa: E402

_WORKER_GOP = int(_DEFAULTS.get("tv_gop", 64))
_WORKER_SAO = str(_DEFAULTS.get("tv_sao", "1")) == "1"
_WORKER_BFRAMES = int(_DEFAULTS.get("tv_bframes", 1))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--res", default=None, choices=sorted(RES), help="default 1080p (tiny with --cpu)")
    ap.add_argument("--batch", type=int, default=0, help="segments per GPU per step (0 = auto)")
    ap.add_argument("--gop", type=int, default=_WORKER_GOP,
                    help="frames per GOP-aligned segment (default: the worker's shipped tv_gop)")
    ap.add_argument("--qp", type=int, default=27)
    ap.add_argument("--sao", dest="sao", action="store_true", default=_WORKER_SAO,
                    help="enable SAO (in-loop sample adaptive offset; default: the worker's shipped tv_sao)")
    ap.add_argument("--no-sao", dest="sao", action="store_false", help="disable SAO")
    ap.add_argument("--bframes", type=int, default=_WORKER_BFRAMES,
                    help="hierarchical-B mini-GOP size (1 = I P P P; default: the worker's tv_bframes)")
    ap.add_argument("--range", type=int, default=64, help="motion search range (full-res pels, multiple of 16)")
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--content", choices=("smooth", "textured"), default="smooth",
                    help="synthetic source: smooth value noise (default) or the textured variant (fine detail, "
                         "per-pixel temporal grain, faster motion; tv/synth.h)")
    ap.add_argument("--ladder", default="", help="ABR mode (config #5): rung heights, e.g. 2160,1440,1080,720,480")
    ap.add_argument("--src", default=None, choices=sorted(SRC), help="ABR mode: HDR10 source resolution (default 8k; tiny with --cpu)")
    ap.add_argument("--job", action="store_true", help="end-to-end job mode (node executor, add -> DONE)")
    ap.add_argument("--job-frames", type=int, default=0)
    ap.add_argument("--source", choices=("synth", "y4m", "mpeg2"), default="synth",
                    help="job mode: synthetic .synth source (generated on each GPU), a raw y4m file read by the job, "
                         "or a DVD title (720x480 interlaced MPEG-2 in Matroska: decode + bwdif + HEVC)")
    ap.add_argument("--job-mode", choices=("direct", "scatter"), default="direct",
                    help="job mode: every rank reads its own range (direct) or rotating-root xGMI scatter")
    ap.add_argument("--codec", default="hevc", choices=["hevc", "av1"], help="av1: BASELINE config #4 engine")
    ap.add_argument("--qindex", type=int, default=0, help="AV1 q-index (0 = matched to --qp)")
    ap.add_argument("--kbps", type=float, default=0.0, help="2-pass rate control to this kbps per 30 fps stream")
    ap.add_argument("--no-4k", action="store_true", help="skip the 4K pass of the default 1080p run")
    ap.add_argument("--no-wpp", dest="wpp", action="store_false",
                    help="one CABAC substream per slice (coded on the host) instead of WPP rows coded on the GPU")
    ap.add_argument("--no-rqt", dest="rqt", action="store_false", help="HEVC: no residual quadtree")
    ap.add_argument("--no-cascade", dest="cascade", action="store_false",
                    help="HEVC: flat QP (no constant-QP I P P P QP cascade)")
    ap.add_argument("--no-pintra", dest="pintra", action="store_false", help="HEVC: no intra CUs in P pictures")
    ap.add_argument("--no-rdoq", dest="rdoq", action="store_false", help="HEVC: no RDOQ-lite coefficient-group trimming")
    ap.add_argument("--entropy", choices=("gpu", "host", "auto"), default=None,
                    help="where WPP substreams are CABAC-coded (default auto: the host writer with >= 12 CPUs "
                         "per rank, else the GPU; TV_ENTROPY); same bytes either way")
    ap.add_argument("--cpu", action="store_true",
                    help="rehearsal on CPU: gloo ranks + the golden encoders (models/cpu_engines.py), tiny geometry")
    args = ap.parse_args()
    if args.res is None:
        args.res = "tiny" if args.cpu else "1080p"
    if args.src is None:
        args.src = "tiny" if args.cpu else "8k"
    if args.cpu and args.job:
        raise SystemExit("--cpu rehearses the step benches; the job bench runs the node executor (tests cover it on CPU)")
    if args.cpu and args.range == 64:
        args.range = 16
    if args.content == "textured":  # tv/synth.h kSynthTextured
        args.seed = (args.seed | 0x80000000) & 0xFFFFFFFF
    if args.job:
        return job_main(args)
    from thinvids_amd.parallel.launch import launched_by_torchrun, spawn_ranks

    if args.gpus > 1 and not launched_by_torchrun():
        # self-launch: N ranks (one per GPU) started before this parent touches the GPU
        sys.exit(spawn_ranks(args.gpus, [os.path.abspath(__file__), *sys.argv[1:]]))
    if args.ladder:
        return ladder_main(args)
    if args.codec == "av1":
        return av1_main(args)

    import torch.distributed as dist

    world, rank, local, dev, cpus = _dist_setup(args)
    out = hevc_pass(args, world, rank, local, dev, cpus)
    if _with_4k(args):
        # the headline metric names 1080p AND 4K: the same process then times a 4K pass
        # (same K / W, same shipped configuration) so the driver's clock covers both
        import copy

        a4 = copy.copy(args)
        a4.res, a4.batch = "4k", 0
        o4 = hevc_pass(a4, world, rank, local, dev, cpus)
        if rank == 0:
            c4 = o4["config"]
            out["config"].update(fps_4k=o4["value"], psnr_y_4k=c4["psnr_y_db"], kbps_4k=c4["kbps_per_30fps_stream"],
                                 ms_per_step_4k=o4["ms_per_step"], segments_per_gpu_4k=c4["segments_per_gpu"],
                                 step_ms_4k=c4["step_ms"])
    if rank == 0:
        print(json.dumps(out), flush=True)
    dist.destroy_process_group()


def _with_4k(args) -> bool:
    """The default driver run (1080p, shipped config, constant QP) also reports 4K."""
    return (not args.no_4k and not args.cpu and args.res == "1080p" and args.kbps <= 0
            and args.bframes == _WORKER_BFRAMES and args.content == "smooth")


def hevc_pass(args, world, rank, local, dev, cpus):
    """One timed HEVC pass (W warm-up + K timed steps) at args.res; returns the JSON record
    on rank 0 (None elsewhere)."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from thinvids_amd.models.gpu_engine import GpuEngine
    from thinvids_amd.parallel.comm import gather_bytes_to_root

    w, h = RES[args.res]
    # segments per GPU: enough CTBs per wavefront diagonal of the I-frame recon and per
    # motion-search launch to fill 256 CUs (measured: 1080p 8 -> 32 segments = +47 %); the
    # engine splits them into two stream groups one frame apart (measured on MI355X:
    # 1080p 32 -> 48 segments +3 %, 4K 16 -> 24 segments +9 %; profiles/README.md)
    batch, sizing = _batch_for(args, local, "hevc", w, h)
    if args.cpu:
        from thinvids_amd.models.cpu_engines import CpuHevcEngine as GpuEngine  # noqa: F811
    tools = dict(wpp=args.wpp, rqt=args.rqt, pintra=args.pintra, entropy=args.entropy, cascade=args.cascade, rdoq=args.rdoq)
    eng = GpuEngine(width=w, height=h, qp=args.qp, batch=batch, gop=args.gop, search_range=args.range, sao=args.sao,
                    seed=args.seed, threads=args.threads or None, device=local, bframes=args.bframes, **tools)
    post = _PostQueue(local, args.cpu)
    # 2-pass: a second engine runs the fast first pass (SAO off: its statistics, decision and
    # filter are ~15 % of the GPU step and only fine-tune the reconstruction; the measured
    # QP-offset response absorbs the pass-1 / pass-2 difference) one step ahead, on its own
    # thread and HIP streams, concurrently with pass 2 of the current step
    eng1 = pre = None
    if args.kbps > 0:
        import concurrent.futures as cf

        eng1 = GpuEngine(width=w, height=h, qp=args.qp, batch=batch, gop=args.gop, search_range=args.range, sao=False,
                         seed=args.seed, threads=args.threads or None, device=local, bframes=args.bframes, **tools)
        pre = cf.ThreadPoolExecutor(1, initializer=None if args.cpu else (lambda: torch.cuda.set_device(local)))

    def comm(segs, sse):
        # rate-control / quality statistics all-reduce + bitstreams -> stitch rank (rank 0)
        stats = torch.tensor([batch * args.gop, sum(len(x) for x in segs), *sse], dtype=torch.float64, device=dev)
        dist.all_reduce(stats)
        gathered = gather_bytes_to_root(b"".join(segs), dev)
        return stats.cpu().numpy(), (sum(len(x) for x in gathered) if gathered else 0)

    from thinvids_amd.models.ratecontrol import (QCOMP, QCOMP_BFRAMES, BatchRateController, frame_sizes,
                                                 plan_frame_qps, round_qps)

    ctl = BatchRateController()
    nominal = args.kbps * 1000.0 * (world * batch * args.gop) / 30.0  # bits per step, whole node
    predicted = {}
    pass1_bits = []

    def plan_pass2(i, segs1):
        """2-pass, post thread (the only thread issuing collectives): pass-1 per-frame bits
        of every rank all-reduced over RCCL -> one global per-frame QP plan for this step's
        share of the target (ratecontrol.plan_frame_qps), corrected by the finished steps'
        bias and debt (BatchRateController) -> this rank's [batch, gop] QP map."""
        flat = torch.zeros(world * batch * args.gop, dtype=torch.float64, device=dev)
        mine = np.concatenate([8.0 * np.asarray(frame_sizes(x), np.float64) for x in segs1])
        flat[rank * batch * args.gop:(rank + 1) * batch * args.gop] = torch.from_numpy(mine).to(dev)
        dist.all_reduce(flat)
        ask, want, u = ctl.request(nominal)
        allb = flat.cpu().numpy().reshape(world * batch, args.gop)
        plan, _ = plan_frame_qps(list(allb), args.qp, ask, qcomp=QCOMP_BFRAMES if args.bframes > 1 else QCOMP)
        qall = np.stack([round_qps(p, u) for p in plan])
        predicted[i] = (want, u)
        pass1_bits.append(float(mine.sum()))
        return qall[rank * batch:(rank + 1) * batch]

    def comm_rc(i, segs, sse):
        out = comm(segs, sse)
        want, u = predicted.pop(i)
        ctl.record(nominal, want, u, 8.0 * float(out[0][1]))
        return out

    counter = [0]
    first = {}

    def starts_of(s: int):
        base = (s * world + rank) * batch
        return [(base + b) * args.gop for b in range(batch)]

    def step(s: int):
        i = counter[0]
        counter[0] += 1
        if args.kbps > 0:
            # pass 1 of step i + 1 (pre thread, eng1) overlaps the plan and pass 2 of step i;
            # every collective is queued on the post thread from this thread, in step order
            if i == 0:
                first[0] = pre.submit(eng1.encode_synthetic, starts_of(0))
            first[i + 1] = pre.submit(eng1.encode_synthetic, starts_of(i + 1))
            qm = post.ex.submit(plan_pass2, i, first.pop(i).result()).result()
            segs = eng.encode_synthetic(starts_of(i), qp=qm)
            post.submit(comm_rc, i, segs, np.array([eng.sse(b) for b in range(batch)]).sum(0))
            return
        segs = eng.encode_synthetic(starts_of(s))
        post.submit(comm, segs, np.array([eng.sse(b) for b in range(batch)]).sum(0))

    from thinvids_amd.parallel.comm import COMM_STATS

    c0 = dict(COMM_STATS)
    el, step_ms, res, ranks = _timed(args, step, dev, world, post,
                                     [len(cpus), eng.threads, lambda: COMM_STATS["p2p_sent_bytes"] - c0["p2p_sent_bytes"],
                                      lambda: COMM_STATS["p2p_recv_bytes"] - c0["p2p_recv_bytes"]])
    for f in first.values():  # the look-ahead pass 1 of the step after the last one
        f.result()
    tot = np.sum([r[0] for r in res], axis=0)
    gathered_bytes = sum(r[1] for r in res)
    frames = tot[0]
    npx = frames * w * h
    psnr = lambda s, n: float(10 * np.log10(255.0 ** 2 * n / s)) if s > 0 else float("inf")
    py, pu, pv = psnr(tot[2], npx), psnr(tot[3], npx / 4), psnr(tot[4], npx / 4)
    fps = frames / el
    kbps = tot[1] * 8 / (frames / 30.0) / 1000.0  # per 30 fps stream
    rec = None
    if rank == 0:
        tm = eng.timing()
        rec = {
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
            "data": CPU_DATA if args.cpu else f"synthetic ({args.content} seeded procedural YUV 4:2:0 source generated on GPU)",
            "config": {
                "model": f"HEVC Main CQP{args.qp} CTB32 {args.res} synthetic" + (" +SAO" if args.sao else "")
                + (f" hier-B{args.bframes}" if args.bframes > 1 else "")
                + (f" 2-pass {args.kbps:g} kbps" if args.kbps > 0 else ""),
                "bframes": args.bframes,
                "rate_control": (f"2-pass: pass-1 per-frame bits all-reduced, per-frame QP plan, target {args.kbps:g} "
                                 "kbps per 30 fps stream, fast first pass (SAO off) one step ahead on a second engine, batch feedback "
                                 "(measured QP offset response + bounded debt)"
                                 if args.kbps > 0 else f"CQP {args.qp}"),
                "kbps_error_pct": round(100 * (kbps / args.kbps - 1), 2) if args.kbps > 0 else None,
                "rc_steps_actual_wanted_offset": ctl.log if args.kbps > 0 else None,
                "pass1_kbps_rank0": round(sum(pass1_bits[-args.steps:]) / (batch * args.gop * args.steps / 30.0) / 1000.0, 1)
                if pass1_bits else None,
                "global_batch": world * batch,
                "seq_len": args.gop,
                "parallelism": f"dp{world}",
                "comm": f"{dist.get_backend()} world={world}: stats all_reduce + bitstream gather to rank 0 (overlapped)",
                "per_rank_comm": [{"transport": "rccl p2p" if dist.get_backend() == "nccl" else dist.get_backend(),
                                   "p2p_sent_mb_incl_warmup": round(r[3] / 1e6, 3), "p2p_recv_mb_incl_warmup": round(r[4] / 1e6, 3)}
                                  for r in ranks],
                "resolution": f"{w}x{h}",
                "segments_per_gpu": batch,
                "batch_sizing": dict(sizing, **({"engine_hbm_gib": round(eng.footprint()["dev"] / 2**30, 2)}
                                               if hasattr(eng, "footprint") else {})),
                "frames_per_segment": args.gop,
                "psnr_y_db": round(py, 3),
                "psnr_yuv_db": round((6 * py + pu + pv) / 8, 3),
                "kbps_per_30fps_stream": round(kbps, 1),
                "gathered_mb_at_root": round(gathered_bytes / 1e6, 6),
                "bytes_all_reduced_mb": round(tot[1] / 1e6, 6),
                "last_step_gpu_ms": round(tm["gpu_ms"], 2),
                "last_step_engine_wall_ms": round(tm["wall_ms"], 2),
                "last_step_entropy_cpu_ms": round(tm["entropy_cpu_ms"], 2),
                "last_step_coef_mb_d2h": round(tm["coef_mb"], 2),
                "entropy": (dict(eng.entropy_stats(), wpp=args.wpp, where=getattr(eng, "entropy", "host"))
                            if hasattr(eng, "entropy_stats") else {"wpp": args.wpp, "where": "cpu rehearsal"}),
                "coding_tools": {"wpp": args.wpp, "rqt": args.rqt, "pintra": args.pintra, "cascade": args.cascade, "rdoq": args.rdoq},
                "per_rank_cpu": [{"busy_cores": r[0], "pinned_cpus": int(r[1]), "cabac_threads": int(r[2])}
                                 for r in ranks],
                "step_ms": step_ms,
            },
        }
    post.close()
    if eng1 is not None:
        pre.shutdown()
        eng1.close()
    eng.close()
    return rec



if __name__ == "__main__":
    main()
