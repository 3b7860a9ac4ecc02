"""Node executor: the job queue's SPMD data plane on one MI355X node.

The reference moves every segment between hosts over HTTP (GET part from the master,
PUT result to the stitcher — reference worker/tasks.py:1497-1525, :1655-1674) and runs one
encode slot per thin client.  On an 8-GPU node the same ``transcode`` job is executed by
one long-lived rank per GPU instead:

    manager  --add_job/scheduler-->  transcode (pipeline queue)
                                        |  node executor alive on this node?
                                        v  yes: RPUSH node:jobs:<host>
    rank 0 BLPOPs the job, broadcasts it to every rank (gloo object broadcast)
    all ranks: parallel.node_job.run_job
        - dynamic segment claim (Huey pull model) from the rendezvous store
        - sources read once per segment (or generated on the GPU), staged on the device
        - RC statistics all-reduced over RCCL (2-pass), per-job SSE all-reduced
        - bitstreams gathered to rank 0 over RCCL (xGMI), muxed into one faststart MP4
    rank 0 publishes the output to the library and the job hash (dest_*, per-job frames/s,
    PSNR, bitrate) and marks it DONE

Engines stay resident across jobs (one EngineCache per rank), so a job pays no process
start-up or HBM allocation.  Progress, heartbeats and cooperative halt go through the same
job-hash fields and keys as the split/encode/stitch path.

    python -m thinvids_amd.worker.node_executor --gpus 8        (self-launches 8 ranks)

The launching process is a :class:`parallel.elastic.Supervisor`: when a rank dies or stops
making progress mid-job, it kills the rank group (communicator abort), quarantines that
GPU, requeues the job at the front of the node queue (it resumes from its per-segment
checkpoints under ``<job dir>/ckpt``) and restarts on the remaining GPUs.
"""
from __future__ import annotations

import argparse
import json
import os
import shutil
import sys
import threading
import time
import traceback

from ..common import Status, emit_activity, get_logging
from ..store import get_store, hmax
from .helpers import (effective_target_height, elapsed_ms, ensure_dirs, final_output_path, is_job_halted,
                      job_base_dir, job_heartbeat, job_key, job_title, now, reset_job_run_state,
                      task_token_is_current)

ACTIVE_JOBS_KEY = "pipeline:active_jobs"
EXECUTORS_KEY = "node:executors"
ALIVE_TTL = 15


def queue_key(host: str) -> str:
    return f"node:jobs:{host}"


def alive_key(host: str) -> str:
    return f"node:executor:{host}"


def live_executor(store=None, prefer: str | None = None) -> str | None:
    """Host of a live node executor (the local one first), or None."""
    st = store or get_store()
    hosts = sorted(st.smembers(EXECUTORS_KEY) or [])
    if prefer in hosts:
        hosts.remove(prefer)
        hosts.insert(0, prefer)
    for h in hosts:
        if st.get(alive_key(h)):
            return h
    return None


def submit(job_id: str, run_token: str | None, host: str, store=None) -> None:
    (store or get_store()).rpush(queue_key(host), json.dumps({"job_id": job_id, "run_token": run_token}))


class _StoreHooks:
    """node_job.JobHooks bound to the job hash (every rank reports its own segments) and to
    the rank heartbeat (per-segment progress, which the supervisor's stall detection reads)."""

    def __init__(self, job_id: str, total: int, stage_t0: float, beat=None):
        self.job_id, self.total, self.t0, self.beat = job_id, total, stage_t0, beat
        self._halt_checked, self._halted = 0.0, False
        self.pass_idx = 0

    def new_pass(self, index: int) -> None:
        """Pass `index` starts: readers switch to its counters (``rc_pass``, see
        common.pass_field) and the progress bar restarts."""
        self.pass_idx = index
        if index:
            get_store().hset(job_key(self.job_id), mapping={"rc_pass": index, "encode_progress": 0})

    def segment_done(self, frames: int) -> None:
        """Every rank increments its segments into the current pass's own counters (pass 0:
        parts_done / completed_chunks / encoded_frames; pass k: the ``_p<k>`` fields) in one
        atomic pipeline -- counters are only ever incremented, never mirrored by a
        read-modify-write, so concurrent ranks cannot move them backwards."""
        if self.beat is not None:
            self.beat.progress("segment")
        st = get_store()
        k = job_key(self.job_id)
        sfx = f"_p{self.pass_idx}" if self.pass_idx else ""
        p = st.pipeline()
        p.hincrby(k, "completed_chunks" + sfx, 1)
        p.hincrby(k, "parts_done" + sfx, 1)
        p.hincrby(k, "encoded_frames" + sfx, int(frames))
        res = p.execute()
        done = int(res[1])
        prog = int(done * 100 / max(1, self.total))
        hmax(st, k, "encode_progress", prog)  # atomic max: ranks never move it backwards
        hmax(st, k, "encode_elapsed", int(now() - self.t0))
        job_heartbeat(self.job_id, "encode", note=f"{done}/{self.total} segments")

    def halted(self) -> bool:
        t = time.monotonic()
        if t - self._halt_checked > 0.5:
            self._halt_checked = t
            self._halted = is_job_halted(self.job_id)
        return self._halted


def _job_params(job: dict) -> dict:
    """Encode parameters of a job (global settings + per-job overrides)."""
    from ..common import as_bool, as_float, as_int, get_settings
    from .tasks import encode_spec_for_job

    s = get_settings()
    spec = encode_spec_for_job(job, s)
    th, deint = effective_target_height(job)
    ladder = [int(x) for x in str(job.get("ladder") or s.get("tv_ladder") or "").split(",") if x.strip()]
    rc = str(job.get("rc_mode") or s.get("tv_rc") or "cqp").lower()
    kbps = as_float(job.get("bitrate_kbps") or s.get("tv_bitrate_kbps"), 0.0) if rc in ("2pass", "abr") else 0.0
    crf = as_int(job.get("crf") or s.get("tv_crf"), 27) if rc == "crf" else 0
    vbv = ([as_float(job.get("vbv_maxrate_kbps") or s.get("tv_vbv_maxrate_kbps"), 0.0),
            as_float(job.get("vbv_bufsize_kbit") or s.get("tv_vbv_bufsize_kbit"), 0.0)] if rc == "abr" else [0.0, 0.0])
    return {"height": th, "qp": spec.qp, "gop": spec.gop, "search_range": spec.search_range, "deblock": spec.deblock,
            "sao": spec.sao, "software": spec.software, "ladder": ladder or None, "bitrate_kbps": kbps,
            "segment_frames": max(spec.gop, as_int(s.get("tv_node_segment_frames"), 256)),
            "mode": str(s.get("tv_node_mode") or "direct"), "batch_segments": as_int(s.get("tv_node_batch"), 8),
            "settings_ok": as_bool(s.get("tv_node_executor"), True), "crf": crf, "rc": rc, "vbv": vbv,
            "scenecut": spec.scenecut, "codec": spec.codec, "qindex": spec.qindex, "bframes": spec.hevc_bframes(),
            "deinterlace": deint}


class CommFailure(RuntimeError):
    """The rank group's communicator failed: the supervisor re-initialises it."""


def execute(job_id: str, run_token: str | None, rank: int, world: int, cache, log, beat=None) -> None:
    """Run one job on every rank (called collectively)."""
    import torch.distributed as dist

    from ..models import media
    from ..parallel.elastic import is_comm_failure
    from ..parallel.node_job import plan_segments, run_job

    st = get_store()
    # rank 0 decides (token, halt) and broadcasts the job so every rank runs the same plan
    box = [None]
    if rank == 0:
        ok = task_token_is_current(job_id, run_token, "transcode") and not is_job_halted(job_id)
        job = st.hgetall(job_key(job_id)) or {}
        if ok:
            try:
                from .tasks import resolve_input_path

                path = resolve_input_path(job)
                info = media.probe(path)
                job.update(source_width=info["width"], source_height=info["height"], source_codec=info["codec"])
                params = _job_params(job)
                segs = plan_segments(int(info["frames"]), params["segment_frames"], params["gop"])
                reset_job_run_state(job_id, job)  # keeps <base>/ckpt: a requeued job resumes
                t0 = now()
                base = job_base_dir(job_id, job)
                ensure_dirs(base)
                st.hset(job_key(job_id), mapping={
                    "status": Status.RUNNING.value, "started_at": job.get("started_at") or t0,
                    "source_codec": info["codec"], "source_resolution": info["resolution"],
                    "source_width": info["width"], "source_height": info["height"], "source_fps": info["fps"],
                    "source_fps_num": info["fps_num"], "source_fps_den": info["fps_den"],
                    "source_duration": info["duration"], "source_file_size": info["size"],
                    "total_frames": info["frames"], "source_bit_depth": info.get("bits", 8),
                    "processing_mode_effective": "node",
                    "processing_mode_reason": f"node executor: {world} GPU rank(s), RCCL data plane",
                    "parts_total": len(segs), "effective_parts": len(segs), "usable_encoder_workers": world,
                    "frames_per_part": params["segment_frames"], "segmented_chunks": len(segs),
                    "segment_progress": 100, "segment_elapsed": 0, "encode_started": t0, "node_world": world,
                    "master_host": os.environ.get("HOSTNAME", ""), "stitch_host": os.environ.get("HOSTNAME", "")})
                job_heartbeat(job_id, "transcode", force=True)
                emit_activity(f'Starting "{job_title(job)}" on {world} GPU rank(s)', job_id=job_id,
                              filename=job.get("filename"), stage="start", source="worker")
                box[0] = {"job": job, "path": path, "params": params, "segs": len(segs), "t0": t0, "base": base,
                          "ckpt": os.path.join(base, "ckpt")}
            except Exception as e:  # probe / planning failure
                _fail(job_id, f"node plan failed: {e}", "split")
    dist.broadcast_object_list(box, src=0, group=_gloo())
    spec = box[0]
    if spec is None:
        return
    p = spec["params"]
    if beat is not None:
        beat.set_job({"job_id": job_id, "run_token": run_token})
    hooks = _StoreHooks(job_id, spec["segs"], spec["t0"], beat)
    out_local = os.path.join(spec["base"], f"job_{job_id}_output.mp4")
    try:
        res = run_job(spec["path"], out_local, height=p["height"], qp=p["qp"], gop=p["gop"],
                      segment_frames=p["segment_frames"], mode=p["mode"], bitrate_kbps=p["bitrate_kbps"],
                      ladder=p["ladder"], search_range=p["search_range"], software=p["software"],
                      batch_segments=p["batch_segments"], hooks=hooks, deblock=p["deblock"], sao=p["sao"],
                      cache=None if p["software"] else cache, crf=p["crf"], resume_dir=spec["ckpt"],
                      scenecut=p.get("scenecut", False), codec=p.get("codec", "hevc"), qindex=p.get("qindex", 0),
                      bframes=p.get("bframes", 1),
                      audio_stream=int(spec["job"].get("selected_a_stream") or 0), rc_mode=p.get("rc", ""),
                      vbv_maxrate_kbps=p.get("vbv", [0, 0])[0], vbv_bufsize_kbit=p.get("vbv", [0, 0])[1],
                      deinterlace=p.get("deinterlace", False))
    except Exception as e:
        if is_comm_failure(e):  # the job is fine, the communicator is not: requeue + re-init
            log.error("[%s] communicator failure on rank %d: %s", job_id, rank, e)
            raise CommFailure(str(e)) from e
        if beat is not None:
            beat.set_job(None)
        if rank == 0:
            log.error("[%s] node job failed:\n%s", job_id, traceback.format_exc())
            if is_job_halted(job_id):
                return
            _fail(job_id, f"node job failed: {e}", "encode")
        return
    if rank == 0:
        _publish(job_id, spec, res)
    if beat is not None:
        beat.set_job(None)


def _publish(job_id: str, spec: dict, res: dict) -> None:
    """Stitch rank: move the muxed output(s) into the library, probe them, write dest_* and
    the per-job throughput / quality fields, mark DONE (reference stitch :2225-2307)."""
    st = get_store()
    job = spec["job"]
    t_comb = now()
    outs = res["outputs"]
    ext = os.path.splitext(outs[0]["path"])[1] or ".mp4"  # .mkv when English subtitles are carried
    final = final_output_path(str(job.get("filename") or f"{job_id}.mp4"), ext)
    ensure_dirs(os.path.dirname(final))
    finals = []
    for k, o in enumerate(outs):
        dst = final if k == 0 else f"{os.path.splitext(final)[0]}_{o['height']}p{os.path.splitext(o['path'])[1]}"
        tmp = dst + ".tmp"
        shutil.move(o["path"], tmp)
        os.replace(tmp, dst)
        finals.append(dst)
    fields = {"status": Status.DONE.value, "output_path": finals[0], "ended_at": now(), "combine_progress": 100,
              "combine_elapsed": round(now() - t_comb, 2), "stitched_chunks": spec["segs"], "encode_progress": 100,
              "encode_elapsed": round(res.get("encode_seconds", 0.0), 2), "job_fps": res.get("fps"),
              "encode_fps": res.get("encode_fps"), "psnr_y": outs[0].get("psnr_y"), "psnr_yuv": outs[0].get("psnr_yuv"),
              "bitrate_kbps": round(outs[0]["kbps"], 1), "rc_passes": res.get("passes", 1),
              "qp_plan_json": json.dumps(res.get("qp_plan", [])[:1]),
              "trace_json": json.dumps(res.get("trace") or {}), "job_seconds": res.get("seconds"),
              "ingest_json": json.dumps([{k: p.get(k) for k in ("reads", "read_bytes", "ingest_s", "read_thread_s", "read_threads", "encoded")}
                                         for p in res.get("per_rank") or []]),
              "stitch_json": json.dumps(res.get("stitch") or {}),
              "ladder_outputs_json": json.dumps(
                  [{"path": f, "width": o["width"], "height": o["height"], "kbps": round(o["kbps"], 1),
                    "psnr_y": o.get("psnr_y")} for f, o in zip(finals, outs)]) if len(outs) > 1 else ""}
    # dest_* from the muxer's own accounting (re-probing a multi-GB output would read it back)
    o = outs[0]
    fps = o["fps_num"] / o["fps_den"]
    dur = o["frames"] / fps if fps else 0.0
    fields.update(dest_file_size=os.path.getsize(finals[0]), dest_duration=f"{dur:.2f}", dest_codec=spec["params"].get("codec", "hevc"),
                  dest_resolution=f"{o['width']}x{o['height']}", dest_fps=f"{fps:.2f}",
                  dest_bitrate_kbps=f"{os.path.getsize(finals[0]) * 8 / dur / 1000 if dur else 0:.0f}",
                  english_subtitles_found=0, english_subtitles_supported=0, english_subtitles_kept=0,
                  subtitle_warning="")
    fields.update(res.get("side_fields") or {})
    st.hset(job_key(job_id), mapping={k: ("" if v is None else v) for k, v in fields.items()})
    st.srem(ACTIVE_JOBS_KEY, job_id)
    shutil.rmtree(spec["base"], ignore_errors=True)
    emit_activity(f'Encoding "{job_title(job)}" completed in {elapsed_ms(spec["t0"])}ms '
                  f'({res.get("fps")} frames/s, PSNR-Y {outs[0].get("psnr_y")} dB)', job_id=job_id,
                  filename=job.get("filename"), stage="encode_complete", source="worker")
    emit_activity(f'Writing "{os.path.basename(finals[0])}"', job_id=job_id, filename=job.get("filename"),
                  stage="write", source="worker")


def _fail(job_id: str, error: str, stage: str) -> None:
    st = get_store()
    st.hset(job_key(job_id), mapping={"status": Status.FAILED.value, "error": error[:2000], "failed_stage": stage,
                                      "failed_worker": os.environ.get("HOSTNAME", ""), "ended_at": now()})
    st.srem(ACTIVE_JOBS_KEY, job_id)
    job = st.hgetall(job_key(job_id)) or {}
    emit_activity(f'Job "{job_title(job)}" failed during {stage}: {error[:200]}', job_id=job_id,
                  filename=job.get("filename"), stage=f"{stage}_error", source="worker")


_gloo_group = None


def _gloo():
    """CPU (gloo) group for object broadcasts next to the RCCL data-plane group."""
    global _gloo_group
    import torch.distributed as dist

    if _gloo_group is None:
        _gloo_group = dist.new_group(backend="gloo") if dist.get_backend() != "gloo" else dist.group.WORLD
    return _gloo_group


def serve(host: str | None = None, max_jobs: int | None = None, idle_exit: float | None = None) -> int:
    """Rank loop: rank 0 pops jobs for this node and broadcasts them; every rank runs them."""
    import datetime

    import torch
    import torch.distributed as dist

    from ..parallel.elastic import EXIT_COMM, RankBeat
    from ..parallel.launch import pin_rank
    from .encoder import EngineCache, gpu_available

    log = get_logging("node-executor")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    host = host or os.environ.get("TV_NODE_HOST") or os.environ.get("HOSTNAME") or "localhost"
    gpu = gpu_available()
    pin_rank(local, int(os.environ.get("LOCAL_WORLD_SIZE", world)))
    if gpu:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local),
                                timeout=datetime.timedelta(seconds=float(os.environ.get("TV_NODE_TIMEOUT", "900"))))
    else:
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=float(os.environ.get("TV_NODE_TIMEOUT", "900"))))
    _gloo()
    cache = EngineCache(device=local, batch=int(os.environ.get("TV_NODE_ENGINE_BATCH", "0")), max_engines=6) if gpu else None
    st = get_store()
    stop = threading.Event()
    gen = int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))
    phys = [int(x) for x in os.environ.get("TV_PHYS_GPUS", "").split(",") if x.strip()] or list(range(world))
    rbeat = RankBeat(st, host, rank, gen, phys[local] if local < len(phys) else local).start()
    if rank == 0:
        st.sadd(EXECUTORS_KEY, host)

        def beat():
            while not stop.is_set():
                st.set(alive_key(host), json.dumps({"world": world, "pid": os.getpid(), "ts": now(), "gen": gen,
                                                    "gpus": phys}), ex=ALIVE_TTL)
                stop.wait(2.0)

        threading.Thread(target=beat, daemon=True, name="node-executor-beat").start()
        log.info("node executor on %s: %d rank(s), %s", host, world, "RCCL" if gpu else "gloo")
    done, idle_since = 0, time.monotonic()
    code = 0
    try:
        while True:
            box = [None]
            if rank == 0:
                item = st.blpop([queue_key(host)], timeout=1)
                if item is not None:
                    box[0] = json.loads(item[1])
                    idle_since = time.monotonic()
                elif idle_exit is not None and time.monotonic() - idle_since > idle_exit:
                    box[0] = {"stop": True}
            dist.broadcast_object_list(box, src=0, group=_gloo())
            msg = box[0]
            if msg is None:
                continue
            if msg.get("stop"):
                break
            try:
                execute(msg["job_id"], msg.get("run_token"), rank, world, cache, log, rbeat)
            except CommFailure:
                code = EXIT_COMM  # leave the broken communicator to the supervisor
                break
            done += 1
            if max_jobs is not None and done >= max_jobs:
                break
    finally:
        stop.set()
        if code == 0:  # a failing rank leaves its last beat (and job) for the supervisor
            rbeat.stop()
        if rank == 0 and code == 0:
            st.delete(alive_key(host))
        if cache is not None and code == 0:
            cache.close()
        if code == 0:
            dist.destroy_process_group()
    if code:
        sys.stdout.flush()
        os._exit(code)  # no teardown collectives on a dead communicator
    return 0


def _requeue(host: str, log):
    """Supervisor callback: put a failed generation's in-flight job back at the front of this
    node's queue (it resumes from its segment checkpoints), or fail it once its restart
    budget (TV_NODE_JOB_RESTARTS, default 3) is spent."""
    def requeue(job: dict, reason: str) -> bool:
        st = get_store()
        jid = job.get("job_id")
        if not jid:
            return False
        n = int(st.hincrby(job_key(jid), "node_restarts", 1))
        if n > int(os.environ.get("TV_NODE_JOB_RESTARTS", "3")):
            _fail(jid, f"node executor failed {n} times: {reason}", "encode")
            return False
        st.hset(job_key(jid), mapping={"node_last_failure": reason[:500]})
        rec = st.hgetall(job_key(jid)) or {}
        emit_activity(f'Requeueing "{job_title(rec)}" after {reason} (restart {n})', job_id=jid,
                      filename=rec.get("filename"), stage="retry", source="worker")
        st.lpush(queue_key(host), json.dumps({"job_id": jid, "run_token": job.get("run_token")}))
        log(f"requeued {jid}: {reason}")
        return True
    return requeue


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="thinvids-amd node executor (one rank per GPU)")
    ap.add_argument("--gpus", type=int, default=int(os.environ.get("TV_NODE_GPUS", "0")) or None)
    ap.add_argument("--host", default=None)
    ap.add_argument("--max-jobs", type=int, default=None)
    ap.add_argument("--idle-exit", type=float, default=None, help="exit after this many idle seconds")
    ap.add_argument("--no-supervise", action="store_true", help="plain launch: no rank restart / GPU fallback")
    a = ap.parse_args(argv)
    from ..parallel.launch import launched_by_torchrun, spawn_ranks

    if not launched_by_torchrun():
        n = a.gpus
        cpu = os.environ.get("TV_FORCE_CPU") == "1"
        if n is None:  # count devices from sysfs / the visibility list: no HIP call here
            from ..parallel.launch import visible_gpu_count

            n = 1 if cpu else max(1, visible_gpu_count())
        rank_argv = ["-m", "thinvids_amd.worker.node_executor", *(argv if argv is not None else sys.argv[1:])]
        if a.no_supervise:
            return spawn_ranks(n, rank_argv)
        from ..parallel.elastic import Supervisor

        host = a.host or os.environ.get("TV_NODE_HOST") or os.environ.get("HOSTNAME") or "localhost"
        log = get_logging("node-supervisor")
        sup = Supervisor(rank_argv, list(range(n)), host, get_store(),
                         stall_sec=float(os.environ.get("TV_NODE_STALL_SEC", "600")),
                         max_restarts=int(os.environ.get("TV_NODE_MAX_RESTARTS", "8")),
                         requeue=_requeue(host, log.warning), log=log.warning, cpu_mode=cpu)
        return sup.run()
    return serve(a.host, a.max_jobs, a.idle_exit)


if __name__ == "__main__":
    sys.exit(main())
