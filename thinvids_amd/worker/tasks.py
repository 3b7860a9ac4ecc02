"""Worker pipeline tasks (reference worker/tasks.py:808-2613).

    transcode(job)  ->  enqueue stitch(job) + split(job)                (pipeline queue)
    split(job)      ->  probe, plan GOP-aligned frame ranges, write parts
                        (split mode) and enqueue encode(job, idx) as each part
                        is ready (streaming dispatch = stage pipelining)
    encode(job,idx) ->  fetch part (HTTP from the master / direct source range),
                        Lanczos-resize on the GPU, HEVC-encode on the MI355X
                        engine, mux MP4, PUT to the stitcher, commit progress
    stitch(job)     ->  wait for parts with the head-of-line retry policy, concat
                        the Annex-B streams into one MP4, publish to the library
    stamp(job)      ->  burn frame numbers (HIP overlay), re-encode, new READY job

The batched consumer (:func:`encode_batch`) is the MI355X-specific part: a per-GPU
consumer pops up to N encode tasks at once and encodes all their GOP chunks in shared
batched engine launches (one part alone cannot fill 256 CUs).

Status values, job-hash fields, set/hash keys and activity messages follow the reference
contract.
"""
from __future__ import annotations

import logging
import os
import shutil
import time
import traceback
from fractions import Fraction

from ..common import Status, emit_activity
from ..models import hevc, media
from ..queue import get_encode_queue, get_pipeline_queue
from ..store import get_store
from ..utils import fault, trace
from . import dataplane, planning
from .config import get_config
from .encoder import EncodeSpec, encode_parts, prepare_frames
from .helpers import (active_gpu_count, disk_free_bytes, effective_target_height, elapsed_ms, ensure_dirs,
                      final_output_path, is_job_halted, job_base_dir, job_heartbeat, job_key, job_title, now,
                      output_geometry, part_paths, reset_job_run_state, task_token_is_current)

log = logging.getLogger("thinvids.worker.tasks")
pipeline_q = get_pipeline_queue()
encode_q = get_encode_queue()
ACTIVE_JOBS_KEY = "pipeline:active_jobs"
STAGE_TTL = 7 * 24 * 3600


def _store():
    return get_store()


def _job(job_id: str) -> dict:
    return _store().hgetall(job_key(job_id)) or {}


def _set(job_id: str, **fields) -> None:
    _store().hset(job_key(job_id), mapping={k: ("" if v is None else v) for k, v in fields.items()})


def _fail_job(job_id: str, error: str, stage: str, part: int = 0) -> None:
    _set(job_id, status=Status.FAILED.value, error=str(error)[:2000], failed_stage=stage, failed_part=part,
         failed_worker=get_config().worker_name, ended_at=now())
    _store().srem(ACTIVE_JOBS_KEY, job_id)
    job = _job(job_id)
    emit_activity(f'Job "{job_title(job)}" failed during {stage}: {str(error)[:200]}', job_id=job_id,
                  filename=job.get("filename"), stage=f"{stage}_error", source="worker")


def resolve_input_path(job: dict) -> str:
    p = str(job.get("input_path") or "").strip()
    if p:
        return p
    return os.path.join(get_config().watch_root, str(job.get("filename") or "").lstrip("/"))


def _fps(job: dict) -> tuple[int, int]:
    try:
        n, d = int(job.get("source_fps_num") or 0), int(job.get("source_fps_den") or 0)
        if n > 0 and d > 0:
            return n, d
    except ValueError:
        pass
    fr = Fraction(str(job.get("source_fps") or "30")).limit_denominator(1001)
    return (fr.numerator, fr.denominator) if fr > 0 else (30, 1)


def encode_spec_for_job(job: dict, settings: dict | None = None) -> EncodeSpec:
    from ..common import as_bool, as_int, get_settings

    s = settings or get_settings()
    w, h = int(job.get("source_width") or 0), int(job.get("source_height") or 0)
    if not (w and h):
        from .helpers import source_dimensions

        w, h = source_dimensions(job)
    th, _ = effective_target_height(job)
    ow, oh = output_geometry(w, h, th)
    return EncodeSpec(width=ow, height=oh, qp=as_int(job.get("qp") or s.get("tv_qp"), get_config().qp),
                      gop=max(1, as_int(s.get("tv_gop"), 64)), search_range=max(16, min(128, as_int(s.get("tv_search_range"), 64) // 16 * 16)),
                      deblock=as_bool(s.get("tv_deblock"), True), sao=as_bool(s.get("tv_sao"), True),
                      software=as_bool(job.get("software_encode")),
                      crf=as_int(job.get("crf") or s.get("tv_crf"), 27)
                      if str(job.get("rc_mode") or s.get("tv_rc") or "cqp").lower() == "crf" else 0,
                      scenecut=as_bool(s.get("tv_scenecut"), True),
                      codec="av1" if str(job.get("codec") or s.get("tv_codec") or "hevc").lower() == "av1" else "hevc",
                      qindex=as_int(job.get("qindex") or s.get("tv_qindex"), 0),
                      bframes=_pow2(as_int(job.get("bframes") or s.get("tv_bframes"), 1)))


def _pow2(n: int) -> int:
    """Largest power of two <= n in 1..16 (the engine's mini-GOP sizes)."""
    n = max(1, min(16, int(n)))
    return 1 << (n.bit_length() - 1)


# =====================================================================  transcode
@pipeline_q.task(retries=999999, retry_delay=5)
def transcode(job_id: str, run_token: str | None = None):
    """Orchestration entry (reference :810-833): reset run state, RUNNING, then enqueue the
    stitcher before the splitter so the receiving side exists first."""
    if not task_token_is_current(job_id, run_token, "transcode") or is_job_halted(job_id):
        return None
    job = _job(job_id)
    host = _node_executor_for(job)
    if host:
        # one node, N GPU ranks, RCCL data plane: the node executor runs the whole job
        from .node_executor import submit

        _set(job_id, processing_mode_effective="node", node_executor_host=host, waiting_node_at=now())
        job_heartbeat(job_id, "transcode", force=True)
        submit(job_id, run_token, host)
        return {"status": "QUEUED_NODE", "host": host}
    reset_job_run_state(job_id, job)
    _set(job_id, status=Status.RUNNING.value, started_at=job.get("started_at") or now())
    job_heartbeat(job_id, "transcode", force=True)
    emit_activity(f'Starting "{job_title(job)}"', job_id=job_id, filename=job.get("filename"), stage="start",
                  source="worker")
    stitch(job_id, run_token)
    split(job_id, run_token)
    return {"status": "DISPATCHED"}


def _node_executor_for(job: dict) -> str | None:
    """A live node executor takes the job (it subsumes the split and direct modes: every
    rank reads its own segment range) unless the setting `tv_node_executor` or the job's
    own `node_executor` field is off."""
    from ..common import as_bool, get_settings

    if not as_bool(get_settings().get("tv_node_executor"), True) or not as_bool(job.get("node_executor"), True):
        return None
    from .node_executor import live_executor

    return live_executor(prefer=get_config().worker_name)


# =========================================================================  split
@pipeline_q.task(retries=0)
def split(job_id: str, run_token: str | None = None):
    """Segmenter / master (reference :836-1351)."""
    from ..common import as_float, get_settings

    if not task_token_is_current(job_id, run_token, "split") or is_job_halted(job_id):
        return None
    st = _store()
    cfg = get_config()
    job = _job(job_id)
    title = job_title(job)
    t0 = now()
    src_path = resolve_input_path(job)
    try:
        info = media.probe(src_path)
    except Exception as e:
        _fail_job(job_id, f"probe failed: {e}", "split")
        return None
    if info["codec"] == "av1" and str(get_settings().get("av1_check_enabled", "1")) == "1":
        _set(job_id, status=Status.REJECTED.value, rejected_reason="AV1 source", rejected_at=now(), ended_at=now())
        st.srem(ACTIVE_JOBS_KEY, job_id)
        return None
    _set(job_id, source_codec=info["codec"], source_resolution=info["resolution"], source_width=info["width"],
         source_height=info["height"], source_fps=info["fps"], source_fps_num=info["fps_num"],
         source_fps_den=info["fps_den"], source_duration=info["duration"], source_file_size=info["size"],
         total_frames=info["frames"])
    job = _job(job_id)
    server = dataplane.start_http_once()
    _set(job_id, master_host=cfg.worker_name, master_endpoint=dataplane.advertised_endpoint())
    settings = get_settings()
    mode, reason = planning.resolve_processing_mode(job, settings, int(info["size"] or 0),
                                                    disk_free_bytes(job_base_dir(job_id, job)))
    spec = encode_spec_for_job(job, settings)
    usable = max(1, active_gpu_count(st))
    plan = planning.plan_parts(int(info["frames"]), usable, gop=spec.gop,
                               segment_frames=int(as_float(settings.get("tv_segment_frames"), 0)),
                               size_b=int(info["size"] or 0),
                               target_segment_mb=as_float(settings.get("target_segment_mb"), 10),
                               est_bytes_per_frame=spec.width * spec.height * 0.02)
    if str(job.get("number_parts_override")) == "1" and str(job.get("number_parts") or "").isdigit() \
            and int(job["number_parts"]) > 0:
        # per-job override (stored but unused by the reference pipeline; honoured here)
        plan = planning.plan_parts(int(info["frames"]), 0, gop=spec.gop,
                                   segment_frames=-(-int(info["frames"]) // int(job["number_parts"])))
    total = len(plan.ranges)
    _set(job_id, processing_mode_effective=mode, processing_mode_reason=reason,
         requested_parts=plan.requested_parts, effective_parts=plan.effective_parts,
         usable_encoder_workers=usable, parts_total=total, frames_per_part=plan.frames_per_part,
         direct_segment_duration=round(plan.frames_per_part * int(info["fps_den"]) / int(info["fps_num"]), 3)
         if mode == "direct" else "", segment_started=now())
    emit_activity(f'Segmenting "{title}" into {total} parts ({mode}: {reason})', job_id=job_id,
                  filename=job.get("filename"), stage="segment", source="worker")
    src = media.open_source(src_path) if mode == "split" else None
    for idx, start, n in plan.ranges:
        if is_job_halted(job_id):
            return {"status": "HALTED"}
        if mode == "split":
            part, _ = part_paths(job_id, idx, job)
            ensure_dirs(os.path.dirname(part))
            tmp = part + ".writing"
            media.write_y4m(tmp, src.read(start, n), int(info["fps_num"]), int(info["fps_den"]))
            os.replace(tmp, part)
        encode(job_id, idx, run_token=run_token, start_frame=start, nframes=n, mode=mode)
        done = st.hincrby(job_key(job_id), "segmented_chunks", 1)
        _set(job_id, segment_progress=int(100 * done / max(1, total)), segment_elapsed=round(now() - t0, 2))
        job_heartbeat(job_id, "split")
    emit_activity(f'Segmenting "{title}" completed in {elapsed_ms(t0)}ms', job_id=job_id,
                  filename=job.get("filename"), stage="segment_complete", source="worker")
    del server
    return {"status": "SEGMENTED", "parts": total}


# ========================================================================  encode
@encode_q.task(retries=0)
def encode(job_id: str, idx: int, run_token: str | None = None, start_frame: int = 0, nframes: int = 0,
           mode: str = "split"):
    """One part (reference :1354-1737).  Queue consumers normally route through
    :func:`encode_batch`; calling the task enqueues it."""
    return encode_batch([dict(job_id=job_id, idx=idx, run_token=run_token, start_frame=start_frame,
                              nframes=nframes, mode=mode)])[0]


def _load_part(job_id: str, job: dict, t: dict) -> list:
    if t.get("mode") == "direct":
        return media.open_source(resolve_input_path(job)).read(int(t["start_frame"]), int(t["nframes"]))
    part, _ = part_paths(job_id, int(t["idx"]), job)
    if os.path.isfile(part):  # same host or shared scratch
        src = media.Y4MSource(part)
        return src.read(0, src.nframes)
    endpoint = job.get("master_endpoint") or job.get("master_host")
    if not endpoint:
        raise RuntimeError("no master endpoint for split-mode part")
    local = os.path.join(get_config().project_root, job_id, "in", f"in_{int(t['idx']):03d}.y4m")
    dataplane.fetch_part(endpoint, job_id, int(t["idx"]), local)
    try:
        src = media.Y4MSource(local)
        return src.read(0, src.nframes)
    finally:
        os.remove(local)


def _deliver(job_id: str, job: dict, idx: int, data: bytes) -> None:
    """PUT to the stitcher (reference :1655-1684); write directly when the stitcher's
    scratch is ours."""
    deadline = now() + get_config().encode_stitcher_wait_sec
    endpoint = job.get("stitch_endpoint")
    while not endpoint and now() < deadline:
        time.sleep(0.2)
        endpoint = _store().hget(job_key(job_id), "stitch_endpoint")
    endpoint = endpoint or job.get("master_endpoint")
    mine = dataplane.advertised_endpoint() if dataplane._server is not None else None
    if endpoint and endpoint != mine:
        dataplane.upload_result(endpoint, job_id, idx, data)
        return
    _, enc = part_paths(job_id, idx, job)
    ensure_dirs(os.path.dirname(enc))
    tmp = f"{enc}.{os.getpid()}.uploading"
    with open(tmp, "wb") as f:
        f.write(data)
    os.replace(tmp, enc)


def _commit(job_id: str, job: dict, idx: int, t0: float) -> None:
    st = _store()
    k = job_key(job_id)
    if st.sadd(f"job_done_parts:{job_id}", idx):
        p = st.pipeline()
        p.hincrby(k, "completed_chunks", 1)
        p.hincrby(k, "parts_done", 1)
        p.execute()
    started = float(st.hget(k, "encode_started") or t0)
    st.hset(k, "encode_elapsed", int(now() - started))
    total = int(st.hget(k, "parts_total") or 0)
    done = int(st.hget(k, "parts_done") or 0)
    emit_activity(f'Encoding "{job_title(job)}" part {idx} completed in {elapsed_ms(t0)}ms', job_id=job_id,
                  filename=job.get("filename"), stage="encode", source="worker")
    if total > 0:
        prog = int(done * 100 / total)
        if prog > int(st.hget(k, "encode_progress") or 0):
            st.hset(k, "encode_progress", prog)
        if done >= total and st.set(f"{k}:encode_stage_complete", "1", nx=True, ex=STAGE_TTL):
            emit_activity(f'Encoding "{job_title(job)}" completed in {elapsed_ms(started)}ms', job_id=job_id,
                          filename=job.get("filename"), stage="encode_complete", source="worker")


def _part_failed(job_id: str, job: dict, t: dict, reason: str, stage: str) -> dict:
    """Retry accounting + requeue, or fail the job when the budget is spent (:1385-1464)."""
    st = _store()
    cfg = get_config()
    idx = int(t["idx"])
    cnt = int(st.hincrby(f"job_retry_counts:{job_id}", idx, 1))
    st.hset(f"job_retry_ts:{job_id}", idx, now())
    st.srem(f"job_retry_inflight:{job_id}", idx)
    why = f"part {idx} ({stage}): {reason}"
    if cnt <= cfg.part_failure_max_retries and not is_job_halted(job_id):
        w = cfg.worker_name
        _set(job_id, last_part_error=why, last_failed_part=idx, last_failed_stage=stage, last_failed_worker=w,
             last_failed_at=now(), last_retry_part=idx, last_retry_stage=stage, last_retry_worker=w,
             last_retry_at=now())
        emit_activity(f'Retrying "{job_title(job)}" part {idx} after failure on {w}', job_id=job_id,
                      filename=job.get("filename"), stage="part_retry", source="worker")
        encode(job_id, idx, run_token=t.get("run_token"), start_frame=t.get("start_frame", 0),
               nframes=t.get("nframes", 0), mode=t.get("mode", "split"))
        return {"status": "RETRYING", "reason": why}
    _fail_job(job_id, f"{why}; retry budget exhausted ({cnt}/{cfg.part_failure_max_retries})", stage, idx)
    return {"status": "FAILED", "reason": why}


def encode_batch(tasks: list[dict]) -> list[dict | None]:
    """Encode several parts (any jobs) with shared batched GPU launches."""
    st = _store()
    results: list = [None] * len(tasks)
    live = []  # (i, task, job, spec, frames, t0)
    for i, t in enumerate(tasks):
        job_id, idx = t["job_id"], int(t["idx"])
        if not task_token_is_current(job_id, t.get("run_token"), "encode") or is_job_halted(job_id):
            results[i] = {"status": "SKIPPED"}
            continue
        if st.sismember(f"job_done_parts:{job_id}", idx):
            results[i] = {"status": "COMPLETED", "idx": idx, "duplicate": True}
            continue
        job = _job(job_id)
        t0 = now()
        if st.set(f"{job_key(job_id)}:encode_stage_started", "1", nx=True, ex=STAGE_TTL):
            _set(job_id, encode_started=t0)
            emit_activity(f'Encoding "{job_title(job)}" started', job_id=job_id, filename=job.get("filename"),
                          stage="encode_start", source="worker")
        job_heartbeat(job_id, "encode", note=f"part {idx}")
        try:
            fault.check("download", idx)
            spec = encode_spec_for_job(job)
            _, deint = effective_target_height(job)  # DVD-native SD keeps its lines + bwdif
            with trace.span("worker.download"):
                raw = _load_part(job_id, job, t)
            with trace.span("worker.prepare"):
                frames = prepare_frames(raw, spec.width, spec.height, deinterlace=deint)
            if not frames:
                raise RuntimeError("part has no frames")
            live.append((i, t, job, spec, frames, t0))
        except Exception as e:
            log.error("[%s] part %s load failed:\n%s", job_id, idx, traceback.format_exc())
            results[i] = _part_failed(job_id, job, t, str(e), "download")
    by_spec: dict = {}
    for item in live:
        by_spec.setdefault(item[3], []).append(item)
    for spec, items in by_spec.items():
        ok = []
        for it in items:
            try:
                fault.check("part", int(it[1]["idx"]))
                ok.append(it)
            except fault.InjectedFault as e:
                results[it[0]] = _part_failed(it[1]["job_id"], it[2], it[1], str(e), "encode")
        items = ok
        if not items:
            continue
        try:
            with trace.span("worker.encode", parts=len(items)):
                bits = encode_parts([it[4] for it in items], spec)
        except Exception as e:
            log.error("encode failed:\n%s", traceback.format_exc())
            for i, t, job, *_ in items:
                results[i] = _part_failed(t["job_id"], job, t, str(e), "encode")
            continue
        for (i, t, job, spec_, frames, t0), annexb in zip(items, bits):
            job_id, idx = t["job_id"], int(t["idx"])
            try:
                fault.check("upload", idx)
                fn, fd = _fps(job)
                with trace.span("worker.upload"):
                    _deliver(job_id, job, idx, hevc.mux_mp4(annexb, spec.width, spec.height, fn, fd))
                _commit(job_id, job, idx, t0)
                results[i] = {"status": "COMPLETED", "idx": idx, "bytes": len(annexb), "frames": len(frames)}
            except Exception as e:
                log.error("[%s] part %s upload failed:\n%s", job_id, idx, traceback.format_exc())
                results[i] = _part_failed(job_id, job, t, str(e), "upload")
    return results


def encode_batch_handler(max_tasks: int | None = None, timeout: float = 1.0) -> bool:
    """Consumer loop body for the encode queue: pop up to N encode tasks, run them as one
    batched call.  Returns False when the queue was empty."""
    n = max_tasks or get_config().encode_batch_tasks
    msgs = encode_q.pop_batch(n, lambda a, b: True, timeout=timeout)
    if not msgs:
        return False
    plain = [m for m in msgs if m["task"] == "encode"]
    for m in msgs:
        if m["task"] != "encode":
            encode_q._execute(m)
    if plain:
        kws = []
        for m in plain:
            kw = dict(m.get("kwargs") or {})
            for name, v in zip(("job_id", "idx"), m.get("args") or []):
                kw[name] = v
            kws.append(kw)
        encode_batch(kws)
    return True


# =========================================================================  stitch
def _ready_set(enc_dir: str, total: int, stable_sec: float) -> set:
    """Parts whose encoded file exists and has been stable for `stable_sec` (:1805-1822)."""
    ready = set()
    t = time.time()
    for i in range(1, total + 1):
        p = os.path.join(enc_dir, f"enc_{i:03d}.mp4")
        try:
            stt = os.stat(p)
        except FileNotFoundError:
            continue
        if stt.st_size > 0 and t - stt.st_mtime >= stable_sec:
            ready.add(i)
    return ready


def concat_parts(paths: list[str], out_path: str, width: int, height: int, fps_num: int, fps_den: int,
                 plan=None) -> tuple[str, int]:
    """Concatenate encoded MP4 parts (each a run of closed GOPs) into one faststart file
    (reference `ffmpeg -f concat -c copy +faststart`, :2047-2120) together with the source's
    side streams of `plan` (:func:`thinvids_amd.models.streams.plan_output`; the reference's
    subtitle remux pass :2126-2223 folds into this one write).  Returns (path, bytes): the
    extension is the plan's (.mkv when English subtitles are carried)."""
    from ..models import streams

    from ..models import av1

    segs = []
    for p in paths:  # each part's elementary stream; the output is streamed from these buffers
        with open(p, "rb") as f:
            data = f.read()
        # tv_codec=av1 parts are av01 MP4s (OBU temporal units), HEVC parts hvc1 (Annex-B)
        segs.append(av1.mp4_av1_stream(data)[1] if av1.mp4_av1_track(data) else hevc.demux_mp4(data)["annexb"])
    ensure_dirs(os.path.dirname(out_path) or ".")
    return streams.write_output(segs, width, height, fps_num, fps_den, out_path, plan)


@pipeline_q.task(retries=0)
def stitch(job_id: str, run_token: str | None = None):
    """Stitcher (reference :1741-2312)."""
    if not task_token_is_current(job_id, run_token, "stitch") or is_job_halted(job_id):
        return None
    st = _store()
    cfg = get_config()
    dataplane.start_http_once()
    _set(job_id, stitch_host=cfg.worker_name, stitch_endpoint=dataplane.advertised_endpoint())
    job = _job(job_id)
    t_stage = now()
    deadline = now() + cfg.stitch_wait_parts_total_sec
    total = 0
    while total <= 0:
        if is_job_halted(job_id):
            return {"status": "HALTED"}
        total = int(st.hget(job_key(job_id), "parts_total") or 0)
        if total > 0:
            break
        if now() > deadline:
            _fail_job(job_id, "timed out waiting for parts_total", "stitch")
            return None
        job_heartbeat(job_id, "stitch_wait")
        time.sleep(cfg.stitch_poll_sec)
    base = job_base_dir(job_id, job)
    enc_dir = os.path.join(base, "encoded")
    tun = planning.StitchTunables()
    ready: set = set()
    last_change = now()
    while True:
        if is_job_halted(job_id):
            return {"status": "HALTED"}
        cur = _ready_set(enc_dir, total, cfg.stitch_stable_sec)
        if cur != ready:
            ready, last_change = cur, now()
        if len(ready) >= total:
            break
        seg = int(st.hget(job_key(job_id), "segmented_chunks") or 0)
        miss = {int(k): float(v) for k, v in (st.hgetall(f"job_missing_first_seen:{job_id}") or {}).items()}
        cnt = {int(k): int(v) for k, v in (st.hgetall(f"job_retry_counts:{job_id}") or {}).items()}
        rts = {int(k): float(v) for k, v in (st.hgetall(f"job_retry_ts:{job_id}") or {}).items()}
        newly, to_retry, give_up = planning.plan_redispatch(ready, total, seg, now(), last_change, miss, cnt, rts,
                                                            est_part_secs=30.0, t=tun)
        for i in newly:
            st.hsetnx(f"job_missing_first_seen:{job_id}", i, now())
        if give_up:
            _fail_job(job_id, "parts missing after retry budget", "stitch")
            return None
        for i in to_retry:
            if st.sadd(f"job_retry_inflight:{job_id}", i):
                st.hincrby(f"job_retry_counts:{job_id}", i, 1)
                st.hset(f"job_retry_ts:{job_id}", i, now())
                _redispatch(job_id, i, run_token)
        job_heartbeat(job_id, "stitch", note=f"{len(ready)}/{total} parts")
        time.sleep(cfg.stitch_poll_sec)
    # ---------------------------------------------------------------- combine
    t_comb = now()
    _set(job_id, combine_progress=0, combine_elapsed=0)
    job = _job(job_id)
    spec = encode_spec_for_job(job)
    fn, fd = _fps(job)
    out_local = os.path.join(base, f"job_{job_id}_output.mp4")
    paths = [os.path.join(enc_dir, f"enc_{i:03d}.mp4") for i in range(1, total + 1)]
    plan = _side_plan(job_id, job)
    try:
        fault.check("stitch", "*")
        with trace.span("stitch.concat"):
            out_local, _ = concat_parts(paths, out_local, spec.width, spec.height, fn, fd, plan)
        final = final_output_path(str(job.get("filename") or f"{job_id}.mp4"), plan.ext if plan else ".mp4")
        ensure_dirs(os.path.dirname(final))
        tmp = final + ".tmp"
        shutil.move(out_local, tmp)
        os.replace(tmp, final)
    except Exception as e:
        log.error("[%s] stitch failed:\n%s", job_id, traceback.format_exc())
        _fail_job(job_id, f"stitch failed: {e}", "stitch")
        return None
    try:
        d = media.probe(final)
        _set(job_id, dest_file_size=d["size"], dest_duration=f"{d['duration']:.2f}", dest_codec=d["codec"],
             dest_resolution=d["resolution"], dest_fps=f"{d['fps']:.2f}",
             dest_bitrate_kbps=f"{d['bitrate_kbps']:.0f}", dest_streams=len(d["streams"]),
             **(plan.fields if plan else {"english_subtitles_found": 0, "english_subtitles_supported": 0,
                                          "english_subtitles_kept": 0, "subtitle_warning": ""}))
    except Exception:
        log.warning("[%s] dest probe failed", job_id)
    shutil.rmtree(base, ignore_errors=True)
    _set(job_id, status=Status.DONE.value, output_path=final, ended_at=now(), combine_progress=100,
         combine_elapsed=round(now() - t_comb, 2), stitched_chunks=total)
    st.srem(ACTIVE_JOBS_KEY, job_id)
    emit_activity(f'Stitching "{job_title(job)}" completed in {elapsed_ms(t_stage)}ms', job_id=job_id,
                  filename=job.get("filename"), stage="stitch_complete", source="worker")
    emit_activity(f'Writing "{os.path.basename(final)}"', job_id=job_id, filename=job.get("filename"),
                  stage="write", source="worker")
    st.delete(f"job_done_parts:{job_id}", f"job_retry_counts:{job_id}", f"job_retry_ts:{job_id}",
              f"job_missing_first_seen:{job_id}", f"job_retry_inflight:{job_id}")
    return {"status": "COMPLETED", "output": final}


def _side_plan(job_id: str, job: dict):
    """Side streams of the job's source for the output (audio copy, English subtitles);
    None (video-only MP4) when the source cannot be indexed — the video is never lost over
    a side-stream problem (the reference likewise keeps the MP4 when its remux fails,
    :2202-2219)."""
    from ..models import streams

    src = resolve_input_path(job)
    try:
        plan = streams.plan_output(src, int(job.get("selected_a_stream") or 0))
    except Exception as e:  # noqa: BLE001
        log.warning("[%s] side streams skipped: %s", job_id, e)
        _set(job_id, subtitle_warning=f"side streams skipped: {e}"[:500])
        return None
    for w in plan.warnings:
        emit_activity(f'{w} for "{job_title(job)}"', job_id=job_id, filename=job.get("filename"),
                      stage="subtitle_warning", source="worker")
    return plan


def _redispatch(job_id: str, idx: int, run_token: str | None) -> None:
    """Re-enqueue a missing part (reference `_retry_part`, :1845-1896)."""
    job = _job(job_id)
    mode = job.get("processing_mode_effective") or "split"
    fpp = int(job.get("frames_per_part") or 0)
    total_frames = int(job.get("total_frames") or 0)
    start = (idx - 1) * fpp
    n = max(0, min(fpp, total_frames - start)) if fpp else 0
    emit_activity(f'Redispatching "{job_title(job)}" part {idx}', job_id=job_id, filename=job.get("filename"),
                  stage="stitch_retry", source="worker")
    encode(job_id, idx, run_token=run_token, start_frame=start, nframes=n, mode=mode)


# ==========================================================================  stamp
STAMP_GOP = 64    # frames per stamped segment (closed GOP)
STAMP_BATCH = 4   # segments per engine launch (bounds host memory)


@pipeline_q.task(retries=0)
def stamp(job_id: str, run_token: str | None = None):
    """Verification encode (reference :2314-2613): burn the frame number into every frame,
    re-encode at high quality next to the source, create a NEW READY job for it."""
    import uuid

    from ..ops.overlay import stamp_ref

    st = _store()
    job = _job(job_id)
    if not task_token_is_current(job_id, run_token, "stamp"):
        return None
    src_path = resolve_input_path(job)
    t0 = now()
    try:
        src = media.open_source(src_path)
        base, _ = os.path.splitext(src_path)
        out = base + ".stamped.mp4"
        _set(job_id, stamp_source=src_path, stamp_tmp=out + ".tmp", stamp_output=out)
        # streamed in closed-GOP chunks (reference :2424-2437 pipes ffmpeg frame by frame): a
        # chunk of STAMP_GOP frames is read, stamped and becomes one IDR-first segment; a few
        # chunks are encoded per engine launch and only their bitstreams are kept, so host
        # memory is bounded by STAMP_BATCH chunks whatever the source length
        spec = EncodeSpec(width=src.width, height=src.height, qp=18, gop=STAMP_GOP, software=not _gpu_ok())
        bits, pending = [], []
        for start in range(0, src.nframes, STAMP_GOP):
            chunk = src.read(start, STAMP_GOP)
            pending.append(_stamp_chunk(chunk, start, stamp_ref))
            del chunk
            if len(pending) == STAMP_BATCH or start + STAMP_GOP >= src.nframes:
                bits.extend(encode_parts(pending, spec))
                pending = []
            job_heartbeat(job_id, "stamp", note=f"{min(src.nframes, start + STAMP_GOP)}/{src.nframes}")
        hevc.mux_mp4_file(bits, src.width, src.height, src.fps_num, src.fps_den, out + ".tmp")
        os.replace(out + ".tmp", out)
    except Exception as e:
        log.error("[%s] stamp failed:\n%s", job_id, traceback.format_exc())
        _fail_job(job_id, f"stamp failed: {e}", "stamp")
        return None
    new_id = str(uuid.uuid4())
    rel = os.path.relpath(out, get_config().watch_root) if out.startswith(get_config().watch_root) else out
    new = {k: v for k, v in job.items() if k in ("target_height", "software_encode", "source_origin",
                                                  "selected_v_stream", "selected_a_stream")}
    new.update(job_id=new_id, filename=rel.lstrip("/"), input_path=out, status=Status.READY.value,
               created_at=now(), stamp_source=src_path)
    st.hset(job_key(new_id), mapping=new)
    st.sadd("jobs:all", job_key(new_id))
    _set(job_id, status=Status.READY.value, stamp_finished_at=now(), stamp_new_job_id=new_id, queue_action="")
    st.srem(ACTIVE_JOBS_KEY, job_id)
    emit_activity(f'Stamped "{job_title(job)}" in {elapsed_ms(t0)}ms -> new job {new_id[:8]}', job_id=job_id,
                  filename=job.get("filename"), stage="stamp", source="worker")
    return {"status": "STAMPED", "new_job_id": new_id, "output": out}


def _gpu_ok() -> bool:
    from .encoder import gpu_available

    return gpu_available()


def _stamp_chunk(chunk: list, start: int, stamp_ref) -> list:
    if not _gpu_ok():
        return [stamp_ref(f, str(start + k)) for k, f in enumerate(chunk)]
    import numpy as np
    import torch

    from ..ops.overlay import stamp_frames_gpu

    h, w = chunk[0][0].shape
    flat = np.stack([np.concatenate([p.ravel() for p in f]) for f in chunk])
    dev = torch.from_numpy(flat).cuda()
    stamp_frames_gpu(dev, w, h, [start + k for k in range(len(chunk))])
    host = dev.cpu().numpy()
    ysz, csz = w * h, (w // 2) * (h // 2)
    return [(r[:ysz].reshape(h, w), r[ysz:ysz + csz].reshape(h // 2, w // 2),
             r[ysz + csz:].reshape(h // 2, w // 2)) for r in host]
