"""Worker helper layer (reference worker/tasks.py:83-654).

Job key/title, heartbeat, scratch layout, active-node discovery, run-state reset,
cooperative cancellation (halt + run-token checks) and target-geometry decisions.  The
Redis contract is unchanged: every key and field named here is the reference's.
"""
from __future__ import annotations

import logging
import os
import re
import shutil
import time

from ..common import Status, get_settings
from ..store import get_store
from .config import get_config

log = logging.getLogger("thinvids.worker")

DISABLED_NODES_KEY = "nodes:disabled"
_HEARTBEAT_CACHE: dict[str, float] = {}


def job_key(job_id: str) -> str:
    return f"job:{job_id}"


def job_title(job: dict) -> str:
    base = os.path.basename((job.get("filename") or "").strip())
    if not base:
        return "Unknown"
    return os.path.splitext(base)[0] or base


def now() -> float:
    return time.time()


def elapsed_ms(started_at) -> int:
    try:
        return max(0, int(round((now() - float(started_at)) * 1000)))
    except (TypeError, ValueError):
        return 0


def job_heartbeat(job_id: str, stage: str, force: bool = False, note: str = "", store=None) -> None:
    """Liveness for the manager watchdog (reference :106-123), rate limited per process."""
    t = now()
    stage = str(stage or "").strip() or "unknown"
    if not force and t - _HEARTBEAT_CACHE.get(job_id, 0.0) < get_config().job_heartbeat_interval_sec:
        return
    mapping = {"last_heartbeat_at": str(t), "last_heartbeat_stage": stage,
               "last_heartbeat_host": get_config().worker_name}
    if note:
        mapping["last_heartbeat_note"] = str(note)[:500]
    try:
        (store or get_store()).hset(job_key(job_id), mapping=mapping)
        _HEARTBEAT_CACHE[job_id] = t
    except Exception:
        pass


def node_is_disabled(store=None, host: str | None = None) -> bool:
    return bool((store or get_store()).sismember(DISABLED_NODES_KEY, host or get_config().worker_name))


def quarantine_current_node(reason: str, job_id: str | None = None, part_idx: int | None = None,
                            store=None) -> None:
    """Disable this node (reference :125-139).  Unlike the reference (defined but never
    called) the encode consumer calls this when the GPU engine cannot be initialised."""
    st = store or get_store()
    host = get_config().worker_name
    try:
        st.sadd(DISABLED_NODES_KEY, host)
        st.hset(f"node:quarantine:{host}", mapping={
            "hostname": host, "reason": str(reason or "")[:1000], "job_id": job_id or "",
            "part_idx": "" if part_idx is None else str(part_idx), "quarantined_at": str(now())})
        st.delete(f"metrics:node:{host}")
    except Exception:
        log.exception("failed to quarantine node %s", host)


def ensure_dirs(*paths: str) -> None:
    for p in paths:
        os.makedirs(p, exist_ok=True)


def active_nodes(store=None) -> list[str]:
    """Hosts from ``nodes:mac`` whose heartbeat ts is within TTL+grace, minus disabled
    (reference :149-177)."""
    st = store or get_store()
    cfg = get_config()
    cutoff = int(now()) - (cfg.metrics_ttl_sec + cfg.metrics_grace_sec)
    hosts = list((st.hgetall("nodes:mac") or {}).keys())
    if not hosts:
        return []
    disabled = set(st.smembers(DISABLED_NODES_KEY) or [])
    p = st.pipeline()
    for h in hosts:
        p.hget(f"metrics:node:{h}", "ts")
    out = []
    for h, ts in zip(hosts, p.execute()):
        try:
            t = int(float(ts or 0))
        except (TypeError, ValueError):
            t = 0
        if t >= cutoff and h not in disabled:
            out.append(h)
    return sorted(out)


def active_gpu_count(store=None) -> int:
    """Encode capacity in GPUs: the agent publishes ``gpu_count`` per node."""
    st = store or get_store()
    total = 0
    for h in active_nodes(st):
        try:
            total += max(1, int(float(st.hget(f"metrics:node:{h}", "gpu_count") or 1)))
        except (TypeError, ValueError):
            total += 1
    return total


# ------------------------------------------------------------------- scratch layout
def job_project_root(job_id: str, job: dict | None = None, store=None) -> str:
    job = job if job is not None else ((store or get_store()).hgetall(job_key(job_id)) or {})
    root = str(job.get("scratch_root_effective") or job.get("scratch_root") or "").strip()
    return root or get_config().project_root


def job_base_dir(job_id: str, job: dict | None = None, store=None) -> str:
    """``{scratch_root or PROJECT_ROOT}/{job_id}`` (reference :276-307)."""
    return os.path.join(job_project_root(job_id, job, store), job_id)


def part_paths(job_id: str, idx: int, job: dict | None = None, store=None) -> tuple[str, str]:
    """(raw part served to encoders, encoded part received by the stitcher).

    The reference's ``parts/part_%03d.ts`` stream-copy chunks become raw YUV4MPEG2 parts
    (this engine owns the decode side); the encoded name ``encoded/enc_%03d.mp4`` is kept."""
    base = job_base_dir(job_id, job, store)
    return (os.path.join(base, "parts", f"part_{idx:03d}.y4m"),
            os.path.join(base, "encoded", f"enc_{idx:03d}.mp4"))


# Per-run counters of a job: zeroed by every restart / requeue path (worker reset and the
# manager's restart route share this list, so a requeued 2-pass job never reads a stale pass)
RUN_COUNTER_FIELDS = ("parts_total", "parts_done", "segmented_chunks", "completed_chunks", "stitched_chunks",
                      "segment_progress", "segment_elapsed", "encode_progress", "encode_elapsed", "combine_progress",
                      "combine_elapsed", "failed_part", "last_heartbeat_at", "ended_at", "rc_pass", "encoded_frames",
                      *(f"{f}_p{k}" for f in ("parts_done", "completed_chunks", "encoded_frames") for k in (1, 2)))


def reset_job_run_state(job_id: str, job: dict | None = None, store=None) -> None:
    """Clear per-run files and counters so restarts never reuse old parts (:318-378)."""
    st = store or get_store()
    base = job_base_dir(job_id, job, st)
    for sub in ("parts", "encoded"):
        shutil.rmtree(os.path.join(base, sub), ignore_errors=True)
        ensure_dirs(os.path.join(base, sub))
    for name in ("concat.txt", f"job_{job_id}_output.mp4"):
        try:
            os.remove(os.path.join(base, name))
        except FileNotFoundError:
            pass
    zero = {k: 0 for k in RUN_COUNTER_FIELDS}
    blank = {k: "" for k in ("error", "failed_stage", "failed_worker", "processing_mode_effective",
                             "processing_mode_reason", "direct_segment_duration", "last_heartbeat_stage",
                             "last_heartbeat_host", "last_heartbeat_note")}
    try:
        st.hset(job_key(job_id), mapping={**zero, **blank})
        st.delete(f"job_done_parts:{job_id}", f"job_retry_counts:{job_id}", f"job_retry_ts:{job_id}",
                  f"job_missing_first_seen:{job_id}", f"job_retry_inflight:{job_id}")
    except Exception:
        pass


def final_output_path(src_filename: str, extension: str = ".mp4") -> str:
    """``LIBRARY_ROOT/<filename without ext>.<ext>`` (reference :380-390)."""
    base, _ = os.path.splitext(src_filename)
    ext = extension if extension.startswith(".") else "." + extension
    return os.path.join(get_config().library_root, base.lstrip("/") + ext)


# ------------------------------------------------------- cooperative cancellation
def is_job_halted(job_id: str, store=None) -> bool:
    s = Status.parse((store or get_store()).hget(job_key(job_id), "status"))
    return s in (Status.FAILED, Status.REJECTED, Status.STOPPED)


def task_token_is_current(job_id: str, run_token: str | None, task_name: str, store=None) -> bool:
    """Ignore replayed work from an older dispatch of the same job (reference :396-424)."""
    token = str(run_token or "").strip()
    current = str((store or get_store()).hget(job_key(job_id), "pipeline_run_token") or "").strip()
    if current:
        if token == current:
            return True
        log.warning("[%s] %s: stale task ignored (token=%s current=%s)", job_id, task_name,
                    token[:8] or "missing", current[:8])
        return False
    if token:
        log.warning("[%s] %s: tokened task ignored because job has no current token", job_id, task_name)
        return False
    return True


# ------------------------------------------------------------------ target geometry
def normalize_target_height(value) -> int:
    cfg = get_config()
    try:
        h = int(value)
    except (TypeError, ValueError):
        return cfg.default_target_height
    return h if h in cfg.allowed_target_heights else cfg.default_target_height


def source_dimensions(job: dict) -> tuple[int, int]:
    m = re.match(r"^\s*(\d+)\s*x\s*(\d+)\s*$", str(job.get("source_resolution") or "").lower())
    return (int(m.group(1)), int(m.group(2))) if m else (0, 0)


def dvd_native_target_height(job: dict) -> int | None:
    """SD DVD material keeps its native 480/576 lines (reference :475-492)."""
    fn = str(job.get("filename") or "").strip().lower()
    codec = str(job.get("source_codec") or "").strip().lower()
    w, h = source_dimensions(job)
    dvd_path = fn.startswith(("dvd/", "movies/")) or "/dvd/" in fn or "/movies/" in fn
    if not dvd_path or not (0 < w <= 720 and 0 < h <= 576) or (codec and codec != "mpeg2video"):
        return None
    return 480 if h <= 480 else 576


def effective_target_height(job: dict) -> tuple[int, bool]:
    dvd = dvd_native_target_height(job)
    if dvd:
        return dvd, True
    return normalize_target_height(job.get("target_height")), False


def output_geometry(src_w: int, src_h: int, target_h: int) -> tuple[int, int]:
    """``scale=-2:H`` semantics: height H, aspect-preserving even width.  Never upscales
    (an upscale buys no quality and costs encode time); odd sources are cropped to even."""
    if src_w <= 0 or src_h <= 0:
        raise ValueError("unknown source geometry")
    h = min(int(target_h), src_h) & ~1
    w = int(round(src_w * h / src_h / 2.0)) * 2
    return max(2, w), max(2, h)


def disk_free_bytes(path: str) -> int:
    try:
        ensure_dirs(path)
        return int(shutil.disk_usage(path).free)
    except OSError:
        return -1


def host_from_endpoint(endpoint: str) -> str:
    raw = re.sub(r"^https?://", "", str(endpoint or "").strip(), flags=re.IGNORECASE)
    return raw.split("/", 1)[0].split(":", 1)[0].strip().lower()


def load_settings() -> dict:
    return get_settings()
