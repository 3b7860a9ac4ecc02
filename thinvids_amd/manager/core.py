"""Manager control logic (reference manager/app.py).

* node discovery / role assignment (C19, C20)            — reference :49-148
* job index with pruning and periodic SCAN reindex (C26) — :919-951
* admission policy (C23) and source probe (C27)          — :872-917, :2120-2220
* pipeline scheduler with the drain-ratio capacity model (C24) and the heartbeat
  watchdog (C25), both under the ``pipeline:scheduler:lock``  — :1057-1494
* warm-up & launch (C21) and power control: WOL / reboot (C22) — :277-377, :2907-3011

The capacity model counts **GPUs** as encoders: an agent publishes ``gpu_count`` in its
``metrics:node:<host>`` hash, and the idle-encoder estimate is in GPUs (one encode
consumer per GPU).  Role names, keys and job-hash fields are the reference's.
"""
from __future__ import annotations

import json
import logging
import os
import socket
import subprocess
import threading
import time
import uuid

from ..common import (JOBS_INDEX_KEY, Status, as_bool, as_float, as_int, emit_activity, get_settings, pass_field,
                      is_base_job_key, natural_host_key)
from ..models import media
from ..store import get_store

log = logging.getLogger("thinvids.manager")

DIRECT_SOURCE_REQUIRED_CODECS = {"vc1", "vc-1", "wmv3"}
DISABLED_NODES_KEY = "nodes:disabled"
PIPELINE_QUEUE_ACTION_TRANSCODE = "TRANSCODE"
PIPELINE_QUEUE_ACTION_STAMP = "STAMP"
PIPELINE_ACTIVE_JOB_KEY = "pipeline:active_job"  # legacy single-job string
PIPELINE_ACTIVE_JOBS_KEY = "pipeline:active_jobs"
PIPELINE_SCHED_LOCK_KEY = "pipeline:scheduler:lock"
PIPELINE_NODE_ROLES_KEY = "pipeline:node_roles"
PIPELINE_NODE_ROLES_META_KEY = "pipeline:node_roles:meta"


def _env_int(name, default, lo=None):
    v = as_int(os.environ.get(name), default)
    return max(lo, v) if lo is not None else v


def _env_float(name, default, lo=None):
    v = as_float(os.environ.get(name), default)
    return max(lo, v) if lo is not None else v


class ManagerConfig:
    def __init__(self):
        self.active_window_sec = _env_int("ACTIVE_WINDOW_SEC", 5)
        self.cluster_warmup_sec = _env_int("CLUSTER_WARMUP_SEC", 60)
        self.min_warmup_workers = _env_int("MIN_WARMUP_WORKERS", 3)
        self.watch_root = os.environ.get("WATCH_ROOT", "/watch")
        self.source_media_root = os.environ.get("SOURCE_MEDIA_ROOT", "/source_media")
        self.library_root = os.environ.get("LIBRARY_ROOT", "/library")
        self.config_root = os.environ.get("CONFIG_ROOT", "/config")
        self.processed_file = os.environ.get("PROCESSED_FILE", os.path.join(self.config_root, "processed.log"))
        self.watcher_service = os.environ.get("WATCHER_SERVICE", "thinvids_watcher.service")
        self.watcher_env_file = os.environ.get("WATCHER_ENV_FILE", os.path.join(self.config_root, "watcher.env"))
        self.local_project_root = os.environ.get("PROJECT_ROOT", "/projects")
        self.nfs_project_root = os.environ.get("NFS_PROJECT_ROOT", "/library/.thinvids-projects")
        self.sched_lock_ttl = _env_int("PIPELINE_SCHED_LOCK_TTL_SEC", 30, 5)
        self.sched_poll_sec = _env_float("PIPELINE_SCHED_POLL_SEC", 2, 0.05)
        self.watchdog_enabled = as_bool(os.environ.get("JOB_WATCHDOG_ENABLED", "1"), True)
        self.watchdog_poll_sec = _env_float("JOB_WATCHDOG_POLL_SEC", 15, 0.05)
        self.starting_stall_sec = _env_int("JOB_STARTING_STALL_SEC", 300, 1)
        self.running_stall_sec = _env_int("JOB_RUNNING_STALL_SEC", 900, 1)
        self.stamping_stall_sec = _env_int("JOB_STAMPING_STALL_SEC", 900, 1)
        self.reindex_sec = _env_float("JOB_INDEX_REINDEX_SEC", 60, 0.0)
        self.allowed_target_heights = (480, 576, 720, 1080, 1440, 2160)
        self.default_target_height = 1080
        self.wol_port = _env_int("WOL_PORT", 9)
        self.wol_broadcast = os.environ.get("WOL_BROADCAST", "255.255.255.255")
        self.manager_hostname = os.environ.get("MANAGER_HOSTNAME", socket.gethostname())


CFG = ManagerConfig()


def reload_config() -> ManagerConfig:
    global CFG
    CFG = ManagerConfig()
    return CFG


def _st(store=None):
    return store or get_store()


def _f(v, d=0.0) -> float:
    return as_float(v, d)


# ------------------------------------------------------------------ nodes (C19)
def get_all_nodes(store=None) -> list[dict]:
    st = _st(store)
    disabled = set(st.smembers(DISABLED_NODES_KEY) or [])
    out = []
    for host, mac in (st.hgetall("nodes:mac") or {}).items():
        host, mac = (host or "").strip(), (mac or "").strip()
        if host and mac:
            out.append({"hostname": host, "mac": mac, "disabled": host in disabled})
    return sorted(out, key=lambda n: natural_host_key(n["hostname"]))


def get_active_nodes(store=None) -> list[dict]:
    st = _st(store)
    nodes = [n for n in get_all_nodes(st) if not n["disabled"]]
    if not nodes:
        return []
    cutoff = int(time.time()) - CFG.active_window_sec
    p = st.pipeline()
    for n in nodes:
        p.hmget(f"metrics:node:{n['hostname']}", ["ts", "gpu_count"])
    out = []
    for n, (ts, gpus) in zip(nodes, p.execute()):
        if int(_f(ts)) >= cutoff:
            out.append({**n, "gpu_count": max(1, as_int(gpus, 1))})
    return out


def active_hostnames(store=None) -> list[str]:
    return [n["hostname"] for n in get_active_nodes(store)]


# ------------------------------------------------------------------ roles (C20)
def pipeline_runtime_settings(settings: dict | None = None) -> dict:
    s = settings or get_settings()
    pwc = max(2, as_int(s.get("pipeline_worker_count"), as_int(os.environ.get("PIPELINE_WORKER_COUNT"), 4)))
    return {
        "max_active_jobs": max(1, pwc // 2),
        "effective_max_active_jobs": max(1, pwc // 2),
        "pipeline_worker_count": pwc,
        "pipeline_drain_ratio_to_start_next": min(1.0, max(0.0, as_float(
            s.get("pipeline_drain_ratio_to_start_next"), 0.75))),
        "pipeline_min_idle_workers_to_start_next": max(1, as_int(
            s.get("pipeline_min_idle_workers_to_start_next"), 4)),
    }


def assign_pipeline_node_roles(settings: dict | None = None, store=None) -> dict:
    """First `pipeline_worker_count` enabled nodes (natural order) -> 'pipeline', rest ->
    'encode'.  Every node still runs an encode consumer per GPU."""
    st = _st(store)
    rt = pipeline_runtime_settings(settings)
    enabled = [n for n in get_all_nodes(st) if not n["disabled"]]
    pipe_hosts = {n["hostname"] for n in enabled[:rt["pipeline_worker_count"]]}
    roles = {n["hostname"]: ("pipeline" if n["hostname"] in pipe_hosts else "encode") for n in enabled}
    stale = [h for h in (st.hkeys(PIPELINE_NODE_ROLES_KEY) or []) if h not in roles]
    p = st.pipeline()
    if stale:
        p.hdel(PIPELINE_NODE_ROLES_KEY, *stale)
    if roles:
        p.hset(PIPELINE_NODE_ROLES_KEY, mapping=roles)
    p.hset(PIPELINE_NODE_ROLES_META_KEY, mapping={
        "updated_at": str(time.time()), "max_active_jobs": str(rt["max_active_jobs"]),
        "effective_max_active_jobs": str(rt["effective_max_active_jobs"]), "active_job_limit_enforced": "0",
        "pipeline_worker_count": str(rt["pipeline_worker_count"]),
        "pipeline_required_for_max_active": str(rt["max_active_jobs"] * 2)})
    p.execute()
    return roles


# -------------------------------------------------------------- job index (C26)
_index_scan_ts = 0.0
_index_guard = threading.Lock()


def job_index_keys(store=None) -> list[str]:
    global _index_scan_ts
    st = _st(store)
    raw = set(st.smembers(JOBS_INDEX_KEY) or [])
    bad = [k for k in raw if not is_base_job_key(k)]
    if bad:
        st.srem(JOBS_INDEX_KEY, *bad)
    keys = {k for k in raw if is_base_job_key(k)}
    legacy = (st.get(PIPELINE_ACTIVE_JOB_KEY) or "").strip()
    if legacy:
        keys.add(f"job:{legacy}")
    t = time.time()
    if not keys or t - _index_scan_ts >= CFG.reindex_sec:
        with _index_guard:
            scanned = [k for k in st.scan_iter("job:*") if is_base_job_key(k)]
            if scanned:
                keys.update(scanned)
                st.sadd(JOBS_INDEX_KEY, *scanned)
            _index_scan_ts = time.time()
    return sorted(keys)


def load_jobs(keys: list[str], store=None) -> list[tuple[str, dict]]:
    st = _st(store)
    p = st.pipeline()
    for k in keys:
        p.hgetall(k)
    return [(k, j) for k, j in zip(keys, p.execute()) if j]


def job_status(job: dict) -> Status | None:
    raw = str(job.get("status") or "").strip().upper()
    if raw == "COMPLETED":  # legacy
        return Status.DONE
    try:
        return Status.parse(raw)
    except Exception:
        return None


# ------------------------------------------------------- policy + probe (C23/C27)
def evaluate_job_policy(details: dict, settings: dict):
    """-> (rejection_reason, message, scratch_mode, scratch_root, processing_mode)."""
    max_gb = as_float(settings.get("max_source_file_size_gb", 15), 15.0)
    large = str(settings.get("large_file_behavior", "direct") or "direct").strip().lower()
    if large not in ("reject", "nfs", "direct"):
        large = "reject"
    size = as_int(details.get("source_file_size"), 0)
    codec = str(details.get("source_codec") or "").strip().lower()
    mode = "direct" if as_bool(settings.get("use_direct_source_for_all_files")) else "split"
    if as_bool(settings.get("av1_check_enabled", "1"), True) and codec in ("av1", "av01"):
        return ("av1_rejected", "AV1 source rejected by global setting (av1_check_enabled).", "local",
                CFG.local_project_root, "split")
    nfs = as_bool(settings.get("use_nfs_for_all_files"))
    scratch_mode, scratch_root = ("nfs", CFG.nfs_project_root) if nfs else ("local", CFG.local_project_root)
    if codec in DIRECT_SOURCE_REQUIRED_CODECS:
        return (None, None, scratch_mode, scratch_root, "direct")
    limit = int(max_gb * 1024 ** 3)
    if limit > 0 and size > limit:
        if large == "nfs":
            return (None, None, "nfs", CFG.nfs_project_root, mode)
        if large == "direct":
            return (None, None, scratch_mode, scratch_root, "direct")
        return ("size_limit", f"Source file too large: {size / 1024 ** 3:.1f} GiB > {max_gb:g} GiB limit",
                scratch_mode, scratch_root, "split")
    return (None, None, scratch_mode, scratch_root, mode)


def get_video_details(path: str) -> dict:
    """Probe a source (our own probe replaces ffprobe; reference :2120-2220)."""
    try:
        info = media.probe(path)
    except Exception as e:
        size = os.path.getsize(path) if os.path.exists(path) else 0
        return {"source_codec": "unknown", "source_resolution": "", "source_duration": "0", "source_fps": "0",
                "source_file_size": size, "total_frames": 0, "streams_json": "[]", "probe_error": str(e)[:500]}
    groups = {"video": [], "audio": [], "subtitle": []}
    for s in info["streams"]:
        kind = s.get("codec_type")
        if kind not in groups:
            continue
        tags = s.get("tags") or {}
        e = {"index": int(s.get("index", 0)), "codec": s.get("codec_name") or "", "title": tags.get("title") or "",
             "language": tags.get("language") or "", "disposition_default": len(groups[kind]) == 0}
        if kind == "video":
            e.update(width=int(s.get("width") or 0), height=int(s.get("height") or 0), fps=info["fps"],
                     nb_frames=info["frames"])
        elif kind == "audio":
            e.update(channels=int(s.get("channels") or 0), sample_rate=int(s.get("sample_rate") or 0))
        groups[kind].append(e)
    # first English audio stream, else the first (reference :2193-2198)
    a_sel = next((i for i, a in enumerate(groups["audio"]) if _is_english(a["language"])), 0)
    return {"source_codec": info["codec"], "source_resolution": info["resolution"],
            "source_width": info["width"], "source_height": info["height"],
            "source_duration": f"{info['duration']:.3f}", "source_fps": f"{info['fps']:.3f}",
            "source_fps_num": info["fps_num"], "source_fps_den": info["fps_den"],
            "source_file_size": info["size"], "source_bitrate_kbps": info["bitrate_kbps"],
            "total_frames": info["frames"], "streams_json": json.dumps(groups), "selected_v_stream": 0,
            "selected_a_stream": a_sel}


def _is_english(lang: str) -> bool:
    lang = (lang or "").strip().lower()
    return lang in ("eng", "en", "english") or lang.startswith("en-")


# ------------------------------------------------------------- scheduler (C24)
def _done_ratio(job: dict) -> float:
    total, done = as_int(job.get("parts_total")), as_int(pass_field(job, "parts_done"))
    return 0.0 if total <= 0 else min(1.0, max(0.0, done / total))


def _remaining(job: dict) -> int:
    total, done = as_int(job.get("parts_total")), as_int(pass_field(job, "parts_done"))
    return max(0, total - done) if total > 0 else 0


def active_job_pipeline_slots(job: dict) -> int:
    s = job_status(job)
    if s == Status.STAMPING:
        return 1
    if s == Status.STARTING or s is None:
        return 2
    if s == Status.RUNNING and as_int(job.get("parts_total")) > 0 and as_int(job.get("segment_progress")) >= 100:
        return 1  # the segmenter returned to the pool; only the stitcher is held
    return 2


def active_job_is_shareable(job: dict, rt: dict) -> bool:
    if job_status(job) != Status.RUNNING:
        return False
    if as_int(job.get("parts_total")) <= 0 or as_int(job.get("segment_progress")) < 100:
        return False
    return _done_ratio(job) >= rt["pipeline_drain_ratio_to_start_next"]


def can_dispatch_next_job(active_jobs: list[dict], store=None) -> tuple[bool, str]:
    st = _st(store)
    rt = pipeline_runtime_settings()
    if not active_jobs:
        return True, "no_active_jobs"
    if any(not active_job_is_shareable(j, rt) for j in active_jobs):
        return False, "active_job_not_shareable"
    roles = assign_pipeline_node_roles(None, st)
    nodes = get_active_nodes(st)
    if not nodes:
        return False, "no_active_workers"
    active_pipeline = sum(1 for n in nodes if roles.get(n["hostname"]) == "pipeline")
    used = sum(active_job_pipeline_slots(j) for j in active_jobs)
    if active_pipeline < used + 2:
        return False, (f"insufficient_pipeline_workers active_pipeline={active_pipeline} used={used} "
                       f"need={used + 2} configured={rt['pipeline_worker_count']}")
    gpus = sum(n["gpu_count"] for n in nodes)
    capacity = max(0, gpus - used)
    remaining = sum(_remaining(j) for j in active_jobs)
    idle = max(0, capacity - remaining)
    need = rt["pipeline_min_idle_workers_to_start_next"]
    if idle < need:
        return False, f"insufficient_idle_workers idle={idle} need={need} encoder_capacity={capacity} " \
                      f"reserved_pipeline_nodes={used}"
    return True, f"idle_workers={idle} remaining_encode_parts={remaining} encoder_capacity={capacity}"


def acquire_sched_lock(store=None) -> str | None:
    token = f"{uuid.uuid4().hex}:{time.time()}"
    return token if _st(store).set(PIPELINE_SCHED_LOCK_KEY, token, nx=True, ex=CFG.sched_lock_ttl) else None


def release_sched_lock(token: str, store=None) -> None:
    st = _st(store)
    if st.get(PIPELINE_SCHED_LOCK_KEY) == token:
        st.delete(PIPELINE_SCHED_LOCK_KEY)


def clear_active_job_refs(job_id: str, store=None) -> None:
    st = _st(store)
    st.srem(PIPELINE_ACTIVE_JOBS_KEY, job_id)
    if (st.get(PIPELINE_ACTIVE_JOB_KEY) or "") == job_id:
        st.delete(PIPELINE_ACTIVE_JOB_KEY)


def active_pipeline_jobs(store=None) -> list[dict]:
    """Members of ``pipeline:active_jobs`` that are still active; prunes the rest."""
    st = _st(store)
    out = []
    for jid in sorted(st.smembers(PIPELINE_ACTIVE_JOBS_KEY) or []):
        job = st.hgetall(f"job:{jid}") or {}
        if job_status(job) in (Status.STARTING, Status.RUNNING, Status.STAMPING):
            job.setdefault("job_id", jid)
            out.append(job)
        else:
            clear_active_job_refs(jid, st)
    return out


def reserve_next_waiting_job(store=None) -> dict | None:
    st = _st(store)
    active = active_pipeline_jobs(st)
    known = {j.get("job_id") for j in active}
    cands = []
    for key, job in load_jobs(job_index_keys(st), st):
        s = job_status(job)
        jid = (job.get("job_id") or key.split(":", 1)[1]).strip()
        if not jid or not (job.get("filename") or "").strip():
            continue
        if s in (Status.STARTING, Status.RUNNING, Status.STAMPING) and jid not in known:
            st.sadd(PIPELINE_ACTIVE_JOBS_KEY, jid)  # adopt orphaned active jobs
            active.append({**job, "job_id": jid})
            known.add(jid)
        elif s == Status.WAITING:
            action = (job.get("queue_action") or PIPELINE_QUEUE_ACTION_TRANSCODE).strip().upper()
            if action not in (PIPELINE_QUEUE_ACTION_TRANSCODE, PIPELINE_QUEUE_ACTION_STAMP):
                action = PIPELINE_QUEUE_ACTION_TRANSCODE
            wait = _f(job.get("waiting_at")) or _f(job.get("started_at")) or _f(job.get("created_at"))
            cands.append((wait, _f(job.get("created_at")), jid, key, job, action))
    if not cands:
        return None
    ok, reason = can_dispatch_next_job(active, st)
    if not ok:
        t = str(time.time())
        for *_, key, _job, _a in cands:
            st.hset(key, mapping={"queue_blocked_reason": reason, "queue_blocked_active_jobs": str(len(active)),
                                  "queue_blocked_at": t})
        return None
    cands.sort(key=lambda c: (c[0], c[1], c[2]))
    _, _, jid, key, job, action = cands[0]
    token = uuid.uuid4().hex
    t = time.time()
    mapping = {"status": (Status.STAMPING if action == PIPELINE_QUEUE_ACTION_STAMP else Status.STARTING).value,
               "queue_reserved_at": str(t),
               "queue_dispatch_attempts": str(as_int(job.get("queue_dispatch_attempts")) + 1),
               "pipeline_run_token": token, "last_heartbeat_at": str(t),
               "last_heartbeat_stage": "stamp_dispatch" if action == PIPELINE_QUEUE_ACTION_STAMP else "dispatch",
               "last_heartbeat_host": "manager", "last_heartbeat_note": action,
               "queue_blocked_reason": "", "queue_blocked_active_jobs": "", "queue_blocked_at": ""}
    if _f(job.get("started_at")) <= 0:
        mapping["started_at"] = str(t)
    st.hset(key, mapping=mapping)
    st.sadd(PIPELINE_ACTIVE_JOBS_KEY, jid)
    return {"job_id": jid, "job_key": key, "filename": job.get("filename"), "action": action, "run_token": token,
            "capacity_reason": reason}


def wait_for_workers(min_count: int, timeout_sec: float, on_tick=None, store=None) -> list[str]:
    deadline = time.time() + max(0.0, timeout_sec)
    best: list[str] = []
    while True:
        cur = active_hostnames(store)
        if on_tick:
            on_tick(cur, best, deadline)
        if len(cur) >= min_count:
            return cur
        if len(cur) > len(best):
            best = cur
        if time.time() >= deadline:
            return best
        time.sleep(min(1.0, max(0.05, deadline - time.time())))


def launch_after_warmup(job_key: str, job_id: str, filename: str, run_token: str, store=None) -> None:
    """WOL, wait for heartbeats when nothing is up, then enqueue `transcode` (C21)."""
    from ..worker import tasks

    st = _st(store)
    job = st.hgetall(job_key) or {}
    if run_token and job.get("pipeline_run_token") != run_token:
        return
    t0 = time.time()
    st.hset(job_key, mapping={"last_heartbeat_at": str(t0), "last_heartbeat_stage": "warmup_start",
                              "last_heartbeat_host": "manager", "last_heartbeat_note": "waking workers",
                              "manager_warmup_started_at": str(t0)})
    try:
        wake_all_nodes(st)
    except Exception as e:
        log.warning("wake_all_nodes failed: %s", e)
    seen = active_hostnames(st)
    if not seen:
        wanted = max(1, min(CFG.min_warmup_workers, max(1, len(get_all_nodes(st)))))

        def tick(cur, best, deadline):
            st.hset(job_key, mapping={"last_heartbeat_at": str(time.time()), "last_heartbeat_stage": "warmup_wait",
                                      "last_heartbeat_host": "manager",
                                      "last_heartbeat_note": f"active={len(cur)} wanted={wanted} "
                                                             f"remaining={max(0, int(deadline - time.time()))}s"})
        seen = wait_for_workers(wanted, CFG.cluster_warmup_sec, tick, st)
    job = st.hgetall(job_key) or {}
    if run_token and job.get("pipeline_run_token") != run_token:
        return
    src = (job.get("input_path") or "").strip() or os.path.join(CFG.watch_root, (filename or "").lstrip("/"))
    st.hset(job_key, mapping={"warmup_workers_json": json.dumps(seen), "warmup_worker_count": len(seen),
                              "warmup_wait_s": CFG.cluster_warmup_sec, "input_path": src,
                              "last_heartbeat_at": str(time.time()), "last_heartbeat_stage": "warmup_complete",
                              "last_heartbeat_host": "manager", "last_heartbeat_note": "launching transcode task",
                              "manager_warmup_completed_at": str(time.time())})
    tid = tasks.transcode(job_id, run_token)
    st.hset(job_key, mapping={"manager_launch_submitted_at": str(time.time()), "manager_launch_task_id": tid})


def launch_reserved_job(reserved: dict | None, store=None) -> None:
    if not reserved:
        return
    from ..worker import tasks

    st = _st(store)
    jid, key = reserved["job_id"], reserved["job_key"]
    try:
        if reserved["action"] == PIPELINE_QUEUE_ACTION_STAMP:
            tasks.stamp(jid, reserved["run_token"])
        else:
            emit_activity(f'Started "{display_title(reserved["filename"])}"', job_id=jid,
                          filename=reserved["filename"], stage="start", source="manager", store=st)
            launch_after_warmup(key, jid, reserved["filename"], reserved["run_token"], st)
    except Exception as e:
        log.exception("[%s] reserved launch failed", jid)
        st.hset(key, mapping={"status": Status.FAILED.value, "error": str(e), "ended_at": str(time.time())})
        clear_active_job_refs(jid, st)


def dispatch_next_waiting_job(store=None) -> bool:
    st = _st(store)
    token = acquire_sched_lock(st)
    if not token:
        return False
    try:
        reserved = reserve_next_waiting_job(st)
    finally:
        release_sched_lock(token, st)
    if not reserved:
        return False
    launch_reserved_job(reserved, st)
    return True


def queue_job_for_dispatch(job_key: str, action: str = PIPELINE_QUEUE_ACTION_TRANSCODE, waiting_at=None,
                           store=None) -> None:
    _st(store).hset(job_key, mapping={"status": Status.WAITING.value, "queue_action": action,
                                      "waiting_at": str(waiting_at or time.time())})


# -------------------------------------------------------------- watchdog (C25)
def _stall_timeout(s: Status) -> float:
    return {Status.STARTING: CFG.starting_stall_sec, Status.RUNNING: CFG.running_stall_sec,
            Status.STAMPING: CFG.stamping_stall_sec}.get(s, 0)


def normalize_watchdog_state(store=None) -> bool:
    """Back-fill missing heartbeat fields of queued/active jobs (:1321-1377)."""
    from ..worker.helpers import host_from_endpoint

    st = _st(store)
    changed = False
    for key, job in load_jobs(job_index_keys(st), st):
        s = job_status(job)
        if s not in (Status.WAITING, Status.STARTING, Status.RUNNING, Status.STAMPING):
            continue
        ref = _f(job.get("started_at")) or _f(job.get("waiting_at")) or _f(job.get("created_at"))
        if s == Status.WAITING:
            ref = _f(job.get("waiting_at")) or _f(job.get("started_at")) or _f(job.get("created_at"))
        m = {}
        if _f(job.get("last_heartbeat_at")) <= 0 and ref > 0:
            m["last_heartbeat_at"] = str(ref)
        if not (job.get("last_heartbeat_stage") or "").strip():
            m["last_heartbeat_stage"] = "queue" if s == Status.WAITING else s.value.lower()
        if not (job.get("last_heartbeat_host") or "").strip():
            h = host_from_endpoint(job.get("master_host") or "") or ("manager" if s == Status.WAITING else "")
            if h:
                m["last_heartbeat_host"] = h
        if not (job.get("last_heartbeat_note") or "").strip() and s == Status.WAITING:
            m["last_heartbeat_note"] = (job.get("queue_action") or PIPELINE_QUEUE_ACTION_TRANSCODE).upper()
        if m:
            st.hset(key, mapping=m)
            changed = True
    return changed


def check_for_stalled_jobs(store=None) -> bool:
    st = _st(store)
    now = time.time()
    changed = normalize_watchdog_state(st)
    for key, job in load_jobs(job_index_keys(st), st):
        s = job_status(job)
        limit = _stall_timeout(s) if s else 0
        if limit <= 0:
            continue
        ref = _f(job.get("last_heartbeat_at")) or _f(job.get("started_at")) or _f(job.get("waiting_at")) \
            or _f(job.get("created_at"))
        if ref <= 0 or now - ref < limit:
            continue
        jid = (job.get("job_id") or key.split(":", 1)[1]).strip()
        stage = (job.get("last_heartbeat_stage") or s.value.lower()).strip()
        host = (job.get("last_heartbeat_host") or "").strip() or "unknown"
        stale = int(now - ref)
        reason = f"watchdog detected stalled job: no heartbeat for {stale}s during {stage}"
        st.hset(key, mapping={"status": Status.FAILED.value, "error": reason, "failed_stage": "watchdog",
                              "failed_worker": host, "ended_at": str(now), "stalled_stage": stage,
                              "stalled_detected_at": str(now)})
        clear_active_job_refs(jid, st)
        revoke_job_tasks(jid, st)
        emit_activity(f'Failed stalled job "{display_title(job.get("filename"))}" after {stale}s without '
                      f'heartbeat ({stage})', job_id=jid, filename=job.get("filename"), stage="watchdog",
                      source="manager", store=st)
        changed = True
    return changed


def revoke_job_tasks(job_id: str, store=None) -> int:
    """Revoke every queued task of a job (fixes reference :1407/:2680, which revoked the
    job id instead of task ids)."""
    from ..queue import get_encode_queue, get_pipeline_queue

    n = 0
    for q in (get_pipeline_queue(), get_encode_queue()):
        for msg in q.pending():
            args = msg.get("args") or []
            if (args and args[0] == job_id) or (msg.get("kwargs") or {}).get("job_id") == job_id:
                q.revoke_by_id(msg["id"])
                n += 1
    return n


def display_title(filename) -> str:
    base = os.path.basename(str(filename or "").strip())
    return os.path.splitext(base)[0] or base or "Unknown"


# ------------------------------------------------------------ loops (C24/C25/C32)
class Housekeeping:
    """Scheduler + watchdog threads (reference manager/housekeeping.py)."""

    def __init__(self, store=None):
        self.store = store
        self._stop = threading.Event()
        self._threads: list[threading.Thread] = []

    def _sched(self):
        while not self._stop.is_set():
            try:
                dispatch_next_waiting_job(self.store)
            except Exception:
                log.exception("scheduler tick failed")
            self._stop.wait(CFG.sched_poll_sec)

    def _watchdog(self):
        while not self._stop.is_set():
            try:
                st = _st(self.store)
                tok = acquire_sched_lock(st)
                if tok:
                    try:
                        changed = check_for_stalled_jobs(st)
                    finally:
                        release_sched_lock(tok, st)
                    if changed:
                        dispatch_next_waiting_job(st)
            except Exception:
                log.exception("watchdog tick failed")
            self._stop.wait(CFG.watchdog_poll_sec)

    def start(self) -> "Housekeeping":
        self._threads = [threading.Thread(target=self._sched, name="pipeline-scheduler", daemon=True)]
        if CFG.watchdog_enabled:
            self._threads.append(threading.Thread(target=self._watchdog, name="job-watchdog", daemon=True))
        for t in self._threads:
            t.start()
        return self

    def stop(self) -> None:
        self._stop.set()
        for t in self._threads:
            t.join(timeout=5)


# ------------------------------------------------------------ power control (C22)
def build_magic_packet(mac: str) -> bytes:
    hexmac = "".join(c for c in mac if c.isalnum())
    if len(hexmac) != 12:
        raise ValueError(f"bad MAC {mac!r}")
    return b"\xff" * 6 + bytes.fromhex(hexmac) * 16


def send_magic_udp(mac: str, repeats: int = 3) -> None:
    pkt = build_magic_packet(mac)
    with socket.socket(socket.AF_INET, socket.SOCK_DGRAM) as s:
        s.setsockopt(socket.SOL_SOCKET, socket.SO_BROADCAST, 1)
        for _ in range(repeats):
            s.sendto(pkt, (CFG.wol_broadcast, CFG.wol_port))


def wake_one_node(host: str, store=None) -> bool:
    mac = _st(store).hget("nodes:mac", host)
    if not mac:
        return False
    try:
        send_magic_udp(mac)
        return True
    except OSError as e:
        log.warning("WOL to %s failed: %s", host, e)
        return False


def wake_all_nodes(store=None) -> int:
    return sum(wake_one_node(n["hostname"], store) for n in get_all_nodes(store) if not n["disabled"])


def reboot_one_node(host: str) -> tuple[bool, str]:
    if host in (CFG.manager_hostname, socket.gethostname(), "localhost", "127.0.0.1"):
        return False, "refusing to reboot the manager itself"
    try:
        r = subprocess.run(["ssh", "-o", "BatchMode=yes", "-o", "ConnectTimeout=5", host, "sudo", "-n",
                            "systemctl", "reboot"], capture_output=True, text=True, timeout=20)
        return r.returncode == 0, (r.stderr or r.stdout or "").strip()[:500]
    except (OSError, subprocess.TimeoutExpired) as e:
        return False, str(e)


def reboot_all_nodes(store=None) -> dict:
    return {n["hostname"]: reboot_one_node(n["hostname"])[0] for n in get_all_nodes(store) if not n["disabled"]}
