"""Worker environment configuration (reference worker/tasks.py:31-80).

Same variable names as the reference where the concept survives (paths, TTLs, HTTP port,
heartbeat interval, retry caps); the VA-API / ffmpeg knobs are replaced by the engine's
(`VEM_QP` keeps its meaning: the constant QP of CQP mode).
"""
from __future__ import annotations

import os
import socket


def env(name: str, default: str = "") -> str:
    v = os.environ.get(name)
    return default if v is None or v == "" else v


def _int(name: str, default: int) -> int:
    try:
        return int(env(name, str(default)))
    except ValueError:
        return default


def _float(name: str, default: float) -> float:
    try:
        return float(env(name, str(default)))
    except ValueError:
        return default


class WorkerConfig:
    """Read at construction so tests can patch the environment and rebuild."""

    def __init__(self):
        self.worker_name = env("HOSTNAME") or socket.gethostname()
        self.project_root = env("PROJECT_ROOT", "/projects")
        self.nfs_project_root = env("NFS_PROJECT_ROOT", "/library/.thinvids-projects")
        self.watch_root = env("WATCH_ROOT", "/watch")
        self.source_media_root = env("SOURCE_MEDIA_ROOT", "/source_media")
        self.library_root = env("LIBRARY_ROOT", "/library")
        self.metrics_ttl_sec = _int("TTL_SEC", 15)
        self.metrics_grace_sec = _int("TTL_GRACE_SEC", 5)
        self.http_bind_host = env("MASTER_HTTP_BIND", "0.0.0.0")
        self.http_port = _int("MASTER_HTTP_PORT", 8000)
        self.http_advertise = env("MASTER_HTTP_ADVERTISE", "")  # host[:port] others use to reach us
        self.allowed_target_heights = (360, 480, 576, 720, 1080, 1440, 2160)
        self.default_target_height = _int("VEM_DEFAULT_TARGET_HEIGHT", 1080)
        self.qp = _int("VEM_QP", 27)
        self.rc_mode = env("VEM_RC_MODE", "CQP").upper()
        self.part_failure_max_retries = _int("PART_FAILURE_MAX_RETRIES", 5)
        self.segment_io_idle_timeout_sec = max(30, _int("SEGMENT_IO_IDLE_TIMEOUT_SEC", 900))
        self.job_heartbeat_interval_sec = max(2.0, _float("JOB_HEARTBEAT_INTERVAL_SEC", 15))
        self.stitch_wait_parts_total_sec = _float("STITCH_WAIT_PARTS_TOTAL_SEC", 300)
        self.stitch_stable_sec = _float("STITCH_STABLE_SEC", 0.8)
        self.stitch_poll_sec = _float("STITCH_POLL_SEC", 0.5)
        self.encode_stitcher_wait_sec = _float("ENCODE_STITCHER_WAIT_SEC", 60)
        self.http_timeout_sec = _float("PART_HTTP_TIMEOUT_SEC", 120)
        # MI355X engine: GOP-chunks per batched launch and the encode consumer's batch window
        self.engine_batch = _int("TV_ENGINE_BATCH", 8)
        self.encode_batch_tasks = _int("TV_ENCODE_BATCH_TASKS", 8)


_cfg: WorkerConfig | None = None


def get_config(reload: bool = False) -> WorkerConfig:
    global _cfg
    if _cfg is None or reload:
        _cfg = WorkerConfig()
    return _cfg
