"""Global settings: store hash ``global:settings`` merged over defaults, cached 10 s
(reference common.py:168-229).  Same keys and defaults as the reference so an existing
thinvids settings hash keeps its meaning; the GPU engine adds ``tv_*`` knobs.
"""
from __future__ import annotations

import os
import threading
import time

from ..store import get_store

SETTINGS_KEY = "global:settings"
LEGACY_SETTINGS_KEY = "settings:global"
CACHED_SETTINGS_TTL = float(os.environ.get("CACHED_SETTINGS_TTL", "10"))

DEFAULT_SETTINGS: dict[str, str] = {
    # reference keys (common.py:173-191)
    "suspend_enabled": "0",
    "suspend_idle_sec": "300",
    "suspend_idle_cpu_pct_max": "15",
    "suspend_gc_enabled": "0",
    "max_source_file_size_gb": "15",
    "av1_check_enabled": "1",
    "use_nfs_for_all_files": "0",
    "use_direct_source_for_all_files": "0",
    "low_disk_direct_enabled": "1",
    "low_disk_min_free_gb": "20",
    "target_segment_mb": "10",
    "large_file_behavior": "direct",
    "default_target_height": "1080",
    "max_active_jobs": "2",
    "pipeline_worker_count": "4",
    "pipeline_drain_ratio_to_start_next": "0.75",
    "pipeline_min_idle_workers_to_start_next": "4",
    # MI355X engine knobs
    "tv_codec": "hevc",
    "tv_qp": "27",
    "tv_rc": "cqp",
    "tv_gop": "64",
    "tv_search_range": "64",
    "tv_deblock": "1",
    "tv_sao": "1",
    "tv_bframes": "1",  # hierarchical-B mini-GOP (1 = I P P P; 2/4/8/16: B pictures, tv/gop.h)
    "tv_segment_frames": "0",  # 0 = derive from target_segment_mb
    "tv_bitrate_kbps": "0",  # tv_rc=2pass / abr target
    "tv_vbv_maxrate_kbps": "0",  # tv_rc=abr: VBV peak rate (0: no VBV)
    "tv_vbv_bufsize_kbit": "0",  # tv_rc=abr: VBV decoder buffer
    "tv_crf": "27",  # tv_rc=crf quality level
    "tv_scenecut": "1",  # IDR (closed-GOP restart) at detected scene cuts
    "tv_ladder": "",  # e.g. "2160,1440,1080,720,480": one MP4 per rung (ABR fan-out)
    # node executor (one rank per GPU, RCCL data plane) — used when one is alive
    "tv_node_executor": "1",
    "tv_node_segment_frames": "256",
    "tv_node_mode": "direct",  # direct (each rank reads its range) | scatter (rank 0 -> xGMI)
    "tv_node_batch": "8",  # segments claimed per rank per batched launch
}

_cache = {"ts": 0.0, "data": {}}
_lock = threading.Lock()


def as_bool(x, default: bool = False) -> bool:
    if x is None:
        return default
    return str(x).strip().lower() in ("1", "true", "yes", "on", "y", "t")


def as_int(x, default: int = 0) -> int:
    try:
        return int(float(x))
    except (TypeError, ValueError):
        return default


def as_float(x, default: float = 0.0) -> float:
    try:
        return float(x)
    except (TypeError, ValueError):
        return default


def get_settings(store=None) -> dict[str, str]:
    """Defaults overlaid by the stored hash (legacy mirror first, primary wins)."""
    now = time.time()
    with _lock:
        if now - _cache["ts"] < CACHED_SETTINGS_TTL and _cache["data"]:
            return dict(_cache["data"])
    st = store or get_store()
    merged = dict(DEFAULT_SETTINGS)
    try:
        merged.update(st.hgetall(LEGACY_SETTINGS_KEY) or {})
        merged.update(st.hgetall(SETTINGS_KEY) or {})
    except Exception:  # store unavailable: serve defaults (reference bug common.py:217 fixed)
        merged = dict(DEFAULT_SETTINGS)
    with _lock:
        _cache["ts"] = now
        _cache["data"] = merged
    return dict(merged)


def invalidate_settings_cache() -> None:
    with _lock:
        _cache["ts"] = 0.0
        _cache["data"] = {}


def save_settings(values: dict, store=None) -> None:
    st = store or get_store()
    clean = {k: str(v) for k, v in values.items()}
    st.hset(SETTINGS_KEY, mapping=clean)
    st.hset(LEGACY_SETTINGS_KEY, mapping=clean)  # mirror (reference manager/app.py:1884-1886)
    invalidate_settings_cache()
