"""Pure planning / policy helpers of the worker pipeline (unit-testable, no I/O).

* parts plan — GOP-aligned frame ranges (reference byte-size plan worker/tasks.py:974-1052
  and direct ranges :584-594, re-expressed in frames because this engine owns the GOP);
* processing-mode decision (reference :619-653);
* stitcher head-of-line redispatch policy (reference :1943-2026).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass, field

from ..common import as_bool, as_float, as_int


@dataclass
class PartsPlan:
    requested_parts: int
    effective_parts: int
    usable_encoder_workers: int
    frames_per_part: int
    ranges: list = field(default_factory=list)  # [(idx (1-based), start_frame, nframes)]


def parts_for_target_size(size_b: int, target_segment_bytes: int) -> int:
    size_b = int(size_b or 0)
    if size_b <= 0:
        return 0
    return max(1, int(math.ceil(size_b / max(1, int(target_segment_bytes or 1)))))


def plan_parts(nframes: int, usable_encoders: int, gop: int = 64, segment_frames: int = 0,
               size_b: int = 0, target_segment_mb: float = 0.0, est_bytes_per_frame: float = 0.0,
               min_frames: int = 8) -> PartsPlan:
    """Frame-range plan.  The requested part count comes from `segment_frames` (if set), else
    from the reference's target segment size applied to the *encoded* size estimate, else
    from the GOP length.  Like the reference, the count is raised to at least one part per
    usable encoder and otherwise rounded up to a multiple of them, so every GPU gets work."""
    nframes = max(0, int(nframes))
    if nframes == 0:
        return PartsPlan(0, 0, usable_encoders, 0, [])
    if segment_frames > 0:
        requested = math.ceil(nframes / segment_frames)
    elif target_segment_mb > 0 and est_bytes_per_frame > 0:
        requested = parts_for_target_size(int(nframes * est_bytes_per_frame), int(target_segment_mb * 1024 * 1024))
        requested = max(requested, math.ceil(nframes / max(gop, 1) / 64))  # never absurdly long
    else:
        requested = math.ceil(nframes / max(1, gop))
    requested = max(1, requested)
    eff = requested
    if usable_encoders > 0:
        eff = usable_encoders if requested <= usable_encoders else math.ceil(requested / usable_encoders) * usable_encoders
    eff = max(1, min(eff, max(1, nframes // max(1, min_frames))))
    fpp = math.ceil(nframes / eff)
    ranges = []
    start, idx = 0, 1
    while start < nframes:
        n = min(fpp, nframes - start)
        ranges.append((idx, start, n))
        start += n
        idx += 1
    return PartsPlan(requested, len(ranges), usable_encoders, fpp, ranges)


def resolve_processing_mode(job: dict, settings: dict, source_size_b: int, free_scratch_b: int | None) -> tuple[str, str]:
    """'split' (parts materialised in scratch, servable to remote encoders) or 'direct'
    (encoders read their frame range straight from the source).  Returns (mode, reason)."""
    requested = str(job.get("processing_mode") or "").strip().lower()
    if requested in ("split", "direct"):
        return requested, "job override"
    if as_bool(settings.get("use_direct_source_for_all_files")):
        return "direct", "global direct-source setting"
    src_origin = str(job.get("source_origin") or "")
    if src_origin == "source_media":
        return "split", "source_media path forces split"
    if as_bool(settings.get("low_disk_direct_enabled"), True) and free_scratch_b is not None:
        min_free = as_float(settings.get("low_disk_min_free_gb"), 20) * 1024 ** 3
        if free_scratch_b < max(min_free, source_size_b):
            return "direct", "low scratch disk"
    max_gb = as_float(settings.get("max_source_file_size_gb"), 15)
    if source_size_b > max_gb * 1024 ** 3 and str(settings.get("large_file_behavior", "direct")) == "direct":
        return "direct", "large source file"
    if str(job.get("source_codec") or "") == "synthetic":
        return "direct", "synthetic source (generated in place)"
    return "split", "default"


@dataclass
class StitchTunables:
    max_retries: int = as_int(os.environ.get("STITCH_MAX_RETRIES"), 3)
    retry_interval_sec: float = as_float(os.environ.get("STITCH_RETRY_INTERVAL_SEC"), 45)
    stall_before_retry_sec: float = as_float(os.environ.get("STITCH_STALL_BEFORE_RETRY_SEC"), 90)
    miss_min_age_sec: float = as_float(os.environ.get("STITCH_MISS_MIN_AGE_SEC"), 90)
    retry_window_ahead: int = as_int(os.environ.get("STITCH_RETRY_WINDOW_AHEAD"), 8)
    max_parallel_redispatch: int = as_int(os.environ.get("STITCH_MAX_PARALLEL_REDISPATCH"), 3)


def plan_redispatch(ready: set, total: int, segmented: int, now: float, last_change: float,
                    miss_seen: dict, retry_cnt: dict, retry_ts: dict, est_part_secs: float,
                    t: StitchTunables) -> tuple[list, list, bool]:
    """Head-of-line conservative retry.  Returns (newly_missing, to_retry, give_up)."""
    frontier = 0
    for i in range(1, total + 1):
        if i in ready:
            frontier = i
        else:
            break
    horizon = min(total, frontier + t.retry_window_ahead)
    if segmented > 0:
        horizon = min(horizon, segmented)
    window = [i for i in range(frontier + 1, horizon + 1) if i not in ready]
    newly = [i for i in window if i not in miss_seen]
    seen = dict(miss_seen)
    for i in newly:
        seen[i] = now
    stalled = (now - last_change) >= t.stall_before_retry_sec
    to_retry = []
    if stalled:
        for i in window:
            if len(to_retry) >= t.max_parallel_redispatch:
                break
            first = float(seen.get(i, 0) or 0)
            if first <= 0 or (now - first) < max(t.miss_min_age_sec, est_part_secs * 1.5):
                continue
            if int(retry_cnt.get(i, 0) or 0) >= t.max_retries:
                continue
            if (now - float(retry_ts.get(i, 0) or 0)) < t.retry_interval_sec:
                continue
            to_retry.append(i)
    give_up = False
    for i in window:
        cnt = int(retry_cnt.get(i, 0) or 0)
        if cnt >= t.max_retries:
            last = max(float(retry_ts.get(i, 0) or 0), float(seen.get(i, 0) or 0))
            if now - last > max(2 * est_part_secs, t.stall_before_retry_sec):
                give_up = True
                break
    return newly, to_retry, give_up
