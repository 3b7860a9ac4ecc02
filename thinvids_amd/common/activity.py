"""Activity log (reference common.py:276-425).

* ``activity:log`` — global capped list (newest first) of JSON events for the UI feed;
* ``joblog:<id>`` — per-job append-only compact text lines
  ``HH:MM:SS [LABEL] jobid8 [name] [part N] [Nms]`` with LABEL in
  START/SEGMENT/ENCODE/STITCH/FINISH/ERROR.
"""
from __future__ import annotations

import json
import os
import re
import time
from datetime import datetime

from ..store import get_store

ACTIVITY_LOG_KEY = "activity:log"
ACTIVITY_LOG_MAX = int(os.environ.get("ACTIVITY_LOG_MAX", "2000"))
ACTIVITY_JOB_LOG_MAX = int(os.environ.get("ACTIVITY_JOB_LOG_MAX", "50000"))

_PART_RE = re.compile(r"\bpart\s+(\d+)\b", re.IGNORECASE)
_MS_RE = re.compile(r"\b(\d+)ms\b", re.IGNORECASE)
_NAME_RE = re.compile(r'"([^"]+)"')


def activity_label(stage: str, message: str) -> str:
    st = (stage or "").strip().lower()
    msg = (message or "").strip().lower()
    if st == "rejected" or "error" in st or " failed" in msg or "error" in msg or "rejected" in msg:
        return "ERROR"
    if st in ("stitch_complete", "write") or msg.startswith('writing "'):
        return "FINISH"
    for prefix, label in (("stitch", "STITCH"), ("encode", "ENCODE")):
        if st.startswith(prefix):
            return label
    if st.startswith("segment") or st == "split":
        return "SEGMENT"
    return "START"


def format_activity_line(ev: dict) -> str:
    try:
        stamp = datetime.fromtimestamp(float(ev.get("ts") or time.time())).strftime("%H:%M:%S")
    except (TypeError, ValueError, OverflowError, OSError):
        stamp = "--:--:--"
    message = str(ev.get("message") or "").strip()
    label = activity_label(str(ev.get("stage") or ""), message)
    jid = str(ev.get("job_id") or "").strip()
    out = [stamp, f"[{label}]", (jid.split("-", 1)[0][:8] if jid else "") or "--------"]
    if label == "START":
        m = _NAME_RE.search(message)
        if m:
            out.append(m.group(1).strip())
    m = _PART_RE.search(message)
    if m:
        out.append(f"part {m.group(1)}")
    m = _MS_RE.search(message)
    if m:
        out.append(f"{m.group(1)}ms")
    return " ".join(out)


def emit_activity(message, job_id=None, filename=None, stage=None, source=None, store=None) -> None:
    st = store or get_store()
    ev = {"ts": time.time(), "message": str(message or "").strip()}
    for k, v in (("job_id", job_id), ("filename", filename), ("stage", stage), ("source", source)):
        if v:
            ev[k] = str(v)
    try:
        p = st.pipeline()
        p.lpush(ACTIVITY_LOG_KEY, json.dumps(ev, separators=(",", ":")))
        p.ltrim(ACTIVITY_LOG_KEY, 0, max(1, ACTIVITY_LOG_MAX) - 1)
        if job_id:
            k = f"joblog:{job_id}"
            p.rpush(k, format_activity_line(ev))
            p.ltrim(k, -max(1, ACTIVITY_JOB_LOG_MAX), -1)
        p.execute()
    except Exception:  # activity is best-effort, never fails a pipeline stage
        pass


def fetch_activity(limit=120, store=None) -> list[dict]:
    st = store or get_store()
    try:
        n = max(1, min(int(limit), 500))
    except (TypeError, ValueError):
        n = 120
    out = []
    for row in st.lrange(ACTIVITY_LOG_KEY, 0, n - 1) or []:
        try:
            d = json.loads(row)
        except (TypeError, ValueError):
            continue
        if isinstance(d, dict):
            out.append(d)
    return out


def fetch_job_activity(job_id, limit=None, store=None) -> list[str]:
    st = store or get_store()
    key = f"joblog:{job_id}"
    if limit is None:
        rows = st.lrange(key, 0, -1) or []
    else:
        try:
            n = max(1, int(limit))
        except (TypeError, ValueError):
            n = 500
        rows = st.lrange(key, -n, -1) or []
    out = []
    for row in rows:
        row = str(row or "").strip()
        if not row:
            continue
        if row.startswith("--:") or (len(row) >= 9 and row[2] == ":" and row[5] == ":"):
            out.append(row)
            continue
        try:  # legacy JSON rows
            d = json.loads(row)
            out.append(format_activity_line(d) if isinstance(d, dict) else str(d).strip())
        except ValueError:
            out.append(row)
    return out
