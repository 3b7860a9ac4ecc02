"""Manager HTTP API and UI (reference manager/app.py).

Every route of the reference is kept with the same method, path, payload and status
codes.  Deliberate fixes of reference defects: ``/dashboard`` renders
the jobs page instead of a missing template, ``/stop_job`` revokes the job's queued task
ids, ``/metrics_snapshot`` gets the ``mem_used``/``mem_total`` the agent now publishes,
and the allowed target heights are one list shared with the worker.

    python -m thinvids_amd.manager [--host 0.0.0.0] [--port 5005] [--no-housekeeping]
"""
from __future__ import annotations

import json
import logging
import math
import os
import re
import shutil
import socket
import subprocess
import time
import uuid

from flask import Flask, jsonify, render_template, request, send_file

from ..common import (JOBS_INDEX_KEY, Status, as_bool, as_float, as_int, emit_activity, fetch_activity,
                      fetch_job_activity, get_settings, invalidate_settings_cache, is_base_job_key,
                      natural_host_key)
from ..common.settings import LEGACY_SETTINGS_KEY, SETTINGS_KEY
from ..store import get_store
from . import core

log = logging.getLogger("thinvids.manager.app")

WATCHER_BOOL_FIELDS = {"USE_WATCHDOG", "USE_SCANNER", "ADOPT_EXISTING_PROCESSED_ON_STARTUP"}
WATCHER_INT_FIELDS = {"SCAN_INTERVAL_SEC": (5, 86400), "STABLE_CHECKS": (1, 60), "STABLE_DELAY_SEC": (1, 600),
                      "WORKERS": (1, 32)}
WATCHER_TEXT_FIELDS = {"PROCESSED_PATH_ALIASES": 1000}
WATCHER_FIELDS = {"WATCH_ROOT", *WATCHER_BOOL_FIELDS, *WATCHER_INT_FIELDS, *WATCHER_TEXT_FIELDS}
VIDEO_EXTS = {".mkv", ".mp4", ".y4m", ".synth", ".hevc", ".265"}


# ------------------------------------------------------------------ path guards
def safe_watch_rel_path(value) -> str:
    raw = str(value or "").replace("\\", "/").strip()
    if "\x00" in raw:
        raise ValueError("Invalid path")
    norm = os.path.normpath(raw.lstrip("/") or ".")
    if norm == ".":
        return ""
    if norm == ".." or norm.startswith("../"):
        raise ValueError("Path must stay under watch root")
    return norm.replace("\\", "/")


def abs_under_root(root: str, rel: str, label: str) -> str:
    rel = safe_watch_rel_path(rel)
    r = os.path.realpath(root)
    p = os.path.realpath(os.path.join(r, rel))
    if p != r and not p.startswith(r + os.sep):
        raise ValueError(f"Path must stay under {label} root")
    return p


def is_video_filename(name: str) -> bool:
    return os.path.splitext(name or "")[1].lower() in VIDEO_EXTS


def safe_existing_input_path(value) -> str:
    raw = str(value or "").strip()
    if not raw:
        return ""
    if "\x00" in raw:
        raise ValueError("Invalid input path")
    p = os.path.realpath(raw)
    for root in (core.CFG.watch_root, core.CFG.source_media_root):
        r = os.path.realpath(root)
        if p == r or p.startswith(r + os.sep):
            if not os.path.isfile(p):
                raise FileNotFoundError(p)
            if not is_video_filename(p):
                raise ValueError("Input path must be a supported video file")
            return p
    raise ValueError("Input path must stay under watch or source media root")


def job_source_path(filename: str, input_path: str = "") -> str:
    if input_path:
        return safe_existing_input_path(input_path)
    return abs_under_root(core.CFG.watch_root, filename, "watch")


def source_origin_for_path(path: str) -> str:
    r = os.path.realpath(core.CFG.source_media_root)
    p = os.path.realpath(path)
    return "source_media" if p == r or p.startswith(r + os.sep) else "watch"


def browse_root(source: str) -> dict:
    s = str(source or "watch").strip().lower()
    if s in ("watch", "archive", ""):
        return {"source": "watch", "label": "Watch Folder", "root_label": core.CFG.watch_root, "root_path": core.CFG.watch_root}
    if s in ("source_media", "source", "media"):
        return {"source": "source_media", "label": "Source Media", "root_label": "/source_media",
                "root_path": core.CFG.source_media_root}
    raise ValueError("Unknown browse source")


def normalize_target_height(value, default: int | None = None) -> int:
    d = default or core.CFG.default_target_height
    h = as_int(value, d)
    return h if h in core.CFG.allowed_target_heights else d


def default_target_height() -> int:
    return normalize_target_height(get_settings().get("default_target_height"))


# ---------------------------------------------------------- watcher control (C29)
def _run(cmd, timeout=15):
    try:
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout)
        return {"ok": r.returncode == 0, "returncode": r.returncode, "stdout": r.stdout[-4000:],
                "stderr": r.stderr[-4000:], "command": cmd}
    except (OSError, subprocess.TimeoutExpired) as e:
        return {"ok": False, "returncode": -1, "stdout": "", "stderr": str(e), "command": cmd}


def read_watcher_env_file() -> dict:
    out = {}
    try:
        with open(core.CFG.watcher_env_file, encoding="utf-8") as f:
            for line in f:
                line = line.strip()
                if not line or line.startswith("#") or "=" not in line:
                    continue
                k, v = line.split("=", 1)
                v = v.strip()
                if len(v) >= 2 and v[0] == v[-1] == '"':
                    v = v[1:-1].replace('\\"', '"').replace("\\$", "$").replace("\\\\", "\\")
                out[k.strip()] = v
    except FileNotFoundError:
        pass
    return out


def _env_quote(v) -> str:
    return '"' + str(v).replace("\\", "\\\\").replace('"', '\\"').replace("$", "\\$") + '"'


def write_watcher_env_file(values: dict) -> dict:
    os.makedirs(os.path.dirname(core.CFG.watcher_env_file) or ".", exist_ok=True)
    cur = read_watcher_env_file()
    cur.update(values)
    lines = ["# Managed by the thinvids manager Watcher page.",
             "# Values here override the watcher service Environment= defaults.", ""]
    lines += [f"{k}={_env_quote(cur[k])}" for k in sorted(cur) if re.fullmatch(r"[A-Za-z_][A-Za-z0-9_]*", k)]
    tmp = f"{core.CFG.watcher_env_file}.tmp.{os.getpid()}"
    with open(tmp, "w", encoding="utf-8") as f:
        f.write("\n".join(lines).rstrip() + "\n")
    os.replace(tmp, core.CFG.watcher_env_file)
    return cur


def normalize_watcher_config(payload) -> dict:
    if not isinstance(payload, dict):
        raise ValueError("Expected a JSON object.")
    out = {}
    if "WATCH_ROOT" in payload:
        raw = str(payload.get("WATCH_ROOT") or "").strip()
        if not raw.startswith("/") or any(c in raw for c in "\x00\r\n"):
            raise ValueError("Watch root must be an absolute path.")
        allowed = {os.path.realpath(core.CFG.watch_root): core.CFG.watch_root,
                   os.path.realpath(core.CFG.source_media_root): core.CFG.source_media_root}
        if os.path.realpath(raw) not in allowed:
            raise ValueError("Watch root must be one of the configured manager media roots.")
        out["WATCH_ROOT"] = allowed[os.path.realpath(raw)]
    for k in WATCHER_BOOL_FIELDS:
        if k in payload:
            out[k] = "1" if as_bool(payload.get(k)) else "0"
    for k, (lo, hi) in WATCHER_INT_FIELDS.items():
        if k in payload:
            v = as_int(payload.get(k), lo)
            if not lo <= v <= hi:
                raise ValueError(f"{k} must be between {lo} and {hi}.")
            out[k] = str(v)
    for k, n in WATCHER_TEXT_FIELDS.items():
        if k in payload:
            v = str(payload.get(k) or "").strip()
            if any(c in v for c in "\x00\r\n") or len(v) > n:
                raise ValueError(f"{k} is invalid.")
            out[k] = v
    return out


def read_watcher_service() -> dict:
    systemctl = shutil.which("systemctl")
    if not systemctl:
        return {"available": False, "name": core.CFG.watcher_service, "active_state": "unknown", "environment": {}}
    r = _run([systemctl, "show", core.CFG.watcher_service, "--no-pager",
              "--property=ActiveState,SubState,MainPID,ExecMainStartTimestamp,Environment"])
    props = dict(line.split("=", 1) for line in r["stdout"].splitlines() if "=" in line)
    env = dict(x.split("=", 1) for x in props.get("Environment", "").split() if "=" in x)
    return {"available": r["ok"], "name": core.CFG.watcher_service, "active_state": props.get("ActiveState", "unknown"),
            "sub_state": props.get("SubState", ""), "main_pid": props.get("MainPID", ""),
            "started_at": props.get("ExecMainStartTimestamp", ""), "environment": env}


def watcher_path_info(path: str) -> dict:
    info = {"path": path, "exists": os.path.isdir(path)}
    try:
        s = os.statvfs(path)
        info.update(total_bytes=s.f_blocks * s.f_frsize, free_bytes=s.f_bavail * s.f_frsize)
    except OSError:
        pass
    fm = shutil.which("findmnt")
    if fm and info["exists"]:
        r = _run([fm, "-n", "-o", "SOURCE,FSTYPE", "--target", path], timeout=5)
        info["mount"] = r["stdout"].strip()
    return info


def watcher_activity(limit=80) -> list[str]:
    jc = shutil.which("journalctl")
    if not jc:
        return []
    r = _run([jc, "-u", core.CFG.watcher_service, "-n", str(int(limit)), "--no-pager", "-o", "short-iso"], timeout=10)
    return r["stdout"].splitlines()[-limit:]


def watcher_status_payload(limit=80) -> dict:
    svc = read_watcher_service()
    envf = read_watcher_env_file()
    config = {"WATCH_ROOT": core.CFG.watch_root, "USE_WATCHDOG": "1", "USE_SCANNER": "1", "SCAN_INTERVAL_SEC": "60",
              "STABLE_CHECKS": "5", "STABLE_DELAY_SEC": "10", "WORKERS": "4",
              "ADOPT_EXISTING_PROCESSED_ON_STARTUP": "0", "PROCESSED_PATH_ALIASES": ""}
    config.update({k: v for k, v in svc.get("environment", {}).items() if k in WATCHER_FIELDS})
    config.update({k: v for k, v in envf.items() if k in WATCHER_FIELDS})
    return {"service": svc, "config": config, "config_fields": sorted(WATCHER_FIELDS),
            "field_types": {"bool": sorted(WATCHER_BOOL_FIELDS),
                            "int": {k: list(v) for k, v in WATCHER_INT_FIELDS.items()},
                            "text": dict(WATCHER_TEXT_FIELDS)},
            "known_roots": [{"label": "Watch folder", "path": core.CFG.watch_root},
                            {"label": "Source media", "path": core.CFG.source_media_root}],
            "env_file": {"path": core.CFG.watcher_env_file, "exists": os.path.exists(core.CFG.watcher_env_file),
                         "values": {k: v for k, v in envf.items() if k in WATCHER_FIELDS}},
            "watch_root": watcher_path_info(config.get("WATCH_ROOT") or core.CFG.watch_root),
            "activity": watcher_activity(limit), "generated_at": time.time()}


def control_watcher(action: str) -> dict:
    action = str(action or "").strip().lower()
    if action not in ("start", "stop", "restart"):
        raise ValueError("Action must be start, stop, or restart.")
    systemctl = shutil.which("systemctl") or "/bin/systemctl"
    cmd = [systemctl, action, core.CFG.watcher_service]
    if os.geteuid() != 0 and shutil.which("sudo"):
        cmd = [shutil.which("sudo"), "-n", *cmd]
    return _run(cmd, timeout=30)


# --------------------------------------------------------------------- settings
def settings_view(s: dict) -> dict:
    out = dict(s)
    out["suspend_enabled"] = as_bool(s.get("suspend_enabled"))
    out["suspend_idle_sec"] = max(30, as_int(s.get("suspend_idle_sec"), 300))
    out["suspend_idle_cpu_pct_max"] = min(100.0, max(1.0, as_float(s.get("suspend_idle_cpu_pct_max"), 15)))
    out["suspend_gc_enabled"] = as_bool(s.get("suspend_gc_enabled"))
    out["max_source_file_size_gb"] = as_float(s.get("max_source_file_size_gb"), 15)
    for k, d in (("av1_check_enabled", True), ("use_nfs_for_all_files", False),
                 ("use_direct_source_for_all_files", False), ("low_disk_direct_enabled", True)):
        out[k] = as_bool(s.get(k), d)
    out["low_disk_min_free_gb"] = as_float(s.get("low_disk_min_free_gb"), 20)
    out["target_segment_mb"] = as_float(s.get("target_segment_mb"), 10) or 10.0
    lfb = str(s.get("large_file_behavior") or "direct").strip().lower()
    out["large_file_behavior"] = lfb if lfb in ("reject", "nfs", "direct") else "reject"
    out["default_target_height"] = normalize_target_height(s.get("default_target_height"))
    rt = core.pipeline_runtime_settings(s)
    out.update(max_active_jobs=rt["max_active_jobs"], effective_max_active_jobs=rt["effective_max_active_jobs"],
               active_job_limit_enforced=False, pipeline_worker_count=rt["pipeline_worker_count"],
               pipeline_required_for_max_active=rt["max_active_jobs"] * 2,
               pipeline_drain_ratio_to_start_next=rt["pipeline_drain_ratio_to_start_next"],
               pipeline_min_idle_workers_to_start_next=rt["pipeline_min_idle_workers_to_start_next"])
    out["tv_qp"] = as_int(s.get("tv_qp"), 27)
    out["tv_gop"] = as_int(s.get("tv_gop"), 64)
    return out


def settings_from_payload(p: dict, cur: dict) -> dict:
    pwc = max(2, int(p.get("pipeline_worker_count", cur.get("pipeline_worker_count", 4))))
    lfb = str(p.get("large_file_behavior", "direct") or "direct").strip().lower()
    m = {
        "suspend_enabled": "1" if as_bool(p.get("suspend_enabled")) else "0",
        "suspend_idle_sec": str(max(30, int(p.get("suspend_idle_sec", 300)))),
        "suspend_idle_cpu_pct_max": str(min(100.0, max(1.0, as_float(p.get("suspend_idle_cpu_pct_max", 15), 15)))),
        "suspend_gc_enabled": "1" if as_bool(p.get("suspend_gc_enabled")) else "0",
        "max_source_file_size_gb": str(as_float(p.get("max_source_file_size_gb", 15), 15) or 15.0),
        "av1_check_enabled": "1" if as_bool(p.get("av1_check_enabled", True), True) else "0",
        "use_nfs_for_all_files": "1" if as_bool(p.get("use_nfs_for_all_files")) else "0",
        "use_direct_source_for_all_files": "1" if as_bool(p.get("use_direct_source_for_all_files")) else "0",
        "low_disk_direct_enabled": "1" if as_bool(p.get("low_disk_direct_enabled", True), True) else "0",
        "low_disk_min_free_gb": str(max(1.0, as_float(p.get("low_disk_min_free_gb", 20), 20))),
        "target_segment_mb": str(as_float(p.get("target_segment_mb", 10), 10) if as_float(
            p.get("target_segment_mb", 10), 10) > 0 else 10.0),
        "large_file_behavior": lfb if lfb in ("reject", "nfs", "direct") else "reject",
        "default_target_height": str(normalize_target_height(p.get("default_target_height"))),
        "max_active_jobs": str(max(1, pwc // 2)),
        "effective_max_active_jobs": str(max(1, pwc // 2)),
        "active_job_limit_enforced": "0",
        "pipeline_worker_count": str(pwc),
        "pipeline_drain_ratio_to_start_next": str(min(1.0, max(0.0, as_float(p.get(
            "pipeline_drain_ratio_to_start_next", cur.get("pipeline_drain_ratio_to_start_next", 0.75)), 0.75)))),
        "pipeline_min_idle_workers_to_start_next": str(max(1, int(p.get(
            "pipeline_min_idle_workers_to_start_next", cur.get("pipeline_min_idle_workers_to_start_next", 4))))),
    }
    for k, lo, hi in (("tv_qp", 0, 51), ("tv_gop", 1, 600), ("tv_search_range", 16, 128), ("tv_segment_frames", 0, 100000)):
        if k in p:
            m[k] = str(min(hi, max(lo, int(p[k]))))
    if "tv_deblock" in p:
        m["tv_deblock"] = "1" if as_bool(p["tv_deblock"], True) else "0"
    return m


# ------------------------------------------------------------------------- app
RC_MODES = ("", "cqp", "crf", "2pass", "abr")
CODECS = ("", "hevc", "av1")


def encoder_overrides(d: dict) -> dict:
    """Validated per-job encoder overrides from a job-settings payload (only the keys
    present; "" clears an override so the global tv_* setting applies).  Raises ValueError
    on out-of-range values."""
    out = {}
    if "rc_mode" in d:
        rc = str(d["rc_mode"] or "").lower()
        if rc not in RC_MODES:
            raise ValueError(f"rc_mode must be one of {RC_MODES[1:]}")
        out["rc_mode"] = rc
    for k, lo, hi in (("qp", 0, 51), ("crf", 1, 51)):
        if k in d:
            v = d[k]
            if v in ("", None):
                out[k] = ""
            elif not lo <= int(v) <= hi:
                raise ValueError(f"{k} out of range")
            else:
                out[k] = int(v)
    for k in ("bitrate_kbps", "vbv_maxrate_kbps", "vbv_bufsize_kbit"):  # VBV: rc_mode abr only
        if k in d:
            v = d[k]
            out[k] = "" if v in ("", None) else float(v)
            if out[k] != "" and out[k] <= 0:
                raise ValueError(f"{k} must be positive")
    if "ladder" in d:
        rungs = [int(x) for x in str(d["ladder"] or "").replace(" ", "").split(",") if x]
        if any(not 64 <= r <= 4320 for r in rungs):
            raise ValueError("ladder rungs must be heights in 64..4320")
        out["ladder"] = ",".join(str(r) for r in rungs)
    if "node_executor" in d:
        out["node_executor"] = "" if d["node_executor"] in ("", None) else ("1" if as_bool(d["node_executor"]) else "0")
    if "codec" in d:
        c = str(d["codec"] or "").lower()
        if c not in CODECS:
            raise ValueError(f"codec must be one of {CODECS[1:]}")
        out["codec"] = c
    return out


def create_app(store=None, housekeeping: bool = False) -> Flask:
    here = os.path.dirname(os.path.abspath(__file__))
    app = Flask("thinvids_manager", template_folder=os.path.join(here, "templates"),
                static_folder=os.path.join(here, "static"))
    st_override = store

    def st():
        return st_override or get_store()

    caches = {"metrics": (0.0, None), "jobs": (0.0, None)}

    def job_or_404(job_id):
        key = f"job:{job_id}"
        if not st().exists(key):
            return key, None
        return key, st().hgetall(key) or {}

    # ------------------------------------------------------------ pages
    @app.get("/")
    def index_page():
        return render_template("index.html", page="jobs")

    @app.get("/dashboard")
    def dashboard_page():  # reference route rendered a missing template (§2.7)
        return render_template("index.html", page="jobs")

    @app.get("/metrics")
    def metrics_page():
        return render_template("metrics.html", page="metrics")

    @app.get("/browse")
    def browse_page():
        return render_template("browse.html", page="browse")

    @app.get("/watcher")
    def watcher_page():
        return render_template("watcher.html", page="watcher")

    @app.get("/nodes")
    def nodes_page():
        return render_template("nodes.html", page="nodes")

    # ---------------------------------------------------------- watcher
    @app.get("/watcher/status")
    def watcher_status():
        return jsonify(watcher_status_payload(as_int(request.args.get("limit"), 80)))

    @app.post("/watcher/config")
    def watcher_config():
        payload = request.get_json(silent=True) or {}
        restart = as_bool(payload.pop("restart", False)) if isinstance(payload, dict) else False
        try:
            values = normalize_watcher_config(payload)
        except ValueError as e:
            return jsonify({"status": "error", "message": str(e)}), 400
        try:
            saved = write_watcher_env_file(values)
        except OSError as e:
            return jsonify({"status": "error", "message": f"could not write env file: {e}"}), 500
        out = {"status": "ok", "saved": {k: v for k, v in saved.items() if k in WATCHER_FIELDS}}
        if restart:
            out["restart"] = control_watcher("restart")
        return jsonify(out)

    @app.post("/watcher/control")
    def watcher_control():
        payload = request.get_json(silent=True) or {}
        try:
            res = control_watcher(payload.get("action"))
        except ValueError as e:
            return jsonify({"status": "error", "message": str(e)}), 400
        return jsonify({"status": "ok" if res["ok"] else "error", "result": res}), (200 if res["ok"] else 500)

    # ----------------------------------------------------------- browse
    @app.get("/browse/list")
    def browse_list():
        try:
            root = browse_root(request.args.get("source"))
            rel = safe_watch_rel_path(request.args.get("path") or "")
            path = abs_under_root(root["root_path"], rel, root["label"])
        except ValueError as e:
            return jsonify({"status": "error", "message": str(e)}), 400
        if not os.path.isdir(path):
            return jsonify({"status": "error", "message": "Directory not found"}), 404
        dirs, files = [], []
        with os.scandir(path) as it:
            for e in it:
                if e.name.startswith("."):
                    continue
                r = f"{rel}/{e.name}" if rel else e.name
                if e.is_dir(follow_symlinks=False):
                    dirs.append({"name": e.name, "path": r})
                elif e.is_file() and is_video_filename(e.name):
                    s = e.stat()
                    files.append({"name": e.name, "path": r, "size": s.st_size, "mtime": s.st_mtime,
                                  "input_path": os.path.join(path, e.name)})
        dirs.sort(key=lambda d: d["name"].lower())
        files.sort(key=lambda f: f["name"].lower())
        parent = os.path.dirname(rel) if rel else None
        return jsonify({"status": "ok", **root, "path": rel, "parent": parent, "dirs": dirs, "files": files})

    # ------------------------------------------------------ nodes/metrics
    def _json_list(v):
        try:
            d = json.loads(v or "[]")
        except ValueError:
            return []
        return d if isinstance(d, list) else []

    def _executor_info(host):
        raw = st().get(f"node:executor:{host}")
        if not raw:
            return None
        try:
            d = json.loads(raw)
        except ValueError:
            return None
        return {"world": as_int(d.get("world"), 0), "pid": as_int(d.get("pid"), 0), "ts": as_float(d.get("ts"))}

    @app.get("/nodes_data")
    def nodes_data():
        nodes = core.get_all_nodes(st())
        active = {n["hostname"] for n in core.get_active_nodes(st())}
        roles = core.assign_pipeline_node_roles(None, st())
        items = []
        for n in nodes:
            h = n["hostname"]
            md = st().hgetall(f"metrics:node:{h}") or {}
            q = st().hgetall(f"node:quarantine:{h}") or {} if n["disabled"] else {}
            try:
                ip = md.get("ip") or socket.gethostbyname(h)
            except OSError:
                ip = ""
            items.append({"hostname": h, "ip": ip, "mac": n["mac"], "last_seen_ts": int(as_float(md.get("ts"))),
                          "active": h in active and not n["disabled"], "disabled": n["disabled"],
                          "worker_role": roles.get(h, "disabled" if n["disabled"] else "encode"),
                          "gpu_count": as_int(md.get("gpu_count"), 0), "gpu_name": md.get("gpu_name", ""),
                          "quarantine_reason": q.get("reason") or "",
                          "quarantined_at": as_float(q.get("quarantined_at")),
                          # detail panel: live utilisation and the node executor's rank group
                          "cpu": as_float(md.get("cpu")), "mem": as_float(md.get("mem")),
                          "gpu": as_float(md.get("gpu"), -1.0), "hbm_used": as_int(md.get("hbm_used")),
                          "hbm_total": as_int(md.get("hbm_total")), "disk": as_int(md.get("disk")),
                          "gpus": _json_list(md.get("gpus_json")), "executor": _executor_info(h),
                          "gpu_quarantine": {g: (json.loads(v) if v.startswith("{") else {"reason": v})
                                             for g, v in (st().hgetall(f"node:gpu_quarantine:{h}") or {}).items()}})
        items.sort(key=lambda x: natural_host_key(x["hostname"]))
        return jsonify({"nodes": items})

    @app.get("/metrics_snapshot")
    def metrics_snapshot():
        now = time.time()
        ts, cached = caches["metrics"]
        if cached and now - ts < 0.5:
            return jsonify(cached)
        hosts = [n["hostname"] for n in core.get_all_nodes(st()) if not n["disabled"]]
        p = st().pipeline()
        for h in hosts:
            p.hgetall(f"metrics:node:{h}")
        nodes = []
        for h, d in zip(hosts, p.execute() if hosts else []):
            if not d:
                continue
            nodes.append({"key": f"metrics:node:{h}", "hostname": d.get("hostname") or h,
                          "ts": int(as_float(d.get("ts"))), "cpu": as_float(d.get("cpu")),
                          "gpu": as_float(d.get("gpu"), -1.0), "mem": as_float(d.get("mem")),
                          "mem_used": as_int(d.get("mem_used")), "mem_total": as_int(d.get("mem_total")),
                          "rx_bps": as_int(d.get("rx_bps")), "tx_bps": as_int(d.get("tx_bps")),
                          "disk": as_int(d.get("disk")), "gpu_count": as_int(d.get("gpu_count")),
                          "hbm_used": as_int(d.get("hbm_used")), "hbm_total": as_int(d.get("hbm_total")),
                          "gpus": json.loads(d.get("gpus_json") or "[]")})
        nodes.sort(key=lambda n: natural_host_key(n["hostname"]))
        payload = {"nodes": nodes}
        caches["metrics"] = (now, payload)
        return jsonify(payload)

    @app.get("/settings")
    def settings_get():
        return jsonify(settings_view(get_settings()))

    @app.post("/settings")
    def settings_post():
        payload = request.get_json(silent=True) or {}
        try:
            mapping = settings_from_payload(payload, get_settings())
        except (TypeError, ValueError):
            return jsonify({"error": "invalid payload"}), 400
        st().hset(SETTINGS_KEY, mapping=mapping)
        st().hset(LEGACY_SETTINGS_KEY, mapping=mapping)
        invalidate_settings_cache()
        core.assign_pipeline_node_roles(None, st())
        return jsonify({"status": "ok", "settings": settings_view(get_settings())})

    # --------------------------------------------------------------- jobs
    status_order = {"READY": 0, "STARTING": 1, "WAITING": 2, "RUNNING": 3, "STAMPING": 4, "STOPPED": 5,
                    "FAILED": 6, "REJECTED": 7, "DONE": 8, "COMPLETED": 8}

    def all_jobs():
        now = time.time()
        ts, cached = caches["jobs"]
        if cached is not None and now - ts < 0.5:
            return cached
        s = st()
        raw = list(s.smembers(JOBS_INDEX_KEY) or [])
        keys = [k for k in raw if is_base_job_key(k)]
        bad = [k for k in raw if not is_base_job_key(k)]
        if bad:
            s.srem(JOBS_INDEX_KEY, *bad)
        if not keys:
            keys = [k for k in s.scan_iter("job:*") if is_base_job_key(k)]
            if keys:
                s.sadd(JOBS_INDEX_KEY, *keys)
        jobs = []
        p = s.pipeline()
        for k in keys:
            p.hgetall(k)
        for k, d in zip(keys, p.execute() if keys else []):
            if not d:
                s.srem(JOBS_INDEX_KEY, k)
                continue
            stt = core.job_status(d)
            started, ended, created = as_float(d.get("started_at")), as_float(d.get("ended_at")), as_float(
                d.get("created_at"))
            elapsed = 0.0
            if stt in (Status.RUNNING, Status.WAITING, Status.STARTING):
                elapsed = now - started if started else 0.0
            elif ended:
                elapsed = ended - started
            jobs.append({"job_id": k.split(":", 1)[1], **d,
                         "segment_progress": as_int(d.get("segment_progress")),
                         "encode_progress": as_int(d.get("encode_progress")),
                         "combine_progress": as_int(d.get("combine_progress")), "elapsed": elapsed,
                         "started": started, "created": created, "stitched_chunks": as_int(d.get("stitched_chunks"))})
        caches["jobs"] = (now, jobs)
        return jobs

    @app.get("/jobs")
    def list_jobs():
        jobs = all_jobs()
        page = max(1, as_int(request.args.get("page"), 1))
        size = as_int(request.args.get("page_size"), 10)
        size = size if size in (10, 25, 50, 100) else 10
        sort_by = (request.args.get("sort_by") or "date").lower()
        reverse = (request.args.get("sort_dir") or "desc").lower() != "asc"
        sf = (request.args.get("status") or "").strip().upper()
        q = (request.args.get("q") or "").strip().lower()
        if sf and sf != "ALL":
            want = {"DONE", "COMPLETED"} if sf == "DONE" else {sf}
            jobs = [j for j in jobs if (j.get("status") or "").upper() in want]
        if q:
            def hit(j):
                fn = j.get("filename") or ""
                base = os.path.basename(fn).lower()
                return q in os.path.splitext(base)[0] or q in base or q in fn.lower()
            jobs = [j for j in jobs if hit(j)]

        def key(j):
            s = (j.get("status") or "").upper()
            fn = os.path.basename(j.get("filename") or "").lower()
            if sort_by == "filename":
                return (fn,)
            if sort_by == "status":
                return (status_order.get(s, 99), fn)
            if sort_by == "encode":
                return (j["encode_progress"], j["started"], fn)
            return (max(j["started"], j["created"]),)
        jobs = sorted(jobs, key=key, reverse=reverse)
        total = len(jobs)
        pages = max(1, math.ceil(total / size))
        page = min(page, pages)
        return jsonify({"page": page, "page_size": size, "total": total, "total_pages": pages,
                        "items": jobs[(page - 1) * size: page * size]})

    @app.get("/activity")
    def activity():
        return jsonify({"items": fetch_activity(min(500, max(1, as_int(request.args.get("limit"), 120))), st())})

    @app.get("/job_activity/<job_id>")
    def job_activity(job_id):
        lim = request.args.get("limit")
        return jsonify({"job_id": job_id, "lines": fetch_job_activity(job_id, as_int(lim) if lim else None, st())})

    def new_job_fields(job_id, filename, full_path, status, now, auto, settings, target_height):
        return {"job_id": job_id, "filename": filename, "input_path": full_path,
                "source_origin": source_origin_for_path(full_path), "status": status.value, "created_at": str(now),
                "started_at": str(now) if auto else "0", "total_chunks": 0, "completed_chunks": 0,
                "stitched_chunks": 0, "segment_duration": as_int(settings.get("segment_duration"), 10),
                "number_parts": as_int(settings.get("number_parts"), 2),
                "serialize_pipeline": "1" if as_bool(settings.get("serialize_pipeline")) else "0",
                "software_encode": "0", "target_height": target_height,
                "queue_action": core.PIPELINE_QUEUE_ACTION_TRANSCODE if auto else "",
                "waiting_at": str(now) if auto else "0", "source_codec": "", "source_resolution": "",
                "source_duration": "0", "source_fps": "0", "source_file_size": 0, "total_frames": 0,
                "scratch_mode": "local", "scratch_root": core.CFG.local_project_root, "processing_mode": "split",
                "processing_mode_effective": "", "processing_mode_reason": ""}

    @app.post("/add_job")
    def add_job():
        data = request.get_json(silent=True) or {}
        try:
            filename = safe_watch_rel_path(data.get("filename"))
        except ValueError as e:
            return jsonify({"status": "error", "message": str(e)}), 400
        force_paused = bool(data.get("force_paused", False))
        manual_review = bool(data.get("manual_review", False))
        if not filename or not is_video_filename(filename):
            return jsonify({"status": "error", "message": "Invalid file format"}), 400
        try:
            full = job_source_path(filename, data.get("input_path") or "")
        except FileNotFoundError:
            return jsonify({"status": "error", "message": "Source file not found"}), 404
        except ValueError as e:
            return jsonify({"status": "error", "message": str(e)}), 400
        if not os.path.isfile(full):
            return jsonify({"status": "error", "message": "Source file not found"}), 404
        s = st()
        settings = get_settings()
        job_id, now = str(uuid.uuid4()), time.time()
        auto = as_bool(settings.get("auto_start", "1"), True) and not force_paused
        th = normalize_target_height(data.get("target_height", default_target_height()))
        job = new_job_fields(job_id, filename, full, Status.WAITING if auto else Status.READY, now, auto, settings, th)
        emit_activity(f'Received "{core.display_title(filename)}"', job_id=job_id, filename=filename,
                      stage="received", source="manager", store=s)
        details = core.get_video_details(full)
        job.update(details)
        reason, message, smode, sroot, pmode = core.evaluate_job_policy(details, settings)
        job.update(scratch_mode=smode, scratch_root=sroot, processing_mode=pmode)
        if job["source_origin"] == "source_media" and pmode == "direct" and \
                str(details.get("source_codec") or "").lower() not in core.DIRECT_SOURCE_REQUIRED_CODECS:
            job.update(processing_mode="split", processing_mode_reason="source_media_forces_split",
                       policy_warning="Source-media jobs are forced to split mode.")
        if not reason and details.get("probe_error"):
            reason, message = "probe_failed", f"Source could not be probed: {details['probe_error']}"
        warning = None
        if reason and manual_review and force_paused:
            warning = message
            job.update(status=Status.READY.value, started_at="0", queue_action="", waiting_at="0",
                       policy_warning=message, policy_warning_reason=reason, policy_warning_at=str(now))
            emit_activity(f'Queued "{core.display_title(filename)}" for review with warning: {message}',
                          job_id=job_id, filename=filename, stage="ready", source="manager", store=s)
            reason = None
        elif reason:
            job.update(status=Status.REJECTED.value, started_at="0", queue_action="", waiting_at="0", error=message,
                       rejected_reason=reason, rejected_at=str(now))
            emit_activity(f'Rejected "{core.display_title(filename)}": {message}', job_id=job_id,
                          filename=filename, stage="rejected", source="manager", store=s)
        s.hset(f"job:{job_id}", mapping=job)
        s.sadd(JOBS_INDEX_KEY, f"job:{job_id}")
        caches["jobs"] = (0.0, None)
        mark_warning = None
        if data.get("mark_watcher_processed"):
            try:
                from ..watcher import mark_processed

                mark_processed(full, core.CFG.watch_root, core.CFG.processed_file)
            except Exception as e:
                mark_warning = str(e)
        if auto and not reason:
            core.queue_job_for_dispatch(f"job:{job_id}", core.PIPELINE_QUEUE_ACTION_TRANSCODE, now, s)
            core.dispatch_next_waiting_job(s)
        if reason:
            out = {"status": "rejected", "job_id": job_id, "message": message, "reason": reason}
        else:
            out = {"status": "success", "job_id": job_id}
            if warning:
                out["policy_warning"] = warning
        if mark_warning:
            out["watcher_mark_warning"] = mark_warning
        return jsonify(out), 201

    @app.post("/copy_job")
    def copy_job():
        data = request.get_json(silent=True) or {}
        src_id = data.get("job_id")
        if not src_id:
            return jsonify({"status": "error", "message": "job_id is required"}), 400
        _, src = job_or_404(src_id)
        if src is None:
            return jsonify({"status": "error", "message": "Source job not found"}), 404
        if not src.get("filename"):
            return jsonify({"status": "error", "message": "Source job missing filename"}), 400
        new_id, now = str(uuid.uuid4()), time.time()
        keep = ("filename", "input_path", "source_origin", "segment_duration", "number_parts", "serialize_pipeline",
                "software_encode", "selected_v_stream", "selected_a_stream", "scratch_mode", "scratch_root",
                "processing_mode", "streams_json", "source_codec", "source_resolution", "source_width",
                "source_height", "source_fps", "source_fps_num", "source_fps_den", "source_duration",
                "source_file_size", "total_frames")
        new = {k: src[k] for k in keep if k in src}
        new.update(job_id=new_id, status=Status.READY.value, created_at=str(now), started_at="0",
                   target_height=normalize_target_height(src.get("target_height", default_target_height())),
                   processing_mode_effective="", processing_mode_reason="", total_chunks=0, completed_chunks=0,
                   stitched_chunks=0)
        st().hset(f"job:{new_id}", mapping=new)
        st().sadd(JOBS_INDEX_KEY, f"job:{new_id}")
        caches["jobs"] = (0.0, None)
        return jsonify({"status": "success", "job_id": new_id}), 201

    @app.post("/start_job/<job_id>")
    def start_job(job_id):
        key, job = job_or_404(job_id)
        if job is None:
            return jsonify({"status": "not found"}), 404
        if core.job_status(job) != Status.READY:
            return jsonify({"status": "invalid", "message": "Job is not in READY state"}), 400
        if not job.get("filename"):
            return jsonify({"status": "invalid", "message": "Missing filename"}), 400
        now = time.time()
        st().hset(key, mapping={"started_at": str(now), "queue_blocked_reason": ""})
        core.queue_job_for_dispatch(key, core.PIPELINE_QUEUE_ACTION_TRANSCODE, now, st())
        emit_activity(f'Queued "{core.display_title(job.get("filename"))}"', job_id=job_id,
                      filename=job.get("filename"), stage="queued", source="manager", store=st())
        caches["jobs"] = (0.0, None)
        core.dispatch_next_waiting_job(st())
        return jsonify({"status": "started"}), 200

    @app.post("/restart_job/<job_id>")
    def restart_job(job_id):
        key, job = job_or_404(job_id)
        if job is None:
            return jsonify({"status": "not found"}), 404
        if core.job_status(job) not in (Status.STOPPED, Status.FAILED, Status.REJECTED, Status.DONE):
            return jsonify({"status": "invalid", "message": "Job is not in STOPPED/FAILED/REJECTED/DONE state."}), 400
        filename = job.get("filename")
        if not filename:
            return jsonify({"status": "invalid", "message": "Missing filename"}), 400
        s = st()
        for k in list(s.scan_iter(f"{key}:*")):
            s.delete(k)
        from ..worker.helpers import job_base_dir

        shutil.rmtree(job_base_dir(job_id, job), ignore_errors=True)
        try:
            full = job_source_path(filename, job.get("input_path") or "")
        except (ValueError, FileNotFoundError):
            full = os.path.join(core.CFG.watch_root, filename.lstrip("/"))
        details = core.get_video_details(full)
        settings = get_settings()
        reason, message, smode, sroot, pmode = core.evaluate_job_policy(details, settings)
        now = time.time()
        clear = {f: "" for f in ("error", "failed_stage", "failed_worker", "rejected_reason", "rejected_at",
                                 "stalled_stage", "stalled_detected_at", "output_path", "queue_blocked_reason",
                                 "pipeline_run_token", "last_part_error")}
        from ..worker.helpers import RUN_COUNTER_FIELDS

        zero = {f: 0 for f in (*RUN_COUNTER_FIELDS, "queue_dispatch_attempts", "node_restarts")}
        mapping = {**clear, **zero, **details, "scratch_mode": smode, "scratch_root": sroot,
                   "processing_mode": pmode, "processing_mode_effective": "", "processing_mode_reason": "",
                   "target_height": normalize_target_height(job.get("target_height", default_target_height()))}
        if reason:
            mapping.update(status=Status.REJECTED.value, error=message, rejected_reason=reason, rejected_at=str(now))
            s.hset(key, mapping=mapping)
            return jsonify({"status": "rejected", "message": message, "reason": reason}), 200
        mapping.update(started_at=str(now))
        s.hset(key, mapping=mapping)
        for k in (f"job_done_parts:{job_id}", f"job_retry_counts:{job_id}", f"job_retry_ts:{job_id}",
                  f"job_missing_first_seen:{job_id}", f"job_retry_inflight:{job_id}"):
            s.delete(k)
        core.queue_job_for_dispatch(key, core.PIPELINE_QUEUE_ACTION_TRANSCODE, now, s)
        emit_activity(f'Restarted "{core.display_title(filename)}"', job_id=job_id, filename=filename,
                      stage="restart", source="manager", store=s)
        caches["jobs"] = (0.0, None)
        core.dispatch_next_waiting_job(s)
        return jsonify({"status": "restarted"}), 200

    @app.post("/stop_job/<job_id>")
    def stop_job(job_id):
        key, job = job_or_404(job_id)
        if job is None:
            return jsonify({"status": "not found"}), 404
        st().hset(key, mapping={"status": Status.STOPPED.value, "ended_at": str(time.time())})
        n = core.revoke_job_tasks(job_id, st())
        core.clear_active_job_refs(job_id, st())
        caches["jobs"] = (0.0, None)
        core.dispatch_next_waiting_job(st())
        return jsonify({"status": "stopped", "revoked_tasks": n}), 200

    @app.delete("/delete_job/<job_id>")
    def delete_job(job_id):
        key, job = job_or_404(job_id)
        if job is None:
            return jsonify({"status": "not found"}), 404
        s = st()
        for k in list(s.scan_iter(f"{key}*")):
            s.delete(k)
        s.delete(f"joblog:{job_id}")
        s.srem(JOBS_INDEX_KEY, key)
        core.revoke_job_tasks(job_id, s)
        core.clear_active_job_refs(job_id, s)
        from ..worker.helpers import job_base_dir

        shutil.rmtree(job_base_dir(job_id, job), ignore_errors=True)
        caches["jobs"] = (0.0, None)
        core.dispatch_next_waiting_job(s)
        return jsonify({"status": "deleted"}), 200

    @app.get("/preview/<job_id>")
    def preview(job_id):
        _, job = job_or_404(job_id)
        if job is None:
            return jsonify({"error": "Job not found"}), 404
        out = job.get("output_path")
        if not out or not os.path.isfile(out):
            return jsonify({"error": "Output not found"}), 404
        return send_file(out, mimetype="video/mp4", conditional=True)

    @app.get("/job_properties/<job_id>")
    def job_properties(job_id):
        _, job = job_or_404(job_id)
        if job is None:
            return jsonify({"error": "Job not found"}), 404
        return jsonify({**job, "activity_log": fetch_job_activity(job_id, None, st())})

    @app.route("/job_settings/<job_id>", methods=["GET", "POST"])
    def job_settings(job_id):
        key, job = job_or_404(job_id)
        if job is None:
            return jsonify({"error": "Job not found"}), 404
        if request.method == "GET":
            return jsonify({"job_id": job_id, "filename": job.get("filename"), "status": job.get("status"),
                            "segment_duration": as_int(job.get("segment_duration"), 10),
                            "number_parts": as_int(job.get("number_parts"), 2),
                            "serialize_pipeline": job.get("serialize_pipeline", "0"),
                            "software_encode": job.get("software_encode", "0"),
                            "target_height": normalize_target_height(job.get("target_height")),
                            "streams": job.get("streams_json") or "[]",
                            "selected_v_stream": job.get("selected_v_stream", "0"),
                            "selected_a_stream": job.get("selected_a_stream", "0"),
                            # encoder knobs of this framework (per-job overrides of tv_*)
                            "rc_mode": job.get("rc_mode", ""), "qp": job.get("qp", ""), "crf": job.get("crf", ""),
                            "bitrate_kbps": job.get("bitrate_kbps", ""), "ladder": job.get("ladder", ""),
                            "vbv_maxrate_kbps": job.get("vbv_maxrate_kbps", ""),
                            "vbv_bufsize_kbit": job.get("vbv_bufsize_kbit", ""),
                            "node_executor": job.get("node_executor", ""), "codec": job.get("codec", ""),
                            "source_fps": job.get("source_fps", "")})
        if core.job_status(job) == Status.RUNNING:
            return jsonify({"error": "Job is RUNNING; stop it or copy/restart to change settings."}), 400
        d = request.get_json(silent=True) or {}
        try:
            mapping = {"segment_duration": int(d.get("segment_duration", job.get("segment_duration", 10))),
                       "number_parts": int(d.get("number_parts", job.get("number_parts", 2))),
                       "selected_v_stream": int(d.get("selected_v_stream", job.get("selected_v_stream", 0))),
                       "selected_a_stream": int(d.get("selected_a_stream", job.get("selected_a_stream", 0))),
                       "serialize_pipeline": "1" if as_bool(d.get("serialize_pipeline",
                                                                  job.get("serialize_pipeline", "0"))) else "0",
                       "software_encode": "1" if as_bool(d.get("software_encode",
                                                               job.get("software_encode", "0"))) else "0",
                       "target_height": normalize_target_height(d.get("target_height", job.get("target_height")))}
            if "number_parts" in d:
                mapping["number_parts_override"] = "1"
            mapping.update(encoder_overrides(d))
        except (TypeError, ValueError) as e:
            return jsonify({"error": f"Failed to update settings: {e}"}), 500
        st().hset(key, mapping=mapping)
        caches["jobs"] = (0.0, None)
        return jsonify({"status": "ok"}), 200

    @app.post("/stamp_job/<job_id>")
    def stamp_job(job_id):
        key, job = job_or_404(job_id)
        if job is None:
            return jsonify({"status": "not found"}), 404
        if core.job_status(job) in (Status.STARTING, Status.WAITING, Status.RUNNING, Status.STAMPING):
            return jsonify({"status": "invalid", "message": "Job is busy; stop it first."}), 400
        fn = job.get("filename") or ""
        try:
            full = job_source_path(fn, job.get("input_path") or "")
        except (ValueError, FileNotFoundError):
            full = os.path.join(core.CFG.watch_root, fn.lstrip("/")) if fn else ""
        if not full or not os.path.exists(full):
            return jsonify({"status": "error", "message": f"Input not found: {full}"}), 400
        started = as_float(job.get("started_at")) or time.time()
        core.queue_job_for_dispatch(key, core.PIPELINE_QUEUE_ACTION_STAMP, started, st())
        st().hset(key, mapping={"encode_progress": 0, "encode_elapsed": 0})
        caches["jobs"] = (0.0, None)
        core.dispatch_next_waiting_job(st())
        return jsonify({"status": "queued"}), 202

    # legacy aliases (reference :2815-2833)
    app.add_url_rule("/tasks", "tasks_legacy", list_jobs, methods=["GET"])
    app.add_url_rule("/add_task", "add_task_legacy", add_job, methods=["POST"])
    app.add_url_rule("/start_task/<job_id>", "start_task_legacy", start_job, methods=["POST"])
    app.add_url_rule("/stop_task/<job_id>", "stop_task_legacy", stop_job, methods=["POST"])
    app.add_url_rule("/delete_task/<job_id>", "delete_task_legacy", delete_job, methods=["DELETE", "POST"])

    # ------------------------------------------------------ node management
    @app.delete("/nodes/delete/<host>")
    def node_delete(host):
        s = st()
        s.hdel("nodes:mac", host)
        s.srem(core.DISABLED_NODES_KEY, host)
        s.delete(f"metrics:node:{host}", f"node:quarantine:{host}")
        s.hdel(core.PIPELINE_NODE_ROLES_KEY, host)
        return jsonify({"status": "deleted", "hostname": host})

    @app.post("/nodes/disable/<host>")
    def node_disable(host):
        st().sadd(core.DISABLED_NODES_KEY, host)
        core.assign_pipeline_node_roles(None, st())
        return jsonify({"status": "disabled", "hostname": host})

    @app.post("/nodes/enable/<host>")
    def node_enable(host):
        st().srem(core.DISABLED_NODES_KEY, host)
        st().delete(f"node:quarantine:{host}")
        core.assign_pipeline_node_roles(None, st())
        return jsonify({"status": "enabled", "hostname": host})

    @app.post("/nodes/wake/<host>")
    def node_wake(host):
        ok = core.wake_one_node(host, st())
        return jsonify({"status": "sent" if ok else "error", "hostname": host}), (200 if ok else 404)

    @app.post("/nodes/wake_all")
    def nodes_wake_all():
        return jsonify({"status": "sent", "count": core.wake_all_nodes(st())})

    @app.post("/nodes/reboot_all")
    def nodes_reboot_all():
        return jsonify({"status": "ok", "results": core.reboot_all_nodes(st())})

    if housekeeping:
        app.housekeeping = core.Housekeeping(st_override).start()
    return app


def main(argv=None) -> int:  # pragma: no cover - service entry
    import argparse

    from ..common import get_logging

    ap = argparse.ArgumentParser()
    ap.add_argument("--host", default=os.environ.get("MANAGER_BIND", "0.0.0.0"))
    ap.add_argument("--port", type=int, default=int(os.environ.get("MANAGER_PORT", "5005")))
    ap.add_argument("--no-housekeeping", action="store_true")
    a = ap.parse_args(argv)
    get_logging("manager")
    app = create_app(housekeeping=not a.no_housekeeping)
    app.run(host=a.host, port=a.port, threaded=True)
    return 0
