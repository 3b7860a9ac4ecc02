"""Node agent (reference agent/agent.py).

A 1 Hz loop that is the cluster's liveness signal:

* publishes ``metrics:node:<host>`` = {ts, hostname, ip, mac, cpu, gpu, mem, mem_used,
  mem_total, disk, rx_bps, tx_bps, worker_role} + MI355X fields {gpu_count, gpu_name,
  hbm_used, hbm_total, xgmi_rx_bps, xgmi_tx_bps, xgmi_read_bytes, xgmi_write_bytes,
  gpus_json} with ``EXPIRE TTL_SEC`` (C7, C8, SURVEY 5.5: xGMI bytes are the node's
  collective traffic, as the NIC counters were the reference's data-plane traffic);
* publishes ``nodes:mac[host]`` hourly (manager discovery / WOL);
* role sync: the encode service always runs, the pipeline service only when
  ``pipeline:node_roles[host] == "pipeline"`` (C9);
* idle suspend gated by global settings: CPU and GPU idle, all jobs idle, idle long
  enough, uptime >= 300 s (C10);
* scratch GC of stale UUID-named job dirs (C11) — reading ``jobs:all`` (the reference read
  the never-written ``jobs:index``).
"""
from __future__ import annotations

import logging
import os
import re
import shutil
import socket
import subprocess
import time

import psutil

from ..common import all_jobs_are_idle, as_bool, as_float, as_int, get_settings
from ..store import get_store
from .gpu import GpuSampler

log = logging.getLogger("thinvids.agent")
_GUID_RE = re.compile(r"^[0-9A-Fa-f]{8}(?:-[0-9A-Fa-f]{4}){3}-[0-9A-Fa-f]{12}$")
ACTIVE = {"STARTING", "WAITING", "RUNNING", "STAMPING"}


class AgentConfig:
    def __init__(self):
        e = os.environ
        self.hostname = e.get("HOSTNAME") or socket.gethostname()
        self.ttl_sec = as_int(e.get("TTL_SEC"), 15)
        self.iface = e.get("AGENT_IFACE", "").strip()
        self.mac = e.get("AGENT_MAC", "").strip()
        self.suspend_enabled = as_bool(e.get("SUSPEND_ENABLED", "1"), True)
        self.suspend_after_idle_sec = as_int(e.get("SUSPEND_AFTER_IDLE_SEC"), 300)
        self.idle_cpu_pct_max = as_float(e.get("IDLE_CPU_PCT_MAX"), 15)
        self.idle_gpu_pct_max = as_float(e.get("IDLE_GPU_PCT_MAX"), 10)
        self.min_uptime_before_suspend = as_int(e.get("MIN_UPTIME_BEFORE_SUSPEND"), 300)
        self.gc_base_dir = e.get("GC_BASE_DIR", e.get("PROJECT_ROOT", "/projects"))
        self.gc_interval_sec = max(60, as_int(e.get("GC_INTERVAL_SEC"), 900))
        self.gc_min_age_sec = max(300, as_int(e.get("GC_MIN_AGE_SEC"), 21600))
        self.role_sync_interval_sec = max(5, as_int(e.get("ROLE_SYNC_INTERVAL_SEC"), 10))
        self.encode_service = e.get("ENCODE_SERVICE", "thinvids-worker-encode.target")
        self.pipeline_service = e.get("PIPELINE_SERVICE", "thinvids-worker-pipeline.service")
        self.manage_services = as_bool(e.get("AGENT_MANAGE_SERVICES", "1"), True) and bool(shutil.which("systemctl"))


def primary_ip_and_iface() -> tuple[str, str]:
    """IP of the default-route interface (UDP connect trick, no packet sent)."""
    ip = ""
    try:
        with socket.socket(socket.AF_INET, socket.SOCK_DGRAM) as s:
            s.connect(("10.255.255.255", 1))
            ip = s.getsockname()[0]
    except OSError:
        pass
    iface = ""
    for name, addrs in psutil.net_if_addrs().items():
        if any(a.family == socket.AF_INET and a.address == ip for a in addrs):
            iface = name
            break
    return ip, iface


def detect_ip_and_mac(cfg: AgentConfig) -> tuple[str, str]:
    ip, iface = primary_ip_and_iface()
    iface = cfg.iface or iface
    mac = cfg.mac
    if not mac and iface:
        for a in psutil.net_if_addrs().get(iface, []):
            if getattr(a, "family", None) == psutil.AF_LINK and a.address and a.address != "00:00:00:00:00:00":
                mac = a.address.lower()
    return ip, mac


def active_job_ids(store) -> set[str]:
    out = set()
    keys = [k for k in (store.smembers("jobs:all") or []) if k.startswith("job:")]
    p = store.pipeline()
    for k in keys:
        p.hget(k, "status")
    for k, s in zip(keys, p.execute() if keys else []):
        if str(s or "").strip().upper() in ACTIVE:
            out.add(k.split(":", 1)[1])
    return out


def remove_stale_projects(base_dir: str, min_age_sec: int, store) -> dict:
    """Delete UUID-named job dirs that are inactive and older than min_age_sec."""
    res = {"removed": 0, "skipped_active": 0, "skipped_recent": 0}
    try:
        names = os.listdir(base_dir)
    except FileNotFoundError:
        return res
    active = active_job_ids(store)
    now = time.time()
    for name in names:
        path = os.path.join(base_dir, name)
        if not os.path.isdir(path) or not _GUID_RE.match(name):
            continue
        if name in active:
            res["skipped_active"] += 1
            continue
        if now - os.path.getmtime(path) < min_age_sec:
            res["skipped_recent"] += 1
            continue
        shutil.rmtree(path, ignore_errors=True)
        res["removed"] += 1
    return res


class Agent:
    def __init__(self, cfg: AgentConfig | None = None, store=None, gpu: GpuSampler | None = None,
                 suspend_fn=None):
        self.cfg = cfg or AgentConfig()
        self.store = store
        self.gpu = gpu if gpu is not None else GpuSampler()
        self.suspend_fn = suspend_fn or (lambda: subprocess.run(["systemctl", "suspend"], check=False))
        self.key = f"metrics:node:{self.cfg.hostname}"
        self.ip, self.mac = "", ""
        self.next_ident = self.next_mac = self.next_role = self.next_gc = 0.0
        self.role = "encode"
        self.idle_since = None
        self.last_suspend = 0.0
        self.last_net = psutil.net_io_counters()
        self.last_ts = time.time()
        self.last_xgmi = None  # (read, write) bytes of the previous sample
        psutil.cpu_percent(interval=None)  # prime

    @property
    def st(self):
        return self.store or get_store()

    # ------------------------------------------------------------- role sync
    def _service_active(self, name: str) -> bool:
        return subprocess.run(["systemctl", "is-active", "--quiet", name], check=False,
                              stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL).returncode == 0

    def _set_service(self, name: str, run: bool) -> None:
        if run != self._service_active(name):
            subprocess.run(["systemctl", "start" if run else "stop", name], check=False)
            log.info("role sync: %s %s", "start" if run else "stop", name)

    def sync_role(self) -> str:
        role = (self.st.hget("pipeline:node_roles", self.cfg.hostname) or "encode").strip().lower()
        role = role if role in ("pipeline", "encode") else "encode"
        if self.cfg.manage_services:
            self._set_service(self.cfg.encode_service, True)
            self._set_service(self.cfg.pipeline_service, role == "pipeline")
        return role

    # ---------------------------------------------------------------- metrics
    def collect(self) -> tuple[dict, dict | None]:
        cpu = psutil.cpu_percent(interval=None)
        vm = psutil.virtual_memory()
        try:
            disk = float(psutil.disk_usage("/").percent)
        except OSError:
            disk = 0.0
        g = self.gpu.sample() if self.gpu else None
        net, ts = psutil.net_io_counters(), time.time()
        dt = max(1e-6, ts - self.last_ts)
        rx = int((net.bytes_recv - self.last_net.bytes_recv) / dt)
        tx = int((net.bytes_sent - self.last_net.bytes_sent) / dt)
        self.last_net, self.last_ts = net, ts
        import json

        payload = {"ts": int(ts), "hostname": self.cfg.hostname, "ip": self.ip, "mac": self.mac, "cpu": float(cpu),
                   "gpu": -1.0 if g is None else float(g["util"]), "mem": float(vm.percent),
                   "mem_used": int(vm.total - vm.available), "mem_total": int(vm.total), "disk": disk,
                   "rx_bps": rx, "tx_bps": tx, "worker_role": self.role,
                   "gpu_count": 0 if g is None else g["gpu_count"], "gpu_name": "" if g is None else g["gpu_name"],
                   "hbm_used": 0 if g is None else g["hbm_used"], "hbm_total": 0 if g is None else g["hbm_total"],
                   "gpus_json": json.dumps([] if g is None else g["gpus"])}
        if g is not None and "xgmi_read_bytes" in g:
            cur = (int(g["xgmi_read_bytes"]), int(g["xgmi_write_bytes"]))
            prev = self.last_xgmi or cur
            payload.update(xgmi_read_bytes=cur[0], xgmi_write_bytes=cur[1],
                           xgmi_rx_bps=max(0, int((cur[0] - prev[0]) / dt)), xgmi_tx_bps=max(0, int((cur[1] - prev[1]) / dt)))
            self.last_xgmi = cur
        return payload, g

    def suspend_settings(self) -> tuple[bool, int, float, bool]:
        s = get_settings()
        idle = as_int(s.get("suspend_idle_sec"), self.cfg.suspend_after_idle_sec)
        cpu = as_float(s.get("suspend_idle_cpu_pct_max"), self.cfg.idle_cpu_pct_max)
        return (self.cfg.suspend_enabled and as_bool(s.get("suspend_enabled"), True),
                idle if idle > 0 else self.cfg.suspend_after_idle_sec,
                cpu if cpu > 0 else self.cfg.idle_cpu_pct_max, as_bool(s.get("suspend_gc_enabled")))

    def tick(self, now: float | None = None) -> dict:
        now = now or time.time()
        st = self.st
        if now >= self.next_ident or not (self.ip and self.mac):
            ip, mac = detect_ip_and_mac(self.cfg)
            self.ip, self.mac = ip or self.ip, mac or self.mac
            self.next_ident = now + 3600
        if self.mac and now >= self.next_mac:
            st.hset("nodes:mac", self.cfg.hostname, self.mac)
            self.next_mac = now + 3600
        if now >= self.next_role:
            try:
                self.role = self.sync_role()
            except Exception as e:
                log.warning("role sync failed: %s", e)
            self.next_role = now + self.cfg.role_sync_interval_sec
        payload, g = self.collect()
        st.hset(self.key, mapping=payload)
        st.expire(self.key, self.cfg.ttl_sec)
        gc = None
        if now >= self.next_gc:
            gc = remove_stale_projects(self.cfg.gc_base_dir, self.cfg.gc_min_age_sec, st)
            self.next_gc = now + self.cfg.gc_interval_sec
        enabled, idle_sec, cpu_max, gc_before = self.suspend_settings()
        gpu_idle = g is None or payload["gpu"] <= self.cfg.idle_gpu_pct_max
        idle = payload["cpu"] <= cpu_max and gpu_idle and all_jobs_are_idle(st)
        action = None
        if idle and enabled:
            self.idle_since = self.idle_since or now
            up = now - psutil.boot_time()
            if (now - self.idle_since >= idle_sec and up >= self.cfg.min_uptime_before_suspend
                    and now - self.last_suspend >= idle_sec):
                if gc_before:
                    remove_stale_projects(self.cfg.gc_base_dir, self.cfg.gc_min_age_sec, st)
                st.delete(self.key)  # drop out of the active set before sleeping
                self.last_suspend = now
                self.idle_since = None
                action = "suspend"
                self.suspend_fn()
        else:
            self.idle_since = None
        return {"payload": payload, "gc": gc, "action": action}

    def run(self) -> None:  # pragma: no cover - service loop
        while True:
            t0 = time.time()
            try:
                self.tick(t0)
            except Exception:
                log.exception("agent tick failed")
            time.sleep(max(0.0, 1.0 - (time.time() - t0)))


def main() -> None:  # pragma: no cover - service entry
    from ..common import get_logging

    get_logging("agent")
    Agent().run()
