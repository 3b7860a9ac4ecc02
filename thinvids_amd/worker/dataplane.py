"""Worker data-plane HTTP server (reference worker/tasks.py:663-806).

One threaded server per worker process (default :8000), acting both as the *master*
(serves raw parts) and the *stitcher* (accepts encoded parts):

* ``GET /job/<id>/part/<idx>``   -> raw part (YUV4MPEG2) from ``parts/part_%03d.y4m``;
* ``PUT /job/<id>/result/<idx>`` -> encoded part, streamed in 1 MiB chunks to
  ``encoded/enc_%03d.mp4.<uuid>.uploading`` and atomically renamed;
* ``GET /healthz``.

This is the *inter-node* path.  Inside one MI355X node the bench/SPMD runner moves frames
and bitstreams with RCCL over xGMI instead (:mod:`thinvids_amd.parallel`).
"""
from __future__ import annotations

import logging
import os
import shutil
import threading
import urllib.request
import uuid
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from urllib.parse import urlparse

from ..common import emit_activity
from ..store import get_store
from .config import get_config
from .helpers import elapsed_ms, ensure_dirs, job_key, job_title, now, part_paths

log = logging.getLogger("thinvids.worker.http")
CHUNK = 1024 * 1024


def _parse(path: str):
    parts = urlparse(path).path.split("/")
    if len(parts) != 5 or parts[1] != "job" or parts[3] not in ("part", "result"):
        return None
    try:
        idx = int(parts[4])
    except ValueError:
        return None
    if not 1 <= idx <= 99999 or not parts[2] or "/" in parts[2] or ".." in parts[2]:
        return None
    return parts[2], parts[3], idx


class _Handler(BaseHTTPRequestHandler):
    server_version = "ThinvidsParts/2.0"
    protocol_version = "HTTP/1.1"

    def log_message(self, fmt, *args):  # route through logging, quietly
        log.debug("HTTP %s - " + fmt, self.address_string(), *args)

    @property
    def store(self):
        return self.server.store or get_store()

    def do_GET(self):
        if self.path == "/healthz":
            body = b"ok"
            self.send_response(200)
            self.send_header("Content-Length", str(len(body)))
            self.end_headers()
            self.wfile.write(body)
            return
        r = _parse(self.path)
        if r is None or r[1] != "part":
            self.send_error(404, "Not found")
            return
        job_id, _, idx = r
        path, _ = part_paths(job_id, idx, store=self.store)
        if not os.path.isfile(path):
            self.send_error(404, "Part not found")
            return
        try:
            self.send_response(200)
            self.send_header("Content-Type", "video/x-yuv4mpeg")
            self.send_header("Content-Length", str(os.path.getsize(path)))
            self.end_headers()
            with open(path, "rb") as f:
                shutil.copyfileobj(f, self.wfile, CHUNK)
        except (BrokenPipeError, ConnectionResetError):
            pass

    def do_PUT(self):
        r = _parse(self.path)
        if r is None or r[1] != "result":
            self.send_error(404, "Not found")
            return
        job_id, _, idx = r
        length = self.headers.get("Content-Length")
        try:
            remaining = int(length)
            if remaining < 0:
                raise ValueError
        except (TypeError, ValueError):
            self.send_error(411 if length is None else 400, "Content-Length required")
            return
        st = self.store
        job = st.hgetall(job_key(job_id)) or {}
        t0 = now()
        _, enc = part_paths(job_id, idx, job)
        tmp = f"{enc}.{uuid.uuid4().hex}.uploading"
        try:
            ensure_dirs(os.path.dirname(enc))
            with open(tmp, "wb") as f:
                while remaining > 0:
                    chunk = self.rfile.read(min(CHUNK, remaining))
                    if not chunk:
                        break
                    f.write(chunk)
                    remaining -= len(chunk)
            if remaining:
                os.remove(tmp)
                self.send_error(400, "Incomplete upload")
                return
            os.replace(tmp, enc)
        except Exception as e:  # never leave a half-written temp behind
            try:
                os.remove(tmp)
            except OSError:
                pass
            log.exception("PUT failed")
            self.send_error(500, f"PUT error: {e}")
            return
        emit_activity(f'Stitching "{job_title(job)}" part {idx} completed in {elapsed_ms(t0)}ms',
                      job_id=job_id, filename=job.get("filename") or "", stage="stitch", source="worker",
                      store=st)
        self.send_response(200)
        self.send_header("Content-Length", "0")
        self.end_headers()


class PartServer(ThreadingHTTPServer):
    daemon_threads = True
    allow_reuse_address = True

    def __init__(self, host: str = "0.0.0.0", port: int = 8000, store=None):
        super().__init__((host, port), _Handler)
        self.store = store
        self._thread: threading.Thread | None = None

    @property
    def port(self) -> int:
        return self.server_address[1]

    def start(self) -> "PartServer":
        self._thread = threading.Thread(target=self.serve_forever, kwargs={"poll_interval": 0.25},
                                        name="tv-dataplane", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self.shutdown()
        self.server_close()


_server: PartServer | None = None
_lock = threading.Lock()


def start_http_once(store=None) -> PartServer:
    global _server
    with _lock:
        if _server is None:
            cfg = get_config()
            _server = PartServer(cfg.http_bind_host, cfg.http_port, store).start()
            log.info("data plane listening on %s:%d", cfg.http_bind_host, _server.port)
        return _server


def advertised_endpoint() -> str:
    """``host:port`` other workers use to reach this process's data plane."""
    cfg = get_config()
    if cfg.http_advertise:
        return cfg.http_advertise
    port = _server.port if _server is not None else cfg.http_port
    return f"{cfg.worker_name}:{port}"


# ------------------------------------------------------------------------- clients
def fetch_part(endpoint: str, job_id: str, idx: int, dest: str, timeout: float | None = None) -> int:
    """GET a raw part into `dest` (atomic); returns bytes written."""
    url = f"http://{endpoint}/job/{job_id}/part/{idx}"
    tmp = f"{dest}.{uuid.uuid4().hex}.part"
    ensure_dirs(os.path.dirname(dest))
    n = 0
    try:
        with urllib.request.urlopen(url, timeout=timeout or get_config().http_timeout_sec) as r, open(tmp, "wb") as f:
            while True:
                chunk = r.read(CHUNK)
                if not chunk:
                    break
                f.write(chunk)
                n += len(chunk)
        os.replace(tmp, dest)
    finally:
        if os.path.exists(tmp):
            os.remove(tmp)
    return n


def upload_result(endpoint: str, job_id: str, idx: int, data: bytes, timeout: float | None = None) -> None:
    req = urllib.request.Request(f"http://{endpoint}/job/{job_id}/result/{idx}", data=data, method="PUT",
                                 headers={"Content-Length": str(len(data)), "Content-Type": "video/mp4"})
    with urllib.request.urlopen(req, timeout=timeout or get_config().http_timeout_sec) as r:
        if r.status != 200:
            raise RuntimeError(f"upload of part {idx} failed: HTTP {r.status}")
