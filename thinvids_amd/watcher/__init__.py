"""Folder watcher (reference manager/watcher.py).

Detects new/changed videos under ``WATCH_ROOT`` with a periodic scanner and a polling
observer, waits until a file is stable (size unchanged for STABLE_CHECKS x
STABLE_DELAY_SEC), then POSTs ``/add_job`` once.  A durable **processed ledger**
(``processed.log``: JSON lines ``{"path", "sig"}`` with ``sig = size:mtime_ns``; legacy
path-only lines accepted; ``fcntl.flock`` for appends; reloaded when the file's mtime
moves) prevents re-submission across restarts.  First run bootstraps the ledger with
everything already present; a one-time adopt migration maps legacy entries; path aliases
(``tv=television``) let a renamed library keep its history.
"""
from __future__ import annotations

import fcntl
import json
import logging
import os
import threading
import time
from concurrent.futures import ThreadPoolExecutor

import requests

log = logging.getLogger("thinvids.watcher")
VIDEO_EXTS = {".mkv", ".mp4", ".y4m", ".synth", ".hevc", ".265"}


def _b(v, d=False):
    return d if v is None else str(v).strip().lower() in ("1", "true", "yes", "on")


class WatcherConfig:
    def __init__(self, env=None):
        e = os.environ if env is None else env
        self.watch_root = e.get("WATCH_ROOT", "/watch")
        self.submit_url = e.get("SUBMIT_URL", "http://localhost:5005/add_job")
        self.use_watchdog = _b(e.get("USE_WATCHDOG", "1"))
        self.use_scanner = _b(e.get("USE_SCANNER", "1"))
        self.scan_interval_sec = float(e.get("SCAN_INTERVAL_SEC", "60"))
        self.poll_interval_sec = float(e.get("POLL_INTERVAL_SEC", "2"))
        self.stable_checks = int(e.get("STABLE_CHECKS", "5"))
        self.stable_delay_sec = float(e.get("STABLE_DELAY_SEC", "10"))
        self.workers = int(e.get("WORKERS", "4"))
        self.processed_file = e.get("PROCESSED_FILE", "/config/processed.log")
        self.adopt_on_startup = _b(e.get("ADOPT_EXISTING_PROCESSED_ON_STARTUP", "0"))
        self.adopt_marker = e.get("ADOPT_EXISTING_PROCESSED_MARKER", "").strip()
        self.path_aliases = e.get("PROCESSED_PATH_ALIASES", "").strip()


def signature_from_stat(st: os.stat_result) -> str:
    return f"{int(st.st_size)}:{int(getattr(st, 'st_mtime_ns', int(st.st_mtime * 1e9)))}"


def signature_for_path(path: str) -> str | None:
    try:
        return signature_from_stat(os.stat(path))
    except FileNotFoundError:
        return None


def is_video_file(path: str) -> bool:
    return os.path.splitext(path)[1].lower() in VIDEO_EXTS


def _norm(p: str) -> str:
    return str(p or "").strip().replace("\\", "/").strip("/")


class FileProcessedStore:
    """File-backed processed ledger (reference watcher.py:73-266)."""

    def __init__(self, file_path: str):
        self.file_path = file_path
        self._entries: dict[str, str | None] = {}
        self._adopted: dict[str, str] = {}
        self._lock = threading.Lock()
        self._mtime = 0.0
        os.makedirs(os.path.dirname(file_path) or ".", exist_ok=True)
        self._load()

    @staticmethod
    def _parse(line: str):
        line = (line or "").strip()
        if not line:
            return None, None
        if line.startswith("{"):
            try:
                d = json.loads(line)
            except ValueError:
                return None, None
            sig = d.get("sig")
            return (str(d.get("path") or "").strip() or None), (str(sig).strip() if sig not in (None, "") else None)
        return line, None  # legacy path-only line

    def _load(self):
        try:
            mtime = os.stat(self.file_path).st_mtime
        except FileNotFoundError:
            return
        with open(self.file_path, encoding="utf-8") as f:
            fcntl.flock(f.fileno(), fcntl.LOCK_SH)
            lines = f.readlines()
            fcntl.flock(f.fileno(), fcntl.LOCK_UN)
        entries = {}
        for line in lines:
            rel, sig = self._parse(line)
            if rel:
                entries[rel] = sig
        with self._lock:
            for rel, sig in self._adopted.items():
                if entries.get(rel) is None:
                    entries[rel] = sig
            self._entries, self._mtime = entries, mtime

    def _maybe_reload(self):
        try:
            if os.stat(self.file_path).st_mtime > self._mtime:
                self._load()
        except FileNotFoundError:
            pass

    def _append(self, records):
        with open(self.file_path, "a+", encoding="utf-8") as f:
            fcntl.flock(f.fileno(), fcntl.LOCK_EX)
            for rel, sig in records:
                f.write(json.dumps({"path": rel, "sig": sig}, separators=(",", ":")) + "\n")
            f.flush()
            os.fsync(f.fileno())
            fcntl.flock(f.fileno(), fcntl.LOCK_UN)
        try:
            self._mtime = os.stat(self.file_path).st_mtime
        except FileNotFoundError:
            pass

    def state_for(self, rel: str, sig: str | None) -> str:
        """'missing' | 'legacy' (path-only entry) | 'matched' | 'changed'."""
        self._maybe_reload()
        with self._lock:
            if rel not in self._entries:
                return "missing"
            stored = self._entries[rel]
            if stored is None:
                return "legacy"
            return "matched" if sig and stored == sig else "changed"

    def adopt_legacy(self, rel: str, sig: str) -> bool:
        if not rel or not sig:
            return False
        self._maybe_reload()
        with self._lock:
            if self._entries.get(rel) is not None:
                return False
            self._entries[rel] = sig
            self._adopted[rel] = sig
            return True

    def add(self, rel: str, sig: str) -> None:
        if not rel or not sig:
            return
        self._maybe_reload()
        with self._lock:
            if self._entries.get(rel) == sig:
                return
            self._entries[rel] = sig
            self._adopted.pop(rel, None)
        self._append([(rel, sig)])

    def add_many(self, items) -> None:
        seen, recs = set(), []
        for rel, sig in items:
            rel, sig = str(rel or "").strip(), str(sig or "").strip()
            if rel and sig and rel not in seen:
                seen.add(rel)
                recs.append((rel, sig))
        if not recs:
            return
        self._append(recs)
        with self._lock:
            for rel, sig in recs:
                self._entries[rel] = sig
                self._adopted.pop(rel, None)

    def count(self) -> int:
        self._maybe_reload()
        with self._lock:
            return len(self._entries)


class Watcher:
    def __init__(self, cfg: WatcherConfig | None = None, submit=None):
        self.cfg = cfg or WatcherConfig()
        self.store = FileProcessedStore(self.cfg.processed_file)
        self._submit = submit or self._http_submit
        self._session = requests.Session()
        self._lock = threading.Lock()
        self._pending: set[str] = set()
        self._submitted: dict[str, str] = {}
        self._seen: dict[str, tuple] = {}
        self._stop = threading.Event()
        self._pool = ThreadPoolExecutor(max_workers=max(1, self.cfg.workers))
        self._threads: list[threading.Thread] = []

    # ---------------------------------------------------------------- paths
    def rel_from_watch(self, path: str) -> str:
        try:
            return os.path.relpath(path, self.cfg.watch_root).replace("\\", "/")
        except ValueError:
            return path

    def aliases(self) -> list[tuple[str, str]]:
        out = []
        for raw in self.cfg.path_aliases.split(","):
            if "=" in raw:
                cur, legacy = (_norm(x) for x in raw.split("=", 1))
                if cur and legacy:
                    out.append((cur, legacy))
        return out

    def candidates(self, rel: str):
        rel = _norm(rel)
        out = [rel] if rel else []
        for cur, legacy in self.aliases():
            if rel == cur:
                c = legacy
            elif rel.startswith(cur + "/"):
                c = legacy + rel[len(cur):]
            else:
                continue
            if c not in out:
                out.append(c)
        return out

    def state_for_rel(self, rel: str, sig: str | None) -> tuple[str, str]:
        for c in self.candidates(rel):
            s = self.store.state_for(c, sig)
            if s != "missing":
                return s, c
        return "missing", _norm(rel)

    def _walk(self):
        for root, dirs, files in os.walk(self.cfg.watch_root):
            dirs[:] = [d for d in dirs if not d.startswith(".")]
            for name in files:
                if not name.startswith(".") and is_video_file(name):
                    yield os.path.join(root, name)

    # ------------------------------------------------------------- submit
    def _http_submit(self, rel: str, path: str) -> bool:
        r = self._session.post(self.cfg.submit_url, json={"filename": rel, "input_path": path}, timeout=20)
        if not r.ok:
            log.error("submit failed %s: %s", r.status_code, r.text[:200])
        return r.ok

    def _settle_known(self, path: str, rel: str, sig: str | None) -> bool:
        """True when the file is already accounted for (matched / legacy)."""
        state, ledger_rel = self.state_for_rel(rel, sig)
        if state == "matched":
            if ledger_rel != rel and sig:
                self.store.add(rel, sig)
            return True
        if state == "legacy":
            if sig:
                self.store.add(rel, sig)
            return True
        return False

    def submit_job_if_stable(self, path: str) -> bool:
        rel = self.rel_from_watch(path)
        try:
            if self._settle_known(path, rel, signature_for_path(path)):
                return False
            last, stable = -1, 0
            while not self._stop.is_set():
                try:
                    size = os.path.getsize(path)
                except FileNotFoundError:
                    return False
                if size == last and size > 0:
                    stable += 1
                    if stable >= self.cfg.stable_checks:
                        break
                else:
                    stable, last = 0, size
                time.sleep(self.cfg.stable_delay_sec)
            sig = signature_for_path(path)
            if not sig or self._settle_known(path, rel, sig):
                return False
            log.info("submitting job for %s", rel)
            if self._submit(rel, path):
                self.store.add(rel, sig)
                with self._lock:
                    self._submitted[path] = sig
                return True
            return False
        except Exception:
            log.exception("submit error for %s", rel)
            return False
        finally:
            with self._lock:
                self._pending.discard(path)

    def schedule_submit(self, path: str):
        rel = self.rel_from_watch(path)
        sig = signature_for_path(path)
        if not sig or self._settle_known(path, rel, sig):
            return None
        with self._lock:
            if path in self._pending or self._submitted.get(path) == sig:
                return None
            self._pending.add(path)
        return self._pool.submit(self.submit_job_if_stable, path)

    # ---------------------------------------------------- startup helpers
    def bootstrap_processed_if_first_run(self) -> int:
        if self.store.count() > 0:
            return 0
        recs = [(self.rel_from_watch(p), signature_for_path(p)) for p in self._walk()]
        recs = [(r, s) for r, s in recs if s]
        self.store.add_many(recs)
        log.info("bootstrap: marked %d existing files as processed", len(recs))
        return len(recs)

    def adopt_marker_file(self) -> str:
        if self.cfg.adopt_marker:
            return self.cfg.adopt_marker
        safe = self.cfg.watch_root.strip(os.sep).replace(os.sep, "_") or "root"
        return f"{self.cfg.processed_file}.{safe}.adopted"

    def adopt_existing_processed_once(self) -> int:
        """One-time migration: files under the (moved) root whose relative path was already
        processed under an alias / legacy entry are adopted with their current signature."""
        marker = self.adopt_marker_file()
        if not self.cfg.adopt_on_startup or os.path.exists(marker):
            return 0
        n = 0
        recs = []
        for p in self._walk():
            rel, sig = self.rel_from_watch(p), signature_for_path(p)
            state, ledger_rel = self.state_for_rel(rel, sig)
            if sig and state in ("legacy", "changed") or (sig and state == "matched" and ledger_rel != rel):
                recs.append((rel, sig))
                n += 1
        self.store.add_many(recs)
        with open(marker, "w") as f:
            f.write(json.dumps({"adopted": n, "at": time.time()}) + "\n")
        return n

    # --------------------------------------------------------------- loops
    def scan_once(self) -> int:
        n = 0
        for p in self._walk():
            if self.schedule_submit(p) is not None:
                n += 1
        return n

    def _scanner(self):
        while not self._stop.wait(self.cfg.scan_interval_sec):
            try:
                self.scan_once()
            except Exception:
                log.exception("scanner pass failed")

    def _observer(self):
        """Polling observer (the reference uses watchdog's PollingObserver): reacts to new
        or modified files between full scanner passes."""
        for p in self._walk():
            try:
                st = os.stat(p)
                self._seen[p] = (st.st_size, st.st_mtime_ns)
            except FileNotFoundError:
                pass
        while not self._stop.wait(self.cfg.poll_interval_sec):
            for p in self._walk():
                try:
                    st = os.stat(p)
                except FileNotFoundError:
                    continue
                key = (st.st_size, st.st_mtime_ns)
                if self._seen.get(p) != key:
                    self._seen[p] = key
                    self.schedule_submit(p)

    def start(self) -> "Watcher":
        os.makedirs(self.cfg.watch_root, exist_ok=True)
        self.bootstrap_processed_if_first_run()
        self.adopt_existing_processed_once()
        if self.cfg.use_scanner:
            self._threads.append(threading.Thread(target=self._scanner, name="watch-scanner", daemon=True))
        if self.cfg.use_watchdog:
            self._threads.append(threading.Thread(target=self._observer, name="watch-observer", daemon=True))
        for t in self._threads:
            t.start()
        return self

    def stop(self):
        self._stop.set()
        for t in self._threads:
            t.join(timeout=5)
        self._pool.shutdown(wait=False, cancel_futures=True)


def mark_processed(path: str, watch_root: str, processed_file: str) -> str:
    """Used by the manager's ``add_job {mark_watcher_processed: true}``."""
    sig = signature_for_path(path)
    if not sig:
        raise FileNotFoundError(path)
    rel = os.path.relpath(path, watch_root).replace("\\", "/")
    FileProcessedStore(processed_file).add(rel, sig)
    return rel


def main() -> None:  # pragma: no cover - service entry
    from ..common import get_logging

    get_logging("watcher")
    w = Watcher().start()
    log.info("watching %s -> %s", w.cfg.watch_root, w.cfg.submit_url)
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        w.stop()
