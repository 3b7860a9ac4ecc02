"""TCP server exposing a :class:`LocalStore` to other processes / hosts.

Stands in for the reference's Redis server (``REDIS_HOST``, reference common.py:23-31,
ansible_workers.yml:20) so the manager, watcher, agents and per-GPU worker processes can
share the same job hashes, heartbeats and queues.  Protocol: one JSON object per line,
``{"op": name, "args": [...], "kwargs": {...}}`` or ``{"batch": [[name, args, kwargs], ...]}``
-> ``{"ok": result}`` / ``{"err": message}``.

    python -m thinvids_amd.store.server --host 0.0.0.0 --port 6390
"""
from __future__ import annotations

import argparse
import json
import socketserver
import threading

from .local import LocalStore


def _check_op(op: str) -> str:
    """The allow-list of remotely callable ops (shared with batches and pipelines)."""
    from .local import Pipeline

    if not isinstance(op, str) or op not in Pipeline._ALLOWED and op != "blpop":
        raise ValueError(f"op not allowed: {op}")
    return op


def _enc(v):
    if isinstance(v, set):
        return {"__set__": sorted(v)}
    if isinstance(v, tuple):
        return list(v)
    if isinstance(v, Exception):
        return {"__err__": str(v)}
    return v


class _Handler(socketserver.StreamRequestHandler):
    def handle(self):
        store: LocalStore = self.server.store  # type: ignore[attr-defined]
        for line in self.rfile:
            if not line.strip():
                continue
            try:
                msg = json.loads(line)
                if "batch" in msg:
                    res = store.execute_batch([(_check_op(n), a, k) for n, a, k in msg["batch"]])
                    out = {"ok": [_enc(r) for r in res]}
                else:
                    op = _check_op(msg["op"])
                    res = getattr(store, op)(*msg.get("args", []), **msg.get("kwargs", {}))
                    out = {"ok": _enc(res)}
            except Exception as e:  # report to the client, keep serving
                out = {"err": f"{type(e).__name__}: {e}"}
            self.wfile.write((json.dumps(out) + "\n").encode())
            self.wfile.flush()


class StoreServer(socketserver.ThreadingTCPServer):
    daemon_threads = True
    allow_reuse_address = True

    def __init__(self, host: str = "127.0.0.1", port: int = 6390, store: LocalStore | None = None):
        self.store = store or LocalStore()
        super().__init__((host, port), _Handler)

    def start_background(self) -> threading.Thread:
        t = threading.Thread(target=self.serve_forever, name="tv-store", daemon=True)
        t.start()
        return t


def main() -> None:
    ap = argparse.ArgumentParser(description="thinvids-amd state store server")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=6390)
    a = ap.parse_args()
    srv = StoreServer(a.host, a.port)
    print(f"store listening on {a.host}:{srv.server_address[1]}", flush=True)
    srv.serve_forever()


if __name__ == "__main__":
    main()
