"""State store factory (reference common.py:33-46 `get_redis`).

``TV_STORE`` selects the backend:

* ``local`` (default) — one in-process :class:`LocalStore` shared by every thread;
* ``tcp://host:port`` — :class:`RemoteStore` against ``python -m thinvids_amd.store.server``;
* ``redis://host:port/db`` — a real redis-py client if the package is installed.
"""
from __future__ import annotations

import os
import threading
from urllib.parse import urlparse

from .local import LocalStore, Pipeline  # noqa: F401
from .remote import RemoteStore  # noqa: F401

_lock = threading.Lock()
_store = None


def make_store(url: str | None = None):
    url = url or os.environ.get("TV_STORE", "local")
    if url in ("", "local", "memory"):
        return LocalStore()
    u = urlparse(url)
    if u.scheme == "tcp":
        return RemoteStore(u.hostname or "127.0.0.1", u.port or 6390)
    if u.scheme == "redis":
        try:
            import redis  # type: ignore
        except ImportError as e:  # pragma: no cover - redis-py not in this image
            raise RuntimeError("TV_STORE=redis://... requires redis-py") from e
        db = int((u.path or "/1").strip("/") or 1)
        return redis.Redis(host=u.hostname, port=u.port or 6379, db=db, decode_responses=True,
                           socket_timeout=5, socket_connect_timeout=5)
    raise ValueError(f"unsupported TV_STORE {url!r}")


def get_store():
    """Process-wide store singleton."""
    global _store
    with _lock:
        if _store is None:
            _store = make_store()
        return _store


def set_store(store) -> None:
    """Install a store (tests / embedded deployments)."""
    global _store
    with _lock:
        _store = store


# reference-compatible name
get_redis = get_store


_HMAX_LUA = ("local v = tonumber(redis.call('HGET', KEYS[1], ARGV[1]) or '0') or 0 "
             "local n = tonumber(ARGV[2]) if n > v then redis.call('HSET', KEYS[1], ARGV[1], n) v = n end "
             "return v")


def hmax(st, key, field, value) -> int:
    """Atomically raise hash field `field` of `key` to at least `value` (monotone progress
    counters written by several ranks: a read-then-write could move them backwards)."""
    if hasattr(st, "hmax"):
        return int(st.hmax(key, field, int(value)))
    return int(st.eval(_HMAX_LUA, 1, key, field, int(value)))  # redis-py
