"""In-process state store with the Redis command subset thinvids uses.

The reference keeps all cross-process state in Redis DB1 (reference common.py:33-46) and
its job queues in Redis DB0 via Huey (common.py:49-64).  Neither redis nor huey exists in
this image, so the control plane talks to a `StateStore` with Redis semantics
(decode_responses=True: every value is a str):

* :class:`LocalStore`  — thread-safe dict store with TTLs and blocking list pops;
* :class:`thinvids_amd.store.remote.RemoteStore` — the same API over TCP to a
  :class:`thinvids_amd.store.server.StoreServer` (multi-process / multi-host);
* a real ``redis.Redis`` when redis-py is installed (``TV_STORE=redis://...``).

Keys and field names follow the reference contract.
"""
from __future__ import annotations

import fnmatch
import threading
import time
from typing import Any, Iterable


def _s(v: Any) -> str:
    if isinstance(v, bytes):
        return v.decode()
    if isinstance(v, bool):
        return "1" if v else "0"
    if isinstance(v, float):
        r = repr(v)
        return r[:-2] if r.endswith(".0") else r
    return str(v)


class WrongType(TypeError):
    pass


class LocalStore:
    def __init__(self):
        self._d: dict[str, Any] = {}
        self._exp: dict[str, float] = {}
        self._lock = threading.RLock()
        self._cv = threading.Condition(self._lock)

    # ------------------------------------------------------------------ internals
    def _alive(self, key: str) -> bool:
        e = self._exp.get(key)
        if e is not None and e <= time.time():
            self._d.pop(key, None)
            self._exp.pop(key, None)
            return False
        return key in self._d

    def _get(self, key: str, typ):
        if not self._alive(key):
            return None
        v = self._d[key]
        if not isinstance(v, typ):
            raise WrongType(f"WRONGTYPE Operation against a key holding the wrong kind of value: {key}")
        return v

    def _new(self, key: str, typ):
        v = self._get(key, typ)
        if v is None:
            v = typ()
            self._d[key] = v
        return v

    def _drop_if_empty(self, key: str):
        v = self._d.get(key)
        if v is not None and not isinstance(v, str) and len(v) == 0:
            self._d.pop(key, None)
            self._exp.pop(key, None)

    # ------------------------------------------------------------------ generic
    def ping(self) -> bool:
        return True

    def delete(self, *keys) -> int:
        with self._lock:
            n = 0
            for k in keys:
                k = _s(k)
                if self._alive(k):
                    n += 1
                self._d.pop(k, None)
                self._exp.pop(k, None)
            return n

    def exists(self, *keys) -> int:
        with self._lock:
            return sum(1 for k in keys if self._alive(_s(k)))

    def expire(self, key, seconds) -> bool:
        with self._lock:
            key = _s(key)
            if not self._alive(key):
                return False
            self._exp[key] = time.time() + float(seconds)
            return True

    def persist(self, key) -> bool:
        with self._lock:
            return self._exp.pop(_s(key), None) is not None

    def ttl(self, key) -> int:
        with self._lock:
            key = _s(key)
            if not self._alive(key):
                return -2
            e = self._exp.get(key)
            return -1 if e is None else max(0, int(round(e - time.time())))

    def keys(self, pattern: str = "*") -> list[str]:
        with self._lock:
            return [k for k in list(self._d) if self._alive(k) and fnmatch.fnmatchcase(k, pattern)]

    def scan_iter(self, match: str = "*", count: int | None = None) -> Iterable[str]:
        return iter(self.keys(match))

    def type(self, key) -> str:
        with self._lock:
            key = _s(key)
            if not self._alive(key):
                return "none"
            v = self._d[key]
            return {str: "string", dict: "hash", set: "set", list: "list"}[type(v)]

    def flushdb(self) -> bool:
        with self._lock:
            self._d.clear()
            self._exp.clear()
            return True

    # ------------------------------------------------------------------ strings
    def get(self, key):
        with self._lock:
            return self._get(_s(key), str)

    def set(self, key, value, ex=None, px=None, nx=False, xx=False):
        with self._lock:
            key = _s(key)
            present = self._alive(key)
            if (nx and present) or (xx and not present):
                return None
            self._d[key] = _s(value)
            self._exp.pop(key, None)
            if ex is not None:
                self._exp[key] = time.time() + float(ex)
            elif px is not None:
                self._exp[key] = time.time() + float(px) / 1000.0
            return True

    def setnx(self, key, value) -> bool:
        return bool(self.set(key, value, nx=True))

    def incrby(self, key, amount=1) -> int:
        with self._lock:
            key = _s(key)
            v = int(self._get(key, str) or 0) + int(amount)
            self._d[key] = str(v)
            return v

    def incr(self, key, amount=1) -> int:
        return self.incrby(key, amount)

    def mget(self, keys, *more):
        ks = list(keys) if isinstance(keys, (list, tuple)) else [keys]
        ks += list(more)
        with self._lock:
            return [self._get(_s(k), str) for k in ks]

    # ------------------------------------------------------------------ hashes
    def hget(self, key, field):
        with self._lock:
            h = self._get(_s(key), dict)
            return None if h is None else h.get(_s(field))

    def hset(self, key, field=None, value=None, mapping=None) -> int:
        with self._lock:
            h = self._new(_s(key), dict)
            n = 0
            items = list((mapping or {}).items())
            if field is not None:
                items.append((field, value))
            for f, v in items:
                f = _s(f)
                n += f not in h
                h[f] = _s(v)
            return n

    def hmset(self, key, mapping) -> bool:
        self.hset(key, mapping=mapping)
        return True

    def hsetnx(self, key, field, value) -> bool:
        with self._lock:
            h = self._new(_s(key), dict)
            if _s(field) in h:
                return False
            h[_s(field)] = _s(value)
            return True

    def hgetall(self, key) -> dict:
        with self._lock:
            h = self._get(_s(key), dict)
            return dict(h) if h else {}

    def hmget(self, key, fields, *more):
        fs = list(fields) if isinstance(fields, (list, tuple)) else [fields]
        fs += list(more)
        with self._lock:
            h = self._get(_s(key), dict) or {}
            return [h.get(_s(f)) for f in fs]

    def hdel(self, key, *fields) -> int:
        with self._lock:
            h = self._get(_s(key), dict)
            if not h:
                return 0
            n = sum(1 for f in fields if h.pop(_s(f), None) is not None)
            self._drop_if_empty(_s(key))
            return n

    def hexists(self, key, field) -> bool:
        with self._lock:
            h = self._get(_s(key), dict)
            return bool(h) and _s(field) in h

    def hkeys(self, key) -> list:
        return list(self.hgetall(key).keys())

    def hlen(self, key) -> int:
        return len(self.hgetall(key))

    def hincrby(self, key, field, amount=1) -> int:
        with self._lock:
            h = self._new(_s(key), dict)
            v = int(float(h.get(_s(field), "0") or 0)) + int(amount)
            h[_s(field)] = str(v)
            return v

    def hmax(self, key, field, value) -> int:
        """Atomic max of an integer hash field (raise it to `value` unless it is already
        higher); returns the field's value afterwards.  Redis has no HMAX: on redis-py the
        store.hmax() helper runs the same as one Lua script."""
        with self._lock:
            h = self._new(_s(key), dict)
            v = max(int(float(h.get(_s(field), "0") or 0)), int(value))
            h[_s(field)] = str(v)
            return v

    def hincrbyfloat(self, key, field, amount=1.0) -> float:
        with self._lock:
            h = self._new(_s(key), dict)
            v = float(h.get(_s(field), "0") or 0) + float(amount)
            h[_s(field)] = _s(v)
            return v

    # ------------------------------------------------------------------ sets
    def sadd(self, key, *members) -> int:
        with self._lock:
            s = self._new(_s(key), set)
            n = 0
            for m in members:
                m = _s(m)
                n += m not in s
                s.add(m)
            return n

    def srem(self, key, *members) -> int:
        with self._lock:
            s = self._get(_s(key), set)
            if not s:
                return 0
            n = 0
            for m in members:
                if _s(m) in s:
                    s.discard(_s(m))
                    n += 1
            self._drop_if_empty(_s(key))
            return n

    def smembers(self, key) -> set:
        with self._lock:
            s = self._get(_s(key), set)
            return set(s) if s else set()

    def sismember(self, key, member) -> bool:
        with self._lock:
            s = self._get(_s(key), set)
            return bool(s) and _s(member) in s

    def scard(self, key) -> int:
        return len(self.smembers(key))

    # ------------------------------------------------------------------ lists
    def lpush(self, key, *values) -> int:
        with self._cv:
            lst = self._new(_s(key), list)
            for v in values:
                lst.insert(0, _s(v))
            self._cv.notify_all()
            return len(lst)

    def rpush(self, key, *values) -> int:
        with self._cv:
            lst = self._new(_s(key), list)
            lst.extend(_s(v) for v in values)
            self._cv.notify_all()
            return len(lst)

    def lpop(self, key):
        with self._lock:
            lst = self._get(_s(key), list)
            if not lst:
                return None
            v = lst.pop(0)
            self._drop_if_empty(_s(key))
            return v

    def rpop(self, key):
        with self._lock:
            lst = self._get(_s(key), list)
            if not lst:
                return None
            v = lst.pop()
            self._drop_if_empty(_s(key))
            return v

    def blpop(self, keys, timeout: float = 0):
        """Blocking left pop over several lists; returns (key, value) or None on timeout."""
        ks = [_s(k) for k in (keys if isinstance(keys, (list, tuple)) else [keys])]
        deadline = None if not timeout else time.time() + float(timeout)
        with self._cv:
            while True:
                for k in ks:
                    v = self.lpop(k)
                    if v is not None:
                        return (k, v)
                left = None if deadline is None else deadline - time.time()
                if left is not None and left <= 0:
                    return None
                self._cv.wait(timeout=min(left, 1.0) if left is not None else 1.0)

    def lrange(self, key, start: int, end: int) -> list:
        with self._lock:
            lst = self._get(_s(key), list) or []
            n = len(lst)
            start = max(0, n + start if start < 0 else start)
            end = n + end if end < 0 else end
            return list(lst[start:end + 1])

    def ltrim(self, key, start: int, end: int) -> bool:
        with self._lock:
            lst = self._get(_s(key), list)
            if lst is None:
                return True
            n = len(lst)
            s = max(0, n + start if start < 0 else start)
            e = n + end if end < 0 else end
            lst[:] = lst[s:e + 1]
            self._drop_if_empty(_s(key))
            return True

    def llen(self, key) -> int:
        with self._lock:
            return len(self._get(_s(key), list) or [])

    def lrem(self, key, count: int, value) -> int:
        with self._lock:
            lst = self._get(_s(key), list)
            if not lst:
                return 0
            value = _s(value)
            removed = 0
            if count >= 0:
                i = 0
                while i < len(lst) and (count == 0 or removed < count):
                    if lst[i] == value:
                        lst.pop(i)
                        removed += 1
                    else:
                        i += 1
            else:
                i = len(lst) - 1
                while i >= 0 and removed < -count:
                    if lst[i] == value:
                        lst.pop(i)
                        removed += 1
                    i -= 1
            self._drop_if_empty(_s(key))
            return removed

    # ------------------------------------------------------------------ pipeline
    def pipeline(self, transaction: bool = False):
        return Pipeline(self)

    # apply a batch of (name, args, kwargs) atomically; used by pipelines and the server
    def execute_batch(self, cmds: list) -> list:
        """Run buffered commands atomically.  Only public data ops are callable: no private
        methods, no nested pipelines/batches and no blocking ``blpop`` (its condition wait
        would release the lock mid-batch and could park the calling thread forever)."""
        bad = [c[0] for c in cmds if c[0] not in Pipeline._ALLOWED]
        if bad:
            raise ValueError(f"op not allowed in a batch: {bad[0]}")
        with self._lock:
            out = []
            for name, args, kwargs in cmds:
                try:
                    out.append(getattr(self, name)(*args, **kwargs))
                except Exception as e:  # mirror redis-py: errors are returned in place
                    out.append(e)
            return out


class Pipeline:
    """Buffered commands executed atomically by `execute()` (redis-py Pipeline subset)."""

    _ALLOWED = {n for n in dir(LocalStore) if not n.startswith("_") and n not in ("pipeline", "execute_batch", "blpop")}

    def __init__(self, store):
        self._store = store
        self._cmds: list = []

    def __getattr__(self, name):
        if name not in self._ALLOWED:
            raise AttributeError(name)

        def queue(*args, **kwargs):
            self._cmds.append((name, list(args), kwargs))
            return self

        return queue

    def execute(self, raise_on_error: bool = True) -> list:
        cmds, self._cmds = self._cmds, []
        res = self._store.execute_batch(cmds)
        if raise_on_error:
            for r in res:
                if isinstance(r, Exception):
                    raise r
        return res

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self._cmds = []
        return False
