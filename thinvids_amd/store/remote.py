"""Client for :mod:`thinvids_amd.store.server` with the LocalStore / redis-py API subset.

Retries connection failures with capped exponential backoff, like the reference's redis
client configuration (``Retry(ExponentialBackoff(cap=10, base=1), retries=16)``,
reference common.py:33-46).
"""
from __future__ import annotations

import json
import socket
import threading
import time


def _dec(v):
    if isinstance(v, dict) and "__set__" in v:
        return set(v["__set__"])
    if isinstance(v, dict) and "__err__" in v:
        return RuntimeError(v["__err__"])
    return v


class RemoteError(RuntimeError):
    pass


class RemoteStore:
    def __init__(self, host: str = "127.0.0.1", port: int = 6390, timeout: float = 30.0,
                 retries: int = 16, backoff_cap: float = 10.0):
        self.addr = (host, port)
        self.timeout = timeout
        self.retries = retries
        self.backoff_cap = backoff_cap
        self._local = threading.local()  # one connection per thread (blocking ops)

    def _conn(self):
        c = getattr(self._local, "conn", None)
        if c is None:
            s = socket.create_connection(self.addr, timeout=self.timeout)
            c = (s, s.makefile("rb"))
            self._local.conn = c
        return c

    def _reset(self):
        c = getattr(self._local, "conn", None)
        if c is not None:
            try:
                c[0].close()
            except OSError:
                pass
        self._local.conn = None

    def _call(self, msg: dict, timeout: float | None = None):
        delay = 1.0
        for attempt in range(self.retries + 1):
            try:
                s, f = self._conn()
                s.settimeout(timeout if timeout is not None else self.timeout)
                s.sendall((json.dumps(msg) + "\n").encode())
                line = f.readline()
                if not line:
                    raise ConnectionError("store closed the connection")
                resp = json.loads(line)
                if "err" in resp:
                    raise RemoteError(resp["err"])
                return resp["ok"]
            except (OSError, ConnectionError):
                self._reset()
                if attempt == self.retries:
                    raise
                time.sleep(delay)
                delay = min(self.backoff_cap, delay * 2)

    def __getattr__(self, op):
        if op.startswith("_"):
            raise AttributeError(op)

        def call(*args, **kwargs):
            t = None
            if op == "blpop":
                to = kwargs.get("timeout", args[1] if len(args) > 1 else 0)
                t = (float(to) + self.timeout) if to else None
            r = _dec(self._call({"op": op, "args": list(args), "kwargs": kwargs}, timeout=t))
            if op == "blpop" and r is not None:
                return tuple(r)
            return r

        return call

    def scan_iter(self, match: str = "*", count: int | None = None):
        return iter(self.keys(match))

    def pipeline(self, transaction: bool = False):
        return _RemotePipeline(self)


class _RemotePipeline:
    def __init__(self, store: RemoteStore):
        self._store = store
        self._cmds: list = []

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)

        def queue(*args, **kwargs):
            self._cmds.append([name, list(args), kwargs])
            return self

        return queue

    def execute(self, raise_on_error: bool = True):
        cmds, self._cmds = self._cmds, []
        res = [_dec(r) for r in self._store._call({"batch": cmds})]
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
