"""Fault injection hooks (SURVEY.md §5.3 "explicit fault-injection hooks for tests").

The reference has no fault injection: its retry paths (per-part re-enqueue,
worker/tasks.py:1385-1464; stitcher head-of-line redispatch, :1943-2026; watchdog,
manager/app.py:1420-1457) are only exercised by real failures on the cluster.  Here every
failure path can be driven deterministically from the environment:

    TV_FAULT="part:3:fail"               encode of part 3 raises (every attempt)
    TV_FAULT="part:3:fail:2"             ... only the first 2 attempts (then succeeds)
    TV_FAULT="upload:2:fail:1"           delivery of part 2 fails once
    TV_FAULT="segment:5:fail:1"          node job: segment 5 fails once (retried by any rank)
    TV_FAULT="rank:1:hang:30"            node job: rank 1 sleeps 30 s before its first segment
    TV_FAULT="rank:1:die:1"              node job: rank 1 exits (code 86) the first time
    TV_FAULT="stitch:*:fail"             stitch raises

Several specs are separated by commas.  ``key`` is an integer index or ``*``.  The
optional count limits how many times a spec fires; counts are kept per process, or in
``TV_FAULT_STATE`` (a directory) so that "fail once" survives an elastic restart of the
whole process group (torchrun --max-restarts).
"""
from __future__ import annotations

import os
import threading
import time
from dataclasses import dataclass

EXIT_CODE = 86


class InjectedFault(RuntimeError):
    """Raised by :func:`check` for a ``fail`` spec."""


@dataclass
class Spec:
    kind: str
    key: str
    action: str
    arg: float | None

    def matches(self, kind: str, key) -> bool:
        return self.kind == kind and (self.key == "*" or self.key == str(key))


_lock = threading.Lock()
_fired: dict[str, int] = {}


def parse(text: str | None) -> list[Spec]:
    out = []
    for item in (text or "").split(","):
        item = item.strip()
        if not item:
            continue
        f = item.split(":")
        if len(f) < 3 or f[2] not in ("fail", "hang", "die"):
            raise ValueError(f"bad TV_FAULT spec {item!r} (kind:key:fail|hang|die[:n])")
        out.append(Spec(f[0], f[1], f[2], float(f[3]) if len(f) > 3 and f[3] else None))
    return out


def _fire_count(tag: str) -> int:
    """Times `tag` has fired so far (process-local, or persisted under TV_FAULT_STATE)."""
    d = os.environ.get("TV_FAULT_STATE")
    if d:
        try:
            return len([n for n in os.listdir(d) if n.startswith(tag + ".")])
        except FileNotFoundError:
            return 0
    return _fired.get(tag, 0)


def _record(tag: str) -> None:
    d = os.environ.get("TV_FAULT_STATE")
    if d:
        os.makedirs(d, exist_ok=True)
        n = _fire_count(tag)
        with open(os.path.join(d, f"{tag}.{n}.{os.getpid()}"), "w") as f:
            f.write(str(time.time()))
    else:
        _fired[tag] = _fired.get(tag, 0) + 1


def check(kind: str, key="*") -> None:
    """Apply the first matching TV_FAULT spec for (kind, key), if any."""
    specs = parse(os.environ.get("TV_FAULT"))
    for i, s in enumerate(specs):
        if not s.matches(kind, key):
            continue
        tag = f"{i}-{s.kind}-{s.key}-{s.action}-{key}".replace("*", "any").replace("/", "_")
        with _lock:
            limit = s.arg if s.action in ("fail", "die") else None
            if limit is not None and _fire_count(tag) >= int(limit):
                continue
            _record(tag)
        if s.action == "fail":
            raise InjectedFault(f"injected fault: {kind} {key}")
        if s.action == "hang":
            time.sleep(s.arg if s.arg is not None else 3600.0)
            return
        if s.action == "die":
            os._exit(EXIT_CODE)


def active() -> bool:
    return bool(os.environ.get("TV_FAULT"))
