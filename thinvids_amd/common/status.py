"""Job status model (reference common.py:72-97).

String-valued so it persists in the state store / JSON unchanged.  `parse` is lenient
(case-insensitive, accepts Status instances) and maps the legacy ``COMPLETED`` value to
DONE, which the reference readers did ad hoc (manager/app.py:953-961, :1976-1978).
"""
from __future__ import annotations

from enum import Enum


class Status(str, Enum):
    READY = "READY"
    STARTING = "STARTING"
    WAITING = "WAITING"
    RUNNING = "RUNNING"
    STAMPING = "STAMPING"
    STOPPED = "STOPPED"
    FAILED = "FAILED"
    REJECTED = "REJECTED"
    DONE = "DONE"

    @staticmethod
    def parse(value) -> "Status":
        if isinstance(value, Status):
            return value
        raw = str(value if value is not None else "").strip().upper()
        if raw == "COMPLETED":
            return Status.DONE
        try:
            return Status[raw]
        except KeyError:
            raise ValueError(f"Unknown Status: {value!r}") from None

    @staticmethod
    def parse_or(value, default: "Status") -> "Status":
        try:
            return Status.parse(value)
        except ValueError:
            return default


ACTIVE_STATUSES = (Status.RUNNING, Status.WAITING, Status.STARTING, Status.STAMPING)
TERMINAL_STATUSES = (Status.DONE, Status.FAILED, Status.STOPPED, Status.REJECTED)
# UI ordering used by the job list sort (reference manager/app.py status_order)
STATUS_ORDER = {s.value: i for i, s in enumerate(
    [Status.RUNNING, Status.STARTING, Status.STAMPING, Status.WAITING, Status.READY,
     Status.STOPPED, Status.FAILED, Status.REJECTED, Status.DONE])}
