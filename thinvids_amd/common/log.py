"""Process logging (reference common.py:100-161 `get_logging`).

One idempotent stdout handler; the line format keeps the reference's fields (time, level,
host, logger, pid, ``VTT`` tag) so journald/grep tooling built for thinvids keeps working.
"""
from __future__ import annotations

import logging
import os
import socket
import sys
import time

_HOST = socket.gethostname()
LOG_FORMAT = "%(asctime)s %(levelname)s %(hostname)s %(name)s [%(process)d] VTT %(message)s"


class _HostFilter(logging.Filter):
    def filter(self, record: logging.LogRecord) -> bool:
        record.hostname = _HOST
        return True


def _level(level) -> int:
    if isinstance(level, int):
        return level
    name = (level or os.environ.get("LOG_LEVEL", "INFO")).upper()
    return getattr(logging, name, logging.INFO)


def get_logging(app_name: str = "thinvids", level=None, use_utc: bool = False,
                quiet_libs: bool = True) -> logging.Logger:
    root = logging.getLogger()
    if not any(getattr(h, "_tv_handler", False) for h in root.handlers):
        h = logging.StreamHandler(sys.stdout)
        h._tv_handler = True  # type: ignore[attr-defined]
        h.addFilter(_HostFilter())
        fmt = logging.Formatter(LOG_FORMAT, datefmt="%Y-%m-%dT%H:%M:%S%z")
        if use_utc:
            fmt.converter = time.gmtime  # type: ignore[assignment]
        h.setFormatter(fmt)
        root.addHandler(h)
        root.setLevel(_level(level))
        if quiet_libs:
            for lib in ("urllib3", "werkzeug", "watchdog"):
                logging.getLogger(lib).setLevel(logging.WARNING)
    elif level is not None:
        root.setLevel(_level(level))
    return logging.getLogger(app_name)
