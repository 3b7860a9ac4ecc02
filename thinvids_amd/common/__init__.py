"""Shared runtime (reference common.py): status model, settings, activity log, logging,
job-index helpers.  The state store itself lives in :mod:`thinvids_amd.store`."""
from __future__ import annotations

import re

from ..store import get_store
from .activity import emit_activity, fetch_activity, fetch_job_activity, format_activity_line  # noqa: F401
from .log import get_logging  # noqa: F401
from .settings import (DEFAULT_SETTINGS, as_bool, as_float, as_int, get_settings,  # noqa: F401
                       invalidate_settings_cache, save_settings)
from .status import ACTIVE_STATUSES, STATUS_ORDER, TERMINAL_STATUSES, Status  # noqa: F401

JOBS_INDEX_KEY = "jobs:all"


def is_base_job_key(key: str) -> bool:
    key = (key or "").strip()
    return key.startswith("job:") and ":" not in key[4:]


def natural_host_key(host: str):
    """Sort key 'thinman2' < 'thinman10' (reference common.py:164-166)."""
    m = re.search(r"(\d+)", host or "")
    return (int(m.group(1)) if m else 0, host or "")


def job_keys(store=None) -> list[str]:
    """Indexed job keys; prunes invalid members and seeds the index by scan when empty."""
    st = store or get_store()
    raw = list(st.smembers(JOBS_INDEX_KEY) or [])
    keys = [k for k in raw if is_base_job_key(k)]
    bad = [k for k in raw if not is_base_job_key(k)]
    if bad:
        st.srem(JOBS_INDEX_KEY, *bad)
    if not keys:
        keys = [k for k in st.scan_iter("job:*") if is_base_job_key(k)]
        if keys:
            st.sadd(JOBS_INDEX_KEY, *keys)
    return keys


def all_jobs_are_idle(store=None) -> bool:
    """True only if no indexed job is RUNNING/WAITING/STARTING (reference common.py:235-274).

    Deliberate fix: with zero jobs the cluster IS idle (the reference returned False)."""
    st = store or get_store()
    keys = job_keys(st)
    if not keys:
        return True
    p = st.pipeline()
    for k in keys:
        p.hget(k, "status")
    busy = {Status.RUNNING.value, Status.WAITING.value, Status.STARTING.value}
    return not any(str(s or "").upper() in busy for s in p.execute())


def pass_field(job: dict, name: str) -> str:
    """Value of a per-pass progress counter (parts_done, completed_chunks, encoded_frames) of
    the job's current rate-control pass: pass 0 keeps the reference's field names, a later
    pass of a 2-pass job counts in ``<name>_p<k>`` (worker/node_executor._StoreHooks)."""
    k = str(job.get("rc_pass") or "0")
    return job.get(f"{name}_p{k}") if k not in ("", "0") else job.get(name)
