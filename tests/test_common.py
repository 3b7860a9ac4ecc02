"""Common control-plane pieces: status model, logging format, settings
cache, activity log, cluster idleness probe — contract pins against the reference's
common.py behaviour (with its documented defects fixed)."""
import logging

import pytest

from thinvids_amd.common import activity, all_jobs_are_idle, job_keys, natural_host_key, settings
from thinvids_amd.common.log import LOG_FORMAT, get_logging
from thinvids_amd.common.status import ACTIVE_STATUSES, TERMINAL_STATUSES, Status
from thinvids_amd.store.local import LocalStore


def test_status_parse_contract():
    assert Status.parse(" running ") is Status.RUNNING
    assert Status.parse("COMPLETED") is Status.DONE  # legacy value read as DONE
    assert Status.parse_or("bogus", Status.FAILED) is Status.FAILED
    with pytest.raises(ValueError):
        Status.parse("bogus")
    assert not set(ACTIVE_STATUSES) & set(TERMINAL_STATUSES)
    assert [s.value for s in Status] == ["READY", "STARTING", "WAITING", "RUNNING", "STAMPING", "STOPPED",
                                         "FAILED", "REJECTED", "DONE"]


def test_logging_format_and_idempotent(capsys):
    assert LOG_FORMAT.endswith("[%(process)d] VTT %(message)s")
    a = get_logging("tv-test")
    n = len(logging.getLogger().handlers)
    get_logging("tv-test")
    assert len(logging.getLogger().handlers) == n  # no duplicate handlers
    a.info("hello")
    assert isinstance(a, logging.Logger)


def test_settings_cache_and_mirror():
    st = LocalStore()
    settings.invalidate_settings_cache()
    base = settings.get_settings(st)
    assert base == dict(settings.DEFAULT_SETTINGS)
    key = next(iter(settings.DEFAULT_SETTINGS))
    settings.save_settings({key: "x1"}, st)
    assert st.hget(settings.SETTINGS_KEY, key) == "x1" and st.hget(settings.LEGACY_SETTINGS_KEY, key) == "x1"
    assert settings.get_settings(st)[key] == "x1"  # a save invalidates this process's cache
    st.hset(settings.SETTINGS_KEY, mapping={key: "x2"})  # another process writes
    assert settings.get_settings(st)[key] == "x1"  # cached for CACHED_SETTINGS_TTL
    settings.invalidate_settings_cache()
    assert settings.get_settings(st)[key] == "x2"
    settings.invalidate_settings_cache()
    assert settings.as_bool("yes") and not settings.as_bool("0") and settings.as_int("7x", 3) == 3


def test_activity_log_capped_and_per_job(monkeypatch):
    st = LocalStore()
    monkeypatch.setattr(activity, "ACTIVITY_LOG_MAX", 5)
    for i in range(8):
        activity.emit_activity(f"part {i} encoded in {i}ms", job_id="j1", stage="encode", store=st)
    ev = activity.fetch_activity(100, store=st)
    assert len(ev) == 5 and ev[0]["message"].startswith("part 7")  # newest first, capped
    lines = activity.fetch_job_activity("j1", store=st)
    assert len(lines) == 8 and "part 0" in lines[0]


def test_idleness_probe_and_job_index():
    st = LocalStore()
    assert all_jobs_are_idle(st)  # no jobs: idle (reference returned False — fixed)
    st.hset("job:a", mapping={"status": "DONE"})
    st.hset("job:b", mapping={"status": "RUNNING"})
    st.hset("job:b:parts", mapping={"x": "1"})  # not a base job key
    assert sorted(job_keys(st)) == ["job:a", "job:b"]
    assert not all_jobs_are_idle(st)
    st.hset("job:b", mapping={"status": "STOPPED"})
    assert all_jobs_are_idle(st)
    assert sorted(["thinman10", "thinman2", "thinman1"], key=natural_host_key) == ["thinman1", "thinman2",
                                                                                    "thinman10"]
