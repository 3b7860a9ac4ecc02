"""Node agent (heartbeat payload, TTL, GC, idle suspend) and folder watcher (stability,
processed ledger, aliases, bootstrap, adopt migration)."""
import json
import os
import time
import uuid

import pytest

from thinvids_amd.store import LocalStore


class FakeGpu:
    def __init__(self, util=0.0):
        self.util = util

    def sample(self):
        return {"gpu_count": 8, "util": self.util, "hbm_used": 10, "hbm_total": 8 * 288 * 2 ** 30,
                "gpu_name": "AMD Instinct MI355X", "gpus": [{"index": i, "util": self.util} for i in range(8)]}


@pytest.fixture()
def agent_env(tmp_path, monkeypatch):
    monkeypatch.setenv("HOSTNAME", "node3")
    monkeypatch.setenv("AGENT_MAC", "aa:bb:cc:00:00:03")
    monkeypatch.setenv("GC_BASE_DIR", str(tmp_path))
    monkeypatch.setenv("AGENT_MANAGE_SERVICES", "0")
    monkeypatch.setenv("MIN_UPTIME_BEFORE_SUSPEND", "0")
    from thinvids_amd.common import invalidate_settings_cache
    from thinvids_amd.store import set_store

    st = LocalStore()
    set_store(st)
    invalidate_settings_cache()
    return st, tmp_path


def test_agent_heartbeat_payload(agent_env):
    from thinvids_amd.agent import Agent

    st, _ = agent_env
    st.hset("pipeline:node_roles", "node3", "pipeline")
    a = Agent(store=st, gpu=FakeGpu(55.0), suspend_fn=lambda: None)
    out = a.tick()
    m = st.hgetall("metrics:node:node3")
    assert m["hostname"] == "node3" and m["mac"] == "aa:bb:cc:00:00:03" and m["worker_role"] == "pipeline"
    assert float(m["gpu"]) == 55.0 and m["gpu_count"] == "8" and int(m["mem_total"]) > 0
    assert len(json.loads(m["gpus_json"])) == 8
    assert 0 < st.ttl("metrics:node:node3") <= 15
    assert st.hget("nodes:mac", "node3") == "aa:bb:cc:00:00:03"
    assert out["action"] is None


def test_agent_gc_and_suspend(agent_env):
    from thinvids_amd.agent import Agent

    st, root = agent_env
    old_inactive, old_active, fresh = (str(uuid.uuid4()) for _ in range(3))
    for d in (old_inactive, old_active, fresh, "not-a-uuid"):
        os.makedirs(root / d)
    past = time.time() - 10 * 3600
    for d in (old_inactive, old_active, "not-a-uuid"):
        os.utime(root / d, (past, past))
    st.hset(f"job:{old_active}", "status", "RUNNING")
    st.sadd("jobs:all", f"job:{old_active}")
    calls = []
    a = Agent(store=st, gpu=FakeGpu(0.0), suspend_fn=lambda: calls.append(1))
    out = a.tick()
    assert out["gc"] == {"removed": 1, "skipped_active": 1, "skipped_recent": 1}
    assert not os.path.exists(root / old_inactive) and os.path.exists(root / "not-a-uuid")
    # suspend: gated by the global setting and by job activity
    st.hset("global:settings", mapping={"suspend_enabled": "1", "suspend_idle_sec": "1",
                                        "suspend_idle_cpu_pct_max": "100"})
    from thinvids_amd.common import invalidate_settings_cache

    invalidate_settings_cache()
    t = time.time()
    a.tick(t)
    assert a.tick(t + 5)["action"] is None  # a RUNNING job exists -> never idle
    st.hset(f"job:{old_active}", "status", "DONE")
    a.tick(t + 10)
    assert a.tick(t + 20)["action"] == "suspend" and calls == [1]
    assert not st.exists("metrics:node:node3")
    busy = Agent(store=st, gpu=FakeGpu(90.0), suspend_fn=lambda: calls.append(2))
    busy.tick(t)
    assert busy.tick(t + 50)["action"] is None


def test_agent_publishes_xgmi_counters_and_rates(agent_env):
    """amdsmi per-link accumulators (KB) -> node totals (bytes) -> per-second rates in
    metrics:node:<host>; unsupported links ("N/A" / sentinel) are skipped, and a GPU whose
    metrics table lacks xGMI falls back to the link-metrics API."""
    from thinvids_amd.agent import Agent
    from thinvids_amd.agent.gpu import GpuSampler, xgmi_bytes

    class FakeSmi:
        class AmdSmiMemoryType:
            VRAM = 0

        def __init__(self):
            self.kb = 0

        def amdsmi_get_gpu_activity(self, h):
            return {"gfx_activity": 50, "umc_activity": 10}

        def amdsmi_get_gpu_metrics_info(self, h):
            if h == 1:
                return {"xgmi_read_data_acc": "N/A"}
            return {"xgmi_read_data_acc": [self.kb, self.kb, "N/A", 2 ** 64 - 1],
                    "xgmi_write_data_acc": [self.kb // 2, 0, "N/A", "N/A"]}

        def amdsmi_get_link_metrics(self, h):
            return {"num_links": 2, "links": [{"read": 7, "write": 3}, {"read": 1, "write": 1}, {"read": 99, "write": 99}]}

    smi = FakeSmi()
    assert xgmi_bytes(smi, 0) == (0, 0)
    assert xgmi_bytes(smi, 1) == (8 * 1024, 4 * 1024)
    gs = GpuSampler.__new__(GpuSampler)
    gs._smi, gs._handles = smi, [0, 1]
    st, _ = agent_env
    a = Agent(store=st, gpu=gs, suspend_fn=lambda: None)
    a.tick()
    m = st.hgetall("metrics:node:node3")
    assert int(m["xgmi_read_bytes"]) == 8 * 1024 and int(m["xgmi_rx_bps"]) == 0
    smi.kb = 1000  # 2 links x 1000 KB read, 500 KB written since the last beat
    a.last_ts -= 1.0
    a.tick()
    m = st.hgetall("metrics:node:node3")
    assert int(m["xgmi_read_bytes"]) == 2000 * 1024 + 8 * 1024 and int(m["xgmi_write_bytes"]) == 500 * 1024 + 4 * 1024
    assert 0.5 * 2000 * 1024 < int(m["xgmi_rx_bps"]) <= 2000 * 1024 and int(m["xgmi_tx_bps"]) > 0
    g = json.loads(m["gpus_json"])
    assert g[0]["xgmi_read_bytes"] == 2000 * 1024


def test_rocm_smi_parser():
    from thinvids_amd.agent.gpu import parse_rocm_smi

    g = parse_rocm_smi({"card1": {"GPU use (%)": "40", "VRAM Total Memory (B)": "1000",
                                  "VRAM Total Used Memory (B)": "10", "Card Series": "MI355X"},
                        "card0": {"GPU use (%)": "20"}, "system": {}})
    assert [x["index"] for x in g] == [0, 1] and g[1]["hbm_total"] == 1000 and g[0]["util"] == 20.0


# --------------------------------------------------------------------- watcher
def _cfg(tmp_path, **kw):
    from thinvids_amd.watcher import WatcherConfig

    env = {"WATCH_ROOT": str(tmp_path / "watch"), "PROCESSED_FILE": str(tmp_path / "cfg" / "processed.log"),
           "STABLE_CHECKS": "2", "STABLE_DELAY_SEC": "0.01", "WORKERS": "2", "SCAN_INTERVAL_SEC": "0.05",
           "POLL_INTERVAL_SEC": "0.05"}
    env.update(kw)
    os.makedirs(env["WATCH_ROOT"], exist_ok=True)
    return WatcherConfig(env)


def test_watcher_submits_once_and_records_ledger(tmp_path):
    from thinvids_amd.watcher import Watcher

    got = []
    w = Watcher(_cfg(tmp_path), submit=lambda rel, path: got.append(rel) or True)
    assert w.bootstrap_processed_if_first_run() == 0  # empty root
    (tmp_path / "watch" / "a.mp4").write_bytes(b"x" * 100)
    (tmp_path / "watch" / "notes.txt").write_bytes(b"x")
    fut = w.schedule_submit(str(tmp_path / "watch" / "a.mp4"))
    assert fut.result(timeout=5) is True and got == ["a.mp4"]
    assert w.schedule_submit(str(tmp_path / "watch" / "a.mp4")) is None  # matched in ledger
    lines = open(tmp_path / "cfg" / "processed.log").read().splitlines()
    assert json.loads(lines[-1])["path"] == "a.mp4"
    # a changed file (new signature) is submitted again; a new process sees the ledger
    time.sleep(0.01)
    (tmp_path / "watch" / "a.mp4").write_bytes(b"y" * 150)
    w2 = Watcher(_cfg(tmp_path), submit=lambda rel, path: got.append(rel) or True)
    assert w2.schedule_submit(str(tmp_path / "watch" / "a.mp4")).result(timeout=5) is True
    assert got == ["a.mp4", "a.mp4"]
    w.stop()
    w2.stop()


def test_watcher_bootstrap_legacy_and_aliases(tmp_path):
    from thinvids_amd.watcher import FileProcessedStore, Watcher, signature_for_path

    os.makedirs(tmp_path / "watch" / "tv", exist_ok=True)
    (tmp_path / "watch" / "tv" / "show.mkv").write_bytes(b"z" * 10)
    (tmp_path / "watch" / "old.mp4").write_bytes(b"o" * 10)
    os.makedirs(tmp_path / "cfg", exist_ok=True)
    # legacy path-only line + an entry under the old library name
    sig = signature_for_path(str(tmp_path / "watch" / "tv" / "show.mkv"))
    with open(tmp_path / "cfg" / "processed.log", "w") as f:
        f.write("old.mp4\n" + json.dumps({"path": "television/show.mkv", "sig": sig}) + "\n")
    got = []
    w = Watcher(_cfg(tmp_path, PROCESSED_PATH_ALIASES="tv=television"), submit=lambda r, p: got.append(r) or True)
    assert w.state_for_rel("old.mp4", "1:2") == ("legacy", "old.mp4")
    assert w.state_for_rel("tv/show.mkv", sig) == ("matched", "television/show.mkv")
    assert w.scan_once() == 0 and got == []
    # both got re-recorded under their current path with a concrete signature
    st = FileProcessedStore(str(tmp_path / "cfg" / "processed.log"))
    assert st.state_for("tv/show.mkv", sig) == "matched"
    assert st.state_for("old.mp4", signature_for_path(str(tmp_path / "watch" / "old.mp4"))) == "matched"
    w.stop()
    # first run on a non-empty root: everything is marked, nothing submitted
    os.remove(tmp_path / "cfg" / "processed.log")
    w3 = Watcher(_cfg(tmp_path), submit=lambda r, p: got.append(r) or True)
    assert w3.bootstrap_processed_if_first_run() == 2 and w3.scan_once() == 0 and got == []
    w3.stop()


def test_watcher_observer_end_to_end(tmp_path):
    from thinvids_amd.watcher import Watcher

    got = []
    w = Watcher(_cfg(tmp_path), submit=lambda r, p: got.append(r) or True).start()
    try:
        time.sleep(0.1)
        (tmp_path / "watch" / "new.mkv").write_bytes(b"n" * 64)
        t0 = time.time()
        while not got and time.time() - t0 < 5:
            time.sleep(0.02)
        assert got == ["new.mkv"]
    finally:
        w.stop()
