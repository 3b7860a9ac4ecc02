"""Manager API contract with the Flask test client, the local store and
temporary media roots.  Scheduler/watchdog policies are exercised directly."""
import json
import os
import time

import pytest

from thinvids_amd.models import hevc, media


@pytest.fixture()
def mgr(tmp_path, monkeypatch):
    for k, v in {"WATCH_ROOT": tmp_path / "watch", "SOURCE_MEDIA_ROOT": tmp_path / "src",
                 "LIBRARY_ROOT": tmp_path / "lib", "PROJECT_ROOT": tmp_path / "proj",
                 "CONFIG_ROOT": tmp_path / "cfg"}.items():
        os.makedirs(v, exist_ok=True)
        monkeypatch.setenv(k, str(v))
    monkeypatch.setenv("CLUSTER_WARMUP_SEC", "0")
    monkeypatch.setenv("JOB_INDEX_REINDEX_SEC", "0")
    from thinvids_amd.common import invalidate_settings_cache
    from thinvids_amd.manager import core
    from thinvids_amd.manager.app import create_app
    from thinvids_amd.queue import get_encode_queue, get_pipeline_queue
    from thinvids_amd.store import LocalStore, set_store

    st = LocalStore()
    set_store(st)
    invalidate_settings_cache()
    core.reload_config()
    get_pipeline_queue().flush()
    get_encode_queue().flush()
    app = create_app()
    app.testing = True
    frames = [hevc.synth_frame(1, t, 64, 64) for t in range(4)]
    media.write_y4m(str(tmp_path / "watch" / "movie.y4m"), frames)
    os.makedirs(tmp_path / "watch" / "shows", exist_ok=True)
    media.write_y4m(str(tmp_path / "watch" / "shows" / "ep1.y4m"), frames)
    return {"c": app.test_client(), "st": st, "root": tmp_path, "core": core}


def _heartbeat(st, host, gpus=8):
    st.hset("nodes:mac", host, "aa:bb:cc:dd:ee:0" + host[-1])
    st.hset(f"metrics:node:{host}", mapping={"ts": str(time.time()), "hostname": host, "cpu": "5", "gpu": "0",
                                             "mem": "10", "gpu_count": str(gpus), "mem_used": "1", "mem_total": "2"})


def test_pages_and_legacy_routes(mgr):
    c = mgr["c"]
    for p in ("/", "/dashboard", "/metrics", "/browse", "/watcher", "/nodes"):
        assert c.get(p).status_code == 200, p
    assert c.get("/tasks").status_code == 200


def test_add_job_validation(mgr):
    c = mgr["c"]
    assert c.post("/add_job", json={"filename": "notes.txt"}).status_code == 400
    assert c.post("/add_job", json={"filename": "../etc/passwd.mp4"}).status_code == 400
    assert c.post("/add_job", json={"filename": "missing.y4m"}).status_code == 404
    r = c.post("/add_job", json={"filename": "movie.y4m", "input_path": "/etc/hosts"})
    assert r.status_code == 400


def test_add_job_auto_starts_and_dispatches(mgr):
    c, st = mgr["c"], mgr["st"]
    r = c.post("/add_job", json={"filename": "movie.y4m"})
    assert r.status_code == 201 and r.json["status"] == "success"
    jid = r.json["job_id"]
    job = st.hgetall(f"job:{jid}")
    # reserved by the scheduler and launched: transcode enqueued with the run token
    assert job["status"] == "STARTING" and job["pipeline_run_token"]
    assert job["source_codec"] == "rawvideo" and job["source_resolution"] == "64x64"
    assert jid in st.smembers("pipeline:active_jobs")
    from thinvids_amd.queue import get_pipeline_queue

    msgs = get_pipeline_queue().pending()
    assert msgs and msgs[0]["task"] == "transcode" and msgs[0]["args"] == [jid, job["pipeline_run_token"]]
    assert f"job:{jid}" in st.smembers("jobs:all")
    lines = c.get(f"/job_activity/{jid}").json["lines"]
    assert any("[START]" in line for line in lines)


def test_second_job_waits_behind_unshareable_active_job(mgr):
    c, st = mgr["c"], mgr["st"]
    a = c.post("/add_job", json={"filename": "movie.y4m"}).json["job_id"]
    b = c.post("/add_job", json={"filename": "shows/ep1.y4m"}).json["job_id"]
    assert st.hget(f"job:{a}", "status") == "STARTING"
    jb = st.hgetall(f"job:{b}")
    assert jb["status"] == "WAITING" and jb["queue_blocked_reason"] == "active_job_not_shareable"
    # job a drains past the ratio, 3 pipeline nodes + plenty of idle GPUs -> b dispatches
    for h in ("node1", "node2", "node3", "node4", "node5"):
        _heartbeat(st, h)
    st.hset(f"job:{a}", mapping={"status": "RUNNING", "segment_progress": 100, "parts_total": 8, "parts_done": 7})
    st.hset("global:settings", mapping={"pipeline_worker_count": "4"})
    from thinvids_amd.common import invalidate_settings_cache

    invalidate_settings_cache()
    assert mgr["core"].dispatch_next_waiting_job() is True
    assert st.hget(f"job:{b}", "status") == "STARTING"


def test_job_lifecycle_routes(mgr):
    c, st = mgr["c"], mgr["st"]
    jid = c.post("/add_job", json={"filename": "movie.y4m", "force_paused": True}).json["job_id"]
    assert st.hget(f"job:{jid}", "status") == "READY"
    g = c.get(f"/job_settings/{jid}").json
    assert g["target_height"] == 1080 and g["software_encode"] == "0"
    assert c.post(f"/job_settings/{jid}", json={"software_encode": True, "target_height": 720}).status_code == 200
    assert st.hget(f"job:{jid}", "software_encode") == "1" and st.hget(f"job:{jid}", "target_height") == "720"
    cp = c.post("/copy_job", json={"job_id": jid})
    assert cp.status_code == 201
    assert st.hget(f"job:{cp.json['job_id']}", "status") == "READY"
    assert c.post(f"/start_job/{jid}").status_code == 200
    assert st.hget(f"job:{jid}", "status") == "STARTING"
    assert c.post(f"/start_job/{jid}").status_code == 400  # not READY any more
    r = c.post(f"/stop_job/{jid}")
    assert r.status_code == 200 and r.json["revoked_tasks"] >= 1
    assert st.hget(f"job:{jid}", "status") == "STOPPED"
    assert jid not in st.smembers("pipeline:active_jobs")
    assert c.post(f"/restart_job/{jid}").status_code == 200
    assert st.hget(f"job:{jid}", "status") in ("WAITING", "STARTING")
    props = c.get(f"/job_properties/{jid}").json
    assert props["filename"] == "movie.y4m" and isinstance(props["activity_log"], list)
    assert c.get(f"/preview/{jid}").status_code == 404
    c.post(f"/stop_job/{jid}")
    assert c.post(f"/stamp_job/{jid}").status_code == 202
    assert c.delete(f"/delete_job/{jid}").status_code == 200
    assert not st.exists(f"job:{jid}") and f"job:{jid}" not in st.smembers("jobs:all")
    assert c.delete(f"/delete_job/{jid}").status_code == 404


def test_jobs_listing_paging_sort_filter(mgr):
    c = mgr["c"]
    ids = [c.post("/add_job", json={"filename": "movie.y4m", "force_paused": True}).json["job_id"] for _ in range(12)]
    d = c.get("/jobs?page=2&page_size=10").json
    assert d["total"] == 12 and d["total_pages"] == 2 and len(d["items"]) == 2
    assert c.get("/jobs?status=DONE").json["total"] == 0
    assert c.get("/jobs?q=movie&page_size=25").json["total"] == 12
    assert c.get("/jobs?q=nothing").json["total"] == 0
    assert {j["job_id"] for j in c.get("/jobs?page_size=100&sort_by=filename").json["items"]} == set(ids)


def test_settings_roundtrip_and_validation(mgr):
    c, st = mgr["c"], mgr["st"]
    s = c.get("/settings").json
    assert s["pipeline_worker_count"] == 4 and s["default_target_height"] == 1080
    r = c.post("/settings", json={"suspend_idle_sec": 5, "pipeline_worker_count": 1, "large_file_behavior": "x",
                                  "default_target_height": 999, "tv_qp": 99})
    assert r.status_code == 200
    s = c.get("/settings").json
    assert s["suspend_idle_sec"] == 30 and s["pipeline_worker_count"] == 2 and s["large_file_behavior"] == "reject"
    assert s["default_target_height"] == 1080 and s["tv_qp"] == 51
    assert st.hget("settings:global", "pipeline_worker_count") == "2"  # legacy mirror
    assert c.post("/settings", json={"suspend_idle_sec": "abc"}).status_code == 400


def test_nodes_and_metrics(mgr):
    c, st = mgr["c"], mgr["st"]
    _heartbeat(st, "node1")
    _heartbeat(st, "node2", gpus=4)
    d = c.get("/nodes_data").json["nodes"]
    assert [n["hostname"] for n in d] == ["node1", "node2"]
    assert all(n["active"] for n in d) and d[0]["worker_role"] == "pipeline"
    m = c.get("/metrics_snapshot").json["nodes"]
    assert m[1]["gpu_count"] == 4 and m[0]["mem_total"] == 2
    assert c.post("/nodes/disable/node2").status_code == 200
    assert st.sismember("nodes:disabled", "node2")
    assert not [n for n in c.get("/nodes_data").json["nodes"] if n["hostname"] == "node2"][0]["active"]
    assert c.post("/nodes/enable/node2").status_code == 200
    assert c.delete("/nodes/delete/node2").status_code == 200
    assert st.hget("nodes:mac", "node2") is None
    assert st.hget("pipeline:node_roles", "node1") == "pipeline"


def test_browse_and_guards(mgr):
    c = mgr["c"]
    d = c.get("/browse/list?source=watch").json
    assert [x["name"] for x in d["dirs"]] == ["shows"] and [x["name"] for x in d["files"]] == ["movie.y4m"]
    d = c.get("/browse/list?source=watch&path=shows").json
    assert d["files"][0]["path"] == "shows/ep1.y4m" and d["parent"] == ""
    assert c.get("/browse/list?source=watch&path=../..").status_code == 400
    assert c.get("/browse/list?source=nope").status_code == 400


def test_watcher_config_validation(mgr):
    c, root = mgr["c"], mgr["root"]
    assert c.post("/watcher/config", json={"STABLE_CHECKS": 0}).status_code == 400
    assert c.post("/watcher/config", json={"WATCH_ROOT": "/tmp/elsewhere"}).status_code == 400
    r = c.post("/watcher/config", json={"STABLE_CHECKS": 3, "USE_SCANNER": False,
                                        "WATCH_ROOT": str(root / "src"), "PROCESSED_PATH_ALIASES": "tv=television"})
    assert r.status_code == 200
    text = open(root / "cfg" / "watcher.env").read()
    assert 'STABLE_CHECKS="3"' in text and 'USE_SCANNER="0"' in text
    s = c.get("/watcher/status").json
    assert s["config"]["STABLE_CHECKS"] == "3" and s["env_file"]["exists"]
    assert c.post("/watcher/control", json={"action": "explode"}).status_code == 400
    # the page's typed form is driven by these: every int field carries its server-side range
    t = s["field_types"]
    assert t["int"]["STABLE_CHECKS"] == [1, 60] and "USE_SCANNER" in t["bool"] and "PROCESSED_PATH_ALIASES" in t["text"]
    assert {"free_bytes", "total_bytes"} <= set(s["watch_root"]) and s["watch_root"]["exists"]


def test_ui_pages_carry_their_controls(mgr):
    """Watcher page: typed config form with range checks, service / root / env panels;
    browse page: both roots, sortable size / modified columns, persistent selection."""
    c = mgr["c"]
    w = c.get("/watcher").get_data(as_text=True)
    for needle in ('type="number"', "p-root", "p-svc", "p-env", "collect()", "field_types"):
        assert needle in w, needle
    b = c.get("/browse").get_data(as_text=True)
    for needle in ("source_media", "sortBy('size')", "sortBy('mtime')", "selectAll", "mark_watcher_processed"):
        assert needle in b, needle


def test_watchdog_fails_stalled_jobs(mgr, monkeypatch):
    c, st, core = mgr["c"], mgr["st"], mgr["core"]
    jid = c.post("/add_job", json={"filename": "movie.y4m"}).json["job_id"]
    st.hset(f"job:{jid}", mapping={"status": "RUNNING", "last_heartbeat_at": str(time.time() - 5000),
                                   "last_heartbeat_stage": "encode", "last_heartbeat_host": "node7"})
    assert core.check_for_stalled_jobs() is True
    job = st.hgetall(f"job:{jid}")
    assert job["status"] == "FAILED" and job["failed_stage"] == "watchdog" and job["stalled_stage"] == "encode"
    assert jid not in st.smembers("pipeline:active_jobs")
    # fresh heartbeat is left alone
    jid2 = c.post("/add_job", json={"filename": "movie.y4m"}).json["job_id"]
    st.hset(f"job:{jid2}", mapping={"status": "RUNNING", "last_heartbeat_at": str(time.time())})
    core.check_for_stalled_jobs()
    assert st.hget(f"job:{jid2}", "status") == "RUNNING"


def test_policy_and_wol(mgr):
    core = mgr["core"]
    s = {"av1_check_enabled": "1", "max_source_file_size_gb": "1", "large_file_behavior": "reject"}
    assert core.evaluate_job_policy({"source_codec": "av1"}, s)[0] == "av1_rejected"
    assert core.evaluate_job_policy({"source_codec": "wmv3"}, s)[4] == "direct"
    assert core.evaluate_job_policy({"source_codec": "h264", "source_file_size": 2 * 1024 ** 3}, s)[0] == "size_limit"
    s["large_file_behavior"] = "nfs"
    assert core.evaluate_job_policy({"source_codec": "h264", "source_file_size": 2 * 1024 ** 3}, s)[2] == "nfs"
    pkt = core.build_magic_packet("aa:bb:cc:dd:ee:ff")
    assert len(pkt) == 102 and pkt[:6] == b"\xff" * 6 and pkt[6:12] == bytes.fromhex("aabbccddeeff")
    ok, msg = core.reboot_one_node("localhost")
    assert not ok and "manager" in msg


def test_unreadable_container_is_rejected_up_front(mgr):
    """A container the engine cannot demux (a broken .mkv, or Matroska whose video is not
    HEVC: no H.264 decoder here) is REJECTED at add_job with the probe reason, never
    dispatched to fail later."""
    from thinvids_amd.models import hevc, streams

    c, st, root = mgr["c"], mgr["st"], mgr["root"]
    (root / "watch" / "film.mkv").write_bytes(b"\x1aE\xdf\xa3" + b"\0" * 64)
    bs, _ = hevc.encode_sequence_cpu([hevc.synth_frame(1, 0, 32, 32)], qp=30, search_range=16)
    avc = str(root / "watch" / "avc.mkv")
    streams.mux([bs], 32, 32, 25, 1, avc, [], streams.CONTAINER_MKV)
    raw = open(avc, "rb").read()
    open(avc, "wb").write(raw.replace(b"V_MPEGH/ISO/HEVC", b"V_MPEG4/ISO/AVC\0"))
    for name, why in (("film.mkv", "mkv"), ("avc.mkv", "HEVC only")):
        r = c.post("/add_job", json={"filename": name})
        assert r.status_code in (200, 201), r.get_data(as_text=True)
        job = st.hgetall(f"job:{r.get_json()['job_id']}")
        assert job["status"] == "REJECTED" and job["rejected_reason"] == "probe_failed"
        assert why in job["error"], job["error"]


def test_job_settings_encoder_overrides(mgr):
    """Per-job encoder knobs from the settings modal reach the node/worker encode spec."""
    c, st = mgr["c"], mgr["st"]
    jid = c.post("/add_job", json={"filename": "movie.y4m", "force_paused": True}).json["job_id"]
    r = c.post(f"/job_settings/{jid}", json={"rc_mode": "2pass", "qp": 30, "bitrate_kbps": "1500",
                                              "ladder": "1080, 720", "node_executor": "0"})
    assert r.status_code == 200
    g = c.get(f"/job_settings/{jid}").json
    assert g["rc_mode"] == "2pass" and g["qp"] == "30" and g["ladder"] == "1080,720" and g["node_executor"] == "0"
    assert float(g["bitrate_kbps"]) == 1500.0
    for bad in ({"rc_mode": "vbr"}, {"qp": 60}, {"crf": 0}, {"bitrate_kbps": -3}, {"ladder": "10"}):
        assert c.post(f"/job_settings/{jid}", json=bad).status_code == 500, bad
    assert st.hget(f"job:{jid}", "rc_mode") == "2pass"  # rejected payloads change nothing
    assert c.post(f"/job_settings/{jid}", json={"qp": "", "rc_mode": ""}).status_code == 200
    assert st.hget(f"job:{jid}", "qp") == "" and st.hget(f"job:{jid}", "rc_mode") == ""
    from thinvids_amd.worker.node_executor import _job_params

    job = {**st.hgetall(f"job:{jid}"), "source_width": 1920, "source_height": 1080, "rc_mode": "crf", "crf": "24"}
    p = _job_params(job)
    assert p["rc"] == "crf" and p["crf"] == 24 and p["ladder"] == [1080, 720] and p["codec"] == "hevc"
    # per-job codec override (AV1 engine, BASELINE config #4)
    assert c.post(f"/job_settings/{jid}", json={"codec": "av1"}).status_code == 200
    assert c.get(f"/job_settings/{jid}").json["codec"] == "av1"
    assert c.post(f"/job_settings/{jid}", json={"codec": "vp9"}).status_code == 500
    assert _job_params({**st.hgetall(f"job:{jid}"), "source_width": 1920, "source_height": 1080})["codec"] == "av1"
    # single-pass ABR under a VBV (per-job overrides, validated)
    assert c.post(f"/job_settings/{jid}", json={"rc_mode": "abr", "bitrate_kbps": 4000, "vbv_maxrate_kbps": 6000,
                                                "vbv_bufsize_kbit": 8000}).status_code == 200
    assert c.get(f"/job_settings/{jid}").json["vbv_maxrate_kbps"] in (6000, "6000", 6000.0, "6000.0")
    assert c.post(f"/job_settings/{jid}", json={"vbv_bufsize_kbit": -1}).status_code == 500
    p = _job_params({**st.hgetall(f"job:{jid}"), "source_width": 1920, "source_height": 1080})
    assert p["rc"] == "abr" and p["bitrate_kbps"] == 4000 and p["vbv"] == [6000.0, 8000.0]


def test_nodes_detail_fields(mgr):
    c, st = mgr["c"], mgr["st"]
    _heartbeat(st, "node1")
    st.hset("metrics:node:node1", mapping={"hbm_used": str(3 << 30), "hbm_total": str(288 << 30),
                                           "gpus_json": json.dumps([{"util": 50.0, "hbm_used": 1, "hbm_total": 2}])})
    st.set("node:executor:node1", json.dumps({"world": 8, "pid": 42, "ts": time.time()}))
    n = c.get("/nodes_data").json["nodes"][0]
    assert n["executor"]["world"] == 8 and n["gpus"][0]["util"] == 50.0 and n["hbm_total"] == 288 << 30
    st.hset("node:gpu_quarantine:node1", "3", json.dumps({"reason": "rank 3 (GPU 3) exited with 86", "ts": 1}))
    assert "exited" in c.get("/nodes_data").json["nodes"][0]["gpu_quarantine"]["3"]["reason"]
    st.hset("metrics:node:node1", "gpus_json", "{bad")
    n = c.get("/nodes_data").json["nodes"][0]
    assert n["gpus"] == []
    # the pages carry the modal / chart hooks the scripts drive
    html = c.get("/").get_data(as_text=True)
    assert 'id="jobset"' in html and 'id="video"' in html and "function step(" in html
    assert "TVHIST" in c.get("/metrics").get_data(as_text=True)
    assert "function detail(" in c.get("/nodes").get_data(as_text=True)


def test_probe_lists_streams_and_prefers_english_audio(mgr):
    """Source probe (reference get_video_details :2120-2220): streams_json groups video /
    audio / subtitle streams with codec + language, and the first English audio stream is
    selected; the stitcher later maps exactly that one (`-map 0:a:{sel}`)."""
    import numpy as np

    from thinvids_amd.models import streams

    c, st, root = mgr["c"], mgr["st"], mgr["root"]
    bs, _ = hevc.encode_sequence_cpu([hevc.synth_frame(1, t, 32, 32) for t in range(3)], qp=30, search_range=16)

    def pcm(lang, fill):
        return streams.SideStream(streams.SIDE_AUDIO, streams.SIDE_PCM_S16LE, "pcm_s16le", lang, 8000, 1, 8000, 16,
                                  data=bytes([fill]) * 1600, offsets=np.zeros(1, np.uint64),
                                  sizes=np.asarray([1600], np.uint32), pts=np.zeros(1, np.int64),
                                  durs=np.asarray([800], np.uint32))
    sub = streams._text_stream([(0, 90, "hi")], "eng", "subrip", "srt")
    src = str(root / "watch" / "multi.mkv")
    streams.mux([bs], 32, 32, 25, 1, src, [pcm("fra", 1), pcm("eng", 2), sub], streams.CONTAINER_MKV)
    jid = c.post("/add_job", json={"filename": "multi.mkv", "force_paused": True}).json["job_id"]
    job = st.hgetall(f"job:{jid}")
    sj = json.loads(job["streams_json"])
    assert [a["language"] for a in sj["audio"]] == ["fra", "eng"] and sj["video"][0]["codec"] == "hevc"
    assert sj["subtitle"][0]["codec"] == "subrip" and int(job["selected_a_stream"]) == 1
    plan = streams.plan_output(src, int(job["selected_a_stream"]))
    assert plan.ext == ".mkv" and [t.language for t in plan.tracks] == ["eng", "eng"]
    assert plan.tracks[0].kind == streams.SIDE_AUDIO and plan.fields["audio_streams_kept"] == 1
