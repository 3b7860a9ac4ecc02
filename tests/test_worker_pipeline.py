"""End-to-end worker pipeline on CPU: transcode -> split -> encode -> stitch through the
real queues with threaded consumers (reference test strategy: SURVEY.md §4 — the reference
exercises these paths only on a live cluster; here they run in-process with the local
store, the HTTP data plane on 127.0.0.1 and the software encoder)."""
import os
import time
import uuid

import numpy as np
import pytest

from thinvids_amd.models import hevc, media


@pytest.fixture(scope="module")
def env(tmp_path_factory):
    root = tmp_path_factory.mktemp("tv")
    old = dict(os.environ)
    os.environ.update({
        "PROJECT_ROOT": str(root / "projects"), "LIBRARY_ROOT": str(root / "library"),
        "WATCH_ROOT": str(root / "watch"), "MASTER_HTTP_PORT": "0", "MASTER_HTTP_BIND": "127.0.0.1",
        "HOSTNAME": "127.0.0.1", "STITCH_STABLE_SEC": "0.05", "STITCH_POLL_SEC": "0.05",
        "TV_FORCE_CPU": "1", "JOB_HEARTBEAT_INTERVAL_SEC": "2",
    })
    from thinvids_amd.common import invalidate_settings_cache, save_settings
    from thinvids_amd.store import LocalStore, set_store
    from thinvids_amd.worker.config import get_config

    store = LocalStore()
    set_store(store)
    get_config(reload=True)
    invalidate_settings_cache()
    save_settings({"tv_gop": "8", "tv_segment_frames": "8"}, store)
    from thinvids_amd.queue import Consumer
    from thinvids_amd.worker import tasks

    tasks.pipeline_q.flush()
    tasks.encode_q.flush()
    cons = [Consumer(tasks.pipeline_q, workers=3).start(),
            Consumer(tasks.encode_q, workers=1, handler=lambda q: tasks.encode_batch_handler(timeout=0.1)).start()]
    yield {"root": root, "store": store, "tasks": tasks}
    for c in cons:
        c.stop()
    os.environ.clear()
    os.environ.update(old)


def _source(root, name, n=20, w=128, h=96):
    watch = root / "watch"
    watch.mkdir(exist_ok=True)
    frames = [hevc.synth_frame(3, t, w, h) for t in range(n)]
    path = watch / name
    media.write_y4m(str(path), frames, 25, 1)
    return path, frames


def _wait_status(store, job_id, want, timeout=90):
    t0 = time.time()
    while time.time() - t0 < timeout:
        s = store.hget(f"job:{job_id}", "status")
        if s in want:
            return s
        time.sleep(0.05)
    raise AssertionError(f"job stuck in {store.hget(f'job:{job_id}', 'status')}: {store.hgetall(f'job:{job_id}')}")


@pytest.mark.parametrize("mode", ["split", "direct"])
def test_transcode_end_to_end(env, mode):
    store, tasks = env["store"], env["tasks"]
    path, frames = _source(env["root"], f"clip_{mode}.y4m")
    job_id, tok = str(uuid.uuid4()), uuid.uuid4().hex
    store.hset(f"job:{job_id}", mapping={
        "job_id": job_id, "filename": f"clip_{mode}.y4m", "input_path": str(path), "status": "STARTING",
        "pipeline_run_token": tok, "software_encode": "1", "target_height": "1080", "processing_mode": mode})
    tasks.transcode(job_id, tok)
    assert _wait_status(store, job_id, {"DONE", "FAILED"}) == "DONE", store.hgetall(f"job:{job_id}")
    job = store.hgetall(f"job:{job_id}")
    assert job["processing_mode_effective"] == mode
    assert int(job["parts_total"]) >= 2 and int(job["parts_done"]) == int(job["parts_total"])
    assert int(job["encode_progress"]) == 100 and int(job["combine_progress"]) == 100
    out = job["output_path"]
    assert out.endswith(f"clip_{mode}.mp4") and os.path.isfile(out)
    assert job["dest_codec"] == "hevc" and job["dest_resolution"] == "128x96"
    with open(out, "rb") as f:
        dm = hevc.demux_mp4(f.read())
    dec = hevc.decode(dm["annexb"], coded=False)
    assert len(dec.frames) == len(frames)
    for a, b in zip(frames, dec.frames):
        assert hevc.psnr(a[0], b[0]) > 30
    # scratch cleaned, activity recorded
    assert not os.path.exists(os.path.join(str(env["root"] / "projects"), job_id))
    log = store.lrange(f"joblog:{job_id}", 0, -1)
    assert any("[FINISH]" in line for line in log) and any("[ENCODE]" in line for line in log)


def test_stale_token_is_ignored(env):
    store, tasks = env["store"], env["tasks"]
    job_id = str(uuid.uuid4())
    store.hset(f"job:{job_id}", mapping={"status": "STARTING", "pipeline_run_token": "new"})
    assert tasks.transcode.call_local(job_id, "old") is None
    assert store.hget(f"job:{job_id}", "status") == "STARTING"


def test_dataplane_roundtrip(env, tmp_path):
    from thinvids_amd.worker import dataplane
    from thinvids_amd.worker.helpers import part_paths

    srv = dataplane.start_http_once()
    ep = f"127.0.0.1:{srv.port}"
    job_id = str(uuid.uuid4())
    part, enc = part_paths(job_id, 7)
    os.makedirs(os.path.dirname(part), exist_ok=True)
    payload = np.random.default_rng(0).integers(0, 255, 3 * 1024 * 1024 + 17, dtype=np.uint8).tobytes()
    with open(part, "wb") as f:
        f.write(payload)
    n = dataplane.fetch_part(ep, job_id, 7, str(tmp_path / "got.y4m"))
    assert n == len(payload) and (tmp_path / "got.y4m").read_bytes() == payload
    dataplane.upload_result(ep, job_id, 7, payload[:1000])
    assert open(enc, "rb").read() == payload[:1000]
    import urllib.error

    with pytest.raises(urllib.error.HTTPError):
        dataplane.fetch_part(ep, job_id, 0, str(tmp_path / "bad"))


def _run_job(env, name, mode="split", n=20):
    store, tasks = env["store"], env["tasks"]
    path, frames = _source(env["root"], name, n=n)
    job_id, tok = str(uuid.uuid4()), uuid.uuid4().hex
    store.hset(f"job:{job_id}", mapping={
        "job_id": job_id, "filename": name, "input_path": str(path), "status": "STARTING",
        "pipeline_run_token": tok, "software_encode": "1", "target_height": "1080", "processing_mode": mode})
    tasks.transcode(job_id, tok)
    return job_id, frames


@pytest.fixture
def fault_env(env, monkeypatch, tmp_path):
    monkeypatch.setenv("TV_FAULT_STATE", str(tmp_path / "faults"))
    return env


def test_injected_part_failure_is_retried(fault_env, monkeypatch):
    """Part 2 fails twice in encode and once in upload: the part is re-enqueued (reference
    `_fail` -> re-enqueue, worker/tasks.py:1385-1464) and the job still finishes."""
    monkeypatch.setenv("TV_FAULT", "part:2:fail:2,upload:1:fail:1")
    store = fault_env["store"]
    job_id, frames = _run_job(fault_env, "fault_retry.y4m")
    assert _wait_status(store, job_id, {"DONE", "FAILED"}) == "DONE", store.hgetall(f"job:{job_id}")
    counts = store.hgetall(f"job_retry_counts:{job_id}") or {}
    job = store.hgetall(f"job:{job_id}")
    assert job["last_retry_part"] in ("1", "2")
    with open(job["output_path"], "rb") as f:
        dec = hevc.decode(hevc.demux_mp4(f.read())["annexb"], coded=False)
    assert len(dec.frames) == len(frames)
    assert not counts  # cleaned at finalize
    log = store.lrange(f"joblog:{job_id}", 0, -1)
    assert sum("Retrying" in line or "retry" in line.lower() for line in log) >= 1 or job["last_retry_stage"]


def test_injected_part_failure_exhausts_budget(fault_env, monkeypatch):
    monkeypatch.setenv("TV_FAULT", "part:1:fail")
    monkeypatch.setenv("PART_FAILURE_MAX_RETRIES", "2")
    from thinvids_amd.worker.config import get_config

    get_config(reload=True)
    try:
        store = fault_env["store"]
        job_id, _ = _run_job(fault_env, "fault_budget.y4m", mode="direct")
        assert _wait_status(store, job_id, {"DONE", "FAILED"}) == "FAILED"
        job = store.hgetall(f"job:{job_id}")
        assert job["failed_stage"] == "encode" and job["failed_part"] == "1"
        assert "retry budget exhausted (3/2)" in job["error"]
    finally:
        monkeypatch.delenv("PART_FAILURE_MAX_RETRIES")
        get_config(reload=True)


def test_injected_stitch_failure_fails_job(fault_env, monkeypatch):
    monkeypatch.setenv("TV_FAULT", "stitch:*:fail")
    store = fault_env["store"]
    job_id, _ = _run_job(fault_env, "fault_stitch.y4m")
    assert _wait_status(store, job_id, {"DONE", "FAILED"}) == "FAILED"
    job = store.hgetall(f"job:{job_id}")
    assert job["failed_stage"] == "stitch" and "injected fault" in job["error"]


def test_fault_spec_parsing(tmp_path, monkeypatch):
    from thinvids_amd.utils import fault

    specs = fault.parse("part:3:fail:2, rank:*:hang:0.01,segment:1:die")
    assert [(s.kind, s.key, s.action, s.arg) for s in specs] == [
        ("part", "3", "fail", 2.0), ("rank", "*", "hang", 0.01), ("segment", "1", "die", None)]
    with pytest.raises(ValueError):
        fault.parse("part:3:explode")
    monkeypatch.setenv("TV_FAULT", "part:3:fail:2")
    monkeypatch.setenv("TV_FAULT_STATE", str(tmp_path))
    fault.check("part", 4)  # other key: no-op
    for _ in range(2):
        with pytest.raises(fault.InjectedFault):
            fault.check("part", 3)
    fault.check("part", 3)  # budget of 2 spent (persisted in TV_FAULT_STATE)
    assert len(os.listdir(tmp_path)) == 2


def test_stamp_streams_in_gop_chunks(env, monkeypatch):
    """Stamp (verification encode) reads, stamps and encodes in closed-GOP chunks and muxes
    the segment bitstreams straight to disk: the output has every frame, each carrying its
    burned-in number, and a new READY job points at it."""
    from thinvids_amd.ops.overlay import stamp_ref

    store, tasks = env["store"], env["tasks"]
    monkeypatch.setattr(tasks, "STAMP_GOP", 8)
    monkeypatch.setattr(tasks, "STAMP_BATCH", 2)
    path, frames = _source(env["root"], "stampme.y4m", n=37, w=96, h=64)
    reads = []
    real_open = media.open_source

    def counting_open(p):
        s = real_open(p)
        real_read = s.read
        s.read = lambda a, n: (reads.append((a, n)), real_read(a, n))[1]
        return s

    monkeypatch.setattr(tasks.media, "open_source", counting_open)
    job_id, tok = str(uuid.uuid4()), uuid.uuid4().hex
    store.hset(f"job:{job_id}", mapping={"job_id": job_id, "filename": "stampme.y4m", "input_path": str(path),
                                         "status": "STAMPING", "pipeline_run_token": tok, "stamp_run_token": tok})
    monkeypatch.setattr(tasks, "task_token_is_current", lambda *a, **k: True)
    res = tasks.stamp.call_local(job_id, tok)
    assert res["status"] == "STAMPED", store.hgetall(f"job:{job_id}")
    assert reads == [(s, 8) for s in range(0, 37, 8)]  # one bounded read per chunk
    with open(res["output"], "rb") as f:
        dec = hevc.decode(hevc.demux_mp4(f.read())["annexb"], coded=False)
    assert len(dec.frames) == 37
    for t in (0, 9, 36):  # the label of frame t is burned in (QP 18: close to the stamped reference)
        ref = stamp_ref(frames[t], str(t))
        assert np.mean(np.abs(dec.frames[t][0].astype(int) - ref[0].astype(int))) < 3.0
        assert np.mean(np.abs(ref[0].astype(int) - frames[t][0].astype(int))) > 0.1
    new = store.hgetall(f"job:{res['new_job_id']}")
    assert new["status"] == "READY" and new["input_path"] == res["output"]


def test_transcode_carries_audio_and_english_subtitles(env):
    """Sidecar audio + English SubRip next to the source: the stitcher carries both and the
    output becomes Matroska (reference rule, worker/tasks.py:2126-2223), with the
    english_subtitles_* job fields set; the HEVC video inside decodes to every frame."""
    import struct

    from thinvids_amd.models import streams

    store, tasks = env["store"], env["tasks"]
    path, frames = _source(env["root"], "withsubs.y4m", n=16)
    base = os.path.splitext(str(path))[0]
    rate, pcm = 8000, (np.arange(8000, dtype=np.int64) % 200 * 50 - 5000).astype("<i2").tobytes()
    with open(base + ".wav", "wb") as f:
        f.write(b"RIFF" + struct.pack("<I", 36 + len(pcm)) + b"WAVE")
        f.write(b"fmt " + struct.pack("<IHHIIHH", 16, 1, 1, rate, rate * 2, 2, 16))
        f.write(b"data" + struct.pack("<I", len(pcm)) + pcm)
    with open(base + ".en.srt", "w") as f:
        f.write("1\n00:00:00,040 --> 00:00:00,300\nfirst cue\n\n2\n00:00:00,320 --> 00:00:00,600\nsecond cue\n")
    job_id, tok = str(uuid.uuid4()), uuid.uuid4().hex
    store.hset(f"job:{job_id}", mapping={
        "job_id": job_id, "filename": "withsubs.y4m", "input_path": str(path), "status": "STARTING",
        "pipeline_run_token": tok, "software_encode": "1", "processing_mode": "split"})
    tasks.transcode(job_id, tok)
    assert _wait_status(store, job_id, {"DONE", "FAILED"}) == "DONE", store.hgetall(f"job:{job_id}")
    job = store.hgetall(f"job:{job_id}")
    out = job["output_path"]
    assert out.endswith("withsubs.mkv") and os.path.isfile(out)
    assert (int(job["english_subtitles_found"]), int(job["english_subtitles_kept"])) == (1, 1)
    assert int(job["audio_streams_kept"]) == 1 and int(job["dest_streams"]) == 3
    assert job["dest_codec"] == "hevc" and job["dest_resolution"] == "128x96"
    annexb, _, _ = streams.mkv_hevc_annexb(out)
    dec = hevc.decode(annexb, coded=False)
    assert len(dec.frames) == len(frames)
    side, _ = streams.mkv_streams(out)
    audio = [s for s in side if s.kind == streams.SIDE_AUDIO][0]
    subs = [s for s in side if s.kind == streams.SIDE_SUBTITLE][0]
    with open(out, "rb") as f:
        got = b""
        for o, n in zip(audio.offsets, audio.sizes):
            f.seek(int(o))
            got += f.read(int(n))
    assert got == pcm
    assert subs.language == "eng" and list(subs.pts) == [40, 320]


def _combed(n=20, w=128, h=96):
    """Interlaced-looking frames: the bottom field is sampled half a frame later (combing)."""
    out = []
    for t in range(n):
        a = hevc.synth_frame(7, 2 * t, w, h)
        b = hevc.synth_frame(7, 2 * t + 1, w, h)
        y = a[0].copy()
        y[1::2] = b[0][1::2]
        out.append((y, a[1], a[2]))
    return out


@pytest.mark.parametrize("mode", ["split", "direct"])
def test_dvd_mpeg2_title_transcodes_with_bwdif(env, mode):
    """A MakeMKV-style DVD title (Matroska V_MPEG2, interlaced, under dvd/) goes through the
    whole pipeline: probed as mpeg2video, kept at its native lines (never upscaled), bwdif
    deinterlaced (K3, reference worker/tasks.py:475-500) and encoded."""
    from thinvids_amd.models import mpeg2, streams
    from thinvids_amd.ops.deint import deinterlace_frames

    store, tasks = env["store"], env["tasks"]
    fr = _combed()
    es, units, disp, rec = mpeg2.encode(fr, interlaced=1, gop=8, closed_gop=0)
    d = env["root"] / "watch" / "dvd"
    d.mkdir(parents=True, exist_ok=True)
    path = d / f"title_{mode}.mkv"
    mpeg2.mkv_write_mpeg2(str(path), units, disp, 128, 96, codec_private=mpeg2.codec_private_of(es))
    job_id, tok = str(uuid.uuid4()), uuid.uuid4().hex
    store.hset(f"job:{job_id}", mapping={
        "job_id": job_id, "filename": f"dvd/title_{mode}.mkv", "input_path": str(path), "status": "STARTING",
        "pipeline_run_token": tok, "software_encode": "1", "target_height": "1080", "processing_mode": mode})
    tasks.transcode(job_id, tok)
    assert _wait_status(store, job_id, {"DONE", "FAILED"}) == "DONE", store.hgetall(f"job:{job_id}")
    job = store.hgetall(f"job:{job_id}")
    assert job["source_codec"] == "mpeg2video" and job["dest_resolution"] == "128x96"
    out = job["output_path"]
    if out.endswith(".mkv"):
        annexb, _, _ = streams.mkv_hevc_annexb(out)
    else:
        with open(out, "rb") as f:
            annexb = hevc.demux_mp4(f.read())["annexb"]
    dec = hevc.decode(annexb, coded=False).frames
    assert len(dec) == len(fr)
    # the output follows the deinterlaced decode, not the combed fields
    deint = deinterlace_frames(rec)
    p_deint = np.mean([hevc.psnr(a[0], b[0]) for a, b in zip(deint, dec)])
    p_comb = np.mean([hevc.psnr(a[0], b[0]) for a, b in zip(rec, dec)])
    assert p_deint > 30 and p_deint > p_comb + 1, (p_deint, p_comb)
