"""Node executor (one rank per GPU, RCCL data plane) under the job queue: a `transcode`
job is handed to a live executor, whose ranks claim segments dynamically, all-reduce
quality statistics, gather bitstreams to rank 0 and publish the output + job hash.  On CPU
the ranks run the software encoder over gloo; the GPU test runs the HIP engine over RCCL."""
import json
import os
import sys
import threading
import time
import uuid

import numpy as np
import pytest

from thinvids_amd.models import hevc, media

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _wait(store, job_id, want, timeout=180):
    t0 = time.time()
    while time.time() - t0 < timeout:
        s = store.hget(f"job:{job_id}", "status")
        if s in want:
            return s
        time.sleep(0.05)
    raise AssertionError(f"job stuck: {store.hgetall(f'job:{job_id}')}")


@pytest.fixture
def node_env(tmp_path, monkeypatch):
    from thinvids_amd.common import invalidate_settings_cache, save_settings
    from thinvids_amd.store import RemoteStore, set_store
    from thinvids_amd.store.server import StoreServer
    from thinvids_amd.worker.config import get_config

    srv = StoreServer("127.0.0.1", 0)
    srv.start_background()
    url = f"tcp://127.0.0.1:{srv.server_address[1]}"
    env = {"TV_STORE": url, "PROJECT_ROOT": str(tmp_path / "projects"), "LIBRARY_ROOT": str(tmp_path / "library"),
           "WATCH_ROOT": str(tmp_path / "watch"), "HOSTNAME": "node-test", "TV_NODE_HOST": "node-test",
           "PYTHONPATH": ROOT}
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    store = RemoteStore("127.0.0.1", srv.server_address[1])
    set_store(store)
    get_config(reload=True)
    invalidate_settings_cache()
    yield {"store": store, "srv": srv, "tmp": tmp_path}
    set_store(None)
    srv.shutdown()
    srv.server_close()


def _start_executor(n, extra_env=None, max_jobs=1):
    from thinvids_amd.parallel.launch import spawn_ranks

    res = {}

    def run():
        env = dict(extra_env or {})
        res["rc"] = spawn_ranks(n, ["-m", "thinvids_amd.worker.node_executor", "--max-jobs", str(max_jobs),
                                    "--idle-exit", "120"], extra_env=env, timeout=300)

    t = threading.Thread(target=run, daemon=True)
    t.start()
    return t, res


def _submit(store, tmp, name, frames, software, extra=None):
    from thinvids_amd.worker import tasks

    watch = tmp / "watch"
    watch.mkdir(exist_ok=True)
    path = watch / name
    media.write_y4m(str(path), frames, 25, 1)
    job_id, tok = str(uuid.uuid4()), uuid.uuid4().hex
    store.hset(f"job:{job_id}", mapping={"job_id": job_id, "filename": name, "input_path": str(path),
                                         "status": "STARTING", "pipeline_run_token": tok,
                                         "software_encode": "1" if software else "0", "target_height": "1080",
                                         **(extra or {})})
    return job_id, tok, tasks


def test_node_executor_runs_transcode_job_over_two_gloo_ranks(node_env, monkeypatch):
    from thinvids_amd.common import save_settings
    from thinvids_amd.worker.node_executor import live_executor

    store, tmp = node_env["store"], node_env["tmp"]
    save_settings({"tv_gop": "8", "tv_node_segment_frames": "8", "tv_node_batch": "1", "tv_sao": "0"}, store)
    th, res = _start_executor(2, {"TV_FORCE_CPU": "1"})
    t0 = time.time()
    while live_executor(store) is None:
        assert time.time() - t0 < 120, "executor did not come up"
        time.sleep(0.1)
    frames = [hevc.synth_frame(4, t, 128, 96) for t in range(40)]
    job_id, tok, tasks = _submit(store, tmp, "clip.y4m", frames, software=True)
    out = tasks.transcode.call_local(job_id, tok)
    assert out["status"] == "QUEUED_NODE" and out["host"] == "node-test"
    assert _wait(store, job_id, {"DONE", "FAILED"}) == "DONE", store.hgetall(f"job:{job_id}")
    th.join(120)
    assert res.get("rc") == 0
    job = store.hgetall(f"job:{job_id}")
    assert job["processing_mode_effective"] == "node" and int(job["node_world"]) == 2
    assert int(job["parts_total"]) == 5 and int(job["parts_done"]) == 5 and int(job["encode_progress"]) == 100
    assert int(job["encoded_frames"]) == 40
    assert float(job["psnr_y"]) > 30 and float(job["job_fps"]) > 0 and float(job["bitrate_kbps"]) > 0
    assert job["dest_resolution"] == "128x96" and job["dest_codec"] == "hevc"
    with open(job["output_path"], "rb") as f:
        dec = hevc.decode(hevc.demux_mp4(f.read())["annexb"], coded=False)
    assert len(dec.frames) == 40
    ps = np.mean([hevc.psnr_yuv(a, b)["y"] for a, b in zip(frames, dec.frames)])
    assert abs(ps - float(job["psnr_y"])) < 0.6  # pooled-SSE vs mean-of-frames PSNR


def test_transcode_without_executor_uses_split_pipeline(node_env):
    from thinvids_amd.worker.tasks import _node_executor_for

    assert _node_executor_for({"processing_mode": "auto"}) is None
    node_env["store"].set("node:executor:other", "{}", ex=15)
    node_env["store"].sadd("node:executors", "other")
    assert _node_executor_for({"processing_mode": "auto"}) == "other"
    assert _node_executor_for({"processing_mode": "split"}) == "other"  # the policy default
    assert _node_executor_for({"node_executor": "0"}) is None


@pytest.mark.gpu
def test_node_executor_gpu_job_with_ladder_and_hdr(node_env):
    """GPU: one RCCL rank; a 10-bit PQ source goes through the device tone-map and a
    two-rung ladder on the HIP engine; both outputs decode and carry per-job PSNR."""
    from thinvids_amd.common import save_settings
    from thinvids_amd.worker.node_executor import live_executor

    store, tmp = node_env["store"], node_env["tmp"]
    save_settings({"tv_gop": "8", "tv_node_segment_frames": "16", "tv_ladder": "192,128"}, store)
    th, res = _start_executor(1)
    t0 = time.time()
    while live_executor(store) is None:
        assert time.time() - t0 < 120, "executor did not come up"
        time.sleep(0.1)
    rng = np.random.default_rng(0)
    base = [hevc.synth_frame(6, t, 256, 192) for t in range(24)]
    frames = [tuple((p.astype(np.uint16) * 3 + 64).astype(np.uint16) for p in f) for f in base]  # 10-bit
    job_id, tok, tasks = _submit(store, tmp, "hdr.y4m", frames, software=False)
    assert tasks.transcode.call_local(job_id, tok)["status"] == "QUEUED_NODE"
    assert _wait(store, job_id, {"DONE", "FAILED"}) == "DONE", store.hgetall(f"job:{job_id}")
    th.join(60)
    job = store.hgetall(f"job:{job_id}")
    outs = json.loads(job["ladder_outputs_json"])
    assert [o["height"] for o in outs] == [192, 128]
    for o in outs:
        with open(o["path"], "rb") as f:
            dec = hevc.decode(hevc.demux_mp4(f.read())["annexb"], coded=False)
        assert len(dec.frames) == 24 and dec.frames[0][0].shape == (o["height"], o["width"])
        assert o["psnr_y"] > 30
    del rng


@pytest.mark.gpu
def test_add_job_end_to_end_on_gpu_node_executor(node_env, monkeypatch):
    """POST /add_job -> scheduler -> transcode (pipeline queue) -> node executor rank on the
    MI355X (HIP engine, RCCL group) -> library output, job hash DONE with dest_*, per-job
    frames/s and PSNR."""
    from thinvids_amd.common import invalidate_settings_cache, save_settings
    from thinvids_amd.manager import core
    from thinvids_amd.manager.app import create_app
    from thinvids_amd.queue import Consumer
    from thinvids_amd.worker import tasks
    from thinvids_amd.worker.node_executor import live_executor

    store, tmp = node_env["store"], node_env["tmp"]
    monkeypatch.setenv("CLUSTER_WARMUP_SEC", "0")
    for d in ("watch", "library", "projects", "cfg", "src"):
        os.makedirs(tmp / d, exist_ok=True)
    monkeypatch.setenv("CONFIG_ROOT", str(tmp / "cfg"))
    monkeypatch.setenv("SOURCE_MEDIA_ROOT", str(tmp / "src"))
    core.reload_config()
    invalidate_settings_cache()
    save_settings({"tv_gop": "16", "tv_node_segment_frames": "32"}, store)
    store.hset("nodes:mac", "node-test", "aa:bb:cc:dd:ee:01")
    store.hset("metrics:node:node-test", mapping={"ts": str(time.time() + 3600), "hostname": "node-test",
                                                  "gpu_count": "1", "cpu": "1", "gpu": "0", "mem": "1"})
    tasks.pipeline_q.flush()
    cons = Consumer(tasks.pipeline_q, workers=2).start()
    th, res = _start_executor(1)
    t0 = time.time()
    while live_executor(store) is None:
        assert time.time() - t0 < 120, "executor did not come up"
        time.sleep(0.1)
    frames = [hevc.synth_frame(8, t, 320, 192) for t in range(96)]
    media.write_y4m(str(tmp / "watch" / "movie.y4m"), frames, 30, 1)
    c = create_app().test_client()
    r = c.post("/add_job", json={"filename": "movie.y4m"})
    assert r.status_code == 201, r.get_data(as_text=True)
    job_id = r.get_json()["job_id"]
    try:
        assert _wait(store, job_id, {"DONE", "FAILED"}) == "DONE", store.hgetall(f"job:{job_id}")
    finally:
        cons.stop()
    job = store.hgetall(f"job:{job_id}")
    assert job["processing_mode_effective"] == "node" and int(job["encoded_frames"]) == 96
    assert job["dest_resolution"] == "320x192" and int(job["dest_file_size"]) > 0
    assert float(job["job_fps"]) > 0 and float(job["psnr_y"]) > 30
    with open(job["output_path"], "rb") as f:
        dec = hevc.decode(hevc.demux_mp4(f.read())["annexb"], coded=False)
    assert len(dec.frames) == 96
    ps = np.mean([hevc.psnr_yuv(a, b)["y"] for a, b in zip(frames, dec.frames)])
    assert abs(ps - float(job["psnr_y"])) < 0.6


def test_run_job_twice_in_one_process_group(tmp_path, monkeypatch):
    """A long-lived executor runs many jobs in one process group: work-queue keys in the
    rendezvous store must not leak from one job into the next."""
    import torch.multiprocessing as mp

    from thinvids_amd.parallel.launch import free_port

    frames = [hevc.synth_frame(4, t, 96, 64) for t in range(24)]
    src = tmp_path / "a.y4m"
    media.write_y4m(str(src), frames, 25, 1)
    mp.spawn(_twice_worker, args=(2, free_port(), str(src), str(tmp_path)), nprocs=2, join=True)
    for k in (0, 1):
        with open(tmp_path / f"o{k}.mp4", "rb") as f:
            assert len(hevc.decode(hevc.demux_mp4(f.read())["annexb"], coded=False).frames) == 24


def _twice_worker(rank, world, port, src, out_dir):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), TV_FORCE_CPU="1")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from thinvids_amd.parallel.node_job import run_job

    for k in (0, 1):
        run_job(src, os.path.join(out_dir, f"o{k}.mp4"), gop=8, segment_frames=8, software=True, batch_segments=1)
    dist.destroy_process_group()


def _start_supervised(n, max_jobs=1):
    from thinvids_amd.worker import node_executor

    res = {}

    def run():
        res["rc"] = node_executor.main(["--gpus", str(n), "--max-jobs", str(max_jobs), "--idle-exit", "120"])

    t = threading.Thread(target=run, daemon=True)
    t.start()
    return t, res


@pytest.mark.parametrize("fault", ["rank:1:die:1", "rank:1:hang:600"])
def test_supervisor_recovers_from_dead_or_hung_rank_on_smaller_world(node_env, monkeypatch, fault):
    """A rank that dies (or hangs mid-job) takes the communicator down: the supervisor kills
    the group, quarantines that GPU, requeues the job and restarts on the remaining GPU; the
    job resumes and completes on the smaller world."""
    from thinvids_amd.common import save_settings
    from thinvids_amd.parallel.elastic import quarantine_key
    from thinvids_amd.worker.node_executor import live_executor

    store, tmp = node_env["store"], node_env["tmp"]
    save_settings({"tv_gop": "8", "tv_node_segment_frames": "8", "tv_node_batch": "1", "tv_sao": "0"}, store)
    monkeypatch.setenv("TV_FORCE_CPU", "1")
    monkeypatch.setenv("TV_FAULT", fault)
    monkeypatch.setenv("TV_FAULT_STATE", str(tmp / "faults"))
    monkeypatch.setenv("TV_NODE_STALL_SEC", "4")
    th, res = _start_supervised(2)
    t0 = time.time()
    while live_executor(store) is None:
        assert time.time() - t0 < 120, "executor did not come up"
        time.sleep(0.1)
    frames = [hevc.synth_frame(4, t, 128, 96) for t in range(32)]
    job_id, tok, tasks = _submit(store, tmp, "clip.y4m", frames, software=True)
    assert tasks.transcode.call_local(job_id, tok)["status"] == "QUEUED_NODE"
    assert _wait(store, job_id, {"DONE", "FAILED"}, timeout=240) == "DONE", store.hgetall(f"job:{job_id}")
    th.join(120)
    assert res.get("rc") == 0
    job = store.hgetall(f"job:{job_id}")
    assert int(job["node_restarts"]) == 1 and int(job["node_world"]) == 1
    assert ("exited with 86" if "die" in fault else "no progress") in job["node_last_failure"]
    assert list(store.hgetall(quarantine_key("node-test"))) == ["1"]
    with open(job["output_path"], "rb") as f:
        dec = hevc.decode(hevc.demux_mp4(f.read())["annexb"], coded=False)
    assert len(dec.frames) == 32


def test_supervisor_stall_culprit_and_requeue_budget(node_env, monkeypatch):
    from thinvids_amd.parallel.elastic import RankBeat, Supervisor, rank_key
    from thinvids_amd.worker.node_executor import _requeue, queue_key

    store = node_env["store"]
    sup = Supervisor([], [0, 1, 2], "h", store, stall_sec=5)
    now = time.time()
    beats = {0: {"job": {"job_id": "a"}, "progress_ts": now - 2}, 1: {"job": {"job_id": "a"}, "progress_ts": now - 9},
             2: {"job": None, "progress_ts": now - 100}}
    assert sup._stalled(beats, 3) == 1  # oldest progress among ranks in the job
    beats[1]["progress_ts"] = now - 1
    assert sup._stalled(beats, 3) is None  # idle rank 2 never counts
    b = RankBeat(store, "h", 0, gen=3, gpu=5, interval=0.05).start()
    b.set_job({"job_id": "a", "run_token": "t"})
    assert sup._beats(1, 3)[0]["gpu"] == 5 and sup._beats(1, 4) == {}
    b.stop()
    assert store.get(rank_key("h", 0)) is None
    monkeypatch.setenv("TV_NODE_JOB_RESTARTS", "1")
    store.hset("job:a", mapping={"job_id": "a", "filename": "x.y4m", "status": "RUNNING"})
    rq = _requeue("h", lambda m: None)
    assert rq({"job_id": "a", "run_token": "t"}, "rank 1 died") is True
    assert json.loads(store.lpop(queue_key("h")))["run_token"] == "t"
    assert rq({"job_id": "a", "run_token": "t"}, "rank 1 died") is False
    assert store.hget("job:a", "status") == "FAILED" and "2 times" in store.hget("job:a", "error")
