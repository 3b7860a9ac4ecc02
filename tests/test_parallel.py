"""Distributed data plane on the gloo backend (world_size 2, CPU): bitstream gather,
frame scatter, RC-stats all-reduce and the SPMD node job (direct / scatter / 2-pass /
ABR ladder).  The same code runs over RCCL on MI355X ranks."""
import json
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from thinvids_amd.parallel.node_job import plan_segments, qp_plan_two_pass


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), TV_FORCE_CPU="1")
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def _comm_worker(rank, world, port, out_dir):
    import torch

    from thinvids_amd.parallel.comm import allreduce_stats, gather_bytes_to_root, scatter_frames_from_root

    dist = _init(rank, world, port)
    dev = torch.device("cpu")
    payload = bytes([rank]) * (rank * 1000)  # rank 0 sends nothing
    got = gather_bytes_to_root(payload, dev)
    frames = [np.full((4, 6), 10 * r, np.uint8) for r in range(world)] if rank == 0 else None
    mine = scatter_frames_from_root(frames, (4, 6), dev).numpy()
    s = allreduce_stats([rank + 1.0, 2.0], dev)
    res = {"scatter_ok": bool((mine == 10 * rank).all()), "stats": s.tolist()}
    if rank == 0:
        res["sizes"] = [len(x) for x in got]
        res["content_ok"] = all(x == bytes([r]) * (r * 1000) for r, x in enumerate(got))
    with open(os.path.join(out_dir, f"r{rank}.json"), "w") as f:
        json.dump(res, f)
    dist.destroy_process_group()


def test_comm_gloo_world2(tmp_path):
    mp.spawn(_comm_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r0 = json.load(open(tmp_path / "r0.json"))
    r1 = json.load(open(tmp_path / "r1.json"))
    assert r0["sizes"] == [0, 1000] and r0["content_ok"]
    assert r0["scatter_ok"] and r1["scatter_ok"]
    assert r0["stats"] == [3.0, 4.0] == r1["stats"]


def test_plan_and_qp_model():
    assert plan_segments(100, 30, 8) == [(0, 32), (32, 32), (64, 32), (96, 4)]
    bits = np.array([8e6, 2e6, 2e6])
    qp = qp_plan_two_pass(bits, [64, 64, 64], 27, target_bits=bits.sum())
    assert qp[0] > 27 > qp[1] - 1 and qp[1] == qp[2]  # complex segment coarser, easy ones finer
    assert (qp_plan_two_pass(bits, [64] * 3, 27, target_bits=bits.sum() / 4) > qp).all()


def _job_worker(rank, world, port, src, out, kw, res_path):
    from thinvids_amd.parallel.node_job import run_job

    dist = _init(rank, world, port)
    res = run_job(src, out, software=True, **kw)
    if rank == 0:
        with open(res_path, "w") as f:
            json.dump(res, f)
    dist.destroy_process_group()


@pytest.fixture(scope="module")
def source(tmp_path_factory):
    from thinvids_amd.models import hevc, media

    d = tmp_path_factory.mktemp("src")
    frames = [hevc.synth_frame(9, t, 128, 96) for t in range(24)]
    p = d / "clip.y4m"
    media.write_y4m(str(p), frames, 24, 1)
    return str(p), frames


@pytest.mark.parametrize("kw", [dict(mode="direct"), dict(mode="scatter"),
                                dict(mode="direct", bitrate_kbps=300.0)])
def test_node_job_world2(tmp_path, source, kw):
    from thinvids_amd.models import hevc

    src, frames = source
    out = str(tmp_path / "out.mp4")
    res_path = str(tmp_path / "res.json")
    kw = dict(gop=8, segment_frames=8, **kw)
    mp.spawn(_job_worker, args=(2, _free_port(), src, out, kw, res_path), nprocs=2, join=True)
    res = json.load(open(res_path))
    assert res["world"] == 2 and res["segments"] == 3
    with open(out, "rb") as f:
        dec = hevc.decode(hevc.demux_mp4(f.read())["annexb"], coded=False)
    assert len(dec.frames) == 24
    assert min(hevc.psnr(a[0], b[0]) for a, b in zip(frames, dec.frames)) > 28
    if kw.get("bitrate_kbps"):
        assert res["passes"] == 2 and len(res["qp_plan"][0]) == 3


def test_node_job_ladder_single_process(tmp_path, source):
    """ABR ladder fan-out (rungs x segments) with Lanczos down-scaling, world 1."""
    from thinvids_amd.models import hevc
    from thinvids_amd.parallel.node_job import run_job

    os.environ["TV_FORCE_CPU"] = "1"
    src, frames = source
    res = run_job(src, str(tmp_path / "lad.mp4"), gop=8, segment_frames=16, ladder=[96, 48], software=True)
    assert [o["height"] for o in res["outputs"]] == [96, 48] and res["outputs"][1]["width"] == 64
    with open(res["outputs"][1]["path"], "rb") as f:
        dec = hevc.decode(hevc.demux_mp4(f.read())["annexb"], coded=False)
    assert len(dec.frames) == 24 and dec.frames[0][0].shape == (48, 64)
