"""File ingest of the node job (verdict r3 item 3): the native parallel reader
(csrc/core/io.cpp) and the GPU y4m staging path (ops/stage.read_y4m_device), the claim-ahead
prefetch in node_job, and the synthetic y4m writer the ingest bench uses."""
import ctypes as C
import os

import numpy as np
import pytest


def _pread(path, off, n, threads):
    from thinvids_amd._native import core_lib

    lib = core_lib()
    lib.tv_pread_parallel.argtypes = [C.c_char_p, C.c_longlong, C.c_longlong, C.c_void_p, C.c_int]
    lib.tv_pread_parallel.restype = C.c_longlong
    buf = np.zeros(n, np.uint8)
    got = lib.tv_pread_parallel(str(path).encode(), off, n, buf.ctypes.data, threads)
    return got, buf


@pytest.mark.parametrize("threads", [1, 3, 8])
def test_pread_parallel_matches_file(tmp_path, threads):
    data = np.random.default_rng(5).integers(0, 256, (40 << 20) + 12345, dtype=np.uint8).tobytes()
    p = tmp_path / "blob"
    p.write_bytes(data)
    got, buf = _pread(p, 777, 30 << 20, threads)
    assert got == 30 << 20 and buf.tobytes() == data[777:777 + (30 << 20)]
    got, buf = _pread(p, len(data) - 1000, 1 << 20, threads)  # the file ends first: short count
    assert got == 1000 and buf[:1000].tobytes() == data[-1000:]
    got, _ = _pread(tmp_path / "missing", 0, 10, threads)
    assert got == -1


@pytest.fixture
def y4m(tmp_path):
    from thinvids_amd.models import hevc, media

    frames = [hevc.synth_frame(4, t, 128, 96) for t in range(20)]
    p = str(tmp_path / "src.y4m")
    media.write_y4m(p, frames, 30, 1)
    return p, frames


@pytest.mark.gpu
def test_read_y4m_device_matches_host_reader(y4m):
    import torch

    from thinvids_amd.models import media
    from thinvids_amd.ops import stage

    p, frames = y4m
    src = media.Y4MSource(p)
    st = {}
    d = stage.read_y4m_device(src, 3, 9, torch.device("cuda", 0), threads=4, stats=st)
    assert d.n == 9 and st["read_bytes"] == 9 * src.info.frame_bytes
    flat = d.buf.reshape(-1)
    for c in range(3):
        off, pw, ph, stride, fs = d.planes[c]
        got = torch.as_strided(flat, (9, ph, pw), (fs, stride, 1), off).cpu().numpy()
        want = np.stack([f[c] for f in frames[3:12]])
        assert np.array_equal(got, want), c


@pytest.mark.gpu
def test_read_y4m_device_10bit(tmp_path):
    import torch

    from thinvids_amd.models import media
    from thinvids_amd.ops import stage

    rng = np.random.default_rng(1)
    frames = [tuple(rng.integers(0, 1024, s, dtype=np.uint16) for s in ((32, 48), (16, 24), (16, 24)))
              for _ in range(4)]
    p = str(tmp_path / "p10.y4m")
    media.write_y4m(p, frames, 30, 1)
    d = stage.read_y4m_device(media.Y4MSource(p), 1, 3, torch.device("cuda", 0))
    assert d.bits == 10
    flat = d.buf.reshape(-1)
    off, pw, ph, stride, fs = d.planes[2]
    got = torch.as_strided(flat, (3, ph, pw), (fs, stride, 1), off).cpu().numpy().astype(np.uint16)
    assert np.array_equal(got, np.stack([f[2] for f in frames[1:4]]))


@pytest.mark.gpu
def test_node_job_y4m_prefetch_is_transparent(tmp_path, y4m, monkeypatch):
    """Claim-ahead prefetch (next claim read + uploaded on a side thread / HIP stream while
    this one encodes) changes nothing in the output, and every byte of the file is read once."""
    from thinvids_amd.models import hevc, media
    from thinvids_amd.parallel.node_job import run_job

    monkeypatch.delenv("TV_FORCE_CPU", raising=False)
    p, frames = y4m
    outs = {}
    for pf in ("1", "0"):
        monkeypatch.setenv("TV_PREFETCH", pf)
        res = run_job(p, str(tmp_path / f"o{pf}.mp4"), gop=4, segment_frames=4, batch_segments=1, software=False)
        outs[pf] = open(res["outputs"][0]["path"], "rb").read()
        pr = res["per_rank"][0]
        assert pr["reads"] == 5 and pr["read_bytes"] == 20 * media.Y4MSource(p).info.frame_bytes
        if pf == "1":
            assert res["trace"]["node_job.prefetch"]["count"] == 4  # every claim after the first
    assert outs["1"] == outs["0"]
    dec = hevc.decode(hevc.demux_mp4(outs["1"])["annexb"], coded=False)
    assert len(dec.frames) == 20
    assert min(hevc.psnr(a[0], b[0]) for a, b in zip(frames, dec.frames)) > 30


@pytest.mark.gpu
def test_write_synth_y4m_matches_host_generator(tmp_path):
    from thinvids_amd.models import hevc, media
    from thinvids_amd.ops import stage

    p = str(tmp_path / "s.y4m")
    size = stage.write_synth_y4m(p, 160, 90, 5, seed=3, chunk=2)
    src = media.Y4MSource(p)
    assert size == os.path.getsize(p) and src.nframes == 5
    for t, f in enumerate(src.read(0, 5)):
        want = hevc.synth_frame(3, t, 160, 90)
        assert all(np.array_equal(a, b) for a, b in zip(f, want)), t


@pytest.mark.gpu
def test_read_y4m_device_many_chunks_over_copy_streams(tmp_path):
    """A range of several 32 MiB ring chunks: each reader thread's chunks go to its own DMA
    stream (TV_INGEST_STREAMS, default 4), all ordered after the caller's stream."""
    import torch

    from thinvids_amd.models import media
    from thinvids_amd.ops import stage

    rng = np.random.default_rng(9)
    w, h, n = 1920, 1080, 44  # ~137 MB: 5 chunks
    frames = [tuple(rng.integers(0, 256, s, dtype=np.uint8) for s in ((h, w), (h // 2, w // 2), (h // 2, w // 2)))
              for _ in range(n)]
    p = str(tmp_path / "big.y4m")
    media.write_y4m(p, frames, 30, 1)
    src = media.Y4MSource(p)
    d = stage.read_y4m_device(src, 2, n - 3, torch.device("cuda", 0), threads=4)
    flat = d.buf.reshape(-1)
    for c in range(3):
        off, pw, ph, stride, fs = d.planes[c]
        got = torch.as_strided(flat, (n - 3, ph, pw), (fs, stride, 1), off).cpu().numpy()
        assert np.array_equal(got, np.stack([f[c] for f in frames[2:n - 1]])), c
