"""AV1 encode path (BASELINE config #4): golden encoder -> OBU stream ->
decoder oracle round trip, the packed-decision writer used by the GPU engine, IVF, and
(GPU) the gfx950 engine against the golden encoder bit for bit.  Conformance with an
independent decoder (dav1d) is pinned in tests/test_av1_conformance.py."""
import numpy as np
import pytest

from thinvids_amd.models import av1, hevc


def _frames(seed, w, h, n, t0=0):
    out = []
    for t in range(n):
        f = hevc.synth_frame(seed, t0 + t, w, h)
        out.append(tuple(f))
    return out


def _psnr_y(res, frames, w, h):
    W, H = av1.coded_size(w, h)
    return [hevc.psnr(f[0], r[:W * H].reshape(H, W)[:h, :w]) for f, r in zip(frames, res.recon)]


@pytest.mark.parametrize("w,h,q", [(72, 40, 100), (128, 96, 60), (160, 90, 160)])
def test_golden_stream_decodes_to_golden_recon(w, h, q):
    frames = _frames(3, w, h, 4)
    res = av1.golden_encode(frames, w, h, q, cascade=False)  # constant q: the PSNR floors below
    dec = av1.decode(res.stream)
    assert (dec.width, dec.height) == (w, h)
    assert dec.frames.shape[0] == 4
    np.testing.assert_array_equal(dec.frames, res.recon)
    ps = _psnr_y(res, frames, w, h)
    assert min(ps) > {60: 40, 100: 36, 160: 30}[q]
    # inter frames code motion (mode bit 0) and most inter blocks are cheap (skip or small)
    assert ((res.mode[1:] & 1) == 1).all()
    assert res.tu_sizes[0] > res.tu_sizes[1]


def test_loop_restoration_units_round_trip():
    """Self-guided restoration units are chosen where they pay and survive the round trip
    (use_sgrproj / lr_sgr_set / subexp-coded weights)."""
    w, h = 192, 128
    frames = _frames(3, w, h, 2)
    res = av1.golden_encode(frames, w, h, 60)
    assert (res.lr[..., 0] >= 0).sum() >= 4
    dec = av1.decode(res.stream)
    np.testing.assert_array_equal(dec.frames, res.recon)


def test_skip_block_merging_on_static_content():
    """Static content: inter blocks are skip with one MV, merged into 32x32 / 64x64 blocks
    (PARTITION_NONE at 32 / 64); the stream round-trips and the P frames get cheaper."""
    w, h = 200, 136
    f0 = _frames(5, w, h, 1)[0]
    frames = [f0] * 4
    res = av1.golden_encode(frames, w, h, 120, cascade=False)
    bsz = (res.mode[1:] >> 13) & 3
    assert (bsz == 2).any() and (bsz == 1).any()
    np.testing.assert_array_equal(av1.decode(res.stream).frames, res.recon)
    # the first P frame still refines the key frame's quantisation error (1/3 dead zone),
    # then the static frames cost next to nothing
    assert max(res.tu_sizes[1:]) < res.tu_sizes[0] / 8 and res.tu_sizes[-1] < 100


def test_higher_qindex_means_fewer_bits_lower_psnr():
    w, h = 128, 64
    frames = _frames(9, w, h, 3)
    lo, hi = av1.golden_encode(frames, w, h, 50), av1.golden_encode(frames, w, h, 180)
    assert len(hi.stream) < len(lo.stream)
    assert np.mean(_psnr_y(hi, frames, w, h)) < np.mean(_psnr_y(lo, frames, w, h))


def test_packed_writer_matches_golden_stream():
    """The GPU engine's entropy path (packed nonzero TBs) writes the same bytes as the
    golden encoder's writer for the same decisions."""
    w, h, q = 96, 64, 110
    frames = _frames(5, w, h, 3)
    res = av1.golden_encode(frames, w, h, q)
    tus = av1.split_temporal_units(res.stream, res.tu_sizes)
    wr = av1.StreamWriter(w, h)
    for k in range(3):
        mode = res.mode[k]
        packed = []
        for p, lev in enumerate((res.ly[k], res.lu[k], res.lv[k])):
            nz = ((mode >> (10 + p)) & 1).astype(bool)
            packed.append(np.ascontiguousarray(lev[nz]) if nz.any() else np.zeros((1, lev.shape[1]), np.int16))
        out = wr.write(res.fparams[k], np.ascontiguousarray(mode), np.ascontiguousarray(res.mv[k]), packed[0],
                       packed[1], packed[2], np.ascontiguousarray(res.cdef_idx[k]), packed=True, seq_header=(k == 0),
                       lr=res.lr[k])
        assert out == tus[k]
    # the GPU engine's eob-truncated scan-order layout (scan_pack == k_av1e_tb_pack)
    wr = av1.StreamWriter(w, h)
    for k in range(3):
        mode = np.ascontiguousarray(res.mode[k])
        sp = [av1.scan_pack(lev, mode, p) for p, lev in enumerate((res.ly[k], res.lu[k], res.lv[k]))]
        out = wr.write(res.fparams[k], mode, np.ascontiguousarray(res.mv[k]), sp[0], sp[1], sp[2],
                       np.ascontiguousarray(res.cdef_idx[k]), packed=2, seq_header=(k == 0), lr=res.lr[k])
        assert out == tus[k]


def test_ivf_round_trip():
    w, h = 64, 48
    frames = _frames(1, w, h, 2)
    res = av1.golden_encode(frames, w, h, 90)
    tus = av1.split_temporal_units(res.stream, res.tu_sizes)
    ivf = av1.ivf_wrap(tus, w, h, 30, 1)
    info, back = av1.ivf_unwrap(ivf)
    assert info["fourcc"] == "AV01" and info["width"] == w and back == tus
    assert av1.probe(b"".join(back))["frames"] == 2


def test_qindex_mapping_monotone():
    qs = [av1.qindex_for_hevc_qp(qp) for qp in (22, 27, 32, 37)]
    assert qs == sorted(qs) and len(set(qs)) == 4
    assert abs(av1.ac_q(255) - 1828) <= 8 and av1.ac_q(0) == 4


# ---------------------------------------------------------------------------- GPU -----
def _gpu_vs_golden(w, h, starts, nframes, q, static=False, seed=11):
    import torch

    from thinvids_amd.models.av1_engine import Av1GpuEngine

    W, H = av1.coded_size(w, h)
    segs = [_frames(seed, w, h, nframes, t0) for t0 in starts]
    if static:  # the first frame repeated: skip-block merging to 32x32 / 64x64
        segs = [[s[0]] * nframes for s in segs]
    eng = Av1GpuEngine(w, h, batch=len(starts), qindex=q)
    dev = eng.dev

    def load(t, planes):
        for b, fr in enumerate(segs):
            for c, (dst, x) in enumerate(zip(planes, av1.pad_frame(fr[t], W, H))):
                dst[b].copy_(torch.from_numpy(np.ascontiguousarray(x)).to(dev))

    g = eng.encode_gop(nframes, load)
    futs = eng.submit_entropy(g)
    for b, fr in enumerate(segs):
        gold = av1.golden_encode(fr, w, h, q)
        np.testing.assert_array_equal(g.mode[:, b], gold.mode, err_msg=f"segment {b}: mode words")
        np.testing.assert_array_equal(g.mv[:, b], gold.mv, err_msg=f"segment {b}: motion vectors")
        np.testing.assert_array_equal(g.tabs[:, b, :8], gold.fparams[:, 9:17])
        np.testing.assert_array_equal(g.fbidx[:, b], gold.cdef_idx)
        np.testing.assert_array_equal(g.lr[:, b], gold.lr, err_msg=f"segment {b}: restoration units")
        tus = futs[b].result()
        assert b"".join(tus) == gold.stream, f"segment {b}: GPU bitstream differs from the golden encoder"
        last = gold.recon[-1]
        fy = eng.fin[0][b].cpu().numpy().reshape(-1)
        np.testing.assert_array_equal(fy, last[:W * H])
    eng.close()
    return g, eng


@pytest.mark.gpu
def test_gpu_av1_engine_matches_golden_small():
    _gpu_vs_golden(200, 120, [0, 7], 4, 100)


@pytest.mark.gpu
def test_gpu_av1_engine_matches_golden_textured():
    """Textured synthetic content (fine detail, per-pixel grain, fast motion: many large
    levels, Golomb escapes, little skip): GPU == golden bit for bit."""
    _gpu_vs_golden(200, 120, [0, 9], 4, 90, seed=3 | 0x80000000)


@pytest.mark.gpu
def test_gpu_av1_engine_matches_golden_merged_blocks():
    g, _ = _gpu_vs_golden(264, 200, [0, 3], 3, 120, static=True)
    assert ((g.mode[1:] >> 13) & 3).max() == 2


@pytest.mark.gpu
def test_gpu_av1_engine_matches_golden_1080p():
    """Benchmark geometry: 1920x1080 (coded 1088, split_or_horz SB rows), key + P frame."""
    g, eng = _gpu_vs_golden(1920, 1080, [3], 2, 110)
    ps = eng.psnr(g)
    assert ps["y"] > 35


def test_worker_software_av1_part_and_mp4_probe(tmp_path):
    """tv_codec=av1 through the worker's segment encoder (software path = golden encoder):
    parts -> OBU streams -> stitched av01 MP4 -> probe / decode back."""
    from thinvids_amd.models import media
    from thinvids_amd.worker.encoder import EncodeSpec, PartStats, encode_parts

    w, h = 80, 48
    parts = [_frames(4, w, h, 5, 0), _frames(4, w, h, 3, 5)]
    spec = EncodeSpec(width=w, height=h, qp=27, gop=4, software=True, codec="av1")
    stats = [PartStats(), PartStats()]
    bits = encode_parts(parts, spec, stats=stats)
    assert all(b[:2] == b"\x12\x00" for b in bits)
    assert [s.frames for s in stats] == [5, 3]
    out = tmp_path / "out.mp4"
    hevc.mux_mp4_file(bits, w, h, 30, 1, str(out))
    info = media.probe(str(out))
    assert info["codec"] == "av1" and info["frames"] == 8 and (info["width"], info["height"]) == (w, h)
    src = media.open_source(str(out))
    got = src.read(5, 3)
    dec = av1.decode(bits[1])
    for k in range(3):
        np.testing.assert_array_equal(got[k][0], dec.planes(k)[0])


def test_stitch_concat_parts_av1(tmp_path):
    """The split/encode/stitch path with tv_codec=av1: two av01 part MP4s through the
    stitcher's concat_parts give one av01 MP4 whose samples are the parts' frames."""
    from thinvids_amd.models import media
    from thinvids_amd.worker.tasks import concat_parts

    w, h = 80, 48
    parts = [_frames(4, w, h, 4, 0), _frames(4, w, h, 3, 4)]
    paths = []
    for i, fr in enumerate(parts):
        bits = av1.golden_encode(fr, w, h, 100).stream
        pth = tmp_path / f"enc_{i + 1:03d}.mp4"
        hevc.mux_mp4_file([bits], w, h, 30, 1, str(pth))
        paths.append(str(pth))
    out, n = concat_parts(paths, str(tmp_path / "job_output.mp4"), w, h, 30, 1)
    info = media.probe(out)
    assert info["codec"] == "av1" and info["frames"] == 7 and n > 0
    src = media.open_source(out)
    got = src.read(4, 3)
    dec = av1.decode(av1.golden_encode(parts[1], w, h, 100).stream)
    for k in range(3):
        np.testing.assert_array_equal(got[k][0], dec.planes(k)[0])


@pytest.mark.gpu
def test_gpu_worker_av1_parts_match_golden():
    """The worker's GPU path for tv_codec=av1 (staging, per-segment q-index map) equals the
    golden encoder on each part's closed GOPs."""
    from thinvids_amd.worker.encoder import EncodeSpec, EngineCache, PartStats, encode_parts

    w, h = 96, 64
    parts = [_frames(6, w, h, 4, 0), _frames(6, w, h, 4, 9)]
    spec = EncodeSpec(width=w, height=h, qp=30, gop=4, codec="av1")
    cache = EngineCache(device=0, batch=4)
    bits = encode_parts(parts, spec, cache=cache, stats=[PartStats(), PartStats()])
    for p, b in zip(parts, bits):
        assert b == av1.golden_encode(p, w, h, spec.av1_qindex()).stream
    # per-frame q-index plan (2-pass / CRF): frame QPs 26..29 -> different streams, still decodable
    qps = [np.array([26, 27, 28, 29]), None]
    bits2 = encode_parts(parts, spec, cache=cache, qps=qps)
    assert bits2[1] == bits[1] and bits2[0] != bits[0]
    assert av1.decode(bits2[0]).frames.shape[0] == 4
    cache.close()


def _av1_rc_worker(rank, world, port, src, out, kbps, res_path):
    import json
    import os

    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from thinvids_amd.parallel.node_job import run_job

    res = run_job(src, out, software=True, gop=4, segment_frames=4, bitrate_kbps=kbps, batch_segments=1,
                  codec="av1")
    if rank == 0:
        with open(res_path, "w") as f:
            json.dump(res, f)
    dist.destroy_process_group()


def test_av1_two_pass_rate_control_on_two_ranks(tmp_path):
    """Config #4's 2-pass RC on AV1: pass-1 per-frame temporal-unit bits all-reduced over a
    2-rank group (gloo here, RCCL on GPUs), per-frame q-index plan in pass 2: achieved
    bitrate within +-5 % of the target; the output is an av01 MP4."""
    import json
    import socket

    import torch.multiprocessing as mp

    from thinvids_amd.models import media
    from thinvids_amd.models.ratecontrol import obu_frame_sizes

    w, h, n = 96, 64, 16
    frames = _frames(13, w, h, n)
    src = str(tmp_path / "rc.y4m")
    media.write_y4m(src, frames, 30, 1)
    base = b"".join(av1.golden_encode(frames[a:a + 4], w, h, av1.qindex_for_hevc_qp(27)).stream
                    for a in range(0, n, 4))
    assert len(obu_frame_sizes(base)) == n
    target = len(base) * 8 / (n / 30) / 1000 * 0.7
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    res_path = str(tmp_path / "res.json")
    mp.spawn(_av1_rc_worker, args=(2, port, src, str(tmp_path / "o.mp4"), target, res_path), nprocs=2, join=True)
    res = json.load(open(res_path))
    assert res["passes"] in (2, 3)
    got = res["outputs"][0]["kbps"]
    assert abs(got / target - 1) < 0.05, (got, target)
    assert media.probe(str(tmp_path / "o.mp4"))["codec"] == "av1"


@pytest.mark.gpu
def test_av1_two_pass_rate_control_gpu_engine(tmp_path, monkeypatch):
    """The same 2-pass on the AV1 GPU engine (per-segment, per-frame q-index maps)."""
    from thinvids_amd.models import media
    from thinvids_amd.parallel.node_job import run_job

    monkeypatch.delenv("TV_FORCE_CPU", raising=False)
    frames = _frames(12, 256, 160, 64)
    src = str(tmp_path / "rc.y4m")
    media.write_y4m(src, frames, 30, 1)
    r1 = run_job(src, str(tmp_path / "a.mp4"), gop=16, segment_frames=16, codec="av1")
    target = r1["outputs"][0]["kbps"] * 0.6
    r2 = run_job(src, str(tmp_path / "b.mp4"), gop=16, segment_frames=16, bitrate_kbps=target, codec="av1")
    assert r2["passes"] in (2, 3) and abs(r2["outputs"][0]["kbps"] / target - 1) < 0.05, (r2["outputs"], target)
    assert media.probe(str(tmp_path / "b.mp4"))["codec"] == "av1"


def test_constant_q_cascade():
    """Without a rate-control plan the key frame and the inter frames follow the low-delay
    q cascade (the HEVC engine's, tv/gop.h), exactly an explicit per-frame q-index map."""
    w, h, q = 96, 64, 100
    frames = _frames(2, w, h, 9)
    qm = av1.cascade_qmap(q, 9)
    assert qm[0] < q and len(set(qm[1:])) > 1
    casc = av1.golden_encode(frames, w, h, q)
    assert casc.stream == av1.golden_encode(frames, w, h, q, qmap=qm).stream
    assert casc.stream != av1.golden_encode(frames, w, h, q, cascade=False).stream
    np.testing.assert_array_equal(av1.decode(casc.stream).frames, casc.recon)
