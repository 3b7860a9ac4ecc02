"""Hierarchical-B coding structure (csrc/include/tv/gop.h): GOP plans, B-slice syntax
(explicit RPS, inter_pred_idc, per-list AMVP with spatial scaling, combined bi-predictive
merge candidates), bi-prediction and the decoder's DPB / output reordering."""
import numpy as np
import pytest

from thinvids_amd.models import hevc
from thinvids_amd.utils.bdrate import bd_rate


def test_gop_plan_mini_gop_4():
    p = hevc.gop_plan(16, 4)
    assert p["disp"] == [0, 4, 2, 1, 3, 8, 6, 5, 7, 12, 10, 9, 11, 15, 13, 14]
    assert p["type"][:5] == [2, 1, 0, 0, 0]
    assert (p["ref0"][2], p["ref1"][2]) == (0, 4)  # B2 between the anchors
    assert (p["ref0"][3], p["ref1"][3]) == (0, 2)  # b1
    assert (p["ref0"][4], p["ref1"][4]) == (2, 4)  # b3
    assert p["layer"][:5] == [0, 0, 1, 2, 2]
    assert (p["dpb_size"], p["num_reorder"]) == (4, 2)


@pytest.mark.parametrize("n,m", [(1, 8), (2, 8), (7, 4), (16, 8), (64, 8), (33, 16), (10, 1)])
def test_gop_plan_invariants(n, m):
    p = hevc.gop_plan(n, m)
    assert sorted(p["disp"]) == list(range(n))
    seen = set()
    for d, t, r0, r1 in zip(p["disp"], p["type"], p["ref0"], p["ref1"]):
        if t == 2:
            assert d == 0 and r0 < 0 and r1 < 0
        if t == 1:
            assert r0 in seen and r0 < d and r1 < 0
        if t == 0:
            assert r0 in seen and r1 in seen and r0 < d < r1
        seen.add(d)
    if m == 1:
        assert p["disp"] == list(range(n)) and p["num_reorder"] == 0


@pytest.mark.parametrize("w,h,n,m,sao", [(320, 192, 13, 4, True), (192, 128, 17, 8, False),
                                         (160, 96, 9, 8, True), (96, 64, 3, 4, False)])
def test_bframes_decode_equals_encoder_recon(w, h, n, m, sao):
    frames = [hevc.synth_frame(7, t, w, h) for t in range(n)]
    bs, recons = hevc.encode_sequence_cpu(frames, qp=27, bframes=m, sao=sao, search_range=32)
    d = hevc.decode(bs)
    assert len(d.coded_frames) == n
    for r, c in zip(recons, d.coded_frames):  # display order on both sides
        for a, b in zip(r, c):
            np.testing.assert_array_equal(a, b)
    info = hevc.probe_annexb(bs)
    assert info["frames"] == n and info["idrs"] == 1


def test_bframes_segments_and_range_decode():
    frames = [hevc.synth_frame(4, t, 128, 96) for t in range(20)]
    bs, recons = hevc.encode_sequence_cpu(frames, qp=30, gop=8, bframes=4, search_range=16)
    full = hevc.decode(bs)
    assert len(full.coded_frames) == 20
    for r, c in zip(recons, full.coded_frames):
        np.testing.assert_array_equal(r[0], c[0])
    part = hevc.decode(bs, first=5, count=9)  # spans two closed GOPs
    assert len(part.coded_frames) == 9
    for a, b in zip(full.coded_frames[5:14], part.coded_frames):
        np.testing.assert_array_equal(a[0], b[0])


def test_bframes_per_frame_base_qp():
    frames = [hevc.synth_frame(3, t, 128, 96) for t in range(9)]
    qps = [22, 30, 26, 34, 28, 40, 25, 31, 29]
    bs, recons = hevc.encode_sequence_cpu(frames, qp=27, frame_qps=qps, bframes=8, search_range=16)
    d = hevc.decode(bs)
    for r, c in zip(recons, d.coded_frames):
        np.testing.assert_array_equal(r[1], c[1])


def test_bframes_lower_rate_at_equal_psnr():
    """The point of the structure: fewer bits at the same PSNR-Y than I P P P (BD-rate over
    three QPs on the bench content, golden encoder = GPU engine)."""
    w, h = 256, 160
    frames = [hevc.synth_frame(1, t, w, h) for t in range(17)]

    def curve(m):
        r, p = [], []
        for qp in (24, 30, 36):
            bs, rec = hevc.encode_sequence_cpu(frames, qp=qp, bframes=m, sao=True, search_range=32)
            mse = np.mean([np.mean((f[0].astype(float) - x[0][:h, :w]) ** 2) for f, x in zip(frames, rec)])
            r.append(len(bs) * 8)
            p.append(10 * np.log10(255 ** 2 / mse))
        return r, p

    ra, pa = curve(1)
    rb, pb = curve(8)
    assert bd_rate(ra, pa, rb, pb) < -5.0


def test_bd_rate_helper():
    r, p = [1000, 600, 360, 220], [45.0, 42.0, 39.0, 36.0]
    assert abs(bd_rate(r, p, r, p)) < 1e-9
    assert abs(bd_rate(r, p, [x * 0.9 for x in r], p) + 10.0) < 1e-6


def _gpu_engine(**kw):
    from thinvids_amd.models.gpu_engine import GpuEngine
    return GpuEngine(**kw)


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,m,gop,sao,seed", [(192, 128, 4, 9, False, 5), (192, 128, 8, 17, True, 5),
                                                (320, 192, 8, 12, True, 7 | 0x80000000), (160, 90, 2, 5, False, 3)])
def test_gpu_bframes_bit_exact(w, h, m, gop, sao, seed):
    """The GPU engine's hierarchical-B streams (per-list fine search, bi decision, exact
    bi-prediction, DPB of phase planes) equal the golden encoder's byte for byte."""
    rng = 32
    eng = _gpu_engine(width=w, height=h, qp=27, batch=2, gop=gop, search_range=rng, sao=sao, seed=seed, bframes=m)
    segs = eng.encode_synthetic([0, 10])
    for b, start in enumerate([0, 10]):
        frames = [hevc.synth_frame(seed, start + f, w, h) for f in range(gop)]
        cpu_bs, recons = hevc.encode_sequence_cpu(frames, qp=27, sao=sao, search_range=rng, bframes=m)
        assert segs[b] == cpu_bs, f"segment {b}: GPU bitstream differs from the golden encoder"
        d = hevc.decode(segs[b])
        assert len(d.coded_frames) == gop
        gy, gu, _ = eng.last_recon(b)  # last display frame
        np.testing.assert_array_equal(d.coded_frames[-1][0], gy)
        np.testing.assert_array_equal(d.coded_frames[-1][1], gu)
    eng.close()


@pytest.mark.gpu
def test_gpu_bframes_qp_map_and_benchmark_geometry():
    """1080p, search range 64, two stream groups, SAO, a per-frame base QP map (display
    order) under the layer offsets: bit-exact with the golden encoder."""
    w, h, gop, m = 1920, 1080, 9, 8
    eng = _gpu_engine(width=w, height=h, qp=27, batch=4, gop=gop, search_range=64, sao=True, seed=3, bframes=m)
    qmap = np.array([[27, 29, 25, 27, 30, 26, 27, 28, 27]] * 4, np.int8)
    qmap[2] += 2
    starts = [0, 100, 200, 300]
    segs = eng.encode_synthetic(starts, qp=qmap)
    for b in (2,):
        frames = [hevc.synth_frame(3, starts[b] + f, w, h) for f in range(gop)]
        cpu_bs, _ = hevc.encode_sequence_cpu(frames, qp=27, sao=True, search_range=64, bframes=m,
                                             frame_qps=list(qmap[b]))
        assert segs[b] == cpu_bs
    eng.close()


def _box_payload(data: bytes, path: list[str]):
    """Payload of the first box at `path` (container boxes descended in order)."""
    import struct

    def find(buf, typ):
        o = 0
        while o + 8 <= len(buf):
            n, t = struct.unpack(">I4s", buf[o:o + 8])
            if t.decode() == typ:
                return buf[o + 8:o + n]
            o += n
        return None

    b = data
    for t in path:
        b = find(b, t)
        if b is None:
            return None
    return b


def test_bframes_mp4_ctts_and_mkv_pts(tmp_path):
    """Containers carry the reordering: MP4 gets ctts (composition offsets, non-negative)
    plus an edit list starting the presentation at the first display frame; Matroska blocks
    stay in decoding order with presentation timestamps; both demux to the same pictures."""
    import struct

    from thinvids_amd.models import streams

    frames = [hevc.synth_frame(2, t, 96, 64) for t in range(9)]
    bs, _ = hevc.encode_sequence_cpu(frames, qp=30, bframes=4, search_range=16)
    mp4 = hevc.mux_mp4(bs, 96, 64, 25, 1)
    ctts = _box_payload(mp4, ["moov", "trak", "mdia", "minf", "stbl", "ctts"])
    assert ctts is not None
    n = struct.unpack(">I", ctts[4:8])[0]
    offs = []
    for k in range(n):
        c, o = struct.unpack(">II", ctts[8 + 8 * k:16 + 8 * k])
        offs += [o] * c
    delta = 1000  # fps_den * 1000
    plan = hevc.gop_plan(9, 4)
    d0 = -min(d - i for i, d in enumerate(plan["disp"]))
    assert offs == [(d - i + d0) * delta for i, d in enumerate(plan["disp"])]
    elst = _box_payload(mp4, ["moov", "trak", "edts", "elst"])
    assert struct.unpack(">I", elst[12:16])[0] == d0 * delta
    dm = hevc.demux_mp4(mp4)
    assert dm["frames"] == 9
    a, b = hevc.decode(bs), hevc.decode(dm["annexb"])
    for x, y in zip(a.frames, b.frames):
        np.testing.assert_array_equal(x[0], y[0])
    # IPPP streams keep the plain layout
    ip, _ = hevc.encode_sequence_cpu(frames, qp=30, search_range=16)
    assert _box_payload(hevc.mux_mp4(ip, 96, 64, 25, 1), ["moov", "trak", "edts"]) is None
    out = str(tmp_path / "b.mkv")
    streams.mux([bs], 96, 64, 25, 1, out, [], streams.CONTAINER_MKV)
    v = streams.mkv_video(streams.mkv_read(out))
    assert [blk[0] for blk in v.blocks] == [40 * d for d in plan["disp"]]
    annexb, _, _ = streams.mkv_hevc_annexb(out)
    for x, y in zip(a.frames, hevc.decode(annexb).frames):
        np.testing.assert_array_equal(x[0], y[0])


def test_bframes_frame_sizes_display_order_and_spec_plumbing():
    """2-pass reads pass-1 bits per DISPLAY frame (the QP map the engine takes is display-
    indexed); the worker spec carries the mini-GOP (in-engine CRF keeps I P P P)."""
    from thinvids_amd.models.ratecontrol import frame_sizes
    from thinvids_amd.worker.encoder import EncodeSpec
    from thinvids_amd.worker.tasks import _pow2

    frames = [hevc.synth_frame(2, t, 96, 64) for t in range(9)]
    bs, _ = hevc.encode_sequence_cpu(frames, qp=30, bframes=8, search_range=16)
    off = hevc.display_offsets(bs)
    plan = hevc.gop_plan(9, 8)
    assert list(off) == [d - i for i, d in enumerate(plan["disp"])]
    sizes = frame_sizes(bs)
    assert len(sizes) == 9 and sum(sizes) == len(bs)
    # the two anchors (the IDR at display 0 and the P at display 8) are the biggest pictures
    assert set(np.argsort(sizes)[-2:].tolist()) == {0, 8}
    ip, _ = hevc.encode_sequence_cpu(frames, qp=30, search_range=16)
    assert not hevc.display_offsets(ip).any()
    assert EncodeSpec(96, 64, bframes=8).hevc_bframes() == 8
    assert EncodeSpec(96, 64, bframes=8, crf=27).hevc_bframes() == 1
    assert [_pow2(n) for n in (0, 1, 3, 4, 7, 8, 40)] == [1, 1, 2, 4, 4, 8, 16]


def _scale_mv_spec(mv, td, tb):
    """H.265 8.5.3.2.7 (8-179..8-183) transcribed independently of csrc/: C division
    truncates toward zero."""
    def cdiv(a, b):
        q = abs(a) // abs(b)
        return q if (a >= 0) == (b >= 0) else -q

    td = max(-128, min(127, td))
    tb = max(-128, min(127, tb))
    tx = cdiv(16384 + (abs(td) >> 1), td)
    dsf = max(-4096, min(4095, (tb * tx + 32) >> 6))
    out = []
    for v in mv:
        p = dsf * v
        s = -1 if p < 0 else 1
        out.append(max(-32768, min(32767, s * ((abs(p) + 127) >> 8))))
    return out


def test_amvp_spatial_scaling_matches_spec_formula():
    import ctypes as C

    from thinvids_amd._native import core_lib

    f = core_lib().tv_hevc_scale_mv
    f.argtypes = [C.c_int] * 4 + [C.POINTER(C.c_int)]
    rng = np.random.default_rng(3)
    out = (C.c_int * 2)()
    cases = [((7, -3), 2, -2), ((-64, 33), -4, 4), ((1, 1), 1, 3), ((5000, -4000), 3, -1), ((-1, 0), -8, 7),
             ((32767, -32768), 1, 127)]
    cases += [((int(a), int(b)), int(td), int(tb)) for a, b, td, tb in
              zip(rng.integers(-2000, 2000, 200), rng.integers(-2000, 2000, 200), rng.choice([-16, -8, -4, -3, -2, -1, 1, 2, 3, 4, 8, 16], 200),
                  rng.choice([-16, -8, -4, -3, -2, -1, 1, 2, 3, 4, 8, 16], 200))]
    for mv, td, tb in cases:
        f(mv[0], mv[1], td, tb, out)
        assert list(out) == _scale_mv_spec(mv, td, tb), (mv, td, tb)


def test_bframes_multi_segment_mp4_order(tmp_path):
    """Two hierarchical-B segments muxed into one MP4 (streaming writer and whole-file
    muxer): composition offsets restart at every IDR and the file decodes to the display
    order of both segments."""
    frames = [hevc.synth_frame(6, t, 96, 64) for t in range(14)]
    segs = [hevc.encode_sequence_cpu(frames[a:b], qp=30, bframes=4, search_range=16)[0] for a, b in ((0, 9), (9, 14))]
    ref = hevc.decode(b"".join(segs)).frames
    assert len(ref) == 14
    p = str(tmp_path / "m.mp4")
    hevc.mux_mp4_file(segs, 96, 64, 30, 1, p)
    with open(p, "rb") as fh:
        dm = hevc.demux_mp4(fh.read())
    assert dm["frames"] == 14
    got = hevc.decode(dm["annexb"]).frames
    for a, b in zip(ref, got):
        np.testing.assert_array_equal(a[0], b[0])
    for i in range(14):  # display order == source order (the two segments' pictures interleave right)
        assert hevc.psnr(frames[i][0], got[i][0]) > 30
