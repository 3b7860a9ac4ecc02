"""CPU codec core: CABAC syntax writer + decoder oracle + reference encoder round trips."""
import numpy as np
import pytest

from thinvids_amd.models import hevc


def _frames(seed, n, w, h):
    return [hevc.synth_frame(seed, t, w, h) for t in range(n)]


@pytest.mark.parametrize("w,h,qp,deblock", [(96, 64, 27, False), (192, 128, 27, True),
                                             (160, 90, 22, True), (128, 96, 40, True),
                                             (64, 64, 12, True)])
def test_decode_equals_encoder_recon(w, h, qp, deblock):
    frames = _frames(3, 4, w, h)
    bs, recons = hevc.encode_sequence_cpu(frames, qp=qp, deblock=deblock, search_range=16)
    d = hevc.decode(bs)
    assert (d.width, d.height) == (w, h)
    assert len(d.frames) == len(frames)
    for r, dd in zip(recons, d.coded_frames):
        for a, b in zip(r, dd):
            np.testing.assert_array_equal(a, b)
    ps = [hevc.psnr_yuv(f, x)["y"] for f, x in zip(frames, d.frames)]
    assert min(ps) > {12: 45, 22: 40, 27: 35, 40: 27}[qp]


def test_multiple_idr_segments_concatenate():
    frames = _frames(5, 6, 96, 64)
    bs, recons = hevc.encode_sequence_cpu(frames, qp=30, gop=3, search_range=16)
    d = hevc.decode(bs)
    assert len(d.frames) == 6
    for r, dd in zip(recons, d.coded_frames):
        np.testing.assert_array_equal(r[0], dd[0])


def test_synth_deterministic_and_moving():
    a = hevc.synth_frame(9, 5, 128, 96)
    b = hevc.synth_frame(9, 5, 128, 96)
    c = hevc.synth_frame(9, 6, 128, 96)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    assert not np.array_equal(a[0], c[0])
    assert a[0].std() > 10


def test_mp4_roundtrip():
    frames = _frames(2, 3, 96, 64)
    bs, _ = hevc.encode_sequence_cpu(frames, qp=27, search_range=16)
    mp4 = hevc.mux_mp4(bs, 96, 64, 30, 1)
    assert mp4[4:8] == b"ftyp"
    assert mp4.index(b"moov") < mp4.index(b"mdat")  # faststart layout
    dm = hevc.demux_mp4(mp4)
    assert (dm["width"], dm["height"], dm["frames"]) == (96, 64, 3)
    assert abs(dm["fps"] - 30.0) < 1e-6
    d1, d2 = hevc.decode(bs), hevc.decode(dm["annexb"])
    for a, b in zip(d1.frames, d2.frames):
        np.testing.assert_array_equal(a[0], b[0])


def test_write_frame_from_decisions_matches_encoder():
    frames = _frames(4, 2, 96, 64)
    # write_frame: one substream, the frame at the sequence QP (no I P P P cascade)
    enc = hevc.CpuEncoder(96, 64, qp=27, search_range=16, wpp=False, cascade=False)
    out = enc.encode(frames[0], True, 0)
    dec = enc.decisions()
    # re-run golden pass B from the decisions and entropy-code it separately
    cbf, coef, rec = hevc.reconstruct_reference(96, 64, 27, tuple(np.pad(p, ((0, (32 - p.shape[0] % 32) % 32 // (1 if i == 0 else 2)), (0, 0)), mode="edge") for i, p in enumerate(frames[0])), None, dec)
    np.testing.assert_array_equal(cbf, dec["cbf"])
    out2 = hevc.write_frame(96, 64, 27, True, 0, dec, coef)
    assert out2 == out


@pytest.mark.parametrize("qp,deblock", [(32, True), (22, True), (27, False)])
def test_sao_roundtrip_and_gain(qp, deblock):
    """SAO (edge/band offsets, merges, chroma-shared type): the oracle decoder reproduces the
    encoder's in-loop reconstruction exactly, and SAO does not lower PSNR."""
    frames = _frames(4, 6, 192, 128)
    res = {}
    for sao in (False, True):
        enc = hevc.CpuEncoder(192, 128, qp=qp, deblock=deblock, sao=sao, search_range=16)
        bs, recons = b"", []
        for i, f in enumerate(frames):
            bs += enc.encode(f, i == 0, i)
            recons.append(enc.recon())
        d = hevc.decode(bs)
        for r, c in zip(recons, d.coded_frames):
            for p in range(3):
                np.testing.assert_array_equal(r[p], c[p])
        res[sao] = np.mean([hevc.psnr(a[0], b[0]) for a, b in zip(frames, d.frames)])
    assert res[True] >= res[False] - 0.01


def test_range_decode_and_header_probe_stream_long_inputs(tmp_path):
    """A source HEVC/MP4 is probed from headers only and read by range from the preceding
    IDR (verdict r1: HevcSource decoded whole files into RAM)."""
    from thinvids_amd.models import media

    frames = [hevc.synth_frame(2, t, 96, 64) for t in range(12)]
    bs, _ = hevc.encode_sequence_cpu(frames, qp=30, gop=4, search_range=16)
    info = hevc.probe_annexb(bs)
    assert info == {"width": 96, "height": 64, "frames": 12, "idrs": 3}
    full = hevc.decode(bs, coded=False).frames
    part = hevc.decode(bs, coded=False, first=5, count=4).frames
    assert len(part) == 4
    for a, b in zip(full[5:9], part):
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)
    p = tmp_path / "s.mp4"
    p.write_bytes(hevc.mux_mp4(bs, 96, 64, 25, 1))
    src = media.HevcSource(str(p))
    assert (src.width, src.height, src.nframes) == (96, 64, 12)
    got = src.read(10, 5)
    assert len(got) == 2 and np.array_equal(got[1][0], full[11][0])


def test_per_frame_slice_qp_round_trips():
    """Rate control sets a slice QP per frame (slice_qp_delta vs the PPS init QP, CABAC
    contexts from SliceQpY): the decoder oracle reproduces the encoder's reconstruction and
    bits fall as QP rises."""
    frames = [hevc.synth_frame(3, t, 128, 96) for t in range(6)]
    qps = [22, 30, 26, 34, 28, 40]
    bs, recons = hevc.encode_sequence_cpu(frames, qp=27, frame_qps=qps, search_range=16)
    d = hevc.decode(bs)
    for r, c in zip(recons, d.coded_frames):
        np.testing.assert_array_equal(r[0], c[0])
        np.testing.assert_array_equal(r[1], c[1])
    lo, _ = hevc.encode_sequence_cpu(frames, qp=24, frame_qps=[24] * 6, search_range=16)
    hi, _ = hevc.encode_sequence_cpu(frames, qp=24, frame_qps=[34] * 6, search_range=16)
    assert len(hi) < 0.6 * len(lo)


def test_crf_picks_per_frame_qp_from_lookahead():
    """In-engine CRF: every frame's QP comes from its quarter-res lookahead complexity
    (tv/rc_model.h); busier content gets a higher QP, the stream decodes exactly."""
    frames = [hevc.synth_frame(3, t, 160, 96) for t in range(6)]
    bs, recons = hevc.encode_sequence_cpu(frames, qp=27, crf=27, search_range=16)
    d = hevc.decode(bs)
    for r, c in zip(recons, d.coded_frames):
        np.testing.assert_array_equal(r[0], c[0])
    flat = [(np.full((96, 160), 100 + t, np.uint8), np.full((48, 80), 128, np.uint8), np.full((48, 80), 128, np.uint8))
            for t in range(6)]
    bf, _ = hevc.encode_sequence_cpu(flat, qp=27, crf=27, search_range=16)
    assert len(bf) < len(bs)


def test_rc_log2_fixed_point():
    import ctypes as C
    import math

    # mirror of tv::rc_log2_q8 (tv/rc_model.h) in Python for a few values
    def ref(x):
        return math.floor(256 * math.log2(x))
    from thinvids_amd.models import ratecontrol  # noqa: F401
    for x in (1, 2, 3, 640, 1024, 12345, 2 ** 31 - 1):
        assert abs(ratecontrol.log2_q8(x) - ref(x)) <= 1
    del C


@pytest.mark.parametrize("w,h,sao", [(192, 128, False), (320, 200, True), (1920, 1080, True)])
def test_wpp_substreams_decode_to_the_same_pictures(w, h, sao):
    """entropy_coding_sync (WPP): one CABAC substream per CTB row, contexts synced after the
    second CTB of the row above, entry points (counting emulation-prevention bytes) in the
    slice header.  The reconstruction is unchanged, the oracle decodes every substream from
    its entry point, and the rate cost of the context resets is small."""
    frames = [hevc.synth_frame(3, t, w, h) for t in range(4)]
    a, ra = hevc.encode_sequence_cpu(frames, qp=27, gop=4, search_range=32, sao=sao, wpp=False)
    b, rb = hevc.encode_sequence_cpu(frames, qp=27, gop=4, search_range=32, sao=sao, wpp=True)
    assert all((x[0] == y[0]).all() for x, y in zip(ra, rb))
    assert len(b) > len(a) and len(b) < 1.03 * len(a)
    dec = hevc.decode(b, coded=False)
    assert len(dec.frames) == 4
    for x, y in zip(dec.frames, rb):
        assert (x[0] == y[0][:h, :w]).all() and (x[1] == y[1][:h // 2, :w // 2]).all()


def test_textured_synthetic_variant():
    """Seed bit 31 selects the textured source: deterministic, different from the smooth
    one, grain that changes every frame, and much harder to code at the same QP."""
    w, h = 160, 96
    a = hevc.synth_frame(9 | 0x80000000, 3, w, h)
    b = hevc.synth_frame(9 | 0x80000000, 3, w, h)
    s = hevc.synth_frame(9, 3, w, h)
    assert all((x == y).all() for x, y in zip(a, b))
    assert (a[0] != s[0]).mean() > 0.5
    t = [hevc.synth_frame(9 | 0x80000000, k, w, h) for k in range(4)]
    sm = [hevc.synth_frame(9, k, w, h) for k in range(4)]
    bt, _ = hevc.encode_sequence_cpu(t, qp=27, gop=4, search_range=32)
    bs, _ = hevc.encode_sequence_cpu(sm, qp=27, gop=4, search_range=32)
    assert len(bt) > 1.5 * len(bs)
