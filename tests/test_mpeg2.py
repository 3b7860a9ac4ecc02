"""MPEG-2 video decoder (csrc/core/mpeg2.cpp) for DVD titles.

The fixtures come from the repo's own MPEG-2 writer (an encoder that shares only the pixel
kernels -- inverse DCT, dequantisation, half-sample prediction -- with the decoder, not the
syntax): every stream must decode to the writer's reconstruction sample for sample.  The VLC
tables are checked structurally (prefix-free, Kraft sums) and against codes quoted from
ISO/IEC 13818-2 Annex B.  Parity against other MPEG-2 decoders is unpinned: none exists in
this image (the reference decodes with ffmpeg, /root/reference/worker/tasks.py:1545-1557).
"""
import numpy as np
import pytest

from thinvids_amd.models import hevc, media, mpeg2


def _frames(n=14, w=96, h=64, seed=3):
    return [hevc.synth_frame(seed, t, w, h) for t in range(n)]


def _static(n=10, w=96, h=64):
    """Mostly still content (a moving square): skipped macroblocks in P and B pictures."""
    base = hevc.synth_frame(5, 0, w, h)
    out = []
    for t in range(n):
        y = base[0].copy()
        y[8:24, 8 + 2 * t:24 + 2 * t] = 200
        out.append((y, base[1].copy(), base[2].copy()))
    return out


CONFIGS = {
    "progressive": dict(),
    "ippp": dict(bframes=0),
    "interlaced_frame_pictures": dict(interlaced=1),
    "field_pictures": dict(interlaced=1, field_pictures=1),
    "bottom_field_first": dict(interlaced=1, field_pictures=1, top_field_first=0),
    "tools": dict(alternate_scan=1, intra_vlc=1, q_scale_type=1, intra_dc_precision=2, custom_matrices=1,
                  vary_quant=1, slices_per_row=3, qscale_code=1),
    "open_gop": dict(closed_gop=0, gop=6, interlaced=1),
    "open_gop_fields_fcode3": dict(closed_gop=0, gop=5, interlaced=1, field_pictures=1, f_code=3, search=12),
}


def test_vlc_tables_are_the_standard_ones():
    def kraft(t):
        return sum(2.0 ** -len(c) for c, _ in t)

    def prefix_free(t):
        codes = sorted(c for c, _ in t)
        return all(not b.startswith(a) for a, b in zip(codes, codes[1:]))

    b14, b15 = dict((v, c) for c, v in mpeg2.table(0)), dict((v, c) for c, v in mpeg2.table(1))
    assert len(b14) == len(b15) == 111 + 2
    for t in range(7):
        assert prefix_free(mpeg2.table(t)), t
    # B.14 is complete except the all-zero prefix (start-code emulation); B.15 also leaves the
    # B.14 codes of the entries it re-codes shorter unused
    assert kraft(mpeg2.table(0)) == 1 - 2 ** -12
    assert kraft(mpeg2.table(1)) == 1 - 9 * 2 ** -12
    assert kraft(mpeg2.table(4)) == kraft(mpeg2.table(5)) == 1.0
    rl = lambda r, lv: r << 8 | lv  # noqa: E731
    assert b14[-1] == "10" and b14[-2] == "000001" and b14[rl(0, 2)] == "0100" and b14[rl(1, 1)] == "011"
    assert b14[rl(0, 40)] == "000000000010000" and b14[rl(31, 1)] == "0000000000011011"
    assert b14[rl(2, 2)] == "0000100" and b14[rl(16, 2)] == "0000000000010101"
    assert b15[-1] == "0110" and b15[rl(0, 1)] == "10" and b15[rl(0, 15)] == "11111111"
    assert b15[rl(9, 1)] == "1111000" and b15[rl(5, 2)] == "000000100" and b15[rl(1, 3)] == "1111001"
    cbp = dict((v, c) for c, v in mpeg2.table(2))
    assert cbp[60] == "111" and cbp[0] == "000000001" and cbp[63] == "001100" and cbp[1] == "01011"
    mv = dict((v, c) for c, v in mpeg2.table(3))
    assert mv[0] == "1" and mv[1] == "01" and mv[4] == "000011" and mv[16] == "0000001100"
    dcl, dcc = dict((v, c) for c, v in mpeg2.table(4)), dict((v, c) for c, v in mpeg2.table(5))
    assert dcl[0] == "100" and dcl[1] == "00" and dcl[11] == "111111111"
    assert dcc[0] == "00" and dcc[3] == "110" and dcc[11] == "1111111111"
    mba = dict((v, c) for c, v in mpeg2.table(6))
    assert mba[1] == "1" and mba[8] == "0000111" and mba[33] == "00000011000" and mba[0] == "00000001000"


def test_writer_tables_are_an_independent_transcription():
    """The fixture writer codes with its own Annex B transcription (csrc/core/mpeg2_wtab.h:
    spec bit strings, zig-zag generated from the anti-diagonals), not the decoder's numeric
    tables: the two must agree entry by entry for every table the writer uses, so a typo in
    either shows up here (and as a mis-decoded round trip below) instead of cancelling out."""
    for t in range(13):
        dec, wr = mpeg2.table(t), mpeg2.table(t, writer=True)
        assert sorted(dec) == sorted(wr), t
    # structure of the writer's copy on its own: the same Kraft sums as the decoder's
    kraft = lambda t: sum(2.0 ** -len(c) for c, _ in t)  # noqa: E731
    assert kraft(mpeg2.table(0, writer=True)) == 1 - 2 ** -12
    assert kraft(mpeg2.table(1, writer=True)) == 1 - 9 * 2 ** -12
    zz = [int(c) for c, _ in mpeg2.table(10, writer=True)]
    assert zz[:10] == [0, 1, 8, 16, 9, 2, 3, 10, 17, 24] and sorted(zz) == list(range(64))


@pytest.mark.parametrize("name", sorted(CONFIGS))
def test_decoder_reproduces_the_writer(name):
    cfg = CONFIGS[name]
    fr = _frames()
    es, units, disp, rec = mpeg2.encode(fr, **cfg)
    info = mpeg2.probe_es(es)
    assert info["frames"] == len(fr) and info["width"] == 96 and info["height"] == 64 and info["mpeg2"] == 1
    assert info["interlaced"] == cfg.get("interlaced", 0) and info["field_pictures"] == cfg.get("field_pictures", 0)
    if cfg.get("interlaced"):
        assert info["top_field_first"] == cfg.get("top_field_first", 1)
    dec = mpeg2.decode_es(es)
    assert len(dec) == len(fr)
    for k, (a, b) in enumerate(zip(rec, dec)):
        for p in range(3):
            np.testing.assert_array_equal(a[p], b[p], err_msg=f"frame {k} plane {p}")
    assert min(hevc.psnr(a[0], b[0]) for a, b in zip(fr, rec)) > 30
    assert sorted(disp) == list(range(len(fr))) and sum(len(u) for u in units) == len(es)


@pytest.mark.parametrize("name", ["progressive", "open_gop", "open_gop_fields_fcode3"])
def test_random_access(name):
    es, _, _, rec = mpeg2.encode(_frames(), **CONFIGS[name])
    rp = mpeg2.raps(es)
    assert len(rp) >= 2 and rp[0][2] == 0
    if name.startswith("open_gop"):
        assert not all(c for _, _, _, c in rp[1:])  # leading B pictures exist
    for s in range(len(rec)):
        for n in (1, 3):
            got = mpeg2.decode_es(es, s, n)
            for a, b in zip(rec[s:s + n], got):
                np.testing.assert_array_equal(a[0], b[0])
                np.testing.assert_array_equal(a[2], b[2])


def test_every_syntax_path_is_exercised():
    stats: dict = {}
    for cfg in CONFIGS.values():
        es, _, _, rec = mpeg2.encode(_frames(), **cfg)
        mpeg2.decode_es(es, stats=stats)
    for cfg in (dict(), dict(interlaced=1, field_pictures=1)):
        fr = _static()
        es, _, _, rec = mpeg2.encode(fr, **cfg)
        dec = mpeg2.decode_es(es, stats=stats)
        for a, b in zip(rec, dec):
            np.testing.assert_array_equal(a[0], b[0])
    missing = [k for k, v in stats.items() if v == 0 and k != "concealed_slices"]
    assert not missing, (missing, stats)


def test_mkv_v_mpeg2_source(tmp_path):
    fr = _frames(16)
    es, units, disp, rec = mpeg2.encode(fr, interlaced=1, closed_gop=0, gop=6)
    path = str(tmp_path / "title.mkv")
    mpeg2.mkv_write_mpeg2(path, units, disp, 96, 64, codec_private=mpeg2.codec_private_of(es))
    src = media.open_source(path)
    assert isinstance(src, mpeg2.Mpeg2Source)
    assert (src.width, src.height, src.nframes) == (96, 64, 16) and (src.fps_num, src.fps_den) == (30000, 1001)
    assert src.field_order == "tt"
    info = media.probe(path)
    assert info["codec"] == "mpeg2video" and info["field_order"] == "tt" and info["frames"] == 16
    for s, n in ((0, 16), (5, 4), (6, 1), (11, 5)):
        got = src.read(s, n)
        assert len(got) == n
        for a, b in zip(rec[s:s + n], got):
            np.testing.assert_array_equal(a[0], b[0])
            np.testing.assert_array_equal(a[1], b[1])


def test_raw_elementary_stream_source(tmp_path):
    fr = _frames(8)
    es, _, _, rec = mpeg2.encode(fr, bframes=1)
    path = tmp_path / "clip.m2v"
    path.write_bytes(es)
    src = media.open_source(str(path))
    assert src.kind == "mpeg2" and src.nframes == 8 and src.field_order == "progressive"
    got = src.read(2, 5)
    for a, b in zip(rec[2:7], got):
        np.testing.assert_array_equal(a[0], b[0])


def test_corrupt_streams_fail_cleanly():
    es, _, _, _ = mpeg2.encode(_frames(6))
    with pytest.raises(ValueError):
        mpeg2.probe_es(b"\x00\x00\x01\xb8" + b"\x00" * 16)  # no sequence header
    # a damaged slice is concealed (the latest reference's samples), the rest decodes
    _, _, _, rec = mpeg2.encode(_frames(6))
    bad = bytearray(es)
    i = bytes(bad).rfind(b"\x00\x00\x01\x02")  # the last picture's second slice
    bad[i + 5:i + 40] = b"\xff" * 35
    st: dict = {}
    got = mpeg2.decode_es(bytes(bad), stats=st)
    assert len(got) == 6 and st["concealed_slices"] >= 1
    assert sum(np.array_equal(a[0], b[0]) for a, b in zip(rec, got)) >= 4


def test_job_entropy_placement(tmp_path, monkeypatch):
    """Node-job CABAC placement: decoded sources from 720p up on the GPU coder, DVD-size
    decoded sources and y4m / synthetic sources by CPU budget (node_job.job_entropy)."""
    from thinvids_amd.parallel.node_job import job_entropy

    monkeypatch.delenv("TV_ENTROPY", raising=False)
    es, _, _, _ = mpeg2.encode(_frames(4), bframes=0)
    path = tmp_path / "clip.m2v"
    path.write_bytes(es)
    src = media.open_source(str(path))
    assert job_entropy(src, 720, 480) == "auto"
    assert job_entropy(src, 1920, 1080) == "gpu"
    y4m = tmp_path / "clip.y4m"
    with open(y4m, "wb") as f:
        f.write(b"YUV4MPEG2 W96 H64 F30:1 Ip A1:1 C420jpeg\n")
        for y, u, v in _frames(2):
            f.write(b"FRAME\n" + y.tobytes() + u.tobytes() + v.tobytes())
    assert job_entropy(media.open_source(str(y4m)), 1920, 1080) == "auto"
    monkeypatch.setenv("TV_ENTROPY", "host")
    assert job_entropy(src, 1920, 1080) == "host"
