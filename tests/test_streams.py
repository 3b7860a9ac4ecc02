"""Side streams and output containers (SURVEY.md §2.3 K8 audio, K10 subtitle remux, K9
concat, K11 probe): MP4 with AAC / PCM / timed-text tracks, Matroska with cues, Matroska
sources, sidecar WAV / SRT, and the stitch rule .mkv iff English subtitles are carried
(reference worker/tasks.py:2126-2223).

No ffmpeg / ffprobe / mkvinfo exists in this image, so the files are checked with our own
parsers (MP4 sample tables, EBML walker) and our own HEVC decoder; playback in third-party
players is parity unpinned.
"""
import os
import struct

import numpy as np
import pytest

from thinvids_amd.models import hevc, media, streams


@pytest.fixture(scope="module")
def clip():
    frames = [hevc.synth_frame(5, t, 96, 64) for t in range(12)]
    bs, _ = hevc.encode_sequence_cpu(frames, qp=27, search_range=16, gop=6)
    return frames, bs


def _aac_stream(n=30, rate=48000):
    rng = np.random.default_rng(1)
    blob = bytearray()
    offs, sizes = [], []
    for _ in range(n):
        k = int(rng.integers(40, 400))
        offs.append(len(blob))
        sizes.append(k)
        blob += rng.integers(0, 256, k, dtype=np.uint8).tobytes()
    return streams.SideStream(streams.SIDE_AUDIO, streams.SIDE_AAC, "aac", "eng", rate, 2, rate, 16,
                              priv=b"\x11\x90", data=bytes(blob), offsets=np.asarray(offs, np.uint64),
                              sizes=np.asarray(sizes, np.uint32), pts=np.arange(n, dtype=np.int64) * 1024,
                              durs=np.full(n, 1024, np.uint32), default=True)


def _payloads(s: streams.SideStream) -> list[bytes]:
    if s.data is not None:
        return [s.data[int(o):int(o) + int(n)] for o, n in zip(s.offsets, s.sizes)]
    with open(s.path, "rb") as f:
        out = []
        for o, n in zip(s.offsets, s.sizes):
            f.seek(int(o))
            out.append(f.read(int(n)))
        return out


def _video_offsets(path) -> np.ndarray:
    import mmap

    with open(path, "rb") as f, mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ) as buf:
        moov = streams._child(buf, 0, len(buf), "moov")
        trak = streams._child(buf, *moov, "trak")  # track 1 is the video
        mdia = streams._child(buf, *trak, "mdia")
        stbl = streams._child(buf, *streams._child(buf, *mdia, "minf"), "stbl")
        return streams._mp4_table(buf, stbl)[0]


def _write_wav(path, rate=8000, ch=2, seconds=1.5):
    t = np.arange(int(rate * seconds))
    pcm = (np.stack([np.sin(t * 0.05 * (c + 1)) for c in range(ch)], 1) * 8000).astype("<i2")
    data = pcm.tobytes()
    with open(path, "wb") as f:
        f.write(b"RIFF" + struct.pack("<I", 36 + len(data)) + b"WAVE")
        f.write(b"fmt " + struct.pack("<IHHIIHH", 16, 1, ch, rate, rate * ch * 2, ch * 2, 16))
        f.write(b"data" + struct.pack("<I", len(data)) + data)
    return data


SRT = """1
00:00:00,100 --> 00:00:00,250
Hello <b>there</b>

2
00:00:00,300 --> 00:00:00,420
Second line
two rows
"""


def test_parse_srt_and_wav(tmp_path):
    cues = streams.parse_srt("﻿" + SRT.replace("\n", "\r\n"))
    assert cues == [(100, 250, "Hello <b>there</b>"), (300, 420, "Second line\ntwo rows")]
    data = _write_wav(tmp_path / "a.wav")
    s = streams.wav_stream(str(tmp_path / "a.wav"))
    assert (s.channels, s.sample_rate, s.codec) == (2, 8000, streams.SIDE_PCM_S16LE)
    assert b"".join(_payloads(s)) == data
    assert list(s.pts) == [0, 8000] and list(s.durs) == [8000, 4000]


def test_mp4_carries_aac_and_text(tmp_path, clip):
    frames, bs = clip
    aac = _aac_stream()
    sub = streams._text_stream([(100, 250, "Hello"), (300, 420, "World\nline 2")], "eng", "subrip", "srt")
    out = str(tmp_path / "o.mp4")
    n = streams.mux([bs], 96, 64, 25, 1, out, [aac, sub], streams.CONTAINER_MP4)
    data = open(out, "rb").read()
    assert n == len(data) and data.index(b"moov") < data.index(b"mdat")
    # video still round-trips through the (chunk-walking) demuxer and decodes bit-exactly
    dm = hevc.demux_mp4(data)
    assert (dm["width"], dm["height"], dm["frames"]) == (96, 64, 12)
    for a, b in zip(hevc.decode(bs).frames, hevc.decode(dm["annexb"]).frames):
        np.testing.assert_array_equal(a[0], b[0])
    side, desc = streams.mp4_streams(out)
    assert [d["codec_type"] for d in desc] == ["video", "audio", "subtitle"]
    a2 = side[0]
    assert a2.codec == streams.SIDE_AAC and a2.priv == aac.priv and a2.language == "eng"
    assert (a2.channels, a2.sample_rate, a2.timescale) == (2, 48000, 48000)
    assert _payloads(a2) == _payloads(aac)
    np.testing.assert_array_equal(a2.pts, aac.pts)
    s2 = side[1]  # tx3g back to cues; gaps were filled with empty samples and dropped again
    assert s2.codec_name == "mov_text" and s2.language == "eng"
    assert _payloads(s2) == [b"Hello", b"World\nline 2"]
    assert list(s2.pts) == [100, 300] and list(s2.durs) == [150, 120]
    # chunks are interleaved (1 s each): at 5 fps the 12 frames span 2.4 s, and the audio's
    # first-second chunk sits between the video chunks instead of after all of them
    slow = str(tmp_path / "slow.mp4")
    streams.mux([bs], 96, 64, 5, 1, slow, [aac], streams.CONTAINER_MP4)
    a3 = streams.mp4_streams(slow)[0][0]
    vo = _video_offsets(slow)
    assert vo.min() < a3.offsets.min() < vo.max() and _payloads(a3) == _payloads(aac)


def test_mkv_roundtrip(tmp_path, clip):
    frames, bs = clip
    data = _write_wav(tmp_path / "a.wav", seconds=0.6)
    pcm = streams.wav_stream(str(tmp_path / "a.wav"), block_sec=0.25)
    sub = streams._text_stream([(40, 200, "Hi"), (240, 400, "Bye")], "eng", "subrip", "srt")
    out = str(tmp_path / "o.mkv")
    n = streams.mux([bs], 96, 64, 25, 1, out, [pcm, sub], streams.CONTAINER_MKV)
    assert n == os.path.getsize(out)
    mk = streams.mkv_read(out)
    assert mk.timestamp_scale == 1000000 and abs(mk.duration_ns / 1e6 - 600) < 1
    v = streams.mkv_video(mk)
    assert (v.codec_id, v.width, v.height, v.default_duration_ns) == ("V_MPEGH/ISO/HEVC", 96, 64, 40000000)
    assert [b[0] for b in v.blocks] == [40 * i for i in range(12)]
    assert [b[3] for b in v.blocks] == [i % 6 == 0 for i in range(12)]  # IDR every 6 frames
    annexb, _, _ = streams.mkv_hevc_annexb(out)
    for a, b in zip(hevc.decode(bs).frames, hevc.decode(annexb).frames):
        np.testing.assert_array_equal(a[0], b[0])
    side, desc = streams.mkv_streams(out)
    assert [d["codec_type"] for d in desc] == ["video", "audio", "subtitle"]
    a2, s2 = side
    assert a2.codec == streams.SIDE_PCM_S16LE and (a2.channels, a2.sample_rate, a2.bits) == (2, 8000, 16)
    assert b"".join(_payloads(a2)) == data
    assert s2.codec == streams.SIDE_SUBRIP and _payloads(s2) == [b"Hi", b"Bye"]
    assert list(s2.pts) == [40, 240] and list(s2.durs) == [160, 160]
    # clusters start at keyframes and are indexed by cues
    raw = open(out, "rb").read()
    assert raw.count(bytes.fromhex("1F43B675")) == 2 and raw.count(bytes.fromhex("BB")) >= 2
    # the MKV is itself a usable source (HEVC in Matroska)
    src = media.open_source(out)
    assert (src.width, src.height, src.nframes, src.fps_num, src.fps_den) == (96, 64, 12, 25, 1)
    pr = media.probe(out)
    assert [s["codec_type"] for s in pr["streams"]] == ["video", "audio", "subtitle"]


def test_mkv_opaque_passthrough(tmp_path, clip):
    """Matroska -> Matroska keeps tracks we do not interpret (here ASS subtitles with their
    header in CodecPrivate) byte for byte, as `-c:s copy` does."""
    _, bs = clip
    hdr = b"[Script Info]\nScriptType: v4.00+\n"
    ass = streams.SideStream(streams.SIDE_SUBTITLE, streams.SIDE_OPAQUE, "ass", "eng", 1000, priv=hdr,
                             mkv_codec_id="S_TEXT/ASS", data=b"0,0,Default,,0,0,0,,Hi",
                             offsets=np.zeros(1, np.uint64), sizes=np.asarray([22], np.uint32),
                             pts=np.asarray([80], np.int64), durs=np.asarray([100], np.uint32))
    first = str(tmp_path / "a.mkv")
    streams.mux([bs], 96, 64, 25, 1, first, [ass], streams.CONTAINER_MKV)
    side, _ = streams.mkv_streams(first)
    assert side[0].codec == streams.SIDE_OPAQUE and side[0].mkv_codec_id == "S_TEXT/ASS" and side[0].priv == hdr
    second = str(tmp_path / "b.mkv")
    streams.mux([bs], 96, 64, 25, 1, second, side, streams.CONTAINER_MKV)
    again, _ = streams.mkv_streams(second)
    assert _payloads(again[0]) == [b"0,0,Default,,0,0,0,,Hi"] and list(again[0].pts) == [80]
    with pytest.raises(RuntimeError, match="Matroska"):
        streams.mux([bs], 96, 64, 25, 1, str(tmp_path / "c.mp4"), side, streams.CONTAINER_MP4)


def test_plan_output_rule(tmp_path, clip):
    _, bs = clip
    base = tmp_path / "movie"
    media.write_y4m(str(base) + ".y4m", [hevc.synth_frame(1, 0, 32, 32)], 25, 1)
    p = streams.plan_output(str(base) + ".y4m")
    assert p.ext == ".mp4" and p.tracks == [] and p.fields["english_subtitles_found"] == 0
    _write_wav(str(base) + ".wav")
    (tmp_path / "movie.fr.srt").write_text(SRT)
    p = streams.plan_output(str(base) + ".y4m")
    assert p.ext == ".mp4" and [t.codec_name for t in p.tracks] == ["pcm_s16le"]  # French subs: not English
    (tmp_path / "movie.en.srt").write_text(SRT)
    p = streams.plan_output(str(base) + ".y4m")
    assert p.ext == ".mkv" and [t.codec_name for t in p.tracks] == ["pcm_s16le", "subrip"]
    assert p.fields["english_subtitles_found"] == 1 and p.fields["english_subtitles_kept"] == 1
    # an English subtitle codec we cannot carry -> warning, MP4
    mk = str(tmp_path / "src.mkv")
    odd = streams.SideStream(streams.SIDE_SUBTITLE, streams.SIDE_OPAQUE, "x", "eng", 1000, mkv_codec_id="S_KATE",
                             data=b"k", offsets=np.zeros(1, np.uint64), sizes=np.ones(1, np.uint32),
                             pts=np.zeros(1, np.int64), durs=np.ones(1, np.uint32))
    streams.mux([bs], 96, 64, 25, 1, mk, [odd], streams.CONTAINER_MKV)
    p = streams.plan_output(mk)
    assert p.ext == ".mp4" and "s_kate" in p.fields["subtitle_warning"]
    assert p.fields["english_subtitles_found"] == 1 and p.fields["english_subtitles_supported"] == 0
