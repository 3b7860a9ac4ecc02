"""Side streams (audio, subtitles) and output containers — the ffprobe / ffmpeg-remux roles
around the video encode.

The reference's encode step re-encodes the source audio (``-c:a aac -ac 2 -b:a 192k``,
reference worker/tasks.py:68, :1570, :1584) and its stitch step copies English subtitles
into a Matroska file when the source has copy-safe ones (ffprobe stream list :503-534,
codec list :536-546, remux :2126-2223), MP4 otherwise.  Here:

* the source's audio and subtitle streams are *indexed*, not decoded: per-sample file
  offsets, sizes and timestamps from the MP4 sample tables or the Matroska clusters (the
  file is memory-mapped, nothing is loaded whole), plus sidecar files next to a raw source
  (``movie.wav`` for PCM audio, ``movie.en.srt`` / ``movie.srt`` for SubRip subtitles);
* the stitcher muxes them with the encoded video in one pass (native
  ``tv_mux_file``: interleaved faststart MP4 or Matroska with cues), reading the side
  samples from the source by offset;
* audio is carried as-is (AAC, PCM and, container permitting, anything else) — no AAC
  encoder exists in this image and a copy is lossless; the reference's 192 kb/s stereo
  re-encode is therefore a deliberate difference;
* the final container follows the reference's rule: ``.mkv`` when English subtitle
  streams we can carry exist, ``.mp4`` otherwise; unsupported English subtitle codecs
  produce the same ``subtitle_warning`` job field.

Matroska sources also provide the HEVC video itself (:func:`mkv_hevc_annexb`), so
``.mkv`` inputs whose video is HEVC are encodable; other codecs are rejected at probe.
"""
from __future__ import annotations

import ctypes as C
import mmap
import os
import re
import struct
from dataclasses import dataclass, field

import numpy as np

SIDE_AUDIO, SIDE_SUBTITLE = 1, 2
SIDE_AAC, SIDE_PCM_S16LE, SIDE_SUBRIP, SIDE_OPAQUE, SIDE_MP4_ENTRY = 1, 2, 3, 4, 5
CONTAINER_MP4, CONTAINER_MKV = 0, 1

# reference :536-546 (copy-safe into Matroska) + what we convert ourselves
COPY_SAFE_SUBS = {"ass", "ssa", "subrip", "srt", "webvtt", "hdmv_pgs_subtitle", "dvd_subtitle", "mov_text"}
ENGLISH = {"en", "eng"}

MKV_CODEC_NAMES = {
    "A_AAC": "aac", "A_AC3": "ac3", "A_EAC3": "eac3", "A_DTS": "dts", "A_OPUS": "opus", "A_VORBIS": "vorbis",
    "A_FLAC": "flac", "A_TRUEHD": "truehd", "A_MPEG/L3": "mp3", "A_MPEG/L2": "mp2", "A_PCM/INT/LIT": "pcm_s16le",
    "S_TEXT/UTF8": "subrip", "S_TEXT/ASS": "ass", "S_TEXT/SSA": "ssa", "S_ASS": "ass", "S_SSA": "ssa",
    "S_TEXT/WEBVTT": "webvtt", "S_HDMV/PGS": "hdmv_pgs_subtitle", "S_VOBSUB": "dvd_subtitle",
    "S_HDMV/TEXTST": "hdmv_text_subtitle", "V_MPEGH/ISO/HEVC": "hevc", "V_MPEG4/ISO/AVC": "h264",
    "V_MPEG2": "mpeg2video", "V_AV1": "av1", "V_VP9": "vp9",
}
MP4_CODEC_NAMES = {"mp4a": "aac", "sowt": "pcm_s16le", "twos": "pcm_s16be", "ac-3": "ac3", "ec-3": "eac3",
                   "Opus": "opus", "fLaC": "flac", "tx3g": "mov_text", "wvtt": "webvtt", "hvc1": "hevc",
                   "hev1": "hevc", "avc1": "h264", "av01": "av1"}


@dataclass
class SideStream:
    """One audio or subtitle stream, indexed (payload stays in `path` unless `data` is set)."""
    kind: int
    codec: int
    codec_name: str               # ffprobe-style name
    language: str = "und"
    timescale: int = 1000
    channels: int = 0
    sample_rate: int = 0
    bits: int = 0
    priv: bytes = b""
    mkv_codec_id: str = ""
    path: str | None = None
    data: bytes | None = None
    offsets: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint64))
    sizes: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint32))
    pts: np.ndarray = field(default_factory=lambda: np.zeros(0, np.int64))
    durs: np.ndarray = field(default_factory=lambda: np.zeros(0, np.uint32))
    default: bool = False
    title: str = ""
    origin: str = ""              # 'mp4' | 'mkv' | 'wav' | 'srt'

    @property
    def nsamples(self) -> int:
        return int(len(self.sizes))

    def carriable(self, container: int) -> bool:
        if self.codec == SIDE_OPAQUE:
            return container == CONTAINER_MKV
        if self.codec == SIDE_MP4_ENTRY:
            return container == CONTAINER_MP4
        return True

    def describe(self) -> dict:
        """ffprobe-like stream entry."""
        d = {"codec_type": "audio" if self.kind == SIDE_AUDIO else "subtitle", "codec_name": self.codec_name,
             "tags": {"language": self.language, **({"title": self.title} if self.title else {})},
             "packets": self.nsamples}
        if self.kind == SIDE_AUDIO:
            d.update(channels=self.channels, sample_rate=self.sample_rate)
        return d


def _lang3(code: str) -> str:
    c = (code or "").strip().lower()
    return {"en": "eng", "fr": "fra", "de": "deu", "es": "spa", "it": "ita", "ja": "jpn"}.get(c, c if len(c) == 3
                                                                                              else "und")


def _text_stream(cues: list[tuple[int, int, str]], language: str, codec_name: str, origin: str,
                 title: str = "") -> SideStream:
    """SubRip stream from (start_ms, end_ms, text) cues, payload in memory."""
    blob = bytearray()
    offs, sizes, pts, durs = [], [], [], []
    for a, b, txt in cues:
        raw = txt.encode("utf-8")
        offs.append(len(blob))
        sizes.append(len(raw))
        pts.append(a)
        durs.append(max(1, b - a))
        blob += raw
    return SideStream(SIDE_SUBTITLE, SIDE_SUBRIP, codec_name, language, 1000, data=bytes(blob),
                      offsets=np.asarray(offs, np.uint64), sizes=np.asarray(sizes, np.uint32),
                      pts=np.asarray(pts, np.int64), durs=np.asarray(durs, np.uint32), origin=origin, title=title)


# ----------------------------------------------------------------------------- SRT
_SRT_TIME = re.compile(r"(\d+):(\d{1,2}):(\d{1,2})[,.](\d{1,3})\s*-->\s*(\d+):(\d{1,2}):(\d{1,2})[,.](\d{1,3})")


def parse_srt(text: str) -> list[tuple[int, int, str]]:
    cues = []
    for block in re.split(r"\r?\n\s*\r?\n", text.lstrip("﻿")):
        lines = [ln.rstrip("\r") for ln in block.strip().splitlines()]
        for i, ln in enumerate(lines):
            m = _SRT_TIME.search(ln)
            if m:
                g = [int(x) for x in m.groups()]
                a = ((g[0] * 60 + g[1]) * 60 + g[2]) * 1000 + int(str(m.group(4)).ljust(3, "0"))
                b = ((g[4] * 60 + g[5]) * 60 + g[6]) * 1000 + int(str(m.group(8)).ljust(3, "0"))
                body = "\n".join(lines[i + 1:]).strip()
                if body and b > a:
                    cues.append((a, b, body))
                break
    cues.sort(key=lambda c: c[0])
    return cues


def srt_stream(path: str, language: str = "und") -> SideStream:
    with open(path, "rb") as f:
        raw = f.read()
    try:
        text = raw.decode("utf-8-sig")
    except UnicodeDecodeError:
        text = raw.decode("latin-1")
    return _text_stream(parse_srt(text), language, "subrip", "srt")


# ----------------------------------------------------------------------------- WAV
def wav_stream(path: str, block_sec: float = 1.0) -> SideStream:
    """16-bit PCM WAV as 1 s blocks (offsets into the file; nothing is read but headers)."""
    with open(path, "rb") as f:
        hdr = f.read(12)
        if len(hdr) < 12 or hdr[:4] != b"RIFF" or hdr[8:12] != b"WAVE":
            raise ValueError(f"{path}: not a RIFF/WAVE file")
        fmt = None
        pos = 12
        size = os.path.getsize(path)
        while pos + 8 <= size:
            f.seek(pos)
            cid, clen = struct.unpack("<4sI", f.read(8))
            if cid == b"fmt ":
                fmt = struct.unpack("<HHIIHH", f.read(16))
            elif cid == b"data":
                if fmt is None:
                    raise ValueError(f"{path}: data before fmt")
                tag, ch, rate, _, align, bits = fmt
                if tag not in (1, 0xFFFE) or bits != 16:
                    raise ValueError(f"{path}: only 16-bit PCM WAV is carried (format {tag}, {bits} bits)")
                data_off, data_len = pos + 8, min(clen, size - pos - 8)
                frames = data_len // align
                blk = max(1, int(rate * block_sec))
                starts = np.arange(0, frames, blk, dtype=np.int64)
                n = np.minimum(blk, frames - starts)
                return SideStream(SIDE_AUDIO, SIDE_PCM_S16LE, "pcm_s16le", "und", rate, ch, rate, 16, path=path,
                                  offsets=(data_off + starts * align).astype(np.uint64),
                                  sizes=(n * align).astype(np.uint32), pts=starts, durs=n.astype(np.uint32),
                                  default=True, origin="wav")
            pos += 8 + clen + (clen & 1)
    raise ValueError(f"{path}: no data chunk")


# ----------------------------------------------------------------------------- MP4
def _boxes(buf, start: int, end: int):
    o = start
    while o + 8 <= end:
        size, typ = struct.unpack_from(">I4s", buf, o)
        hdr = 8
        if size == 1:
            size = struct.unpack_from(">Q", buf, o + 8)[0]
            hdr = 16
        elif size == 0:
            size = end - o
        if size < hdr or o + size > end:
            raise ValueError("mp4: bad box size")
        yield typ.decode("latin-1"), o + hdr, o + size
        o += size


def _child(buf, start, end, typ):
    for t, a, b in _boxes(buf, start, end):
        if t == typ:
            return a, b
    return None


def _descr(buf, o):
    tag = buf[o]
    o += 1
    n = 0
    for _ in range(4):
        b = buf[o]
        o += 1
        n = (n << 7) | (b & 0x7F)
        if not b & 0x80:
            break
    return tag, o, n


def _esds_asc(buf, a, b) -> bytes:
    o = a + 4
    tag, o, n = _descr(buf, o)
    if tag != 3:
        return b""
    flags = buf[o + 2]
    o += 3 + (2 if flags & 0x80 else 0) + (2 if flags & 0x20 else 0)
    if flags & 0x40:
        o += 1 + buf[o]
    tag, o, n = _descr(buf, o)
    if tag != 4:
        return b""
    o += 13
    tag, o, n = _descr(buf, o)
    return bytes(buf[o:o + n]) if tag == 5 else b""


def _mp4_table(buf, stbl):
    a, b = stbl
    stts = _child(buf, a, b, "stts")
    stsz = _child(buf, a, b, "stsz")
    stsc = _child(buf, a, b, "stsc")
    co = _child(buf, a, b, "stco")
    wide = co is None
    if wide:
        co = _child(buf, a, b, "co64")
    if not (stts and stsz and stsc and co):
        raise ValueError("mp4: incomplete sample table")
    const, count = struct.unpack_from(">II", buf, stsz[0] + 4)
    sizes = (np.full(count, const, np.uint32) if const else
             np.frombuffer(buf, ">u4", count, stsz[0] + 12).astype(np.uint32))
    n_tts = struct.unpack_from(">I", buf, stts[0] + 4)[0]
    runs = np.frombuffer(buf, ">u4", 2 * n_tts, stts[0] + 8).reshape(-1, 2).astype(np.int64)
    durs = np.repeat(runs[:, 1], runs[:, 0])[:count].astype(np.uint32)
    pts = np.concatenate([[0], np.cumsum(durs.astype(np.int64))[:-1]]) if count else np.zeros(0, np.int64)
    nco = struct.unpack_from(">I", buf, co[0] + 4)[0]
    chunk_off = np.frombuffer(buf, ">u8" if wide else ">u4", nco, co[0] + 8).astype(np.uint64)
    nsc = struct.unpack_from(">I", buf, stsc[0] + 4)[0]
    sc = np.frombuffer(buf, ">u4", 3 * nsc, stsc[0] + 8).reshape(-1, 3).astype(np.int64)
    offsets = np.zeros(count, np.uint64)
    i = 0
    for e in range(nsc):
        first, per = int(sc[e, 0]), int(sc[e, 1])
        last = int(sc[e + 1, 0]) - 1 if e + 1 < nsc else nco
        for c in range(first, last + 1):
            if i >= count:
                break
            k = min(per, count - i)
            within = np.concatenate([[0], np.cumsum(sizes[i:i + k].astype(np.uint64))[:-1]]).astype(np.uint64)
            offsets[i:i + k] = chunk_off[c - 1] + within
            i += k
    if i < count:
        raise ValueError("mp4: chunk table shorter than the sample table")
    return offsets, sizes, pts.astype(np.int64), durs


def _mp4_lang(v: int) -> str:
    s = "".join(chr(((v >> sh) & 31) + 0x60) for sh in (10, 5, 0))
    return s if s.isalpha() else "und"


def mp4_streams(path: str) -> tuple[list[SideStream], list[dict]]:
    """(side streams we index, ffprobe-like entries for every trak incl. video)."""
    out, desc = [], []
    with open(path, "rb") as f, mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ) as buf:
        moov = _child(buf, 0, len(buf), "moov")
        if moov is None:
            raise ValueError(f"{path}: no moov")
        for t, a, b in _boxes(buf, *moov):
            if t != "trak":
                continue
            mdia = _child(buf, a, b, "mdia")
            if not mdia:
                continue
            hd = _child(buf, *mdia, "hdlr")
            handler = bytes(buf[hd[0] + 8:hd[0] + 12]).decode("latin-1") if hd else ""
            mdhd = _child(buf, *mdia, "mdhd")
            ver = buf[mdhd[0]]
            ts = struct.unpack_from(">I", buf, mdhd[0] + (20 if ver == 1 else 12))[0]
            lang = _mp4_lang(struct.unpack_from(">H", buf, mdhd[0] + (32 if ver == 1 else 20))[0])
            minf = _child(buf, *mdia, "minf")
            stbl = _child(buf, *minf, "stbl") if minf else None
            stsd = _child(buf, *stbl, "stsd") if stbl else None
            if not stsd:
                continue
            e0 = stsd[0] + 8
            esize, etype = struct.unpack_from(">I4s", buf, e0)
            etype = etype.decode("latin-1")
            name = MP4_CODEC_NAMES.get(etype, etype.strip())
            kind = {"soun": SIDE_AUDIO, "sbtl": SIDE_SUBTITLE, "text": SIDE_SUBTITLE, "subt": SIDE_SUBTITLE}.get(handler)
            desc.append({"codec_type": {"vide": "video", "soun": "audio"}.get(handler, "subtitle" if kind else handler),
                         "codec_name": name, "tags": {"language": lang}})
            if kind is None:
                continue
            offsets, sizes, pts, durs = _mp4_table(buf, stbl)
            if kind == SIDE_AUDIO:
                ch, _, _, _, rate = struct.unpack_from(">HHHHI", buf, e0 + 8 + 16)
                rate >>= 16
                s = SideStream(SIDE_AUDIO, SIDE_MP4_ENTRY, name, lang, ts, ch, rate or ts, 16, path=path,
                               offsets=offsets, sizes=sizes, pts=pts, durs=durs, origin="mp4",
                               priv=bytes(buf[e0:e0 + esize]))
                if etype == "mp4a":
                    es = _child(buf, e0 + 8 + 28, e0 + esize, "esds")
                    asc = _esds_asc(buf, *es) if es else b""
                    if asc:
                        s.codec, s.priv = SIDE_AAC, asc
                elif etype == "sowt":
                    s.codec, s.priv = SIDE_PCM_S16LE, b""
                out.append(s)
            elif etype == "tx3g":  # 3GPP timed text -> SubRip cues (u16 length + UTF-8, styles dropped)
                cues = []
                for o, n, p, d in zip(offsets, sizes, pts, durs):
                    if n < 2:
                        continue
                    ln = struct.unpack_from(">H", buf, int(o))[0]
                    txt = bytes(buf[int(o) + 2:int(o) + 2 + min(ln, int(n) - 2)]).decode("utf-8", "replace")
                    if txt.strip():
                        cues.append((int(p) * 1000 // ts, int(p + d) * 1000 // ts, txt))
                out.append(_text_stream(cues, lang, "mov_text", "mp4"))
            else:  # other subtitle codecs: listed (so they count as found) but not carried
                out.append(SideStream(SIDE_SUBTITLE, SIDE_MP4_ENTRY, name, lang, ts, origin="mp4"))
    return out, desc


# ----------------------------------------------------------------------------- MKV
_MKV_LEVEL1 = {0x114D9B74, 0x1549A966, 0x1654AE6B, 0x1F43B675, 0x1C53BB6B, 0x1043A770, 0x1254C367, 0x1941A469}


def _ebml_id(buf, o):
    b = buf[o]
    n = 9 - b.bit_length() if b else 0
    if not 1 <= n <= 4:
        raise ValueError("mkv: bad element id")
    return int.from_bytes(buf[o:o + n], "big"), o + n


def _ebml_size(buf, o):
    b = buf[o]
    n = 9 - b.bit_length() if b else 0
    if not 1 <= n <= 8:
        raise ValueError("mkv: bad element size")
    v = b & ((1 << (8 - n)) - 1)
    for i in range(1, n):
        v = (v << 8) | buf[o + i]
    return (None if v == (1 << (7 * n)) - 1 else v), o + n


def _elements(buf, start, end):
    o = start
    while o < end:
        eid, p = _ebml_id(buf, o)
        size, p = _ebml_size(buf, p)
        if size is None:  # unknown size (live-written segment / cluster): up to the next level-1 element
            q = p
            while q < end:
                cid, qq = _ebml_id(buf, q)
                if cid in _MKV_LEVEL1 and q != p:
                    break
                csz, qq = _ebml_size(buf, qq)
                if csz is None:
                    q = qq
                    continue
                q = qq + csz
            size = min(q, end) - p
        yield eid, p, min(p + size, end)
        o = p + size


def _uint(buf, a, b):
    return int.from_bytes(buf[a:b], "big")


def _float(buf, a, b):
    return struct.unpack(">d" if b - a == 8 else ">f", bytes(buf[a:b]))[0]


@dataclass
class MkvTrack:
    number: int
    type: int
    codec_id: str
    priv: bytes = b""
    language: str = "eng"   # Matroska's default when the element is absent
    default: bool = True
    name: str = ""
    default_duration_ns: int = 0
    width: int = 0
    height: int = 0
    rate: float = 0.0
    channels: int = 1
    bits: int = 0
    blocks: list = field(default_factory=list)   # (ts_ticks, offset, size, key, dur_ticks)


@dataclass
class MkvFile:
    timestamp_scale: int
    duration_ns: float
    tracks: dict


def _lace_sizes(buf, o, end, lacing):
    count = buf[o] + 1
    o += 1
    if lacing == 2:  # Xiph
        sizes = []
        for _ in range(count - 1):
            n = 0
            while True:
                b = buf[o]
                o += 1
                n += b
                if b != 255:
                    break
            sizes.append(n)
    elif lacing == 6:  # EBML
        first, o = _ebml_size(buf, o)
        sizes = [first]
        for _ in range(count - 2):
            b = buf[o]
            n = 9 - b.bit_length()
            raw, o2 = _ebml_size(buf, o)
            sizes.append(sizes[-1] + raw - ((1 << (7 * n - 1)) - 1))
            o = o2
    else:  # fixed
        return o, [(end - o) // count] * count
    sizes.append(end - o - sum(sizes))
    return o, sizes


def mkv_read(path: str) -> MkvFile:
    """Index a Matroska file: tracks and every block's (timestamp, file offset, size, key)."""
    with open(path, "rb") as f, mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ) as buf:
        n = len(buf)
        eid, p = _ebml_id(buf, 0)
        if eid != 0x1A45DFA3:
            raise ValueError(f"{path}: not an EBML file")
        size, p = _ebml_size(buf, p)
        seg = None
        for eid, a, b in _elements(buf, p + (size or 0), n):
            if eid == 0x18538067:
                seg = (a, b)
                break
        if seg is None:
            raise ValueError(f"{path}: no Matroska segment")
        scale, dur, tracks = 1000000, 0.0, {}
        for eid, a, b in _elements(buf, *seg):
            if eid == 0x1549A966:
                for cid, ca, cb in _elements(buf, a, b):
                    if cid == 0x2AD7B1:
                        scale = _uint(buf, ca, cb)
                    elif cid == 0x4489:
                        dur = _float(buf, ca, cb)
            elif eid == 0x1654AE6B:
                for cid, ca, cb in _elements(buf, a, b):
                    if cid != 0xAE:
                        continue
                    t = MkvTrack(0, 0, "")
                    for k, ka, kb in _elements(buf, ca, cb):
                        if k == 0xD7:
                            t.number = _uint(buf, ka, kb)
                        elif k == 0x83:
                            t.type = _uint(buf, ka, kb)
                        elif k == 0x86:
                            t.codec_id = bytes(buf[ka:kb]).decode("ascii", "replace").rstrip("\0")
                        elif k == 0x63A2:
                            t.priv = bytes(buf[ka:kb])
                        elif k == 0x22B59C:
                            t.language = bytes(buf[ka:kb]).decode("ascii", "replace").rstrip("\0")
                        elif k == 0x88:
                            t.default = bool(_uint(buf, ka, kb))
                        elif k == 0x536E:
                            t.name = bytes(buf[ka:kb]).decode("utf-8", "replace")
                        elif k == 0x23E383:
                            t.default_duration_ns = _uint(buf, ka, kb)
                        elif k == 0xE0:
                            for v, va, vb in _elements(buf, ka, kb):
                                if v == 0xB0:
                                    t.width = _uint(buf, va, vb)
                                elif v == 0xBA:
                                    t.height = _uint(buf, va, vb)
                        elif k == 0xE1:
                            for v, va, vb in _elements(buf, ka, kb):
                                if v == 0xB5:
                                    t.rate = _float(buf, va, vb)
                                elif v == 0x9F:
                                    t.channels = _uint(buf, va, vb)
                                elif v == 0x6264:
                                    t.bits = _uint(buf, va, vb)
                    tracks[t.number] = t
            elif eid == 0x1F43B675:
                cts = 0
                for cid, ca, cb in _elements(buf, a, b):
                    if cid == 0xE7:
                        cts = _uint(buf, ca, cb)
                    elif cid in (0xA3, 0xA0):
                        bdur = None
                        key = None
                        if cid == 0xA0:
                            blk = None
                            for g, ga, gb in _elements(buf, ca, cb):
                                if g == 0xA1:
                                    blk = (ga, gb)
                                elif g == 0x9B:
                                    bdur = _uint(buf, ga, gb)
                                elif g == 0xFB:
                                    key = False
                            if blk is None:
                                continue
                            ca, cb = blk
                            key = True if key is None else key
                        tn, o = _ebml_size(buf, ca)
                        rel = struct.unpack_from(">h", buf, o)[0]
                        flags = buf[o + 2]
                        o += 3
                        if key is None:
                            key = bool(flags & 0x80)
                        t = tracks.get(tn)
                        if t is None:
                            continue
                        lacing = flags & 0x06
                        if lacing:
                            o, sizes = _lace_sizes(buf, o, cb, lacing)
                        else:
                            sizes = [cb - o]
                        step = t.default_duration_ns // scale if t.default_duration_ns else 0
                        for j, sz in enumerate(sizes):
                            t.blocks.append((cts + rel + j * step, o, sz, key, bdur if len(sizes) == 1 else step))
                            o += sz
        return MkvFile(scale, dur * scale, tracks)


def _hvcc_to_ps(priv: bytes) -> tuple[int, bytes]:
    """(NAL length size, Annex-B parameter sets) of an HEVCDecoderConfigurationRecord."""
    if len(priv) < 23:
        raise ValueError("mkv: short hvcC")
    nls = (priv[21] & 3) + 1
    o, out = 23, bytearray()
    for _ in range(priv[22]):
        cnt = struct.unpack_from(">H", priv, o + 1)[0]
        o += 3
        for _ in range(cnt):
            ln = struct.unpack_from(">H", priv, o)[0]
            out += b"\0\0\0\1" + priv[o + 2:o + 2 + ln]
            o += 2 + ln
    return nls, bytes(out)


def mkv_video(mk: MkvFile) -> MkvTrack:
    vids = [t for t in mk.tracks.values() if t.type == 1]
    if not vids:
        raise ValueError("mkv: no video track")
    return vids[0]


def mkv_hevc_annexb(path: str) -> tuple[bytes, MkvTrack, MkvFile]:
    """The HEVC video track of a Matroska file as an Annex-B elementary stream."""
    mk = mkv_read(path)
    v = mkv_video(mk)
    if v.codec_id != "V_MPEGH/ISO/HEVC":
        raise ValueError(f"{path}: video codec {MKV_CODEC_NAMES.get(v.codec_id, v.codec_id)} is not decodable "
                         f"here (HEVC only)")
    nls, ps = _hvcc_to_ps(v.priv)
    out = bytearray(ps)
    with open(path, "rb") as f, mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ) as buf:
        for _, o, sz, _, _ in sorted(v.blocks, key=lambda x: x[1]):
            q, end = o, o + sz
            while q + nls <= end:
                ln = int.from_bytes(buf[q:q + nls], "big")
                q += nls
                out += b"\0\0\0\1" + buf[q:q + ln]
                q += ln
    return bytes(out), v, mk


def mkv_streams(path: str, mk: MkvFile | None = None) -> tuple[list[SideStream], list[dict]]:
    mk = mk or mkv_read(path)
    tb = 10 ** 9 // mk.timestamp_scale if mk.timestamp_scale and 10 ** 9 % mk.timestamp_scale == 0 else 1000
    out, desc = [], []
    for t in sorted(mk.tracks.values(), key=lambda x: x.number):
        name = MKV_CODEC_NAMES.get(t.codec_id, t.codec_id.lower())
        lang = _lang3(t.language) if t.language else "eng"
        desc.append({"codec_type": {1: "video", 2: "audio", 0x11: "subtitle"}.get(t.type, "data"),
                     "codec_name": name, "tags": {"language": lang, **({"title": t.name} if t.name else {})}})
        if t.type not in (2, 0x11) or not t.blocks:
            continue
        bl = sorted(t.blocks, key=lambda x: x[0])
        ts = np.asarray([x[0] for x in bl], np.int64)
        dflt = (t.default_duration_ns // mk.timestamp_scale) if t.default_duration_ns else 0
        durs = np.asarray([x[4] if x[4] else 0 for x in bl], np.int64)
        nxt = np.append(np.diff(ts), dflt or (np.median(np.diff(ts)) if len(ts) > 1 else 1))
        durs = np.where(durs > 0, durs, np.maximum(nxt, 1))
        s = SideStream(SIDE_AUDIO if t.type == 2 else SIDE_SUBTITLE, SIDE_OPAQUE, name, lang, tb,
                       t.channels, int(t.rate), t.bits, t.priv, t.codec_id, path,
                       offsets=np.asarray([x[1] for x in bl], np.uint64), sizes=np.asarray([x[2] for x in bl], np.uint32),
                       pts=ts, durs=durs.astype(np.uint32), default=t.default, title=t.name, origin="mkv")
        if t.codec_id == "S_TEXT/UTF8":
            s.codec = SIDE_SUBRIP
        elif t.codec_id == "A_PCM/INT/LIT" and t.bits == 16:
            s.codec = SIDE_PCM_S16LE
        elif t.codec_id == "A_AAC" and t.priv and t.rate:
            # AAC access units are 1024 samples: exact timing at the sample rate for MP4
            rate = int(t.rate)
            s.codec, s.timescale, s.sample_rate = SIDE_AAC, rate, rate
            s.pts = (ts * rate // tb).astype(np.int64)
            s.durs = np.full(len(ts), 1024, np.uint32)
        out.append(s)
    return out, desc


# ------------------------------------------------------------------- collection
def sidecars(src_path: str) -> list[SideStream]:
    """``base.wav`` (PCM audio) and ``base[.lang].srt`` subtitles next to the source."""
    base, _ = os.path.splitext(src_path)
    out = []
    if os.path.exists(base + ".wav"):
        out.append(wav_stream(base + ".wav"))
    d = os.path.dirname(src_path) or "."
    stem = os.path.basename(base)
    try:
        names = sorted(os.listdir(d))
    except OSError:
        names = []
    for nm in names:
        if not nm.lower().endswith(".srt") or not nm.startswith(stem):
            continue
        mid = nm[len(stem):-4]
        if mid and not re.fullmatch(r"\.[A-Za-z]{2,3}", mid):
            continue
        out.append(srt_stream(os.path.join(d, nm), _lang3(mid[1:]) if mid else "und"))
    return out


def source_streams(src_path: str) -> tuple[list[SideStream], list[dict]]:
    """Every side stream of a source (container + sidecars) and its ffprobe-like list."""
    ext = os.path.splitext(src_path)[1].lower()
    streams, desc = [], []
    try:
        if ext == ".mp4":
            streams, desc = mp4_streams(src_path)
        elif ext == ".mkv":
            streams, desc = mkv_streams(src_path)
    except (ValueError, struct.error, IndexError) as e:
        raise ValueError(f"{src_path}: cannot index streams: {e}") from e
    extra = sidecars(src_path)
    return streams + extra, desc + [s.describe() | {"codec_type": "audio" if s.kind == SIDE_AUDIO else "subtitle"}
                                    for s in extra]


@dataclass
class OutputPlan:
    container: int
    ext: str
    tracks: list
    fields: dict
    warnings: list


def plan_output(src_path: str | None, audio_index: int | None = 0) -> OutputPlan:
    """Which side streams go into the output and in which container (reference rule,
    worker/tasks.py:2126-2164: Matroska iff copy-safe English subtitles exist).  Like the
    reference's ``-map 0:a:{selected_a_stream}?`` (:1151, :1553) one audio stream is kept —
    the job's selected one (out of range: the first); ``audio_index=None`` keeps them all."""
    streams = source_streams(src_path)[0] if src_path and os.path.exists(src_path) else []
    audio = [s for s in streams if s.kind == SIDE_AUDIO]
    if audio_index is not None and audio:
        audio = [audio[audio_index if 0 <= audio_index < len(audio) else 0]]
    audio = [s for s in audio if s.nsamples]
    subs_en = [s for s in streams if s.kind == SIDE_SUBTITLE and s.language in ENGLISH]
    ok = [s for s in subs_en if s.codec_name in COPY_SAFE_SUBS and s.nsamples and s.codec != SIDE_MP4_ENTRY]
    bad = [s for s in subs_en if s not in ok]
    container = CONTAINER_MKV if ok else CONTAINER_MP4
    warnings = []
    if bad:
        warnings.append("Skipped unsupported English subtitle codecs: " +
                        ", ".join(sorted({s.codec_name or "unknown" for s in bad})))
    keep_audio = [s for s in audio if s.carriable(container)]
    dropped = [s for s in audio if s not in keep_audio]
    if dropped:
        warnings.append("Skipped audio streams the output container cannot carry: " +
                        ", ".join(sorted({s.codec_name for s in dropped})))
    for k, s in enumerate(keep_audio):
        s.default = k == 0
    tracks = keep_audio + ok
    fields = {"english_subtitles_found": len(subs_en), "english_subtitles_supported": len(ok),
              "english_subtitles_kept": len(ok), "audio_streams_kept": len(keep_audio),
              "subtitle_warning": warnings[0] if bad else ""}
    return OutputPlan(container, ".mkv" if container == CONTAINER_MKV else ".mp4", tracks, fields, warnings)


# ------------------------------------------------------------------------- muxing
class _CSide(C.Structure):
    _fields_ = [("kind", C.c_int32), ("codec", C.c_int32), ("timescale", C.c_int32), ("channels", C.c_int32),
                ("sample_rate", C.c_int32), ("bits", C.c_int32), ("is_default", C.c_int32), ("reserved", C.c_int32),
                ("lang", C.c_char * 4), ("mkv_codec_id", C.c_char_p), ("priv", C.c_void_p), ("priv_size", C.c_uint64),
                ("path", C.c_char_p), ("data", C.c_void_p), ("nsamples", C.c_int64),
                ("offsets", C.c_void_p), ("sizes", C.c_void_p), ("pts", C.c_void_p), ("durs", C.c_void_p)]


def mux(segments, width: int, height: int, fps_num: int, fps_den: int, path: str,
        tracks: list[SideStream] = (), container: int = CONTAINER_MP4) -> int:
    """Write the Annex-B segments + side streams to `path` (native writer).  Returns bytes."""
    from .hevc import check, core_lib

    lib = core_lib()
    if not getattr(lib, "_muxfile_sig", False):
        lib.tv_mux_file.argtypes = [C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.c_int, C.c_int, C.c_int, C.c_int,
                                    C.c_int, C.POINTER(_CSide), C.c_int, C.c_int, C.c_char_p,
                                    C.POINTER(C.c_ulonglong)]
        lib.tv_mux_file.restype = C.c_int
        lib.tv_side_track_size.restype = C.c_size_t
        if lib.tv_side_track_size() != C.sizeof(_CSide):
            raise RuntimeError("SideTrack layout mismatch between Python and libtvcore")
        lib._muxfile_sig = True
    segs = [s for s in segments if len(s)]
    keep = [np.frombuffer(s, np.uint8) for s in segs]
    ptrs = (C.c_void_p * max(1, len(keep)))(*[k.ctypes.data for k in keep])
    sizes = (C.c_size_t * max(1, len(keep)))(*[len(k) for k in keep])
    arr = (_CSide * max(1, len(tracks)))()
    hold = []
    for i, s in enumerate(tracks):
        offs = np.ascontiguousarray(s.offsets, np.uint64)
        szs = np.ascontiguousarray(s.sizes, np.uint32)
        pts = np.ascontiguousarray(s.pts, np.int64)
        durs = np.ascontiguousarray(s.durs, np.uint32)
        priv = np.frombuffer(s.priv, np.uint8) if s.priv else None
        data = np.frombuffer(s.data, np.uint8) if s.data is not None and len(s.data) else None
        hold += [offs, szs, pts, durs, priv, data]
        c = arr[i]
        c.kind, c.codec, c.timescale = s.kind, s.codec, int(s.timescale)
        c.channels, c.sample_rate, c.bits, c.is_default = int(s.channels), int(s.sample_rate), int(s.bits), int(s.default)
        c.lang = (s.language or "und")[:3].encode("ascii", "replace")
        c.mkv_codec_id = s.mkv_codec_id.encode() if s.mkv_codec_id else None
        c.priv = priv.ctypes.data if priv is not None else None
        c.priv_size = len(s.priv)
        c.path = s.path.encode() if (s.path and data is None) else None
        c.data = data.ctypes.data if data is not None else None
        c.nsamples = s.nsamples
        c.offsets, c.sizes, c.pts, c.durs = offs.ctypes.data, szs.ctypes.data, pts.ctypes.data, durs.ctypes.data
    out = C.c_ulonglong()
    check(lib.tv_mux_file(ptrs, sizes, len(keep), width, height, fps_num, fps_den, arr, len(tracks), container,
                          path.encode(), C.byref(out)))
    del hold
    return int(out.value)


def write_output(segments, width: int, height: int, fps_num: int, fps_den: int, base_path: str,
                 plan: OutputPlan | None) -> tuple[str, int]:
    """Mux to ``base_path`` with the plan's extension (atomically, via ``.tmp``)."""
    plan = plan or OutputPlan(CONTAINER_MP4, ".mp4", [], {}, [])
    path = os.path.splitext(base_path)[0] + plan.ext
    tmp = path + ".tmp"
    n = mux(segments, width, height, fps_num, fps_den, tmp, plan.tracks, plan.container)
    os.replace(tmp, path)
    return path, n
