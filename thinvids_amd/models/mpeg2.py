"""MPEG-2 video (DVD titles) as a transcode source.

The reference's DVD path rips titles with MakeMKV and remuxes the MPEG-2 video with
``-c copy`` (/root/reference/rips/dvd_rip_queue.py:1649-1668); the transcode worker then
deinterlaces DVD-native 480/576 material with bwdif (/root/reference/worker/tasks.py:475-500)
from whatever ffmpeg decodes (:1545-1557).  Here the decoder is native
(``csrc/core/mpeg2.cpp``): Matroska ``V_MPEG2`` tracks and raw elementary streams
(``.m2v``/``.mpv``) open as :class:`Mpeg2Source`, whose ``read`` decodes only the GOPs a range
needs (random access at I pictures, one GOP earlier for open GOPs).

``encode`` is the fixture writer of the same library (an independent MPEG-2 encoder whose
reconstruction the decoder must reproduce) and ``mkv_write_mpeg2`` a minimal Matroska muxer
for the tests' DVD-like inputs.  Parity against other decoders is unpinned (no other MPEG-2
decoder exists in this image); the inverse DCT is the 13818-2 Annex A definition.
"""
from __future__ import annotations

import ctypes as C
import mmap
import os
import struct
from fractions import Fraction

import numpy as np

from .._native import Bytes, core_lib, ptr, u8p

i32p = C.POINTER(C.c_int32)
i64p = C.POINTER(C.c_int64)

ES_EXTS = (".m2v", ".mpv", ".m2video")


def _lib():
    lib = core_lib()
    if not getattr(lib, "_mpeg2_sigs", False):
        lib.tv_mpeg2_last_error.restype = C.c_char_p
        lib.tv_mpeg2_encode.argtypes = [i32p, C.c_int, C.c_int, u8p, C.c_void_p, i64p, i32p, u8p]
        lib.tv_mpeg2_probe.argtypes = [u8p, C.c_size_t, i32p]
        lib.tv_mpeg2_raps.argtypes = [u8p, C.c_size_t, i64p, i64p, i32p, i32p, C.c_int]
        lib.tv_mpeg2_decode.argtypes = [u8p, C.c_size_t, C.c_int64, C.c_int64, C.c_int32, C.c_int32, C.c_int32, u8p,
                                        i32p, i64p]
        lib.tv_mpeg2_stat_name.restype = C.c_char_p
        lib.tv_mpeg2_stat_name.argtypes = [C.c_int]
        lib.tv_mpeg2_table.argtypes = [C.c_int, i32p, i32p, i32p, C.c_int]
        lib._mpeg2_sigs = True
    return lib


def _check(rc: int) -> int:
    if rc < 0:
        raise ValueError(_lib().tv_mpeg2_last_error().decode())
    return rc


def _buf(data) -> tuple[np.ndarray, int]:
    a = np.frombuffer(data, np.uint8) if not isinstance(data, np.ndarray) else data
    return a, a.size


# ------------------------------------------------------------------ writer (fixtures)
_CFG = ("width", "height", "frame_rate_code", "gop", "bframes", "qscale_code", "interlaced", "field_pictures",
        "top_field_first", "alternate_scan", "intra_vlc", "q_scale_type", "intra_dc_precision", "custom_matrices",
        "closed_gop", "vary_quant", "slices_per_row", "f_code", "search", "seed")
_DEFAULTS = dict(frame_rate_code=4, gop=12, bframes=2, qscale_code=6, interlaced=0, field_pictures=0, top_field_first=1,
                 alternate_scan=0, intra_vlc=0, q_scale_type=0, intra_dc_precision=0, custom_matrices=0, closed_gop=1,
                 vary_quant=0, slices_per_row=1, f_code=2, search=6, seed=1)


def encode(frames, **cfg):
    """Display-order I420 frames ``[(y, u, v)]`` -> (elementary stream, decoding-order frame
    units, each unit's display index, display-order reconstruction)."""
    h, w = frames[0][0].shape
    c = dict(_DEFAULTS, **cfg, width=w, height=h)
    arr = np.asarray([c[k] for k in _CFG], np.int32)
    n = len(frames)
    yuv = np.concatenate([np.concatenate([f[0].ravel(), f[1].ravel(), f[2].ravel()]) for f in frames]).astype(np.uint8)
    out = Bytes()
    sizes = np.zeros(n, np.int64)
    disp = np.zeros(n, np.int32)
    rec = np.zeros(n * w * h * 3 // 2, np.uint8)
    _check(_lib().tv_mpeg2_encode(ptr(arr, i32p), len(arr), n, ptr(yuv), out.h, ptr(sizes, i64p), ptr(disp, i32p),
                                  ptr(rec)))
    es = out.tobytes()
    units, o = [], 0
    for s in sizes:
        units.append(es[o:o + int(s)])
        o += int(s)
    return es, units, [int(d) for d in disp], _split(rec, n, w, h)


def _split(buf: np.ndarray, n: int, w: int, h: int):
    cw, ch = (w + 1) // 2, (h + 1) // 2
    fs = w * h + 2 * cw * ch
    out = []
    for i in range(n):
        f = buf[i * fs:(i + 1) * fs]
        out.append((f[:w * h].reshape(h, w), f[w * h:w * h + cw * ch].reshape(ch, cw),
                    f[w * h + cw * ch:].reshape(ch, cw)))
    return out


# ------------------------------------------------------------------ elementary streams
def probe_es(data) -> dict:
    a, n = _buf(data)
    info = np.zeros(16, np.int32)
    _check(_lib().tv_mpeg2_probe(ptr(a), n, ptr(info, i32p)))
    keys = ("width", "height", "frames", "fps_num", "fps_den", "interlaced", "top_field_first", "field_pictures",
            "progressive_sequence", "aspect", "profile_level", "raps", "mb_width", "mb_height", "mpeg2")
    return {k: int(v) for k, v in zip(keys, info)}


def raps(data) -> list[tuple[int, int, int, bool]]:
    """(offset, sequence-header offset, frames before, closed) of every I picture."""
    a, n = _buf(data)
    cnt = _check(_lib().tv_mpeg2_raps(ptr(a), n, None, None, None, None, 0))
    off, so = np.zeros(cnt, np.int64), np.zeros(cnt, np.int64)
    fb, cl = np.zeros(cnt, np.int32), np.zeros(cnt, np.int32)
    _check(_lib().tv_mpeg2_raps(ptr(a), n, ptr(off, i64p), ptr(so, i64p), ptr(fb, i32p), ptr(cl, i32p), cnt))
    return [(int(off[i]), int(so[i]), int(fb[i]), bool(cl[i])) for i in range(cnt)]


def _decode(a: np.ndarray, n: int, seq_off: int, start: int, base: int, first: int, count: int, w: int, h: int,
            stats: dict | None = None):
    cw, ch = (w + 1) // 2, (h + 1) // 2
    out = np.zeros(count * (w * h + 2 * cw * ch), np.uint8)
    got = np.zeros(count, np.int32)
    st = np.zeros(_lib().tv_mpeg2_num_stats(), np.int64)
    _check(_lib().tv_mpeg2_decode(ptr(a), n, seq_off, start, base, first, count, ptr(out), ptr(got, i32p),
                                  ptr(st, i64p)))
    if stats is not None:
        for i, v in enumerate(st):
            name = _lib().tv_mpeg2_stat_name(i).decode()
            stats[name] = stats.get(name, 0) + int(v)
    frames = _split(out, count, w, h)
    missing = [first + i for i in range(count) if not got[i]]
    if missing:
        raise ValueError(f"mpeg2: frames {missing[:4]} could not be decoded")
    return frames


def decode_es(data, first: int = 0, count: int | None = None, stats: dict | None = None):
    """Display-order frames ``[first, first + count)`` of an elementary stream (``stats``: the
    decoder's syntax-element counters are added to it)."""
    a, n = _buf(data)
    info = probe_es(a)
    count = info["frames"] - first if count is None else min(count, info["frames"] - first)
    if count <= 0:
        return []
    rp = raps(a)
    j = max(k for k in range(len(rp)) if rp[k][2] <= first) if rp and rp[0][2] <= first else 0
    if not rp[j][3] and j > 0:  # open GOP: its leading B pictures need the previous one
        j -= 1
    off, so, fb, _ = rp[j]
    return _decode(a, n, so, off, fb, first, count, info["width"], info["height"], stats)


def table(which: int, writer: bool = False) -> list[tuple[str, int]]:
    """A VLC table of the decoder (or, writer=True, of the fixture writer's independent
    transcription, csrc/core/mpeg2_wtab.h) as (code bits, value): 0 B.14 and 1 B.15 (value
    run << 8 | level; EOB -1, escape -2), 2 B.9 coded_block_pattern, 3 B.10 motion_code
    magnitude, 4 / 5 B.12 / B.13 dct_dc_size, 6 B.1 macroblock_address_increment (escape 0),
    7 / 8 / 9 macroblock_type of I / P / B (value = flags MQ 1, MF 2, MB 4, MP 8, MI 16);
    10 / 11 the zig-zag / alternate scans and 12 the non-linear quantiser_scale as
    (str(entry), index)."""
    w = which + (100 if writer else 0)
    n = _lib().tv_mpeg2_table(w, None, None, None, 0)
    code, ln, val = np.zeros(n, np.int32), np.zeros(n, np.int32), np.zeros(n, np.int32)
    _lib().tv_mpeg2_table(w, ptr(code, i32p), ptr(ln, i32p), ptr(val, i32p), n)
    if which >= 10:
        return [(str(int(c)), int(v)) for c, v in zip(code, val)]
    return [(format(int(c), f"0{int(l)}b"), int(v)) for c, l, v in zip(code, ln, val)]


# ------------------------------------------------------------------ Matroska
def _ebml_id(eid: int) -> bytes:
    n = (eid.bit_length() + 7) // 8
    return eid.to_bytes(n, "big")


def _ebml_size(n: int) -> bytes:
    for k in range(1, 9):
        if n < (1 << (7 * k)) - 1:
            return ((1 << (7 * k)) | n).to_bytes(k, "big")
    raise ValueError("EBML size")


def _el(eid: int, payload: bytes) -> bytes:
    return _ebml_id(eid) + _ebml_size(len(payload)) + payload


def _uint(eid: int, v: int) -> bytes:
    return _el(eid, v.to_bytes(max(1, (v.bit_length() + 7) // 8), "big"))


def mkv_write_mpeg2(path: str, units, unit_display, width: int, height: int, fps_num: int = 30000,
                    fps_den: int = 1001, codec_private: bytes = b"", keys=None) -> None:
    """A minimal Matroska file with one ``V_MPEG2`` track: one SimpleBlock per frame unit in
    decoding order, timestamps (ms) from the display index (MakeMKV's layout for DVD video)."""
    dur_ns = int(round(1e9 * fps_den / fps_num))
    ebml = _el(0x1A45DFA3, _uint(0x4286, 1) + _uint(0x42F7, 1) + _uint(0x42F2, 4) + _uint(0x42F3, 8)
               + _el(0x4282, b"matroska") + _uint(0x4287, 4) + _uint(0x4285, 2))
    info = _el(0x1549A966, _uint(0x2AD7B1, 1000000) + _el(0x4489, struct.pack(">d", len(units) * dur_ns / 1e6))
               + _el(0x4D80, b"thinvids-amd") + _el(0x5741, b"thinvids-amd"))
    video = _el(0xE0, _uint(0xB0, width) + _uint(0xBA, height))
    track = _el(0xAE, _uint(0xD7, 1) + _uint(0x73C5, 1) + _uint(0x83, 1) + _el(0x86, b"V_MPEG2")
                + _uint(0x23E383, dur_ns) + (_el(0x63A2, codec_private) if codec_private else b"") + video)
    tracks = _el(0x1654AE6B, track)
    if keys is None:
        keys = [u[:4] == b"\x00\x00\x01\xb3" for u in units]
    clusters = b""
    i = 0
    while i < len(units):  # a cluster per key frame (relative timestamps fit in int16)
        j = i + 1
        while j < len(units) and not keys[j]:
            j += 1
        t0 = min(int(unit_display[k] * dur_ns // 1000000) for k in range(i, j))
        body = _uint(0xE7, t0)
        for k in range(i, j):
            rel = int(unit_display[k] * dur_ns // 1000000) - t0
            blk = b"\x81" + struct.pack(">hB", rel, 0x80 if keys[k] else 0) + units[k]
            body += _el(0xA3, blk)
        clusters += _el(0x1F43B675, body)
        i = j
    seg = info + tracks + clusters
    with open(path, "wb") as f:
        f.write(ebml + _ebml_id(0x18538067) + _ebml_size(len(seg)) + seg)


def codec_private_of(es: bytes) -> bytes:
    """The sequence header (+ extensions) at the start of an elementary stream."""
    p = es.find(b"\x00\x00\x01\xb8")
    q = es.find(b"\x00\x00\x01\x00")
    cut = min(x for x in (p, q, len(es)) if x >= 0)
    return es[:cut]


# ------------------------------------------------------------------ source
class Mpeg2Source:
    """A DVD title (Matroska ``V_MPEG2``) or a raw MPEG-2 elementary stream; ``read`` decodes
    a display-order range from the random-access point before it."""
    kind = "mpeg2"

    def __init__(self, path: str):
        self.path = path
        self.fps_num, self.fps_den = 30000, 1001
        self._mkv = None
        if path.lower().endswith(".mkv"):
            from .streams import mkv_read, mkv_video

            mk = mkv_read(path)
            v = mkv_video(mk)
            if v.codec_id != "V_MPEG2":
                raise ValueError(f"{path}: not an MPEG-2 video track ({v.codec_id})")
            blocks = sorted(v.blocks, key=lambda b: b[1])  # file (= decoding) order
            if not blocks:
                raise ValueError(f"{path}: empty MPEG-2 track")
            self._priv = v.priv
            self._blocks = [(int(o), int(sz), bool(key)) for _, o, sz, key, _ in blocks]
            ts = np.asarray([b[0] for b in blocks], np.int64)
            self._disp_to_dec = np.argsort(ts, kind="stable")  # display index -> decoding index
            self._mkv = mk
            head = self._unit_bytes(0, min(len(blocks), 2))
            info = probe_es(head)
            if v.default_duration_ns:
                fr = Fraction(10 ** 9, v.default_duration_ns).limit_denominator(1001)
                self.fps_num, self.fps_den = fr.numerator, fr.denominator
            else:
                self.fps_num, self.fps_den = info["fps_num"], info["fps_den"]
            self.nframes = len(blocks)
        else:
            with open(path, "rb") as f:
                self._es = np.frombuffer(mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ), np.uint8)
            info = probe_es(self._es)
            self.fps_num, self.fps_den = info["fps_num"], info["fps_den"]
            self.nframes = info["frames"]
            self._raps = raps(self._es)
        self.width, self.height = info["width"], info["height"]
        self.interlaced = bool(info["interlaced"])
        self.top_field_first = bool(info["top_field_first"])
        self.field_order = ("tt" if self.top_field_first else "bb") if self.interlaced else "progressive"
        self.info = info

    def _unit_bytes(self, a: int, b: int) -> bytes:
        with open(self.path, "rb") as f:
            parts = [self._priv]
            for o, sz, _ in self._blocks[a:b]:
                f.seek(o)
                parts.append(f.read(sz))
        return b"".join(parts)

    def _picture_type(self, k: int) -> int:
        """picture_coding_type of block k (1 I, 2 P, 3 B; 0 unknown)."""
        o, sz, _ = self._blocks[k]
        with open(self.path, "rb") as f:
            f.seek(o)
            head = f.read(min(sz, 4096))
        i = head.find(b"\x00\x00\x01\x00")
        return (head[i + 5] >> 3) & 7 if 0 <= i and i + 5 < len(head) else 0

    def read(self, start: int, n: int):
        n = max(0, min(n, self.nframes - start))
        if n == 0:
            return []
        if self._mkv is None:
            return decode_es(self._es, start, n)
        dec = self._disp_to_dec[start:start + n]
        lo, hi = int(dec.min()), int(dec.max())
        # the B pictures after the last one needed precede the held reference in display
        # order: decode through them, or that reference would be numbered too early
        while hi + 1 < len(self._blocks) and self._picture_type(hi + 1) == 3:
            hi += 1
        keys = [i for i, b in enumerate(self._blocks) if b[2] and i <= lo]
        k = keys[-1] if keys else 0
        if len(keys) > 1:  # open GOPs: leading B pictures reference the previous GOP
            k = keys[-2]
        data = np.frombuffer(self._unit_bytes(k, hi + 1), np.uint8)
        return _decode(data, data.size, 0, 0, k, start, n, self.width, self.height)


def is_mpeg2_mkv(path: str) -> bool:
    from .streams import mkv_read, mkv_video

    try:
        return mkv_video(mkv_read(path)).codec_id == "V_MPEG2"
    except (ValueError, OSError):
        return False


def write_dvd_title(path: str, frames: int, width: int = 720, height: int = 480, unique: int = 30, seed: int = 1,
                    gop: int = 15) -> dict:
    """A DVD-like title for benchmarks: ``unique`` interlaced synthetic frames (fields half a
    frame apart) coded as closed GOPs of ``gop`` at DVD rates, repeated to ``frames`` frames in
    a Matroska ``V_MPEG2`` track (29.97 fps)."""
    from . import hevc

    src = []
    for t in range(unique):
        a = hevc.synth_frame(seed, 2 * t, width, height)
        b = hevc.synth_frame(seed, 2 * t + 1, width, height)
        y = a[0].copy()
        y[1::2] = b[0][1::2]
        src.append((y, a[1], a[2]))
    es, units, disp, _ = encode(src, interlaced=1, gop=gop, bframes=2, closed_gop=1, qscale_code=4, seed=seed)
    reps = -(-frames // unique)
    all_units, all_disp = [], []
    for r in range(reps):
        for u, d in zip(units, disp):
            all_units.append(u)
            all_disp.append(r * unique + d)
    # whole closed GOPs only: trim to the GOP boundary at or after `frames`
    keep = [k for k, d in enumerate(all_disp) if d < -(-frames // gop) * gop]
    all_units = [all_units[k] for k in keep]
    all_disp = [all_disp[k] for k in keep]
    mkv_write_mpeg2(path, all_units, all_disp, width, height, codec_private=codec_private_of(es))
    return {"frames": len(all_units), "unique": unique, "bytes": os.path.getsize(path),
            "kbps": round(sum(len(u) for u in units) * 8 / (unique / 29.97) / 1000, 1)}
