"""Media sources, sinks and probing (replaces the reference's ffprobe / ffmpeg demux role,
SURVEY.md §2.3 K1/K11).

Readable inputs (no ffmpeg in this image, so only formats we can decode ourselves):

* ``.y4m``   — YUV4MPEG2 4:2:0, 8-bit or 10-bit (``C420p10``: HDR10 PQ masters; frames
  come back as uint16 planes and are tone-mapped on the GPU before encoding);
* ``.synth`` — JSON ``{"width", "height", "frames", "fps", "seed"}``: the procedural source
  of :mod:`thinvids_amd.models.hevc` (P5 "direct source" with zero I/O);
* ``.hevc`` / ``.265`` / ``.mp4`` / ``.mkv`` whose video is HEVC (decoded with the oracle
  decoder; Matroska is indexed by :mod:`thinvids_amd.models.streams`).  Audio and subtitle
  streams of a source (and sidecar ``.wav`` / ``.srt`` files) are listed by :func:`probe`
  and carried into the output by the stitcher.

Every source exposes ``width, height, fps_num, fps_den, nframes`` and
``read(start, n) -> list[(Y, U, V)]``.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass
from fractions import Fraction

import numpy as np

from . import hevc, mpeg2

VIDEO_EXTS = (".y4m", ".synth", ".hevc", ".265", ".mp4", ".mkv")


# ------------------------------------------------------------------------------ Y4M
@dataclass
class Y4MInfo:
    width: int
    height: int
    fps_num: int
    fps_den: int
    header_len: int
    frame_bytes: int
    nframes: int
    bits: int = 8


def _y4m_info(path: str) -> Y4MInfo:
    with open(path, "rb") as f:
        header = f.readline()
        if not header.startswith(b"YUV4MPEG2"):
            raise ValueError(f"{path}: not a YUV4MPEG2 file")
        w = h = 0
        fn, fd = 30, 1
        bits = 8
        for tok in header.decode().split()[1:]:
            if tok[0] == "W":
                w = int(tok[1:])
            elif tok[0] == "H":
                h = int(tok[1:])
            elif tok[0] == "F":
                a, b = tok[1:].split(":")
                fn, fd = int(a), int(b)
            elif tok[0] == "C":
                if tok[1:] in ("420p10",):
                    bits = 10
                elif not tok[1:].startswith("420") or tok[1:].startswith("420p1"):
                    raise ValueError(f"{path}: only 4:2:0 8-bit or 10-bit Y4M is supported (got {tok})")
        frame_hdr = f.readline()
        if frame_hdr and not frame_hdr.startswith(b"FRAME"):
            raise ValueError(f"{path}: malformed frame header")
        fhl = len(frame_hdr) if frame_hdr else 6
    plane = w * h * 3 // 2 * (2 if bits > 8 else 1)
    size = os.path.getsize(path)
    n = max(0, (size - len(header)) // (fhl + plane))
    return Y4MInfo(w, h, fn, fd, len(header), fhl + plane, n, bits)


def write_y4m(path: str, frames, fps_num: int = 30, fps_den: int = 1) -> None:
    """Write 8-bit (uint8 planes) or 10-bit (uint16 planes, ``C420p10`` little-endian) Y4M."""
    frames = list(frames)
    h, w = frames[0][0].shape
    ten = frames[0][0].dtype == np.uint16
    dt = np.dtype("<u2") if ten else np.uint8
    tmp = path + ".tmp"
    with open(tmp, "wb") as f:
        f.write(f"YUV4MPEG2 W{w} H{h} F{fps_num}:{fps_den} Ip A1:1 {'C420p10 XYSCSS=420P10' if ten else 'C420jpeg'}\n"
                .encode())
        for y, u, v in frames:
            f.write(b"FRAME\n")
            f.write(np.ascontiguousarray(y, dt).tobytes())
            f.write(np.ascontiguousarray(u, dt).tobytes())
            f.write(np.ascontiguousarray(v, dt).tobytes())
    os.replace(tmp, path)


class Y4MSource:
    kind = "rawvideo"

    def __init__(self, path: str):
        self.path = path
        self.info = _y4m_info(path)
        self.width, self.height = self.info.width, self.info.height
        self.fps_num, self.fps_den = self.info.fps_num, self.info.fps_den
        self.nframes = self.info.nframes
        self.bits = self.info.bits

    def read(self, start: int, n: int):
        """Frames [start, start + n) read straight from their byte range (random access:
        nothing before `start` is touched, so a long file streams segment by segment)."""
        out = []
        i = self.info
        n = max(0, min(n, self.nframes - start))
        ysz, csz = i.width * i.height, i.width * i.height // 4
        dt = np.dtype("<u2") if i.bits > 8 else np.uint8
        with open(self.path, "rb") as f:
            f.seek(i.header_len + start * i.frame_bytes)
            for _ in range(n):
                raw = f.read(i.frame_bytes)
                hdr = raw.index(b"\n") + 1
                buf = np.frombuffer(raw, dt, offset=hdr)
                y = buf[:ysz].reshape(i.height, i.width)
                u = buf[ysz:ysz + csz].reshape(i.height // 2, i.width // 2)
                v = buf[ysz + csz:ysz + 2 * csz].reshape(i.height // 2, i.width // 2)
                out.append((y, u, v))
        return out


# ---------------------------------------------------------------------------- synth
class SynthSource:
    kind = "synthetic"

    def __init__(self, path: str | None = None, spec: dict | None = None):
        if spec is None:
            with open(path) as f:
                spec = json.load(f)
        self.path = path
        self.spec = spec
        self.width, self.height = int(spec["width"]), int(spec["height"])
        fps = Fraction(str(spec.get("fps", 30))).limit_denominator(1001)
        self.fps_num, self.fps_den = fps.numerator, fps.denominator
        self.nframes = int(spec["frames"])
        self.seed = int(spec.get("seed", 1))
        self.start = int(spec.get("start_frame", 0))

    def read(self, start: int, n: int):
        n = max(0, min(n, self.nframes - start))
        return [hevc.synth_frame(self.seed, self.start + start + k, self.width, self.height) for k in range(n)]


def write_synth_spec(path: str, width: int, height: int, frames: int, fps=30, seed: int = 1) -> None:
    with open(path, "w") as f:
        json.dump({"width": width, "height": height, "frames": frames, "fps": fps, "seed": seed}, f)


# ----------------------------------------------------------------------------- HEVC
class HevcSource:
    """Our own HEVC elementary stream / MP4 output as a source.  Only the header is parsed
    up front (geometry, picture count); ``read`` decodes just the requested range from the
    preceding IDR, so a long file is never decoded (or held decoded) as a whole."""
    kind = "hevc"

    def __init__(self, path: str):
        self.path = path
        self.fps_num, self.fps_den = 30, 1
        if path.lower().endswith(".mkv"):
            from .streams import mkv_hevc_annexb

            data, vt, _ = mkv_hevc_annexb(path)
            if vt.default_duration_ns:
                fr = Fraction(10 ** 9, vt.default_duration_ns).limit_denominator(1001)
                self.fps_num, self.fps_den = fr.numerator, fr.denominator
        else:
            with open(path, "rb") as f:
                data = f.read()
        if path.lower().endswith(".mp4"):
            dm = hevc.demux_mp4(data)
            data = dm["annexb"]
            ts, d = dm["timescale"], dm["sample_delta"]
            if ts and d:
                fr = Fraction(ts, d).limit_denominator(1001)
                self.fps_num, self.fps_den = fr.numerator, fr.denominator
        self._annexb = data
        info = hevc.probe_annexb(data)
        self.width, self.height = info["width"], info["height"]
        self.nframes = info["frames"]

    def read(self, start: int, n: int):
        n = max(0, min(n, self.nframes - start))
        if n == 0:
            return []
        return list(hevc.decode(self._annexb, coded=False, first=start, count=n).frames)


# ----------------------------------------------------------------------------- AV1
class Av1Source:
    """Our own AV1 output (MP4 'av01' track or IVF) as a source: the header walk gives the
    geometry and frame count; ``read`` decodes a range with the decoder oracle from the
    preceding key frame (models/av1.py)."""
    kind = "av1"

    def __init__(self, path: str):
        from . import av1

        self.path = path
        with open(path, "rb") as f:
            head = f.read(4)
        self.fps_num, self.fps_den = 30, 1
        if head == b"DKIF":
            with open(path, "rb") as f:
                info, tus = av1.ivf_unwrap(f.read())
            self.fps_num, self.fps_den = info["fps"]
            self._tus = tus
            self.width, self.height, self.nframes = info["width"], info["height"], len(tus)
        else:
            with open(path, "rb") as f:
                tr = av1.mp4_av1_track(f.read())
            if tr is None:
                raise ValueError(f"{path}: no AV1 track")
            self._tus = None
            if tr["timescale"] and tr["delta"]:
                fr = Fraction(tr["timescale"], tr["delta"]).limit_denominator(1001)
                self.fps_num, self.fps_den = fr.numerator, fr.denominator
            self.width, self.height, self.nframes = tr["width"], tr["height"], len(tr["samples"])

    def read(self, start: int, n: int):
        from . import av1

        n = max(0, min(n, self.nframes - start))
        if n == 0:
            return []
        if self._tus is not None:
            k = start
            stream = b"".join(self._tus[:start + n])  # IVF: decode from the start (closed GOPs)
            k = 0
        else:
            with open(self.path, "rb") as f:
                data = f.read()
            tr, stream = av1.mp4_av1_stream(data, start, n)
            k = start
            while k > 0 and not tr["samples"][k][2]:
                k -= 1
        dec = av1.decode(stream)
        return [dec.planes(i) for i in range(start - k, start - k + n)]


def _is_av1_file(path: str) -> bool:
    try:
        with open(path, "rb") as f:
            head = f.read(1 << 16)
    except OSError:
        return False
    return head[:4] == b"DKIF" or (path.lower().endswith(".mp4") and b"av01" in head[:4096] + _moov_probe(path))


def _moov_probe(path: str) -> bytes:
    """The bytes of the moov box's sample description area (faststart files keep it first)."""
    try:
        with open(path, "rb") as f:
            data = f.read(1 << 20)
        i = data.find(b"stsd")
        return data[i:i + 64] if i >= 0 else b""
    except OSError:
        return b""


def open_source(path: str):
    ext = os.path.splitext(path)[1].lower()
    if ext == ".y4m":
        return Y4MSource(path)
    if ext == ".synth":
        return SynthSource(path)
    if ext == ".ivf" or (ext == ".mp4" and _is_av1_file(path)):
        return Av1Source(path)
    if ext in mpeg2.ES_EXTS or (ext == ".mkv" and mpeg2.is_mpeg2_mkv(path)):
        return mpeg2.Mpeg2Source(path)  # DVD titles (MakeMKV V_MPEG2) / raw MPEG-2 video
    if ext in (".hevc", ".265", ".mp4", ".mkv"):
        return HevcSource(path)
    raise ValueError(f"unsupported input format: {path}")


def probe(path: str) -> dict:
    """ffprobe-like summary used for the job hash `source_*` / `dest_*` fields."""
    src = open_source(path)
    size = os.path.getsize(path) if os.path.exists(path) else 0
    fps = src.fps_num / src.fps_den
    dur = src.nframes / fps if fps else 0.0
    codec = {"rawvideo": "rawvideo", "synthetic": "synthetic", "hevc": "hevc", "av1": "av1",
             "mpeg2": "mpeg2video"}[src.kind]
    return {
        "codec": codec,
        "width": src.width,
        "height": src.height,
        "resolution": f"{src.width}x{src.height}",
        "fps": round(fps, 3),
        "fps_num": src.fps_num,
        "fps_den": src.fps_den,
        "frames": src.nframes,
        "duration": round(dur, 3),
        "size": size,
        "bits": int(getattr(src, "bits", 8)),
        "field_order": getattr(src, "field_order", "progressive"),
        "bitrate_kbps": round(size * 8 / dur / 1000.0, 1) if dur else 0.0,
        "streams": _stream_list(path, codec, src),
    }


def _stream_list(path: str, codec: str, src) -> list[dict]:
    """ffprobe-like stream list: the video stream, then the source's audio / subtitle streams
    (container tracks and sidecar files, :func:`thinvids_amd.models.streams.source_streams`)."""
    from .streams import source_streams

    out = [{"index": 0, "codec_type": "video", "codec_name": codec, "width": src.width, "height": src.height}]
    try:
        side, desc = source_streams(path)
    except ValueError:
        return out
    for d in desc:
        if d.get("codec_type") in ("audio", "subtitle"):
            out.append({"index": len(out), **d})
    return out
