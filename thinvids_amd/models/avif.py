"""AVIF / AVIS containers for the AV1 encoder's temporal units, and an independent AV1
decoder for conformance checks.

* :func:`avif_still` wraps one key-frame temporal unit as an AVIF image item (HEIF
  ``meta``: ``hdlr pict``, ``pitm``, ``iloc``, ``iinf``/``infe av01``, ``iprp`` with
  ``ispe`` + ``av1C`` + ``pixi``, ``ipma``).
* :func:`avis_sequence` wraps a closed GOP as an AVIF image sequence (``avis`` brand,
  one ``pict`` track whose ``av01`` sample entry carries ``av1C``; every temporal unit
  is one sample, the key frame the only sync sample).
* :func:`dav1d_decode` decodes either through libavif's bundled dav1d (the AVIF plugin
  library that ships with Pillow; called through its public C API with ``ctypes``) and
  returns the decoder's Y/U/V planes exactly, without any YUV->RGB conversion.

dav1d is an independent, conformance-tested AV1 decoder, so ``dav1d_decode(stream) ==
golden recon`` pins the encoder's bitstream to the AV1 specification.
The reference never writes AV1 (it rejects AV1 sources, /root/reference/worker/tasks.py:
929-939, and encodes H.264 at :1573-1586); AVIF output is this framework's own addition.
"""
from __future__ import annotations

import ctypes as C
import glob
import os
import struct

import numpy as np

OBU_SEQUENCE_HEADER, OBU_TEMPORAL_DELIMITER = 1, 2


# ------------------------------------------------------------------ OBU helpers --------
def _leb128(data: bytes, i: int) -> tuple[int, int]:
    v = 0
    for k in range(8):
        b = data[i + k]
        v |= (b & 0x7F) << (7 * k)
        if not b & 0x80:
            return v, i + k + 1
    raise ValueError("bad leb128")


def obus(data: bytes):
    """(type, full OBU bytes) of a low-overhead-format OBU sequence (sizes present)."""
    i = 0
    while i < len(data):
        h = data[i]
        typ, ext, has_size = (h >> 3) & 15, (h >> 2) & 1, (h >> 1) & 1
        if not has_size:
            raise ValueError("OBU without obu_size")
        j = i + 1 + ext
        size, j = _leb128(data, j)
        yield typ, data[i:j + size]
        i = j + size


def strip_td(tu: bytes) -> bytes:
    return b"".join(o for t, o in obus(tu) if t != OBU_TEMPORAL_DELIMITER)


def sequence_header(tu: bytes) -> bytes:
    for t, o in obus(tu):
        if t == OBU_SEQUENCE_HEADER:
            return o
    raise ValueError("no sequence header OBU in the temporal unit")


def seq_frame_size(seq_obu: bytes) -> tuple[int, int]:
    """max_frame_width / height of a sequence header OBU (one operating point, no timing
    or decoder-model info: the encoder's headers)."""
    h = seq_obu[0]
    _, i = _leb128(seq_obu, 1 + ((h >> 2) & 1))
    bits = int.from_bytes(seq_obu[i:i + 16].ljust(16, b"\0"), "big")
    pos = [0]

    def u(n):
        pos[0] += n
        return (bits >> (128 - pos[0])) & ((1 << n) - 1)

    u(3), u(1)
    if u(1):  # reduced_still_picture_header
        raise ValueError("reduced still-picture headers are not written by this encoder")
    if u(1) or u(1):
        raise ValueError("timing / display-delay info not supported")
    if u(5) != 0:
        raise ValueError("one operating point expected")
    u(12)
    if u(5) > 7:
        u(1)
    wb, hb = u(4) + 1, u(4) + 1
    return u(wb) + 1, u(hb) + 1


def av1c(seq_obu: bytes) -> bytes:
    """AV1CodecConfigurationRecord for the encoder's sequence header (Main profile, 8-bit
    4:2:0, colocated-unknown chroma position; seq_level_idx 31 as written)."""
    b1 = (0 << 5) | 31      # seq_profile 0 | seq_level_idx_0
    b2 = (0 << 7) | (0 << 6) | (0 << 5) | (0 << 4) | (1 << 3) | (1 << 2) | 0  # tier, hbd, 12b, mono, ssx, ssy, csp
    return bytes([0x81, b1, b2, 0]) + seq_obu


# ------------------------------------------------------------------ ISO-BMFF ----------
def _box(typ: bytes, payload: bytes) -> bytes:
    return struct.pack(">I", 8 + len(payload)) + typ + payload


def _fbox(typ: bytes, version: int, flags: int, payload: bytes) -> bytes:
    return _box(typ, struct.pack(">I", (version << 24) | flags) + payload)


def _item_props(width: int, height: int, seq_obu: bytes) -> tuple[bytes, int]:
    """ipco and its property count.  ispe is the coded frame size: readers rescale a frame
    whose size differs from ispe (libavif does), so the display size lives only in the
    stream's render_size."""
    del width, height
    W, H = seq_frame_size(seq_obu)
    ispe = _fbox(b"ispe", 0, 0, struct.pack(">II", W, H))
    pixi = _fbox(b"pixi", 0, 0, bytes([3, 8, 8, 8]))
    return _box(b"ipco", ispe + _box(b"av1C", av1c(seq_obu)) + pixi), 3


def _meta(width: int, height: int, seq: bytes, off: int, size: int) -> bytes:
    """HEIF meta box of one av01 item whose data is `size` bytes at file offset `off`."""
    hdlr = _fbox(b"hdlr", 0, 0, b"\0\0\0\0pict" + b"\0" * 12 + b"\0")
    pitm = _fbox(b"pitm", 0, 0, struct.pack(">H", 1))
    infe = _fbox(b"infe", 2, 0, struct.pack(">HH", 1, 0) + b"av01" + b"\0")
    iinf = _fbox(b"iinf", 0, 0, struct.pack(">H", 1) + infe)
    ipco, nprop = _item_props(width, height, seq)
    ipma = _fbox(b"ipma", 0, 0, struct.pack(">IHB", 1, 1, nprop) + bytes([0x81, 0x82, 0x03, 0x84][:nprop]))
    iprp = _box(b"iprp", ipco + ipma)
    iloc = _fbox(b"iloc", 0, 0, bytes([0x44, 0x00]) + struct.pack(">HHHHII", 1, 1, 0, 1, off, size))
    return _fbox(b"meta", 0, 0, hdlr + pitm + iloc + iinf + iprp)


def avif_still(tu: bytes, width: int, height: int) -> bytes:
    """One key-frame temporal unit -> AVIF file bytes (the item holds the sequence header
    and frame OBUs; the temporal delimiter is dropped, as MIAF requires)."""
    item = strip_td(tu)
    seq = sequence_header(tu)
    ftyp = _box(b"ftyp", b"avif" + struct.pack(">I", 0) + b"avifmif1miaf")
    n = len(_meta(width, height, seq, 0, len(item)))
    meta = _meta(width, height, seq, len(ftyp) + n + 8, len(item))
    return ftyp + meta + _box(b"mdat", item)


def avis_sequence(tus: list, width: int, height: int, fps: int = 30) -> bytes:
    """Temporal units of one closed GOP (key frame first) -> AVIF image-sequence bytes."""
    samples = [strip_td(t) for t in tus]
    seq = sequence_header(tus[0])
    W, H = seq_frame_size(seq)
    n = len(samples)
    ftyp = _box(b"ftyp", b"avis" + struct.pack(">I", 0) + b"avisavifmsf1iso8mif1miaf")
    ts, dur = fps, 1
    mvhd = _fbox(b"mvhd", 0, 0, struct.pack(">IIII", 0, 0, ts, n * dur) + struct.pack(">IH", 0x00010000, 0x0100)
                 + b"\0" * 10 + struct.pack(">9I", 0x10000, 0, 0, 0, 0x10000, 0, 0, 0, 0x40000000) + b"\0" * 24
                 + struct.pack(">I", 2))
    tkhd = _fbox(b"tkhd", 0, 3, struct.pack(">IIIII", 0, 0, 1, 0, n * dur) + b"\0" * 8 + struct.pack(">hhhH", 0, 0, 0, 0)
                 + struct.pack(">9I", 0x10000, 0, 0, 0, 0x10000, 0, 0, 0, 0x40000000)
                 + struct.pack(">II", W << 16, H << 16))
    mdhd = _fbox(b"mdhd", 0, 0, struct.pack(">IIII", 0, 0, ts, n * dur) + struct.pack(">HH", 0x55C4, 0))
    hdlr = _fbox(b"hdlr", 0, 0, b"\0\0\0\0pict" + b"\0" * 12 + b"\0")
    vmhd = _fbox(b"vmhd", 0, 1, b"\0" * 8)
    dref = _fbox(b"dref", 0, 0, struct.pack(">I", 1) + _fbox(b"url ", 0, 1, b""))
    dinf = _box(b"dinf", dref)
    av01 = _box(b"av01", b"\0" * 6 + struct.pack(">H", 1) + b"\0" * 16 + struct.pack(">HH", W, H)
                + struct.pack(">II", 0x00480000, 0x00480000) + b"\0" * 4 + struct.pack(">H", 1) + b"\0" * 32
                + struct.pack(">Hh", 0x18, -1) + _box(b"av1C", av1c(seq)))
    stsd = _fbox(b"stsd", 0, 0, struct.pack(">I", 1) + av01)
    stts = _fbox(b"stts", 0, 0, struct.pack(">III", 1, n, dur))
    stsc = _fbox(b"stsc", 0, 0, struct.pack(">IIII", 1, 1, n, 1))
    stsz = _fbox(b"stsz", 0, 0, struct.pack(">II", 0, n) + b"".join(struct.pack(">I", len(s)) for s in samples))
    stss = _fbox(b"stss", 0, 0, struct.pack(">II", 1, 1))

    def build(off: int) -> bytes:
        stco = _fbox(b"stco", 0, 0, struct.pack(">II", 1, off))
        stbl = _box(b"stbl", stsd + stts + stsc + stsz + stco + stss)
        minf = _box(b"minf", vmhd + dinf + stbl)
        mdia = _box(b"mdia", mdhd + hdlr + minf)
        return _box(b"moov", mvhd + _box(b"trak", tkhd + mdia))

    # the first frame is also the primary image item (what still-image readers show)
    nm = len(_meta(width, height, seq, 0, len(samples[0])))
    data_off = len(ftyp) + nm + len(build(0)) + 8
    meta = _meta(width, height, seq, data_off, len(samples[0]))
    return ftyp + meta + build(data_off) + _box(b"mdat", b"".join(samples))


# ------------------------------------------------------------------ dav1d via libavif --
_LIB = None


def _libavif():
    global _LIB
    if _LIB is None:
        import PIL

        cands = sorted(glob.glob(os.path.join(os.path.dirname(os.path.dirname(PIL.__file__)), "pillow.libs",
                                              "libavif*.so*")))
        if not cands:
            raise RuntimeError("libavif (Pillow's AVIF plugin) not found")
        lib = C.CDLL(cands[0])
        vp = C.c_void_p
        lib.avifDecoderCreate.restype = vp
        lib.avifDecoderSetIOMemory.argtypes = [vp, vp, C.c_size_t]
        lib.avifDecoderParse.argtypes = [vp]
        lib.avifDecoderNextImage.argtypes = [vp]
        lib.avifDecoderDestroy.argtypes = [vp]
        for f in ("avifImagePlaneRowBytes", "avifImagePlaneWidth", "avifImagePlaneHeight"):
            getattr(lib, f).argtypes = [vp, C.c_int]
            getattr(lib, f).restype = C.c_uint32
        lib.avifImagePlane.argtypes = [vp, C.c_int]
        lib.avifImagePlane.restype = vp
        lib.avifResultToString.restype = C.c_char_p
        _LIB = lib
    return _LIB


def dav1d_available() -> bool:
    try:
        _libavif()
        from PIL import _avif

        return _avif.decoder_codec_available("dav1d")
    except Exception:
        return False


# avifDecoder field offsets (libavif 1.x avif.h: 11 leading 32-bit settings, strictFlags
# the 11th, then the `image` pointer)
_STRICT_FLAGS_IDX, _IMAGE_PTR_OFF = 10, 48


def dav1d_decode(data: bytes) -> list:
    """Decode an AVIF / AVIS file with libavif's dav1d; returns [(Y, U, V)] uint8 planes
    per frame at the decoded frame size (libavif applies no clean-aperture crop; it does
    rescale to an ``ispe`` that differs from the frame size, which this module's writers
    never produce)."""
    lib = _libavif()
    d = lib.avifDecoderCreate()
    if not d:
        raise RuntimeError("avifDecoderCreate failed")
    buf = C.create_string_buffer(bytes(data), len(data))
    try:
        (C.c_uint32 * 12).from_address(d)[_STRICT_FLAGS_IDX] = 0
        r = lib.avifDecoderSetIOMemory(d, buf, len(data))
        if r == 0:
            r = lib.avifDecoderParse(d)
        if r != 0:
            raise RuntimeError(f"libavif parse: {lib.avifResultToString(r).decode()}")
        frames = []
        while True:
            r = lib.avifDecoderNextImage(d)
            if r == 16:  # AVIF_RESULT_NO_IMAGES_REMAINING
                break
            if r != 0:
                raise RuntimeError(f"libavif/dav1d decode frame {len(frames)}: {lib.avifResultToString(r).decode()}")
            img = C.c_void_p.from_address(d + _IMAGE_PTR_OFF).value
            planes = []
            for c in range(3):
                w, h = lib.avifImagePlaneWidth(img, c), lib.avifImagePlaneHeight(img, c)
                rb = lib.avifImagePlaneRowBytes(img, c)
                a = np.frombuffer(C.string_at(lib.avifImagePlane(img, c), rb * h), np.uint8).reshape(h, rb)
                planes.append(a[:, :w].copy())
            frames.append(tuple(planes))
        return frames
    finally:
        lib.avifDecoderDestroy(d)
