"""AV1 codec "model" API (BASELINE config #4): golden encoder, decoder
oracle, IVF container, and the temporal-unit writer the GPU engine's entropy stage uses.

Coding-tool subset and the tables substituted for the ones the AV1 specification defines
but this offline image does not hold (default CDFs, q-index lookup, transform rounding):
``csrc/include/tv/av1_enc.h``.  The stream syntax is AV1's (OBUs, uncompressed header,
partition / mode / MV / coefficient symbols with the spec's context derivations) and the
decoder oracle here parses it back bit-exactly; decoding by libaom / dav1d is parity
unpinned (neither exists in the image).

Reference parity: thinvids rejects AV1 sources (/root/reference/worker/tasks.py:929-939)
and only emits H.264 (:1532-1586); this is the north-star AV1 path of BASELINE.json.
"""
from __future__ import annotations

import ctypes as C
import struct
from dataclasses import dataclass

import numpy as np

from .._native import Bytes, core_lib, ptr, u8p

i16p = C.POINTER(C.c_int16)
u32p = C.POINTER(C.c_uint32)
i32p = C.POINTER(C.c_int32)
i64p = C.POINTER(C.c_int64)
i8p = C.POINTER(C.c_int8)
vp = C.c_void_p

# mirrored from av1_enc.h
INTRA_CANDS = (0, 1, 2, 9, 10, 11, 12)


def coded_size(width: int, height: int) -> tuple[int, int]:
    return (width + 15) & ~15, (height + 15) & ~15


def _lib():
    lib = core_lib()
    if not getattr(lib, "_av1c_sigs", False):
        i = C.c_int
        lib.tv_av1c_last_error.restype = C.c_char_p
        lib.tv_av1c_golden_encode.argtypes = [i, i, i, u8p, i, i32p, vp, i64p, u8p, u32p, u32p, i16p, i16p, i16p, i32p,
                                                i8p, i32p]
        lib.tv_av1c_golden_encode.restype = i
        lib.tv_av1c_decode.argtypes = [u8p, C.c_size_t, i, u8p, i32p, i32p]
        lib.tv_av1c_decode.restype = i
        lib.tv_av1c_write_tu.argtypes = [vp, i, i, i32p, u32p, u32p, i16p, i16p, i16p, i8p, i32p, i, i, vp]
        lib.tv_av1c_state_new.restype = vp
        lib.tv_av1c_state_free.argtypes = [vp]
        lib.tv_av1c_write_tu.restype = i
        lib._av1c_sigs = True
    return lib


def _check(rc: int):
    if rc != 0:
        raise RuntimeError(_lib().tv_av1c_last_error().decode())


def ac_q(q: int) -> int:
    """Substitute AC quantiser step (av1_enc.h ac_q), for rate-control mapping."""
    q = min(max(q, 0), 255)
    if q == 0:
        return 4
    if q <= 96:
        return q + 7
    e = (q - 96) * 1711
    ip, fp = e >> 16, e & 65535
    two_f = 65536 + ((fp * (43025 + ((22511 * fp) >> 16))) >> 16)
    return min(1828, ((103 * two_f << ip) + 32768) >> 16)


_QP_TO_QINDEX: dict = {}


def qindex_for_hevc_qp(qp: int) -> int:
    """The q-index whose AC step matches HEVC QP `qp`'s (x8 transform scale): qstep =
    2^((qp-4)/6) in orthonormal units."""
    qp = int(qp)
    if qp not in _QP_TO_QINDEX:
        target = 8.0 * 2.0 ** ((qp - 4) / 6.0)
        _QP_TO_QINDEX[qp] = int(min(range(1, 256), key=lambda q: abs(ac_q(q) - target)))
    return _QP_TO_QINDEX[qp]


@dataclass
class GoldenResult:
    stream: bytes
    tu_sizes: list
    recon: np.ndarray  # (n, W*H*3/2) uint8, coded size
    mode: np.ndarray   # (n, nblk) uint32
    mv: np.ndarray
    ly: np.ndarray     # (n, nblk, 256) int16
    lu: np.ndarray
    lv: np.ndarray
    fparams: np.ndarray  # (n, 25) int32 (frame_params layout)
    cdef_idx: np.ndarray  # (n, nsb) int8
    lr: np.ndarray  # (n, 3, nu, 3) int32: per plane / 64x64 unit (sgr set | -1, xqd0, xqd1)


def pack_i420(frames, W: int, H: int) -> np.ndarray:
    """[(Y, U, V)] of coded size -> (n, W*H*3/2) uint8."""
    out = np.empty((len(frames), W * H * 3 // 2), np.uint8)
    for k, (y, u, v) in enumerate(frames):
        out[k, :W * H] = y.reshape(-1)
        out[k, W * H:W * H * 5 // 4] = u.reshape(-1)
        out[k, W * H * 5 // 4:] = v.reshape(-1)
    return out


def pad_frame(frame, W: int, H: int):
    """Edge-replicate a display-size (Y, U, V) to the coded size."""
    y, u, v = frame
    h, w = y.shape
    return (np.pad(y, ((0, H - h), (0, W - w)), mode="edge"),
            np.pad(u, ((0, H // 2 - h // 2), (0, W // 2 - w // 2)), mode="edge"),
            np.pad(v, ((0, H // 2 - h // 2), (0, W // 2 - w // 2)), mode="edge"))


def golden_encode(frames, width: int, height: int, qindex: int, qmap=None) -> GoldenResult:
    """C++ golden encoder over display-size (Y, U, V) frames (one closed GOP); `qmap`
    (optional): per-frame q-index of a rate-control plan."""
    W, H = coded_size(width, height)
    n = len(frames)
    yuv = pack_i420([pad_frame(f, W, H) for f in frames], W, H)
    nb = (W // 16) * (H // 16)
    out = Bytes()
    sizes = np.zeros(n, np.int64)
    recon = np.empty_like(yuv)
    mode = np.zeros((n, nb), np.uint32)
    mv = np.zeros((n, nb), np.uint32)
    ly = np.zeros((n, nb, 256), np.int16)
    lu = np.zeros((n, nb, 64), np.int16)
    lv = np.zeros((n, nb, 64), np.int16)
    fparams = np.zeros((n, 25), np.int32)
    cdef = np.zeros((n, ((W + 63) // 64) * ((H + 63) // 64)), np.int8)
    lr = np.zeros((n, 3, lr_units(W, H), 3), np.int32)
    qm = None if qmap is None else np.ascontiguousarray(np.asarray(qmap, np.int32).reshape(n))
    _check(_lib().tv_av1c_golden_encode(width, height, n, ptr(yuv), qindex,
                                        None if qm is None else qm.ctypes.data_as(i32p), out.h,
                                        sizes.ctypes.data_as(i64p),
                                        ptr(recon), mode.ctypes.data_as(u32p), mv.ctypes.data_as(u32p),
                                        ly.ctypes.data_as(i16p), lu.ctypes.data_as(i16p), lv.ctypes.data_as(i16p),
                                        fparams.ctypes.data_as(i32p), cdef.ctypes.data_as(i8p),
                                        lr.ctypes.data_as(i32p)))
    return GoldenResult(out.tobytes(), sizes.tolist(), recon, mode, mv, ly, lu, lv, fparams, cdef, lr)


def lr_units(W: int, H: int) -> int:
    """64x64 restoration units of the luma plane (ceil layout; the lr array's unit stride)."""
    return ((W + 63) // 64) * ((H + 63) // 64)


@dataclass
class Av1Decoded:
    width: int
    height: int
    W: int
    H: int
    frames: np.ndarray  # (n, W*H*3/2) coded size

    def planes(self, k: int, display: bool = True):
        W, H = self.W, self.H
        f = self.frames[k]
        y = f[:W * H].reshape(H, W)
        u = f[W * H:W * H * 5 // 4].reshape(H // 2, W // 2)
        v = f[W * H * 5 // 4:].reshape(H // 2, W // 2)
        if display:
            return y[:self.height, :self.width], u[:self.height // 2, :self.width // 2], v[:self.height // 2,
                                                                                             :self.width // 2]
        return y, u, v


def probe(stream: bytes) -> dict:
    geo = np.zeros(4, np.int32)
    n = C.c_int32(0)
    buf = np.frombuffer(stream, np.uint8)
    _check(_lib().tv_av1c_decode(ptr(buf), len(buf), 0, None, geo.ctypes.data_as(i32p), C.byref(n)))
    return {"width": int(geo[0]), "height": int(geo[1]), "coded": (int(geo[2]), int(geo[3])), "frames": n.value}


def decode(stream: bytes) -> Av1Decoded:
    """Decoder oracle: parse + reconstruct every frame of a stream of temporal units."""
    info = probe(stream)
    W, H = info["coded"]
    frames = np.empty((info["frames"], W * H * 3 // 2), np.uint8)
    geo = np.zeros(4, np.int32)
    n = C.c_int32(0)
    buf = np.frombuffer(stream, np.uint8)
    _check(_lib().tv_av1c_decode(ptr(buf), len(buf), info["frames"], ptr(frames), geo.ctypes.data_as(i32p),
                                 C.byref(n)))
    return Av1Decoded(info["width"], info["height"], W, H, frames)


# cdef / frame parameter vector of tv_av1c_write_tu
def frame_params(key: bool, qindex: int, lf, sharp: int, damping: int, cdef_y, cdef_uv, cdef_bits: int = 3):
    p = np.zeros(25, np.int32)
    p[0], p[1] = int(key), qindex
    p[2:6] = lf
    p[6], p[7], p[8] = sharp, damping, cdef_bits
    p[9:17] = cdef_y
    p[17:25] = cdef_uv
    return p


def zigzag_scan(N: int) -> np.ndarray:
    """Raster position of each scan index (av1_enc.h zigzag_scan)."""
    out = []
    for s in range(2 * N - 1):
        lo, hi = max(0, s - N + 1), min(s, N - 1)
        rows = range(lo, hi + 1) if s & 1 else range(hi, lo - 1, -1)
        out.extend(r * N + (s - r) for r in rows)
    return np.asarray(out, np.int64)


def scan_pack(lev: np.ndarray, mode: np.ndarray, plane: int) -> np.ndarray:
    """Host model of the GPU engine's device->host level layout (k_av1e_tb_pack): each TB
    with the plane's nonzero bit as [eob, eob levels in zigzag order], back to back."""
    n = lev.shape[-1]
    sc = zigzag_scan(16 if n == 256 else 8)
    parts = []
    for b in np.nonzero((mode >> (10 + plane)) & 1)[0]:
        z = lev[b][sc]
        eob = int(np.nonzero(z)[0][-1]) + 1
        parts.append(np.concatenate([[eob], z[:eob]]).astype(np.int16))
    return np.concatenate(parts) if parts else np.zeros(1, np.int16)


class StreamWriter:
    """Writes one stream's temporal units in order from engine decisions; carries the
    frame-to-frame CDF state (frame-end CDF update, primary_ref_frame of inter frames)."""

    def __init__(self, width: int, height: int):
        self.w, self.h = width, height
        self.lib = _lib()
        self.st = self.lib.tv_av1c_state_new()

    def __del__(self):
        if getattr(self, "st", None):
            self.lib.tv_av1c_state_free(self.st)
            self.st = None

    def write(self, fparams: np.ndarray, mode: np.ndarray, mv: np.ndarray, ly: np.ndarray, lu: np.ndarray,
              lv: np.ndarray, cdef_idx: np.ndarray, packed: int, seq_header: bool, lr: np.ndarray | None = None,
              out: Bytes | None = None) -> bytes | None:
        """packed: 0 = full [nblk][N*N] levels, 1 = nonzero TBs back to back, 2 = scan_pack."""
        o = out if out is not None else Bytes()
        _check(self.lib.tv_av1c_write_tu(self.st, self.w, self.h, fparams.ctypes.data_as(i32p),
                                         mode.ctypes.data_as(u32p), mv.ctypes.data_as(u32p),
                                         ly.ctypes.data_as(i16p), lu.ctypes.data_as(i16p), lv.ctypes.data_as(i16p),
                                         cdef_idx.ctypes.data_as(i8p),
                                         None if lr is None else np.ascontiguousarray(lr, np.int32).ctypes.data_as(i32p),
                                         int(packed), int(seq_header), o.h))
        return None if out is not None else o.tobytes()


# ------------------------------------------------------------------------------- IVF ----
def ivf_header(width: int, height: int, fps_num: int, fps_den: int, nframes: int) -> bytes:
    return struct.pack("<4sHH4sHHIIII", b"DKIF", 0, 32, b"AV01", width, height, fps_num, fps_den, nframes, 0)


def ivf_wrap(tus, width: int, height: int, fps_num: int = 30, fps_den: int = 1) -> bytes:
    """Temporal units -> an IVF file (the AV1 elementary-stream container of aomenc)."""
    out = [ivf_header(width, height, fps_num, fps_den, len(tus))]
    for k, tu in enumerate(tus):
        out.append(struct.pack("<IQ", len(tu), k))
        out.append(tu)
    return b"".join(out)


def ivf_unwrap(data: bytes) -> tuple[dict, list]:
    if data[:4] != b"DKIF":
        raise ValueError("not an IVF file")
    _, _, hlen, fourcc, w, h, num, den, n, _ = struct.unpack("<4sHH4sHHIIII", data[:32])
    pos, tus = hlen, []
    while pos + 12 <= len(data):
        sz, _pts = struct.unpack("<IQ", data[pos:pos + 12])
        tus.append(data[pos + 12:pos + 12 + sz])
        pos += 12 + sz
    return {"fourcc": fourcc.decode(), "width": w, "height": h, "fps": (num, den)}, tus


def split_temporal_units(stream: bytes, sizes) -> list:
    out, pos = [], 0
    for s in sizes:
        out.append(stream[pos:pos + s])
        pos += s
    return out


# ------------------------------------------------------------------------------- MP4 ----
TD_OBU = b"\x12\x00"  # temporal delimiter OBU (stripped from ISO-BMFF samples)


def _boxes(data: bytes, start: int, end: int):
    pos = start
    while pos + 8 <= end:
        size, typ = struct.unpack(">I4s", data[pos:pos + 8])
        hdr = 8
        if size == 1:
            size = struct.unpack(">Q", data[pos + 8:pos + 16])[0]
            hdr = 16
        elif size == 0:
            size = end - pos
        if size < hdr:
            raise ValueError("mp4: bad box size")
        yield typ.decode("latin-1"), pos + hdr, pos + size
        pos += size


def mp4_av1_track(data: bytes) -> dict | None:
    """The 'av01' video track of an MP4 (our muxer's output): geometry, timing and the
    sample (offset, size, sync) table; None when the file has no AV1 track."""
    def find(path, start, end):
        for t, a, b in _boxes(data, start, end):
            if t == path[0]:
                return (a, b) if len(path) == 1 else find(path[1:], a, b)
        return None

    moov = find(["moov"], 0, len(data))
    if not moov:
        return None
    for t, a, b in _boxes(data, *moov):
        if t != "trak":
            continue
        stbl = find(["mdia", "minf", "stbl"], a, b)
        mdhd = find(["mdia", "mdhd"], a, b)
        if not stbl or not mdhd:
            continue
        boxes = {t2: (a2, b2) for t2, a2, b2 in _boxes(data, *stbl)}
        sa, sb = boxes["stsd"]
        entry = data[sa + 8:sa + 16]
        if entry[4:8] != b"av01":
            continue
        ea = sa + 8
        width, height = struct.unpack(">HH", data[ea + 8 + 24:ea + 8 + 28])
        ver = data[mdhd[0]]
        timescale = struct.unpack(">I", data[mdhd[0] + (20 if ver == 1 else 12):][:4])[0]
        a2 = boxes["stts"][0]
        delta = struct.unpack(">I", data[a2 + 12:a2 + 16])[0] if struct.unpack(">I", data[a2 + 4:a2 + 8])[0] else 0
        a2 = boxes["stsz"][0]
        fixed, count = struct.unpack(">II", data[a2 + 4:a2 + 12])
        sizes = [fixed] * count if fixed else list(struct.unpack(f">{count}I", data[a2 + 12:a2 + 12 + 4 * count]))
        if "stco" in boxes:
            a2 = boxes["stco"][0]
            n = struct.unpack(">I", data[a2 + 4:a2 + 8])[0]
            chunk_off = struct.unpack(f">{n}I", data[a2 + 8:a2 + 8 + 4 * n])
        else:
            a2 = boxes["co64"][0]
            n = struct.unpack(">I", data[a2 + 4:a2 + 8])[0]
            chunk_off = struct.unpack(f">{n}Q", data[a2 + 8:a2 + 8 + 8 * n])
        a2 = boxes["stsc"][0]
        n = struct.unpack(">I", data[a2 + 4:a2 + 8])[0]
        stsc = [struct.unpack(">III", data[a2 + 8 + 12 * i:a2 + 20 + 12 * i]) for i in range(n)]
        offsets, k = [], 0
        for ci, co in enumerate(chunk_off):
            spc = next(e[1] for e in reversed(stsc) if e[0] <= ci + 1)
            o = co
            for _ in range(spc):
                if k >= count:
                    break
                offsets.append(o)
                o += sizes[k]
                k += 1
        sync = set(range(1, count + 1))
        if "stss" in boxes:
            a2 = boxes["stss"][0]
            n = struct.unpack(">I", data[a2 + 4:a2 + 8])[0]
            sync = set(struct.unpack(f">{n}I", data[a2 + 8:a2 + 8 + 4 * n]))
        return {"width": width, "height": height, "timescale": timescale, "delta": delta,
                "samples": [(o, z, (i + 1) in sync) for i, (o, z) in enumerate(zip(offsets, sizes))]}
    return None


def mp4_av1_stream(data: bytes, first: int = 0, count: int = -1) -> tuple[dict, bytes]:
    """Temporal units [first, first + count) of an AV1 MP4 back as a decodable OBU stream
    (temporal delimiters restored), starting from the preceding key frame."""
    tr = mp4_av1_track(data)
    if tr is None:
        raise ValueError("mp4: no AV1 track")
    smp = tr["samples"]
    end = len(smp) if count < 0 else min(len(smp), first + count)
    k = first
    while k > 0 and not smp[k][2]:
        k -= 1
    return tr, b"".join(TD_OBU + data[o:o + z] for o, z, _ in smp[k:end])
