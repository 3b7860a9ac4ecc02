"""HEVC codec "model" API: synthetic source, CPU reference encoder, decoder oracle,
MP4 mux/demux — thin numpy wrappers over ``libtvcore.so``.

Frames are ``(Y, U, V)`` tuples of uint8 numpy arrays (4:2:0, Y shape ``(H, W)``).
"""
from __future__ import annotations

import ctypes as C
import threading
from dataclasses import dataclass

import numpy as np

from .._native import u8p, Bytes, check, core_lib, i16p, ptr

Frame = tuple  # (Y, U, V)


def coded_size(width: int, height: int, ctb: int = 32) -> tuple[int, int]:
    return (width + ctb - 1) // ctb * ctb, (height + ctb - 1) // ctb * ctb


def synth_frame(seed: int, t: int, width: int, height: int) -> Frame:
    """Deterministic synthetic frame (same bytes as the GPU generator kernel)."""
    y = np.empty((height, width), np.uint8)
    u = np.empty((height // 2, width // 2), np.uint8)
    v = np.empty_like(u)
    core_lib().tv_synth_frame(seed & 0xFFFFFFFF, t, width, height, ptr(y), ptr(u), ptr(v))
    return y, u, v


def psnr(a: np.ndarray, b: np.ndarray) -> float:
    mse = np.mean((a.astype(np.float64) - b.astype(np.float64)) ** 2)
    return float("inf") if mse == 0 else 10.0 * np.log10(255.0 ** 2 / mse)


def psnr_yuv(ref: Frame, dec: Frame) -> dict:
    py, pu, pv = (psnr(r, d) for r, d in zip(ref, dec))
    return {"y": py, "u": pu, "v": pv, "yuv": (6 * py + pu + pv) / 8}


def codec_flags(deblock: bool = True, sao: bool = False, wpp: bool = True, rqt: bool = True, pintra: bool = True,
                cascade: bool = False, rdoq: bool = True) -> int:
    """The native APIs' configuration bits (tv::SeqConfig::set_flags): 1 deblocking, 2 SAO,
    4 WPP substreams, 8 no residual quadtree, 16 no intra CUs in P pictures, 64 the constant-QP
    I P P P QP cascade (tv/gop.h ippp_qp_offset), 128 no RDOQ-lite coefficient-group trimming
    (tv/hevc_defs.h kRdoqMode)."""
    return (int(bool(deblock)) | (2 if sao else 0) | (4 if wpp else 0) | (0 if rqt else 8) | (0 if pintra else 16)
            | (64 if cascade else 0) | (0 if rdoq else 128))


IPPP_CASCADE_IDR = -5
IPPP_CASCADE_P = (1, 0, 1, -1, 1, 0, 1, -3)


def ippp_cascade_qps(qp: int, nframes: int) -> list[int]:
    """Per-frame slice QPs of one constant-QP I P P P GOP under the cascade (mirror of tv/gop.h
    ippp_qp_offset): what the engines code when no explicit map is given."""
    return [max(0, min(51, qp + (IPPP_CASCADE_IDR if i == 0 else IPPP_CASCADE_P[(i - 1) % 8]))) for i in range(nframes)]


class CpuEncoder:
    """Scalar C++ HEVC encoder (software path; reference `software_encode`)."""

    def __init__(self, width: int, height: int, qp: int = 27, deblock: bool = True,
                 search_range: int = 64, max_merge: int = 5, sao: bool = False, crf: int = 0, wpp: bool = True,
                 bframes: int = 1, rqt: bool = True, pintra: bool = True, cascade: bool = True, rdoq: bool = True):
        """`wpp`: one CABAC substream per CTB row (entropy_coding_sync; the GPU engine's
        default, it codes them on the device); `rqt` / `pintra` / `rdoq`: residual quadtree for
        inter CUs, intra 16x16 CUs in P pictures, trailing lone-level coefficient groups of inter
        TBs dropped (coding tools; part of the bitstream identity)."""
        if width % 2 or height % 2:
            raise ValueError("width/height must be even")
        self.lib = core_lib()
        self.width, self.height, self.qp = width, height, qp
        self.cw, self.ch = coded_size(width, height)
        self.bframes = int(bframes)
        if self.bframes > 1:
            if crf:
                raise ValueError("CRF with B frames is not supported by the golden encoder")
            f = self.lib.tv_cpu_encoder_new_b
            f.restype = C.c_void_p
            f.argtypes = [C.c_int] * 7
            self.h = f(width, height, qp, codec_flags(deblock, sao, wpp, rqt, pintra, cascade, rdoq), search_range, max_merge,
                       self.bframes)
        elif crf:
            f = self.lib.tv_cpu_encoder_new_crf
            f.restype = C.c_void_p
            f.argtypes = [C.c_int] * 7
            self.h = f(width, height, qp, codec_flags(deblock, sao, wpp, rqt, pintra, cascade, rdoq), search_range, max_merge,
                       int(crf))
        else:
            self.h = self.lib.tv_cpu_encoder_new(width, height, qp, codec_flags(deblock, sao, wpp, rqt, pintra, cascade, rdoq),
                                                 search_range, max_merge)
        if not self.h:
            raise ValueError(self.lib.tv_last_error().decode())
        self.out = Bytes()

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.tv_cpu_encoder_free(self.h)
            self.h = None

    def begin_gop(self, nframes: int) -> list[int]:
        """Hierarchical-B mode: plan the next segment; returns the display index of every
        picture in coding order (feed the frames to :meth:`encode` in that order)."""
        disp = (C.c_int * nframes)()
        f = self.lib.tv_cpu_encoder_begin_gop
        f.restype = C.c_int
        f.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int)]
        check(f(self.h, nframes, disp))
        return list(disp)

    def encode(self, frame: Frame, idr: bool, poc: int, qp: int | None = None) -> bytes:
        """One frame; `qp` overrides the slice QP of this frame (rate control)."""
        y, u, v = (np.ascontiguousarray(p) for p in frame)
        self.out.clear()
        if qp is None:
            check(self.lib.tv_cpu_encoder_encode(self.h, ptr(y), ptr(u), ptr(v), y.shape[1], u.shape[1],
                                                 int(idr), poc, self.out.h))
        else:
            f = self.lib.tv_cpu_encoder_encode_qp
            f.restype = C.c_int
            f.argtypes = [C.c_void_p, u8p, u8p, u8p] + [C.c_int] * 5 + [C.c_void_p]
            check(f(self.h, ptr(y), ptr(u), ptr(v), y.shape[1], u.shape[1], int(idr), poc, int(qp), self.out.h))
        return self.out.tobytes()

    def recon(self) -> Frame:
        y = np.empty((self.ch, self.cw), np.uint8)
        u = np.empty((self.ch // 2, self.cw // 2), np.uint8)
        v = np.empty_like(u)
        self.lib.tv_cpu_encoder_recon(self.h, ptr(y), ptr(u), ptr(v))
        return y, u, v

    def decisions(self) -> dict:
        w8, h8 = self.cw // 8, self.ch // 8
        d = {k: np.empty((h8, w8), np.uint8) for k in ("cu_log2", "intra", "ipm", "cbf")}
        mv = np.empty((h8, w8, 2), np.int16)
        self.lib.tv_cpu_encoder_decisions(self.h, ptr(d["cu_log2"]), ptr(d["intra"]), ptr(d["ipm"]),
                                          ptr(mv, i16p), ptr(d["cbf"]))
        d["mv"] = mv
        return d


def gop_plan(nframes: int, bframes: int) -> dict:
    """Coding structure of one segment (tv/gop.h): per coded picture the display index,
    slice type (2 I / 1 P / 0 B), references and temporal layer, plus DPB size / reorder."""
    lib = core_lib()
    arrs = [(C.c_int * max(1, nframes))() for _ in range(5)]
    info = (C.c_int * 2)()
    f = lib.tv_gop_plan
    f.restype = C.c_int
    f.argtypes = [C.c_int, C.c_int] + [C.POINTER(C.c_int)] * 6
    n = f(nframes, bframes, *arrs, info)
    keys = ("disp", "type", "ref0", "ref1", "layer")
    out = {k: list(a)[:n] for k, a in zip(keys, arrs)}
    out["dpb_size"], out["num_reorder"] = info[0], info[1]
    return out


def encode_sequence_cpu(frames, qp: int = 27, gop: int = 0, frame_qps=None, bframes: int = 1,
                        **kw) -> tuple[bytes, list]:
    """Encode frames (first is IDR; IDR every `gop` frames if gop>0). Returns (annexb, recons)
    with the reconstructions in display order.  `frame_qps`: optional per-frame slice QP
    (display order; with B frames the base to which the layer offset is added); `qp` stays
    the PPS init QP.  `bframes` > 1: hierarchical-B mini-GOPs of that size (tv/gop.h)."""
    frames = list(frames)
    h, w = frames[0][0].shape
    if bframes > 1:
        enc = CpuEncoder(w, h, qp=qp, bframes=bframes, **kw)
        seg = gop if gop > 0 else len(frames)
        out, recons = bytearray(), [None] * len(frames)
        for s0 in range(0, len(frames), seg):
            n = min(seg, len(frames) - s0)
            for d in enc.begin_gop(n):
                i = s0 + d
                out += enc.encode(frames[i], d == 0, d, None if frame_qps is None else int(frame_qps[i]))
                recons[i] = enc.recon()
        return bytes(out), recons
    enc = CpuEncoder(w, h, qp=qp, **kw)
    out, recons, poc = bytearray(), [], 0
    for i, f in enumerate(frames):
        idr = i == 0 or (gop > 0 and i % gop == 0)
        poc = 0 if idr else poc + 1
        out += enc.encode(f, idr, poc, None if frame_qps is None else int(frame_qps[i]))
        recons.append(enc.recon())
    return bytes(out), recons


def display_offsets(annexb: bytes) -> np.ndarray:
    """Per picture in decoding order: display index - decoding index (all zero for I P P P;
    hierarchical-B streams are reordered), from the slice headers only."""
    lib = core_lib()
    buf = np.frombuffer(annexb, np.uint8)
    cap = max(1, annexb.count(b"\x00\x00\x01"))
    out = np.zeros(cap, np.int32)
    f = lib.tv_hevc_display_offsets
    f.restype = C.c_int
    f.argtypes = [C.POINTER(C.c_uint8), C.c_size_t, C.POINTER(C.c_int), C.c_int]
    n = f(buf.ctypes.data_as(C.POINTER(C.c_uint8)), len(buf), out.ctypes.data_as(C.POINTER(C.c_int)), cap)
    if n < 0:
        raise ValueError(lib.tv_last_error().decode())
    return out[:n]


@dataclass
class DecodedStream:
    width: int
    height: int
    coded_w: int
    coded_h: int
    frames: list  # cropped (Y, U, V)
    coded_frames: list  # coded-size (Y, U, V)


def probe_annexb(annexb: bytes) -> dict:
    """Header-only probe (SPS geometry, picture and IDR counts): nothing is decoded."""
    lib = core_lib()
    if not getattr(lib, "_probe_sig", False):
        lib.tv_hevc_probe.argtypes = [C.POINTER(C.c_uint8), C.c_size_t] + [C.POINTER(C.c_int)] * 4
        lib.tv_hevc_probe.restype = C.c_int
        lib.tv_decoder_decode_range.argtypes = [C.c_void_p, C.POINTER(C.c_uint8), C.c_size_t, C.c_int, C.c_int]
        lib.tv_decoder_decode_range.restype = C.c_int
        lib._probe_sig = True
    buf = np.frombuffer(annexb, np.uint8)
    w, h, n, k = (C.c_int() for _ in range(4))
    check(lib.tv_hevc_probe(ptr(buf), len(annexb), C.byref(w), C.byref(h), C.byref(n), C.byref(k)))
    return {"width": w.value, "height": h.value, "frames": n.value, "idrs": k.value}


def decode(annexb: bytes, coded: bool = True, first: int = 0, count: int = -1) -> DecodedStream:
    """Decode an Annex-B HEVC stream with the native decoder oracle; `first`/`count` decode
    only that picture range (from the nearest preceding IDR)."""
    lib = core_lib()
    probe_annexb(b"")  # signatures
    h = lib.tv_decoder_new()
    try:
        buf = np.frombuffer(annexb, np.uint8)
        check(lib.tv_decoder_decode_range(h, ptr(buf), len(annexb), int(first), int(count)))
        w, hh, cw, ch, n = (C.c_int() for _ in range(5))
        lib.tv_decoder_info(h, C.byref(w), C.byref(hh), C.byref(cw), C.byref(ch), C.byref(n))
        frames, coded_frames = [], []
        for i in range(n.value):
            for crop, sink, (W, H) in ((1, frames, (w.value, hh.value)),
                                       (0, coded_frames, (cw.value, ch.value))):
                if crop == 0 and not coded:
                    continue
                y = np.empty((H, W), np.uint8)
                u = np.empty((H // 2, W // 2), np.uint8)
                v = np.empty_like(u)
                check(lib.tv_decoder_frame(h, i, crop, ptr(y), ptr(u), ptr(v)))
                sink.append((y, u, v))
        return DecodedStream(w.value, hh.value, cw.value, ch.value, frames, coded_frames)
    finally:
        lib.tv_decoder_free(h)


def write_frame(width: int, height: int, qp: int, idr: bool, poc: int, dec: dict,
                coef: tuple, deblock: bool = True, max_merge: int = 5) -> bytes:
    """Entropy-code one frame from decision arrays (cu_log2/intra/ipm/mv/cbf + coef planes)."""
    lib = core_lib()
    out = Bytes()
    cy, cu, cv = (np.ascontiguousarray(c, dtype=np.int16) for c in coef)
    check(lib.tv_write_frame(width, height, qp, int(deblock), max_merge, int(idr), poc,
                             ptr(np.ascontiguousarray(dec["cu_log2"])), ptr(np.ascontiguousarray(dec["intra"])),
                             ptr(np.ascontiguousarray(dec["ipm"])),
                             ptr(np.ascontiguousarray(dec["mv"], dtype=np.int16), i16p),
                             ptr(np.ascontiguousarray(dec["cbf"])), ptr(cy, i16p), ptr(cu, i16p),
                             ptr(cv, i16p), out.h))
    return out.tobytes()


def reconstruct_reference(width: int, height: int, qp: int, src: Frame, ref: Frame | None,
                          dec: dict, deblock: bool = True):
    """Golden-model pass B: decisions -> (cbf, coef planes, recon) on the CPU."""
    lib = core_lib()
    cw, ch = coded_size(width, height)
    cbf = np.zeros((ch // 8, cw // 8), np.uint8)
    cy = np.zeros((ch, cw), np.int16)
    cu = np.zeros((ch // 2, cw // 2), np.int16)
    cv = np.zeros_like(cu)
    ry = np.zeros((ch, cw), np.uint8)
    ru = np.zeros((ch // 2, cw // 2), np.uint8)
    rv = np.zeros_like(ru)
    s = [np.ascontiguousarray(p) for p in src]
    r = [np.ascontiguousarray(p) for p in ref] if ref is not None else None
    null = C.cast(None, C.POINTER(C.c_uint8))
    check(lib.tv_reconstruct_frame(
        width, height, qp, int(deblock), ptr(s[0]), ptr(s[1]), ptr(s[2]),
        ptr(r[0]) if r else null, ptr(r[1]) if r else null, ptr(r[2]) if r else null,
        ptr(np.ascontiguousarray(dec["cu_log2"])), ptr(np.ascontiguousarray(dec["intra"])),
        ptr(np.ascontiguousarray(dec["ipm"])), ptr(np.ascontiguousarray(dec["mv"], dtype=np.int16), i16p),
        ptr(cbf), ptr(cy, i16p), ptr(cu, i16p), ptr(cv, i16p), ptr(ry), ptr(ru), ptr(rv)))
    return cbf, (cy, cu, cv), (ry, ru, rv)


def mux_mp4(annexb: bytes, width: int, height: int, fps_num: int = 30, fps_den: int = 1) -> bytes:
    lib = core_lib()
    out = Bytes()
    buf = np.frombuffer(annexb, np.uint8).copy()
    check(lib.tv_mux_mp4(ptr(buf), len(annexb), width, height, fps_num, fps_den, out.h))
    return out.tobytes()


def mux_mp4_file(segments, width: int, height: int, fps_num: int, fps_den: int, path: str) -> int:
    """Write the concatenation of Annex-B segments as a faststart MP4 at `path`, streaming
    the payload from the segment buffers (no joined copy).  Returns the file size."""
    lib = core_lib()
    if not getattr(lib, "_muxf_sig", False):
        lib.tv_mux_mp4_file.argtypes = [C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.c_int, C.c_int, C.c_int,
                                        C.c_int, C.c_int, C.c_char_p, C.POINTER(C.c_ulonglong)]
        lib.tv_mux_mp4_file.restype = C.c_int
        lib._muxf_sig = True
    segs = [s for s in segments if len(s)]
    keep = [np.frombuffer(s, np.uint8) for s in segs]
    ptrs = (C.c_void_p * len(keep))(*[k.ctypes.data for k in keep])
    sizes = (C.c_size_t * len(keep))(*[len(k) for k in keep])
    out = C.c_ulonglong()
    check(lib.tv_mux_mp4_file(ptrs, sizes, len(keep), width, height, fps_num, fps_den, path.encode(), C.byref(out)))
    return int(out.value)


class Mp4StreamWriter:
    """Streaming faststart MP4 of one video track (csrc/core/mp4.cpp Mp4Stream): Annex-B (or
    AV1 OBU) segments are appended as they are encoded and written straight to `path`; the
    head (ftyp + moov + free padding) is reserved for `max_samples` frames and filled in by
    close(), so the finished file is faststart without re-copying the payload.  Segments
    must share one set of parameter sets (one encoder configuration per job)."""

    def __init__(self, path: str, width: int, height: int, fps_num: int, fps_den: int, max_samples: int):
        lib = core_lib()
        if not getattr(lib, "_mp4s_sig", False):
            lib.tv_mp4s_open.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_ulonglong]
            lib.tv_mp4s_open.restype = C.c_void_p
            lib.tv_mp4s_append.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
            lib.tv_mp4s_append.restype = C.c_int
            lib.tv_mp4s_close.argtypes = [C.c_void_p, C.POINTER(C.c_ulonglong)]
            lib.tv_mp4s_close.restype = C.c_int
            lib.tv_mp4s_abort.argtypes = [C.c_void_p]
            lib.tv_mp4s_last_error.restype = C.c_char_p
            lib._mp4s_sig = True
        self.lib, self.path = lib, path
        self.h = lib.tv_mp4s_open(path.encode(), width, height, fps_num, fps_den, max(1, int(max_samples)))
        if not self.h:
            raise RuntimeError(lib.tv_mp4s_last_error().decode())
        self.payload = 0
        # the native calls release the GIL: append / close / abort from different threads
        # must never overlap on one handle (abort deletes it)
        self.lock = threading.Lock()

    def append(self, segment) -> None:
        buf = np.frombuffer(segment, np.uint8)
        if not len(buf):
            return
        with self.lock:
            if not self.h:
                raise RuntimeError("stream writer closed")
            if self.lib.tv_mp4s_append(self.h, buf.ctypes.data, len(buf)) != 0:
                raise RuntimeError(self.lib.tv_mp4s_last_error().decode())
        self.payload += len(buf)

    def close(self) -> int:
        """Finish the file; returns its size."""
        with self.lock:
            h, self.h = self.h, None
            if not h:
                raise RuntimeError("stream writer closed")
            out = C.c_ulonglong()
            if self.lib.tv_mp4s_close(h, C.byref(out)) != 0:
                raise RuntimeError(self.lib.tv_mp4s_last_error().decode())
        return int(out.value)

    def abort(self) -> None:
        with self.lock:
            if self.h:
                self.lib.tv_mp4s_abort(self.h)
                self.h = None

    def __del__(self):
        self.abort()


def demux_mp4(data: bytes) -> dict:
    lib = core_lib()
    out = Bytes()
    buf = np.frombuffer(data, np.uint8).copy()
    w, h, n, ts, d = (C.c_int() for _ in range(5))
    check(lib.tv_demux_mp4(ptr(buf), len(data), C.byref(w), C.byref(h), C.byref(n), C.byref(ts),
                           C.byref(d), out.h))
    return {"annexb": out.tobytes(), "width": w.value, "height": h.value, "frames": n.value,
            "timescale": ts.value, "sample_delta": d.value,
            "fps": ts.value / d.value if d.value else 0.0}
