"""Rate control (BASELINE config #4 "2-pass RC all-reduce").

The reference only ever runs constant QP (`-rc_mode CQP -qp 27`, reference
worker/tasks.py:66-67, :1573-1586) or libx264 CRF 23 (:1558-1571).  Here:

* ``cqp``   — one QP everywhere (parity with the reference's hardware path);
* ``crf``   — per-frame QP from the engine's own lookahead: the quarter-resolution coarse
  motion search cost of a frame (or its quarter-res intra activity for an IDR) sets
  QP = crf + 2.4 * log2(complexity / reference) (x264's qcomp = 0.6 curve), I frames -3;
  the same integer formula runs on the GPU and in the CPU golden model;
* ``2pass`` — frame-level two-pass: pass 1 encodes at the base QP and yields every frame's
  bits; the per-frame statistics of all ranks are all-reduced (RCCL), a global allocation
  (bits^qcomp complexity compression) becomes a per-frame QP plan, and pass 2 encodes it
  with rank-local rate feedback between batches (each completed batch corrects the QP
  offset of the segments a rank still has to encode);
* ``abr``   — single pass at a target bitrate (no pass 1, so it streams the stitch): every
  rank plans each claimed batch at one uniform QP offset from its own finished batches
  (AbrController, the offset regression of BatchRateController), optionally under a VBV:
  the decoder-buffer model is checked per segment and a violating segment is re-encoded
  coarser (vbv_scale / vbv_repair_offset).

VBV decomposition.  Segments are closed GOPs encoded on different ranks in any order, so a
global leaky-bucket simulation would serialise the node.  Instead every segment must, starting
from the buffer at ``init`` x bufsize, never underflow and end at least that full again; then
any concatenation of segments is compliant (each one hands the next a buffer at least as full
as the one it assumed), and the check is local to the rank that encoded the segment.

The bits(QP) model is bits = b1 * 2^(-(QP - QP1) / SLOPE) with SLOPE QP steps per halving
(measured on this encoder: 5.9 - 7.5 between QP 17 and 42).
"""
from __future__ import annotations

import math

import numpy as np

SLOPE = 6.5  # QP steps per halving of the bits
QCOMP = 0.6
# Hierarchical-B streams keep their layer QP cascade (tv/gop.h) under 2-pass: bits follow
# complexity 1:1, i.e. one uniform QP shift for the whole plan.  The I P P P qcomp (0.6) moves
# bits from the anchors to the cheap B pictures, which then predict from starved anchors
# (measured: 1500 kbps hit within -3.6 % but at 38.5 dB instead of ~43 dB).
QCOMP_BFRAMES = 1.0


def log2_q8(x: int) -> int:
    """floor(256 * log2(x)) by repeated squaring — the integer form tv/rc_model.h uses on
    both the CPU and the GPU (so CRF decisions are bit-identical)."""
    x = max(1, int(x))
    e = x.bit_length() - 1
    y = x << (31 - e) if e <= 31 else x >> (e - 31)
    r = e << 8
    for b in range(7, -1, -1):
        y = (y * y) >> 31
        if y >= 1 << 32:
            r |= 1 << b
            y >>= 1
    return r


def obu_frame_sizes(stream: bytes) -> list[int]:
    """Bytes per temporal unit of an AV1 low-overhead OBU stream (one shown frame per
    temporal unit here; the temporal delimiter and sequence header count toward it)."""
    out: list[int] = []
    pos, n, cur = 0, len(stream), -1
    while pos < n:
        start = pos
        h = stream[pos]
        pos += 1 + ((h >> 2) & 1)
        size, shift = 0, 0
        while True:
            b = stream[pos]
            pos += 1
            size |= (b & 0x7F) << shift
            shift += 7
            if not b & 0x80:
                break
        pos += size
        if (h >> 3) & 15 == 2:  # temporal delimiter: a new unit
            out.append(0)
            cur = len(out) - 1
        if cur >= 0:
            out[cur] += pos - start
    return out


def frame_sizes(annexb: bytes, decode_order: bool = False) -> list[int]:
    """Bytes per coded picture of an Annex-B stream in DISPLAY order (parameter sets count
    toward the next picture in decoding order, start codes included; hierarchical-B streams
    are mapped back by their POCs, so the list lines up with a display-order QP map); AV1
    OBU streams (leading temporal delimiter) are split per temporal unit.  `decode_order`:
    the pictures as they enter the decoder (VBV buffer model)."""
    if annexb[:2] == b"\x12\x00":
        return obu_frame_sizes(annexb)
    out: list[int] = []
    pending = 0
    i, n = 0, len(annexb)
    starts = []
    while True:
        j = annexb.find(b"\x00\x00\x01", i)
        if j < 0:
            break
        s = j - 1 if j > 0 and annexb[j - 1] == 0 else j
        starts.append((s, j + 3))
        i = j + 3
    for k, (s, h) in enumerate(starts):
        e = starts[k + 1][0] if k + 1 < len(starts) else n
        size = e - s
        t = (annexb[h] >> 1) & 0x3F if h < n else 63
        if t <= 31:  # a slice: one picture per slice here
            out.append(pending + size)
            pending = 0
        else:
            pending += size
    from .hevc import display_offsets

    if decode_order:
        return out
    off = display_offsets(annexb)
    if len(off) == len(out) and off.any():
        disp = [0] * len(out)
        for i, o in enumerate(off):
            disp[i + int(o)] = out[i]
        return disp
    return out


def predict_bits(b1: np.ndarray, q1, q, slope: float = SLOPE) -> np.ndarray:
    return np.asarray(b1, np.float64) * np.power(2.0, -(np.asarray(q, np.float64) - np.asarray(q1, np.float64)) / slope)


def plan_frame_qps(bits1: list, q1: int, target_bits: float, qcomp: float = QCOMP, qp_min: int = 10,
                   qp_max: int = 51, key_offset: float | None = None, slope: float = SLOPE) -> tuple[list, float]:
    """Per-frame real-valued QPs for pass 2.  bits1: per segment, the pass-1 bits of every
    frame (encoded at q1).  Frame f gets a share t_f proportional to b_f^qcomp (compressed
    complexity, as x264's qcomp), scaled so sum(t) == target_bits; its QP is the one the
    model says yields t_f.  `key_offset` (AV1 path): the first frame of every segment (its
    key frame) is instead pinned `key_offset` QP from its segment's mean inter-frame QP —
    the inter frames predict from it, so starving it costs more bits than it saves (the
    frame-independent bits model misses that) — and one uniform shift of every QP, found
    by bisection, restores the target.  `slope`: QP steps per halving of the bits (a fitted
    value from BatchRateController, else SLOPE).  Returns (per-segment QP arrays, predicted
    total)."""
    flat = np.concatenate([np.maximum(np.asarray(b, np.float64), 1.0) for b in bits1])
    w = flat ** qcomp
    t = target_bits * w / w.sum()
    q = np.clip(q1 + slope * np.log2(flat / t), qp_min, qp_max)
    if key_offset is not None:
        k, keys = 0, []
        for b in bits1:
            if len(b) > 1:
                q[k] = float(np.mean(q[k + 1:k + len(b)])) + key_offset
            keys.append(k)
            k += len(b)
        lo, hi = -30.0, 30.0
        for _ in range(50):  # predicted bits fall monotonically with a uniform shift
            mid = (lo + hi) / 2
            if predict_bits(flat, q1, np.clip(q + mid, qp_min, qp_max), slope).sum() > target_bits:
                lo = mid
            else:
                hi = mid
        q = np.clip(q + (lo + hi) / 2, qp_min, qp_max)
    out, k = [], 0
    for b in bits1:
        out.append(q[k:k + len(b)])
        k += len(b)
    return out, float(predict_bits(flat, q1, q, slope).sum())


def round_qps(qf: np.ndarray, offset: float = 0.0, qp_min: int = 10, qp_max: int = 51) -> np.ndarray:
    """Integer QPs from real-valued ones with error diffusion along the segment (the
    rounding error of one frame is carried into the next, so a segment's mean QP — and its
    bits — follow the real-valued plan)."""
    out = np.empty(len(qf), np.int64)
    carry = 0.0
    for i, v in enumerate(np.asarray(qf, np.float64) + offset):
        r = int(np.clip(math.floor(v + carry + 0.5), qp_min, qp_max))
        carry += v - r
        out[i] = r
    return out


# AV1 (this repo's q-index map, qindex_for_hevc_qp): measured 4.4-5.6 QP per halving of the
# bits around the 4K 20 Mbps operating point (profiles/README.md, round 4)
AV1_SLOPE = 5.0


class BatchRateController:
    """Batch-sequential 2-pass feedback (the bench's steps, a worker's claims).  Each batch
    is planned from its own pass-1 statistics (plan_frame_qps: the relative per-frame
    allocation) plus one uniform QP offset u chosen here from the finished batches: the
    miss r = log2(actual / wanted) of every finished batch is regressed on its offset
    (r = a + b u, the local bits(QP) response -- measured, since the log-linear model's slope
    is neither codec- nor operating-point-independent: 5 to 10 QP per halving on this repo's
    AV1 between q-index 60 and 100), and the next offset is the root -u = a / b- (a Newton
    step with the SLOPE prior while every finished batch shares one offset).  A quarter of
    the accumulated overshoot / undershoot is repaid by the next batch, at most 4 % of its
    share.  Deterministic in the (all-reduced) inputs, so every rank plans the same."""

    def __init__(self, repay: float = 0.25, max_repay: float = 0.04, window: int = 4, max_offset: float = 12.0,
                 slope: float | None = None):
        self.target = self.actual = 0.0
        self.repay, self.max_repay, self.window, self.max_offset = repay, max_repay, window, max_offset
        # QP per halving of the bits until two operating points measure it (codec-dependent:
        # AV1_SLOPE for the AV1 q-index map)
        self.slope = SLOPE if slope is None else float(slope)
        self.pts: list = []  # (offset u, log2(actual / wanted)) per finished batch
        self.log: list = []  # per finished batch: actual / nominal, wanted / nominal, offset

    def offset(self) -> float:
        pts = self.pts[-self.window:]
        if not pts:
            return 0.0
        u = np.array([p[0] for p in pts])
        r = np.array([p[1] for p in pts])
        b = -1.0 / self.slope
        if np.ptp(u) > 0.25:  # two operating points: the measured response
            bu = float(np.polyfit(u, r, 1)[0])
            b = float(np.clip(bu, -1.0 / 3.5, -1.0 / 16.0))
        # the root of the line through the centroid with slope b
        u_next = float(u.mean() - r.mean() / b)
        return float(np.clip(u_next, -self.max_offset, self.max_offset))

    def request(self, nominal: float) -> tuple[float, float, float]:
        """(bits to ask the planner for, bits this batch should produce, QP offset to add)."""
        lim = self.max_repay * nominal
        want = nominal + float(np.clip(self.repay * (self.target - self.actual), -lim, lim))
        return want, want, self.offset()

    def record(self, nominal: float, wanted: float, offset: float, actual: float) -> None:
        self.target += nominal
        self.actual += actual
        self.pts.append((float(offset), math.log2(max(actual, 1.0) / max(wanted, 1.0))))
        self.log.append([round(actual / nominal, 4), round(wanted / nominal, 4), round(offset, 3)])


class RateFeedback:
    """Rank-local pass-2 correction: the log-ratio of actual to planned bits over the
    segments encoded so far becomes a QP offset for the segments still to come."""

    def __init__(self, gain: float = 1.0, limit: float = 6.0):
        self.actual = 0.0
        self.planned = 0.0
        self.gain, self.limit = gain, limit

    def offset(self) -> float:
        if self.actual <= 0 or self.planned <= 0:
            return 0.0
        return float(np.clip(self.gain * SLOPE * math.log2(self.actual / self.planned), -self.limit, self.limit))

    def record(self, actual_bits: float, planned_bits: float) -> None:
        self.actual += actual_bits
        self.planned += planned_bits


def vbv_levels(bits, fps: float, maxrate_bps: float, bufsize_bits: float, init: float = 0.9) -> tuple[float, float]:
    """Decoder-buffer (leaky bucket) levels of one segment: the buffer starts at init x
    bufsize, frame f's bits leave it at its removal time, and it refills at maxrate per frame
    interval up to bufsize.  Returns (lowest level right after a removal, level at the end of
    the segment's last interval); the segment is compliant iff the first is >= 0 and the
    second >= the starting level (see the module docstring)."""
    fill = maxrate_bps / fps
    level = init * bufsize_bits
    low = level
    for b in bits:
        level -= float(b)
        low = min(low, level)
        level = min(bufsize_bits, level + fill)
    return low, level


def vbv_ok(bits, fps: float, maxrate_bps: float, bufsize_bits: float, init: float = 0.9) -> bool:
    low, end = vbv_levels(bits, fps, maxrate_bps, bufsize_bits, init)
    return low >= 0.0 and end >= init * bufsize_bits - 1e-6


def vbv_scale(bits, fps: float, maxrate_bps: float, bufsize_bits: float, init: float = 0.9) -> float:
    """Largest uniform factor s <= 1 such that s x bits is compliant (bisection; the levels
    fall monotonically in s)."""
    b = np.asarray(bits, np.float64)
    if vbv_ok(b, fps, maxrate_bps, bufsize_bits, init):
        return 1.0
    lo, hi = 0.0, 1.0
    for _ in range(40):
        mid = (lo + hi) / 2
        if vbv_ok(b * mid, fps, maxrate_bps, bufsize_bits, init):
            lo = mid
        else:
            hi = mid
    return lo


def vbv_repair_offset(scale: float, attempt: int, slope: float = SLOPE) -> int:
    """QP increase for a re-encode that must shrink a segment by `scale`: the model's
    -slope*log2(scale), plus one step per previous failed attempt (the I frame at the head of
    the segment responds less than the model)."""
    return max(1, int(math.ceil(-slope * math.log2(max(scale, 1e-6)))) + attempt)


class AbrController:
    """Single-pass average-bitrate control of one rank's batches on one rung.  A batch of
    segments is encoded at base QP + u.  The finished batches' misses r = log2(actual /
    nominal) are regressed on their offsets (r = a + b u over the last `window` batches; slope
    b measured once two operating points differ, else the SLOPE prior, clipped to 3.5..16 QP
    per halving) and the next u puts the line at log2(want / nominal), where want repays 25 %
    of the accumulated miss (at most 10 % of the batch).  Rank-local: every rank meets the
    target on its own segments, so the node meets it with no collective per batch."""

    def __init__(self, base_qp: float, qp_min: int = 10, qp_max: int = 51, max_offset: float = 16.0,
                 window: int = 4, repay: float = 0.25, max_repay: float = 0.10):
        self.base = float(base_qp)
        self.qp_min, self.qp_max, self.max_offset = qp_min, qp_max, max_offset
        self.window, self.repay, self.max_repay = window, repay, max_repay
        self.target = self.actual = 0.0
        self.pts: list = []  # (u, log2(actual / nominal)) per finished batch
        self.log: list = []  # per finished batch: actual / nominal, want / nominal, u
        self.pending: tuple | None = None

    def offset(self, want_ratio: float = 1.0) -> float:
        pts = self.pts[-self.window:]
        if not pts:
            return 0.0
        u = np.array([p[0] for p in pts])
        r = np.array([p[1] for p in pts])
        b = -1.0 / SLOPE
        if np.ptp(u) > 0.25:
            b = float(np.clip(np.polyfit(u, r, 1)[0], -1.0 / 3.5, -1.0 / 16.0))
        u_next = u.mean() + (math.log2(max(want_ratio, 1e-6)) - r.mean()) / b
        return float(np.clip(u_next, -self.max_offset, self.max_offset))

    def plan(self, nominal_bits: float, frames: list) -> list:
        """Per-segment integer QP arrays (lengths `frames`) for a batch worth nominal_bits;
        the fractional QP is error-diffused along each segment."""
        lim = self.max_repay * nominal_bits
        want = nominal_bits + float(np.clip(self.repay * (self.target - self.actual), -lim, lim))
        u = self.offset(want / max(nominal_bits, 1.0))
        q = float(np.clip(self.base + u, self.qp_min, self.qp_max))
        self.pending = (nominal_bits, want, q - self.base)
        return [round_qps(np.full(n, q), 0.0, self.qp_min, self.qp_max) for n in frames]

    def record(self, actual_bits: float) -> None:
        if self.pending is None:
            return
        nominal, want, u = self.pending
        self.pending = None
        self.target += nominal
        self.actual += actual_bits
        self.pts.append((u, math.log2(max(actual_bits, 1.0) / max(nominal, 1.0))))
        self.log.append([round(actual_bits / nominal, 4), round(want / nominal, 4), round(u, 3)])
