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
  offset of the segments a rank still has to encode).

The bits(QP) model is bits = b1 * 2^(-(QP - QP1) / SLOPE) with SLOPE QP steps per halving
(measured on this encoder: 5.9 - 7.5 between QP 17 and 42).
"""
from __future__ import annotations

import math

import numpy as np

SLOPE = 6.5  # QP steps per halving of the bits
QCOMP = 0.6


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


def frame_sizes(annexb: bytes) -> list[int]:
    """Bytes per coded picture of an Annex-B stream (parameter sets count toward the next
    picture, start codes included); AV1 OBU streams (leading temporal delimiter) are split
    per temporal unit."""
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

    def __init__(self, repay: float = 0.25, max_repay: float = 0.04, window: int = 4, max_offset: float = 12.0):
        self.target = self.actual = 0.0
        self.repay, self.max_repay, self.window, self.max_offset = repay, max_repay, window, max_offset
        self.pts: list = []  # (offset u, log2(actual / wanted)) per finished batch
        self.log: list = []  # per finished batch: actual / nominal, wanted / nominal, offset

    def offset(self) -> float:
        pts = self.pts[-self.window:]
        if not pts:
            return 0.0
        u = np.array([p[0] for p in pts])
        r = np.array([p[1] for p in pts])
        b = -1.0 / SLOPE
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
