"""Scene-cut detection: an IDR (closed-GOP restart) at every abrupt content change.

A P-frame across a cut has no useful reference, and the P-frame engine codes inter CUs
only, so it would spend bits on a full-frame residual and still lose quality.  The
reference never faces this: its segmenter cuts at the source's keyframes (`ffmpeg -f segment`,
reference worker/tasks.py:1163-1213), which encoders place at scene changes, and x264 inserts
scenecut IDRs itself.  Here the encoder restarts the closed GOP at each detected cut: a
part's chunk plan (:func:`thinvids_amd.worker.encoder.chunk_plan`) gets a boundary there, so
the cut frame is coded as an IDR by the same batched engine (chunks of any length batch
together), on the GPU and the CPU paths alike.

Detector: luma thumbnails (8x8 mean pool) of consecutive frames; frame t is a cut when the
mean absolute thumbnail difference d(t) exceeds both an absolute floor and `ratio` times the
recent typical motion (median of the previous differences), and the last boundary is at
least `min_gap` frames back.  Thumbnails are computed on the device for staged frames (one
pooled tensor, a few KB back to the host) and with numpy for host frames.
"""
from __future__ import annotations

import numpy as np

FLOOR = 12.0   # mean |delta| of 8x8-pooled luma (8-bit levels) below which nothing is a cut
RATIO = 3.0    # ... and it must exceed RATIO x the recent median difference
MIN_GAP = 4    # frames between boundaries
HISTORY = 8


def thumbs_host(frames) -> np.ndarray:
    """(n, h/8, w/8) float32 8x8-pooled luma of host (Y, U, V) frames (10-bit scaled to 8)."""
    out = []
    for f in frames:
        y = np.asarray(f[0])
        h, w = (y.shape[0] // 8) * 8, (y.shape[1] // 8) * 8
        t = y[:h, :w].astype(np.float32).reshape(h // 8, 8, w // 8, 8).mean(axis=(1, 3))
        out.append(t / 4.0 if y.dtype == np.uint16 else t)
    return np.stack(out) if out else np.zeros((0, 1, 1), np.float32)


def diffs_device(dev_frames) -> np.ndarray:
    """d(t) for t = 1..n-1 of a :class:`~thinvids_amd.ops.stage.DevFrames`, computed on its
    device: the 8x8 thumbnails come from one HIP kernel straight from the samples
    (csrc/gpu/k_stage.hip k_thumbs8; a float copy of every luma plane + avg_pool2d cost ~5 %
    of a y4m job's GPU time), only n - 1 floats come back."""
    import torch

    from ..ops import stage

    off, w, h, stride, fs = dev_frames.planes[0]
    n = dev_frames.n
    if n < 2:
        return np.zeros(0, np.float32)
    tw, th = w // 8, h // 8
    t = torch.empty((n, th, tw), dtype=torch.float32, device=dev_frames.buf.device)
    stage.thumbs8(dev_frames.ptr(0), dev_frames.bits, w, h, stride, fs, n, t)
    return (t[1:] - t[:-1]).abs().mean(dim=(1, 2)).cpu().numpy()


def diffs_host(frames) -> np.ndarray:
    t = thumbs_host(frames)
    return np.abs(t[1:] - t[:-1]).mean(axis=(1, 2)) if len(t) > 1 else np.zeros(0, np.float32)


def detect(d: np.ndarray, floor: float = FLOOR, ratio: float = RATIO, min_gap: int = MIN_GAP) -> list[int]:
    """Cut frames (indices t >= 1 into the part) from consecutive-frame differences d[t-1]."""
    cuts, hist, last = [], [], 0
    for t in range(1, len(d) + 1):
        v = float(d[t - 1])
        base = float(np.median(hist)) if hist else 0.0
        if v > floor and v > ratio * base + 1.0 and t - last >= min_gap:
            cuts.append(t)
            last = t
            hist = []  # the new scene's motion sets the new baseline
            continue
        hist = (hist + [v])[-HISTORY:]
    return cuts


def part_cuts(part) -> list[int]:
    """Cuts of an encoder part: host frames, device frames, or a synthetic range (none)."""
    if hasattr(part, "select"):
        return detect(diffs_device(part))
    if isinstance(part, (list, tuple)) and part and isinstance(part[0], (list, tuple)):
        return detect(diffs_host(part))
    return []
