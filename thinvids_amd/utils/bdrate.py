"""Bjontegaard delta rate (BD-rate) between two rate-distortion curves.

The "fixed PSNR" part of the headline metric (BASELINE.json) is judged as a rate difference
at equal quality: fit log10(rate) as a cubic in PSNR for each curve, integrate both over the
overlapping PSNR interval and report the average rate change in percent (negative = the test
curve needs fewer bits for the same PSNR).  Used by ``tools/rd_curve.py`` and the compression
tool tests.
"""
from __future__ import annotations

import numpy as np


def bd_rate(rate_a, psnr_a, rate_b, psnr_b) -> float:
    """Average % rate change of curve b against anchor a over their common PSNR range."""
    ra, pa = np.log10(np.asarray(rate_a, np.float64)), np.asarray(psnr_a, np.float64)
    rb, pb = np.log10(np.asarray(rate_b, np.float64)), np.asarray(psnr_b, np.float64)
    if len(ra) < 2 or len(rb) < 2:
        raise ValueError("need at least two rate points per curve")
    deg = min(3, len(ra) - 1, len(rb) - 1)
    fa, fb = np.polyfit(pa, ra, deg), np.polyfit(pb, rb, deg)
    lo, hi = max(pa.min(), pb.min()), min(pa.max(), pb.max())
    if hi <= lo:
        raise ValueError("curves do not overlap in PSNR")
    ia, ib = np.polyint(fa), np.polyint(fb)
    avg_a = (np.polyval(ia, hi) - np.polyval(ia, lo)) / (hi - lo)
    avg_b = (np.polyval(ib, hi) - np.polyval(ib, lo)) / (hi - lo)
    return float((10.0 ** (avg_b - avg_a) - 1.0) * 100.0)


def rate_at_psnr(rates, psnrs, target: float) -> float:
    """Rate of a curve interpolated (log-rate, piecewise linear in PSNR) at `target` dB."""
    p = np.asarray(psnrs, np.float64)
    r = np.log10(np.asarray(rates, np.float64))
    o = np.argsort(p)
    return float(10.0 ** np.interp(target, p[o], r[o]))
