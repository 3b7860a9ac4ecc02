#!/usr/bin/env python3
"""Throughput of the AV1 in-loop filter kernels (CDEF direction + strength search + filter,
Wiener / self-guided restoration search + apply) on batches of synthetic frames.

    python tools/av1_tools_bench.py [--res 4k] [--batch 8] [--iters 5] [--lr]

Reconstructions are synthetic frames with added quantisation-like noise (seeded), so the
searches see realistic statistics.  Prints one JSON line with frames/s per stage.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

RES = {"1080p": (1920, 1088), "4k": (3840, 2160), "720p": (1280, 720)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--res", default="4k", choices=sorted(RES))
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--lr", action="store_true", help="also time the loop-restoration search")
    a = ap.parse_args()
    import numpy as np
    import torch

    from thinvids_amd.models import hevc
    from thinvids_amd.ops import av1

    dev = torch.device("cuda", 0)
    w, h = RES[a.res]
    g = torch.Generator(device="cpu").manual_seed(1)
    planes = []
    for c, (pw, ph) in enumerate(((w, h), (w // 2, h // 2), (w // 2, h // 2))):
        base = np.stack([hevc.synth_frame(4, t, w, h)[c] for t in range(a.batch)])
        src = torch.from_numpy(base).to(dev)
        noise = (torch.randn((a.batch, ph, pw), generator=g) * 3).round().to(torch.int16).to(dev)
        rec = (src.to(torch.int16) + noise).clamp(0, 255).to(torch.uint8)
        planes.append((src, rec))
    (Ys, Yr), (Us, Ur), (Vs, Vr) = planes

    def cdef_step():
        d, v = av1.cdef_dirs(Yr)
        sy = av1.cdef_search(Ys, Yr, d, v, False)
        su = av1.cdef_search(Us, Ur, d, v, True)
        sv = av1.cdef_search(Vs, Vr, d, v, True)
        nfb = sy.shape[1]
        pr = torch.full((a.batch, nfb), 38, dtype=torch.int8)
        return [av1.cdef_apply(Yr, d, v, pr, False), av1.cdef_apply(Ur, d, v, pr, True),
                av1.cdef_apply(Vr, d, v, pr, True)], (sy, su, sv)

    def timed(fn, n):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n

    res = {"res": f"{w}x{h}", "batch": a.batch}
    t = timed(cdef_step, a.iters)
    res["cdef_search_apply_ms_per_batch"] = round(1000 * t, 3)
    res["cdef_fps"] = round(a.batch / t, 1)
    nu = av1.n_units(w, h)
    coef = np.tile(np.array([3, -7, 15, -2, 5, 20], np.int32), (a.batch, nu, 1))
    t = timed(lambda: av1.wiener_apply(Yr, coef), a.iters)
    res["wiener_apply_luma_fps"] = round(a.batch / t, 1)
    t = timed(lambda: av1.wiener_stats(Ys, Yr, 0, np.zeros((a.batch, nu, 3), np.int32)), a.iters)
    res["wiener_stats_luma_fps"] = round(a.batch / t, 1)
    prm = np.tile(np.array([0, -20, 40], np.int32), (a.batch, nu, 1))
    t = timed(lambda: av1.sgr_apply(Yr, prm), a.iters)
    res["sgr_apply_luma_fps"] = round(a.batch / t, 1)
    rng = np.random.default_rng(0)
    lf = [np.stack([av1.random_lf_info(pw, ph, rng, chroma=c > 0, lvl_max=40) for _ in range(a.batch)])
          for c, (pw, ph) in enumerate(((w, h), (w // 2, h // 2), (w // 2, h // 2)))]
    lf = [torch.as_tensor(x.view(np.int32)).to(dev) for x in lf]
    t = timed(lambda: [av1.deblock(r, i, c > 0) for c, (r, i) in enumerate(zip((Yr, Ur, Vr), lf))], a.iters)
    res["deblock_yuv_fps"] = round(a.batch / t, 1)
    res["deblock_yuv_gbps"] = round(a.batch * w * h * 1.5 * 2 / t / 1e9, 1)
    if a.lr:
        t = timed(lambda: av1.loop_restoration_search(Ys, Yr, sgr_sets=(0, 10, 14)), max(1, a.iters // 2))
        res["lr_search_luma_fps"] = round(a.batch / t, 1)
    out, (sy, su, sv) = cdef_step()
    res["psnr_y_in"] = round(av1.psnr(Ys, Yr), 3)
    res["psnr_y_cdef38"] = round(av1.psnr(Ys, out[0]), 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
