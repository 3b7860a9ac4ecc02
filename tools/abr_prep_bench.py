#!/usr/bin/env python3
"""Isolated timing of the ABR ladder's pre-processing (no encode running alongside):
synthetic HDR10 generation, PQ tone-map, and the rung resamples (fused 2-D vs two-pass,
cascaded vs direct), per 8K source frame.

    python tools/abr_prep_bench.py [--src 7680x4320] [--frames 16] [--iters 5]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--src", default="7680x4320")
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    import torch

    from thinvids_amd.models.abr import LADDER, AbrLadder

    sw, sh = (int(x) for x in a.src.split("x"))
    n = a.frames

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.iters):
            fn()
        torch.cuda.synchronize()
        return 1000 * (time.perf_counter() - t) / a.iters / n  # ms per source frame

    out = {"src": a.src, "frames_per_launch": n}
    for cascade in (True, False):
        for fused in (True, False):
            lad = AbrLadder(sw, sh, LADDER, segments=1, gop=n, cascade=cascade, fused=fused, slots=1)
            key = f"{'cascade' if cascade else 'direct'}_{'fused' if fused else 'twopass'}"
            if cascade and fused:
                out["synth_ms_per_frame"] = round(timed(lambda: lad.synth_p010(0, n)), 4)
                lad.synth_p010(0, n)
                out["tonemap_ms_per_frame"] = round(timed(lambda: lad.lib.tv_tonemap_pq_batch(
                    lad.y16.data_ptr(), lad.uv16.data_ptr(), sw, sh, n, lad.sdr.data_ptr(),
                    __import__("ctypes").c_float(1000.0), __import__("ctypes").c_float(100.0), lad._stream())), 4)
            lad.synth_p010(0, n)
            out[f"ladder_chunk_ms_per_frame_{key}"] = round(timed(lambda: lad.ladder_chunk(0, n)), 4)
            lad.close()
            del lad
            torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
