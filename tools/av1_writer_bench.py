"""CPU cost of the AV1 OBU writer (the engine's entropy stage) per frame.

    python tools/av1_writer_bench.py --res 3840x2160 --frames 3 --reps 5

Golden-encodes a short GOP of the bench content (q-index matched to QP 27), then times
``StreamWriter.write`` (tv_av1c_write_tu, the engine's scan-packed level layout) on each
frame's decisions, single-threaded, and prints ms per key / inter frame.
"""
from __future__ import annotations

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np

    from thinvids_amd.models import av1, hevc

    ap = argparse.ArgumentParser()
    ap.add_argument("--res", default="1920x1080")
    ap.add_argument("--frames", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--dump", default="", help="write the decisions for tools/native/bench_av1w.cpp")
    a = ap.parse_args()
    w, h = map(int, a.res.split("x"))
    q = av1.qindex_for_hevc_qp(27)
    frames = [hevc.synth_frame(a.seed, t, w, h) for t in range(a.frames)]
    t0 = time.time()
    g = av1.golden_encode(frames, w, h, q)
    t_gold = time.time() - t0
    packs = [[av1.scan_pack(lv, g.mode[i], p) for p, lv in enumerate((g.ly[i], g.lu[i], g.lv[i]))]
             for i in range(a.frames)]
    if a.dump:
        import struct

        with open(a.dump, "wb") as f:
            f.write(struct.pack("<3i", w, h, a.frames))
            for i in range(a.frames):
                for arr in (g.fparams[i], g.mode[i], g.mv[i], *packs[i], g.cdef_idx[i], g.lr[i]):
                    arr = np.ascontiguousarray(arr)
                    f.write(struct.pack("<q", arr.size))
                    f.write(arr.tobytes())
    best = [1e9] * a.frames
    sizes = [0] * a.frames
    for _ in range(a.reps):
        wr = av1.StreamWriter(w, h)
        for i in range(a.frames):
            t1 = time.perf_counter()
            tu = wr.write(g.fparams[i], g.mode[i], g.mv[i], packs[i][0], packs[i][1], packs[i][2], g.cdef_idx[i], 2,
                          i == 0, g.lr[i])
            best[i] = min(best[i], time.perf_counter() - t1)
            sizes[i] = len(tu)
    assert b"".join(av1.split_temporal_units(g.stream, g.tu_sizes)) == g.stream
    ok = sizes == list(map(int, g.tu_sizes))
    print({"res": a.res, "qindex": q, "golden_s": round(t_gold, 1),
           "writer_ms": [round(1000 * b, 2) for b in best], "bytes": sizes,
           "golden_bytes": list(map(int, g.tu_sizes)), "ok": ok})


if __name__ == "__main__":
    main()
