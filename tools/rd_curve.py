"""Rate-distortion curve of the golden HEVC encoder on the bench's synthetic content.

    python tools/rd_curve.py --res 640x360 --frames 32 --qps 22,27,32,37 [--cascade 1,3,2,3] [--textured]

Prints one JSON line per QP (kbps per 30 fps stream, PSNR-Y / YUV over the whole clip) and,
with --anchor FILE (a previous run's output), the BD-rate against it.  The GPU engine is bit-
exact with this encoder, so the curve is the engine's curve too.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from concurrent.futures import ProcessPoolExecutor

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run_point(args):
    qp, a = args
    from thinvids_amd.models import hevc

    w, h = map(int, a["res"].split("x"))
    seed = a["seed"] | (1 << 31 if a["textured"] else 0)
    frames = [hevc.synth_frame(seed, t, w, h) for t in range(a["frames"])]
    cascade = a["cascade"]
    fq = None
    if cascade:
        fq, k = [], 0
        for i in range(len(frames)):
            idr = i % a["gop"] == 0
            fq.append(max(0, min(51, qp + (a["iqp"] if idr else cascade[(i % a["gop"] - 1) % len(cascade)]))))
    import numpy as np

    if a.get("codec") == "av1":
        from thinvids_amd.models import av1

        q = av1.qindex_for_hevc_qp(qp)
        W, H = av1.coded_size(w, h)
        stream, ys = b"", []
        for s0 in range(0, len(frames), a["gop"]):
            n = min(a["gop"], len(frames) - s0)
            qm = None
            if fq is not None:  # a QP cascade in HEVC QP units, mapped to q-indices
                qm = [av1.qindex_for_hevc_qp(x) for x in fq[s0:s0 + n]]
            r = av1.golden_encode(frames[s0:s0 + a["gop"]], w, h, q, qmap=qm)
            stream += r.stream
            ys += [hevc.psnr(f[0], rec[:W * H].reshape(H, W)[:h, :w]) for f, rec in zip(frames[s0:], r.recon)]
    else:
        kw = dict(sao=a["sao"], rqt=a["rqt"], pintra=a["pintra"], wpp=a["wpp"], cascade=a["ippp_cascade"], rdoq=a["rdoq"])
        stream, recons = hevc.encode_sequence_cpu(frames, qp=qp, gop=a["gop"], frame_qps=fq, bframes=a["bframes"], **kw)
        ys = [hevc.psnr(f[0], r[0][:h, :w]) for f, r in zip(frames, recons)]

    mse_y = np.mean([10 ** (-p / 10) for p in ys])
    py = -10 * np.log10(mse_y)
    kbps = len(stream) * 8 * 30 / len(frames) / 1000
    return {"qp": qp, "kbps": round(kbps, 2), "psnr_y": round(float(py), 4), "frames": len(frames)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--res", default="640x360")
    ap.add_argument("--frames", type=int, default=32)
    ap.add_argument("--gop", type=int, default=64)
    ap.add_argument("--qps", default="22,27,32,37")
    ap.add_argument("--cascade", default="", help="P-frame QP offsets repeating over the GOP, e.g. 3,2,3,1")
    ap.add_argument("--iqp", type=int, default=0, help="I-frame QP offset (with --cascade)")
    ap.add_argument("--sao", type=int, default=1)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--textured", action="store_true")
    ap.add_argument("--bframes", type=int, default=1, help="hierarchical-B mini-GOP size (1 = IPPP)")
    ap.add_argument("--codec", choices=("hevc", "av1"), default="hevc",
                    help="av1: the golden AV1 encoder at the q-index matched to each QP")
    # coding tools: explicit flags; this tool alone also honours TV_RQT=0 / TV_PINTRA=0 / TV_WPP=0
    # (A/B sweeps), nothing else in the framework reads them from the environment
    env_on = lambda k: os.environ.get(k, "1") != "0"
    ap.add_argument("--rqt", type=int, default=int(env_on("TV_RQT")))
    ap.add_argument("--ippp-cascade", type=int, default=1, help="built-in constant-QP I P P P QP cascade (tv/gop.h)")
    ap.add_argument("--pintra", type=int, default=int(env_on("TV_PINTRA")))
    ap.add_argument("--wpp", type=int, default=int(env_on("TV_WPP")))
    ap.add_argument("--rdoq", type=int, default=1, help="RDOQ-lite coefficient-group trimming")
    ap.add_argument("--anchor", default="")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    cfg = dict(res=a.res, frames=a.frames, gop=a.gop, sao=bool(a.sao), seed=a.seed, textured=a.textured,
               cascade=[int(x) for x in a.cascade.split(",")] if a.cascade else [], iqp=a.iqp,
               bframes=a.bframes, codec=a.codec, rqt=bool(a.rqt), pintra=bool(a.pintra), wpp=bool(a.wpp),
               ippp_cascade=bool(a.ippp_cascade), rdoq=bool(a.rdoq))
    qps = [int(q) for q in a.qps.split(",")]
    with ProcessPoolExecutor(len(qps)) as ex:
        pts = list(ex.map(run_point, [(q, cfg) for q in qps]))
    for p in pts:
        print(json.dumps(p))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(pts, f)
    if a.anchor:
        from thinvids_amd.utils.bdrate import bd_rate

        with open(a.anchor) as f:
            anc = json.load(f)
        print(json.dumps({"bd_rate_pct": round(bd_rate([p["kbps"] for p in anc], [p["psnr_y"] for p in anc],
                                                        [p["kbps"] for p in pts], [p["psnr_y"] for p in pts]), 2)}))


if __name__ == "__main__":
    main()
