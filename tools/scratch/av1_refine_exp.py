"""Bits / PSNR of the golden AV1 encoder on the synthetic source (used to evaluate the
rejected MV-refinement pass, profiles/README.md).  Usage: w h frames qindex."""
import os, sys, numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from thinvids_amd.models import av1, hevc
w, h, n, q = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
frames = [tuple(hevc.synth_frame(3, t, w, h)) for t in range(n)]
r = av1.golden_encode(frames, w, h, q)
W, H = av1.coded_size(w, h)
rec = r.recon.reshape(n, -1)
mse = []
for t in range(n):
    y = rec[t, :W * H].reshape(H, W)[:h, :w].astype(np.float64)
    mse.append(np.mean((y - frames[t][0].astype(np.float64)) ** 2))
ps = 10 * np.log10(255 ** 2 / np.mean(mse))
m = r.mode
print(f"bytes={len(r.stream)} I={r.tu_sizes[0]} P={sum(r.tu_sizes[1:])} psnrY={ps:.3f} mvs_distinct={[len(set(r.mv[t].tolist())) for t in range(1, n)]}")
for t in range(1, n):
    md = r.mode[t]
    skip = ((md >> 9) & 1).sum()
    nzy = ((md >> 10) & 1).sum(); nzu = ((md >> 11) & 1).sum(); nzv = ((md >> 12) & 1).sum()
    cy = (r.ly[t] != 0).sum(); cu = (r.lu[t] != 0).sum() + (r.lv[t] != 0).sum()
    zero = (r.mv[t] == 0).sum()
    print(f"f{t}: blocks={md.size} skip={skip} nzY={nzy} nzU={nzu} nzV={nzv} coefY={cy} coefUV={cu} zeromv={zero} bytes={r.tu_sizes[t]}")
