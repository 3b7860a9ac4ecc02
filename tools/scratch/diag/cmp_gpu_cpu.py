"""Diagnose a GPU-vs-CPU bitstream mismatch: per-NAL comparison and per-frame recon diff."""
import sys

import numpy as np

sys.path.insert(0, ".")
from thinvids_amd.models import hevc  # noqa: E402
from thinvids_amd.models.gpu_engine import GpuEngine  # noqa: E402


def nals(bs):
    out, i = [], 0
    idx = [k for k in range(len(bs) - 3) if bs[k:k + 4] == b"\x00\x00\x00\x01"]
    idx.append(len(bs))
    return [bs[idx[j]:idx[j + 1]] for j in range(len(idx) - 1)]


w, h, qp, gop = 192, 128, 27, int(sys.argv[1]) if len(sys.argv) > 1 else 4
batch = int(sys.argv[2]) if len(sys.argv) > 2 else 2
eng = GpuEngine(width=w, height=h, qp=qp, batch=batch, gop=gop, search_range=16, seed=5)
segs = eng.encode_synthetic([0, 10][:batch])
seg = int(sys.argv[3]) if len(sys.argv) > 3 else 0
start = [0, 10][seg]
frames = [hevc.synth_frame(5, start + f, w, h) for f in range(gop)]
cpu_bs, recons = hevc.encode_sequence_cpu(frames, qp=qp, search_range=16)
a, b = nals(segs[seg]), nals(cpu_bs)
print("nals", len(a), len(b), [len(x) for x in a], [len(x) for x in b])
for k, (x, y) in enumerate(zip(a, b)):
    if x != y:
        d = next(i for i in range(min(len(x), len(y))) if x[i] != y[i]) if x[:min(len(x), len(y))] != y[:min(len(x), len(y))] else min(len(x), len(y))
        print("first differing NAL", k, "at byte", d)
        break
dg = hevc.decode(segs[seg])
for f in range(gop):
    gy = dg.coded_frames[f][0]
    cy = recons[f][0]
    diff = np.argwhere(gy != cy)
    print("frame", f, "luma mismatches", len(diff), diff[:5].tolist())
    for c in (1, 2):
        dd = np.argwhere(dg.coded_frames[f][c] != recons[f][c])
        print("   chroma", c, len(dd), dd[:5].tolist())
