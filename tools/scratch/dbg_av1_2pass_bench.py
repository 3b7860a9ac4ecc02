"""Debug: the bench's 2-pass AV1 flow on one GPU with per-frame bits of segment 0."""
import ctypes as C
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
from thinvids_amd.models import av1 as av1m
from thinvids_amd.models.av1_engine import Av1GpuEngine
from thinvids_amd.models.ratecontrol import frame_sizes, plan_frame_qps, round_qps
from thinvids_amd.ops import stage

w, h, B, G = 1920, 1080, 4, 16
eng = Av1GpuEngine(w, h, batch=B, qindex=av1m.qindex_for_hevc_qp(27))
W, H = eng.W, eng.H
lib = stage._lib()
dev = eng.dev


def load(t, planes):
    st = C.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    src = stage.synth_frames(1, w, h, [b * G + t for b in range(B)], dev)
    for c, dst in enumerate(planes):
        off, pw, ph, stride, fs = src.planes[c]
        cw, chh = (W, H) if c == 0 else (W // 2, H // 2)
        stage._ok(lib.tv_pad_batch(C.c_void_p(src.ptr(c)), pw, ph, stride, fs, C.c_void_p(dst.data_ptr()), cw, chh, cw,
                                   cw * chh, B, st))


g1 = eng.encode_gop(G, load)
s1 = [b"".join(f.result()) for f in eng.submit_entropy(g1)]
b1 = [8.0 * np.array(frame_sizes(x)) for x in s1]
plan, pred = plan_frame_qps(b1, 27, sum(x.sum() for x in b1) * 0.6, key_offset=-2.0)
qm = np.array([[av1m.qindex_for_hevc_qp(int(v)) for v in round_qps(p)] for p in plan], np.int32).T
g2 = eng.encode_gop(G, load, qmap=qm)
s2 = [b"".join(f.result()) for f in eng.submit_entropy(g2)]
b2 = [8.0 * np.array(frame_sizes(x)) for x in s2]
print("pass1 bits seg0", (b1[0] / 1000).round(1))
print("plan qp seg0", np.round(plan[0], 1))
print("qindex seg0", qm[:, 0])
print("pass2 bits seg0", (b2[0] / 1000).round(1))
print("ratio", sum(x.sum() for x in b2) / sum(x.sum() for x in b1), "pred", pred / sum(x.sum() for x in b1))
print("psnr1", eng.psnr(g1), "psnr2", eng.psnr(g2))
