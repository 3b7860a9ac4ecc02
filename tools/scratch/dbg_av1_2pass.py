import sys, numpy as np, torch
sys.path.insert(0, '.')
from thinvids_amd.models import av1 as av1m
from thinvids_amd.models.av1_engine import Av1GpuEngine
from thinvids_amd.models.ratecontrol import frame_sizes, plan_frame_qps, round_qps
from tests.test_av1_codec import _frames
w, h, B, G = 480, 272, 2, 8
segs = [_frames(3, w, h, G, 0), _frames(3, w, h, G, 8)]
W, H = av1m.coded_size(w, h)
eng = Av1GpuEngine(w, h, batch=B, qindex=av1m.qindex_for_hevc_qp(27))
def load(t, planes):
    for b, fr in enumerate(segs):
        for dst, x in zip(planes, av1m.pad_frame(fr[t], W, H)):
            dst[b].copy_(torch.from_numpy(np.ascontiguousarray(x)).to(eng.dev))
g1 = eng.encode_gop(G, load)
s1 = [b"".join(f.result()) for f in eng.submit_entropy(g1)]
b1 = [8.0 * np.array(frame_sizes(x)) for x in s1]
plan, _ = plan_frame_qps(b1, 27, sum(x.sum() for x in b1) * 0.6)
qm = np.array([[av1m.qindex_for_hevc_qp(int(v)) for v in round_qps(p)] for p in plan], np.int32).T
print('qm', qm.T)
g2 = eng.encode_gop(G, load, qmap=qm)
print('g2.qm', g2.qm.T)
s2 = [b"".join(f.result()) for f in eng.submit_entropy(g2)]
print('ratio', sum(map(len, s2)) / sum(map(len, s1)))
gold = [av1m.golden_encode(s, w, h, 102, qmap=qm[:, b]) for b, s in enumerate(segs)]
print('golden ratio', sum(len(x.stream) for x in gold) / sum(map(len, s1)), [x.stream == y for x, y in zip(gold, s2)])
