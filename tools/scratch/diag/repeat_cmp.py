"""Repeat a GPU-vs-CPU bit-exactness check N times in one process (flakiness hunt)."""
import sys

sys.path.insert(0, ".")
from thinvids_amd.models import hevc  # noqa: E402
from thinvids_amd.models.gpu_engine import GpuEngine  # noqa: E402

w, h, qp, gop, batch, threads, reps = 192, 128, 27, 4, 2, int(sys.argv[1]), int(sys.argv[2])
frames = [[hevc.synth_frame(5, s + f, w, h) for f in range(gop)] for s in (0, 10)]
cpu = [hevc.encode_sequence_cpu(fr, qp=qp, search_range=16)[0] for fr in frames]
res = []
for r in range(reps):
    eng = GpuEngine(width=w, height=h, qp=qp, batch=batch, gop=gop, search_range=16, seed=5, threads=threads)
    segs = eng.encode_synthetic([0, 10])
    segs2 = eng.encode_synthetic([0, 10])  # a second call on a warm engine
    res.append("".join("ok"[int(a == c)] if a == c else "X" for a, c in zip(segs + segs2, cpu + cpu)))
    eng.close()
print("threads", threads, res)
