"""Debug: per-chunk PSNR of the batched worker encode path."""
from thinvids_amd.models import hevc
from thinvids_amd.models.gpu_engine import GpuEngine

frames = [hevc.synth_frame(5, t, 192, 128) for t in range(40)]
for batch, nseg, n in ((4, 3, 8), (4, 1, 8), (1, 1, 8), (4, 2, 5), (2, 2, 8)):
    eng = GpuEngine(192, 128, qp=30, batch=batch, gop=8, search_range=16)
    segs = [frames[8 * i:8 * i + n] for i in range(nseg)]
    bits = eng.encode_frames(segs)
    for i, b in enumerate(bits):
        d = hevc.decode(b, coded=False)
        cpu = hevc.encode_sequence_cpu(segs[i], qp=30, search_range=16)[0]
        print(batch, nseg, n, i, len(d.frames), [round(hevc.psnr(a[0], x[0]), 1) for a, x in zip(segs[i], d.frames)],
              "eq_cpu", b == cpu, len(b), len(cpu))
    eng.close()
