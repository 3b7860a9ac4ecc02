"""Residual quadtree (hevc_defs.h rqt_split): inter 32x32 / 16x16 CUs code four half-size
TBs when their luma residual is unevenly spread.  The golden encoder's streams decode to its
reconstruction with the split transform trees (split_transform_flag, depth-1 chroma cbfs,
internal TB edges in the deblocking filter), and the tool lowers the bitrate at equal or
better PSNR on the bench's synthetic content (the GPU engine is bit-exact with the golden
model: tests/test_gpu_engine.py)."""

import numpy as np

from thinvids_amd.models import hevc

W, H = 256, 160


def _clip(seed):
    return [hevc.synth_frame(seed, t, W, H) for t in range(6)]


def test_split_streams_decode_exactly():
    for seed in (2, 2 | (1 << 31)):
        frames = _clip(seed)
        for bf in (1, 4):
            bs, recons = hevc.encode_sequence_cpu(frames, qp=27, bframes=bf, search_range=32)
            dec = hevc.decode(bs)
            for r, d in zip(recons, dec.frames if bf > 1 else dec.coded_frames):
                for c in range(3):
                    np.testing.assert_array_equal(r[c][:d[c].shape[0], :d[c].shape[1]], d[c])


def _bytes_psnr(rqt: bool, seed: int) -> tuple[int, float]:
    fr = _clip(seed)
    bs, rec = hevc.encode_sequence_cpu(fr, qp=27, search_range=32, rqt=rqt)
    return len(bs), float(np.mean([hevc.psnr(f[0], r[0][:H, :W]) for f, r in zip(fr, rec)]))


def test_rqt_lowers_the_rate():
    n1, p1 = _bytes_psnr(True, 2)
    n0, p0 = _bytes_psnr(False, 2)
    assert n1 < n0 and p1 > p0 - 0.01, (n1, p1, n0, p0)
