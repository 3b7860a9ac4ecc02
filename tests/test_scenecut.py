"""Scene-cut IDRs: the detector finds an abrupt content switch (and ignores ordinary
motion), the chunk plan restarts the closed GOP there, and the encoded part carries an IDR
at the cut frame — cheaper and better than coding the cut as a P-frame."""
import numpy as np
import pytest

from thinvids_amd.models import hevc, scenecut
from thinvids_amd.worker.encoder import EncodeSpec, chunk_plan, encode_parts


def _clip(n=24, cut=13, w=128, h=96):
    a = [hevc.synth_frame(3, t, w, h) for t in range(cut)]
    b = [hevc.synth_frame(77, 500 + t, w, h) for t in range(n - cut)]
    return a + b


def _slice_types(annexb: bytes) -> list[int]:
    out, i = [], 0
    while True:
        j = annexb.find(b"\x00\x00\x01", i)
        if j < 0:
            return out
        t = (annexb[j + 3] >> 1) & 0x3F
        if t <= 31:
            out.append(t)
        i = j + 3


def test_detector_and_plan():
    frames = _clip()
    assert scenecut.detect(scenecut.diffs_host(frames)) == [13]
    still = [hevc.synth_frame(3, t, 128, 96) for t in range(24)]  # panning content: no cut
    assert scenecut.detect(scenecut.diffs_host(still)) == []
    assert chunk_plan(24, 8, [13]) == [(0, 8), (8, 5), (13, 8), (21, 3)]
    assert chunk_plan(24, 8) == [(0, 8), (8, 8), (16, 8)]
    assert chunk_plan(10, 64, [3, 5]) == [(0, 3), (3, 2), (5, 5)]
    d = np.array([1, 1, 30, 31, 1, 40], np.float32)  # d[t-1] for frames t = 1..6
    # t=3 is within min_gap of the part start (an IDR anyway), t=6 within min_gap of t=4
    assert scenecut.detect(d, min_gap=4) == [4]


def test_scenecut_idr_in_cpu_encode():
    frames = _clip()
    base = EncodeSpec(128, 96, qp=30, gop=16, software=True, search_range=16)
    on = EncodeSpec(128, 96, qp=30, gop=16, software=True, search_range=16, scenecut=True)
    b_off, b_on = encode_parts([frames], base)[0], encode_parts([frames], on)[0]
    idr = lambda bs: [k for k, t in enumerate(_slice_types(bs)) if t in (19, 20)]
    assert idr(b_off) == [0, 16] and idr(b_on) == [0, 13]  # the cadence restarts at the cut
    d_on = hevc.decode(b_on, coded=False).frames
    d_off = hevc.decode(b_off, coded=False).frames
    ps = lambda dec: np.mean([hevc.psnr_yuv(a, b)["y"] for a, b in zip(frames[13:16], dec[13:16])])
    # the cut frame as an IDR: no worse quality around the cut, and not more bits overall
    assert ps(d_on) >= ps(d_off) - 0.05 and len(b_on) <= len(b_off) * 1.02


@pytest.mark.gpu
def test_scenecut_idr_gpu_matches_cpu():
    frames = _clip(n=32, cut=13, w=192, h=128)
    spec = dict(qp=30, gop=16, search_range=16, scenecut=True)
    g = encode_parts([frames], EncodeSpec(192, 128, **spec))[0]
    c = encode_parts([frames], EncodeSpec(192, 128, software=True, **spec))[0]
    assert g == c


@pytest.mark.gpu
def test_device_thumbnails_equal_host():
    """k_thumbs8 (csrc/gpu/k_stage.hip) against the numpy 8x8 means (exact), 8-bit and
    10-bit, whole buffers and a view at an offset; d(t) equal to the host's up to the order
    of the final mean."""
    import torch

    from thinvids_amd.ops import stage

    frames = _clip(n=6, cut=3, w=136, h=72)
    dev = stage.upload_frames(frames, torch.device("cuda", 0))
    close = lambda a, b: np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-5)  # noqa: E731 (mean order)
    close(scenecut.diffs_device(dev), scenecut.diffs_host(frames))
    f10 = [tuple((p.astype(np.uint16) * 4 + (p & 3)) for p in f) for f in frames]
    d10 = stage.upload_frames(f10, torch.device("cuda", 0))
    close(scenecut.diffs_device(d10), scenecut.diffs_host(f10))
    # planes at an offset into the buffer: a view one frame in
    close(scenecut.diffs_device(dev.select(1, 5)), scenecut.diffs_host(frames[1:]))
    # the thumbnails themselves
    t = torch.empty((6, 9, 17), dtype=torch.float32, device="cuda")
    off, w, h, stride, fs = dev.planes[0]
    stage.thumbs8(dev.ptr(0), 8, w, h, stride, fs, 6, t)
    np.testing.assert_array_equal(t.cpu().numpy(), scenecut.thumbs_host(frames))
