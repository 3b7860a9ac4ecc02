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
