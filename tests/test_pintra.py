"""Intra 16x16 CUs in P pictures (tv/me_model.h pintra_*): the golden encoder codes badly
predicted quadrants as intra, only in the pattern the four-pass parallel GPU reconstruction
can honour, the streams decode to the encoder's reconstruction, a cut coded as P gets
cheaper, and the GPU engine is bit-exact with the golden model."""

import numpy as np
import pytest

from thinvids_amd.models import hevc

W, H = 320, 192


def _cut_clip(n=8, cut=4):
    return [hevc.synth_frame(3, t, W, H) for t in range(cut)] + \
           [hevc.synth_frame(77, 500 + t, W, H) for t in range(n - cut)]


def _encode(frames, qp=30, pintra=True):
    enc = hevc.CpuEncoder(W, H, qp=qp, search_range=32, pintra=pintra)
    stream, intra, recons = b"", [], []
    for t, f in enumerate(frames):
        stream += enc.encode(f, t == 0, t)
        intra.append(enc.decisions()["intra"].copy())
        recons.append(enc.recon())
    return stream, intra, recons


def _later_pass_neighbours(q):
    """Quadrants (dx CTBs, dy CTBs, quadrant) whose acceptance would break pass q: the
    z-scan-available intra-prediction neighbours reconstructed in a later pass."""
    return {3: [], 2: [(-1, 0, 3)], 1: [(0, -1, 3), (0, -1, 2), (1, -1, 2)],
            0: [(-1, 0, 1), (-1, 0, 3), (-1, -1, 3), (0, -1, 2), (0, -1, 3)]}[q]


def test_cut_coded_as_p_uses_intra_quadrants_in_a_parallel_safe_pattern():
    frames = _cut_clip()
    stream, intra, recons = _encode(frames)
    p_intra = intra[4]  # the first picture after the cut (a P picture)
    assert p_intra.sum() >= 0.2 * p_intra.size, "a cut should be coded mostly intra"
    for k, m in enumerate(intra[1:], 1):  # P pictures: intra units form whole 16x16 quadrants
        q16 = m.reshape(m.shape[0] // 2, 2, m.shape[1] // 2, 2)
        assert np.all((q16.min(axis=(1, 3)) == q16.max(axis=(1, 3)))), f"picture {k}: partial intra quadrant"
        qa = q16[:, 0, :, 0]  # [rows of 16][cols of 16]
        hc, wc = qa.shape[0] // 2, qa.shape[1] // 2
        for j in range(hc):
            for i in range(wc):
                for q in range(4):
                    if not qa[2 * j + (q >> 1), 2 * i + (q & 1)]:
                        continue
                    for dx, dy, nq in _later_pass_neighbours(q):
                        ii, jj = i + dx, j + dy
                        if 0 <= ii < wc and 0 <= jj < hc:
                            assert not qa[2 * jj + (nq >> 1), 2 * ii + (nq & 1)], (k, i, j, q, dx, dy, nq)
    dec = hevc.decode(stream)
    for d, r in zip(dec.coded_frames, recons):
        for c in range(3):
            np.testing.assert_array_equal(d[c], r[c])


def _bytes_and_psnr(on: bool) -> tuple[int, float]:
    fr = _cut_clip()
    st, _, rec = _encode(fr, pintra=on)
    return len(st), float(np.mean([hevc.psnr(f[0], r[0][:H, :W]) for f, r in zip(fr, rec)]))


def test_intra_in_p_makes_a_cut_cheaper():
    n_on, p_on = _bytes_and_psnr(True)
    n_off, p_off = _bytes_and_psnr(False)
    assert n_on < 0.985 * n_off and p_on > p_off - 0.02, (n_on, p_on, n_off, p_off)


@pytest.mark.gpu
def test_gpu_intra_in_p_bit_exact():
    from thinvids_amd.models.gpu_engine import GpuEngine

    frames = _cut_clip()
    eng = GpuEngine(width=W, height=H, qp=30, batch=1, gop=len(frames), search_range=32)
    try:
        seg = eng.encode_frames([frames])[0]
    finally:
        eng.close()
    cpu_bs, _ = hevc.encode_sequence_cpu(frames, qp=30, search_range=32)
    assert seg == cpu_bs, "GPU bitstream with intra quadrants in P pictures differs from the golden model"
