"""ABR ladder (BASELINE config #5): rung planning on CPU; on the GPU the batched
tone-map / Lanczos kernels against the single-frame HIP ops + numpy edge padding (exact),
and a small ladder end to end through the oracle decoder."""
import numpy as np
import pytest

from thinvids_amd.models import abr


def test_plan_rungs_8k():
    r = abr.plan_rungs(7680, 4320)
    assert r == [(3840, 2160), (2560, 1440), (1920, 1080), (1280, 720), (854, 480)]
    # never upscales, duplicates collapse
    assert abr.plan_rungs(1920, 1080, (2160, 1080, 720)) == [(1920, 1080), (1280, 720)]


def test_split_threads_proportional():
    t = abr.split_threads(abr.plan_rungs(7680, 4320), 16)
    assert t[0] >= t[1] >= t[2] >= 2 and t[-1] == 2
    assert sum(t) <= 16 + 2 * len(t)


def test_resize2d_plan_fits_lds():
    for geo in ((7680, 4320, 3840, 2160, 3840, 2176), (3840, 2160, 854, 480, 864, 480),
                (640, 360, 426, 240, 448, 256)):
        th, wp, smem = abr.resize2d_plan(*geo)
        assert th >= 8 and wp % 4 == 0 and 0 < smem <= 40 * 1024


def test_staging_layout_coded_size():
    L = abr.staging_layout(854, 480)
    assert (L["cw"], L["ch"]) == (864, 480)
    assert L["fsz"] == 864 * 480 * 3 // 2
    y, u, v = L["planes"]
    assert y == (0, 854, 480, 864, 864, 480)
    assert u[0] == 864 * 480 and v[0] == 864 * 480 + 432 * 240


@pytest.mark.gpu
@pytest.mark.parametrize("cascade,fused", [(False, True), (True, True), (True, False)])
def test_ladder_chunk_matches_single_frame_ops(cascade, fused):
    import torch

    from thinvids_amd.models.gpu_engine import pad_frame
    from thinvids_amd.ops import color, resize

    lad = abr.AbrLadder(src_w=640, src_h=360, heights=(240, 180, 120), segments=2, gop=3, cascade=cascade,
                        fused=fused)
    try:
        lad.synth_p010(5, 3)
        y16, uv16 = lad.y16.clone(), lad.uv16.clone()
        lad.ladder_chunk(3, 3, slot=1)
        lad.staging = lad.staging_slots[1]
        torch.cuda.synchronize()
        assert int(y16.to(torch.int32).min()) >= 64 << 6 and int(y16.to(torch.int32).max()) <= 940 << 6
        for f in range(3):
            sdr = color.tonemap_pq(y16[f], uv16[f])
            got_sdr = lad.sdr[f].cpu().numpy()
            want_sdr = np.concatenate([p.cpu().numpy().ravel() for p in sdr])
            assert np.array_equal(got_sdr, want_sdr)
            first = None
            for (w, h), L, st in zip(lad.rungs, lad.layouts, lad.staging):
                planes = resize.resize_frame(first if (cascade and first is not None) else sdr, w, h)
                first = first or planes
                want = pad_frame(*[p.cpu().numpy() for p in planes], L["cw"], L["ch"])
                assert np.array_equal(st[3 + f].cpu().numpy(), want), (w, h, f)
    finally:
        lad.close()


@pytest.mark.gpu
def test_ladder_encode_decodes():
    from thinvids_amd.models import hevc

    lad = abr.AbrLadder(src_w=640, src_h=360, heights=(360, 240, 180), segments=2, gop=4)
    try:
        segs = lad.encode_synthetic([0, 4])
        assert len(segs) == 3 and all(len(s) == 2 for s in segs)
        for r, (eng, rung) in enumerate(zip(lad.engines, segs)):
            for b, bs in enumerate(rung):
                d = hevc.decode(bs)
                assert len(d.frames) == 4
                gy, _, _ = eng.last_recon(b)
                assert np.array_equal(d.coded_frames[-1][0], gy)
        q = lad.psnr()
        assert [(x["w"], x["h"]) for x in q] == lad.rungs
        assert all(x["y"] > 30 for x in q), q
    finally:
        lad.close()


@pytest.mark.gpu
def test_ladder_overlapped_equals_serial():
    lad = abr.AbrLadder(src_w=640, src_h=360, heights=(240, 180), segments=2, gop=4)
    try:
        serial = [lad.encode_synthetic([0, 4]), lad.encode_synthetic([8, 12])]
        lad.prepare_synthetic([0, 4], slot=0)
        import torch

        torch.cuda.synchronize()
        a = lad.encode_overlapped(2, 0, prepare_next=lambda: (lad.prepare_synthetic([8, 12], slot=1),
                                                               torch.cuda.synchronize()))
        b = lad.encode_overlapped(2, 1)
        assert [a, b] == serial
    finally:
        lad.close()
