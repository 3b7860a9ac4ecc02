"""AV1 bitstream conformance against an independent decoder.

The encoder's streams are wrapped as AVIF (key frame) / AVIS (image sequence) and decoded
by dav1d 1.5.3 through libavif (the AVIF plugin library bundled with Pillow, called with
ctypes: ``thinvids_amd.models.avif.dav1d_decode``, which returns the decoder's Y/U/V
planes, no colour conversion).  Every decoded frame must equal the encoder's
reconstruction exactly -- any error in a CDF, context, scan, quantiser, transform or
loop filter shows up as a mismatch.  Coverage: key + inter frames with deblocking, CDEF
and self-guided loop restoration on, frame sizes that are multiples of 16, a render size
that is not (coded size padded), the benchmark geometry (1920x1080), and the GPU engine's
own streams (GPU tests).

Reference parity: the reference never writes AV1 (it rejects AV1 sources,
/root/reference/worker/tasks.py:929-939, and encodes H.264 at :1573-1586); this is
BASELINE config #4's codec.
"""
import numpy as np
import pytest

from thinvids_amd.models import av1, avif, hevc

pytestmark = pytest.mark.skipif(not avif.dav1d_available(), reason="libavif / dav1d (Pillow AVIF plugin) missing")


def _frames(seed, w, h, n, t0=0):
    return [tuple(hevc.synth_frame(seed, t0 + t, w, h)) for t in range(n)]


def _planes(rec, W, H):
    return (rec[:W * H].reshape(H, W), rec[W * H:W * H * 5 // 4].reshape(H // 2, W // 2),
            rec[W * H * 5 // 4:].reshape(H // 2, W // 2))


def _check(stream, tu_sizes, recon, w, h):
    """dav1d-decode a stream (AVIF for one frame, AVIS otherwise) and compare every plane
    of every frame with the encoder's coded-size reconstruction."""
    W, H = av1.coded_size(w, h)
    tus = av1.split_temporal_units(stream, tu_sizes)
    data = avif.avif_still(tus[0], w, h) if len(tus) == 1 else avif.avis_sequence(tus, w, h)
    dec = avif.dav1d_decode(data)
    assert len(dec) == len(tus)
    for k, (got, rec) in enumerate(zip(dec, recon)):
        for c, (g, r) in enumerate(zip(got, _planes(rec, W, H))):
            assert g.shape == r.shape, (k, c, g.shape, r.shape)
            bad = np.argwhere(g != r)
            assert not len(bad), f"frame {k} plane {c}: {len(bad)} samples differ, first {bad[0].tolist()}"


def test_key_frame_avif_decodes_exactly():
    w, h = 160, 96
    res = av1.golden_encode(_frames(3, w, h, 1), w, h, 100)
    _check(res.stream, res.tu_sizes, res.recon, w, h)


@pytest.mark.parametrize("w,h,q", [(160, 96, 100), (200, 120, 60), (264, 200, 160)])
def test_gop_avis_decodes_exactly(w, h, q):
    """Key + 15 inter frames, deblocking + CDEF + restoration on; 200x120 and 264x200 have
    a render size smaller than the coded size and partial superblocks / restoration units."""
    res = av1.golden_encode(_frames(7, w, h, 16), w, h, q)
    assert (res.lr[..., 0] >= 0).any(), "restoration never used: the LR path is not exercised"
    assert (res.fparams[:, 2] > 0).all(), "deblocking off"
    _check(res.stream, res.tu_sizes, res.recon, w, h)


def test_static_content_merged_blocks_decode_exactly():
    """Skip-block merging (32x32 / 64x64 inter blocks, TX_64X64 edges) on static content."""
    w, h = 200, 136
    f0 = _frames(5, w, h, 1)[0]
    res = av1.golden_encode([f0] * 4, w, h, 120)
    assert (((res.mode[1:] >> 13) & 3) == 2).any()
    _check(res.stream, res.tu_sizes, res.recon, w, h)


def test_benchmark_geometry_1080p_decodes_exactly():
    """1920x1080 (coded 1088: split_or_horz superblock row, 17 restoration unit rows)."""
    w, h = 1920, 1080
    res = av1.golden_encode(_frames(11, w, h, 3), w, h, 110)
    _check(res.stream, res.tu_sizes, res.recon, w, h)


def test_spec_tables_match_libavif_copies():
    """The committed tables (csrc/include/tv/av1_tables.h) equal what the generator reads
    out of the bundled libaom / dav1d today, and the q lookups have the spec's end points."""
    import re
    from pathlib import Path

    text = (Path(__file__).resolve().parents[1] / "csrc/include/tv/av1_tables.h").read_text()
    acq = [int(v) for v in re.search(r"kAcQLookup\[256\] = \{([^}]*)\}", text).group(1).split(",") if v.strip()]
    dcq = [int(v) for v in re.search(r"kDcQLookup\[256\] = \{([^}]*)\}", text).group(1).split(",") if v.strip()]
    assert acq[0] == 4 and acq[255] == 1828 and dcq[0] == 4 and dcq[255] == 1336
    assert av1.ac_q(255) == 1828 and av1.ac_q(100) == acq[100]


# ---------------------------------------------------------------------------- GPU -----
@pytest.mark.gpu
def test_gpu_engine_stream_decodes_exactly_1080p():
    """The GPU engine's own 1080p GOP (key + 15 inter frames, all loop filters) through
    dav1d equals the engine's final reconstruction of every frame."""
    import torch

    from thinvids_amd.models.av1_engine import Av1GpuEngine

    w, h, n = 1920, 1080, 16
    W, H = av1.coded_size(w, h)
    frames = [av1.pad_frame(f, W, H) for f in _frames(21, w, h, n)]
    eng = Av1GpuEngine(w, h, batch=1, qindex=110)
    recon = []

    def load(t, planes):
        if t:  # the previous frame's final reconstruction is complete once frame t starts
            recon.append(np.concatenate([x[0].cpu().numpy().reshape(-1) for x in eng.fin]))
        for dst, x in zip(planes, frames[t]):
            dst[0].copy_(torch.from_numpy(np.ascontiguousarray(x)).to(eng.dev))

    g = eng.encode_gop(n, load)
    recon.append(np.concatenate([x[0].cpu().numpy().reshape(-1) for x in eng.fin]))
    tus = eng.submit_entropy(g)[0].result()
    eng.close()
    stream = b"".join(tus)
    _check(stream, [len(t) for t in tus], recon, w, h)


def test_directional_intra_decodes_exactly(monkeypatch):
    """D135 / D113 / D157 (7.11.2.4 without the edge filter, av1_enc.h intra_dir_px): with the
    search widened to them (TV_AV1_DBG bit 32) key frames use them and dav1d reproduces the
    encoder's reconstruction bit for bit, luma and chroma."""
    monkeypatch.setenv("TV_AV1_DBG", "32")
    w, h = 200, 120
    fr = _frames(1, w, h, 2) + _frames(1 | (1 << 31), w, h, 1, t0=5)
    for f in (fr[:2], fr[2:]):
        r = av1.golden_encode(f, w, h, 100)
        ym = (np.asarray(r.mode[0]).astype(np.uint32) >> 1) & 15
        uvm = (np.asarray(r.mode[0]).astype(np.uint32) >> 5) & 15
        assert np.isin(ym, (4, 5, 6)).sum() > 0 and np.isin(uvm, (4, 5, 6)).sum() > 0
        _check(r.stream, r.tu_sizes, r.recon, w, h)
