"""GPU CABAC (csrc/gpu/k_entropy.hip): the engine's WPP substreams, binarised and
arithmetic-coded on the device, are byte-identical to the host CABAC writer
(csrc/core/hevc_writer.cpp, SeqConfig::wpp) driven by the golden CPU encoder — and to the same
engine with the host writer (entropy="host") — across slice types (I / P / B), SAO, RQT,
intra-in-P, CRF and textured content.  Runs only on an MI355X."""
import numpy as np
import pytest

from thinvids_amd.models import hevc

pytestmark = pytest.mark.gpu


def _engine(**kw):
    from thinvids_amd.models.gpu_engine import GpuEngine
    kw.setdefault("entropy", "gpu")  # "auto" would pick the host writer on a many-CPU box
    return GpuEngine(**kw)


def _golden(seed, starts, w, h, gop, **kw):
    out = []
    for s in starts:
        frames = [hevc.synth_frame(seed, s + f, w, h) for f in range(gop)]
        out.append(hevc.encode_sequence_cpu(frames, **kw)[0])
    return out


@pytest.mark.parametrize("w,h,qp,sao,extra", [
    (192, 128, 27, False, {}),
    (160, 96, 32, True, {}),
    (256, 160, 22, True, {}),
    (192, 128, 27, True, {"rqt": False, "pintra": False}),
    (320, 192, 37, False, {"rqt": False}),
])
def test_gpu_entropy_equals_host_writer(w, h, qp, sao, extra):
    gop, rng, seed, starts = 5, 16, 5, [0, 7, 20]
    eng = _engine(width=w, height=h, qp=qp, batch=3, gop=gop, search_range=rng, sao=sao, seed=seed, **extra)
    assert eng.entropy == "gpu"
    segs = eng.encode_synthetic(starts)
    st = eng.entropy_stats()
    assert (st["gpu"], st["fallbacks"], st["status"], st["host_pictures"]) == (True, 0, 0, 0), st
    gold = _golden(seed, starts, w, h, gop, qp=qp, sao=sao, search_range=rng, **extra)
    for b in range(len(starts)):
        assert segs[b] == gold[b], f"segment {b}: GPU CABAC differs from the host writer"
        d = hevc.decode(segs[b])
        gy, _, _ = eng.last_recon(b)
        np.testing.assert_array_equal(d.coded_frames[-1][0], gy)
    eng.close()


@pytest.mark.parametrize("qp", [0, 3, 51])
def test_cascade_edge_qps_clip_like_the_golden_encoder(qp):
    """Constant QP with the I P P P cascade at the ends of the range: the IDR's -5 and the
    P pictures' +1 clip to 0..51 (as cpu_encoder.cpp does) instead of failing the encode."""
    w, h, gop, rng, seed = 128, 96, 9, 16, 5
    for ent in ("gpu", "host"):
        eng = _engine(width=w, height=h, qp=qp, batch=2, gop=gop, search_range=rng, seed=seed, entropy=ent)
        segs = eng.encode_synthetic([0, 10])
        eng.close()
        assert segs == _golden(seed, [0, 10], w, h, gop, qp=qp, search_range=rng), ent


def test_gpu_entropy_equals_host_entropy_same_engine_config():
    """entropy="host" (the C++ writer on the engine's thread pool, WPP) and "gpu" give the
    same bytes at the bench geometry's width (60 CTB columns) on textured content."""
    w, h, gop, rng = 1920, 192, 3, 32
    seed = 7 | 0x80000000
    outs = []
    for ent in ("gpu", "host"):
        eng = _engine(width=w, height=h, qp=27, batch=2, gop=gop, search_range=rng, sao=True, seed=seed, entropy=ent)
        outs.append(eng.encode_synthetic([0, 30]))
        if ent == "gpu":
            assert eng.entropy_stats()["fallbacks"] == 0
        eng.close()
    assert outs[0] == outs[1]


def test_gpu_entropy_b_frames():
    """Hierarchical-B (B slices: inter_pred_idc, two AMVP lists with POC scaling, combined
    bi-predictive merge candidates) coded on the GPU equals the golden B encoder."""
    w, h, gop, rng, seed = 192, 128, 9, 16, 9
    eng = _engine(width=w, height=h, qp=27, batch=2, gop=gop, search_range=rng, sao=True, seed=seed, bframes=4)
    segs = eng.encode_synthetic([0, 40])
    assert eng.entropy_stats()["fallbacks"] == 0
    gold = _golden(seed, [0, 40], w, h, gop, qp=27, sao=True, search_range=rng, bframes=4)
    for b in range(2):
        assert segs[b] == gold[b], f"segment {b}"
        assert len(hevc.decode(segs[b]).frames) == gop
    eng.close()


def test_gpu_entropy_crf_and_qp_map():
    """Per-frame slice QPs (in-engine CRF; an explicit 2-pass QP map) reach the GPU
    coder's context initialisation and the host's slice_qp_delta."""
    w, h, gop, rng, seed = 192, 128, 5, 16, 5
    eng = _engine(width=w, height=h, qp=27, batch=2, gop=gop, search_range=rng, seed=seed, crf=30)
    segs = eng.encode_synthetic([0, 10])
    gold = _golden(seed, [0, 10], w, h, gop, qp=27, crf=30, search_range=rng)
    assert segs == gold
    eng.close()
    qmap = np.array([[24, 30, 33, 28, 35], [40, 22, 27, 27, 31]], np.int8)
    eng = _engine(width=w, height=h, qp=27, batch=2, gop=gop, search_range=rng, seed=seed)
    segs = eng.encode_synthetic([0, 10], qp=qmap)
    for b, s in enumerate([0, 10]):
        frames = [hevc.synth_frame(seed, s + f, w, h) for f in range(gop)]
        g, _ = hevc.encode_sequence_cpu(frames, qp=27, search_range=rng, frame_qps=qmap[b])
        assert segs[b] == g, f"segment {b}"
    eng.close()


def test_gpu_entropy_capacity_fallback(monkeypatch):
    """A token budget too small for the picture: the device reports it, the host writer codes
    that picture instead, and the stream is unchanged."""
    monkeypatch.setenv("TV_ENT_TOKENS_PER_PX", "0.0001")
    w, h, gop, rng, seed = 192, 128, 3, 16, 5
    eng = _engine(width=w, height=h, qp=22, batch=2, gop=gop, search_range=rng, seed=seed)
    segs = eng.encode_synthetic([0, 10])
    st = eng.entropy_stats()
    gold = _golden(seed, [0, 10], w, h, gop, qp=22, search_range=rng)
    assert segs == gold
    eng.close()
    assert st["gpu"] and st["fallbacks"] > 0 and st["status"] & 1, st


def test_two_coder_lanes_dense_routing_is_byte_identical(monkeypatch):
    """The second coder lane (pictures alternate between two entropy streams and their
    scratch once the content is dense): forced from the first picture with
    TV_ENT_DENSE_AFTER=0 on textured content, the stream equals the host writer's and the
    golden encoder's, and both lanes coded pictures."""
    monkeypatch.setenv("TV_ENT_LANES", "2")
    monkeypatch.setenv("TV_ENT_DENSE_AFTER", "0")
    w, h, gop, rng = 256, 160, 8, 16
    seed = 11 | 0x80000000
    eng = _engine(width=w, height=h, qp=22, batch=3, gop=gop, search_range=rng, seed=seed, sao=True)
    segs = eng.encode_synthetic([0, 9, 30])
    st = eng.entropy_stats()
    eng.close()
    assert st["fallbacks"] == 0 and min(st["lane_pictures"]) > 0, st
    host = _engine(width=w, height=h, qp=22, batch=3, gop=gop, search_range=rng, seed=seed, sao=True, entropy="host")
    assert segs == host.encode_synthetic([0, 9, 30])
    host.close()
    assert segs == _golden(seed, [0, 9, 30], w, h, gop, qp=22, search_range=rng, sao=True)


def test_lane_coder_is_byte_identical(monkeypatch):
    """TV_ENT_CODER=lanes (one wave per CTB row index, one lane per segment, the WPP hand-off
    between waves) codes the same bytes as the host writer on I / P pictures with SAO and on
    textured content."""
    monkeypatch.setenv("TV_ENT_CODER", "lanes")
    for seed, qp in ((5, 27), (3 | 0x80000000, 22)):
        w, h, gop, rng = 256, 160, 5, 16
        eng = _engine(width=w, height=h, qp=qp, batch=3, gop=gop, search_range=rng, seed=seed, sao=True)
        segs = eng.encode_synthetic([0, 7, 20])
        st = eng.entropy_stats()
        eng.close()
        assert st["fallbacks"] == 0, st
        assert segs == _golden(seed, [0, 7, 20], w, h, gop, qp=qp, search_range=rng, sao=True)


def test_hybrid_entropy_routes_pictures_to_the_host(monkeypatch):
    """TV_ENT_HOST=n: while fewer than n pictures sit in the host writer pool the next one is
    coded there instead of on the GPU; the stream is the same either way."""
    monkeypatch.setenv("TV_ENT_HOST", "1")
    w, h, gop, rng, seed = 192, 128, 6, 16, 5
    eng = _engine(width=w, height=h, qp=27, batch=2, gop=gop, search_range=rng, seed=seed, sao=True)
    segs = eng.encode_synthetic([0, 10])
    st = eng.entropy_stats()
    eng.close()
    assert st["gpu"] and st["host_pictures"] > 0 and st["fallbacks"] == 0, st
    assert segs == _golden(seed, [0, 10], w, h, gop, qp=27, search_range=rng, sao=True)
