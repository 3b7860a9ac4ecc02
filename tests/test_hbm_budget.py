"""HBM-aware engine sizing (verdict r3 item 8): the native footprint ledger and its
no-allocation estimate, the byte-budgeted EngineCache (LRU eviction by bytes) and the
budget-capped auto_batch."""
import pytest

from thinvids_amd.worker.encoder import EncodeSpec, EngineCache, auto_batch, engine_bytes

GiB = 1 << 30


def test_estimate_scales_with_batch_sao_and_dpb():
    from thinvids_amd.models.gpu_engine import estimate_footprint

    a = estimate_footprint(1920, 1080, 24, 64)["dev"]
    b = estimate_footprint(1920, 1080, 48, 64)["dev"]
    assert 1.9 < b / a < 2.05  # per-segment buffers dominate
    assert estimate_footprint(1920, 1080, 48, 64, sao=True)["dev"] > b  # the SAO scratch set
    assert estimate_footprint(1920, 1080, 48, 64, bframes=8)["dev"] > b  # a deeper DPB
    assert 3 * GiB < b < 8 * GiB  # 1080p x 48: the measured order of magnitude
    assert estimate_footprint(3840, 2160, 24, 64)["dev"] > 1.9 * a


class _FakeEngine:
    def __init__(self, spec, batch):
        self.spec, self.batch, self.closed = spec, batch, False
        from thinvids_amd.models.gpu_engine import estimate_footprint

        self._fp = estimate_footprint(spec.width, spec.height, batch, spec.gop, spec.sao)

    def footprint(self):
        return self._fp

    def close(self):
        self.closed = True


def test_engine_cache_evicts_by_bytes(monkeypatch):
    monkeypatch.setenv("TV_ENTROPY", "host")  # footprints without the GPU coder's scratch
    cache = EngineCache(batch=0, max_engines=16, budget=64 * GiB)
    monkeypatch.setattr(cache, "_build", lambda spec, batch: _FakeEngine(spec, batch))
    hd = [EncodeSpec(1920, 1080, qp=q) for q in (22, 25, 27, 30, 32)]
    uhd = EncodeSpec(3840, 2160, qp=27)
    engines = [cache.get(s) for s in hd]  # 5 x ~15 GiB (engine + staging): the oldest go
    assert cache.used_bytes() <= cache.budget
    assert engines[0].closed and not engines[4].closed and cache.evicted == 1
    assert cache.get(hd[1]) is engines[1]  # a hit refreshes the LRU order
    e4 = cache.get(uhd)  # ~30 GiB: evicts the least recently used (2, 3), keeps 1 and 4
    assert cache.used_bytes() <= cache.budget and not e4.closed
    assert engines[2].closed and engines[3].closed and not engines[1].closed and not engines[4].closed
    assert e4.batch == 24 and engines[4].batch == 48  # CU-fill heuristic, inside the budget


def test_engine_cache_refuses_an_engine_over_budget(monkeypatch):
    cache = EngineCache(batch=48, budget=4 * GiB)
    monkeypatch.setattr(cache, "_build", lambda spec, batch: _FakeEngine(spec, batch))
    with pytest.raises(MemoryError):
        cache.get(EncodeSpec(3840, 2160))


def test_auto_batch_is_capped_by_the_budget():
    spec = EncodeSpec(3840, 2160, gop=64)
    assert auto_batch(spec) == 24 and auto_batch(spec, 1000 * GiB) == 24
    small = auto_batch(spec, 24 * GiB)
    assert 1 <= small < 24 and engine_bytes(spec, small) <= 12 * GiB
    assert auto_batch(EncodeSpec(1920, 1080, codec="av1"), 1000 * GiB) == 32
    assert auto_batch(EncodeSpec(3840, 2160, codec="av1"), 1000 * GiB) == 16


@pytest.mark.gpu
@pytest.mark.parametrize("w,h,batch,gop,sao,bframes", [(1920, 1080, 48, 64, True, 1), (320, 180, 8, 16, False, 8),
                                                       (3840, 2160, 6, 8, True, 1)])
def test_native_footprint_equals_estimate(w, h, batch, gop, sao, bframes):
    from thinvids_amd.models.gpu_engine import GpuEngine, estimate_footprint

    eng = GpuEngine(width=w, height=h, qp=27, batch=batch, gop=gop, sao=sao, bframes=bframes)
    try:
        assert eng.footprint() == estimate_footprint(w, h, batch, gop, sao, bframes)
    finally:
        eng.close()


@pytest.mark.gpu
def test_8k_ladder_and_4k_av1_engine_fit_together():
    """The shipped 8K HDR10 -> 5-rung ladder shape and a concurrent 4K AV1 engine are
    resident on one MI355X at once, each runs a step, and the budget model accounts for
    what the device actually lost."""
    import torch

    from thinvids_amd.models.abr import AbrLadder
    from thinvids_amd.models.av1_engine import Av1GpuEngine
    from thinvids_amd.worker.encoder import device_budget

    free0, total = torch.cuda.mem_get_info(0)
    lad = AbrLadder(7680, 4320, [2160, 1440, 1080, 720, 480], segments=24, gop=64, device=0)
    av = Av1GpuEngine(3840, 2160, batch=16, qindex=100, device=0)
    try:
        lad.prepare_synthetic([64 * b for b in range(24)], slot=0)
        segs = lad.encode_prepared(24, slot=0)
        assert len(segs) == 5 and all(len(r) == 24 for r in segs)

        def load(t, planes):
            for p in planes:
                p.fill_(100 + t)

        g = av.encode_gop(64, load)
        assert g.sse.shape[:2] == (64, 16)
        torch.cuda.synchronize()
        free1, _ = torch.cuda.mem_get_info(0)
        used = free0 - free1
        model = (sum(e.footprint()["dev"] for e in lad.engines)
                 + engine_bytes(EncodeSpec(3840, 2160, gop=64, codec="av1"), 16))
        assert used < device_budget(0), (used / GiB, device_budget(0) / GiB)
        assert model < used * 1.5, (model / GiB, used / GiB)
    finally:
        av.close()
        lad.close()
