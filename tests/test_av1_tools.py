"""AV1 coding tools: range coder, CDEF, loop restoration.

CPU tests pin the C++ golden model against independent numpy re-implementations of the
filter arithmetic and against the tools' purpose (round trip, compression near entropy,
PSNR gains on real HEVC reconstructions).  GPU tests pin the gfx950 kernels bit-exactly to
the golden model.  Parity with libaom/dav1d is unpinned (no AV1 decoder in the image)."""
import numpy as np
import pytest

from thinvids_amd.ops import av1


def _rec_pair(w=192, h=128, qp=37, t=1):
    from thinvids_amd.models import hevc

    frames = [hevc.synth_frame(3, k, w, h) for k in range(t + 1)]
    bs, _ = hevc.encode_sequence_cpu(frames, qp=qp)
    dec = hevc.decode(bs, coded=False)
    return tuple(np.ascontiguousarray(p) for p in frames[t]), tuple(np.ascontiguousarray(p) for p in dec.frames[t])


# ------------------------------------------------------------------ range coder -------
@pytest.mark.parametrize("adapt", [True, False])
def test_range_coder_roundtrip_random(adapt):
    rng = np.random.default_rng(7)
    for n in (1, 2, 17, 500, 5000):
        alpha = rng.choice([2, 3, 5, 8, 13, 16], n)
        ctx = np.searchsorted([2, 3, 5, 8, 13, 16], alpha)
        sym = np.minimum(alpha - 1, rng.geometric(0.4, n) - 1)
        data, dec = av1.range_coder_roundtrip(sym, alpha, ctx, adapt)
        np.testing.assert_array_equal(dec, sym)


def test_range_coder_compresses_to_entropy():
    rng = np.random.default_rng(1)
    p = np.array([0.7, 0.15, 0.1, 0.05])
    n = 20000
    sym = rng.choice(4, n, p=p)
    data, dec = av1.range_coder_roundtrip(sym, np.full(n, 4), np.zeros(n, int), adapt=True)
    np.testing.assert_array_equal(dec, sym)
    ent = -(p * np.log2(p)).sum() * n / 8
    assert len(data) < 1.03 * ent + 16, (len(data), ent)
    # without adaptation the uniform CDF costs 2 bits / symbol
    data_u, _ = av1.range_coder_roundtrip(sym, np.full(n, 4), np.zeros(n, int), adapt=False)
    assert abs(len(data_u) - n * 2 / 8) < 8


def test_range_coder_rejects_bad_symbols():
    with pytest.raises(ValueError):
        av1.range_coder_roundtrip([4], [4], [0])
    with pytest.raises(ValueError):
        av1.range_coder_roundtrip([0], [17], [0])


# ------------------------------------------------------------------------- CDEF --------
def _np_cdef_dir(block):
    x = block.astype(np.int64) - 128
    part = np.zeros((8, 15), np.int64)
    for i in range(8):
        for j in range(8):
            bins = [i + j, i + j // 2, i, 3 + i - j // 2, 7 + i - j, 3 - i // 2 + j, j, i // 2 + j]
            for d in range(8):
                part[d, bins[d]] += x[i, j]
    div = [0, 840, 420, 280, 210, 168, 140, 120, 105]
    cost = np.zeros(8, np.int64)
    for d in (2, 6):
        cost[d] = (part[d, :8] ** 2).sum() * 105
    for d in (0, 4):
        cost[d] = sum((part[d, i] ** 2 + part[d, 14 - i] ** 2) * div[i + 1] for i in range(7)) + part[d, 7] ** 2 * 105
    for d in (1, 3, 5, 7):
        c = (part[d, 3:8] ** 2).sum() * 105
        c += sum((part[d, j] ** 2 + part[d, 10 - j] ** 2) * div[2 * j + 2] for j in range(3))
        cost[d] = c
    best = int(np.argmax(cost))
    return best, int((cost[best] - cost[(best + 4) & 7]) >> 10)


def test_cdef_directions_match_numpy_and_orientation():
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (32, 48), dtype=np.uint8)
    img[:8, :8] = np.repeat(np.arange(8, dtype=np.uint8)[:, None] * 30, 8, 1)   # rows constant: horizontal
    img[:8, 8:16] = np.repeat(np.arange(8, dtype=np.uint8)[None, :] * 30, 8, 0)  # columns constant: vertical
    d, v = av1.cdef_dirs(img)
    for by in range(4):
        for bx in range(6):
            assert (int(d[by, bx]), int(v[by, bx])) == _np_cdef_dir(img[by * 8:by * 8 + 8, bx * 8:bx * 8 + 8])
    assert d[0, 0] == 2 and d[0, 1] == 6


def _np_cdef_pixel(P, x, y, pri, sec, damping, d):
    dirs = [[(-1, 1), (-2, 2)], [(0, 1), (-1, 2)], [(0, 1), (0, 2)], [(0, 1), (1, 2)],
            [(1, 1), (2, 2)], [(1, 0), (2, 1)], [(1, 0), (2, 0)], [(1, 0), (2, -1)]]
    h, w = P.shape

    def get(dy, dx):
        yy, xx = y + dy, x + dx
        return int(P[yy, xx]) if 0 <= yy < h and 0 <= xx < w else None

    def constrain(diff, t, dmp):
        if not t:
            return 0
        adj = max(0, dmp - (t.bit_length() - 1))
        return int(np.sign(diff)) * min(abs(diff), max(0, t - (abs(diff) >> adj)))

    c = int(P[y, x])
    s, mx, mn = 0, c, c
    for k in range(2):
        pt = [[4, 2], [3, 3]][pri & 1][k]
        st = [2, 1][k]
        for sg in (-1, 1):
            v = get(sg * dirs[d][k][0], sg * dirs[d][k][1])
            if pri and v is not None:
                s += pt * constrain(v - c, pri, damping)
                mx, mn = max(mx, v), min(mn, v)
            for off in (-2, 2):
                if not sec:
                    continue
                v = get(sg * dirs[(d + off) & 7][k][0], sg * dirs[(d + off) & 7][k][1])
                if v is not None:
                    s += st * constrain(v - c, sec, damping)
                    mx, mn = max(mx, v), min(mn, v)
    return min(mx, max(mn, c + ((8 + s - (s < 0)) >> 4)))


def test_cdef_apply_matches_numpy_reference():
    src, rec = _rec_pair(64, 64, qp=40)
    Y = rec[0]
    d, v = av1.cdef_dirs(Y)
    preset = 9 * 4 + 2  # primary 9, secondary 2
    out = av1.cdef_apply(Y, d, v, np.array([preset], np.int8), chroma=False, damping=5)
    for (y, x) in [(0, 0), (5, 7), (31, 33), (63, 63), (40, 2), (17, 50)]:
        var = int(v[y // 8, x // 8])
        i = (var >> 6).bit_length() - 1 if var >> 6 else 0
        pri = (9 * (4 + min(i, 12)) + 8) >> 4 if var else 0
        assert out[y, x] == _np_cdef_pixel(Y, x, y, pri, 2, 5, int(d[y // 8, x // 8])), (y, x)
    # preset 0 (no primary, no secondary) and "off" are the identity
    np.testing.assert_array_equal(av1.cdef_apply(Y, d, v, np.array([0], np.int8), False), Y)
    np.testing.assert_array_equal(av1.cdef_apply(Y, d, v, np.array([-1], np.int8), False), Y)


def test_cdef_search_consistent_with_apply_and_improves_psnr():
    src, rec = _rec_pair(128, 64, qp=40)
    d, v = av1.cdef_dirs(rec[0])
    sse = av1.cdef_search(src[0], rec[0], d, v, chroma=False)
    assert sse.shape == (2, 64)
    for p in (0, 5, 27, 63):
        out = av1.cdef_apply(rec[0], d, v, np.array([p, p], np.int8), chroma=False)
        e = (out.astype(np.int64) - src[0]) ** 2
        assert e[:, :64].sum() == sse[0, p] and e[:, 64:].sum() == sse[1, p]
    # chroma planes use the luma directions of the co-located blocks
    suv = av1.cdef_search(src[1], rec[1], d, v, chroma=True)
    assert suv.shape == (2, 64)
    out, rep = av1.postfilter_frames(src, rec, restore=False)
    assert all(b >= a - 1e-9 for a, b in zip(rep["psnr_in"], rep["psnr_cdef"]))
    assert rep["psnr_cdef"][0] > rep["psnr_in"][0] + 0.05


def test_cdef_select_greedy_table():
    rng = np.random.default_rng(0)
    sy = rng.integers(1000, 2000, (20, 64)).astype(np.float64)
    su = rng.integers(100, 200, (20, 64)).astype(np.float64)
    table, idx, total = av1.cdef_select(sy, su, max_presets=8)
    assert 1 <= len(table) <= 8 and idx.shape == (20,) and idx.max() < len(table)
    one, _, t1 = av1.cdef_select(sy, su, max_presets=1)
    assert total <= t1 and len(one) == 1
    best_single = (sy[:, :, None] + su[:, None, :]).reshape(20, -1).sum(0).min()
    assert t1 == best_single


# ------------------------------------------------------------- loop restoration --------
def _np_wiener_unit(P, coef):
    """Independent numpy Wiener of a whole plane with one set of taps (single unit)."""
    h, w = P.shape
    taps = lambda c: np.array([c[0], c[1], c[2], 128 - 2 * sum(c), c[2], c[1], c[0]], np.int64)
    ht, vt = taps(coef[:3]), taps(coef[3:])
    pad = np.pad(P.astype(np.int64), 3, mode="edge")
    mid = sum(ht[t] * pad[:, t:t + w] for t in range(7))
    mid = np.clip((mid + 4) >> 3, -(1 << 11), (1 << 13) - 1 - (1 << 11))
    out = sum(vt[t] * mid[t:t + h, :] for t in range(7))
    return np.clip((out + (1 << 10)) >> 11, 0, 255).astype(np.uint8)


def test_wiener_apply_matches_numpy_reference():
    src, rec = _rec_pair(64, 64, qp=37)
    for coef in ([3, -7, 15, -2, 5, 20], [10, 8, 46, -5, -23, -17], [0, 0, 0, 1, 0, 0]):
        out = av1.wiener_apply(rec[0], np.array([coef], np.int32))
        np.testing.assert_array_equal(out, _np_wiener_unit(rec[0], coef))
    np.testing.assert_array_equal(av1.wiener_apply(rec[0], np.zeros((1, 6), np.int32)), rec[0])


def test_loop_restoration_search_never_hurts():
    src, rec = _rec_pair(192, 128, qp=40)
    dec = av1.loop_restoration_search(src[0], rec[0], sgr_sets=(0, 6, 10, 14))
    assert dec.kind.shape == (1, 6)
    assert (dec.sse_best <= dec.sse_off).all()
    out = av1.loop_restoration_apply(rec[0], dec)
    e = (out.astype(np.int64) - src[0]) ** 2
    assert e.sum() == pytest.approx(dec.sse_best.sum())
    assert av1.psnr(src[0], out) > av1.psnr(src[0], rec[0])


def test_sgr_filter_smooths_and_projection_identity():
    src, rec = _rec_pair(64, 64, qp=40)
    # w0 = w1 = 0 projects back onto the input exactly
    np.testing.assert_array_equal(av1.sgr_apply(rec[0], np.array([[0, 0, 0]], np.int32)), rec[0])
    np.testing.assert_array_equal(av1.sgr_apply(rec[0], np.array([[-1, 5, 5]], np.int32)), rec[0])
    st = av1.sgr_stats(src[0], rec[0], 0)
    assert st.shape == (1, 5) and st[0, 0] > 0 and st[0, 2] > 0


# ---------------------------------------------------------------------- GPU --------
@pytest.mark.gpu
def test_gpu_av1_tools_bit_exact():
    import torch

    dev = torch.device("cuda", 0)
    pairs = [_rec_pair(192, 128, qp=q, t=1) for q in (32, 40)]
    stack = lambda c: torch.stack([torch.from_numpy(p[k][c]) for p in pairs for k in (0,)]).to(dev)
    S = [torch.stack([torch.from_numpy(p[0][c]) for p in pairs]).to(dev) for c in range(3)]
    R = [torch.stack([torch.from_numpy(p[1][c]) for p in pairs]).to(dev) for c in range(3)]
    del stack
    d, v = av1.cdef_dirs(R[0])
    for b, (s, r) in enumerate(pairs):
        dc, vc = av1.cdef_dirs(r[0])
        np.testing.assert_array_equal(d[b].cpu().numpy(), dc.ravel())
        np.testing.assert_array_equal(v[b].cpu().numpy(), vc.ravel())
        for c, chroma in ((0, False), (1, True)):
            ssg = av1.cdef_search(S[c], R[c], d, v, chroma)[b].cpu().numpy()
            ssc = av1.cdef_search(s[c], r[c], dc, vc, chroma)
            np.testing.assert_array_equal(ssg, ssc.astype(np.int64))
    presets = torch.tensor([[3, 17, -1, 63, 40, 0], [63, 1, 2, 3, 4, 5]], dtype=torch.int8)
    for c, chroma in ((0, False), (2, True)):
        og = av1.cdef_apply(R[c], d, v, presets, chroma).cpu().numpy()
        for b, (s, r) in enumerate(pairs):
            dc, vc = av1.cdef_dirs(r[0])
            np.testing.assert_array_equal(og[b], av1.cdef_apply(r[c], dc, vc, presets[b].numpy(), chroma))
    coef = np.array([[[3, -7, 15, -2, 5, 20]] * 6, [[0] * 6] + [[10, 8, 46, -5, -23, -17]] * 5], np.int32)
    og = av1.wiener_apply(R[0], coef).cpu().numpy()
    other = np.array([[[1, -3, 9]] * 6, [[0, 0, 0]] * 6], np.int32)
    for dirn in (0, 1):
        sg = av1.wiener_stats(S[0], R[0], dirn, other).cpu().numpy()
        for b, (s, r) in enumerate(pairs):
            np.testing.assert_array_equal(sg[b], av1.wiener_stats(s[0], r[0], dirn, other[b]))
    for b, (s, r) in enumerate(pairs):
        np.testing.assert_array_equal(og[b], av1.wiener_apply(r[0], coef[b]))
    prm = np.array([[[0, -20, 40], [-1, 0, 0], [10, 5, -9], [14, 31, 95], [7, -96, -32], [3, 0, 0]]] * 2, np.int32)
    og = av1.sgr_apply(R[0], prm).cpu().numpy()
    for st in (0, 10, 14):
        sg = av1.sgr_stats(S[0], R[0], st).cpu().numpy()
        for b, (s, r) in enumerate(pairs):
            np.testing.assert_array_equal(sg[b], av1.sgr_stats(s[0], r[0], st))
    for b, (s, r) in enumerate(pairs):
        np.testing.assert_array_equal(og[b], av1.sgr_apply(r[0], prm[b]))


@pytest.mark.gpu
def test_gpu_postfilter_equals_cpu():
    import torch

    dev = torch.device("cuda", 0)
    s, r = _rec_pair(192, 128, qp=38)
    S = tuple(torch.from_numpy(p)[None].to(dev) for p in s)
    R = tuple(torch.from_numpy(p)[None].to(dev) for p in r)
    og, rg = av1.postfilter_frames(S, R, sgr_sets=(0, 10, 14))
    oc, rc = av1.postfilter_frames(s, r, sgr_sets=(0, 10, 14))
    for a, b in zip(og, oc):
        np.testing.assert_array_equal(a[0].cpu().numpy(), b)
    assert rg["psnr_lr"] == pytest.approx(rc["psnr_lr"])


# -------------------------------------------------------------------- transforms -------
_TX = [(n, c, r) for n in (4, 8, 16, 32, 64) for c in ("dct", "adst", "flipadst", "idtx")
       for r in ("dct", "adst", "idtx") if not ((c in ("adst", "flipadst") or r == "adst") and n > 16)
       and not ((c == "idtx" or r == "idtx") and n > 32)]


def test_txfm_basis_matches_av1_constants():
    assert list(av1.txfm_basis("adst", 4)[0]) == [1321, 2482, 3344, 3803]  # AV1 sinpi(1..4)
    d8 = av1.txfm_basis("dct", 8)
    assert d8[0, 0] == 2896 and d8[1, 0] == 4017 and d8[2, 0] == 3784  # cospi 32, 4(56), 8(48)
    assert av1.txfm_basis("idtx", 4)[0, 0] == 5793  # NewSqrt2
    for n in (4, 8, 16, 32, 64):  # rows are orthogonal with norm 4096 sqrt(n/2)
        b = av1.txfm_basis("dct", n).astype(np.float64)
        g = b @ b.T / (4096.0 ** 2 * n / 2)
        assert np.abs(g - np.eye(n)).max() < 2e-3


@pytest.mark.parametrize("n,col,row", [t for t in _TX if t[0] <= 32])
def test_txfm_roundtrip(n, col, row):
    rng = np.random.default_rng(n)
    x = rng.integers(-255, 256, (6, n, n)).astype(np.int16)
    c = av1.txfm2d(x, col, row)
    y = av1.txfm2d(c, col, row, inverse=True)
    assert np.abs(y.astype(int) - x).max() <= 1
    # energy compaction: a smooth ramp puts (nearly) everything into few DCT coefficients
    if col == row == "dct":
        ramp = np.add.outer(np.arange(n), np.arange(n)).astype(np.int16)[None] * (200 // (2 * n))
        cc = np.abs(av1.txfm2d(ramp, col, row)[0].astype(np.int64)) ** 2
        assert cc[:2, :2].sum() > 0.95 * cc.sum()


@pytest.mark.gpu
def test_gpu_txfm_bit_exact():
    import torch

    rng = np.random.default_rng(5)
    for n, col, row in _TX:
        x = rng.integers(-255, 256, (9, n, n)).astype(np.int16)
        xg = torch.from_numpy(x).cuda()
        cg = av1.txfm2d(xg, col, row)
        cc = av1.txfm2d(x, col, row)
        np.testing.assert_array_equal(cg.cpu().numpy(), cc, err_msg=f"fwd {n} {col} {row}")
        ig = av1.txfm2d(cg, col, row, inverse=True)
        np.testing.assert_array_equal(ig.cpu().numpy(), av1.txfm2d(cc, col, row, inverse=True),
                                      err_msg=f"inv {n} {col} {row}")
