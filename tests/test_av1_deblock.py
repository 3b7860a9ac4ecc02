"""AV1 deblocking loop filter (SURVEY.md §2.3 K16 ``av1_deblock``; AV1 spec 7.14).

The C++ golden model (csrc/core/av1_tools.cpp ``deblock`` over tv/av1_defs.h) is pinned to an
independent pure-Python model written from the spec's edge rules and libaom's explicit
4/6/8/14-tap formulas (not the generic tap loop the C++ uses).  The fused gfx950 kernel
(k_deblock: both passes per 64x64 LDS tile) is pinned bit-exactly to the golden model.
Parity with libaom/dav1d binaries is unpinned (none in the image)."""
import numpy as np
import pytest

from thinvids_amd.ops import av1


def R(v, n):
    return (v + (1 << (n - 1))) >> n


def s8(v):
    return max(-128, min(127, v))


def _filter_line(px, size, lvl, sharp):
    """px: dict k -> value, k >= 0 q side, k < 0 p side (-1 = p0).  Returns updates."""
    shift = 2 if sharp > 4 else (1 if sharp > 0 else 0)
    limit = lvl >> shift
    limit = max(1, min(9 - sharp, limit)) if sharp > 0 else max(1, limit)
    blimit, thresh = 2 * (lvl + 2) + limit, lvl >> 4
    p = [px.get(-k - 1) for k in range(7)]
    q = [px.get(k) for k in range(7)]
    pairs = {4: 1, 6: 2, 8: 3, 16: 3}[size]
    if abs(p[0] - q[0]) * 2 + abs(p[1] - q[1]) // 2 > blimit:
        return {}
    for k in range(1, pairs + 1):
        if abs(p[k] - p[k - 1]) > limit or abs(q[k] - q[k - 1]) > limit:
            return {}
    flat = size >= 6 and all(abs(p[k] - p[0]) <= 1 and abs(q[k] - q[0]) <= 1 for k in range(1, pairs + 1))
    if not flat:
        hev = abs(p[1] - p[0]) > thresh or abs(q[1] - q[0]) > thresh
        ps1, ps0, qs0, qs1 = p[1] - 128, p[0] - 128, q[0] - 128, q[1] - 128
        f = s8(ps1 - qs1) if hev else 0
        f = s8(f + 3 * (qs0 - ps0))
        f1, f2 = s8(f + 4) >> 3, s8(f + 3) >> 3
        out = {0: s8(qs0 - f1) + 128, -1: s8(ps0 + f2) + 128}
        if not hev:
            f3 = R(f1, 1)
            out[1], out[-2] = s8(qs1 - f3) + 128, s8(ps1 + f3) + 128
        return out
    flat2 = size == 16 and all(abs(p[k] - p[0]) <= 1 and abs(q[k] - q[0]) <= 1 for k in range(4, 7))
    p0, p1, p2, p3, p4, p5, p6 = p
    q0, q1, q2, q3, q4, q5, q6 = q
    if size == 6:
        return {-2: R(p2 * 3 + p1 * 2 + p0 * 2 + q0, 3), -1: R(p2 + p1 * 2 + p0 * 2 + q0 * 2 + q1, 3),
                0: R(p1 + p0 * 2 + q0 * 2 + q1 * 2 + q2, 3), 1: R(p0 + q0 * 2 + q1 * 2 + q2 * 3, 3)}
    if not flat2:
        return {-3: R(3 * p3 + 2 * p2 + p1 + p0 + q0, 3), -2: R(2 * p3 + p2 + 2 * p1 + p0 + q0 + q1, 3),
                -1: R(p3 + p2 + p1 + 2 * p0 + q0 + q1 + q2, 3), 0: R(p2 + p1 + p0 + 2 * q0 + q1 + q2 + q3, 3),
                1: R(p1 + p0 + q0 + 2 * q1 + q2 + 2 * q3, 3), 2: R(p0 + q0 + q1 + 2 * q2 + 3 * q3, 3)}
    return {
        -6: R(p6 * 7 + p5 * 2 + p4 * 2 + p3 + p2 + p1 + p0 + q0, 4),
        -5: R(p6 * 5 + p5 * 2 + p4 * 2 + p3 * 2 + p2 + p1 + p0 + q0 + q1, 4),
        -4: R(p6 * 4 + p5 + p4 * 2 + p3 * 2 + p2 * 2 + p1 + p0 + q0 + q1 + q2, 4),
        -3: R(p6 * 3 + p5 + p4 + p3 * 2 + p2 * 2 + p1 * 2 + p0 + q0 + q1 + q2 + q3, 4),
        -2: R(p6 * 2 + p5 + p4 + p3 + p2 * 2 + p1 * 2 + p0 * 2 + q0 + q1 + q2 + q3 + q4, 4),
        -1: R(p6 + p5 + p4 + p3 + p2 + p1 * 2 + p0 * 2 + q0 * 2 + q1 + q2 + q3 + q4 + q5, 4),
        0: R(p5 + p4 + p3 + p2 + p1 + p0 * 2 + q0 * 2 + q1 * 2 + q2 + q3 + q4 + q5 + q6, 4),
        1: R(p4 + p3 + p2 + p1 + p0 + q0 * 2 + q1 * 2 + q2 * 2 + q3 + q4 + q5 + q6 * 2, 4),
        2: R(p3 + p2 + p1 + p0 + q0 + q1 * 2 + q2 * 2 + q3 * 2 + q4 + q5 + q6 * 3, 4),
        3: R(p2 + p1 + p0 + q0 + q1 + q2 * 2 + q3 * 2 + q4 * 2 + q5 + q6 * 4, 4),
        4: R(p1 + p0 + q0 + q1 + q2 + q3 * 2 + q4 * 2 + q5 * 2 + q6 * 5, 4),
        5: R(p0 + q0 + q1 + q2 + q3 + q4 * 2 + q5 * 2 + q6 * 7, 4),
    }


def _decode_info(word):
    return dict(txw=4 << (word & 7), txh=4 << (word >> 3 & 7), bw=4 << (word >> 6 & 7), bh=4 << (word >> 9 & 7),
                lv=word >> 12 & 63, lh=word >> 18 & 63, sk=word >> 24 & 1)


def deblock_py(plane, info, chroma, sharp=0):
    out = plane.astype(np.int64).copy()
    h, w = plane.shape
    inf = [[_decode_info(int(v)) for v in row] for row in info]
    for pas in (0, 1):
        for y in range(h):
            for x in range(w):
                pos, dim = (x, w) if pas == 0 else (y, h)
                if pos == 0 or pos % 4:
                    continue
                cur = inf[y // 4][x // 4]
                prev = inf[y // 4][x // 4 - 1] if pas == 0 else inf[y // 4 - 1][x // 4]
                ts = cur["txw" if pas == 0 else "txh"]
                if pos % ts:
                    continue
                if cur["sk"] and pos % cur["bw" if pas == 0 else "bh"]:
                    continue
                key = "lv" if pas == 0 else "lh"
                lvl = cur[key] or prev[key]
                if not lvl:
                    continue
                fs = min(ts, prev["txw" if pas == 0 else "txh"])
                if chroma:
                    size = 6 if fs >= 8 and pos >= 3 and pos + 3 <= dim else 4
                elif fs >= 16 and pos >= 7 and pos + 7 <= dim:
                    size = 16
                elif fs >= 8 and pos >= 4 and pos + 4 <= dim:
                    size = 8
                else:
                    size = 4
                n = {4: 2, 6: 3, 8: 4, 16: 7}[size]
                at = (lambda k: (y, x + k)) if pas == 0 else (lambda k: (y + k, x))
                px = {k: int(out[at(k)]) for k in range(-n, n)}
                for k, v in _filter_line(px, size, lvl, sharp).items():
                    out[at(k)] = v
    return out.astype(np.uint8)


def _blocky(w, h, seed=0, bs=8, step=24):
    """Smooth gradient + texture, coarsely quantised per bs x bs DCT block (visible seams)."""
    from scipy.fft import dctn, idctn

    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    img = 128 + 60 * np.sin(xx / 23.0) * np.cos(yy / 17.0) + rng.normal(0, 3, (h, w))
    img[: h // 2, : w // 3] += 25 * (((xx[: h // 2, : w // 3] // 5) + (yy[: h // 2, : w // 3] // 5)) % 2)
    out = np.empty_like(img)
    for y in range(0, h, bs):
        for x in range(0, w, bs):
            c = dctn(img[y:y + bs, x:x + bs], norm="ortho")
            out[y:y + bs, x:x + bs] = idctn(np.round(c / step) * step, norm="ortho")
    return np.clip(np.round(img), 0, 255).astype(np.uint8), np.clip(np.round(out), 0, 255).astype(np.uint8)


@pytest.mark.parametrize("chroma", [False, True])
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_deblock_golden_matches_spec_model(chroma, seed):
    rng = np.random.default_rng(seed)
    w, h = (72, 40) if chroma else (136, 72)
    _, rec = _blocky(w, h, seed, bs=4 if chroma else 8, step=20)
    info = av1.random_lf_info(w, h, rng, chroma=chroma, lvl_max=63)
    for sharp in (0, 3, 6):
        got = av1.deblock(rec, info, chroma, sharp)
        np.testing.assert_array_equal(got, deblock_py(rec, info, chroma, sharp))


def test_deblock_uses_every_filter_length():
    """A plane with 4/8/16 tx grids and flat / textured areas exercises the narrow, 8-tap and
    14-tap paths; each changes pixels only within its reach of an edge."""
    w, h = 192, 64
    _, rec = _blocky(w, h, 3, bs=8, step=28)
    tx = np.zeros((h // 4, w // 4), np.int64)
    tx[:, :16], tx[:, 16:32], tx[:, 32:] = 4, 8, 16
    big = np.full_like(tx, 64)
    info = av1.lf_info(tx, tx, big, big, np.full_like(tx, 40), np.full_like(tx, 40))
    got = av1.deblock(rec, info)
    np.testing.assert_array_equal(got, deblock_py(rec, info, False))
    # vertical edges only (horizontal level 0): each length stays within its reach
    info_v = av1.lf_info(tx, tx, big, big, np.full_like(tx, 40), np.zeros_like(tx))
    diff = av1.deblock(rec, info_v) != rec
    assert diff[:, :64].any() and diff[:, 64:128].any() and diff[:, 128:].any()
    # 8-tap region: the pixel 4 away from an 8-aligned edge is never written
    assert not diff[:, list(range(68, 124, 8))].any()
    # 14-tap region: pixels 6..9 away from 16-aligned edges changed (wide filter used),
    # pixel 8 away never (reach is 6)
    assert diff[:, [c for c in range(134, 186) if c % 16 in (10, 11, 12, 13, 3, 4, 5)]].any()
    assert not diff[:, list(range(136, 186, 16))].any()


def test_deblock_level_zero_and_skip_are_identity():
    w, h = 128, 64
    _, rec = _blocky(w, h, 4)
    z = np.zeros((h // 4, w // 4), np.int64)
    info = av1.lf_info(z + 8, z + 8, z + 64, z + 64, z, z)
    np.testing.assert_array_equal(av1.deblock(rec, info), rec)
    # skip && inter inside one 64x64 block: only the 64-aligned block edges filter
    info = av1.lf_info(z + 8, z + 8, z + 64, z + 64, z + 30, z + 30, z + 1)
    got = av1.deblock(rec, info)
    changed = np.nonzero((got != rec).any(axis=0))[0]
    assert changed.size and np.all(np.abs(changed - 64) <= 4)


def test_deblock_improves_blocky_reconstruction():
    for bs, tx in ((8, 8), (16, 16)):
        src, rec = _blocky(256, 128, 5, bs=bs, step=40)
        z = np.zeros((32, 64), np.int64)
        info = av1.lf_info(z + tx, z + tx, z + 64, z + 64, z + 36, z + 36)
        got = av1.deblock(rec, info)
        assert av1.psnr(src, got) > av1.psnr(src, rec) + 0.2


def test_deblock_rejects_bad_dims():
    with pytest.raises(RuntimeError):
        av1.deblock(np.zeros((10, 16), np.uint8), np.zeros((2, 4), np.uint32))


@pytest.mark.gpu
def test_gpu_deblock_bit_exact():
    import torch

    rng = np.random.default_rng(11)
    for chroma, (w, h), B in ((False, (1920, 1080), 2), (False, (200, 136), 3), (True, (960, 540), 2),
                              (True, (100, 68), 3)):
        planes, infos = [], []
        for b in range(B):
            _, rec = _blocky(w, h, 20 + b, bs=4 if chroma else 8, step=24)
            planes.append(rec)
            infos.append(av1.random_lf_info(w, h, rng, chroma=chroma))
        for sharp in (0, 5):
            got = av1.deblock(torch.as_tensor(np.stack(planes)).cuda(), np.stack(infos), chroma, sharp).cpu().numpy()
            for b in range(B):
                np.testing.assert_array_equal(got[b], av1.deblock(planes[b], infos[b], chroma, sharp))
