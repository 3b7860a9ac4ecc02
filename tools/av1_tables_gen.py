"""Generate csrc/include/tv/av1_tables.h: the AV1 specification's constant tables the
encoder needs (8-bit Dc_Qlookup / Ac_Qlookup and the default CDFs of every symbol the
encoder codes), read out of the AV1 reference implementations that ship in this image.

This container has no network and no copy of the AV1 specification text, but Pillow's
AVIF plugin bundles libavif, which statically links libaom 3.13.2 (encoder) and dav1d
1.5.3 (decoder).  Both carry the specification's default CDFs in their read-only data:

* libaom lays every CDF out as CDF_SIZE(n) = n + 1 uint16 words: the n - 1 inverse-CDF
  values (32768 - cdf), the terminal 0 and the adaptation counter 0, padded to the array's
  CDF_SIZE(max symbols) -- so a table is found by the byte pattern of its first entries
  and read with a fixed stride;
* dav1d keeps the same inverse-CDF values with its own padding; tables libaom's encoder
  image lacks are read from dav1d's copy (stride measured between the first two CDFs).

Every table read from one library is checked against the other when both hold it.  Only
numbers are extracted (nothing is executed); the output is a plain C++ header committed to
the repository, so the build never needs Pillow.  Run: ``python tools/av1_tables_gen.py``.
"""
from __future__ import annotations

import glob
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "csrc", "include", "tv", "av1_tables.h")


def _blob() -> bytes:
    import PIL

    p = sorted(glob.glob(os.path.join(os.path.dirname(os.path.dirname(PIL.__file__)), "pillow.libs", "libavif*.so*")))
    if not p:
        sys.exit("libavif (Pillow AVIF plugin) not found")
    return open(p[0], "rb").read()


B = _blob()


def find(words) -> list:
    pat = np.asarray(words, dtype="<u2").tobytes()
    out, i = [], B.find(pat)
    while i >= 0:
        if i % 2 == 0:
            out.append(i)
        i = B.find(pat, i + 1)
    return out


def u16(off: int, n: int) -> list:
    return np.frombuffer(B[off:off + 2 * n], dtype="<u2").tolist()


def icdf(vals) -> list:
    return [32768 - v for v in vals]


def aom_table(name, first, count, stride, nsym, second=None, first_hit=False):
    """libaom layout: CDF k at base + 2*stride*k; nsym(k) symbols."""
    n0 = nsym(0) if callable(nsym) else nsym
    pat = icdf(first) + ([0, 0] if len(first) == n0 - 1 else [])
    if second is not None:
        for nxt in (second if isinstance(second[0], list) else [second]):
            pat = pat + [0] * (stride - len(pat) % stride if len(pat) % stride else 0) + icdf(nxt)
    def plausible(base):
        for k in range(count):
            n = nsym(k) if callable(nsym) else nsym
            w = u16(base + 2 * stride * k, stride)
            if w[n - 1:n + 1] != [0, 0] or any(v == 0 for v in w[:n - 1]):
                return False
        return True

    hits = [h for h in find(pat) if plausible(h)]
    if not hits:
        raise SystemExit(f"{name}: no match for the libaom layout")
    # identical layouts in both libraries (e.g. CDF_SIZE(7) == dav1d's [8]) must agree
    if first_hit:  # periodic table (identical rows per q context): the lowest match is its start
        hits = hits[:1]
    reads = [[u16(h + 2 * stride * k, stride) for k in range(count)] for h in hits]
    if any(r != reads[0] for r in reads[1:]):
        raise SystemExit(f"{name}: {len(hits)} differing matches for the libaom layout")
    base = hits[0]
    rows = []
    for k in range(count):
        n = nsym(k) if callable(nsym) else nsym
        w = u16(base + 2 * stride * k, stride)
        vals, term = w[:n - 1], w[n - 1:n + 1]
        if term != [0, 0] or any(v == 0 for v in vals) or vals != sorted(vals, reverse=True):
            raise SystemExit(f"{name}[{k}]: not an inverse CDF of {n} symbols: {w}")
        rows.append(icdf(vals))
    return rows


def dav1d_table(name, first, second, count, nsym):
    """dav1d layout: locate the first two CDFs (icdf values then the counter), derive the
    stride from their distance."""
    n = nsym
    if count == 1:
        hits = find(icdf(first) + [0])
        if not hits:
            raise SystemExit(f"{name}: not in dav1d's tables")
        return [list(first)]
    a = find(icdf(first) + [0])
    b = find(icdf(second) + [0])
    cands = [(x, y - x) for x in a for y in b if 0 < y - x <= 64 and (y - x) % 2 == 0]
    if not cands:
        raise SystemExit(f"{name}: no dav1d candidates")
    reads = []
    for base, step in cands:
        rows = []
        for k in range(count):
            w = u16(base + step * k, n)
            vals = w[:n - 1]
            if w[n - 1] != 0 or any(v == 0 for v in vals):
                raise SystemExit(f"{name}[{k}]: not a dav1d inverse CDF: {w}")
            rows.append(icdf(vals))
        reads.append(rows)
    if any(r != reads[0] for r in reads[1:]):
        raise SystemExit(f"{name}: {len(cands)} differing dav1d candidates")
    return reads[0]


def in_dav1d(name, rows, n):
    """Cross-check: the first two CDFs of a libaom table also appear in dav1d's copy."""
    for r in rows[:2]:
        if not find(icdf(r) + [0]) and n > 2:
            raise SystemExit(f"{name}: entry {r} not found in dav1d's tables")


T = {}
# ---- quantizer lookup (8-bit)
dcq = find([4, 8, 8, 9, 10, 11, 12, 12, 13, 14, 15, 16, 17, 18, 19, 19, 20])
acq = find([4, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22, 23])
if len(dcq) != 1 or len(acq) != 1:
    raise SystemExit("q lookup tables not unique")
DCQ, ACQ = u16(dcq[0], 256), u16(acq[0], 256)
assert DCQ[255] == 1336 and ACQ[255] == 1828 and DCQ == sorted(DCQ) and ACQ == sorted(ACQ)

# ---- mode info (libaom entropymode.c layouts)
T["kf_y_mode"] = ((5, 5), 13, aom_table("kf_y_mode", [15588, 17027, 19338, 20218, 20682, 21110, 21825, 23244, 24189,
                                                      28165, 29093, 30466], 25, 14, 13))
T["y_mode"] = ((4,), 13, aom_table("y_mode", [22801, 23489, 24293, 24756, 25601, 26123, 26606, 27418], 4, 14, 13))
uv0 = aom_table("uv_mode_cfl_not_allowed", [22631, 24152, 25378, 25661, 25986, 26520, 27055, 27923], 13, 15, 13)
uv1 = aom_table("uv_mode_cfl_allowed", [10407, 11208, 12900, 13181, 13823, 14175, 14899, 15656], 13, 15, 14)
T["uv_mode0"] = ((13,), 13, uv0)
T["uv_mode1"] = ((13,), 14, uv1)
T["angle_delta"] = ((8,), 7, aom_table("angle_delta", [2180, 5032, 7567, 22776, 26989, 30217], 8, 8, 7))
part = aom_table("partition", [19132, 25510, 30392], 20, 11, lambda k: 4 if k < 4 else (10 if k < 16 else 8))
T["partition"] = ((20,), 10, part)
# intra_ext_tx [set 0..2][txSzSqr 4][mode 13], CDF_SIZE(16) = 17; set 0 is all zero
s1 = aom_table("intra_ext_tx_set1", [1535, 8035, 9461, 12751, 23467, 27825], 52, 17, 7)
s2base = find(icdf([1535, 8035, 9461, 12751, 23467, 27825]) + [0, 0])[0] + 2 * 17 * 52
s2 = []
for k in range(52):
    w = u16(s2base + 34 * k, 17)
    assert w[4:6] == [0, 0] and all(w[:4]), w
    s2.append(icdf(w[:4]))
T["intra_tx_set1"] = ((4, 13), 7, s1)
T["intra_tx_set2"] = ((4, 13), 5, s2)
# inter_ext_tx [set 0..3][4], CDF_SIZE(16)
i1 = aom_table("inter_ext_tx_set1", [4458, 5560, 7695, 9709, 13330, 14789, 17537, 20266, 21504, 22848, 23934, 25474,
                                     27727, 28915, 30631], 4, 17, 16)
ibase = find(icdf([4458, 5560, 7695, 9709, 13330, 14789, 17537, 20266]))[0]
i2 = [icdf(u16(ibase + 34 * (4 + k), 17)[:11]) for k in range(4)]
i3 = [icdf(u16(ibase + 34 * (8 + k), 17)[:1]) for k in range(4)]
for k in range(4):
    assert u16(ibase + 34 * (4 + k), 17)[11:13] == [0, 0] and u16(ibase + 34 * (8 + k), 17)[1:3] == [0, 0]
T["inter_tx_set1"] = ((4,), 16, i1)
T["inter_tx_set2"] = ((4,), 12, i2)
T["inter_tx_set3"] = ((4,), 2, i3)
T["newmv"] = ((6,), 2, aom_table("newmv", [24035], 6, 3, 2, second=[16630]))
T["refmv"] = ((6,), 2, aom_table("refmv", [23974], 6, 3, 2, second=[24188]))
T["single_ref"] = ((3, 6), 2, aom_table("single_ref", [4897], 18, 3, 2, second=[1555]))
T["txfm_split"] = ((21,), 2, aom_table("txfm_partition", [28581], 21, 3, 2, second=[23846]))
tx0 = aom_table("tx_size_cat0", [19968], 3, 4, 2, second=[19968])
tx1 = aom_table("tx_size_cat1", [12272, 30172], 9, 4, 3, second=[12272, 30172])
T["tx_size_cat0"] = ((3,), 2, tx0)
T["tx_size_cat123"] = ((3, 3), 3, tx1)
T["filter_intra"] = ((22,), 2, aom_table("filter_intra", [4621], 22, 3, 2, second=[6743]))
# dav1d-only small tables
T["skip"] = ((3,), 2, dav1d_table("skip", [31671], [16515], 3, 2))
T["intra_inter"] = ((4,), 2, dav1d_table("intra_inter", [806], [16662], 4, 2))
T["zeromv"] = ((2,), 2, dav1d_table("zeromv", [2175], [1054], 2, 2))
T["drl"] = ((3,), 2, dav1d_table("drl", [13104], [24560], 3, 2))
# motion vectors (libaom entropymv.c default_nmv_context; dav1d holds the same values)
T["mv_joint"] = ((), 4, dav1d_table("mv_joint", [4096, 11264, 19328], [4096, 11264, 19328], 1, 4))
T["mv_class"] = ((), 11, dav1d_table("mv_class", [28672, 30976, 31858, 32320, 32551, 32656, 32740, 32757, 32762,
                                                 32767], [28672, 30976, 31858, 32320, 32551, 32656, 32740, 32757,
                                                          32762, 32767], 1, 11))
T["mv_class0_fr"] = ((2,), 4, dav1d_table("mv_class0_fr", [16384, 24576, 26624], [12288, 21248, 24128], 2, 4))
T["mv_class0_bit"] = ((), 2, dav1d_table("mv_class0_bit", [27648], [27648], 1, 2))
T["mv_bits"] = ((10,), 2, dav1d_table("mv_bits", [17408], [17920], 10, 2))
T["mv_fr"] = ((), 4, dav1d_table("mv_fr", [8192, 17408, 21248], [8192, 17408, 21248], 1, 4))
# restoration (dav1d: restore_switchable CDF3, wiener / sgrproj CDF2)
T["restore_switchable"] = ((), 3, dav1d_table("restore_switchable", [9413, 22581], [9413, 22581], 1, 3))
T["use_wiener"] = ((), 2, dav1d_table("use_wiener", [11570], [11570], 1, 2))
T["use_sgrproj"] = ((), 2, dav1d_table("use_sgrproj", [16855], [16855], 1, 2))

# ---- coefficients (libaom token_cdfs.h), [qctx 4][txSz 5][ptype 2][ctx]
T["txb_skip"] = ((4, 5, 13), 2, aom_table("txb_skip", [31849], 260, 3, 2, second=[5892]))
T["eob_extra"] = ((4, 5, 2, 9), 2, aom_table("eob_extra", [16961], 360, 3, 2, second=[17223]))
T["dc_sign"] = ((4, 2, 3), 2, aom_table("dc_sign", [16000], 24, 3, 2, second=[[13056], [18816], [15232], [12928]], first_hit=True))
for nm, n, first in (("eob_pt_16", 5, [840, 1039, 1980, 4895]),
                     ("eob_pt_32", 6, [400, 520, 977, 2102, 6542]),
                     ("eob_pt_64", 7, [329, 498, 1101, 1784, 3265, 7758]),
                     ("eob_pt_128", 8, [219, 482, 1140, 2091, 3680, 6028, 12586]),
                     ("eob_pt_256", 9, [310, 584, 1887, 3589, 6168, 8611, 11352, 15652]),
                     ("eob_pt_512", 10, [641, 983, 3707, 5430, 10234, 14958, 18788, 23412, 26061]),
                     ("eob_pt_1024", 11, [393, 421, 751, 1623, 3160, 6352, 13345, 18047, 22571, 25830])):
    T[nm] = ((4, 2, 2), n, aom_table(nm, first, 16, n + 1, n))
T["coeff_base_eob"] = ((4, 5, 2, 4), 3, aom_table("coeff_base_eob", [17837, 29055], 160, 4, 3))
T["coeff_base"] = ((4, 5, 2, 42), 4, aom_table("coeff_base", [4034, 8930, 12727], 1680, 5, 4))
brbase = find(icdf([4034, 8930, 12727]) + [0, 0])[0] + 2 * 5 * 1680
br = []
for k in range(840):
    w = u16(brbase + 10 * k, 5)
    assert w[3:5] == [0, 0] and w[:3] == sorted(w[:3], reverse=True), (k, w)
    br.append(icdf(w[:3]))
T["coeff_br"] = ((4, 5, 2, 21), 4, br)

for nm, (dims, n, rows) in T.items():
    if nm not in ("skip", "intra_inter", "zeromv", "drl") and not nm.startswith(("mv_", "restore", "use_")):
        in_dav1d(nm, [r for r in rows if r and any(r)], n)


def emit() -> str:
    L = ["// av1_tables.h — GENERATED by tools/av1_tables_gen.py; do not edit.",
         "// Constant tables of the AV1 specification used by the encoder (8-bit), read out of the",
         "// libaom 3.13.2 / dav1d 1.5.3 reference implementations bundled with this image's libavif",
         "// (see the generator's docstring).  CDFs are listed as the n - 1 cumulative values",
         "// 32768 * P(X <= i) of each n-symbol distribution (the specification's Default_*_Cdf rows",
         "// without the trailing 32768 and counter); av1_codec.cpp converts them to inverse CDFs.",
         "#pragma once", "#include <cstdint>", "", "namespace tv {", "namespace av1 {", "namespace tab {", ""]

    def arr(name, typ, vals, per=16):
        s = [f"constexpr {typ} {name}[{len(vals)}] = {{"]
        for i in range(0, len(vals), per):
            s.append("    " + ", ".join(str(v) for v in vals[i:i + per]) + ",")
        s.append("};")
        return s

    L += arr("kDcQLookup", "int16_t", DCQ) + arr("kAcQLookup", "int16_t", ACQ) + [""]
    for nm, (dims, n, rows) in T.items():
        width = n - 1
        flat = []
        for r in rows:
            flat += list(r) + [0] * (width - len(r))
        shape = "".join(f"[{d}]" for d in dims)
        cname = "k" + "".join(p.capitalize() for p in nm.split("_"))
        L.append(f"// {nm}: {n}-symbol CDFs{'' if dims else ''} {list(dims)}")
        body = [", ".join(str(v) for v in flat[i:i + width]) for i in range(0, len(flat), width)]
        L.append(f"constexpr uint16_t {cname}{shape}[{width}] = {{")
        for i in range(0, len(body), 4):  # flat list: brace elision fills the array
            L.append("    " + ", ".join(body[i:i + 4]) + ",")
        L.append("};")
        L.append("")
    L += ["}  // namespace tab", "}  // namespace av1", "}  // namespace tv", ""]
    return "\n".join(L)


open(OUT, "w").write(emit())
print("wrote", OUT, "tables:", len(T))
