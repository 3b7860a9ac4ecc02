"""Independent check of the HEVC (H.265) tables the encoder codes with.

No HEVC decoder is importable here, so the decoder oracle (csrc/core/hevc_decoder.cpp)
shares its grammar and tables with the writer; a transcription error in a shared table
would pass every round trip.  This file is a second transcription, written against the
spec's own layout -- context init values as the ctxIdx tables list them (initType 0, 1, 2
concatenated, Tables 9-5 .. 9-37), the LPS range / transition tables (9-52, 9-53), the
deblocking beta / tC table (8-12), the chroma QP table (8-10), the intra angle tables (8-4,
8-5), the interpolation filters (8-39 / 8-40 equations' coefficient lists), the scan
orders (6.5.3 .. 6.5.5) and the transform matrix (8.6.4.2) -- and shares no header with
csrc/.  The encoder's tables are read back through ``tv_hevc_spec_table``
(csrc/core/hevc_writer.cpp) and diffed here entry by entry.

Generated tables (scans, the DCT matrix, intra filter flags) are rebuilt from the spec's
definitions rather than typed in.
"""
import ctypes as C

import numpy as np
import pytest

CNU = 154  # "context not used" init value

# ---------------------------------------------------------------- context init values
# element -> values for ctxIdx 0.. over initType 0 | 1 | 2 (the spec table's column order)
CTX_INIT = {
    "sao_merge_flag": [153, 153, 153],
    "sao_type_idx": [200, 185, 160],
    "split_cu_flag": [139, 141, 157, 107, 139, 126, 107, 139, 126],
    "cu_transquant_bypass_flag": [154, 154, 154],
    "cu_skip_flag": [CNU, CNU, CNU, 197, 185, 201, 197, 185, 201],  # initType 0 has no skip ctx
    "pred_mode_flag": [CNU, 149, 134],
    "part_mode": [184, 154, 154],  # first bin only (2Nx2N decision) per initType
    "prev_intra_luma_pred_flag": [184, 154, 183],
    "intra_chroma_pred_mode": [63, 152, 152],
    "rqt_root_cbf": [CNU, 79, 79],
    "merge_flag": [CNU, 110, 154],
    "merge_idx": [CNU, 122, 137],
    "inter_pred_idc": [CNU] * 5 + [95, 79, 63, 31, 31] * 2,
    "ref_idx": [CNU, CNU, 153, 153, 153, 153],
    "mvp_flag": [CNU, 168, 168],
    "split_transform_flag": [153, 138, 138, 124, 138, 94, 224, 167, 122],
    "cbf_luma": [111, 141, 153, 111, 153, 111],
    "cbf_chroma": [94, 138, 182, 154, 149, 107, 167, 154, 149, 92, 167, 154],
    "abs_mvd_greater0_flag": [CNU, 140, 169],
    "abs_mvd_greater1_flag": [CNU, 198, 198],
    "cu_qp_delta_abs": [154] * 6,
    "transform_skip_flag": [139] * 6,
    "last_sig_coeff_x_prefix": [
        110, 110, 124, 125, 140, 153, 125, 127, 140, 109, 111, 143, 127, 111, 79, 108, 123, 63,
        125, 110, 94, 110, 95, 79, 125, 111, 110, 78, 110, 111, 111, 95, 94, 108, 123, 108,
        125, 110, 124, 110, 95, 94, 125, 111, 111, 79, 125, 126, 111, 111, 79, 108, 123, 93],
    "coded_sub_block_flag": [91, 171, 134, 141, 121, 140, 61, 154, 121, 140, 61, 154],
    # 42 regular contexts per initType, then the two transform-skip contexts (range extension)
    "sig_coeff_flag": [
        111, 111, 125, 110, 110, 94, 124, 108, 124, 107, 125, 141, 179, 153, 125, 107, 125, 141,
        179, 153, 125, 107, 125, 141, 179, 153, 125, 140, 139, 182, 182, 152, 136, 152, 136, 153,
        136, 139, 111, 136, 139, 111,
        155, 154, 139, 153, 139, 123, 123, 63, 153, 166, 183, 140, 136, 153, 154, 166, 183, 140,
        136, 153, 154, 166, 183, 140, 136, 153, 154, 170, 153, 123, 123, 107, 121, 107, 121, 167,
        151, 183, 140, 151, 183, 140,
        170, 154, 139, 153, 139, 123, 123, 63, 124, 166, 183, 140, 136, 153, 154, 166, 183, 140,
        136, 153, 154, 166, 183, 140, 136, 153, 154, 170, 153, 138, 138, 122, 121, 122, 121, 167,
        151, 183, 140, 151, 183, 140],
    "sig_coeff_flag_transform_skip": [141, 111, 140, 140, 140, 140],
    "coeff_abs_level_greater1_flag": [
        140, 92, 137, 138, 140, 152, 138, 139, 153, 74, 149, 92, 139, 107, 122, 152, 140, 179,
        166, 182, 140, 227, 122, 197,
        154, 196, 196, 167, 154, 152, 167, 182, 182, 134, 149, 136, 153, 121, 136, 122, 169, 208,
        166, 167, 154, 152, 167, 182,
        154, 196, 167, 167, 154, 152, 167, 182, 182, 134, 149, 136, 153, 121, 136, 137, 169, 194,
        166, 167, 154, 167, 137, 182],
    "coeff_abs_level_greater2_flag": [138, 153, 136, 167, 152, 152, 107, 167, 91, 122, 107, 167,
                                      107, 167, 91, 107, 107, 167],
}
CTX_INIT["last_sig_coeff_y_prefix"] = CTX_INIT["last_sig_coeff_x_prefix"]  # same table (9-27)

# --------------------------------------------------------------- arithmetic coder tables
RANGE_TAB_LPS = [
    (128, 176, 208, 240), (128, 167, 197, 227), (128, 158, 187, 216), (123, 150, 178, 205),
    (116, 142, 169, 195), (111, 135, 160, 185), (105, 128, 152, 175), (100, 122, 144, 166),
    (95, 116, 137, 158), (90, 110, 130, 150), (85, 104, 123, 142), (81, 99, 117, 135),
    (77, 94, 111, 128), (73, 89, 105, 122), (69, 85, 100, 116), (66, 80, 95, 110),
    (62, 76, 90, 104), (59, 72, 86, 99), (56, 69, 81, 94), (53, 65, 77, 89),
    (51, 62, 73, 85), (48, 59, 69, 80), (46, 56, 66, 76), (43, 53, 63, 72),
    (41, 50, 59, 69), (39, 48, 56, 65), (37, 45, 54, 62), (35, 43, 51, 59),
    (33, 41, 48, 56), (32, 39, 46, 53), (30, 37, 43, 50), (29, 35, 41, 48),
    (27, 33, 39, 45), (26, 31, 37, 43), (24, 30, 35, 41), (23, 28, 33, 39),
    (22, 27, 32, 37), (21, 26, 30, 35), (20, 24, 29, 33), (19, 23, 27, 31),
    (18, 22, 26, 30), (17, 21, 25, 28), (16, 20, 23, 27), (15, 19, 22, 25),
    (14, 18, 21, 24), (14, 17, 20, 23), (13, 16, 19, 22), (12, 15, 18, 21),
    (12, 14, 17, 20), (11, 14, 16, 19), (11, 13, 15, 18), (10, 12, 15, 17),
    (10, 12, 14, 16), (9, 11, 13, 15), (9, 11, 12, 14), (8, 10, 12, 14),
    (8, 9, 11, 13), (7, 9, 11, 12), (7, 9, 10, 12), (7, 8, 10, 11),
    (6, 8, 9, 11), (6, 7, 9, 10), (6, 7, 8, 9), (2, 2, 2, 2),
]
TRANS_IDX_LPS = [0, 0, 1, 2, 2, 4, 4, 5, 6, 7, 8, 9, 9, 11, 11, 12, 13, 13, 15, 15, 16, 16, 18, 18,
                 19, 19, 21, 21, 22, 22, 23, 24, 24, 25, 26, 26, 27, 27, 28, 29, 29, 30, 30, 30,
                 31, 32, 32, 33, 33, 33, 34, 34, 35, 35, 35, 36, 36, 36, 37, 37, 37, 38, 38, 63]
TRANS_IDX_MPS = [min(i + 1, 62) for i in range(63)] + [63]

# sig_coeff_flag ctxIdxMap for 4x4 TBs (9.3.4.2.5) and last-position prefix grouping
CTX_IDX_MAP = [0, 1, 4, 5, 2, 3, 4, 5, 6, 6, 8, 8, 7, 7, 8, 8]
GROUP_IDX = [0, 1, 2, 3, 4, 4, 5, 5, 6, 6, 6, 6, 7, 7, 7, 7] + [8] * 8 + [9] * 8
MIN_IN_GROUP = [0, 1, 2, 3, 4, 6, 8, 12, 16, 24]

# ------------------------------------------------------------------- quant / deblock
LEVEL_SCALE = [40, 45, 51, 57, 64, 72]
BETA = [0] * 16 + [6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18] + list(range(20, 65, 2))
TC = [0] * 18 + [1] * 9 + [2] * 4 + [3] * 4 + [4] * 3 + [5] * 2 + [6] * 2 + [7, 8, 9, 10, 11, 13, 14, 16, 18, 20, 22, 24]
QPC_30_42 = [29, 30, 31, 32, 33, 33, 34, 34, 35, 35, 36, 36, 37]


def chroma_qp(qpi):
    return qpi if qpi < 30 else (qpi - 6 if qpi > 42 else QPC_30_42[qpi - 30])


# --------------------------------------------------------------------------- intra
ANGLE_2_34 = [32, 26, 21, 17, 13, 9, 5, 2, 0, -2, -5, -9, -13, -17, -21, -26, -32,
              -26, -21, -17, -13, -9, -5, -2, 0, 2, 5, 9, 13, 17, 21, 26, 32]
INTRA_PRED_ANGLE = [0, 0] + ANGLE_2_34
INV_ANGLE_11_25 = [-4096, -1638, -910, -630, -482, -390, -315, -256, -315, -390, -482, -630, -910, -1638, -4096]


def intra_filter_flag(log2n, mode):
    """8.4.4.2.3 filterFlag (no strong smoothing): minDistVerHor > intraHorVerDistThres."""
    if mode == 1 or log2n == 2:  # DC, 4x4
        return 0
    thres = {3: 7, 4: 1, 5: 0}[log2n]
    return int(min(abs(mode - 26), abs(mode - 10)) > thres)


def scan_idx(log2n, mode):
    """7.4.9.11 scanIdx for intra luma 4x4 / 8x8: vertical scan for near-horizontal modes
    6..14, horizontal scan for near-vertical modes 22..30."""
    if 6 <= mode <= 14:
        return 2
    if 22 <= mode <= 30:
        return 1
    return 0


# --------------------------------------------------------------------------- inter
LUMA_FILTER = [[0, 0, 0, 64, 0, 0, 0, 0], [-1, 4, -10, 58, 17, -5, 1, 0], [-1, 4, -11, 40, 40, -11, 4, -1],
               [0, 1, -5, 17, 58, -10, 4, -1]]
CHROMA_FILTER = [[0, 64, 0, 0], [-2, 58, 10, -2], [-4, 54, 16, -2], [-6, 46, 28, -4], [-4, 36, 36, -4],
                 [-4, 28, 46, -6], [-2, 16, 54, -4], [-2, 10, 58, -2]]


# ------------------------------------------------------------------- scans (6.5.3-6.5.5)
def up_right_diagonal(blk):
    """6.5.3: (x, y) of scan positions of a blk x blk block, packed x | y << log2(blk)."""
    out, x, y = [], 0, 0
    sh = blk.bit_length() - 1
    while len(out) < blk * blk:
        while y >= 0:
            if x < blk and y < blk:
                out.append(x | (y << sh))
            y -= 1
            x += 1
        y, x = x, 0
    return out


def horizontal(blk):
    sh = blk.bit_length() - 1
    return [x | (y << sh) for y in range(blk) for x in range(blk)]


def vertical(blk):
    sh = blk.bit_length() - 1
    return [x | (y << sh) for x in range(blk) for y in range(blk)]


# -------------------------------------------------------------- transform (8.6.4.2)
# the 32-point matrix's distinct odd-row magnitudes per size (coefficient list of the spec's
# transMatrix columns 0..15): 4-pt {64, 83, 36}, 8-pt odd {89, 75, 50, 18}, 16-pt odd
# {90, 87, 80, 70, 57, 43, 25, 9}, 32-pt odd {90, 90, 88, 85, 82, 78, 73, 67, 61, 54, 46,
# 38, 31, 22, 13, 4}
ODD32 = [90, 90, 88, 85, 82, 78, 73, 67, 61, 54, 46, 38, 31, 22, 13, 4]
ODD16 = [90, 87, 80, 70, 57, 43, 25, 9]
ODD8 = [89, 75, 50, 18]


def dct32_matrix():
    """transMatrix[k][n], rebuilt from the cosine sign pattern: row k, column n uses the
    magnitude of angle (2n+1)k (units of pi/64) from the row's frequency class."""
    import math

    m = np.zeros((32, 32), np.int64)
    for k in range(32):
        for n in range(32):
            if k == 0:
                m[k, n] = 64
                continue
            a = ((2 * n + 1) * k) % 128
            c = math.cos(math.pi * a / 64)
            tz = (k & -k).bit_length() - 1  # k = odd * 2^tz
            if tz == 4:
                mag = 64
            elif tz == 3:
                mag = [83, 36][0 if abs(c) > 0.7 else 1]
            else:
                lst = {2: ODD8, 1: ODD16, 0: ODD32}[tz]
                # the magnitude index orders |cos| descending within the class
                step = 1 << tz
                idx = [abs(math.cos(math.pi * (2 * j + 1) * step / 64)) for j in range(len(lst))]
                mag = lst[int(np.argmin([abs(abs(c) - v) for v in idx]))]
            m[k, n] = mag if c > 0 else -mag
    return m


# ------------------------------------------------------------------------------ tests
@pytest.fixture(scope="module")
def enc():
    from thinvids_amd._native import core_lib

    lib = core_lib()
    lib.tv_hevc_spec_table.argtypes = [C.c_char_p, C.POINTER(C.c_int), C.c_int]
    lib.tv_hevc_spec_table.restype = C.c_int

    def get(name):
        n = lib.tv_hevc_spec_table(name.encode(), None, 0)
        assert n >= 0, f"encoder does not export {name}"
        buf = (C.c_int * n)()
        lib.tv_hevc_spec_table(name.encode(), buf, n)
        return list(buf)

    return get


def _per_type(vals, n):
    return [vals[t * n:(t + 1) * n] for t in range(3)]


@pytest.mark.parametrize("element", sorted(k for k in CTX_INIT if k != "sig_coeff_flag_transform_skip"))
def test_context_init_values(enc, element):
    spec = CTX_INIT[element]
    got = enc("ctx:" + element)
    if element == "sig_coeff_flag":  # the encoder keeps the 2 transform-skip contexts after the 42
        ts = _per_type(CTX_INIT["sig_coeff_flag_transform_skip"], 2)
        spec = sum((s + t for s, t in zip(_per_type(spec, 42), ts)), [])
    n = len(spec) // 3
    assert len(got) == len(spec), (element, len(got), len(spec))
    for t, (g, s) in enumerate(zip(_per_type(got, n), _per_type(spec, n))):
        # a context the encoder never codes for this initType may hold any value: only the
        # spec's CNU placeholders are exempt
        bad = [i for i, (a, b) in enumerate(zip(g, s)) if a != b and b != CNU]
        assert not bad, f"{element} initType {t}: ctx {bad} encoder {[g[i] for i in bad]} spec {[s[i] for i in bad]}"


def test_arithmetic_coder_tables(enc):
    assert enc("range_tab_lps") == [v for row in RANGE_TAB_LPS for v in row]
    assert enc("trans_idx_lps") == TRANS_IDX_LPS
    assert enc("trans_idx_mps") == TRANS_IDX_MPS


def test_residual_coding_tables(enc):
    assert enc("ctx_idx_map") == CTX_IDX_MAP
    assert enc("group_idx") == GROUP_IDX and enc("min_in_group") == MIN_IN_GROUP
    assert enc("scan_diag4x4") == up_right_diagonal(4)
    assert enc("scan_hor4x4") == horizontal(4) and enc("scan_ver4x4") == vertical(4)
    assert enc("scan_diag8x8") == up_right_diagonal(8)
    assert enc("scan_idx") == [scan_idx(l, m) for l in (2, 3) for m in range(35)]


def test_quant_deblock_chroma_qp_tables(enc):
    assert len(BETA) == 52 and len(TC) == 54
    assert enc("level_scale") == LEVEL_SCALE
    assert enc("beta") == BETA and enc("tc") == TC
    assert enc("chroma_qp") == [chroma_qp(q) for q in range(58)]


def test_intra_tables(enc):
    assert enc("intra_pred_angle") == INTRA_PRED_ANGLE
    assert enc("inv_angle") == INV_ANGLE_11_25
    # invAngle = round(8192 / angle) for the negative angles (8.4.4.2.6)
    assert INV_ANGLE_11_25 == [-round(8192 / -a) for a in ANGLE_2_34[9:24]]
    assert enc("intra_filter") == [intra_filter_flag(l, m) for l in range(2, 6) for m in range(35)]


def test_interpolation_filters(enc):
    assert enc("luma_filter") == sum(LUMA_FILTER, [])
    assert enc("chroma_filter") == sum(CHROMA_FILTER, [])
    assert all(sum(r) == 64 for r in LUMA_FILTER + CHROMA_FILTER)


def test_transform_matrix(enc):
    m = dct32_matrix()
    got = np.array(enc("dct32")).reshape(32, 32)
    assert (got == m).all(), np.argwhere(got != m)[:5].tolist()
    # the first column lists every distinct magnitude once per row class
    assert list(m[:, 0]) == [64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67, 64, 61, 57,
                             54, 50, 46, 43, 38, 36, 31, 25, 22, 18, 13, 9, 4]
