"""Independent check of the HEVC high-level syntax the encoder writes for hierarchical-B and
WPP streams: the writer (csrc/core/hevc_writer.cpp) and the decoder oracle
(csrc/core/hevc_decoder.cpp) share cabac.h / bitstream.h / hevc_codec.h, so a shared
misreading of the specification would pass every round-trip test.  This file parses the
streams with a bit reader written from the H.265 text (7.3.1.1 NAL header, 7.3.2.2 SPS,
7.3.2.3 PPS, 7.3.6.1 slice segment header, 7.3.7 st_ref_pic_set, 8.3.1 POC, C.5.2 DPB
bumping) and an ISO/IEC 14496-12 box walker for the MP4 ``stts`` / ``ctts`` tables; it
imports nothing from csrc/ beyond running the encoder.  Every syntax branch is taken from
the parsed flags (not from what this encoder happens to set), so a header the writer
gets wrong fails here even when the oracle agrees with it.

Parity with a third-party HEVC decoder stays unpinned (none is installed in this image);
this pins the high-level syntax, POC and reference structure, DPB constraints, WPP entry
points and the MP4 timing tables."""
import struct

import numpy as np
import pytest

from thinvids_amd.models import hevc

IDR_W_RADL, IDR_N_LP, BLA_W_LP, RSV_IRAP_23 = 19, 20, 16, 23
VPS, SPS, PPS = 32, 33, 34


# ------------------------------------------------------------------ bit reading --------
def nal_units(annexb: bytes):
    """(nal_unit_type, rbsp bytes, emulation-prevention byte positions in the NAL) per NAL."""
    starts, i = [], 0
    while True:
        j = annexb.find(b"\x00\x00\x01", i)
        if j < 0:
            break
        starts.append(j + 3)
        i = j + 3
    out = []
    for k, s in enumerate(starts):
        e = starts[k + 1] - 3 if k + 1 < len(starts) else len(annexb)
        nal = annexb[s:e]
        while nal and nal[-1] == 0:  # trailing_zero_8bits / the next start code's leading zero
            nal = nal[:-1]
        rbsp, epb, z = bytearray(), [], 0
        for p, byte in enumerate(nal):
            if z >= 2 and byte == 3:
                epb.append(p)
                z = 0
                continue
            rbsp.append(byte)
            z = z + 1 if byte == 0 else 0
        hdr = (nal[0] << 8) | nal[1]
        assert hdr >> 15 == 0, "forbidden_zero_bit"
        assert hdr & 7 == 1, "nuh_temporal_id_plus1"
        out.append(((hdr >> 9) & 63, bytes(rbsp[2:]), epb, len(nal)))
    return out


class Bits:
    def __init__(self, data: bytes):
        self.d, self.p = data, 0

    def u(self, n: int) -> int:
        v = 0
        for _ in range(n):
            v = (v << 1) | ((self.d[self.p >> 3] >> (7 - (self.p & 7))) & 1)
            self.p += 1
        return v

    def ue(self) -> int:
        z = 0
        while self.u(1) == 0:
            z += 1
        return (1 << z) - 1 + self.u(z)

    def se(self) -> int:
        k = self.ue()
        return (k + 1) // 2 if k & 1 else -(k // 2)


def profile_tier_level(b: Bits, max_sub_layers_minus1: int) -> dict:
    r = {"profile_space": b.u(2), "tier": b.u(1), "profile_idc": b.u(5)}
    r["compat"] = b.u(32)
    b.u(4)  # progressive / interlaced / non_packed / frame_only
    b.u(43)
    b.u(1)
    r["level_idc"] = b.u(8)
    sub_p, sub_l = [], []
    for _ in range(max_sub_layers_minus1):
        sub_p.append(b.u(1))
        sub_l.append(b.u(1))
    if max_sub_layers_minus1 > 0:
        for _ in range(max_sub_layers_minus1, 8):
            b.u(2)
    for i in range(max_sub_layers_minus1):
        if sub_p[i]:
            b.u(88)
        if sub_l[i]:
            b.u(8)
    return r


def st_ref_pic_set(b: Bits, idx: int, num_sets: int, sets: list) -> dict:
    """7.3.7 + the 7.4.8 derivation: DeltaPocS0/S1 and UsedByCurrPicS0/S1."""
    inter = b.u(1) if idx != 0 else 0
    if inter:
        delta_idx = b.ue() + 1 if idx == num_sets else 1
        ref = sets[idx - delta_idx]
        sign, absd = b.u(1), b.ue() + 1
        delta_rps = (1 - 2 * sign) * absd
        n_ref = len(ref["s0"]) + len(ref["s1"])
        used, use_delta = [], []
        for _ in range(n_ref + 1):
            u = b.u(1)
            used.append(u)
            use_delta.append(1 if u else b.u(1))
        # (7-61) / (7-62)
        s0, s1 = [], []
        for j in range(len(ref["s1"]) - 1, -1, -1):
            d = ref["s1"][j][0] + delta_rps
            if d < 0 and use_delta[len(ref["s0"]) + j]:
                s0.append((d, used[len(ref["s0"]) + j]))
        if delta_rps < 0 and use_delta[n_ref]:
            s0.append((delta_rps, used[n_ref]))
        for j in range(len(ref["s0"])):
            d = ref["s0"][j][0] + delta_rps
            if d < 0 and use_delta[j]:
                s0.append((d, used[j]))
        for j in range(len(ref["s0"]) - 1, -1, -1):
            d = ref["s0"][j][0] + delta_rps
            if d > 0 and use_delta[j]:
                s1.append((d, used[j]))
        if delta_rps > 0 and use_delta[n_ref]:
            s1.append((delta_rps, used[n_ref]))
        for j in range(len(ref["s1"])):
            d = ref["s1"][j][0] + delta_rps
            if d > 0 and use_delta[len(ref["s0"]) + j]:
                s1.append((d, used[len(ref["s0"]) + j]))
        return {"s0": s0, "s1": s1}
    nneg, npos = b.ue(), b.ue()
    s0, s1, prev = [], [], 0
    for _ in range(nneg):
        prev -= b.ue() + 1
        s0.append((prev, b.u(1)))
    prev = 0
    for _ in range(npos):
        prev += b.ue() + 1
        s1.append((prev, b.u(1)))
    return {"s0": s0, "s1": s1}


def parse_sps(rbsp: bytes) -> dict:
    b = Bits(rbsp)
    b.u(4)  # sps_video_parameter_set_id
    msl = b.u(3)
    b.u(1)
    s = {"ptl": profile_tier_level(b, msl)}
    s["id"] = b.ue()
    s["chroma_format_idc"] = b.ue()
    if s["chroma_format_idc"] == 3:
        b.u(1)
    s["w"], s["h"] = b.ue(), b.ue()
    s["conf"] = [b.ue() for _ in range(4)] if b.u(1) else [0, 0, 0, 0]
    s["bd_y"], s["bd_c"] = b.ue() + 8, b.ue() + 8
    s["poc_lsb_bits"] = b.ue() + 4
    sub = b.u(1)
    s["dpb"], s["reorder"] = [], []
    for _ in range(0 if sub else msl, msl + 1):
        s["dpb"].append(b.ue() + 1)
        s["reorder"].append(b.ue())
        b.ue()
    s["min_cb"] = b.ue() + 3
    s["ctb"] = s["min_cb"] + b.ue()
    s["min_tb"] = b.ue() + 2
    s["max_tb"] = s["min_tb"] + b.ue()
    b.ue()
    b.ue()
    if b.u(1):  # scaling_list_enabled_flag
        assert b.u(1) == 0, "sps_scaling_list_data not exercised by this parser"
    s["amp"], s["sao"], pcm = b.u(1), b.u(1), b.u(1)
    assert pcm == 0
    n = b.ue()
    sets = []
    for i in range(n):
        sets.append(st_ref_pic_set(b, i, n, sets))
    s["st_rps"] = sets
    s["long_term"] = b.u(1)
    assert s["long_term"] == 0
    s["tmvp"] = b.u(1)
    s["strong_intra"] = b.u(1)
    return s


def parse_pps(rbsp: bytes) -> dict:
    b = Bits(rbsp)
    p = {"id": b.ue(), "sps": b.ue(), "dep_slices": b.u(1), "output_flag": b.u(1), "extra_bits": b.u(3),
         "sdh": b.u(1), "cabac_init_present": b.u(1), "l0_default": b.ue() + 1, "l1_default": b.ue() + 1,
         "init_qp": 26 + b.se(), "cip": b.u(1), "ts": b.u(1)}
    p["cu_qp_delta"] = b.u(1)
    if p["cu_qp_delta"]:
        b.ue()
    p["cb_off"], p["cr_off"] = b.se(), b.se()
    p["slice_chroma_offsets"], p["wp"], p["wbp"], p["tqb"] = b.u(1), b.u(1), b.u(1), b.u(1)
    p["tiles"], p["wpp"] = b.u(1), b.u(1)
    assert p["tiles"] == 0
    p["lf_across_slices"] = b.u(1)
    p["dbk_override_enabled"], p["dbk_disabled"] = 0, 0
    if b.u(1):  # deblocking_filter_control_present_flag
        p["dbk_override_enabled"] = b.u(1)
        p["dbk_disabled"] = b.u(1)
        if not p["dbk_disabled"]:
            b.se()
            b.se()
    assert b.u(1) == 0  # pps_scaling_list_data_present_flag
    p["lists_mod"] = b.u(1)
    b.ue()
    p["sh_ext"] = b.u(1)
    return p


def parse_slice(nut: int, rbsp: bytes, sps: dict, pps: dict) -> dict:
    b = Bits(rbsp)
    sh = {"first": b.u(1)}
    if BLA_W_LP <= nut <= RSV_IRAP_23:
        b.u(1)
    sh["pps"] = b.ue()
    assert sh["first"], "one slice per picture"
    for _ in range(pps["extra_bits"]):
        b.u(1)
    sh["type"] = b.ue()  # 0 B, 1 P, 2 I
    if pps["output_flag"]:
        b.u(1)
    sh["rps"] = {"s0": [], "s1": []}
    sh["tmvp"] = 0
    if nut not in (IDR_W_RADL, IDR_N_LP):
        sh["poc_lsb"] = b.u(sps["poc_lsb_bits"])
        if not b.u(1):  # short_term_ref_pic_set_sps_flag
            n = len(sps["st_rps"])
            sh["rps"] = st_ref_pic_set(b, n, n, sps["st_rps"])
        else:
            n = len(sps["st_rps"])
            idx = b.u(max(1, (n - 1).bit_length())) if n > 1 else 0
            sh["rps"] = sps["st_rps"][idx]
        if sps["tmvp"]:
            sh["tmvp"] = b.u(1)
    sao_l = sao_c = 0
    if sps["sao"]:
        sao_l = b.u(1)
        sao_c = b.u(1) if sps["chroma_format_idc"] else 0
    sh["sao"] = (sao_l, sao_c)
    if sh["type"] in (0, 1):
        n0, n1 = pps["l0_default"], pps["l1_default"]
        if b.u(1):  # num_ref_idx_active_override_flag
            n0 = b.ue() + 1
            if sh["type"] == 0:
                n1 = b.ue() + 1
        sh["n_ref"] = (n0, n1 if sh["type"] == 0 else 0)
        num_total = sum(u for _, u in sh["rps"]["s0"]) + sum(u for _, u in sh["rps"]["s1"])
        assert not (pps["lists_mod"] and num_total > 1), "list modification not exercised"
        if sh["type"] == 0:
            sh["mvd_l1_zero"] = b.u(1)
        if pps["cabac_init_present"]:
            b.u(1)
        if sh["tmvp"]:
            col_l0 = b.u(1) if sh["type"] == 0 else 1
            if (col_l0 and n0 > 1) or (not col_l0 and n1 > 1):
                b.ue()
        assert not ((pps["wp"] and sh["type"] == 1) or (pps["wbp"] and sh["type"] == 0))
        sh["max_merge"] = 5 - b.ue()
    sh["qp"] = pps["init_qp"] + b.se()
    if pps["slice_chroma_offsets"]:
        b.se()
        b.se()
    dbk_disabled = pps["dbk_disabled"]
    if pps["dbk_override_enabled"] and b.u(1):
        dbk_disabled = b.u(1)
        if not dbk_disabled:
            b.se()
            b.se()
    if pps["lf_across_slices"] and (sao_l or sao_c or not dbk_disabled):
        b.u(1)
    sh["entry_points"] = []
    if pps["tiles"] or pps["wpp"]:
        n = b.ue()
        if n:
            bits = b.ue() + 1
            sh["entry_points"] = [b.u(bits) + 1 for _ in range(n)]
    if pps["sh_ext"]:
        for _ in range(b.ue()):
            b.u(8)
    assert b.u(1) == 1  # byte_alignment(): alignment_bit_equal_to_one
    while b.p & 7:
        assert b.u(1) == 0
    sh["data_rbsp_offset"] = b.p >> 3
    return sh


def decode_structure(annexb: bytes) -> tuple[dict, dict, list]:
    """SPS, PPS and per picture (decoding order): nal type, slice header, POC (8.3.1)."""
    sps = pps = None
    pics, prev_tid0 = [], 0
    for nut, rbsp, epb, nal_len in nal_units(annexb):
        if nut == SPS:
            sps = parse_sps(rbsp)
        elif nut == PPS:
            pps = parse_pps(rbsp)
        elif nut < 32:
            sh = parse_slice(nut, rbsp, sps, pps)
            if nut in (IDR_W_RADL, IDR_N_LP):
                poc = 0
            else:
                mx = 1 << sps["poc_lsb_bits"]
                lsb, plsb, pmsb = sh["poc_lsb"], prev_tid0 % mx, prev_tid0 - prev_tid0 % mx
                if lsb < plsb and plsb - lsb >= mx // 2:
                    msb = pmsb + mx
                elif lsb > plsb and lsb - plsb > mx // 2:
                    msb = pmsb - mx
                else:
                    msb = pmsb
                poc = msb + lsb
            if nut not in (0, 2, 4, 6, 8, 10, 12, 14) or nut >= 16:  # not a sub-layer non-reference picture
                prev_tid0 = poc
            # slice data size in NAL bytes (emulation prevention included, 7.4.7.1): the NAL
            # index at which the header's RBSP bytes (NAL header + slice header) are used up
            want, seen, pos, eps = 2 + sh["data_rbsp_offset"], 0, 0, set(epb)
            while seen < want:
                if pos not in eps:
                    seen += 1
                pos += 1
            hdr_nal = pos
            pics.append({"nut": nut, "sh": sh, "poc": poc, "data_bytes": nal_len - hdr_nal})
    return sps, pps, pics


# ------------------------------------------------------------------------ tests --------
@pytest.fixture(scope="module")
def b4_stream():
    w, h, n = 128, 96, 12
    frames = [hevc.synth_frame(6, t, w, h) for t in range(n)]
    data, _ = hevc.encode_sequence_cpu(frames, qp=30, gop=n, bframes=4, sao=True, search_range=16, wpp=True)
    return data, w, h, n


def test_parameter_sets_parse_from_the_spec(b4_stream):
    data, w, h, n = b4_stream
    sps, pps, pics = decode_structure(data)
    assert sps["ptl"]["profile_idc"] == 1 and sps["chroma_format_idc"] == 1  # Main, 4:2:0
    cw, ch = hevc.coded_size(w, h)
    assert (sps["w"], sps["h"]) == (cw, ch) and sps["bd_y"] == sps["bd_c"] == 8
    assert sps["w"] - 2 * (sps["conf"][0] + sps["conf"][1]) == w and sps["h"] - 2 * (sps["conf"][2] + sps["conf"][3]) == h
    assert sps["sao"] == 1 and sps["ctb"] == 5 and pps["wpp"] == 1
    assert len(pics) == n


def test_poc_order_and_reference_sets_follow_the_gop_plan(b4_stream):
    """Decoding order / POC / slice types equal tv/gop.h's plan; every reference a picture
    uses is in its RPS as used_by_curr, and every RPS entry is a picture still in the DPB."""
    data, w, h, n = b4_stream
    sps, pps, pics = decode_structure(data)
    plan = hevc.gop_plan(n, 4)
    assert [p["poc"] for p in pics] == plan["disp"]
    assert [p["sh"]["type"] for p in pics] == plan["type"]
    decoded = set()
    for k, p in enumerate(pics):
        rps = p["sh"]["rps"]
        entries = [(p["poc"] + d, u) for d, u in rps["s0"] + rps["s1"]]
        for poc, _ in entries:
            assert poc in decoded, f"picture {p['poc']}: RPS names {poc}, never decoded"
        used = {poc for poc, u in entries if u}
        refs = {plan["ref0"][k], plan["ref1"][k]} - {-1}
        assert refs <= used, (p["poc"], refs, used)
        if p["sh"]["type"] == 1:
            assert len(rps["s1"]) == 0 or not any(u for _, u in rps["s1"])
        # references not in the RPS are dropped (marked unused) before decoding this picture
        decoded = {poc for poc, _ in entries} | {p["poc"]}
        assert len(decoded) <= sps["dpb"][-1], "DPB overflow"


def test_dpb_bumping_respects_num_reorder(b4_stream):
    """C.5.2.2 'bumping': with sps_max_num_reorder_pics and the DPB size the stream
    declares, pictures come out in POC order without exceeding either."""
    data, *_ = b4_stream
    sps, pps, pics = decode_structure(data)
    reorder, dpb_size = sps["reorder"][-1], sps["dpb"][-1]
    waiting, out = [], []
    for p in pics:
        waiting.append(p["poc"])
        while len(waiting) > reorder:
            m = min(waiting)
            waiting.remove(m)
            out.append(m)
        assert len(waiting) <= dpb_size
    out += sorted(waiting)
    assert out == sorted(out) == list(range(len(pics)))


def test_wpp_entry_points_cover_the_slice_data(b4_stream):
    """entropy_coding_sync: one entry point per CTB row after the first, and the substream
    sizes add up to the slice data (NAL bytes incl. emulation prevention, 7.4.7.1)."""
    data, w, h, n = b4_stream
    sps, pps, pics = decode_structure(data)
    rows = -(-sps["h"] // (1 << sps["ctb"]))
    for p in pics:
        eps = p["sh"]["entry_points"]
        assert len(eps) == rows - 1
        assert sum(eps) < p["data_bytes"]  # the last substream holds the rest


def _boxes(data: bytes, start: int, end: int):
    i = start
    while i + 8 <= end:
        size, typ = struct.unpack(">I4s", data[i:i + 8])
        hdr = 8
        if size == 1:
            size, hdr = struct.unpack(">Q", data[i + 8:i + 16])[0], 16
        elif size == 0:
            size = end - i
        yield typ.decode("latin1"), i + hdr, i + size
        i += size


def _find(data: bytes, path: list, start: int = 0, end: int | None = None):
    end = len(data) if end is None else end
    for typ, s, e in _boxes(data, start, end):
        if typ == path[0]:
            if len(path) == 1:
                return s, e
            return _find(data, path[1:], s, e)
    return None


def test_mp4_ctts_orders_samples_by_poc(b4_stream):
    """ISO/IEC 14496-12 stts + ctts (version 1, signed offsets allowed): composition times
    of the decode-order samples put them in POC order at one frame duration apart, and the
    first presented sample starts at the edit list's media time (or 0)."""
    data, w, h, n = b4_stream
    mp4 = hevc.mux_mp4(data, w, h, 30, 1)
    stbl = _find(mp4, ["moov", "trak", "mdia", "minf", "stbl"])
    assert stbl is not None
    stts = _find(mp4, ["stts"], *stbl)
    ctts = _find(mp4, ["ctts"], *stbl)
    assert stts is not None and ctts is not None, "B-frame MP4 needs ctts"
    s, _ = stts
    cnt = struct.unpack(">I", mp4[s + 4:s + 8])[0]
    dts, t = [], 0
    for k in range(cnt):
        c, d = struct.unpack(">II", mp4[s + 8 + 8 * k:s + 16 + 8 * k])
        for _ in range(c):
            dts.append(t)
            t += d
    dur = dts[1] - dts[0]
    s, _ = ctts
    ver = mp4[s]
    cnt = struct.unpack(">I", mp4[s + 4:s + 8])[0]
    offs = []
    for k in range(cnt):
        c, o = struct.unpack(">I" + ("i" if ver else "I"), mp4[s + 8 + 8 * k:s + 16 + 8 * k])
        offs += [o] * c
    assert len(offs) == len(dts) == n
    cts = np.array(dts) + np.array(offs)
    _, _, pics = decode_structure(data)
    order = np.argsort(cts, kind="stable")
    assert [pics[i]["poc"] for i in order] == list(range(n))
    assert np.all(np.diff(np.sort(cts)) == dur)
    elst = _find(mp4, ["moov", "trak", "edts", "elst"])
    media_time = 0
    if elst is not None:
        s, _ = elst
        ver = mp4[s]
        media_time = struct.unpack(">q" if ver else ">i", mp4[s + 8 + (8 if ver else 4):s + 8 + (16 if ver else 8)])[0]
    assert int(np.min(cts)) == media_time
