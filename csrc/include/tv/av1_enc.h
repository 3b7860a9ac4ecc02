// av1_enc.h — AV1 encoder primitives shared (TV_HD) by the C++ golden encoder / decoder
// oracle (csrc/core/av1_codec.cpp) and the gfx950 encode kernels (csrc/gpu/k_av1_enc.hip),
// so GPU and CPU reconstructions are identical bit for bit (BASELINE
// config #4 "4K60 AV1 with CDEF + loop-restoration HIP kernels").
//
// Coding structure (a GPU-friendly subset of AV1 Main, 8-bit 4:2:0):
//   * 64x64 superblocks, coded size padded to a multiple of 16 (render_size = display size);
//     every superblock splits to 16x16 coding blocks (PARTITION_SPLIT / split_or_* at edges);
//   * TX_MODE_LARGEST: one 16x16 luma and two 8x8 chroma transforms per block, reduced_tx_set;
//   * key frames: intra modes DC / V / H / SMOOTH / SMOOTH_V / SMOOTH_H / PAETH searched (D113 /
//     D135 / D157 predicted and decodable too); all read no above-right / below-left samples,
//     so the I-frame wavefront is a plain diagonal; angle delta 0; intra edge filter / filter
//     intra / CfL / palette off;
//   * inter frames: one reference (LAST = previous frame), quarter-pel motion, EIGHTTAP
//     (regular) filters; the NEWMV / NEARESTMV / NEARMV / GLOBALMV choice is made by the
//     syntax writer from the spatial MV stack (the mode does not change the reconstruction);
//   * deblocking with frame levels, CDEF (8 presets per frame, 64x64 cdef_idx).
//
// Every normative table (q lookup, default CDFs) is the specification's (tv/av1_tables.h)
// and the inverse transforms are the specification's (tv/av1_itx.h): streams decode with
// any conformant AV1 decoder (tests/test_av1_conformance.py decodes them with dav1d).
#pragma once
#include <cstdint>

#include "tv/av1_tables.h"
#include "tv/hevc_defs.h"  // TV_HD, clip3, tv_abs

namespace tv {
namespace av1 {

constexpr int kBlk = 16;   // coding block (luma)
constexpr int kCBlk = 8;   // chroma block
constexpr int kSb = 64;    // superblock
constexpr int kMaxPresets = 8;

// intra modes (AV1 numbering)
enum : int { DC_PRED = 0, V_PRED = 1, H_PRED = 2, D135_PRED = 4, D113_PRED = 5, D157_PRED = 6, SMOOTH_PRED = 9,
             SMOOTH_V_PRED = 10, SMOOTH_H_PRED = 11, PAETH_PRED = 12 };
// inter modes (YModes of inter blocks)
enum : int { NEARESTMV = 13, NEARMV = 14, GLOBALMV = 15, NEWMV = 16 };
// Mode search candidates.  D113 / D135 / D157 are predicted exactly (intra_dir_px; dav1d
// decodes them bit-exactly) but the SATD-driven search picked them where they cost more than
// they saved: key-frame-only clips at QP 27 +1.0 % bytes at -0.09 dB even with a 10-bit mode
// penalty (profiles/README.md, round 4), so the search keeps the seven non-directional-delta
// modes until it gets a rate-aware decision.
constexpr int kNumIntraCand = 7;
TV_HD int intra_cand(int i) {
  constexpr int8_t m[kNumIntraCand] = {DC_PRED, V_PRED, H_PRED, SMOOTH_PRED, SMOOTH_V_PRED, SMOOTH_H_PRED, PAETH_PRED};
  return m[i];
}
// 1-D transform types (av1_txfm.h: 0 DCT, 1 ADST) of the chroma intra transform
// (Mode_To_Txfm: V -> ADST_DCT, H -> DCT_ADST, SMOOTH / PAETH -> ADST_ADST, ...): vertical
// (column) type in bit 0, horizontal (row) type in bit 1.
TV_HD int uv_txtype(int uv_mode) {
  switch (uv_mode) {
    case V_PRED: case D113_PRED: case SMOOTH_V_PRED: return 1;      // ADST_DCT
    case H_PRED: case D157_PRED: case SMOOTH_H_PRED: return 2;      // DCT_ADST
    case D135_PRED: case SMOOTH_PRED: case PAETH_PRED: return 3;    // ADST_ADST
    default: return 0;                                      // DCT_DCT
  }
}

// ---------------------------------------------------------------- quantizer ------------
// Dc_Qlookup / Ac_Qlookup (8-bit) of the specification (tv/av1_tables.h)
TV_HD int ac_q(int q) { return tab::kAcQLookup[clip3(0, 255, q)]; }
TV_HD int dc_q(int q) { return tab::kDcQLookup[clip3(0, 255, q)]; }
// encoder quantisation rounding (1/128 of the step): 1/3 for intra blocks; inter frames
// choose per frame (inter_rounding).  With the refined motion field a clean source leaves a
// small, coherent residual that is worth keeping (1/3: -2.3 % BD-rate against 1/6 on the
// smooth bench content), while sensor grain is not (1/6: -5.5 % on the textured variant).
// The frame's mean luma SATD per pixel at its final MVs tells them apart: 1.8-3.5 on the
// smooth content, 6.3-10 on the textured one at QP 22..37 (tools/rd_curve.py --codec av1).
constexpr int kRndIntra = 43, kRndInter = 43, kRndInterNoisy = 21;
constexpr int kNoisySatdPerPx = 5;
TV_HD int inter_rounding(long long satd_sum, int W, int H) {
  return satd_sum > (long long)kNoisySatdPerPx * W * H ? kRndInterNoisy : kRndInter;
}
TV_HD int quant(int c, int q, int rnd) {
  const int a = c < 0 ? -c : c;
  const int l = (a + ((q * rnd) >> 7)) / q;
  return c < 0 ? -l : l;
}
// AV1 dequantisation (7.12.3, dqDenom 0 for <= 16x16): |l * q| & 0xFFFFFF, clamp to int16
TV_HD int dequant(int l, int q) {
  if (!l) return 0;
  const long long a = ((long long)(l < 0 ? -l : l) * q) & 0xFFFFFF;
  const int v = (int)(l < 0 ? -a : a);
  return clip3(-32768, 32767, v);
}
// frame loop-filter level from the AC step (libaom-style linear guess), 0..63
TV_HD int lf_level_for_q(int q) {
  const long long v = ((long long)ac_q(q) * 20723 + 1015158) >> 18;
  return (int)clip3(0LL, 63LL, v);
}
// lambda for SAD/SATD-domain decisions (bits -> distortion units, x16)
TV_HD int lambda16(int q) { return tv_max(16, (ac_q(q) * 16 * 3) / 32); }

// Coefficient scan (zigzag over anti-diagonals, odd diagonals top-down): raster position of
// scan index k for N x N, written to out[0..N*N).  The syntax writer's scan and the order
// of the GPU's eob-truncated level packing (k_av1e_tb_pack).
TV_HD void zigzag_scan(int N, int16_t* out) {
  int k = 0;
  for (int s = 0; s <= 2 * N - 2; ++s) {
    const int lo = s - N + 1 > 0 ? s - N + 1 : 0, hi = s < N - 1 ? s : N - 1;
    if (s & 1)
      for (int r = lo; r <= hi; ++r) out[k++] = (int16_t)(r * N + (s - r));
    else
      for (int r = hi; r >= lo; --r) out[k++] = (int16_t)(r * N + (s - r));
  }
}

// ------------------------------------------------------------------ intra prediction ----
// Smooth weights (Sm_Weights_Tx_*)
TV_HD int sm_weight(int N, int i) {
  constexpr uint8_t w8[8] = {255, 197, 146, 105, 73, 50, 37, 32};
  constexpr uint8_t w16[16] = {255, 225, 196, 170, 145, 123, 102, 84, 68, 54, 43, 33, 26, 20, 17, 16};
  return N == 8 ? w8[i] : w16[i];
}

// Edge samples of an N x N block at (x, y) of a plane (7.11.2 without the intra edge
// filter): above[0..N-1], left[0..N-1], top-left.  get(x, y) reads reconstructed samples.
struct IntraEdge {
  int above[16], left[16], tl;
  bool have_a, have_l;
};
template <class G>
TV_HD void intra_edges(G get, int x, int y, int N, IntraEdge& e) {
  e.have_a = y > 0;
  e.have_l = x > 0;
  for (int i = 0; i < N; ++i) {
    if (e.have_a) e.above[i] = get(x + i, y - 1);
    else if (e.have_l) e.above[i] = get(x - 1, y);
    else e.above[i] = 127;
    if (e.have_l) e.left[i] = get(x - 1, y + i);
    else if (e.have_a) e.left[i] = get(x, y - 1);
    else e.left[i] = 129;
  }
  if (e.have_a && e.have_l) e.tl = get(x - 1, y - 1);
  else if (e.have_a) e.tl = get(x, y - 1);
  else if (e.have_l) e.tl = get(x - 1, y);
  else e.tl = 128;
}

TV_HD int intra_dc(const IntraEdge& e, int N) {
  const int lg = N == 8 ? 3 : 4;
  int s = 0;
  if (e.have_a && e.have_l) {
    for (int i = 0; i < N; ++i) s += e.above[i] + e.left[i];
    return (s + N) >> (lg + 1);
  }
  if (e.have_a) {
    for (int i = 0; i < N; ++i) s += e.above[i];
    return (s + (N >> 1)) >> lg;
  }
  if (e.have_l) {
    for (int i = 0; i < N; ++i) s += e.left[i];
    return (s + (N >> 1)) >> lg;
  }
  return 128;
}

// Directional prediction for 90 < pAngle < 180 (7.11.2.4; no edge filter, no upsampling):
// the above row at x = j - (i + 1) * dx / 64 while that lands at or right of the corner
// (index -1 = top-left), else the left column at y = i - (j + 1) * dy / 64; linear
// interpolation in 1/32 steps.  dx = Dr_Intra_Derivative[180 - pAngle], dy = [pAngle - 90].
// Every read is inside above[-1 .. N-1] / left[-1 .. N-1]: no above-right, no below-left.
TV_HD int intra_dir_px(const IntraEdge& e, int i, int j, int dx, int dy) {
  int idx = (j << 6) - (i + 1) * dx;
  int base = idx >> 6;
  if (base >= -1) {
    const int shift = (idx >> 1) & 0x1f;
    const int a0 = base < 0 ? e.tl : e.above[base], a1 = e.above[base + 1];
    return (a0 * (32 - shift) + a1 * shift + 16) >> 5;
  }
  idx = (i << 6) - (j + 1) * dy;
  base = idx >> 6;
  const int shift = (idx >> 1) & 0x1f;
  const int l0 = base < 0 ? e.tl : e.left[base], l1 = e.left[base + 1];
  return (l0 * (32 - shift) + l1 * shift + 16) >> 5;
}

// predicted sample (row i, col j); dc = intra_dc(e, N) precomputed for DC_PRED
TV_HD int intra_pred_px(int mode, const IntraEdge& e, int N, int i, int j, int dc) {
  switch (mode) {
    case D113_PRED: return intra_dir_px(e, i, j, 27, 151);  // Dr_Intra_Derivative[67], [23]
    case D135_PRED: return intra_dir_px(e, i, j, 64, 64);   // [45], [45]
    case D157_PRED: return intra_dir_px(e, i, j, 151, 27);  // [23], [67]
    case V_PRED: return e.above[j];
    case H_PRED: return e.left[i];
    case SMOOTH_PRED: {
      const int wy = sm_weight(N, i), wx = sm_weight(N, j);
      const int s = wy * e.above[j] + (256 - wy) * e.left[N - 1] + wx * e.left[i] + (256 - wx) * e.above[N - 1];
      return (s + 256) >> 9;
    }
    case SMOOTH_V_PRED: {
      const int wy = sm_weight(N, i);
      return (wy * e.above[j] + (256 - wy) * e.left[N - 1] + 128) >> 8;
    }
    case SMOOTH_H_PRED: {
      const int wx = sm_weight(N, j);
      return (wx * e.left[i] + (256 - wx) * e.above[N - 1] + 128) >> 8;
    }
    case PAETH_PRED: {
      const int base = e.above[j] + e.left[i] - e.tl;
      const int pl = tv_abs(base - e.left[i]), pa = tv_abs(base - e.above[j]), pt = tv_abs(base - e.tl);
      if (pl <= pa && pl <= pt) return e.left[i];
      if (pa <= pt) return e.above[j];
      return e.tl;
    }
    default: return dc;
  }
}

// ------------------------------------------------------------------ inter prediction ----
// EIGHTTAP (regular) sub-pixel filters, 1/16 positions.
TV_HD int subpel_tap(int f, int t) {
  constexpr int16_t k[16][8] = {
      {0, 0, 0, 128, 0, 0, 0, 0},      {0, 2, -6, 126, 8, -2, 0, 0},    {0, 2, -10, 122, 18, -4, 0, 0},
      {0, 2, -12, 116, 28, -8, 2, 0},  {0, 2, -14, 110, 38, -10, 2, 0}, {0, 2, -14, 102, 48, -12, 2, 0},
      {0, 2, -16, 94, 58, -12, 2, 0},  {0, 2, -14, 84, 66, -12, 2, 0},  {0, 2, -14, 76, 76, -14, 2, 0},
      {0, 2, -12, 66, 84, -14, 2, 0},  {0, 2, -12, 58, 94, -16, 2, 0},  {0, 2, -12, 48, 102, -14, 2, 0},
      {0, 2, -10, 38, 110, -14, 2, 0}, {0, 2, -8, 28, 116, -12, 2, 0},  {0, 0, -4, 18, 122, -10, 2, 0},
      {0, 0, -2, 8, 126, -6, 2, 0}};
  return k[f][t];
}
constexpr int kInterRound0 = 3, kInterRound1 = 11;

// Predicted sample at integer position (x, y) of a block displaced by (ix + fx/16, iy +
// fy/16); get(x, y) reads the reference with coordinates clamped to the plane (7.11.3.3).
template <class G>
TV_HD int inter_pred_px(G get, int x, int y, int fx, int fy) {
  if (!fx && !fy) return get(x, y);
  int col[8];
  for (int r = 0; r < 8; ++r) {
    int s = 0;
    for (int t = 0; t < 8; ++t) s += subpel_tap(fx, t) * get(x + t - 3, y + r - 3);
    col[r] = (s + (1 << (kInterRound0 - 1))) >> kInterRound0;
  }
  int s = 0;
  for (int t = 0; t < 8; ++t) s += subpel_tap(fy, t) * col[t];
  return clip_pixel((s + (1 << (kInterRound1 - 1))) >> kInterRound1);
}
// Motion vectors are (row, col) in 1/8 luma samples, always even (quarter-pel, no hp).
// Luma: integer mv >> 3, phase (mv & 7) * 2; chroma (4:2:0): integer mv >> 4, phase mv & 15.
TV_HD int mv_int(int mv, bool chroma) { return chroma ? (mv >> 4) : (mv >> 3); }
TV_HD int mv_frac(int mv, bool chroma) { return chroma ? (mv & 15) : ((mv & 7) << 1); }

// ------------------------------------------------------------------------- costs --------
// 4x4 Hadamard SATD of a difference block d[16] (row-major)
TV_HD int satd4(const int* d) {
  int m[16];
  for (int i = 0; i < 4; ++i) {
    const int a0 = d[i * 4] + d[i * 4 + 3], a1 = d[i * 4 + 1] + d[i * 4 + 2];
    const int a2 = d[i * 4 + 1] - d[i * 4 + 2], a3 = d[i * 4] - d[i * 4 + 3];
    m[i * 4] = a0 + a1;
    m[i * 4 + 1] = a3 + a2;
    m[i * 4 + 2] = a0 - a1;
    m[i * 4 + 3] = a3 - a2;
  }
  int s = 0;
  for (int j = 0; j < 4; ++j) {
    const int a0 = m[j] + m[12 + j], a1 = m[4 + j] + m[8 + j];
    const int a2 = m[4 + j] - m[8 + j], a3 = m[j] - m[12 + j];
    s += tv_abs(a0 + a1) + tv_abs(a3 + a2) + tv_abs(a0 - a1) + tv_abs(a3 - a2);
  }
  return (s + 1) >> 1;
}
// approximate bits of one MV component difference (1/8 units, even)
TV_HD int mv_comp_bits(int d) {
  int a = (d < 0 ? -d : d) >> 1;  // quarter-pel units
  if (!a) return 1;
  int b = 0;
  while (a) {
    ++b;
    a >>= 1;
  }
  return 2 * b + 2;
}
// approximate mode bits of the key-frame intra candidates (x16)
TV_HD int intra_mode_bits16(int m) {
  switch (m) {
    case DC_PRED: return 32;
    case V_PRED: case H_PRED: return 48;
    case SMOOTH_PRED: return 40;
    case PAETH_PRED: return 48;
    default: return 56;
  }
}

// CDEF presets the encoder evaluates (preset = pri * 4 + sec_idx): luma primary strengths
// {0,1,2,3,5,7,10,13} x secondary {0, 2}; chroma {0,2,4,7} x {0, 2} (a libaom-style fast
// strength subset: 16 / 8 of the 64 presets, 4x / 8x less CDEF search work).
constexpr uint64_t cdef_mask(const int* pri, int npri, const int* sec, int nsec) {
  uint64_t m = 0;
  for (int i = 0; i < npri; ++i)
    for (int j = 0; j < nsec; ++j) m |= 1ull << (pri[i] * 4 + sec[j]);
  return m;
}
constexpr int kCdefPriY[8] = {0, 1, 2, 3, 5, 7, 10, 13}, kCdefPriUV[4] = {0, 2, 4, 7}, kCdefSec[2] = {0, 2};
constexpr uint64_t kCdefMaskY = cdef_mask(kCdefPriY, 8, kCdefSec, 2);
constexpr uint64_t kCdefMaskUV = cdef_mask(kCdefPriUV, 4, kCdefSec, 2);

// ---------------------------------------------------------------- loop restoration ------
// Self-guided restoration (SGRPROJ) per 64x64 unit of each plane: candidate parameter sets
// (Sgr_Params rows), projection weights by an integer least-squares solve, unit on/off by
// SSE + rate.  xqd ranges / reference mid of the AV1 syntax (Sgrproj_Xqd_Min/Max/Mid).
constexpr int kNumLrSets = 2;
TV_HD int lr_set(int i) { return i == 0 ? 4 : 10; }
constexpr int kXqdMin0 = -96, kXqdMax0 = 31, kXqdMin1 = -32, kXqdMax1 = 95, kXqdMid0 = -32, kXqdMid1 = 31;
TV_HD int bitlen64(unsigned long long v) {
  int n = 0;
  while (v) {
    ++n;
    v >>= 1;
  }
  return n;
}
TV_HD long long div_round(long long n, long long d) { return n >= 0 ? (n + d / 2) / d : -((-n + d / 2) / d); }
// Coded weights (xqd0, xqd1) of a unit from its sgr_stats (H00 H01 H11 c0 c1: normal
// equations of the weights a, b of F0 - u and F1 - u, 1/128 units).  The decoder applies
// a to F0, 128 - xqd0 - xqd1 to F1 and xqd1 to u (sgr_project_xqd), so xqd0 = a and
// xqd1 = 128 - a - b, each clamped to its coded range (one weight clamped, the other
// re-solved given it); radius-0 passes get the syntax's implied values.  Stats are scaled
// below 2^30 so the 2x2 Cramer solve stays in 64 bits.
TV_HD void sgr_solve(const long long* st, int r0, int r1, int* xqd0, int* xqd1) {
  unsigned long long m = 0;
  for (int i = 0; i < 5; ++i) {
    const unsigned long long a = (unsigned long long)(st[i] < 0 ? -st[i] : st[i]);
    m = a > m ? a : m;
  }
  const int sh = tv_max(0, bitlen64(m) - 30);
  const long long H00 = (st[0] >> sh) + 1, H01 = st[1] >> sh, H11 = (st[2] >> sh) + 1, c0 = st[3] >> sh,
                  c1 = st[4] >> sh;
  long long a = 0, b = 0;
  if (r0 && r1) {
    const long long det = H00 * H11 - H01 * H01;
    if (det > 0) {
      a = div_round(c0 * H11 - c1 * H01, det);
      b = div_round(H00 * c1 - H01 * c0, det);
    }
    if (a < kXqdMin0 || a > kXqdMax0) {
      a = clip3((long long)kXqdMin0, (long long)kXqdMax0, a);
      b = div_round(c1 - H01 * a, H11);
    } else if (b < 128 - kXqdMax1 - a || b > 128 - kXqdMin1 - a) {
      b = clip3(128 - kXqdMax1 - a, 128 - kXqdMin1 - a, b);
      a = clip3((long long)kXqdMin0, (long long)kXqdMax0, div_round(c0 - H01 * b, H00));
    }
    *xqd0 = (int)a;
    *xqd1 = (int)clip3((long long)kXqdMin1, (long long)kXqdMax1, 128 - a - b);
  } else if (r0) {
    *xqd0 = (int)clip3((long long)kXqdMin0, (long long)kXqdMax0, div_round(c0, H00));
    *xqd1 = clip3(kXqdMin1, kXqdMax1, 128 - *xqd0);
  } else {
    *xqd0 = 0;
    *xqd1 = (int)clip3((long long)kXqdMin1, (long long)kXqdMax1, 128 - div_round(c1, H11));
  }
}
// rate of a restored unit (~16 bits) in SSE units
TV_HD long long lr_rate_cost(int q) {
  const long long a = ac_q(q);
  return ((a * a * 9) >> 10) * 16;
}

// ------------------------------------------------------------------ motion search -------
// Full-pel search of +-kMeRange around the co-located block on a 2-pel grid (17 x 17), then
// the 8 full-pel neighbours of the best grid point, then 8 half-pel and 8 quarter-pel
// refinements (SAD / SATD + lambda * mv bits, first minimum wins at every stage).
constexpr int kMeRange = 16;
constexpr int kMeGrid = kMeRange + 1;  // grid points per axis (step 2)
constexpr int kMeSide = 2 * kMeRange + 1;
TV_HD int me_cand_dx(int k) { return 2 * (k % kMeGrid) - kMeRange; }
TV_HD int me_cand_dy(int k) { return 2 * (k / kMeGrid) - kMeRange; }
TV_HD int me_ring_dx(int k) { constexpr int8_t t[8] = {-1, 0, 1, -1, 1, -1, 0, 1}; return t[k]; }
TV_HD int me_ring_dy(int k) { constexpr int8_t t[8] = {-1, -1, -1, 0, 0, 1, 1, 1}; return t[k]; }

// Motion-field refinement (inter frames): after the per-block search, kMvRefineRounds
// Jacobi rounds in which every 16x16 block re-chooses, by luma SATD alone (first minimum
// wins, its own MV first), among the current MVs of its neighbours.  The field becomes
// coherent (the writer codes most blocks as NEARESTMV / NEARMV, and skip blocks merge)
// and the search's local minima are escaped: on the bench content -31 % BD-rate against
// the independent per-block search (tools/rd_curve.py --codec av1, profiles/README.md).
constexpr int kMvRefineRounds = 3;
constexpr int kMvRefineMaxCand = 11;
// candidate list of block (bx, by) from the current field `cur` (bw x bh blocks):
// own, left, above, above-right, right, below, zero, then the distance-2 neighbours
// (left, above, right, below); duplicates dropped.  Returns the count.
TV_HD int mv_refine_cands(const uint32_t* cur, int bw, int bh, int bx, int by, uint32_t* out) {
  const int b = by * bw + bx;
  uint32_t c[kMvRefineMaxCand];
  int n = 0;
  c[n++] = cur[b];
  if (bx) c[n++] = cur[b - 1];
  if (by) c[n++] = cur[b - bw];
  if (by && bx + 1 < bw) c[n++] = cur[b - bw + 1];
  if (bx + 1 < bw) c[n++] = cur[b + 1];
  if (by + 1 < bh) c[n++] = cur[b + bw];
  c[n++] = 0u;
  if (bx > 1) c[n++] = cur[b - 2];
  if (by > 1) c[n++] = cur[b - 2 * bw];
  if (bx + 2 < bw) c[n++] = cur[b + 2];
  if (by + 2 < bh) c[n++] = cur[b + 2 * bw];
  int m = 0;
  for (int i = 0; i < n; ++i) {
    bool dup = false;
    for (int j = 0; j < m; ++j) dup |= out[j] == c[i];
    if (!dup) out[m++] = c[i];
  }
  return m;
}

// MV unification after the refinement: a complete 32x32 quad (blocks k = 0..3 in raster
// order, sat[k][c] = SATD of block k at member c's MV) takes the member MV of least total
// SATD when that is at most kQuadUnifyBits' worth (lambda) above its blocks' own MVs; then
// a complete 64x64 superblock likewise takes one of its quads' (top-left block) MVs
// (own = its 16 blocks at their MVs, tot[c] = at quad c's).  Same-MV skip blocks merge into
// 32x32 / 64x64 blocks: -5 % BD-rate on the bench content (tools/rd_curve.py --codec av1).
constexpr int kQuadUnifyBits = 6, kSbUnifyBits = 16;
TV_HD int quad_unify(const int (*sat)[4], int lam) {
  const int own = sat[0][0] + sat[1][1] + sat[2][2] + sat[3][3];
  int bc = 1 << 30, bi = 0;
  for (int c = 0; c < 4; ++c) {
    const int t = sat[0][c] + sat[1][c] + sat[2][c] + sat[3][c];
    if (t < bc) bc = t, bi = c;
  }
  return bc <= own + ((lam * kQuadUnifyBits) >> 4) ? bi : -1;
}
TV_HD int sb_unify(int own, const int* tot, int lam) {
  int bc = tot[0], bi = 0;
  for (int c = 1; c < 4; ++c)
    if (tot[c] < bc) bc = tot[c], bi = c;
  return bc <= own + ((lam * kSbUnifyBits) >> 4) ? bi : -1;
}

// ------------------------------------------------------------------ per-block record ----
// One 32-bit word per 16x16 block: bit 0 inter, 1-4 y mode, 5-8 uv mode, 9 skip (no
// nonzero level in any plane), 10-12 nonzero mask (Y, U, V); mv word: row (low 16, signed)
// and col (high 16).
TV_HD uint32_t pack_mode(int inter, int ym, int uvm, int skip, int nzmask) {
  return (uint32_t)(inter & 1) | ((uint32_t)(ym & 15) << 1) | ((uint32_t)(uvm & 15) << 5) |
         ((uint32_t)(skip & 1) << 9) | ((uint32_t)(nzmask & 7) << 10);
}
TV_HD int mode_inter(uint32_t m) { return m & 1; }
TV_HD int mode_y(uint32_t m) { return (m >> 1) & 15; }
TV_HD int mode_uv(uint32_t m) { return (m >> 5) & 15; }
TV_HD int mode_skip(uint32_t m) { return (m >> 9) & 1; }
TV_HD int mode_nz(uint32_t m) { return (m >> 10) & 7; }
// bits 13-14: size of the (merged) block covering this 16x16 cell: 0 = 16x16, 1 = 32x32, 2 = 64x64
TV_HD int mode_bsz(uint32_t m) { return (m >> 13) & 3; }
TV_HD uint32_t with_bsz(uint32_t m, int s) { return (m & ~(3u << 13)) | ((uint32_t)(s & 3) << 13); }

// Skip-block merging of inter frames (one 64x64 superblock at sb (sx, sy)): a fully inside
// 32x32 quad whose four 16x16 blocks are all inter + skip with one motion vector becomes one
// 32x32 block; four such quads with one motion vector become one 64x64 block.  Prediction is
// unchanged (same MV), only the block size seen by the syntax and the deblocking differs.
TV_HD void merge_sb(uint32_t* mode, const uint32_t* mv, int bw, int bh, int sx, int sy) {
  bool q_ok[4];
  int nq = 0;
  for (int q = 0; q < 4; ++q) {
    const int qx = sx * 4 + (q & 1) * 2, qy = sy * 4 + (q >> 1) * 2;
    bool ok = qx + 1 < bw && qy + 1 < bh;
    if (ok) {
      const uint32_t v0 = mv[qy * bw + qx];
      for (int k = 0; k < 4 && ok; ++k) {
        const int c = (qy + (k >> 1)) * bw + qx + (k & 1);
        ok = mode_inter(mode[c]) && mode_skip(mode[c]) && mv[c] == v0;
      }
    }
    q_ok[q] = ok;
    nq += ok;
  }
  const int x0 = sx * 4, y0 = sy * 4;
  bool sb = nq == 4;
  if (sb) {
    const uint32_t v0 = mv[y0 * bw + x0];
    for (int q = 1; q < 4 && sb; ++q) sb = mv[(y0 + (q >> 1) * 2) * bw + x0 + (q & 1) * 2] == v0;
  }
  for (int q = 0; q < 4; ++q) {
    if (!q_ok[q]) continue;
    const int qx = x0 + (q & 1) * 2, qy = y0 + (q >> 1) * 2;
    for (int k = 0; k < 4; ++k) {
      const int c = (qy + (k >> 1)) * bw + qx + (k & 1);
      mode[c] = with_bsz(mode[c], sb ? 2 : 1);
    }
  }
}
TV_HD uint32_t pack_mv(int row, int col) { return (uint32_t)(row & 0xFFFF) | ((uint32_t)(col & 0xFFFF) << 16); }
TV_HD int mv_row(uint32_t v) { return (int)(int16_t)(v & 0xFFFF); }
TV_HD int mv_col(uint32_t v) { return (int)(int16_t)(v >> 16); }

// deblocking info word for a 4x4 unit (av1_defs.h layout): tx = block = 16 << bsz luma,
// 8 << bsz chroma
TV_HD uint32_t lf_word(bool chroma, int lvl_v, int lvl_h, bool skip_inter, int bsz = 0) {
  const uint32_t l = (chroma ? 1u : 2u) + (uint32_t)bsz;
  return l | (l << 3) | (l << 6) | (l << 9) | ((uint32_t)(lvl_v & 63) << 12) | ((uint32_t)(lvl_h & 63) << 18) |
         ((uint32_t)skip_inter << 24);
}

}  // namespace av1
}  // namespace tv
