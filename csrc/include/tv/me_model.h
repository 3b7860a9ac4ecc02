// me_model.h — the hierarchical motion-search model shared by the CPU golden encoder and
// the gfx950 kernels (TV_HD: host + device), so both make bit-identical decisions.
//
//   1. quarter-resolution luma of every SOURCE frame: q = (sum of a 4x4 block + 8) >> 4;
//   2. coarse search per 32x32 CTB (an 8x8 block at quarter resolution) of the current
//      quarter frame against the previous quarter SOURCE frame, full search over
//      [-Rq, Rq]^2 with Rq = range / 4 (range = +-64 full-res pels by default): the
//      coarse field is fully parallel (no recon dependency) and doubles as lookahead;
//   3. full-resolution refinement per CTB around a small candidate set — zero, the CTB's
//      coarse vector, its four coarse neighbours and the co-located vector of the previous
//      frame — with a [-4, +3] x [-3, +3] integer window per candidate and the SAD of all
//      21 blocks (16 x 8x8, 4 x 16x16, 1 x 32x32) at every position;
//   4. half- then quarter-pel refinement per block;
//   5. the rate term charges the MVD against a CTB predictor (median of the left / top /
//      top-right coarse vectors), not |MV|: coherent fields are cheap, as AMVP/merge make
//      them in the bitstream.
#pragma once
#include "hevc_defs.h"

namespace tv {

constexpr int kMeMaxCand = 7;
constexpr int kMeWinX0 = -4, kMeWinX1 = 3;  // integer window around a candidate
constexpr int kMeWinY0 = -3, kMeWinY1 = 3;
constexpr int kMeWinW = kMeWinX1 - kMeWinX0 + 1;  // 8
constexpr int kMeWinH = kMeWinY1 - kMeWinY0 + 1;  // 7
constexpr int kMePosPerCand = kMeWinW * kMeWinH;  // 56

TV_HD int me_pen_index(int dx, int dy) { return tv_min(63, mv_bits_est(dx, dy)); }

// coarse rate term for a quarter-res displacement (dxq, dyq): the full-res penalty / 16
// (a quarter-res SAD sums 16x fewer, 16x averaged samples)
TV_HD int me_coarse_pen(const int* penmv, int dxq, int dyq) {
  return (penmv[me_pen_index(16 * dxq, 16 * dyq)] + 8) >> 4;
}

TV_HD int me_median3(int a, int b, int c) { return tv_max(tv_min(a, b), tv_min(tv_max(a, b), c)); }

// floor division of a quarter-pel component to integer pels
TV_HD int me_qpel_to_int(int v) { return (v + 2) >> 2; }

// Candidate centres (integer full-res pels) of CTB (cxi, cyi) and its MVD predictor pmv
// (quarter pels).  cmv: coarse field [hc][wc][2] in integer full-res pels.  (tmx, tmy):
// co-located quarter-pel MV of the previous frame.  Centres are clamped to [-lim, lim] so
// every integer position stays inside +-range.  Exact duplicates are dropped (first kept).
TV_HD int me_candidates(const int16_t* cmv, int wc, int hc, int cxi, int cyi, int tmx, int tmy, int lim,
                        int cand[kMeMaxCand][2], int pmv[2]) {
  const int self = cyi * wc + cxi;
  int raw[kMeMaxCand][2];
  int n = 0;
  raw[n][0] = 0;
  raw[n][1] = 0;
  ++n;
  raw[n][0] = cmv[2 * self];
  raw[n][1] = cmv[2 * self + 1];
  ++n;
  const int nx[4] = {cxi - 1, cxi, cxi + 1, cxi};
  const int ny[4] = {cyi, cyi - 1, cyi, cyi + 1};
  for (int k = 0; k < 4; ++k) {
    if (nx[k] < 0 || ny[k] < 0 || nx[k] >= wc || ny[k] >= hc) continue;
    const int o = ny[k] * wc + nx[k];
    raw[n][0] = cmv[2 * o];
    raw[n][1] = cmv[2 * o + 1];
    ++n;
  }
  raw[n][0] = me_qpel_to_int(tmx);
  raw[n][1] = me_qpel_to_int(tmy);
  ++n;
  int m = 0;
  for (int i = 0; i < n; ++i) {
    const int x = clip3(-lim, lim, raw[i][0]), y = clip3(-lim, lim, raw[i][1]);
    bool dup = false;
    for (int j = 0; j < m; ++j) dup = dup || (tv_abs(cand[j][0] - x) <= 3 && tv_abs(cand[j][1] - y) <= 2);
    if (dup) continue;
    cand[m][0] = x;
    cand[m][1] = y;
    ++m;
  }
  // predictor: median of left / top / top-right coarse vectors (missing -> own coarse)
  int px[3], py[3];
  const int ax[3] = {cxi - 1, cxi, cxi + 1}, ay[3] = {cyi, cyi - 1, cyi - 1};
  for (int k = 0; k < 3; ++k) {
    const bool ok = ax[k] >= 0 && ay[k] >= 0 && ax[k] < wc && ay[k] < hc;
    const int o = ok ? ay[k] * wc + ax[k] : self;
    px[k] = cmv[2 * o];
    py[k] = cmv[2 * o + 1];
  }
  pmv[0] = 4 * me_median3(px[0], px[1], px[2]);
  pmv[1] = 4 * me_median3(py[0], py[1], py[2]);
  return m;
}

// position index within the candidate windows -> integer MV (full-res pels)
TV_HD void me_pos_to_mv(int pos, const int cand[kMeMaxCand][2], int& mx, int& my) {
  const int k = pos / kMePosPerCand, r = pos - k * kMePosPerCand;
  mx = cand[k][0] + (r % kMeWinW) + kMeWinX0;
  my = cand[k][1] + (r / kMeWinW) + kMeWinY0;
}

// sub-pel neighbour k (0..7) of a centre
TV_HD void me_cand_offset(int k, int& ox, int& oy) {
  ox = (k == 0 || k == 3 || k == 5) ? -1 : ((k == 1 || k == 6) ? 0 : 1);
  oy = k < 3 ? -1 : (k < 5 ? 0 : 1);
}

// ---- intra mode pre-selection (I-frame analysis, CPU == GPU) ---------------------------
// stage 1: planar, DC and the angular modes 2, 6, 10, ..., 34 (11 modes); stage 2: the
// +-1 / +-2 neighbours of the best stage-1 angular mode (never stage-1 modes themselves).
// 15 SATD evaluations per block instead of 35.
constexpr int kIntraCoarseModes = 11;
TV_HD int intra_coarse_mode(int i) { return i < 2 ? i : 2 + 4 * (i - 2); }
// i-th refinement mode around angular mode m (0..3 -> m-2, m-1, m+1, m+2); -1 if outside 2..34
TV_HD int intra_refine_mode(int m, int i) {
  const int d = i < 2 ? i - 2 : i - 1;
  const int r = m + d;
  return (r >= 2 && r <= 34) ? r : -1;
}

// ---- intra CUs in P pictures (CPU == GPU) -----------------------------------------------
// Unit of decision: the four 16x16 quadrants q (z-order) of a 32x32 CTB.  A quadrant whose
// best 16x16 inter cost (SAD + MV rate, after sub-pel refinement) exceeds kPIntraGate per
// sample is evaluated for intra: the 15-mode SATD search of the I-frame analysis on SOURCE
// neighbours picks the mode, and it becomes a candidate when that mode's SAD + pintra
// penalty beats the inter cost (a 16x16 intra CU, 2Nx2N, chroma DM).
//
// Reconstruction is four passes, pass q coding quadrant q of every CTB in parallel after the
// inter reconstruction.  Intra prediction reads the reconstructed left / above / above-right
// / below-left / corner neighbours that are available in z-scan order; a candidate is
// accepted only if none of those neighbours is an accepted intra quadrant of a LATER pass
// (which would not be reconstructed yet).  For quadrant q of CTB (i, j) those are:
//   q = 3: none;   q = 2: quadrant 3 of (i-1, j);
//   q = 1: quadrant 3 of (i, j-1), quadrant 2 of (i, j-1) and (i+1, j-1);
//   q = 0: quadrant 1 and 3 of (i-1, j), 3 of (i-1, j-1), 2 and 3 of (i, j-1).
// Deciding 3 -> 2 -> 1 -> 0 makes acceptance a pure function of the candidate flags of a
// 3 x 2 CTB neighbourhood (no sequential pass over the picture).
constexpr int kPIntraGate = 6;  // mean inter SAD per sample before intra is tried
// intra cost against the inter SAD + MV rate: SAD * 5/4 (intra residuals cost more bits per
// unit of SAD) + lambda * kPIntraPenBits (mode, CU overhead).  Tuned on the golden encoder
// (tests/test_pintra.py clip, QP 30): a scene cut coded as P -3.9 % bytes at +0.13 dB Y-PSNR,
// panning content neutral; gate 6 instead of 4 gives up 0.2 % of that for fewer searches.
constexpr int kPIntraPenBits = 16;
TV_HD int pintra_cost(int sad, int pen) { return sad * 5 / 4 + pen; }
// the 15-mode search runs only when the DC prediction's cost is within 2x of the inter cost
// (textured / fast-moving quadrants past the gate stop after one prediction)
TV_HD bool pintra_worth_search(int sad_dc, int pen, int inter_cost) { return pintra_cost(sad_dc, pen) < 2 * inter_cost; }
// cand: the frame's [hc][wc][4] quadrant bytes (0x80 | mode for a candidate, else 0)
TV_HD bool pintra_c(const uint8_t* cand, int wc, int hc, int i, int j, int q) {
  return i >= 0 && j >= 0 && i < wc && j < hc && (cand[((long)j * wc + i) * 4 + q] & 0x80);
}
TV_HD bool pintra_acc2(const uint8_t* c, int wc, int hc, int i, int j) {
  return pintra_c(c, wc, hc, i, j, 2) && !pintra_c(c, wc, hc, i - 1, j, 3);
}
TV_HD bool pintra_acc1(const uint8_t* c, int wc, int hc, int i, int j) {
  return pintra_c(c, wc, hc, i, j, 1) && !pintra_c(c, wc, hc, i, j - 1, 3) && !pintra_acc2(c, wc, hc, i, j - 1) &&
         !pintra_acc2(c, wc, hc, i + 1, j - 1);
}
TV_HD bool pintra_accepted(const uint8_t* c, int wc, int hc, int i, int j, int q) {
  switch (q) {
    case 3: return pintra_c(c, wc, hc, i, j, 3);
    case 2: return pintra_acc2(c, wc, hc, i, j);
    case 1: return pintra_acc1(c, wc, hc, i, j);
    default:
      return pintra_c(c, wc, hc, i, j, 0) && !pintra_acc1(c, wc, hc, i - 1, j) && !pintra_c(c, wc, hc, i - 1, j, 3) &&
             !pintra_c(c, wc, hc, i - 1, j - 1, 3) && !pintra_acc2(c, wc, hc, i, j - 1) &&
             !pintra_c(c, wc, hc, i, j - 1, 3);
  }
}

}  // namespace tv
