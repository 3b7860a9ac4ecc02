// hevc_mvpred.h — HEVC motion-vector prediction (H.265 8.5.3.2): merge and AMVP candidate
// lists for the engine's 2Nx2N PUs, P and B slices.  Host + device (TV_HD): the CABAC syntax
// writer, the decoder oracle and the GPU entropy binariser (csrc/gpu/k_entropy.hip) derive
// skip / merge / AMVP syntax from the same lists.
#pragma once
#include "hevc_defs.h"

namespace tv {

// ------------------------------------ MV prediction -------------------------------------
struct Mv {
  int x = 0, y = 0;
  TV_HD bool operator==(const Mv& o) const { return x == o.x && y == o.y; }
  TV_HD bool operator!=(const Mv& o) const { return !(*this == o); }
};
// Merge candidate list for a 2Nx2N PU (P slice, one reference).  `inter_at(xN,yN,mv)` must
// return true iff the location is available (z-scan, decoded, in picture) and inter coded.
template <class F>
TV_HD int merge_candidates(int xPb, int yPb, int nW, int nH, int maxCand, F&& inter_at, Mv* out) {
  Mv a1, b1, b0, a0, b2;
  const bool avA1 = inter_at(xPb - 1, yPb + nH - 1, a1);
  const bool avB1 = inter_at(xPb + nW - 1, yPb - 1, b1);
  const bool avB0 = inter_at(xPb + nW, yPb - 1, b0);
  const bool avA0 = inter_at(xPb - 1, yPb + nH, a0);
  const bool avB2 = inter_at(xPb - 1, yPb - 1, b2);
  const bool fA1 = avA1;
  const bool fB1 = avB1 && !(avA1 && a1 == b1);
  const bool fB0 = avB0 && !(avB1 && b1 == b0);
  const bool fA0 = avA0 && !(avA1 && a1 == a0);
  bool fB2 = avB2 && !(avA1 && a1 == b2) && !(avB1 && b1 == b2);
  if ((int)fA0 + (int)fA1 + (int)fB0 + (int)fB1 == 4) fB2 = false;
  int n = 0;
  if (fA1 && n < maxCand) out[n++] = a1;
  if (fB1 && n < maxCand) out[n++] = b1;
  if (fB0 && n < maxCand) out[n++] = b0;
  if (fA0 && n < maxCand) out[n++] = a0;
  if (fB2 && n < maxCand) out[n++] = b2;
  while (n < maxCand) out[n++] = Mv{0, 0};
  return n;
}

// AMVP candidate list (2 entries) for a 2Nx2N PU, P slice, single reference picture.
template <class F>
TV_HD void amvp_candidates(int xPb, int yPb, int nW, int nH, F&& inter_at, Mv* out) {
  Mv a0, a1, b0, b1, b2;
  const bool avA0 = inter_at(xPb - 1, yPb + nH, a0);
  const bool avA1 = inter_at(xPb - 1, yPb + nH - 1, a1);
  const bool isScaled = avA0 || avA1;
  bool fA = false, fB = false;
  Mv A, B;
  if (avA0) { fA = true; A = a0; }
  else if (avA1) { fA = true; A = a1; }
  const bool avB0 = inter_at(xPb + nW, yPb - 1, b0);
  const bool avB1 = inter_at(xPb + nW - 1, yPb - 1, b1);
  const bool avB2 = inter_at(xPb - 1, yPb - 1, b2);
  if (avB0) { fB = true; B = b0; }
  else if (avB1) { fB = true; B = b1; }
  else if (avB2) { fB = true; B = b2; }
  if (!isScaled && fB) { fA = true; A = B; }
  // (!isScaled): B re-derived by the scaled pass -> same first available B candidate
  Mv list[3];
  int n = 0;
  if (fA) list[n++] = A;
  if (fB) list[n++] = B;
  if (n == 2 && list[0] == list[1]) n = 1;
  while (n < 2) list[n++] = Mv{0, 0};
  out[0] = list[0];
  out[1] = list[1];
}

// ---------------------------- B-slice motion (one ref per list) --------------------------
// Motion of a B-slice PU: prediction direction (1 = L0, 2 = L1, 3 = bi) and both lists'
// vectors (refIdx is always 0: each list holds one picture, tv/gop.h).
struct Motion {
  int dir = 1;
  Mv mv[2];
  TV_HD bool operator==(const Motion& o) const {
    return dir == o.dir && (!(dir & 1) || mv[0] == o.mv[0]) && (!(dir & 2) || mv[1] == o.mv[1]);
  }
};

// Merge candidate list of a 2Nx2N PU in a B slice (8.5.3.2.2-8.5.3.2.5, no temporal
// candidate): spatial candidates, combined bi-predictive candidates, zero candidates.
// `same_ref` = RefPicList0[0] and RefPicList1[0] are the same picture.
template <class F>
TV_HD int merge_candidates_b(int xPb, int yPb, int nW, int nH, int maxCand, bool same_ref, F&& at, Motion* out) {
  Motion a1, b1, b0, a0, b2;
  const bool avA1 = at(xPb - 1, yPb + nH - 1, a1);
  const bool avB1 = at(xPb + nW - 1, yPb - 1, b1);
  const bool avB0 = at(xPb + nW, yPb - 1, b0);
  const bool avA0 = at(xPb - 1, yPb + nH, a0);
  const bool avB2 = at(xPb - 1, yPb - 1, b2);
  const bool fA1 = avA1;
  const bool fB1 = avB1 && !(avA1 && a1 == b1);
  const bool fB0 = avB0 && !(avB1 && b1 == b0);
  const bool fA0 = avA0 && !(avA1 && a1 == a0);
  bool fB2 = avB2 && !(avA1 && a1 == b2) && !(avB1 && b1 == b2);
  if ((int)fA0 + (int)fA1 + (int)fB0 + (int)fB1 == 4) fB2 = false;
  int n = 0;
  if (fA1 && n < maxCand) out[n++] = a1;
  if (fB1 && n < maxCand) out[n++] = b1;
  if (fB0 && n < maxCand) out[n++] = b0;
  if (fA0 && n < maxCand) out[n++] = a0;
  if (fB2 && n < maxCand) out[n++] = b2;
  const int orig = n;
  if (orig > 1 && orig < maxCand) {
    constexpr int l0i[12] = {0, 1, 0, 2, 1, 2, 0, 3, 1, 3, 2, 3};
    constexpr int l1i[12] = {1, 0, 2, 0, 2, 1, 3, 0, 3, 1, 3, 2};
    for (int c = 0; c < orig * (orig - 1) && n < maxCand; ++c) {
      const Motion& p = out[l0i[c]];
      const Motion& q = out[l1i[c]];
      if ((p.dir & 1) && (q.dir & 2) && (!same_ref || p.mv[0] != q.mv[1])) {
        Motion m;
        m.dir = 3;
        m.mv[0] = p.mv[0];
        m.mv[1] = q.mv[1];
        out[n++] = m;
      }
    }
  }
  while (n < maxCand) {
    Motion z;
    z.dir = 3;
    out[n++] = z;
  }
  return n;
}

// Spatial MV scaling (8.5.3.2.7): td / tb are POC distances to the candidate's and the
// target reference picture.
TV_HD Mv scale_mv(Mv m, int td, int tb) {
  td = clip3(-128, 127, td);
  tb = clip3(-128, 127, tb);
  const int tx = (16384 + (tv_abs(td) >> 1)) / td;
  const int dsf = clip3(-4096, 4095, (tb * tx + 32) >> 6);
  auto s = [&](int v) {
    const long long p = (long long)dsf * v;
    const long long a = ((p < 0 ? -p : p) + 127) >> 8;
    return (int)clip3<long long>(-32768, 32767, p < 0 ? -a : a);
  };
  return Mv{s(m.x), s(m.y)};
}

// AMVP candidate list (2 entries) of list X for a 2Nx2N PU in a B slice with one picture
// per list (POCs ref_poc[0..1], current POC cur_poc): spatial candidates with the
// other-list and scaled fallbacks, no temporal candidate.
template <class F>
TV_HD void amvp_candidates_b(int xPb, int yPb, int nW, int nH, int X, const int* ref_poc, int cur_poc, F&& at, Mv* out) {
  const int Y = 1 - X, target = ref_poc[X];
  Motion nA[2], nB[3];
  const bool avA[2] = {at(xPb - 1, yPb + nH, nA[0]), at(xPb - 1, yPb + nH - 1, nA[1])};
  const bool isScaled = avA[0] || avA[1];
  // first pass: a neighbour vector that points at the target picture as it is
  auto same_pic = [&](const Motion& m, Mv& v) {
    if ((m.dir >> X) & 1) {  // list X of the neighbour holds the same picture
      v = m.mv[X];
      return true;
    }
    if (((m.dir >> Y) & 1) && ref_poc[Y] == target) {
      v = m.mv[Y];
      return true;
    }
    return false;
  };
  // second pass: any vector of the neighbour, scaled to the target picture's distance
  auto scaled = [&](const Motion& m, Mv& v) {
    int l;
    if ((m.dir >> X) & 1) l = X;
    else if ((m.dir >> Y) & 1) l = Y;
    else return false;
    v = m.mv[l];
    v = scale_mv(v, cur_poc - ref_poc[l], cur_poc - target);
    return true;
  };
  bool fA = false, fB = false;
  Mv A, B;
  for (int k = 0; k < 2 && !fA; ++k)
    if (avA[k]) fA = same_pic(nA[k], A);
  for (int k = 0; k < 2 && !fA; ++k)
    if (avA[k]) fA = scaled(nA[k], A);
  const bool avB[3] = {at(xPb + nW, yPb - 1, nB[0]), at(xPb + nW - 1, yPb - 1, nB[1]), at(xPb - 1, yPb - 1, nB[2])};
  for (int k = 0; k < 3 && !fB; ++k)
    if (avB[k]) fB = same_pic(nB[k], B);
  if (!isScaled && fB) {
    fA = true;
    A = B;
  }
  if (!isScaled) {
    fB = false;
    for (int k = 0; k < 3 && !fB; ++k)
      if (avB[k]) fB = scaled(nB[k], B);
  }
  Mv list[2];
  int n = 0;
  if (fA) list[n++] = A;
  if (fB) list[n++] = B;
  if (n == 2 && list[0] == list[1]) n = 1;
  while (n < 2) list[n++] = Mv{0, 0};
  out[0] = list[0];
  out[1] = list[1];
}

}  // namespace tv
