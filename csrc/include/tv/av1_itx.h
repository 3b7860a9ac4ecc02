// av1_itx.h — the AV1 specification's inverse transforms (section 7.13: inverse DCT /
// ADST / identity 1-D processes and the 2-D inverse transform process), bit exact.
// Shared (TV_HD) by the C++ golden encoder / decoder oracle (csrc/core/av1_codec.cpp) and
// the gfx950 encode kernels (csrc/gpu/k_av1_enc.hip), so reconstructions equal what any
// conformant decoder (dav1d in tests/test_av1_conformance.py) reconstructs.
//
// The DCT is the specification's butterfly network written as its recursive structure:
// bit-reversal permutation, the even half is the N/2-point DCT, the odd half is a ladder of
// rotations (12-bit cos128 / sin128 constants, Round2(.., 12) after every rotation) and
// Hadamard butterflies, then one output butterfly.  ADST4 uses the sinpi(k/9) constants,
// ADST8 / ADST16 the butterfly networks of 7.13.2.7 / 7.13.2.8.  Additions are clamped to
// the stage range as dav1d / libaom do (no effect on conformant streams).
//
// The forward transforms the encoder uses are not normative (any forward transform gives a
// valid stream); av1_txfm.h keeps the integer basis-matrix forward path (MFMA on gfx950).
#pragma once
#include <cstdint>

#include "tv/hevc_defs.h"  // TV_HD, clip3

namespace tv {
namespace av1 {

// round(4096 * cos(i * pi / 128)), i = 0..64
constexpr int16_t kCos128[65] = {4096, 4095, 4091, 4085, 4076, 4065, 4052, 4036, 4017, 3996, 3973, 3948, 3920,
                                 3889, 3857, 3822, 3784, 3745, 3703, 3659, 3612, 3564, 3513, 3461, 3406, 3349,
                                 3290, 3229, 3166, 3102, 3035, 2967, 2896, 2824, 2751, 2675, 2598, 2520, 2440,
                                 2359, 2276, 2191, 2106, 2019, 1931, 1842, 1751, 1660, 1567, 1474, 1380, 1285,
                                 1189, 1092, 995,  897,  799,  700,  601,  501,  401,  301,  201,  101,  0};
// round(4096 * 2 sqrt(2) / 3 * sin(k * pi / 9)), k = 0..4
constexpr int16_t kSinPi9[5] = {0, 1321, 2482, 3344, 3803};

TV_HD int cospi(int i) { return kCos128[i]; }
TV_HD int32_t hbtf(int w0, int32_t a, int w1, int32_t b) {
  return (int32_t)(((int64_t)w0 * a + (int64_t)w1 * b + 2048) >> 12);
}
TV_HD int brev(int nbits, int x) {
  int r = 0;
  for (int i = 0; i < nbits; ++i) r |= ((x >> i) & 1) << (nbits - 1 - i);
  return r;
}
struct Range {
  int32_t lo, hi;
  TV_HD int32_t operator()(int64_t v) const { return (int32_t)(v < lo ? lo : (v > hi ? hi : v)); }
};

// ---- inverse DCT (N = 2^n, n = 1..6) ----------------------------------------------------
// odd half of an N-point DCT (M = N/2 values at o[0..M)), inputs already permuted
TV_HD void idct_odd(int32_t* o, int n, Range c) {
  const int N = 1 << n, M = N >> 1;
  if (n == 1) return;
  for (int i = 0; i < M / 2; ++i) {  // input rotations
    const int a = (64 >> n) * (1 + 4 * brev(n - 2, i));
    const int32_t lo = o[i], hi = o[M - 1 - i];
    o[i] = hbtf(cospi(64 - a), lo, -cospi(a), hi);
    o[M - 1 - i] = hbtf(cospi(a), lo, cospi(64 - a), hi);
  }
  const int L = n - 2;
  for (int l = 1; l <= L; ++l) {
    const int G = 1 << l;
    for (int q = 0; q < M / G; ++q)  // Hadamard butterflies over blocks of G
      for (int i = 0; i < G / 2; ++i) {
        const int x = q * G + i, y = q * G + G - 1 - i;
        const int32_t a = o[x], b = o[y];
        if (q & 1) {
          o[x] = c((int64_t)b - a);
          o[y] = c((int64_t)a + b);
        } else {
          o[x] = c((int64_t)a + b);
          o[y] = c((int64_t)a - b);
        }
      }
    const int S = 2 * G;
    if (l < L) {  // rotations of the middle of every lower-half block of S
      const int nblk = (M / 2) / S, np = n - l - 1;  // angles of the (N >> (l+1))-point DCT
      int lb = 0;
      while ((1 << lb) < nblk) ++lb;
      for (int r = 0; r < nblk; ++r) {
        const int th = (64 >> np) * (1 + 4 * brev(lb, r));
        for (int j = r * S + S / 4; j < r * S + 3 * S / 4; ++j) {
          const int32_t lo = o[j], hi = o[M - 1 - j];
          if (j < r * S + S / 2) {
            o[j] = hbtf(-cospi(th), lo, cospi(64 - th), hi);
            o[M - 1 - j] = hbtf(cospi(64 - th), lo, cospi(th), hi);
          } else {
            o[j] = hbtf(-cospi(64 - th), lo, -cospi(th), hi);
            o[M - 1 - j] = hbtf(-cospi(th), lo, cospi(64 - th), hi);
          }
        }
      }
    } else {  // final level: pi / 4 rotations
      for (int j = M / 4; j < M / 2; ++j) {
        const int32_t lo = o[j], hi = o[M - 1 - j];
        o[j] = hbtf(-2896, lo, 2896, hi);
        o[M - 1 - j] = hbtf(2896, lo, 2896, hi);
      }
    }
  }
}

// N-point DCT of a bit-reversal-permuted array: the 2-point core, then for every size
// 4, 8, .. N the odd half of that size and its output butterfly (the recursion over the
// even half, unrolled bottom-up)
TV_HD void idct_core(int32_t* t, int n, Range c) {
  {
    const int32_t a = t[0], b = t[1];
    t[0] = hbtf(2896, a, 2896, b);
    t[1] = hbtf(2896, a, -2896, b);
  }
  for (int m = 2; m <= n; ++m) {
    const int M = 1 << m;
    idct_odd(t + M / 2, m, c);
    for (int i = 0; i < M / 2; ++i) {
      const int32_t a = t[i], b = t[M - 1 - i];
      t[i] = c((int64_t)a + b);
      t[M - 1 - i] = c((int64_t)a - b);
    }
  }
}

template <int n> TV_HD void idct(int32_t* t, Range c) {
  constexpr int N = 1 << n;
  int32_t p[N];
  for (int i = 0; i < N; ++i) p[i] = t[brev(n, i)];
  idct_core(p, n, c);
  for (int i = 0; i < N; ++i) t[i] = p[i];
}

// ---- inverse ADST ---------------------------------------------------------------------
TV_HD void iadst4(int32_t* t) {
  const int64_t x0 = t[0], x1 = t[1], x2 = t[2], x3 = t[3];
  int64_t s0 = kSinPi9[1] * x0, s1 = kSinPi9[2] * x0, s2 = kSinPi9[3] * x1, s3 = kSinPi9[4] * x2;
  const int64_t s4 = kSinPi9[1] * x2, s5 = kSinPi9[2] * x3, s6 = kSinPi9[4] * x3, s7 = x0 - x2 + x3;
  s0 = s0 + s3;
  s1 = s1 - s4;
  s3 = s2;
  s2 = kSinPi9[3] * s7;
  s0 = s0 + s5;
  s1 = s1 - s6;
  const int64_t y0 = s0 + s3, y1 = s1 + s3, y2 = s2, y3 = s0 + s1 - s3;
  t[0] = (int32_t)((y0 + 2048) >> 12);
  t[1] = (int32_t)((y1 + 2048) >> 12);
  t[2] = (int32_t)((y2 + 2048) >> 12);
  t[3] = (int32_t)((y3 + 2048) >> 12);
}

TV_HD void iadst8(int32_t* t, Range c) {
  int32_t b[8], a[8];
  b[0] = t[7], b[1] = t[0], b[2] = t[5], b[3] = t[2], b[4] = t[3], b[5] = t[4], b[6] = t[1], b[7] = t[6];
  for (int i = 0; i < 4; ++i) {
    const int k = 4 + 16 * i;  // cospi 4, 20, 36, 52
    a[2 * i] = hbtf(cospi(k), b[2 * i], cospi(64 - k), b[2 * i + 1]);
    a[2 * i + 1] = hbtf(cospi(64 - k), b[2 * i], -cospi(k), b[2 * i + 1]);
  }
  for (int i = 0; i < 4; ++i) {
    b[i] = c((int64_t)a[i] + a[i + 4]);
    b[i + 4] = c((int64_t)a[i] - a[i + 4]);
  }
  a[0] = b[0], a[1] = b[1], a[2] = b[2], a[3] = b[3];
  a[4] = hbtf(cospi(16), b[4], cospi(48), b[5]);
  a[5] = hbtf(cospi(48), b[4], -cospi(16), b[5]);
  a[6] = hbtf(-cospi(48), b[6], cospi(16), b[7]);
  a[7] = hbtf(cospi(16), b[6], cospi(48), b[7]);
  b[0] = c((int64_t)a[0] + a[2]), b[1] = c((int64_t)a[1] + a[3]);
  b[2] = c((int64_t)a[0] - a[2]), b[3] = c((int64_t)a[1] - a[3]);
  b[4] = c((int64_t)a[4] + a[6]), b[5] = c((int64_t)a[5] + a[7]);
  b[6] = c((int64_t)a[4] - a[6]), b[7] = c((int64_t)a[5] - a[7]);
  a[0] = b[0], a[1] = b[1], a[4] = b[4], a[5] = b[5];
  a[2] = hbtf(cospi(32), b[2], cospi(32), b[3]);
  a[3] = hbtf(cospi(32), b[2], -cospi(32), b[3]);
  a[6] = hbtf(cospi(32), b[6], cospi(32), b[7]);
  a[7] = hbtf(cospi(32), b[6], -cospi(32), b[7]);
  t[0] = a[0], t[1] = -a[4], t[2] = a[6], t[3] = -a[2];
  t[4] = a[3], t[5] = -a[7], t[6] = a[5], t[7] = -a[1];
}

TV_HD void iadst16(int32_t* t, Range c) {
  int32_t b[16], a[16];
  constexpr int8_t perm[16] = {15, 0, 13, 2, 11, 4, 9, 6, 7, 8, 5, 10, 3, 12, 1, 14};
  for (int i = 0; i < 16; ++i) b[i] = t[perm[i]];
  for (int i = 0; i < 8; ++i) {
    const int k = 2 + 8 * i;  // cospi 2, 10, ..., 58
    a[2 * i] = hbtf(cospi(k), b[2 * i], cospi(64 - k), b[2 * i + 1]);
    a[2 * i + 1] = hbtf(cospi(64 - k), b[2 * i], -cospi(k), b[2 * i + 1]);
  }
  for (int i = 0; i < 8; ++i) {
    b[i] = c((int64_t)a[i] + a[i + 8]);
    b[i + 8] = c((int64_t)a[i] - a[i + 8]);
  }
  for (int i = 0; i < 8; ++i) a[i] = b[i];
  a[8] = hbtf(cospi(8), b[8], cospi(56), b[9]);
  a[9] = hbtf(cospi(56), b[8], -cospi(8), b[9]);
  a[10] = hbtf(cospi(40), b[10], cospi(24), b[11]);
  a[11] = hbtf(cospi(24), b[10], -cospi(40), b[11]);
  a[12] = hbtf(-cospi(56), b[12], cospi(8), b[13]);
  a[13] = hbtf(cospi(8), b[12], cospi(56), b[13]);
  a[14] = hbtf(-cospi(24), b[14], cospi(40), b[15]);
  a[15] = hbtf(cospi(40), b[14], cospi(24), b[15]);
  for (int g = 0; g < 16; g += 8)
    for (int i = 0; i < 4; ++i) {
      b[g + i] = c((int64_t)a[g + i] + a[g + i + 4]);
      b[g + i + 4] = c((int64_t)a[g + i] - a[g + i + 4]);
    }
  for (int g = 0; g < 16; g += 8) {
    a[g + 0] = b[g + 0], a[g + 1] = b[g + 1], a[g + 2] = b[g + 2], a[g + 3] = b[g + 3];
    a[g + 4] = hbtf(cospi(16), b[g + 4], cospi(48), b[g + 5]);
    a[g + 5] = hbtf(cospi(48), b[g + 4], -cospi(16), b[g + 5]);
    a[g + 6] = hbtf(-cospi(48), b[g + 6], cospi(16), b[g + 7]);
    a[g + 7] = hbtf(cospi(16), b[g + 6], cospi(48), b[g + 7]);
  }
  for (int g = 0; g < 16; g += 4) {
    b[g + 0] = c((int64_t)a[g + 0] + a[g + 2]);
    b[g + 1] = c((int64_t)a[g + 1] + a[g + 3]);
    b[g + 2] = c((int64_t)a[g + 0] - a[g + 2]);
    b[g + 3] = c((int64_t)a[g + 1] - a[g + 3]);
  }
  for (int g = 0; g < 16; g += 4) {
    a[g + 0] = b[g + 0], a[g + 1] = b[g + 1];
    a[g + 2] = hbtf(cospi(32), b[g + 2], cospi(32), b[g + 3]);
    a[g + 3] = hbtf(cospi(32), b[g + 2], -cospi(32), b[g + 3]);
  }
  t[0] = a[0], t[1] = -a[8], t[2] = a[12], t[3] = -a[4];
  t[4] = a[6], t[5] = -a[14], t[6] = a[10], t[7] = -a[2];
  t[8] = a[3], t[9] = -a[11], t[10] = a[15], t[11] = -a[7];
  t[12] = a[5], t[13] = -a[13], t[14] = a[9], t[15] = -a[1];
}

template <int n> TV_HD void iidentity(int32_t* t) {
  constexpr int N = 1 << n;
  for (int i = 0; i < N; ++i) {
    const int64_t v = t[i];
    t[i] = n == 2 ? (int32_t)((v * 5793 + 2048) >> 12)
         : n == 3 ? (int32_t)(v * 2)
         : n == 4 ? (int32_t)((v * 11586 + 2048) >> 12)
                  : (int32_t)(v * 4);
  }
}

// 1-D inverse of type (0 DCT, 1 ADST, 3 IDTX; tv::av1::TxType1D) on T[0..2^n)
template <int n> TV_HD void inv_1d(int32_t* t, int type, Range c) {
  if (type == 3) iidentity<n>(t);
  else if (type == 1 && n == 2) iadst4(t);
  else if (type == 1 && n == 3) iadst8(t, c);
  else if (type == 1 && n == 4) iadst16(t, c);
  else idct<n>(t, c);
}

// Transform_Row_Shift of the square sizes (log2 N = 2..6)
TV_HD constexpr int row_shift(int lg) { return lg == 2 ? 0 : (lg == 3 ? 1 : 2); }
constexpr int32_t kRowLo = -(1 << 15), kRowHi = (1 << 15) - 1;  // BitDepth + 8
constexpr int32_t kColLo = -(1 << 15), kColHi = (1 << 15) - 1;  // Max(BitDepth + 6, 16)

// One row of the 2-D inverse transform (7.13.3): dequantised coefficients in[0..N) ->
// the row transform, Round2(.., rowShift), clamped to the column range.  Row i >= 32 of a
// 64-point transform and all-zero rows stay zero.
template <int lg> TV_HD void inv_row(const int32_t* in, int trow, int32_t* out) {
  constexpr int N = 1 << lg, nz = N < 32 ? N : 32, rs = row_shift(lg);
  const Range rr{kRowLo, kRowHi}, cr{kColLo, kColHi};
  int32_t t[N];
  bool any = false;
  for (int j = 0; j < N; ++j) {
    t[j] = j < nz ? rr(in[j]) : 0;
    any |= t[j] != 0;
  }
  if (!any) {
    for (int j = 0; j < N; ++j) out[j] = 0;
    return;
  }
  inv_1d<lg>(t, trow, rr);
  for (int j = 0; j < N; ++j) out[j] = cr(((int64_t)t[j] + ((1 << rs) >> 1)) >> rs);
}
// One column: the column transform and Round2(.., 4) (colShift, 8-bit).
template <int lg> TV_HD void inv_col(int32_t* t, int tcol) {
  constexpr int N = 1 << lg;
  inv_1d<lg>(t, tcol, Range{kColLo, kColHi});
  for (int i = 0; i < N; ++i) t[i] = (t[i] + 8) >> 4;
}

// 2-D inverse transform process (7.13.3) of an N x N block, 8-bit: `coef` are the
// dequantised coefficients in raster order (row i = vertical frequency), `res` the
// residual.  tcol / trow: 1-D types of the columns (vertical) and rows (horizontal).
template <int lg> TV_HD void inv_txfm2d(const int32_t* coef, int tcol, int trow, int32_t* res) {
  constexpr int N = 1 << lg, nz = N < 32 ? N : 32;
  for (int i = 0; i < N; ++i) {
    if (i < nz) inv_row<lg>(coef + i * N, trow, res + i * N);
    else
      for (int j = 0; j < N; ++j) res[i * N + j] = 0;
  }
  int32_t t[N];
  for (int j = 0; j < N; ++j) {
    for (int i = 0; i < N; ++i) t[i] = res[i * N + j];
    inv_col<lg>(t, tcol);
    for (int i = 0; i < N; ++i) res[i * N + j] = t[i];
  }
}
inline void inv_txfm2d(const int32_t* coef, int lg, int tcol, int trow, int32_t* res) {
  switch (lg) {
    case 2: inv_txfm2d<2>(coef, tcol, trow, res); break;
    case 3: inv_txfm2d<3>(coef, tcol, trow, res); break;
    case 4: inv_txfm2d<4>(coef, tcol, trow, res); break;
    case 5: inv_txfm2d<5>(coef, tcol, trow, res); break;
    default: inv_txfm2d<6>(coef, tcol, trow, res); break;
  }
}

}  // namespace av1
}  // namespace tv
