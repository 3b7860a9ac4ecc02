// hevc_defs.h — HEVC (H.265) constants, tables and bit-exact scalar primitives shared by
// the C++ host code (syntax writer, decoder oracle, CPU reference encoder) and the HIP
// kernels for gfx950.  Everything here is `TV_HD` (host+device) and header-only so the GPU
// and CPU paths compute byte-identical reconstructions.
//
// Reference parity: thinvids encodes with ffmpeg h264_vaapi CQP 27 (reference
// worker/tasks.py:66-67, :1573-1586); this engine replaces that hot path with its own
// HEVC encoder (SURVEY.md §2.3 K5a–K5h).  Tables are transcribed from ITU-T H.265.
#pragma once
#include <cstdint>
#include <cmath>
#include <cstdlib>

#if defined(__HIPCC__)
#define TV_HD __host__ __device__ __forceinline__
#else
#define TV_HD inline
#endif

namespace tv {

template <typename T> TV_HD T clip3(T lo, T hi, T v) { return v < lo ? lo : (v > hi ? hi : v); }
TV_HD int clip_pixel(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }
TV_HD int tv_abs(int v) { return v < 0 ? -v : v; }
TV_HD int tv_min(int a, int b) { return a < b ? a : b; }
TV_HD int tv_max(int a, int b) { return a > b ? a : b; }

// ---------------------------------------------------------------------------------------
// Fixed coding-structure configuration of this engine (GPU-friendly subset of Main profile)
//   CTB 32x32, min CB 8x8, TB = CB (no residual quadtree), min TB 4 (chroma of 8x8 CB),
//   2Nx2N partitions only, one slice per picture, 1 reference picture (previous frame).
// ---------------------------------------------------------------------------------------
constexpr int kCtbLog2 = 5;
constexpr int kCtb = 1 << kCtbLog2;
constexpr int kMinCbLog2 = 3;
constexpr int kMinTbLog2 = 2;
constexpr int kMaxTbLog2 = 5;

// --------------------------------- transform matrix -------------------------------------
// HEVC 32-point integer DCT.  T32[k][n]; smaller sizes use rows k*(32/N).
// The 33 distinct magnitudes indexed by m = ((2n+1)k mod 128) folded to [0,32].
constexpr int8_t kDctMag[33] = {64, 90, 90, 90, 89, 88, 87, 85, 83, 82, 80, 78, 75, 73, 70, 67, 64,
                                61, 57, 54, 50, 46, 43, 38, 36, 31, 25, 22, 18, 13, 9,  4,  0};

struct DctMat32 {
  int8_t m[32][32];
};
constexpr DctMat32 make_dct32() {
  DctMat32 d{};
  for (int k = 0; k < 32; ++k)
    for (int n = 0; n < 32; ++n) {
      int mm = ((2 * n + 1) * k) % 128;
      int v = 0;
      if (mm <= 32) v = kDctMag[mm];
      else if (mm < 64) v = -kDctMag[64 - mm];
      else if (mm <= 96) v = -kDctMag[mm - 64];
      else v = kDctMag[128 - mm];
      d.m[k][n] = (int8_t)v;
    }
  return d;
}
constexpr DctMat32 kDct32 = make_dct32();

// coefficient of the N-point DCT (N = 1<<log2N): row k (frequency), column n (sample)
TV_HD int dct_coef(int log2N, int k, int n) { return kDct32.m[k << (5 - log2N)][n]; }

// ------------------------------------ quantisation --------------------------------------
constexpr int kQuantScale[6] = {26214, 23302, 20560, 18396, 16384, 14564};
constexpr int kLevelScale[6] = {40, 45, 51, 57, 64, 72};
// Table reads as select chains: indexing the constexpr arrays from device code becomes a
// global-memory load per coefficient (a ~1 us round trip inside the I-frame wavefront's
// serial TB chain); the selects are a handful of ALU ops.
TV_HD int quant_scale(int qp) {
  const int r = qp % 6;
  return r == 0 ? 26214 : r == 1 ? 23302 : r == 2 ? 20560 : r == 3 ? 18396 : r == 4 ? 16384 : 14564;
}
TV_HD int level_scale(int qp) {
  const int r = qp % 6;
  return r == 0 ? 40 : r == 1 ? 45 : r == 2 ? 51 : r == 3 ? 57 : r == 4 ? 64 : 72;
}

// chroma QP mapping for 4:2:0 (H.265 Table 8-10)
TV_HD int chroma_qp(int qpy, int offset) {
  int qpi = clip3(-0, 57, qpy + offset);
  if (qpi < 30) return qpi;
  if (qpi >= 43) return qpi - 6;
  constexpr int tab[13] = {29, 30, 31, 32, 33, 33, 34, 34, 35, 35, 36, 36, 37};
  return tab[qpi - 30];
}

// Decoder-exact scaling (dequantisation) of one level, flat scaling matrix (m = 16).
TV_HD int dequant_level(int level, int qp, int log2N) {
  const int bdShift = 8 + log2N - 5;  // BitDepth + log2(nTbS) + 10 - 15
  long long v = (long long)level * 16 * level_scale(qp);
  v = v * (1LL << (qp / 6)) + (1LL << (bdShift - 1));  // multiply: v may be negative
  v >>= bdShift;
  return (int)clip3<long long>(-32768, 32767, v);
}

// RDOQ-lite trailing coefficient-group trimming of inter TBs (tv code_tb / k_inter_recon;
// SeqConfig::rdoq, flag bit 128 off): mode 1 any group after the DC group, 2 groups on or
// beyond the TB's anti-diagonal, 3 groups beyond it.  1080p BD-rate against the tool off
// (profiles/r6_rdoq/): mode 1 +0.85 % smooth / -2.27 % textured, 2 -0.46 / -1.08, 3 -0.16 / -0.64.
constexpr int kRdoqMode = 2;
// first CG diagonal (x + y in CG units, s CGs per side) the trimming may drop
TV_HD int rdoq_dmin(int mode, int s) { return mode == 1 ? 1 : (mode == 2 ? tv_max(1, s - 1) : s); }

// Encoder deadzone quantiser (not normative).  `coef` is the forward-transform output.
// Rounding 1/3 (intra) and 1/4 (inter): the inter 1/6 of HM cost +0.9 % BD-rate on the bench
// content against 1/4 (tools/rd_curve.py, 640x360 GOP 64 + SAO; 1/3: +0.7 %).
TV_HD int quant_level(int coef, int qp, int log2N, bool intra) {
  const int qbits = 14 + qp / 6 + (15 - 8 - log2N);
  const int add = (intra ? 171 : 128) << (qbits - 9);
  int a = tv_abs(coef);
  int l = (int)(((long long)a * quant_scale(qp) + add) >> qbits);
  if (l > 32767) l = 32767;
  return coef < 0 ? -l : l;
}

// Exact scalar inverse 2-D transform (H.265 8.6.4.2) — `coef` and `res` are N*N row-major
// (row = y, column = x).  Output residual is what the decoder adds to the prediction.
TV_HD void inverse_transform(const int* coef, int log2N, int* res) {
  const int N = 1 << log2N;
  int tmp[32 * 32];
  // stage 1: columns (vertical 1-D inverse), clip to 16 bit after >>7
  for (int x = 0; x < N; ++x)
    for (int y = 0; y < N; ++y) {
      int s = 0;
      for (int k = 0; k < N; ++k) s += dct_coef(log2N, k, y) * coef[k * N + x];
      tmp[y * N + x] = clip3(-32768, 32767, (s + 64) >> 7);
    }
  // stage 2: rows, bdShift = 20 - BitDepth = 12
  for (int y = 0; y < N; ++y)
    for (int x = 0; x < N; ++x) {
      long long s = 0;
      for (int k = 0; k < N; ++k) s += (long long)dct_coef(log2N, k, x) * tmp[y * N + k];
      res[y * N + x] = (int)((s + 2048) >> 12);
    }
}

// Forward 2-D transform (encoder side; HM scaling convention).  residual -> coefficients.
TV_HD void forward_transform(const int* res, int log2N, int* coef) {
  const int N = 1 << log2N;
  const int sh1 = log2N - 1, sh2 = log2N + 6;
  int tmp[32 * 32];
  for (int k = 0; k < N; ++k)  // vertical: tmp[k][x] = sum_y T[k][y] * r[y][x]
    for (int x = 0; x < N; ++x) {
      int s = 0;
      for (int y = 0; y < N; ++y) s += dct_coef(log2N, k, y) * res[y * N + x];
      tmp[k * N + x] = (s + (1 << (sh1 - 1))) >> sh1;
    }
  for (int k = 0; k < N; ++k)
    for (int j = 0; j < N; ++j) {  // horizontal: coef[k][j] = sum_x T[j][x] * tmp[k][x]
      long long s = 0;
      for (int x = 0; x < N; ++x) s += (long long)dct_coef(log2N, j, x) * tmp[k * N + x];
      coef[k * N + j] = (int)((s + (1LL << (sh2 - 1))) >> sh2);
    }
}

// ---------------------------------- intra prediction ------------------------------------
constexpr int8_t kIntraPredAngle[35] = {0,   0,   32,  26,  21,  17,  13,  9,  5,  2,  0,  -2,
                                        -5,  -9,  -13, -17, -21, -26, -32, -26, -21, -17, -13, -9,
                                        -5,  -2,  0,   2,   5,   9,   13,  17,  21,  26,  32};
// invAngle for modes 11..25
constexpr int16_t kInvAngle[15] = {-4096, -1638, -910, -630, -482, -390, -315, -256,
                                   -315,  -390,  -482, -630, -910, -1638, -4096};

// One intra-predicted sample at (x, y) of an N x N block from its (already substituted,
// optionally smoothed) reference samples:
//   left[i] = p[-1][i-1] for i = 0..2N   (left[0] = corner p[-1][-1])
//   top[i]  = p[i-1][-1] for i = 0..2N   (top[0]  = corner)
// `dc` is the DC value of the block (only used by mode 1), `fe` enables the DC/H/V boundary
// smoothing (luma, N < 32).  Used per lane by the HIP kernels and per block on the CPU.
template <typename R>
TV_HD int intra_pred_pixel_ai(const R* left, const R* top, int log2N, int mode, int angle, int inv, bool fe,
                              int dc, int x, int y);
// angle / inverse angle of an angular mode (device callers hoist these table reads out of
// their per-sample loops: an indexed constexpr table is a global-memory load on the GPU)
TV_HD int intra_angle(int mode) { return kIntraPredAngle[mode]; }
TV_HD int intra_inv_angle(int mode) { return mode >= 11 && mode <= 25 ? kInvAngle[mode - 11] : 0; }
template <typename R>
TV_HD int intra_pred_pixel(const R* left, const R* top, int log2N, int mode, bool fe, int dc, int x,
                           int y) {
  return intra_pred_pixel_ai(left, top, log2N, mode, mode >= 2 ? intra_angle(mode) : 0,
                             mode >= 2 ? intra_inv_angle(mode) : 0, fe, dc, x, y);
}
template <typename R>
TV_HD int intra_pred_pixel_ai(const R* left, const R* top, int log2N, int mode, int angle, int inv, bool fe,
                              int dc, int x, int y) {
  const int N = 1 << log2N;
  if (mode == 0)
    return ((N - 1 - x) * left[y + 1] + (x + 1) * top[N + 1] + (N - 1 - y) * top[x + 1] +
            (y + 1) * left[N + 1] + N) >> (log2N + 1);
  if (mode == 1) {
    if (fe) {
      if (x == 0 && y == 0) return (left[1] + 2 * dc + top[1] + 2) >> 2;
      if (y == 0) return (top[x + 1] + 3 * dc + 2) >> 2;
      if (x == 0) return (left[y + 1] + 3 * dc + 2) >> 2;
    }
    return dc;
  }
  const bool vert = mode >= 18;
  const R* mainr = vert ? top : left;
  const R* side = vert ? left : top;
  const int i = vert ? x : y, j = vert ? y : x;
  const int pos = (j + 1) * angle;
  const int idx = pos >> 5, fact = pos & 31;
  auto ref = [&](int k) -> int { return k >= 0 ? (int)mainr[k] : (int)side[(k * inv + 128) >> 8]; };
  int v = fact ? ((32 - fact) * ref(i + idx + 1) + fact * ref(i + idx + 2) + 16) >> 5 : ref(i + idx + 1);
  if (fe) {
    if (mode == 26 && x == 0) v = clip_pixel(top[1] + ((left[y + 1] - left[0]) >> 1));
    else if (mode == 10 && y == 0) v = clip_pixel(left[1] + ((top[x + 1] - top[0]) >> 1));
  }
  return v;
}

template <typename R> TV_HD int intra_dc_value(const R* left, const R* top, int log2N) {
  const int N = 1 << log2N;
  int s = N;
  for (int i = 0; i < N; ++i) s += top[i + 1] + left[i + 1];
  return s >> (log2N + 1);
}

// Whole-block intra prediction (CPU path), pred[y*N+x].
TV_HD void intra_pred_from_refs(const int* left, const int* top, int log2N, int mode,
                                bool filter_edges, int* pred) {
  const int N = 1 << log2N;
  const int dc = mode == 1 ? intra_dc_value(left, top, log2N) : 0;
  for (int y = 0; y < N; ++y)
    for (int x = 0; x < N; ++x)
      pred[y * N + x] = intra_pred_pixel(left, top, log2N, mode, filter_edges, dc, x, y);
}

// [1 2 1] reference smoothing decision (H.265 8.4.4.2.3), luma only, no strong smoothing.
TV_HD bool intra_filter_refs(int log2N, int mode) {
  if (mode == 1 || log2N == 2) return false;
  const int d = tv_min(tv_abs(mode - 26), tv_abs(mode - 10));
  const int thr = log2N == 3 ? 7 : (log2N == 4 ? 1 : 0);
  return d > thr;
}

// Apply [1 2 1] filtering in place to left/top arrays (length 2N+1 each, index 0 = corner).
TV_HD void intra_smooth_refs(int* left, int* top, int N) {
  int l[65], t[65];
  const int c = (left[1] + 2 * left[0] + top[1] + 2) >> 2;
  for (int i = 1; i < 2 * N; ++i) {
    l[i] = (left[i + 1] + 2 * left[i] + left[i - 1] + 2) >> 2;
    t[i] = (top[i + 1] + 2 * top[i] + top[i - 1] + 2) >> 2;
  }
  for (int i = 1; i < 2 * N; ++i) {
    left[i] = l[i];
    top[i] = t[i];
  }
  left[0] = top[0] = c;
}

// Reference-sample substitution (H.265 8.4.4.2.2) given availability flags.
//   Canonical order: left[2N] (bottom) ... left[1], corner, top[1] ... top[2N].
template <typename R>
TV_HD void intra_substitute(R* left, R* top, const bool* lavail, const bool* tavail, int N) {
  const int total = 4 * N + 1;
  auto get = [&](int i) -> R& { return i < 2 * N ? left[2 * N - i] : top[i - 2 * N]; };
  auto av = [&](int i) -> bool { return i < 2 * N ? lavail[2 * N - i] : tavail[i - 2 * N]; };
  int first = -1;
  for (int i = 0; i < total; ++i)
    if (av(i)) {
      first = i;
      break;
    }
  if (first < 0) {
    for (int i = 0; i < total; ++i) get(i) = 128;
    left[0] = 128;
    return;
  }
  if (first > 0) get(0) = get(first);
  for (int i = 1; i < total; ++i)
    if (!av(i)) get(i) = get(i - 1);
  left[0] = top[0];  // the corner is stored in both arrays; index 2N maps to top[0]
}

// MPM candidate list (H.265 8.4.2)
TV_HD void intra_mpm_list(int candA, int candB, int* list) {
  if (candA == candB) {
    if (candA < 2) {
      list[0] = 0;
      list[1] = 1;
      list[2] = 26;
    } else {
      list[0] = candA;
      list[1] = 2 + ((candA + 29) % 32);
      list[2] = 2 + ((candA - 2 + 1) % 32);
    }
  } else {
    list[0] = candA;
    list[1] = candB;
    if (candA != 0 && candB != 0) list[2] = 0;
    else if (candA != 1 && candB != 1) list[2] = 1;
    else list[2] = 26;
  }
}

// ------------------------------- inter interpolation ------------------------------------
constexpr int8_t kLumaFilter[4][8] = {{0, 0, 0, 64, 0, 0, 0, 0},
                                      {-1, 4, -10, 58, 17, -5, 1, 0},
                                      {-1, 4, -11, 40, 40, -11, 4, -1},
                                      {0, 1, -5, 17, 58, -10, 4, -1}};
constexpr int8_t kChromaFilter[8][4] = {{0, 64, 0, 0},     {-2, 58, 10, -2}, {-4, 54, 16, -2},
                                        {-6, 46, 28, -4},  {-4, 36, 36, -4}, {-4, 28, 46, -6},
                                        {-2, 16, 54, -4},  {-2, 10, 58, -2}};

// One luma prediction sample at integer position (xi, yi) with fraction (fx, fy) in quarter
// pel, reference plane clamped at its borders (w x h).  Returns the final 8-bit sample
// (uni-prediction, default weighting).
TV_HD int mc_luma_inter(const uint8_t* ref, int stride, int w, int h, int xi, int yi, int fx,
                        int fy);
TV_HD int mc_chroma_inter(const uint8_t* ref, int stride, int w, int h, int xi, int yi, int fx,
                          int fy);
TV_HD int mc_luma_sample(const uint8_t* ref, int stride, int w, int h, int xi, int yi, int fx, int fy) {
  return clip_pixel((mc_luma_inter(ref, stride, w, h, xi, yi, fx, fy) + 32) >> 6);
}
TV_HD int mc_chroma_sample(const uint8_t* ref, int stride, int w, int h, int xi, int yi, int fx, int fy) {
  return clip_pixel((mc_chroma_inter(ref, stride, w, h, xi, yi, fx, fy) + 32) >> 6);
}
// bi-prediction of one sample from the two 14-bit intermediates (8.5.3.3.4.2, 8-bit)
TV_HD int bipred_sample(int p0, int p1) { return clip_pixel((p0 + p1 + 64) >> 7); }
// 14-bit intermediate luma prediction sample (8.5.3.3.3.1: shift1 = 0, shift2 = 6, shift3 = 6)
TV_HD int mc_luma_inter(const uint8_t* ref, int stride, int w, int h, int xi, int yi, int fx,
                        int fy) {
  auto px = [&](int x, int y) -> int {
    x = clip3(0, w - 1, x);
    y = clip3(0, h - 1, y);
    return ref[y * stride + x];
  };
  int v;
  if (fx == 0 && fy == 0) {
    v = px(xi, yi) << 6;
  } else if (fy == 0) {
    v = 0;
    for (int i = 0; i < 8; ++i) v += kLumaFilter[fx][i] * px(xi + i - 3, yi);
  } else if (fx == 0) {
    v = 0;
    for (int i = 0; i < 8; ++i) v += kLumaFilter[fy][i] * px(xi, yi + i - 3);
  } else {
    v = 0;
    for (int j = 0; j < 8; ++j) {
      int t = 0;
      for (int i = 0; i < 8; ++i) t += kLumaFilter[fx][i] * px(xi + i - 3, yi + j - 3);
      v += kLumaFilter[fy][j] * t;
    }
    v >>= 6;
  }
  return v;
}

TV_HD int mc_chroma_inter(const uint8_t* ref, int stride, int w, int h, int xi, int yi, int fx,
                          int fy) {
  auto px = [&](int x, int y) -> int {
    x = clip3(0, w - 1, x);
    y = clip3(0, h - 1, y);
    return ref[y * stride + x];
  };
  int v;
  if (fx == 0 && fy == 0) {
    v = px(xi, yi) << 6;
  } else if (fy == 0) {
    v = 0;
    for (int i = 0; i < 4; ++i) v += kChromaFilter[fx][i] * px(xi + i - 1, yi);
  } else if (fx == 0) {
    v = 0;
    for (int i = 0; i < 4; ++i) v += kChromaFilter[fy][i] * px(xi, yi + i - 1);
  } else {
    v = 0;
    for (int j = 0; j < 4; ++j) {
      int t = 0;
      for (int i = 0; i < 4; ++i) t += kChromaFilter[fx][i] * px(xi + i - 1, yi + j - 1);
      v += kChromaFilter[fy][j] * t;
    }
    v >>= 6;
  }
  return v;
}

// ------------------------------------ deblocking ----------------------------------------
constexpr uint8_t kBetaTable[52] = {0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,  0,
                                    0,  0,  0,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15,
                                    16, 17, 18, 20, 22, 24, 26, 28, 30, 32, 34, 36, 38,
                                    40, 42, 44, 46, 48, 50, 52, 54, 56, 58, 60, 62, 64};
constexpr uint8_t kTcTable[54] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  0,  0,  0,  0,  0,
                                  1, 1, 1, 1, 1, 1, 1, 1, 1, 2, 2, 2,  2,  3,  3,  3,  3,  4,
                                  4, 4, 5, 5, 6, 6, 7, 8, 9, 10, 11, 13, 14, 16, 18, 20, 22, 24};

// Luma deblocking of one 4-sample edge segment.  `p` points at sample p0 of line 0,
// `step` is the distance p0->q0 direction (across the edge), `lstep` between lines.
// Returns nothing; modifies samples in place.  bs in {1,2}, qp = (QpP+QpQ+1)>>1.
TV_HD void deblock_luma_edge4(uint8_t* q0ptr, int xstep, int lstep, int bs, int qp) {
  // q0ptr points at q0 of line 0; p_i = q0ptr[-(i+1)*xstep], q_i = q0ptr[i*xstep]
  const int beta = kBetaTable[clip3(0, 51, qp)];
  const int tc = kTcTable[clip3(0, 53, qp + 2 * (bs - 1))];
  if (tc == 0) return;
  auto P = [&](int line, int i) -> uint8_t& { return q0ptr[line * lstep - (i + 1) * xstep]; };
  auto Q = [&](int line, int i) -> uint8_t& { return q0ptr[line * lstep + i * xstep]; };
  const int dp0 = tv_abs(P(0, 2) - 2 * P(0, 1) + P(0, 0));
  const int dp3 = tv_abs(P(3, 2) - 2 * P(3, 1) + P(3, 0));
  const int dq0 = tv_abs(Q(0, 2) - 2 * Q(0, 1) + Q(0, 0));
  const int dq3 = tv_abs(Q(3, 2) - 2 * Q(3, 1) + Q(3, 0));
  const int dpq0 = dp0 + dq0, dpq3 = dp3 + dq3;
  const int dp = dp0 + dp3, dq = dq0 + dq3;
  const int d = dpq0 + dpq3;
  if (d >= beta) return;
  auto dsam = [&](int line, int dpq) -> bool {
    return 2 * dpq < (beta >> 2) &&
           tv_abs(P(line, 3) - P(line, 0)) + tv_abs(Q(line, 0) - Q(line, 3)) < (beta >> 3) &&
           tv_abs(P(line, 0) - Q(line, 0)) < ((5 * tc + 1) >> 1);
  };
  const bool strong = dsam(0, dpq0) && dsam(3, dpq3);
  const bool dEp = dp < ((beta + (beta >> 1)) >> 3);
  const bool dEq = dq < ((beta + (beta >> 1)) >> 3);
  for (int k = 0; k < 4; ++k) {
    const int p0 = P(k, 0), p1 = P(k, 1), p2 = P(k, 2), p3 = P(k, 3);
    const int q0 = Q(k, 0), q1 = Q(k, 1), q2 = Q(k, 2), q3 = Q(k, 3);
    if (strong) {
      P(k, 0) = (uint8_t)clip3(p0 - 2 * tc, p0 + 2 * tc, (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3);
      P(k, 1) = (uint8_t)clip3(p1 - 2 * tc, p1 + 2 * tc, (p2 + p1 + p0 + q0 + 2) >> 2);
      P(k, 2) = (uint8_t)clip3(p2 - 2 * tc, p2 + 2 * tc, (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3);
      Q(k, 0) = (uint8_t)clip3(q0 - 2 * tc, q0 + 2 * tc, (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3);
      Q(k, 1) = (uint8_t)clip3(q1 - 2 * tc, q1 + 2 * tc, (p0 + q0 + q1 + q2 + 2) >> 2);
      Q(k, 2) = (uint8_t)clip3(q2 - 2 * tc, q2 + 2 * tc, (p0 + q0 + q1 + 3 * q2 + 2 * q3 + 4) >> 3);
    } else {
      int delta = (9 * (q0 - p0) - 3 * (q1 - p1) + 8) >> 4;
      if (tv_abs(delta) < tc * 10) {
        delta = clip3(-tc, tc, delta);
        P(k, 0) = (uint8_t)clip_pixel(p0 + delta);
        Q(k, 0) = (uint8_t)clip_pixel(q0 - delta);
        if (dEp) {
          int dP = clip3(-(tc >> 1), tc >> 1, (((p2 + p0 + 1) >> 1) - p1 + delta) >> 1);
          P(k, 1) = (uint8_t)clip_pixel(p1 + dP);
        }
        if (dEq) {
          int dQ = clip3(-(tc >> 1), tc >> 1, (((q2 + q0 + 1) >> 1) - q1 - delta) >> 1);
          Q(k, 1) = (uint8_t)clip_pixel(q1 + dQ);
        }
      }
    }
  }
}

// Chroma deblocking of one edge segment of `len` lines (only for bs == 2).
TV_HD void deblock_chroma_edge(uint8_t* q0ptr, int xstep, int lstep, int len, int qpc) {
  const int tc = kTcTable[clip3(0, 53, qpc + 2)];
  if (tc == 0) return;
  for (int k = 0; k < len; ++k) {
    uint8_t* q0p = q0ptr + k * lstep;
    const int p0 = q0p[-xstep], p1 = q0p[-2 * xstep], q0 = q0p[0], q1 = q0p[xstep];
    const int delta = clip3(-tc, tc, ((((q0 - p0) * 4) + p1 - q1 + 4) >> 3));
    q0p[-xstep] = (uint8_t)clip_pixel(p0 + delta);
    q0p[0] = (uint8_t)clip_pixel(q0 - delta);
  }
}

// Boundary strength of the deblocking edge between luma positions P and Q (H.265 8.7.2.4)
// for this engine's structure (TB = PU = CU, one reference picture).  Arrays are the
// per-8x8-unit decision planes (see hevc_codec.h).  Returns 0 for edges inside a CU.
// B slices (dir != nullptr): the two lists hold different pictures (tv/gop.h), so the
// reference sets of P and Q match iff their directions do; then every used list's vectors
// are compared (8.7.2.4).
TV_HD int deblock_edge_bs(const uint8_t* cu_log2, const uint8_t* intra, const uint8_t* cbf,
                          const int16_t* mv, int w8, int xp, int yp, int xq, int yq,
                          const uint8_t* dir = nullptr, const int16_t* mv1 = nullptr,
                          const uint8_t* tu = nullptr) {
  const int up = (yp >> 3) * w8 + (xp >> 3), uq = (yq >> 3) * w8 + (xq >> 3);
  const int sp = cu_log2[up], sq = cu_log2[uq];
  if (sp == sq) {
    const int m = ~((1 << sp) - 1);
    if ((xp & m) == (xq & m) && (yp & m) == (yq & m)) {
      // inside one CU: an edge only between the TBs of an RQT-split inter CU (half its size;
      // one motion: bS 1 iff either TB has luma levels)
      if (!(tu && tu[up] && (((xp ^ xq) | (yp ^ yq)) & (1 << (sp - 1))))) return 0;
      return ((cbf[up] & 1) || (cbf[uq] & 1)) ? 1 : 0;
    }
  }
  if (intra[up] || intra[uq]) return 2;
  if ((cbf[up] & 1) || (cbf[uq] & 1)) return 1;
  auto differ = [&](const int16_t* v) {
    return tv_abs(v[2 * up] - v[2 * uq]) >= 4 || tv_abs(v[2 * up + 1] - v[2 * uq + 1]) >= 4;
  };
  if (!dir) return differ(mv) ? 1 : 0;
  const int d = dir[up];
  if (d != dir[uq]) return 1;
  if ((d & 1) && differ(mv)) return 1;
  if ((d & 2) && differ(mv1)) return 1;
  return 0;
}

// RQT decision of an inter 32x32 CU (CPU == GPU, before the transform): four 16x16 TBs when
// the luma residual is unevenly spread -- the cleanest quadrant's SAD is below half the
// busiest one's (and below kRqtClean per sample), so its TB can drop out (cbf 0) instead of
// spreading the busy quadrant's energy over a 32x32 transform.  Swept on the golden encoder
// (640x360, 32 frames, QP 22-37): -1.51 % BD-rate smooth, -1.15 % textured against no RQT;
// a quarter instead of half: -0.5 / -0.2 %.
constexpr int kRqtClean = 6;
constexpr int kRqtMinLog2 = 4;  // 32x32 and 16x16 inter CUs may split (TV_RQT16 experiments)
TV_HD bool rqt_split(const int* sad4, int npx = 256) {  // npx: samples per quadrant
  int lo = sad4[0], hi = sad4[0];
  for (int q = 1; q < 4; ++q) {
    lo = sad4[q] < lo ? sad4[q] : lo;
    hi = sad4[q] > hi ? sad4[q] : hi;
  }
  return 2 * lo < hi && lo < npx * kRqtClean;
}

// Rough bin count of an mvd pair (encoder cost model; CPU and GPU use the same).
TV_HD int mv_bits_est(int dx, int dy) {
  int bits = 0;
  for (int c = 0; c < 2; ++c) {
    int a = tv_abs(c ? dy : dx);
    if (a == 0) {
      bits += 1;
      continue;
    }
    int v = a + 1, n = 0;
    while (v > 1) {
      v >>= 1;
      ++n;
    }
    bits += 2 * n + 1;
  }
  return bits;
}

// ------------------------------------ scan orders ---------------------------------------
// 4x4 up-right diagonal scan: position i -> (x, y) packed as x | y<<2
constexpr uint8_t kScanDiag4x4[16] = {0, 4, 1, 8, 5, 2, 12, 9, 6, 3, 13, 10, 7, 14, 11, 15};
constexpr uint8_t kScanHor4x4[16] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15};
constexpr uint8_t kScanVer4x4[16] = {0, 4, 8, 12, 1, 5, 9, 13, 2, 6, 10, 14, 3, 7, 11, 15};
// 2x2 sub-block scans (for 8x8 TBs): packed x | y<<2
constexpr uint8_t kScanDiag2x2[4] = {0, 4, 1, 5};
constexpr uint8_t kScanHor2x2[4] = {0, 1, 4, 5};
constexpr uint8_t kScanVer2x2[4] = {0, 4, 1, 5};
// 8x8 diagonal sub-block scan (for 32x32 TBs): packed x | y<<3
struct Scan8 {
  uint8_t s[64];
};
constexpr Scan8 make_diag8() {
  Scan8 r{};
  int i = 0, x = 0, y = 0;
  while (i < 64) {
    while (y >= 0) {
      if (x < 8 && y < 8) r.s[i++] = (uint8_t)(x | (y << 3));
      --y;
      ++x;
    }
    y = x;
    x = 0;
  }
  return r;
}
constexpr Scan8 kScanDiag8x8 = make_diag8();
// 4x4 diagonal sub-block scan for 16x16 TBs: packed x | y<<2 (same as kScanDiag4x4)

// sub-block (xS,yS) of scan position i for a TB with log2 size L and scanIdx s
TV_HD void subblock_pos(int log2N, int scanIdx, int i, int& xs, int& ys) {
  if (log2N == 2) {
    xs = ys = 0;
  } else if (log2N == 3) {
    const uint8_t v = scanIdx == 0 ? kScanDiag2x2[i] : (scanIdx == 1 ? kScanHor2x2[i] : kScanVer2x2[i]);
    xs = v & 3;
    ys = v >> 2;
  } else if (log2N == 4) {
    xs = kScanDiag4x4[i] & 3;
    ys = kScanDiag4x4[i] >> 2;
  } else {
    xs = kScanDiag8x8.s[i] & 7;
    ys = kScanDiag8x8.s[i] >> 3;
  }
}
TV_HD void coef_pos_in_sb(int scanIdx, int n, int& x, int& y) {
  const uint8_t v = scanIdx == 0 ? kScanDiag4x4[n] : (scanIdx == 1 ? kScanHor4x4[n] : kScanVer4x4[n]);
  x = v & 3;
  y = v >> 2;
}

// scanIdx (H.265 7.4.9.11): mode dependent for intra 4x4/8x8 luma, 4x4 chroma (4:2:0)
TV_HD int scan_idx_for(bool intra, int log2TrafoSize, int cIdx, int predMode) {
  if (!intra) return 0;
  if (log2TrafoSize == 2 || (log2TrafoSize == 3 && cIdx == 0)) {
    if (predMode >= 6 && predMode <= 14) return 2;
    if (predMode >= 22 && predMode <= 30) return 1;
  }
  return 0;
}

// z-order index of a 4x4 unit inside a 32x32 CTB (x4,y4 in 0..7)
TV_HD int zorder4(int x4, int y4) {
  // bit interleave x2 y2 x1 y1 x0 y0 -> y2 x2 y1 x1 y0 x0
  return (x4 & 1) | ((y4 & 1) << 1) | ((x4 & 2) << 1) | ((y4 & 2) << 2) | ((x4 & 4) << 2) | ((y4 & 4) << 3);
}

// Availability of luma location (xN,yN) for the block at (xC,yC) (H.265 6.4.1), for a
// picture with a single slice and no tiles.
TV_HD bool zscan_available(int xC, int yC, int xN, int yN, int picW, int picH) {
  if (xN < 0 || yN < 0 || xN >= picW || yN >= picH) return false;
  const int wCtb = (picW + kCtb - 1) >> kCtbLog2;
  const int aN = (yN >> kCtbLog2) * wCtb + (xN >> kCtbLog2);
  const int aC = (yC >> kCtbLog2) * wCtb + (xC >> kCtbLog2);
  if (aN != aC) return aN < aC;
  const int zN = zorder4((xN & (kCtb - 1)) >> 2, (yN & (kCtb - 1)) >> 2);
  const int zC = zorder4((xC & (kCtb - 1)) >> 2, (yC & (kCtb - 1)) >> 2);
  return zN <= zC;
}

// ------------------------------------------------------------------------------ SAO
// Sample adaptive offset (H.265 7.3.8.3 / 8.7.3), 8-bit.  One CTB/component parameter set
// is packed in 32 bits: type (0 off, 1 band, 2 edge) | class (EO class or band position)
// << 2 | (offset[i] + 8) << (7 + 4 i), offsets in [-7, 7] with the EO sign convention
// (categories 1, 2 >= 0; 3, 4 <= 0) already applied.  Encoder decisions are integer RD so
// the CPU golden model and the GPU kernels choose identical parameters.
constexpr int kSaoMaxOff = 7;  // (1 << (Min(bitDepth, 10) - 5)) - 1
TV_HD uint32_t sao_pack(int type, int cls, const int* off) {
  uint32_t p = (uint32_t)type | ((uint32_t)cls << 2);
  for (int i = 0; i < 4; ++i) p |= (uint32_t)(off[i] + 8) << (7 + 4 * i);
  return p;
}
TV_HD int sao_type(uint32_t p) { return (int)(p & 3); }
TV_HD int sao_class(uint32_t p) { return (int)((p >> 2) & 31); }
TV_HD int sao_offset(uint32_t p, int i) { return (int)((p >> (7 + 4 * i)) & 15) - 8; }
TV_HD uint32_t sao_off_param() {
  const int z[4] = {0, 0, 0, 0};
  return sao_pack(0, 0, z);
}
// neighbour displacement of EO class c: (dx, dy) of sample a; sample b is the mirror
TV_HD void sao_eo_dir(int c, int& dx, int& dy) {
  dx = c == 1 ? 0 : (c == 3 ? 1 : -1);
  dy = c == 0 ? 0 : -1;
}
// EO category (0 = none, 1 local min .. 4 local max) of p against neighbours a, b
TV_HD int sao_eo_category(int p, int a, int b) {
  const int e = 2 + (p > a) - (p < a) + (p > b) - (p < b);
  return e == 2 ? 0 : (e < 2 ? e + 1 : e);
}
// one SAO'd sample from its deblocked value v and the two EO neighbours of the parameter
// set's class (a, b < 0: outside the picture -> the sample is left unchanged)
TV_HD int sao_sample_nb(int v, int a, int b, uint32_t p) {
  const int t = sao_type(p);
  if (t == 1) {
    const int k = ((v >> 3) - sao_class(p)) & 31;
    return k < 4 ? clip_pixel(v + sao_offset(p, k)) : v;
  }
  if (t == 2) {
    if (a < 0 || b < 0) return v;
    const int c = sao_eo_category(v, a, b);
    return c ? clip_pixel(v + sao_offset(p, c - 1)) : v;
  }
  return v;
}
// one SAO'd sample.  x, y: component coordinates; src: deblocked plane (w x h).
TV_HD int sao_sample(const uint8_t* src, int w, int h, int x, int y, uint32_t p) {
  const int v = src[y * w + x];
  if (sao_type(p) != 2) return sao_sample_nb(v, 0, 0, p);
  int dx, dy;
  sao_eo_dir(sao_class(p), dx, dy);
  const int ax = x + dx, ay = y + dy, bx = x - dx, by = y - dy;
  const bool in = !(ax < 0 || ay < 0 || bx < 0 || by < 0 || ax >= w || ay >= h || bx >= w || by >= h);
  return sao_sample_nb(v, in ? src[ay * w + ax] : -1, in ? src[by * w + bx] : -1, p);
}

// Statistics of one CTB component: count and sum(orig - deblocked) per EO class/category
// and per band.
struct SaoStats {
  int eo_n[4][5], eo_s[4][5];
  int bo_n[32], bo_s[32];
};
TV_HD int sao_tr_bits(int a) { return a < kSaoMaxOff ? a + 1 : kSaoMaxOff; }
// best offset for one category given (n, s): minimises 16*dSSE + lam16*bits; sign_lo/hi
// bound the allowed range; `sign_bit` adds one bit for non-zero values (band offsets).
TV_HD long long sao_best_offset(int n, int s, int lo, int hi, long long lam16, bool sign_bit, int& best) {
  best = 0;
  long long bj = lam16 * sao_tr_bits(0);
  if (n == 0) return bj;
  int o = (2 * s + (s >= 0 ? n : -n)) / (2 * n);  // round(s / n)
  o = o < lo ? lo : (o > hi ? hi : o);
  const int step = o > 0 ? -1 : 1;
  for (int v = o; v != 0; v += step) {
    const long long dd = (long long)n * v * v - 2LL * v * s;
    const long long j = 16 * dd + lam16 * (sao_tr_bits(v < 0 ? -v : v) + (sign_bit ? 1 : 0));
    if (j < bj) {
      bj = j;
      best = v;
    }
  }
  return bj;
}
// The decision runs in three data-parallel phases so a GPU block can spread it over its
// lanes while the CPU golden model runs the same steps in loops:
//   1. 144 independent items: the best offset + cost of every (component, EO class,
//      category) [3 x 16] and every (component, band) [3 x 32];
//   2. for every component and band position, the cost of the 4-band window [3 x 32];
//   3. the final choice per component (luma) / jointly for Cb+Cr (shared type + EO class).
struct SaoTables {
  long long eo_j[3][4][4];
  long long bo_j[3][32];
  long long win_j[3][32];
  int8_t eo_o[3][4][4];
  int8_t bo_o[3][32];
};
constexpr int kSaoItems = 3 * 48;
TV_HD void sao_item(const SaoStats* st, long long lam16, int idx, SaoTables& t) {
  const int c = idx / 48, r = idx % 48;
  int o;
  if (r < 16) {
    const int cls = r >> 2, k = r & 3;
    const bool pos = k < 2;  // categories 1, 2 >= 0; 3, 4 <= 0
    t.eo_j[c][cls][k] = sao_best_offset(st[c].eo_n[cls][k + 1], st[c].eo_s[cls][k + 1], pos ? 0 : -kSaoMaxOff,
                                        pos ? kSaoMaxOff : 0, lam16, false, o);
    t.eo_o[c][cls][k] = (int8_t)o;
  } else {
    const int b = r - 16;
    t.bo_j[c][b] = sao_best_offset(st[c].bo_n[b], st[c].bo_s[b], -kSaoMaxOff, kSaoMaxOff, lam16, true, o);
    t.bo_o[c][b] = (int8_t)o;
  }
}
TV_HD void sao_window(int idx, SaoTables& t) {  // idx in [0, 96)
  const int c = idx / 32, p = idx % 32;
  long long j = 0;
  for (int k = 0; k < 4; ++k) j += t.bo_j[c][(p + k) & 31];
  t.win_j[c][p] = j;
}
TV_HD int sao_best_band(const SaoTables& t, int c) {
  int best = 0;
  for (int p = 1; p < 32; ++p)
    if (t.win_j[c][p] < t.win_j[c][best]) best = p;
  return best;
}
TV_HD uint32_t sao_pack_eo(const SaoTables& t, int c, int cls) {
  int off[4];
  for (int k = 0; k < 4; ++k) off[k] = t.eo_o[c][cls][k];
  return sao_pack(2, cls, off);
}
TV_HD uint32_t sao_pack_bo(const SaoTables& t, int c, int pos) {
  int off[4];
  for (int k = 0; k < 4; ++k) off[k] = t.bo_o[c][(pos + k) & 31];
  return sao_pack(1, pos, off);
}
TV_HD long long sao_eo_j(const SaoTables& t, int c, int cls) {
  return t.eo_j[c][cls][0] + t.eo_j[c][cls][1] + t.eo_j[c][cls][2] + t.eo_j[c][cls][3];
}
// Band offsets are not chosen: with this RD estimate they cost more than they gain (golden,
// 640x360, 32 frames, QP 22-37: dropping them -1.04 % BD-rate smooth, -0.38 % textured) and
// their statistics were a third of k_sao_decide's statistics phase (LDS histogram atomics).
constexpr bool kSaoBandOffsets = false;
// Rate in bits: type TR bins (off 1, band 2, edge 2), EO class 2, band position 5, offsets.
// the final choice given each component's best band position (sao_best_band; the GPU finds
// it with a wave-parallel argmin)
TV_HD void sao_finish_pos(const SaoTables& t, long long lam16, const int* pos, uint32_t* out) {
  {  // luma
    long long best = lam16 * 1;
    out[0] = sao_off_param();
    for (int cls = 0; cls < 4; ++cls) {
      const long long j = sao_eo_j(t, 0, cls) + lam16 * 4;
      if (j < best) {
        best = j;
        out[0] = sao_pack_eo(t, 0, cls);
      }
    }
    if (kSaoBandOffsets && t.win_j[0][pos[0]] + lam16 * 7 < best) out[0] = sao_pack_bo(t, 0, pos[0]);
  }
  {  // chroma: one type (and EO class) for Cb and Cr
    long long best = lam16 * 1;
    out[1] = out[2] = sao_off_param();
    for (int cls = 0; cls < 4; ++cls) {
      const long long j = sao_eo_j(t, 1, cls) + sao_eo_j(t, 2, cls) + lam16 * 4;
      if (j < best) {
        best = j;
        out[1] = sao_pack_eo(t, 1, cls);
        out[2] = sao_pack_eo(t, 2, cls);
      }
    }
    if (kSaoBandOffsets && t.win_j[1][pos[1]] + t.win_j[2][pos[2]] + lam16 * 12 < best) {
      out[1] = sao_pack_bo(t, 1, pos[1]);
      out[2] = sao_pack_bo(t, 2, pos[2]);
    }
  }
}
TV_HD void sao_finish(const SaoTables& t, long long lam16, uint32_t* out) {
  int pos[3];
  for (int c = 0; c < 3; ++c) pos[c] = sao_best_band(t, c);
  sao_finish_pos(t, lam16, pos, out);
}
// Sequential form of the three phases (CPU golden model).
inline void sao_decide(const SaoStats* st, long long lam16, uint32_t* out) {
  SaoTables t;
  for (int i = 0; i < kSaoItems; ++i) sao_item(st, lam16, i, t);
  for (int i = 0; i < 96; ++i) sao_window(i, t);
  sao_finish(t, lam16, out);
}
// lambda for SSE-domain decisions in 1/16 units (lam_sse = lam_sad^2)
inline long long sao_lambda16(int qp) {
  const double l = 0.57 * std::pow(2.0, (qp - 12) / 3.0);
  return (long long)(l * 16.0);
}

}  // namespace tv
