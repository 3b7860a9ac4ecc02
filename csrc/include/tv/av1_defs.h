// av1_defs.h — AV1 in-loop filter arithmetic shared by the C++ golden model (av1_tools.cpp)
// and the gfx950 kernels (k_av1.hip): CDEF direction search + filter, Wiener and
// self-guided loop restoration (BASELINE config #4).
//
// Everything is integer and written once as TV_HD functions, so GPU == CPU bit for bit.
// 8-bit video only (BitDepth 8: coeff_shift 0, InterRound0 3 / InterRound1 11).
#pragma once
#include <cstdint>

#include "tv/hevc_defs.h"  // TV_HD, clip3, tv_abs

namespace tv {
namespace av1 {

// ------------------------------------------------------------------------------ CDEF ----
// Direction offsets (dy, dx) of the primary taps k = 0, 1 for the 8 directions.
TV_HD int cdef_dir_dy(int d, int k) {
  constexpr int8_t t[8][2] = {{-1, -2}, {0, -1}, {0, 0}, {0, 1}, {1, 2}, {1, 2}, {1, 2}, {1, 2}};
  return t[d & 7][k];
}
TV_HD int cdef_dir_dx(int d, int k) {
  constexpr int8_t t[8][2] = {{1, 2}, {1, 2}, {1, 2}, {1, 2}, {1, 2}, {0, 1}, {0, 0}, {0, -1}};
  return t[d & 7][k];
}
TV_HD int floor_log2(unsigned v) { return v ? 31 - __builtin_clz(v) : -1; }

// Partial-sum bin of pixel (i = row, j = col) of an 8x8 block for direction d.
TV_HD int cdef_bin(int d, int i, int j) {
  switch (d) {
    case 0: return i + j;
    case 1: return i + (j >> 1);
    case 2: return i;
    case 3: return 3 + i - (j >> 1);
    case 4: return 7 + i - j;
    case 5: return 3 - (i >> 1) + j;
    case 6: return j;
    default: return (i >> 1) + j;
  }
}

// Direction cost from the 15 partial sums (of pixel - 128) of direction d.
TV_HD int cdef_cost(const int* partial /* [15] */, int d) {
  constexpr int div[9] = {0, 840, 420, 280, 210, 168, 140, 120, 105};
  int cost = 0;
  if (d == 2 || d == 6) {
    for (int i = 0; i < 8; ++i) cost += partial[i] * partial[i];
    return cost * div[8];
  }
  if (d == 0 || d == 4) {
    for (int i = 0; i < 7; ++i) cost += (partial[i] * partial[i] + partial[14 - i] * partial[14 - i]) * div[i + 1];
    return cost + partial[7] * partial[7] * div[8];
  }
  for (int j = 0; j < 5; ++j) cost += partial[3 + j] * partial[3 + j];
  cost *= div[8];
  for (int j = 0; j < 3; ++j) cost += (partial[j] * partial[j] + partial[10 - j] * partial[10 - j]) * div[2 * j + 2];
  return cost;
}

// best direction (first maximum) and variance from the 8 costs
TV_HD int cdef_pick(const int* cost, int* var) {
  int best = 0, bc = cost[0];
  for (int d = 1; d < 8; ++d)
    if (cost[d] > bc) {
      bc = cost[d];
      best = d;
    }
  *var = (bc - cost[(best + 4) & 7]) >> 10;
  return best;
}

TV_HD int cdef_constrain(int diff, int threshold, int damping) {
  if (!threshold) return 0;
  const int adj = damping - floor_log2((unsigned)threshold);
  const int a = tv_abs(diff);
  int lim = threshold - (a >> (adj > 0 ? adj : 0));
  lim = lim > 0 ? lim : 0;
  const int v = a < lim ? a : lim;
  return diff < 0 ? -v : v;
}

// luma primary strength adjusted by the block variance
TV_HD int cdef_adjust_strength(int strength, int var) {
  if (!var) return 0;
  int i = (var >> 6) ? floor_log2((unsigned)(var >> 6)) : 0;
  i = i < 12 ? i : 12;
  return (strength * (4 + i) + 8) >> 4;
}

// Filter one pixel with value c.  get(dy, dx) returns the neighbour sample or -1 when it
// is unavailable (outside the frame).  `pri`/`sec` are final strengths (sec in {0,1,2,4}).
template <class G>
TV_HD int cdef_filter(G get, int c, int pri, int sec, int damping, int dir) {
  int sum = 0, mx = c, mn = c;
  const int pt = pri & 1;
  for (int k = 0; k < 2; ++k) {
    const int ptap = pt ? 3 : (k ? 2 : 4);
    const int stap = k ? 1 : 2;
    for (int sg = -1; sg <= 1; sg += 2) {
      if (pri) {
        const int v = get(sg * cdef_dir_dy(dir, k), sg * cdef_dir_dx(dir, k));
        if (v >= 0) {
          sum += ptap * cdef_constrain(v - c, pri, damping);
          mx = v > mx ? v : mx;
          mn = v < mn ? v : mn;
        }
      }
      if (!sec) continue;
      for (int off = -2; off <= 2; off += 4) {
        const int d2 = (dir + off) & 7;
        const int v = get(sg * cdef_dir_dy(d2, k), sg * cdef_dir_dx(d2, k));
        if (v >= 0) {
          sum += stap * cdef_constrain(v - c, sec, damping);
          mx = v > mx ? v : mx;
          mn = v < mn ? v : mn;
        }
      }
    }
  }
  const int y0 = c + ((8 + sum - (sum < 0)) >> 4);
  return clip3(mn, mx, y0);
}

// plane form: pixel (x, y) of a w x h plane with pitch p
TV_HD int cdef_filter_pixel(const uint8_t* P, int p, int w, int h, int x, int y, int pri, int sec, int damping,
                            int dir) {
  auto get = [=](int dy, int dx) -> int {
    const int yy = y + dy, xx = x + dx;
    return (xx >= 0 && xx < w && yy >= 0 && yy < h) ? (int)P[(long)yy * p + xx] : -1;
  };
  return cdef_filter(get, (int)P[(long)y * p + x], pri, sec, damping, dir);
}

// CDEF strength preset: index = pri * 4 + sec_idx; sec_idx 3 means strength 4.
TV_HD int cdef_sec_value(int sec_idx) { return sec_idx == 3 ? 4 : sec_idx; }
// Direction-array flag of an 8x8 block whose four 4x4 units are all skip (7.15 cdef_block:
// such blocks are not filtered); set by the callers that know the block modes.
constexpr int kCdefSkipBlock = 0x80;
// 7.15.1: the filter direction is the block's direction unless the preset's (unadjusted)
// primary strength is 0, then 0 (the secondary taps still run along directions 2 / 6)
TV_HD int cdef_dir_used(int preset, int d) { return (preset >> 2) == 0 ? 0 : (d & 7); }
constexpr int kCdefPresets = 64;  // 16 primary x 4 secondary
constexpr uint64_t kCdefSkipped = 1ull << 40;  // SSE reported for presets a search skipped

// ------------------------------------------------------------------ loop restoration ----
constexpr int kWienerTaps = 7;
constexpr int kRound0 = 3, kRound1 = 11;  // 8-bit: InterRound0 / InterRound1 (sum = 2 * FILTER_BITS)
TV_HD int wiener_min(int k) { return k == 0 ? -5 : (k == 1 ? -23 : -17); }
TV_HD int wiener_max(int k) { return k == 0 ? 10 : (k == 1 ? 8 : 46); }
TV_HD int wiener_tap(const int* c3 /* c0, c1, c2 */, int t) {
  if (t == 3) return 128 - 2 * (c3[0] + c3[1] + c3[2]);
  return c3[t < 3 ? t : 6 - t];
}
// horizontal stage: value stored in the 16-bit intermediate; get(t) = sample at x + t - 3
template <class G>
TV_HD int wiener_h(G get, const int* hc) {
  int s = 0;
  for (int t = 0; t < kWienerTaps; ++t) s += wiener_tap(hc, t) * get(t);
  const int off = 1 << (8 + 7 - kRound0 - 1), lim = (1 << (8 + 1 + 7 - kRound0)) - 1;
  return clip3(-off, lim - off, (s + (1 << (kRound0 - 1))) >> kRound0);
}
// 1-D 7-tap filter of 8-bit samples back to the 8-bit scale (/128, no clipping): the fixed
// direction of the separable Wiener least-squares passes
template <class G>
TV_HD int lr_tap_filter(G get, const int* c3) {
  int s = 0;
  for (int t = 0; t < kWienerTaps; ++t) s += wiener_tap(c3, t) * get(t);
  return (s + 64) >> 7;
}
TV_HD int wiener_v(const int* col /* 7 intermediates, stride cs */, int cs, const int* vc) {
  int s = 0;
  for (int t = 0; t < kWienerTaps; ++t) s += wiener_tap(vc, t) * col[t * cs];
  return clip3(0, 255, (s + (1 << (kRound1 - 1))) >> kRound1);
}

// Self-guided restoration: parameter sets {r0, s0, r1, s1} (radius, scale of each pass).
TV_HD int sgr_param(int set, int k) {
  constexpr int16_t t[16][4] = {{2, 140, 1, 3236}, {2, 112, 1, 2158}, {2, 93, 1, 1618}, {2, 80, 1, 1438},
                                {2, 70, 1, 1295},  {2, 58, 1, 1177},  {2, 47, 1, 1079}, {2, 37, 1, 996},
                                {2, 30, 1, 925},   {2, 25, 1, 863},   {0, -1, 1, 2589}, {0, -1, 1, 1618},
                                {0, -1, 1, 1177},  {0, -1, 1, 925},   {2, 56, 0, -1},   {2, 22, 0, -1}};
  return t[set & 15][k];
}
constexpr int kSgrMtableBits = 20, kSgrSgrBits = 8, kSgrRecipBits = 12, kSgrRstBits = 4, kSgrPrjBits = 7;

// x_by_xplus1: 256 * z / (z + 1) rounded, 1 at 0, 256 from 255 on
TV_HD int sgr_xbyx1(unsigned z) {
  if (z >= 255) return 256;
  if (z == 0) return 1;
  return (int)(((z << kSgrSgrBits) + (z / 2)) / (z + 1));
}
// (a, b) guide coefficients of one pixel from its (2r+1)^2 box sum / square sum; `xb(z)`
// evaluates sgr_xbyx1 (the GPU passes a lookup in an LDS table of it)
// `s` is the parameter set's scale (the Sgr_Params entry next to the radius: the table holds
// the scale factor itself, not an epsilon)
template <class XB>
TV_HD void sgr_ab_x(int sum, int sq, int r, int s_param, XB xb, int* A, int* B) {
  const int n = (2 * r + 1) * (2 * r + 1);
  const unsigned s = (unsigned)s_param;
  const long long p0 = (long long)sq * n - (long long)sum * sum;
  const unsigned p = p0 > 0 ? (unsigned)p0 : 0u;
  const unsigned z = (unsigned)(((unsigned long long)p * s + (1u << (kSgrMtableBits - 1))) >> kSgrMtableBits);
  const int a2 = xb(z);
  const int one_over_n = ((1 << kSgrRecipBits) + n / 2) / n;
  // 8-bit: (256 - a2) * sum * one_over_n <= 255 * 6375 * 164 < 2^31, so B < 2^16 and both
  // coefficients fit 16-bit storage (the GPU keeps them as uint16 in LDS)
  const int b2 = ((1 << kSgrSgrBits) - a2) * sum * one_over_n;
  *A = a2;
  *B = (b2 + (1 << (kSgrRecipBits - 1))) >> kSgrRecipBits;
}
struct SgrXbDiv {
  TV_HD int operator()(unsigned z) const { return sgr_xbyx1(z); }
};
TV_HD void sgr_ab(int sum, int sq, int r, int s, int* A, int* B) { sgr_ab_x(sum, sq, r, s, SgrXbDiv{}, A, B); }

// projection of the two guided outputs (flt = filtered << RST_BITS domain) onto the pixel
TV_HD int sgr_project(int x, int f0, int f1, int r0, int r1, int w0, int w1) {
  const int u = x << kSgrRstBits;
  int v = u << kSgrPrjBits;
  if (r0) v += w0 * (f0 - u);
  if (r1) v += w1 * (f1 - u);
  const int s = kSgrRstBits + kSgrPrjBits;
  return clip3(0, 255, (v + (1 << (s - 1))) >> s);
}


// ------------------------------------------------ normative self-guided restoration ----
// 7.17 with 64x64 restoration units (lr_unit_shift 0, lr_uv_shift 0) and 4:2:0 chroma
// (ss = 1): units are counted with rounding (the last row / column of units absorbs up to
// half a unit), unit rows are offset 8 luma rows up, and the filters read the CDEF output
// inside the current 64-luma-row stripe (also offset by 8) and up to 2 rows of the
// deblocked, pre-CDEF frame beyond it.
TV_HD int lr_count_units(int size) { int n = (size + 32) / 64; return n > 1 ? n : 1; }
TV_HD int lr_unit_row(int y, int h, int ss) {
  const int r = (y + (8 >> ss)) / 64, n = lr_count_units(h);
  return r < n ? r : n - 1;
}
TV_HD int lr_unit_col(int x, int w) {
  const int c = x / 64, n = lr_count_units(w);
  return c < n ? c : n - 1;
}
// rows [y0, y1) of unit row ur / columns [x0, x1) of unit column uc
TV_HD void lr_unit_rows(int ur, int h, int ss, int* y0, int* y1) {
  const int off = 8 >> ss, n = lr_count_units(h);
  *y0 = ur ? ur * 64 - off : 0;
  *y1 = ur == n - 1 ? h : (ur + 1) * 64 - off;
}
TV_HD void lr_unit_cols(int uc, int w, int* x0, int* x1) {
  *x0 = uc * 64;
  *x1 = uc == lr_count_units(w) - 1 ? w : (uc + 1) * 64;
}
// stripe of row y: first row StripeStartY and last row StripeEndY (may lie outside the plane)
TV_HD int lr_stripe_start(int y, int ss) {
  const int S = 64 >> ss, off = 8 >> ss;
  return ((y + off) / S) * S - off;
}
// get_source_sample: the plane row that feeds (x, y) of the stripe [s0, s0 + S) and whether
// it comes from the deblocked (pre-CDEF) frame
TV_HD int lr_src_row(int y, int h, int s0, int ss, bool* dbk) {
  const int s1 = s0 + (64 >> ss) - 1;
  y = clip3(0, h - 1, y);
  *dbk = false;
  if (y < s0) {
    *dbk = true;
    return y > s0 - 2 ? y : s0 - 2;
  }
  if (y > s1) {
    *dbk = true;
    return y < s1 + 2 ? y : s1 + 2;
  }
  return y;
}
// guided-filter output of pixel (row y, value c) from the 3x3 (A, B) neighbourhood (pass 0:
// radius-2 filter, (A, B) used on odd rows only; pass 1: radius 1, all rows).  getA(dy, dx)
// / getB(dy, dx) read the neighbour's coefficients.
template <class GA, class GB>
TV_HD int sgr_output(int pass, int y, int c, GA getA, GB getB) {
  int a = 0, b = 0, shift = 5;
  if (pass == 0) {
    if (y & 1) shift = 4;
    for (int dy = -1; dy <= 1; ++dy) {
      if (!((y + dy) & 1)) continue;
      for (int dx = -1; dx <= 1; ++dx) {
        const int wt = dx == 0 ? 6 : 5;
        a += wt * getA(dy, dx);
        b += wt * getB(dy, dx);
      }
    }
  } else {
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        const int wt = (dy == 0 || dx == 0) ? 4 : 3;
        a += wt * getA(dy, dx);
        b += wt * getB(dy, dx);
      }
  }
  const int s = kSgrSgrBits + shift - kSgrRstBits;
  return (a * c + b + (1 << (s - 1))) >> s;
}
// projection with the coded weights (7.17.? self guided filter process): w0 = xqd0 weights
// F0, w1 = xqd1 weights the CDEF sample u, w2 = 128 - w0 - w1 weights F1 (a radius-0 pass
// contributes u instead)
TV_HD int sgr_project_xqd(int x, int f0, int f1, int r0, int r1, int xqd0, int xqd1) {
  const int u = x << kSgrRstBits, w2 = (1 << kSgrPrjBits) - xqd0 - xqd1;
  const int v = xqd1 * u + xqd0 * (r0 ? f0 : u) + w2 * (r1 ? f1 : u);
  const int s = kSgrRstBits + kSgrPrjBits;
  return clip3(0, 255, (v + (1 << (s - 1))) >> s);
}

// ------------------------------------------------------------ deblocking loop filter ----
// One 32-bit info word per 4x4 unit of a plane (row-major, w/4 per row):
//   bits 0-2  log2(tx width) - 2      bits 3-5   log2(tx height) - 2
//   bits 6-8  log2(block width) - 2   bits 9-11  log2(block height) - 2
//   bits 12-17 filter level for vertical edges, 18-23 for horizontal edges (0..63)
//   bit 24    skip && is_inter (internal tx edges of such blocks are not filtered)
// Transform and coding blocks are aligned to their size (true for every AV1 partition), so
// "x is a tx / block edge" is x % size == 0.
TV_HD int lf_tx(uint32_t i, int pass) { return 4 << ((i >> (pass ? 3 : 0)) & 7); }
TV_HD int lf_bs(uint32_t i, int pass) { return 4 << ((i >> (pass ? 9 : 6)) & 7); }
TV_HD int lf_lvl(uint32_t i, int pass) { return (int)((i >> (pass ? 18 : 12)) & 63); }

// Filter length of the edge between 4x4 units `prev` (p side) and `cur` (q side) whose q
// side starts at `pos` (x for pass 0 = vertical edges, y for pass 1) in a plane of extent
// `dim` along the filter: 0 = not filtered, else 4 / 6 (chroma) / 8 / 16 (luma 13-tap).
// AV1 7.14.2 / 7.14.3: tx edge, block edge or not (skip && inter), level fallback to the
// p side, size = min of both tx sizes capped at 16 (luma) / 6 (chroma).  Sizes are also
// capped so the taps stay inside the plane (only reachable with a tx map crossing the
// frame edge).
TV_HD int lf_edge(uint32_t prev, uint32_t cur, int pos, int dim, int pass, int chroma, int* lvl) {
  const int ts = lf_tx(cur, pass);
  if (pos <= 0 || pos % ts) return 0;
  if ((cur >> 24 & 1) && pos % lf_bs(cur, pass)) return 0;
  int l = lf_lvl(cur, pass);
  if (!l) l = lf_lvl(prev, pass);
  if (!l) return 0;
  *lvl = l;
  const int ps = lf_tx(prev, pass);
  int fs = ts < ps ? ts : ps;
  if (chroma) return fs >= 8 && pos >= 3 && pos + 3 <= dim ? 6 : 4;
  if (fs >= 16 && pos >= 7 && pos + 7 <= dim) return 16;
  if (fs >= 8 && pos >= 4 && pos + 4 <= dim) return 8;
  return 4;
}

TV_HD int lf_s8(int v) { return v < -128 ? -128 : (v > 127 ? 127 : v); }

// AV1 7.14.6: filter one line of an edge.  q0 points at the first q-side pixel, `step` is
// the distance between taps (1 for a vertical edge, the pitch for a horizontal one).  Every
// loop bound is a template constant, so the tap arrays live in registers (a runtime-sized
// version spilled them to scratch memory in the GPU deblocking kernel).
template <int n, int log2, int n2> TV_HD void lf_wide(uint8_t* q0, int step, const int* p, const int* q) {
  // wide filter (7.14.6.4): n taps modified per side, weight 2 within |j| <= n2
  int F[14];  // F[7 + k]: k >= 0 -> q[k], k < 0 -> p[-k-1]
#pragma unroll
  for (int k = 0; k <= n; ++k) {
    F[7 + k] = q[k];
    F[6 - k] = p[k];
  }
  int o[12];
#pragma unroll
  for (int i = -n; i < n; ++i) {
    int t = 0;
#pragma unroll
    for (int j = -n; j <= n; ++j) {
      const int k = clip3(-(n + 1), n, i + j);
      t += F[7 + k] * ((j <= n2 && j >= -n2) ? 2 : 1);
    }
    o[i + n] = (t + (1 << (log2 - 1))) >> log2;
  }
#pragma unroll
  for (int i = -n; i < n; ++i) q0[i * step] = (uint8_t)o[i + n];
}

template <int SIZE> TV_HD void lf_filter_n(uint8_t* q0, int step, int lvl, int sharp) {
  const int shift = sharp > 4 ? 2 : (sharp > 0 ? 1 : 0);
  int limit = lvl >> shift;
  limit = sharp > 0 ? clip3(1, 9 - sharp, limit) : (limit < 1 ? 1 : limit);
  const int blimit = 2 * (lvl + 2) + limit, thresh = lvl >> 4;
  constexpr int nr = SIZE == 16 ? 7 : (SIZE == 8 ? 4 : (SIZE == 6 ? 3 : 2));  // taps read per side
  constexpr int lm = SIZE == 4 ? 2 : (SIZE == 6 ? 3 : 4);
  int p[7], q[7];
#pragma unroll
  for (int k = 0; k < nr; ++k) {
    q[k] = q0[k * step];
    p[k] = q0[-(k + 1) * step];
  }
  bool mask = tv_abs(p[0] - q[0]) * 2 + (tv_abs(p[1] - q[1]) >> 1) <= blimit;
#pragma unroll
  for (int k = 1; k < lm; ++k) mask = mask && tv_abs(p[k] - p[k - 1]) <= limit && tv_abs(q[k] - q[k - 1]) <= limit;
  if (!mask) return;
  bool flat = SIZE >= 6;
#pragma unroll
  for (int k = 1; k < lm; ++k) flat = flat && tv_abs(p[k] - p[0]) <= 1 && tv_abs(q[k] - q[0]) <= 1;
  if (!flat) {  // narrow filter (7.14.6.3)
    const bool hev = tv_abs(p[1] - p[0]) > thresh || tv_abs(q[1] - q[0]) > thresh;
    const int ps1 = p[1] - 128, ps0 = p[0] - 128, qs0 = q[0] - 128, qs1 = q[1] - 128;
    int f = hev ? lf_s8(ps1 - qs1) : 0;
    f = lf_s8(f + 3 * (qs0 - ps0));
    const int f1 = lf_s8(f + 4) >> 3, f2 = lf_s8(f + 3) >> 3;
    q0[0] = (uint8_t)(lf_s8(qs0 - f1) + 128);
    q0[-step] = (uint8_t)(lf_s8(ps0 + f2) + 128);
    if (!hev) {
      const int f3 = (f1 + 1) >> 1;
      q0[step] = (uint8_t)(lf_s8(qs1 - f3) + 128);
      q0[-2 * step] = (uint8_t)(lf_s8(ps1 + f3) + 128);
    }
    return;
  }
  if constexpr (SIZE == 16) {
    bool flat2 = true;
#pragma unroll
    for (int k = 4; k < 7; ++k) flat2 = flat2 && tv_abs(p[k] - p[0]) <= 1 && tv_abs(q[k] - q[0]) <= 1;
    if (flat2) lf_wide<6, 4, 1>(q0, step, p, q);
    else lf_wide<3, 3, 0>(q0, step, p, q);
  } else if constexpr (SIZE == 8) {
    lf_wide<3, 3, 0>(q0, step, p, q);
  } else if constexpr (SIZE == 6) {
    lf_wide<2, 3, 1>(q0, step, p, q);
  }
}

TV_HD void lf_filter(uint8_t* q0, int step, int size, int lvl, int sharp) {
  switch (size) {
    case 16: lf_filter_n<16>(q0, step, lvl, sharp); break;
    case 8: lf_filter_n<8>(q0, step, lvl, sharp); break;
    case 6: lf_filter_n<6>(q0, step, lvl, sharp); break;
    default: lf_filter_n<4>(q0, step, lvl, sharp); break;
  }
}

}  // namespace av1
}  // namespace tv
