// av1_tools.cpp — C++ golden model of the AV1 tools: CDEF
// direction search / filter / strength search, Wiener and self-guided loop restoration
// with their least-squares statistics, and the AV1 range coder.  The per-pixel arithmetic
// lives in tv/av1_defs.h and is shared with the gfx950 kernels (csrc/gpu/k_av1.hip).
#include "tv/av1.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <thread>
#include <vector>
#include <stdexcept>
#include <string>

#include "tv/av1_defs.h"

namespace tv {
namespace av1 {

// ========================================================================== CDEF ======
void cdef_find_dirs(const uint8_t* Y, int w, int h, uint8_t* dir, int* var) {
  const int w8 = w / 8, h8 = h / 8;
  for (int by = 0; by < h8; ++by)
    for (int bx = 0; bx < w8; ++bx) {
      int partial[8][15] = {};
      for (int i = 0; i < 8; ++i)
        for (int j = 0; j < 8; ++j) {
          const int x = (int)Y[(long)(by * 8 + i) * w + bx * 8 + j] - 128;
          for (int d = 0; d < 8; ++d) partial[d][cdef_bin(d, i, j)] += x;
        }
      int cost[8];
      for (int d = 0; d < 8; ++d) cost[d] = cdef_cost(partial[d], d);
      int v;
      dir[by * w8 + bx] = (uint8_t)cdef_pick(cost, &v);
      var[by * w8 + bx] = v;
    }
}

namespace {
// filter block (64x64 luma, 32x32 chroma) geometry
inline int fb_size(bool chroma) { return chroma ? 32 : 64; }
inline int nfb_of(int w, int h, bool chroma) {
  const int f = fb_size(chroma);
  return ((w + f - 1) / f) * ((h + f - 1) / f);
}
// final strengths of block (bx, by) for preset index p
inline void block_strengths(int p, bool chroma, int v, int& pri, int& sec) {
  pri = p >> 2;
  sec = cdef_sec_value(p & 3);
  if (!chroma) pri = cdef_adjust_strength(pri, v);
}
}  // namespace

void cdef_search(const uint8_t* src, const uint8_t* rec, int w, int h, bool chroma, const uint8_t* dir,
                 const int* var, int luma_w8, int damping, uint64_t* sse, uint64_t pmask, bool checker) {
  const int bs = chroma ? 4 : 8, fbs = fb_size(chroma), nfx = (w + fbs - 1) / fbs;
  const int dmp = chroma ? damping - 1 : damping;
  std::memset(sse, 0, sizeof(uint64_t) * nfb_of(w, h, chroma) * kCdefPresets);
  // bands of filter-block rows on separate threads (each writes only its own fb rows)
  const int nband = (h + fbs - 1) / fbs;
  const int nt = std::max(1, std::min(nband, (int)std::thread::hardware_concurrency()));
  std::atomic<int> next{0};
  auto band = [&](int fr) {
    for (int by = fr * fbs / bs; by < std::min(h / bs, (fr + 1) * fbs / bs); ++by)
    for (int bx = 0; bx < w / bs; ++bx) {
      if (checker && ((bx + by) & 1)) continue;  // encoder search on a checkerboard of blocks
      const int d0 = dir[by * luma_w8 + bx], v = var[by * luma_w8 + bx];
      uint64_t* S = sse + (long)((by * bs / fbs) * nfx + bx * bs / fbs) * kCdefPresets;
      for (int p = 0; p < kCdefPresets; ++p) {
        if (!(pmask >> p & 1)) {
          S[p] = kCdefSkipped;
          continue;
        }
        int pri, sec;
        block_strengths(p, chroma, v, pri, sec);
        if (d0 & kCdefSkipBlock) pri = sec = 0;  // skip blocks are not filtered
        const int d = cdef_dir_used(p, d0);
        uint64_t acc = 0;
        for (int i = 0; i < bs; ++i)
          for (int j = 0; j < bs; ++j) {
            const int x = bx * bs + j, y = by * bs + i;
            const int f = (pri | sec) ? cdef_filter_pixel(rec, w, w, h, x, y, pri, sec, dmp, d) : rec[(long)y * w + x];
            const int e = f - (int)src[(long)y * w + x];
            acc += (uint64_t)(e * e);
          }
        S[p] += acc;
      }
    }
  };
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t)
    th.emplace_back([&] {
      for (int r; (r = next.fetch_add(1)) < nband;) band(r);
    });
  for (auto& x : th) x.join();
}

void cdef_apply(const uint8_t* rec, int w, int h, bool chroma, const uint8_t* dir, const int* var, int luma_w8,
                int damping, const int8_t* fb_preset, uint8_t* out) {
  const int bs = chroma ? 4 : 8, fbs = fb_size(chroma), nfx = (w + fbs - 1) / fbs;
  const int dmp = chroma ? damping - 1 : damping;
  for (int by = 0; by < h / bs; ++by)
    for (int bx = 0; bx < w / bs; ++bx) {
      const int p = fb_preset[(by * bs / fbs) * nfx + bx * bs / fbs];
      const int d0 = dir[by * luma_w8 + bx], v = var[by * luma_w8 + bx];
      int pri = 0, sec = 0;
      if (p >= 0 && !(d0 & kCdefSkipBlock)) block_strengths(p, chroma, v, pri, sec);
      const int d = cdef_dir_used(p, d0);
      for (int i = 0; i < bs; ++i)
        for (int j = 0; j < bs; ++j) {
          const int x = bx * bs + j, y = by * bs + i;
          out[(long)y * w + x] = (uint8_t)((pri | sec) ? cdef_filter_pixel(rec, w, w, h, x, y, pri, sec, dmp, d)
                                                       : rec[(long)y * w + x]);
        }
    }
}

// ============================================================== loop restoration ======
namespace {
inline int units_x(int w) { return (w + kRu - 1) / kRu; }
inline int nunits(int w, int h) { return units_x(w) * ((h + kRu - 1) / kRu); }
inline int unit_of(int x, int y, int w) { return (y / kRu) * units_x(w) + x / kRu; }
inline int px(const uint8_t* P, int w, int h, int x, int y) {
  return P[(size_t)clip3(0, h - 1, y) * w + clip3(0, w - 1, x)];
}
}  // namespace

// Each 64x64 unit is filtered with its own taps in both directions, including the three
// rows / columns of context beyond the unit (edge-replicated at the frame border).
void wiener_apply(const uint8_t* rec, int w, int h, const int* coef, uint8_t* out) {
  int mid[70][kRu];
  for (int uy = 0; uy < h; uy += kRu)
    for (int ux = 0; ux < w; ux += kRu) {
      const int* c = coef + 6 * unit_of(ux, uy, w);
      const int uw = std::min(kRu, w - ux), uh = std::min(kRu, h - uy);
      const bool id = !(c[0] | c[1] | c[2] | c[3] | c[4] | c[5]);
      for (int r = 0; r < uh + 6; ++r)
        for (int j = 0; j < uw; ++j)
          mid[r][j] = wiener_h([&](int t) { return px(rec, w, h, ux + j + t - 3, uy + r - 3); }, c);
      for (int i = 0; i < uh; ++i)
        for (int j = 0; j < uw; ++j) {
          const size_t o = (size_t)(uy + i) * w + ux + j;
          out[o] = id ? rec[o] : (uint8_t)wiener_v(&mid[i][j], kRu, c + 3);
        }
    }
}

void wiener_stats(const uint8_t* src, const uint8_t* rec, int w, int h, int dir, const int* other, int64_t* stats) {
  std::memset(stats, 0, sizeof(int64_t) * 9 * nunits(w, h));
  for (int uy = 0; uy < h; uy += kRu)
    for (int ux = 0; ux < w; ux += kRu) {
      const int u = unit_of(ux, uy, w);
      const int* c = other + 3 * u;
      const int uw = std::min(kRu, w - ux), uh = std::min(kRu, h - uy);
      // z = rec filtered with the unit's fixed taps of the other direction
      auto Z = [&](int x, int y) {
        return dir == 0 ? lr_tap_filter([&](int t) { return px(rec, w, h, x, y + t - 3); }, c)
                        : lr_tap_filter([&](int t) { return px(rec, w, h, x + t - 3, y); }, c);
      };
      int64_t* S = stats + 9 * u;
      for (int i = 0; i < uh; ++i)
        for (int j = 0; j < uw; ++j) {
          const int x = ux + j, y = uy + i;
          auto at = [&](int d) { return dir == 0 ? Z(clip3(0, w - 1, x + d), y) : Z(x, clip3(0, h - 1, y + d)); };
          const int zc = at(0);
          int f[3];
          for (int k = 0; k < 3; ++k) f[k] = at(k - 3) + at(3 - k) - 2 * zc;
          const int64_t e = 128 * ((int)src[(size_t)y * w + x] - zc);
          S[0] += f[0] * f[0];
          S[1] += f[0] * f[1];
          S[2] += f[0] * f[2];
          S[3] += f[1] * f[1];
          S[4] += f[1] * f[2];
          S[5] += f[2] * f[2];
          S[6] += f[0] * e;
          S[7] += f[1] * e;
          S[8] += f[2] * e;
        }
    }
}

namespace {
// box sum / square sum of radius r around (x, y), edge-clamped
inline void box(const uint8_t* P, int w, int h, int x, int y, int r, int& sum, int& sq) {
  sum = sq = 0;
  for (int dy = -r; dy <= r; ++dy)
    for (int dx = -r; dx <= r; ++dx) {
      const int v = P[(size_t)clip3(0, h - 1, y + dy) * w + clip3(0, w - 1, x + dx)];
      sum += v;
      sq += v * v;
    }
}
void guided(const uint8_t* P, int w, int h, int r, int eps, int32_t* F) {
  std::vector<int> A((size_t)w * h), B((size_t)w * h);
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      int s, q;
      box(P, w, h, x, y, r, s, q);
      sgr_ab(s, q, r, eps, &A[(size_t)y * w + x], &B[(size_t)y * w + x]);
    }
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      int a = 0, b = 0;
      for (int dy = -1; dy <= 1; ++dy)
        for (int dx = -1; dx <= 1; ++dx) {
          const int wt = (dx && dy) ? 3 : 4;
          const size_t k = (size_t)clip3(0, h - 1, y + dy) * w + clip3(0, w - 1, x + dx);
          a += wt * A[k];
          b += wt * B[k];
        }
      const int s = kSgrSgrBits + 5 - kSgrRstBits;
      F[(size_t)y * w + x] = (a * (int)P[(size_t)y * w + x] + b + (1 << (s - 1))) >> s;
    }
}
}  // namespace

void sgr_filter_planes(const uint8_t* rec, int w, int h, int set, int32_t* f0, int32_t* f1) {
  const int r0 = sgr_param(set, 0), r1 = sgr_param(set, 2);
  for (long i = 0; i < (long)w * h; ++i) f0[i] = f1[i] = (int)rec[i] << kSgrRstBits;
  if (r0) guided(rec, w, h, r0, sgr_param(set, 1), f0);
  if (r1) guided(rec, w, h, r1, sgr_param(set, 3), f1);
}

void sgr_apply(const uint8_t* rec, int w, int h, const int* params, uint8_t* out) {
  std::vector<int32_t> f0((size_t)w * h), f1((size_t)w * h);
  // units may use different sets: filter once per distinct set
  std::vector<int> sets;
  for (int u = 0; u < nunits(w, h); ++u)
    if (params[3 * u] >= 0 && std::find(sets.begin(), sets.end(), params[3 * u]) == sets.end())
      sets.push_back(params[3 * u]);
  std::memcpy(out, rec, (size_t)w * h);
  for (int set : sets) {
    sgr_filter_planes(rec, w, h, set, f0.data(), f1.data());
    const int r0 = sgr_param(set, 0), r1 = sgr_param(set, 2);
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        const int* p = params + 3 * unit_of(x, y, w);
        if (p[0] != set) continue;
        const size_t i = (size_t)y * w + x;
        out[i] = (uint8_t)sgr_project(rec[i], f0[i], f1[i], r0, r1, p[1], p[2]);
      }
  }
}

void sgr_stats(const uint8_t* src, const uint8_t* rec, int w, int h, int set, int64_t* stats) {
  std::vector<int32_t> f0((size_t)w * h), f1((size_t)w * h);
  sgr_filter_planes(rec, w, h, set, f0.data(), f1.data());
  std::memset(stats, 0, sizeof(int64_t) * 5 * nunits(w, h));
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      const size_t i = (size_t)y * w + x;
      const int u = (int)rec[i] << kSgrRstBits;
      const int64_t a = f0[i] - u, b = f1[i] - u;
      const int64_t e = (((int64_t)src[i] << kSgrRstBits) - u) << kSgrPrjBits;
      int64_t* S = stats + 5 * unit_of(x, y, w);
      S[0] += a * a;
      S[1] += a * b;
      S[2] += b * b;
      S[3] += a * e;
      S[4] += b * e;
    }
}

// ------------------------------------------------- normative self-guided restoration ----
void sgr_flt(const uint8_t* cdef, const uint8_t* dbk, int w, int h, int ss, int set, int32_t* f0, int32_t* f1) {
  const int S = 64 >> ss, off = 8 >> ss;
  for (long i = 0; i < (long)w * h; ++i) f0[i] = f1[i] = (int)cdef[i] << kSgrRstBits;
  std::vector<int> A, B;
  for (int s0 = -off; s0 < h; s0 += S) {  // stripes: rows [max(0, s0), min(h, s0 + S))
    const int y0 = std::max(0, s0), y1 = std::min(h, s0 + S);
    if (y0 >= y1) continue;
    auto src = [&](int x, int y) -> int {
      bool db;
      const int yy = lr_src_row(y, h, s0, ss, &db);
      return (db ? dbk : cdef)[(size_t)yy * w + clip3(0, w - 1, x)];
    };
    const int ah = y1 - y0 + 2, aw = w + 2;  // (A, B) rows y0-1 .. y1, columns -1 .. w
    for (int pass = 0; pass < 2; ++pass) {
      const int r = sgr_param(set, 2 * pass), eps = sgr_param(set, 2 * pass + 1);
      if (!r) continue;
      A.assign((size_t)ah * aw, 0);
      B.assign((size_t)ah * aw, 0);
      for (int i = 0; i < ah; ++i)
        for (int j = 0; j < aw; ++j) {
          const int y = y0 - 1 + i, x = j - 1;
          int sum = 0, sq = 0;
          for (int dy = -r; dy <= r; ++dy)
            for (int dx = -r; dx <= r; ++dx) {
              const int v = src(x + dx, y + dy);
              sum += v;
              sq += v * v;
            }
          sgr_ab(sum, sq, r, eps, &A[(size_t)i * aw + j], &B[(size_t)i * aw + j]);
        }
      int32_t* F = pass ? f1 : f0;
      for (int y = y0; y < y1; ++y)
        for (int x = 0; x < w; ++x) {
          const size_t c = (size_t)(y - y0 + 1) * aw + x + 1;
          F[(size_t)y * w + x] = sgr_output(
              pass, y, cdef[(size_t)y * w + x], [&](int dy, int dx) { return A[c + dy * aw + dx]; },
              [&](int dy, int dx) { return B[c + dy * aw + dx]; });
        }
    }
  }
}

void lr_apply(const uint8_t* cdef, const uint8_t* dbk, int w, int h, int ss, const int* params, uint8_t* out) {
  const int ux = lr_count_units(w), uy = lr_count_units(h);
  std::vector<int> sets;
  for (int u = 0; u < ux * uy; ++u)
    if (params[3 * u] >= 0 && std::find(sets.begin(), sets.end(), params[3 * u]) == sets.end())
      sets.push_back(params[3 * u]);
  std::memcpy(out, cdef, (size_t)w * h);
  std::vector<int32_t> f0((size_t)w * h), f1((size_t)w * h);
  for (int set : sets) {
    sgr_flt(cdef, dbk, w, h, ss, set, f0.data(), f1.data());
    const int r0 = sgr_param(set, 0), r1 = sgr_param(set, 2);
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        const int* p = params + 3 * (lr_unit_row(y, h, ss) * ux + lr_unit_col(x, w));
        if (p[0] != set) continue;
        const size_t i = (size_t)y * w + x;
        out[i] = (uint8_t)sgr_project_xqd(cdef[i], f0[i], f1[i], r0, r1, p[1], p[2]);
      }
  }
}

void lr_stats(const uint8_t* src, const uint8_t* cdef, const uint8_t* dbk, int w, int h, int ss, int set,
              int64_t* stats) {
  const int ux = lr_count_units(w), uy = lr_count_units(h);
  std::vector<int32_t> f0((size_t)w * h), f1((size_t)w * h);
  sgr_flt(cdef, dbk, w, h, ss, set, f0.data(), f1.data());
  std::memset(stats, 0, sizeof(int64_t) * 5 * ux * uy);
  for (int y = 0; y < h; ++y)
    for (int x = 0; x < w; ++x) {
      const size_t i = (size_t)y * w + x;
      const int u = (int)cdef[i] << kSgrRstBits;
      const int64_t a = f0[i] - u, b = f1[i] - u;
      const int64_t e = (((int64_t)src[i] << kSgrRstBits) - u) << kSgrPrjBits;
      int64_t* S = stats + 5 * (lr_unit_row(y, h, ss) * ux + lr_unit_col(x, w));
      S[0] += a * a;
      S[1] += a * b;
      S[2] += b * b;
      S[3] += a * e;
      S[4] += b * e;
    }
}

// ================================================================== range coder ======

// ---------------------------------------------------------------- deblocking loop filter ----
// AV1 7.14: every vertical edge of the plane (pass 0), then every horizontal edge (pass 1).
// Edges of one pass never share a tap (a size-n filter needs tx >= n on both sides), so the
// raster order inside a pass does not matter; the GPU kernel relies on the same property.
void deblock(const uint8_t* in, int w, int h, bool chroma, const uint32_t* info, int sharp, uint8_t* out) {
  if (w % 4 || h % 4) throw std::invalid_argument("deblock: plane dims must be multiples of 4");
  std::memcpy(out, in, (size_t)w * h);
  const int w4 = w / 4;
  for (int y = 0; y < h; ++y)
    for (int x = 4; x < w; x += 4) {
      const uint32_t* row = info + (size_t)(y / 4) * w4;
      int lvl = 0;
      const int size = lf_edge(row[x / 4 - 1], row[x / 4], x, w, 0, chroma, &lvl);
      if (size) lf_filter(out + (size_t)y * w + x, 1, size, lvl, sharp);
    }
  for (int y = 4; y < h; y += 4)
    for (int x = 0; x < w; ++x) {
      int lvl = 0;
      const int size = lf_edge(info[(size_t)(y / 4 - 1) * w4 + x / 4], info[(size_t)(y / 4) * w4 + x / 4], y, h, 1,
                               chroma, &lvl);
      if (size) lf_filter(out + (size_t)y * w + x, w, size, lvl, sharp);
    }
}

void cdf_init_uniform(uint16_t* icdf, int n) {
  if (n < 2 || n > 16) throw std::runtime_error("cdf: 2..16 symbols");
  for (int i = 0; i < n; ++i) icdf[i] = (uint16_t)(32768 - ((i + 1) * 32768 + n / 2) / n);
  icdf[n - 1] = 0;
  icdf[n] = 0;
}

namespace {
constexpr int kProbShift = 6, kMinProb = 4;
inline int ilog(uint32_t v) { return 32 - __builtin_clz(v); }
inline uint32_t bound(uint32_t r, int icdf_v, int n, int k) {
  return ((r >> 8) * (uint32_t)(icdf_v >> kProbShift) >> (7 - kProbShift)) + kMinProb * (n - 1 - k);
}
}  // namespace

size_t RangeEncoder::bits_written() const { return pre_.size() * 8 + (size_t)(cnt_ + 10); }

std::vector<uint8_t> RangeEncoder::finish() {
  // round low up to a value that identifies the final interval with the fewest bytes
  uint64_t l = low_;
  int c = cnt_, s = 10;
  const uint64_t m = 0x3FFF;
  uint64_t e = ((l + m) & ~m) | (m + 1);
  s += c;
  std::vector<uint16_t> buf = pre_;
  if (s > 0) {
    uint64_t n = (1ull << (c + 16)) - 1;
    do {
      buf.push_back((uint16_t)(e >> (c + 16)));
      e &= n;
      s -= 8;
      c -= 8;
      n >>= 8;
    } while (s > 0);
  }
  std::vector<uint8_t> out(buf.size());
  uint32_t carry = 0;
  for (size_t i = buf.size(); i-- > 0;) {
    carry = buf[i] + carry;
    out[i] = (uint8_t)carry;
    carry >>= 8;
  }
  return out;
}

namespace {
constexpr int kWindow = 64;
}

RangeDecoder::RangeDecoder(const uint8_t* data, size_t size) : p_(data), end_(data + size) {
  dif_ = (1ull << (kWindow - 1)) - 1;
  rng_ = 0x8000;
  cnt_ = -15;
  refill();
}

void RangeDecoder::refill() {
  int s = kWindow - 9 - (cnt_ + 15);
  for (; s >= 0 && p_ < end_; s -= 8, ++p_) {
    dif_ ^= (uint64_t)p_[0] << s;
    cnt_ += 8;
  }
  if (p_ >= end_) cnt_ = 0x4000;  // past the end: zeros (already in dif as complemented ones)
}

void RangeDecoder::normalize(uint32_t r) {
  const int d = 16 - ilog(r);
  cnt_ -= d;
  dif_ = ((dif_ + 1) << d) - 1;
  rng_ = r << d;
  if (cnt_ < 0) refill();
}

int RangeDecoder::decode(uint16_t* icdf, int n, bool adapt) {
  const uint32_t r = rng_;
  const uint32_t c = (uint32_t)(dif_ >> (kWindow - 16));
  uint32_t u, v = r;
  int k = -1;
  do {
    u = v;
    ++k;
    v = bound(r, icdf[k], n, k);
  } while (c < v);
  dif_ -= (uint64_t)v << (kWindow - 16);
  normalize(u - v);
  if (adapt) cdf_adapt(icdf, n, k);
  return k;
}

int RangeDecoder::decode_bool(int p0_q15) {
  uint16_t icdf[3] = {(uint16_t)(32768 - clip3(1, 32767, p0_q15)), 0, 0};
  return decode(icdf, 2, false);
}

uint32_t RangeDecoder::decode_literal(int bits) {
  uint32_t v = 0;
  for (int b = 0; b < bits; ++b) v = (v << 1) | (uint32_t)decode_bool(16384);
  return v;
}

}  // namespace av1
}  // namespace tv

// ================================================================== C API ============
namespace {
thread_local std::string g_av1_err;
template <class F> int av1_guard(F&& f) {
  try {
    f();
    return 0;
  } catch (const std::exception& e) {
    g_av1_err = e.what();
    return -1;
  }
}
}  // namespace

extern "C" {
using namespace tv::av1;
const char* tv_av1_last_error() { return g_av1_err.c_str(); }
void tv_av1_cdef_find_dirs(const uint8_t* Y, int w, int h, uint8_t* dir, int* var) { cdef_find_dirs(Y, w, h, dir, var); }
void tv_av1_cdef_search(const uint8_t* src, const uint8_t* rec, int w, int h, int chroma, const uint8_t* dir,
                        const int* var, int luma_w8, int damping, uint64_t* sse) {
  cdef_search(src, rec, w, h, chroma != 0, dir, var, luma_w8, damping, sse, ~0ull, false);
}
void tv_av1_cdef_apply(const uint8_t* rec, int w, int h, int chroma, const uint8_t* dir, const int* var, int luma_w8,
                       int damping, const int8_t* fb_preset, uint8_t* out) {
  cdef_apply(rec, w, h, chroma != 0, dir, var, luma_w8, damping, fb_preset, out);
}
void tv_av1_wiener_apply(const uint8_t* rec, int w, int h, const int* coef, uint8_t* out) {
  wiener_apply(rec, w, h, coef, out);
}
void tv_av1_wiener_stats(const uint8_t* src, const uint8_t* rec, int w, int h, int dir, const int* other,
                         int64_t* stats) {
  wiener_stats(src, rec, w, h, dir, other, stats);
}
void tv_av1_sgr_apply(const uint8_t* rec, int w, int h, const int* params, uint8_t* out) {
  sgr_apply(rec, w, h, params, out);
}
void tv_av1_sgr_stats(const uint8_t* src, const uint8_t* rec, int w, int h, int set, int64_t* stats) {
  sgr_stats(src, rec, w, h, set, stats);
}
int tv_av1_deblock(const uint8_t* in, int w, int h, int chroma, const uint32_t* info, int sharp, uint8_t* out) {
  return av1_guard([&] { deblock(in, w, h, chroma != 0, info, sharp, out); });
}
void tv_av1_sgr_filter_planes(const uint8_t* rec, int w, int h, int set, int32_t* f0, int32_t* f1) {
  sgr_filter_planes(rec, w, h, set, f0, f1);
}

// Range coder round trip driver: encode n symbols (alphabet sizes alpha[i], values sym[i];
// adaptive contexts ctx[i] in [0, nctx)) -> bytes; decode them back into `dec`.
int tv_av1_rc_roundtrip(const int* sym, const int* alpha, const int* ctx, int n, int nctx, int adapt, void* out_bytes,
                        int* dec) {
  return av1_guard([&] {
    std::vector<std::vector<uint16_t>> cdf(nctx, std::vector<uint16_t>(17));
    std::vector<int> csize(nctx, 0);
    RangeEncoder enc;
    for (int i = 0; i < n; ++i) {
      auto& c = cdf[ctx[i]];
      if (!csize[ctx[i]]) {
        cdf_init_uniform(c.data(), alpha[i]);
        csize[ctx[i]] = alpha[i];
      }
      enc.encode(sym[i], c.data(), alpha[i], adapt != 0);
    }
    auto bytes = enc.finish();
    auto* v = static_cast<std::vector<uint8_t>*>(out_bytes);
    v->assign(bytes.begin(), bytes.end());
    std::fill(csize.begin(), csize.end(), 0);
    RangeDecoder d(bytes.data(), bytes.size());
    for (int i = 0; i < n; ++i) {
      auto& c = cdf[ctx[i]];
      if (!csize[ctx[i]]) {
        cdf_init_uniform(c.data(), alpha[i]);
        csize[ctx[i]] = alpha[i];
      }
      dec[i] = d.decode(c.data(), alpha[i], adapt != 0);
    }
  });
}
}

// ================================================================ AV1 transforms ======
#include "tv/av1_txfm.h"

namespace tv {
namespace av1 {
namespace {
inline int32_t rshift_round(int64_t v, int s) { return (int32_t)((v + (1LL << (s - 1))) >> s); }
inline int32_t clamp16(int32_t v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }
}  // namespace

// Golden 2-D transform of nblk N x N blocks (row-major int16): forward (columns then rows)
// or inverse (rows then columns), same integer stages as k_av1_txfm.hip.
void txfm2d_ref(const int16_t* in, int16_t* out, int nblk, int log2N, int tcol, int trow, bool inverse) {
  const int N = 1 << log2N;
  if (!txfm_valid(tcol, N) || !txfm_valid(trow, N)) throw std::runtime_error("av1 txfm: bad type/size");
  std::vector<int32_t> Bc(N * N), Br(N * N), t(N * N);
  for (int k = 0; k < N; ++k)
    for (int n = 0; n < N; ++n) {
      Bc[k * N + n] = txfm_basis(tcol, N, k, n);
      Br[k * N + n] = txfm_basis(trow, N, k, n);
    }
  int f1, f2, i1, i2;
  txfm_shifts(log2N, f1, f2, i1, i2);
  for (int b = 0; b < nblk; ++b) {
    const int16_t* X = in + (size_t)b * N * N;
    int16_t* Y = out + (size_t)b * N * N;
    for (int r = 0; r < N; ++r)
      for (int c = 0; c < N; ++c) {
        int64_t s = 0;
        for (int k = 0; k < N; ++k)
          s += inverse ? (int64_t)X[r * N + k] * Br[k * N + c]    // g[r][c] = sum_j C[r][j] Br[j][c]
                       : (int64_t)Bc[r * N + k] * X[k * N + c];   // tmp[r][c] = sum_y Bc[r][y] X[y][c]
        t[r * N + c] = clamp16(rshift_round(s, inverse ? i1 : f1));
      }
    for (int r = 0; r < N; ++r)
      for (int c = 0; c < N; ++c) {
        int64_t s = 0;
        for (int k = 0; k < N; ++k)
          s += inverse ? (int64_t)Bc[k * N + r] * t[k * N + c]    // X[r][c] = sum_k Bc[k][r] g[k][c]
                       : (int64_t)t[r * N + k] * Br[c * N + k];   // C[r][c] = sum_x tmp[r][x] Br[c][x]
        Y[r * N + c] = (int16_t)clamp16(rshift_round(s, inverse ? i2 : f2));
      }
  }
}

}  // namespace av1
}  // namespace tv

extern "C" {
int tv_av1_txfm_ref(const int16_t* in, int16_t* out, int nblk, int log2N, int tcol, int trow, int inverse) {
  return av1_guard([&] { tv::av1::txfm2d_ref(in, out, nblk, log2N, tcol, trow, inverse != 0); });
}
int tv_av1_txfm_basis(int type, int N, int32_t* out) {
  if (!tv::av1::txfm_valid(type, N)) return -1;
  for (int k = 0; k < N; ++k)
    for (int n = 0; n < N; ++n) out[k * N + n] = tv::av1::txfm_basis(type, N, k, n);
  return 0;
}
}
