// mpeg2.cpp — MPEG-2 video decoder + fixture writer (see tv/mpeg2.h).
#include "tv/mpeg2.h"
#include "mpeg2_wtab.h"

#include <algorithm>
#include <array>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <string>

namespace tv::mpeg2 {
const char* const kStatNames[kNumStats] = {
    "intra", "p_mc", "p_no_mc", "b_fwd", "b_bwd", "b_bi", "p_skipped", "b_skipped", "frame_mc", "field_mc_frame_pic",
    "field_mc_field_pic", "mc_16x8", "field_dct", "escapes", "quant_changes", "intra_blocks", "inter_blocks",
    "concealed_slices"};

namespace {

[[noreturn]] void fail(const std::string& m) { throw std::runtime_error("mpeg2: " + m); }

// ---------------------------------------------------------------- tables (Annex B) ------
struct Vc {
  uint16_t code;
  uint8_t len;
};

// B.14 / B.15 by run: the codes of levels 1.. (sign bit not included)
struct RunRow {
  int n;
  Vc c[40];
};
const RunRow kB14[32] = {
    {40, {{3, 2},     {4, 4},     {5, 5},     {6, 7},     {0x26, 8},  {0x21, 8},  {0xa, 10},  {0x1d, 12},
          {0x18, 12}, {0x13, 12}, {0x10, 12}, {0x1a, 13}, {0x19, 13}, {0x18, 13}, {0x17, 13}, {0x1f, 14},
          {0x1e, 14}, {0x1d, 14}, {0x1c, 14}, {0x1b, 14}, {0x1a, 14}, {0x19, 14}, {0x18, 14}, {0x17, 14},
          {0x16, 14}, {0x15, 14}, {0x14, 14}, {0x13, 14}, {0x12, 14}, {0x11, 14}, {0x10, 14}, {0x18, 15},
          {0x17, 15}, {0x16, 15}, {0x15, 15}, {0x14, 15}, {0x13, 15}, {0x12, 15}, {0x11, 15}, {0x10, 15}}},
    {18, {{3, 3},     {6, 6},     {0x25, 8},  {0xc, 10},  {0x1b, 12}, {0x16, 13}, {0x15, 13}, {0x1f, 15},
          {0x1e, 15}, {0x1d, 15}, {0x1c, 15}, {0x1b, 15}, {0x1a, 15}, {0x19, 15}, {0x13, 16}, {0x12, 16},
          {0x11, 16}, {0x10, 16}}},
    {5, {{5, 4}, {4, 7}, {0xb, 10}, {0x14, 12}, {0x14, 13}}},
    {4, {{7, 5}, {0x24, 8}, {0x1c, 12}, {0x13, 13}}},
    {3, {{6, 5}, {0xf, 10}, {0x12, 12}}},
    {3, {{7, 6}, {9, 10}, {0x12, 13}}},
    {3, {{5, 6}, {0x1e, 12}, {0x14, 16}}},
    {2, {{4, 6}, {0x15, 12}}},
    {2, {{7, 7}, {0x11, 12}}},
    {2, {{5, 7}, {0x11, 13}}},
    {2, {{0x27, 8}, {0x10, 13}}},
    {2, {{0x23, 8}, {0x1a, 16}}},
    {2, {{0x22, 8}, {0x19, 16}}},
    {2, {{0x20, 8}, {0x18, 16}}},
    {2, {{0xe, 10}, {0x17, 16}}},
    {2, {{0xd, 10}, {0x16, 16}}},
    {2, {{8, 10}, {0x15, 16}}},
    {1, {{0x1f, 12}}},
    {1, {{0x1a, 12}}},
    {1, {{0x19, 12}}},
    {1, {{0x17, 12}}},
    {1, {{0x16, 12}}},
    {1, {{0x1f, 13}}},
    {1, {{0x1e, 13}}},
    {1, {{0x1d, 13}}},
    {1, {{0x1c, 13}}},
    {1, {{0x1b, 13}}},
    {1, {{0x1f, 16}}},
    {1, {{0x1e, 16}}},
    {1, {{0x1d, 16}}},
    {1, {{0x1c, 16}}},
    {1, {{0x1b, 16}}},
};
// B.15 differs from B.14 for runs 0..16 (levels 16.. of run 0 and 8.. of run 1 are shared)
const RunRow kB15Low[17] = {
    {15, {{2, 2}, {6, 3}, {7, 4}, {0x1c, 5}, {0x1d, 5}, {5, 6}, {4, 6}, {0x7b, 7}, {0x7c, 7}, {0x23, 8},
          {0x22, 8}, {0xfa, 8}, {0xfb, 8}, {0xfe, 8}, {0xff, 8}}},
    {7, {{2, 3}, {6, 5}, {0x79, 7}, {0x27, 8}, {0x20, 8}, {0x16, 13}, {0x15, 13}}},
    {5, {{5, 5}, {7, 7}, {0xfc, 8}, {0xc, 10}, {0x14, 13}}},
    {4, {{7, 5}, {0x26, 8}, {0x1c, 12}, {0x13, 13}}},
    {3, {{6, 6}, {0xfd, 8}, {0x12, 12}}},
    {3, {{7, 6}, {4, 9}, {0x12, 13}}},
    {3, {{6, 7}, {0x1e, 12}, {0x14, 16}}},
    {2, {{4, 7}, {0x15, 12}}},
    {2, {{5, 7}, {0x11, 12}}},
    {2, {{0x78, 7}, {0x11, 13}}},
    {2, {{0x7a, 7}, {0x10, 13}}},
    {2, {{0x21, 8}, {0x1a, 16}}},
    {2, {{0x25, 8}, {0x19, 16}}},
    {2, {{0x24, 8}, {0x18, 16}}},
    {2, {{5, 9}, {0x17, 16}}},
    {2, {{7, 9}, {0x16, 16}}},
    {2, {{0xd, 10}, {0x15, 16}}},
};
constexpr Vc kEob14{2, 2}, kEob15{6, 4}, kEsc{1, 6};

// B.1 macroblock_address_increment 1..33, escape = +33
const Vc kMba[34] = {{0, 0},     {1, 1},     {3, 3},     {2, 3},     {3, 4},     {2, 4},     {3, 5},
                     {2, 5},     {7, 7},     {6, 7},     {0xb, 8},   {0xa, 8},   {9, 8},     {8, 8},
                     {7, 8},     {6, 8},     {0x17, 10}, {0x16, 10}, {0x15, 10}, {0x14, 10}, {0x13, 10},
                     {0x12, 10}, {0x23, 11}, {0x22, 11}, {0x21, 11}, {0x20, 11}, {0x1f, 11}, {0x1e, 11},
                     {0x1d, 11}, {0x1c, 11}, {0x1b, 11}, {0x1a, 11}, {0x19, 11}, {0x18, 11}};
constexpr Vc kMbaEscape{8, 11};

// macroblock_type flags
enum { MQ = 1, MF = 2, MB = 4, MP = 8, MI = 16 };
struct TypeCode {
  Vc c;
  int flags;
};
const TypeCode kTypeI[] = {{{1, 1}, MI}, {{1, 2}, MI | MQ}};
const TypeCode kTypeP[] = {{{1, 1}, MF | MP}, {{1, 2}, MP},          {{1, 3}, MF},
                           {{3, 5}, MI},      {{2, 5}, MF | MP | MQ}, {{1, 5}, MP | MQ},
                           {{1, 6}, MI | MQ}};
const TypeCode kTypeB[] = {{{2, 2}, MF | MB},           {{3, 2}, MF | MB | MP}, {{2, 3}, MB},
                           {{3, 3}, MB | MP},           {{2, 4}, MF},           {{3, 4}, MF | MP},
                           {{3, 5}, MI},                {{2, 5}, MF | MB | MP | MQ},
                           {{3, 6}, MF | MP | MQ},      {{2, 6}, MB | MP | MQ}, {{1, 6}, MI | MQ}};

// B.9 coded_block_pattern (4:2:0), indexed by the pattern
const Vc kCbp[64] = {
    {1, 9},    {0xb, 5},  {9, 5},    {0xd, 6},  {0xd, 4},  {0x17, 7}, {0x13, 7}, {0x1f, 8}, {0xc, 4},  {0x16, 7},
    {0x12, 7}, {0x1e, 8}, {0x13, 5}, {0x1b, 8}, {0x17, 8}, {0x13, 8}, {0xb, 4},  {0x15, 7}, {0x11, 7}, {0x1d, 8},
    {0x11, 5}, {0x19, 8}, {0x15, 8}, {0x11, 8}, {0xf, 6},  {0xf, 8},  {0xd, 8},  {3, 9},    {0xf, 5},  {0xb, 8},
    {7, 8},    {7, 9},    {0xa, 4},  {0x14, 7}, {0x10, 7}, {0x1c, 8}, {0xe, 6},  {0xe, 8},  {0xc, 8},  {2, 9},
    {0x10, 5}, {0x18, 8}, {0x14, 8}, {0x10, 8}, {0xe, 5},  {0xa, 8},  {6, 8},    {6, 9},    {0x12, 5}, {0x1a, 8},
    {0x16, 8}, {0x12, 8}, {0xd, 5},  {9, 8},    {5, 8},    {5, 9},    {0xc, 5},  {8, 8},    {4, 8},    {4, 9},
    {7, 3},    {0xa, 5},  {8, 5},    {0xc, 6}};
// B.10 motion_code magnitude 0..16 (a sign bit follows non-zero codes)
const Vc kMotion[17] = {{1, 1},   {1, 2},   {1, 3},   {1, 4},    {3, 6},    {5, 7},    {4, 7},    {3, 7},   {0xb, 9},
                        {0xa, 9}, {9, 9},   {0x11, 10}, {0x10, 10}, {0xf, 10}, {0xe, 10}, {0xd, 10}, {0xc, 10}};
// B.12 / B.13 dct_dc_size
const Vc kDcLuma[12] = {{4, 3}, {0, 2}, {1, 2}, {5, 3}, {6, 3}, {0xe, 4}, {0x1e, 5}, {0x3e, 6},
                        {0x7e, 7}, {0xfe, 8}, {0x1fe, 9}, {0x1ff, 9}};
const Vc kDcChroma[12] = {{0, 2},    {1, 2},    {2, 2},     {6, 3},     {0xe, 4},    {0x1e, 5},
                          {0x3e, 6}, {0x7e, 7}, {0xfe, 8}, {0x1fe, 9}, {0x3fe, 10}, {0x3ff, 10}};

const uint8_t kScan[2][64] = {
    {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
     41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
     30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63},
    {0,  8,  16, 24, 1,  9,  2,  10, 17, 25, 32, 40, 48, 56, 57, 49, 41, 33, 26, 18, 3,  11,
     4,  12, 19, 27, 34, 42, 50, 58, 35, 43, 51, 59, 20, 28, 5,  13, 6,  14, 21, 29, 36, 44,
     52, 60, 37, 45, 53, 61, 22, 30, 7,  15, 23, 31, 38, 46, 54, 62, 39, 47, 55, 63}};
const uint8_t kDefaultIntra[64] = {8,  16, 19, 22, 26, 27, 29, 34, 16, 16, 22, 24, 27, 29, 34, 37,
                                   19, 22, 26, 27, 29, 34, 34, 38, 22, 22, 26, 27, 29, 34, 37, 40,
                                   22, 26, 27, 29, 32, 35, 40, 48, 26, 27, 29, 32, 35, 40, 48, 58,
                                   26, 27, 29, 34, 38, 46, 56, 69, 27, 29, 35, 38, 46, 56, 69, 83};
const uint8_t kNonLinearQ[32] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  10, 12, 14, 16,  18,  20,  22,
                                 24, 28, 32, 36, 40, 44, 48, 52, 56, 64, 72, 80, 88, 96, 104, 112};
const int kFrameRate[9][2] = {{0, 1}, {24000, 1001}, {24, 1}, {25, 1}, {30000, 1001}, {30, 1}, {50, 1}, {60000, 1001}, {60, 1}};

// ---------------------------------------------------------------- VLC lookup ------------
// peek(bits) -> (len << 16) | (value + 32768); len 0 = invalid
struct Lut {
  int bits = 0;
  std::vector<uint32_t> t;
  void init(int b) {
    bits = b;
    t.assign(size_t(1) << b, 0);
  }
  void add(Vc c, int value) {
    if (c.len > bits) fail("lut width");
    const uint32_t lo = uint32_t(c.code) << (bits - c.len), n = 1u << (bits - c.len);
    for (uint32_t k = 0; k < n; ++k) {
      if (t[lo + k]) fail("ambiguous code table");
      t[lo + k] = (uint32_t(c.len) << 16) | uint32_t(value + 32768);
    }
  }
};

// DCT coefficient table: entry = len | run << 5 | (level + 2048) << 11 | kind << 24
enum { kCoef = 0, kEobK = 1, kEscK = 2 };
struct CoefLut {
  std::vector<uint32_t> t;  // 16-bit peek
  Vc enc[32][41];           // (run, level) -> code; len 0 = escape
  Vc eob;
  void build(bool b15) {
    t.assign(1 << 16, 0);
    std::memset(enc, 0, sizeof(enc));
    auto add = [&](Vc c, int run, int level, int kind) {
      const uint32_t lo = uint32_t(c.code) << (16 - c.len), n = 1u << (16 - c.len);
      for (uint32_t k = 0; k < n; ++k) {
        if (t[lo + k]) fail("ambiguous coefficient table");
        t[lo + k] = uint32_t(c.len) | uint32_t(run) << 5 | uint32_t(level + 2048) << 11 | uint32_t(kind) << 24;
      }
      if (kind == kCoef) enc[run][level] = c;
    };
    for (int r = 0; r < 32; ++r) {
      const RunRow& row = kB14[r];
      for (int l = 1; l <= row.n; ++l) {
        Vc c = row.c[l - 1];
        if (b15 && r < 17 && (r > 1 || l <= kB15Low[r].n) && !(r == 0 && l > 15) && !(r == 1 && l > 7))
          c = kB15Low[r].c[l - 1];
        add(c, r, l, kCoef);
      }
    }
    eob = b15 ? kEob15 : kEob14;
    add(eob, 0, 0, kEobK);
    add(kEsc, 0, 0, kEscK);
  }
};

struct Tables {
  Lut mba, type[4], cbp, motion, dcl, dcc;
  CoefLut coef[2];
  double cosx[8][8];  // C(u)/2 cos((2x+1) u pi / 16)
  float cosf[8][8];   // the same in single precision (inverse DCT)
  Tables() {
    mba.init(11);
    for (int i = 1; i <= 33; ++i) mba.add(kMba[i], i);
    mba.add(kMbaEscape, 0);
    type[1].init(2);
    for (auto& e : kTypeI) type[1].add(e.c, e.flags);
    type[2].init(6);
    for (auto& e : kTypeP) type[2].add(e.c, e.flags);
    type[3].init(6);
    for (auto& e : kTypeB) type[3].add(e.c, e.flags);
    cbp.init(9);
    for (int i = 0; i < 64; ++i) cbp.add(kCbp[i], i);
    motion.init(10);
    for (int i = 0; i <= 16; ++i) motion.add(kMotion[i], i);
    dcl.init(9);
    for (int i = 0; i < 12; ++i) dcl.add(kDcLuma[i], i);
    dcc.init(10);
    for (int i = 0; i < 12; ++i) dcc.add(kDcChroma[i], i);
    coef[0].build(false);
    coef[1].build(true);
    for (int u = 0; u < 8; ++u)
      for (int x = 0; x < 8; ++x) {
        cosx[u][x] = (u == 0 ? std::sqrt(0.125) : 0.5) * std::cos((2 * x + 1) * u * M_PI / 16.0);
        cosf[u][x] = (float)cosx[u][x];
      }
  }
};
const Tables& tabs() {
  static const Tables t;
  return t;
}

// ---------------------------------------------------------------- bit I/O ---------------
class Reader {
 public:
  Reader(const uint8_t* d, size_t n, size_t byte) : d_(d), n_(n), pos_(byte * 8) {}
  uint32_t peek(int k) const {
    const size_t b = pos_ >> 3;
    uint64_t v;
    if (b + 8 <= n_) {
      std::memcpy(&v, d_ + b, 8);
      v = __builtin_bswap64(v);
    } else {
      v = 0;
      for (int i = 0; i < 8; ++i) v = (v << 8) | (b + i < n_ ? d_[b + i] : 0);
    }
    return uint32_t((v << (pos_ & 7)) >> (64 - k));
  }
  uint32_t get(int k) {
    if (k == 0) return 0;
    const uint32_t v = peek(k);
    pos_ += k;
    return v;
  }
  void skip(int k) { pos_ += k; }
  int vlc(const Lut& l) {
    const uint32_t e = l.t[peek(l.bits)];
    if (!e) fail("invalid variable-length code");
    pos_ += e >> 16;
    return int(e & 0xffff) - 32768;
  }
  bool next_is_start_code() const { return peek(23) == 0; }
  bool exhausted() const { return (pos_ >> 3) >= n_; }

 private:
  const uint8_t* d_;
  size_t n_, pos_;
};

class Writer {
 public:
  explicit Writer(std::vector<uint8_t>& o) : out_(o) {}
  void put(uint32_t v, int n) {
    if (n == 0) return;
    acc_ = (acc_ << n) | (uint64_t(v) & ((uint64_t(1) << n) - 1));
    nacc_ += n;
    while (nacc_ >= 8) {
      nacc_ -= 8;
      out_.push_back(uint8_t(acc_ >> nacc_));
    }
  }
  void put(Vc c) { put(c.code, c.len); }
  void put(wtab::Code c) { put(c.code, c.len); }
  void align() {
    if (nacc_) put(0, 8 - nacc_);
  }
  void start_code(uint8_t c) {
    align();
    const uint8_t sc[4] = {0, 0, 1, c};
    out_.insert(out_.end(), sc, sc + 4);
  }
  size_t size() const { return out_.size(); }

 private:
  std::vector<uint8_t>& out_;
  uint64_t acc_ = 0;
  int nacc_ = 0;
};

size_t next_start_code(const uint8_t* d, size_t n, size_t p) {
  while (p + 3 < n) {
    if (d[p + 2] > 1) {
      p += 3;
    } else if (d[p] == 0 && d[p + 1] == 0 && d[p + 2] == 1) {
      return p;
    } else {
      ++p;
    }
  }
  return n;
}

// ---------------------------------------------------------------- pixel kernels --------
// Separable inverse DCT in single precision (|coefficient| <= 2048: the float sums stay within
// ~1e-3 of the exact transform, far inside the IEEE 1180 accuracy 13818-2 Annex A asks for),
// all-zero rows skipped.  The writer's reconstruction uses this same function, so decoder
// and writer agree sample for sample.
void idct(const int32_t* F, int16_t* out) {
  const auto& c = tabs().cosf;
  float t[64];
  int rows[8], nr = 0;  // rows with a coefficient (all-zero rows add exact zeros: skipped)
  for (int v = 0; v < 8; ++v) {
    const int32_t* r = F + v * 8;
    bool any = false;
    for (int u = 0; u < 8; ++u) any |= r[u] != 0;
    if (!any) continue;
    rows[nr++] = v;
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int u = 0; u < 8; ++u) {
      if (!r[u]) continue;  // exact: a zero coefficient adds zeros
      const float f = (float)r[u];
      for (int x = 0; x < 8; ++x) s[x] += c[u][x] * f;
    }
    for (int x = 0; x < 8; ++x) t[v * 8 + x] = s[x];
  }
  if (nr == 0) {
    std::memset(out, 0, 64 * sizeof(int16_t));
    return;
  }
  for (int y = 0; y < 8; ++y) {
    float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // x innermost (vectorised); per element the
    for (int k = 0; k < nr; ++k) {          // same ascending-row order of additions
      const float cv = c[rows[k]][y];
      const float* tr = t + rows[k] * 8;
      for (int x = 0; x < 8; ++x) s[x] += cv * tr[x];
    }
    for (int x = 0; x < 8; ++x) out[y * 8 + x] = int16_t(std::clamp((int)std::floor(s[x] + 0.5f), -256, 255));
  }
}

void fdct(const int16_t* in, double* F) {
  const auto& c = tabs().cosx;
  double t[64];
  for (int y = 0; y < 8; ++y)
    for (int u = 0; u < 8; ++u) {
      double s = 0;
      for (int x = 0; x < 8; ++x) s += c[u][x] * in[y * 8 + x];
      t[y * 8 + u] = s;
    }
  for (int v = 0; v < 8; ++v)
    for (int u = 0; u < 8; ++u) {
      double s = 0;
      for (int y = 0; y < 8; ++y) s += c[v][y] * t[y * 8 + u];
      F[v * 8 + u] = s;
    }
}

// 7.4.2-7.4.4: QF (raster) -> F (raster) in place, saturation + mismatch control
void dequant(int32_t* b, bool intra, const uint8_t* W, int qs, int dc_mult) {
  int sum = 0;
  for (int i = 0; i < 64; ++i) {
    int f;
    if (intra && i == 0) {
      f = b[0] * dc_mult;
    } else if (b[i]) {
      const int v = b[i];
      f = ((2 * v + (intra ? 0 : (v > 0 ? 1 : -1))) * int(W[i]) * qs) / 32;
    } else {
      f = 0;
    }
    f = std::clamp(f, -2048, 2047);
    b[i] = f;
    sum += f;
  }
  if ((sum & 1) == 0) b[63] ^= 1;
}

struct View {  // a plane (frame or field) of a reference
  const uint8_t* p;
  int stride, w, h;
};

// 7.6.4 half-sample prediction of a w x h block at integer (x, y) + half flags
void mc(const View& r, int x, int y, int hx, int hy, int w, int h, uint8_t* dst, int ds) {
  const bool inside = x >= 0 && y >= 0 && x + w + hx <= r.w && y + h + hy <= r.h;
  if (inside) {  // the common case, one loop per half-sample phase
    const uint8_t* q = r.p + (size_t)y * r.stride + x;
    const int s = r.stride;
    for (int j = 0; j < h; ++j, q += s, dst += ds) {
      if (hx && hy)
        for (int i = 0; i < w; ++i) dst[i] = uint8_t((q[i] + q[i + 1] + q[i + s] + q[i + s + 1] + 2) >> 2);
      else if (hx)
        for (int i = 0; i < w; ++i) dst[i] = uint8_t((q[i] + q[i + 1] + 1) >> 1);
      else if (hy)
        for (int i = 0; i < w; ++i) dst[i] = uint8_t((q[i] + q[i + s] + 1) >> 1);
      else
        std::memcpy(dst, q, w);
    }
    return;
  }
  for (int j = 0; j < h; ++j)
    for (int i = 0; i < w; ++i) {
      int a, b, c, d;
      if (inside) {
        const uint8_t* q = r.p + (size_t)(y + j) * r.stride + x + i;
        a = q[0];
        b = q[hx];
        c = q[hy * r.stride];
        d = q[hy * r.stride + hx];
      } else {  // out-of-picture vectors (non-conforming streams): edge samples
        const int x0 = std::clamp(x + i, 0, r.w - 1), x1 = std::clamp(x + i + hx, 0, r.w - 1);
        const int y0 = std::clamp(y + j, 0, r.h - 1), y1 = std::clamp(y + j + hy, 0, r.h - 1);
        a = r.p[(size_t)y0 * r.stride + x0];
        b = r.p[(size_t)y0 * r.stride + x1];
        c = r.p[(size_t)y1 * r.stride + x0];
        d = r.p[(size_t)y1 * r.stride + x1];
      }
      int v;
      if (hx && hy)
        v = (a + b + c + d + 2) >> 2;
      else if (hx)
        v = (a + b + 1) >> 1;
      else if (hy)
        v = (a + c + 1) >> 1;
      else
        v = a;
      dst[j * ds + i] = uint8_t(v);
    }
}

// ---------------------------------------------------------------- shared prediction ----
struct PicInfo {
  int type = 1;       // 1 I, 2 P, 3 B
  int structure = 3;  // 1 top field, 2 bottom field, 3 frame
  bool second_field = false;
  int fcode[2][2] = {{15, 15}, {15, 15}};
  int dc_prec = 0, tff = 0, fpfd = 1, concealment = 0, qst = 0, ivlc = 0, alt = 0, rff = 0, progressive = 1;
  int temporal_ref = 0;
};

struct Motion {
  int dirs = 0;   // 1 forward, 2 backward
  int mtype = 2;  // frame pictures: 1 field, 2 frame; field pictures: 1 field, 2 16x8
  int mv[2][2][2] = {};
  int sel[2][2] = {};
};

struct Refs {
  const Image* fwd = nullptr;
  const Image* bwd = nullptr;
  const Image* cur = nullptr;  // the frame being decoded (the first field of a P second field)
};

View plane_view(const Image& im, int comp, int parity /* -1 frame */) {
  const uint8_t* p = comp == 0 ? im.y.data() : comp == 1 ? im.u.data() : im.v.data();
  const int w = comp ? im.w / 2 : im.w, h = comp ? im.h / 2 : im.h;
  if (parity < 0) return {p, w, w, h};
  return {p + (size_t)parity * w, 2 * w, w, h / 2};
}

// prediction of one macroblock (MB-local layout: frame lines for frame pictures, field lines
// for field pictures) -- 7.6.3 / 7.6.4
void predict(const PicInfo& pi, const Refs& rf, const Motion& m, int mbx, int mby, uint8_t* py, uint8_t* pu,
             uint8_t* pv) {
  uint8_t t[2][384];
  int nd = 0;
  const int cur_par = pi.structure == 2 ? 1 : 0;
  for (int s = 0; s < 2; ++s) {
    if (!(m.dirs & (1 << s))) continue;
    uint8_t* oy = t[nd];
    uint8_t* ou = oy + 256;
    uint8_t* ov = ou + 64;
    ++nd;
    auto ref_of = [&](int parity) -> const Image* {
      if (pi.structure != 3 && pi.type == 2 && pi.second_field && s == 0 && parity != cur_par) return rf.cur;
      return s == 0 ? rf.fwd : rf.bwd;
    };
    auto part = [&](const Image* im, int parity, int mvx, int mvy, int lx, int ly, int w, int h, int dy0, int dstep,
                    int cdy0) {
      // luma w x h at picture position (lx, ly) + mv, into rows dy0, dy0 + dstep, ...
      if (!im) fail("missing reference picture");
      if (im->w < 16 || im->h < 32) fail("reference picture too small");
      uint8_t blk[256], cb[64], cr[64];
      mc(plane_view(*im, 0, parity), lx + (mvx >> 1), ly + (mvy >> 1), mvx & 1, mvy & 1, w, h, blk, w);
      const int cx = mvx / 2, cy = mvy / 2;
      const int cw = w / 2, ch = h / 2;
      mc(plane_view(*im, 1, parity), lx / 2 + (cx >> 1), ly / 2 + (cy >> 1), cx & 1, cy & 1, cw, ch, cb, cw);
      mc(plane_view(*im, 2, parity), lx / 2 + (cx >> 1), ly / 2 + (cy >> 1), cx & 1, cy & 1, cw, ch, cr, cw);
      for (int j = 0; j < h; ++j) std::memcpy(oy + (dy0 + j * dstep) * 16, blk + j * w, w);
      for (int j = 0; j < ch; ++j) {
        std::memcpy(ou + (cdy0 + j * dstep) * 8, cb + j * cw, cw);
        std::memcpy(ov + (cdy0 + j * dstep) * 8, cr + j * cw, cw);
      }
    };
    if (pi.structure == 3) {
      if (m.mtype == 2) {  // frame prediction
        const Image* im = s == 0 ? rf.fwd : rf.bwd;
        part(im, -1, m.mv[0][s][0], m.mv[0][s][1], mbx * 16, mby * 16, 16, 16, 0, 1, 0);
      } else if (m.mtype == 1) {  // field prediction: top lines from mv[0], bottom from mv[1]
        const Image* im = s == 0 ? rf.fwd : rf.bwd;
        for (int r = 0; r < 2; ++r)
          part(im, m.sel[r][s], m.mv[r][s][0], m.mv[r][s][1], mbx * 16, mby * 8, 16, 8, r, 2, r);
      } else {
        fail("dual-prime prediction is not supported");
      }
    } else {
      if (m.mtype == 1) {
        part(ref_of(m.sel[0][s]), m.sel[0][s], m.mv[0][s][0], m.mv[0][s][1], mbx * 16, mby * 16, 16, 16, 0, 1, 0);
      } else if (m.mtype == 2) {  // 16x8
        for (int r = 0; r < 2; ++r)
          part(ref_of(m.sel[r][s]), m.sel[r][s], m.mv[r][s][0], m.mv[r][s][1], mbx * 16, mby * 16 + 8 * r, 16, 8,
               8 * r, 1, 4 * r);
      } else {
        fail("dual-prime prediction is not supported");
      }
    }
  }
  if (nd == 0) fail("prediction without a direction");
  if (nd == 2)
    for (int i = 0; i < 384; ++i) t[0][i] = uint8_t((t[0][i] + t[1][i] + 1) >> 1);
  std::memcpy(py, t[0], 256);
  std::memcpy(pu, t[0] + 256, 64);
  std::memcpy(pv, t[0] + 320, 64);
}

// block b of a macroblock: (x0, y0, row step) in the MB-local 16x16 / 8x8 layout
inline void block_geom(int b, int dct_type, int& x0, int& y0, int& step) {
  if (b >= 4) {
    x0 = y0 = 0;
    step = 1;
  } else if (dct_type) {
    x0 = (b & 1) * 8;
    y0 = b >> 1;
    step = 2;
  } else {
    x0 = (b & 1) * 8;
    y0 = (b >> 1) * 8;
    step = 1;
  }
}

// the macroblock's rows in the picture (frame or field lines of the current frame buffer)
struct Dest {
  uint8_t* y;
  uint8_t* u;
  uint8_t* v;
  int ys, cs;
};
Dest mb_dest(Image& im, const PicInfo& pi, int mbx, int mby) {
  const int par = pi.structure == 3 ? 0 : pi.structure == 2 ? 1 : 0;
  const int f = pi.structure == 3 ? 1 : 2;
  Dest d;
  d.ys = im.w * f;
  d.cs = im.w / 2 * f;
  d.y = im.y.data() + (size_t)par * im.w + (size_t)mby * 16 * d.ys + mbx * 16;
  d.u = im.u.data() + (size_t)par * (im.w / 2) + (size_t)mby * 8 * d.cs + mbx * 8;
  d.v = im.v.data() + (size_t)par * (im.w / 2) + (size_t)mby * 8 * d.cs + mbx * 8;
  return d;
}

inline int quant_scale(int code, int qst) { return qst ? kNonLinearQ[code] : 2 * code; }

}  // namespace

// ================================================================= public helpers ========
SeqHeader::SeqHeader() {
  std::memcpy(intra_q, kDefaultIntra, 64);
  std::memset(inter_q, 16, 64);
  std::memcpy(cintra_q, kDefaultIntra, 64);
  std::memset(cinter_q, 16, 64);
}

void SeqHeader::fps(int& num, int& den) const {
  const int c = (frame_rate_code >= 1 && frame_rate_code <= 8) ? frame_rate_code : 4;
  num = kFrameRate[c][0] * (fr_ext_n + 1);
  den = kFrameRate[c][1] * (fr_ext_d + 1);
}

void Image::alloc(int cw, int ch) {
  w = cw;
  h = ch;
  y.assign((size_t)cw * ch, 0);
  u.assign((size_t)cw * ch / 4, 128);
  v.assign((size_t)cw * ch / 4, 128);
}

namespace {

void parse_seq_header(Reader& r, SeqHeader& s) {
  s.width = r.get(12);
  s.height = r.get(12);
  s.aspect = r.get(4);
  s.frame_rate_code = r.get(4);
  s.bit_rate = r.get(18);
  r.skip(1);
  s.vbv = r.get(10);
  r.skip(1);  // constrained_parameters_flag
  if (r.get(1)) {
    for (int i = 0; i < 64; ++i) s.intra_q[kScan[0][i]] = uint8_t(r.get(8));
  } else {
    std::memcpy(s.intra_q, kDefaultIntra, 64);
  }
  if (r.get(1)) {
    for (int i = 0; i < 64; ++i) s.inter_q[kScan[0][i]] = uint8_t(r.get(8));
  } else {
    std::memset(s.inter_q, 16, 64);
  }
  std::memcpy(s.cintra_q, s.intra_q, 64);
  std::memcpy(s.cinter_q, s.inter_q, 64);
  s.mpeg2 = false;
  if (s.width <= 0 || s.height <= 0) fail("bad sequence header");
}

// extension_start_code payloads; returns the identifier
int parse_extension(Reader& r, SeqHeader& s, PicInfo* pi) {
  const int id = r.get(4);
  if (id == 1) {  // sequence_extension
    s.profile_level = r.get(8);
    s.progressive_seq = r.get(1);
    s.chroma_format = r.get(2);
    s.width |= r.get(2) << 12;
    s.height |= r.get(2) << 12;
    s.bit_rate |= r.get(12) << 18;
    r.skip(1);
    s.vbv |= r.get(8) << 10;
    s.low_delay = r.get(1);
    s.fr_ext_n = r.get(2);
    s.fr_ext_d = r.get(5);
    s.mpeg2 = true;
    if (s.chroma_format != 1) fail("only 4:2:0 MPEG-2 video is supported");
  } else if (id == 3) {  // quant_matrix_extension
    if (r.get(1))
      for (int i = 0; i < 64; ++i) s.intra_q[kScan[0][i]] = s.cintra_q[kScan[0][i]] = uint8_t(r.get(8));
    if (r.get(1))
      for (int i = 0; i < 64; ++i) s.inter_q[kScan[0][i]] = s.cinter_q[kScan[0][i]] = uint8_t(r.get(8));
    if (r.get(1))
      for (int i = 0; i < 64; ++i) s.cintra_q[kScan[0][i]] = uint8_t(r.get(8));
    if (r.get(1))
      for (int i = 0; i < 64; ++i) s.cinter_q[kScan[0][i]] = uint8_t(r.get(8));
  } else if (id == 8 && pi) {  // picture_coding_extension
    pi->fcode[0][0] = r.get(4);
    pi->fcode[0][1] = r.get(4);
    pi->fcode[1][0] = r.get(4);
    pi->fcode[1][1] = r.get(4);
    pi->dc_prec = r.get(2);
    pi->structure = r.get(2);
    pi->tff = r.get(1);
    pi->fpfd = r.get(1);
    pi->concealment = r.get(1);
    pi->qst = r.get(1);
    pi->ivlc = r.get(1);
    pi->alt = r.get(1);
    pi->rff = r.get(1);
    r.skip(1);  // chroma_420_type
    pi->progressive = r.get(1);
    if (pi->structure == 0) fail("reserved picture_structure");
  }
  return id;
}

void parse_picture_header(Reader& r, PicInfo& pi) {
  pi.temporal_ref = r.get(10);
  pi.type = r.get(3);
  r.skip(16);  // vbv_delay
  if (pi.type < 1 || pi.type > 3) fail("unsupported picture_coding_type (D pictures)");
  if (pi.type >= 2) {  // MPEG-1 f codes (MPEG-2 takes them from the coding extension)
    r.skip(1);
    pi.fcode[0][0] = pi.fcode[0][1] = r.get(3);
  }
  if (pi.type == 3) {
    r.skip(1);
    pi.fcode[1][0] = pi.fcode[1][1] = r.get(3);
  }
  // MPEG-2 defaults unless a coding extension follows (MPEG-1 streams: frame, progressive)
  pi.structure = 3;
  pi.fpfd = 1;
  pi.progressive = 1;
  pi.dc_prec = pi.concealment = pi.qst = pi.ivlc = pi.alt = pi.rff = pi.tff = 0;
}

}  // namespace

// ================================================================= index =================
StreamIndex index_stream(const uint8_t* d, size_t n) {
  StreamIndex ix;
  bool have_seq = false, seen_interlaced = false, first_seq_open = false;
  size_t last_seq = 0, hdr_start = SIZE_MAX;  // first header byte since the last picture
  bool gop_pending = false, gop_closed = false;
  int fields_open = 0;  // 1 after a first field
  struct P {
    int type;
    size_t rap;  // index into raps + 1, or 0
  };
  std::vector<P> pics;
  SeqHeader seq;
  for (size_t p = next_start_code(d, n, 0); p < n; p = next_start_code(d, n, p + 4)) {
    const uint8_t c = d[p + 3];
    if (c == 0xB3) {
      Reader r(d, n, p + 4);
      parse_seq_header(r, seq);
      if (!have_seq) {
        ix.seq = seq;
        first_seq_open = true;
      }
      have_seq = true;
      last_seq = p;
      if (hdr_start == SIZE_MAX) hdr_start = p;
    } else if (c == 0xB5 && have_seq) {
      Reader r(d, n, p + 4);
      if (r.peek(4) == 1 || r.peek(4) == 3) {
        parse_extension(r, seq, nullptr);
        if (first_seq_open) ix.seq = seq;
      }
    } else if (c == 0xB8) {
      Reader r(d, n, p + 4);
      r.skip(25);
      gop_closed = r.get(1);
      gop_pending = true;
      if (hdr_start == SIZE_MAX) hdr_start = p;
    } else if (c == 0x00 && have_seq) {
      first_seq_open = false;
      PicInfo pi;
      Reader r(d, n, p + 4);
      try {
        parse_picture_header(r, pi);
      } catch (const std::runtime_error&) {
        continue;  // a damaged picture header: the decoder skips that picture too
      }
      // the coding extension (before the first slice)
      for (size_t q = next_start_code(d, n, p + 4); q < n; q = next_start_code(d, n, q + 4)) {
        const uint8_t e = d[q + 3];
        if (e >= 0x01 && e <= 0xAF) break;
        if (e == 0x00 || e == 0xB3 || e == 0xB8 || e == 0xB7) break;
        if (e == 0xB5) {
          Reader x(d, n, q + 4);
          if (x.peek(4) == 8) parse_extension(x, seq, &pi);
        }
      }
      const bool first_of_frame = pi.structure == 3 || fields_open == 0;
      if (pi.structure != 3) {
        ix.field_pictures = true;
        fields_open ^= 1;
      }
      if (first_of_frame) {
        if (!pi.progressive && !seen_interlaced) {
          seen_interlaced = true;
          ix.interlaced = true;
          ix.top_field_first = pi.structure == 3 ? pi.tff : (pi.structure == 1 ? 1 : 0);
        }
        P rec{pi.type, 0};
        if (pi.type == 1) {
          Rap rap;
          rap.offset = hdr_start != SIZE_MAX ? hdr_start : p;
          rap.seq_offset = last_seq;
          rap.frames_before = ix.frames;
          rap.closed = gop_pending && gop_closed;
          ix.raps.push_back(rap);
          rec.rap = ix.raps.size();
        }
        pics.push_back(rec);
        ++ix.frames;
      }
      hdr_start = SIZE_MAX;
      gop_pending = false;
    }
  }
  if (!have_seq) fail("no sequence header");
  // an I picture not followed by B pictures has no leading pictures: random access is clean
  for (size_t k = 0; k < pics.size(); ++k)
    if (pics[k].rap && (k + 1 == pics.size() || pics[k + 1].type != 3)) ix.raps[pics[k].rap - 1].closed = true;
  if (!ix.raps.empty()) ix.raps[0].closed = true;  // nothing precedes the first GOP
  return ix;
}

// ================================================================= decoder ===============
struct Decoder::Impl {
  SeqHeader seq;
  PicInfo pi;
  bool in_picture = false;  // a picture header was seen, slices may follow
  bool pic_started = false;
  bool broken_link = false, gop_closed = false;
  bool skip_pic = false;  // undecodable (leading B after a random access)
  std::shared_ptr<Image> cur, fwd, bwd, held;
  int cur_type = 0, cur_fields = 0, cur_first_structure = 0;
  bool cur_broken = false;
  int disp = 0;
  const Sink* sink = nullptr;
  bool stop = false;
  // slice state
  int qcode = 0, dc_pred[3] = {}, pmv[2][2][2] = {};
  Motion prev{};
  bool prev_intra = false;
  // syntax coverage (Decoder::stats): see kStatNames
  int64_t st[kNumStats] = {};

  std::shared_ptr<Image> new_image() {
    auto im = std::make_shared<Image>();
    im->alloc(seq.mb_width() * 16, seq.mb_height() * 16);
    return im;
  }

  void output(const std::shared_ptr<Image>& im, bool broken) {
    const int k = disp++;
    if (!broken && im && !stop && !(*sink)(k, *im)) stop = true;
  }

  void begin_picture() {
    pic_started = true;
    const bool second = pi.structure != 3 && cur_fields == 1 && cur && pi.structure != cur_first_structure;
    pi.second_field = second;
    if (!second) {
      if (cur_fields == 1) finish_frame();  // a lone field: finish what there is
      cur = new_image();
      // concealment base: a slice lost to a bitstream error leaves the latest reference's
      // samples there instead of grey
      if (bwd && bwd->w == cur->w && bwd->h == cur->h) {
        cur->y = bwd->y;
        cur->u = bwd->u;
        cur->v = bwd->v;
      }
      cur_type = pi.type;
      cur_first_structure = pi.structure;
      cur_fields = 0;
      // references: B needs both, P the most recent, leading B pictures after a random
      // access (or a broken link) have none
      cur_broken = pi.type == 3 ? (!fwd || !bwd || broken_link) : pi.type == 2 ? !bwd : false;
    }
    skip_pic = cur_broken;
  }

  void end_picture() {
    if (!pic_started) return;
    pic_started = false;
    in_picture = false;
    if (pi.structure == 3) {
      finish_frame();
    } else if (++cur_fields == 2) {
      finish_frame();
    }
  }

  void finish_frame() {
    if (!cur) return;
    if (cur_type == 3) {
      output(cur, cur_broken);
    } else {
      if (held) output(held, false);
      fwd = bwd;
      bwd = cur;
      held = cur;
      broken_link = false;  // the link is repaired by the next reference
    }
    cur.reset();
    cur_fields = 0;
  }

  void flush() {
    if (cur_fields == 1) finish_frame();
    if (held) output(held, false);
    held.reset();
  }

  // ------------------------------------------------------------- slice ----------------
  void reset_pmv() { std::memset(pmv, 0, sizeof(pmv)); }
  void reset_dc() { dc_pred[0] = dc_pred[1] = dc_pred[2] = 128 << pi.dc_prec; }

  int motion_delta(Reader& r, int s, int t) {
    const int code_mag = r.vlc(tabs().motion);
    int mc = code_mag;
    if (mc && r.get(1)) mc = -mc;
    const int rsize = pi.fcode[s][t] - 1;
    if (rsize < 0 || rsize > 8) fail("bad f_code");
    const int f = 1 << rsize;
    if (f == 1 || mc == 0) return mc;
    const int resid = r.get(rsize);
    const int dlt = (std::abs(mc) - 1) * f + resid + 1;
    return mc < 0 ? -dlt : dlt;
  }

  void motion_vector(Reader& r, Motion& m, int rr, int s, bool field_in_frame) {
    for (int t = 0; t < 2; ++t) {
      const int delta = motion_delta(r, s, t);
      const int f = 1 << (pi.fcode[s][t] - 1);
      const int high = 16 * f - 1, low = -16 * f, range = 32 * f;
      int pred = pmv[rr][s][t];
      if (field_in_frame && t == 1) pred >>= 1;
      int v = pred + delta;
      if (v < low) v += range;
      if (v > high) v -= range;
      m.mv[rr][s][t] = v;
      pmv[rr][s][t] = (field_in_frame && t == 1) ? v * 2 : v;
    }
  }

  void motion_vectors(Reader& r, Motion& m, int s) {
    const bool frame_pic = pi.structure == 3;
    int count, field_fmt;
    if (frame_pic) {
      if (m.mtype == 1) {
        count = 2;
        field_fmt = 1;
      } else if (m.mtype == 2) {
        count = 1;
        field_fmt = 0;
      } else {
        fail("dual-prime prediction is not supported");
      }
    } else {
      if (m.mtype == 3) fail("dual-prime prediction is not supported");
      count = m.mtype == 2 ? 2 : 1;
      field_fmt = 1;
    }
    if (count == 1) {
      if (field_fmt) m.sel[0][s] = r.get(1);
      motion_vector(r, m, 0, s, false);
      pmv[1][s][0] = pmv[0][s][0];
      pmv[1][s][1] = pmv[0][s][1];
    } else {
      for (int rr = 0; rr < 2; ++rr) {
        m.sel[rr][s] = r.get(1);
        motion_vector(r, m, rr, s, frame_pic);
      }
    }
  }

  void read_block(Reader& r, int b, bool intra, int32_t* blk) {
    ++st[intra ? 15 : 16];
    std::memset(blk, 0, 64 * sizeof(int32_t));
    const uint8_t* scan = kScan[pi.alt];
    int n = 0;
    const CoefLut* lut = &tabs().coef[0];
    if (intra) {
      const int cc = b < 4 ? 0 : b - 3;
      const int size = r.vlc(cc == 0 ? tabs().dcl : tabs().dcc);
      int diff = 0;
      if (size) {
        const int bits = r.get(size);
        diff = (bits >> (size - 1)) ? bits : bits + 1 - (1 << size);
      }
      dc_pred[cc] += diff;
      blk[0] = dc_pred[cc];
      n = 1;
      if (pi.ivlc) lut = &tabs().coef[1];
    } else if (r.peek(1)) {  // first coefficient '1s' = (0, +-1)
      r.skip(1);
      blk[scan[0]] = r.get(1) ? -1 : 1;
      n = 1;
    }
    while (true) {
      const uint32_t e = lut->t[r.peek(16)];
      if (!e) fail("invalid DCT coefficient code");
      const int kind = int(e >> 24);
      r.skip(int(e & 31));
      if (kind == kEobK) break;
      int run, level;
      if (kind == kEscK) {
        run = r.get(6);
        level = r.get(12);
        if (level & 0x800) level -= 4096;
        if (level == 0 || level == -2048) fail("forbidden escape level");
        ++st[13];
      } else {
        run = int((e >> 5) & 63);
        level = int((e >> 11) & 0x1fff) - 2048;
        if (r.get(1)) level = -level;
      }
      n += run;
      if (n > 63) fail("coefficient index past the block");
      blk[scan[n]] = level;
      ++n;
    }
  }

  void decode_slice(const uint8_t* d, size_t n, size_t p) {
    const int mbw = seq.mb_width();
    const int mbh = pi.structure == 3 ? seq.mb_height() : seq.mb_height() / 2;
    Reader r(d, n, p + 4);
    int row = d[p + 3] - 1;
    if (seq.height > 2800) row += r.get(3) << 7;
    if (row >= mbh) fail("slice below the picture");
    qcode = r.get(5);
    if (r.peek(1)) {  // intra_slice_flag, intra_slice, reserved; extra_information_slice
      r.skip(1 + 1 + 7);
      while (r.get(1)) r.skip(8);
    } else {
      r.skip(1);
    }
    reset_dc();
    reset_pmv();
    prev = Motion{};
    prev_intra = false;
    int addr = row * mbw - 1;
    bool first = true;
    const int nmb = mbw * mbh;
    while (true) {
      int inc = 0;
      while (r.peek(11) == 8) {
        r.skip(11);
        inc += 33;
      }
      inc += r.vlc(tabs().mba);
      if (addr + inc >= nmb) fail("macroblock address past the picture");
      if (!first && inc > 1) {
        for (int k = 1; k < inc; ++k) skipped_mb(addr + k, mbw);
      }
      addr += inc;
      first = false;
      if (addr >= nmb) fail("macroblock address past the picture");
      macroblock(r, addr % mbw, addr / mbw);
      if (r.next_is_start_code() || r.exhausted()) break;
    }
  }

  void put_mb(const uint8_t* py, const uint8_t* pu, const uint8_t* pv, int mbx, int mby) {
    const int rows = pi.structure == 3 ? cur->h / 16 : cur->h / 32;
    if (mbx >= cur->w / 16 || mby >= rows) fail("macroblock outside the picture buffer");
    Dest dd = mb_dest(*cur, pi, mbx, mby);
    for (int j = 0; j < 16; ++j) std::memcpy(dd.y + (size_t)j * dd.ys, py + j * 16, 16);
    for (int j = 0; j < 8; ++j) {
      std::memcpy(dd.u + (size_t)j * dd.cs, pu + j * 8, 8);
      std::memcpy(dd.v + (size_t)j * dd.cs, pv + j * 8, 8);
    }
  }

  Refs refs() const {
    Refs rf;
    if (pi.type == 2) {
      rf.fwd = bwd.get();
    } else {
      rf.fwd = fwd.get();
      rf.bwd = bwd.get();
    }
    rf.cur = cur.get();
    return rf;
  }

  void skipped_mb(int addr, int mbw) {
    const int mbx = addr % mbw, mby = addr / mbw;
    reset_dc();
    uint8_t py[256], pu[64], pv[64];
    Motion m;
    const int cur_par = pi.structure == 2 ? 1 : 0;
    ++st[pi.type == 2 ? 6 : 7];
    if (pi.type == 2) {  // zero vector from the same-parity / whole reference, PMVs reset
      reset_pmv();
      m.dirs = 1;
      m.mtype = pi.structure == 3 ? 2 : 1;
      m.sel[0][0] = cur_par;
    } else if (pi.type == 3) {  // the previous macroblock's directions and vectors (PMV)
      if (prev_intra) fail("skipped macroblock after an intra macroblock in a B picture");
      m.dirs = prev.dirs;
      m.mtype = pi.structure == 3 ? 2 : 1;
      for (int s = 0; s < 2; ++s) {
        m.mv[0][s][0] = pmv[0][s][0];
        m.mv[0][s][1] = pmv[0][s][1];
        m.sel[0][s] = cur_par;
      }
    } else {
      fail("skipped macroblock in an I picture");
    }
    if (skip_pic) return;
    predict(pi, refs(), m, mbx, mby, py, pu, pv);
    put_mb(py, pu, pv, mbx, mby);
  }

  void macroblock(Reader& r, int mbx, int mby) {
    const int flags = r.vlc(tabs().type[pi.type]);
    const bool frame_pic = pi.structure == 3;
    Motion m;
    m.dirs = ((flags & MF) ? 1 : 0) | ((flags & MB) ? 2 : 0);
    int dct_type = 0;
    if (frame_pic) {
      if (m.dirs) m.mtype = pi.fpfd ? 2 : int(r.get(2));
      if (!pi.fpfd && (flags & (MI | MP))) dct_type = r.get(1);
    } else if (m.dirs) {
      m.mtype = r.get(2);
    }
    if (m.dirs && m.mtype == 0) fail("reserved motion type");
    if (flags & MQ) qcode = r.get(5);
    const bool intra = flags & MI;
    if ((flags & MF) || (intra && pi.concealment)) {
      Motion cm = m;
      if (intra) cm.mtype = frame_pic ? 2 : 1;
      motion_vectors(r, cm, 0);
      if (!intra) m = cm;
    }
    if (flags & MB) motion_vectors(r, m, 1);
    if (intra && pi.concealment) r.skip(1);
    int cbp = intra ? 63 : (flags & MP) ? r.vlc(tabs().cbp) : 0;
    // predictor state (7.2.1, 7.6.3.4)
    if (intra) {
      if (!pi.concealment) reset_pmv();
    } else {
      reset_dc();
      if (pi.type == 2 && !(flags & MF)) {  // P "no MC": zero vector, PMVs reset
        reset_pmv();
        m.dirs = 1;
        m.mtype = frame_pic ? 2 : 1;
        m.sel[0][0] = pi.structure == 2 ? 1 : 0;
        std::memset(m.mv, 0, sizeof(m.mv));
      }
    }
    prev = m;
    prev_intra = intra;
    if (intra) {
      ++st[0];
    } else if (pi.type == 2) {
      ++st[(flags & MF) ? 1 : 2];
    } else {
      ++st[m.dirs == 1 ? 3 : m.dirs == 2 ? 4 : 5];
    }
    if (!intra && (flags & (MF | MB))) ++st[frame_pic ? (m.mtype == 2 ? 8 : 9) : (m.mtype == 1 ? 10 : 11)];
    if (dct_type) ++st[12];
    if (flags & MQ) ++st[14];
    const int qs = quant_scale(qcode, pi.qst);
    if (qs == 0) fail("quantiser_scale_code 0");
    int32_t blk[6][64];
    int16_t res[6][64];
    for (int b = 0; b < 6; ++b) {
      if (!(cbp & (32 >> b))) continue;
      read_block(r, b, intra, blk[b]);
    }
    if (skip_pic) return;
    uint8_t py[256], pu[64], pv[64];
    if (intra) {
      std::memset(py, 0, 256);
      std::memset(pu, 0, 64);
      std::memset(pv, 0, 64);
    } else {
      predict(pi, refs(), m, mbx, mby, py, pu, pv);
    }
    for (int b = 0; b < 6; ++b) {
      if (!(cbp & (32 >> b))) continue;
      const uint8_t* W = intra ? (b < 4 ? seq.intra_q : seq.cintra_q) : (b < 4 ? seq.inter_q : seq.cinter_q);
      dequant(blk[b], intra, W, qs, 8 >> pi.dc_prec);
      idct(blk[b], res[b]);
      int x0, y0, step;
      block_geom(b, dct_type, x0, y0, step);
      uint8_t* dst = b < 4 ? py : b == 4 ? pu : pv;
      const int ds = b < 4 ? 16 : 8;
      for (int j = 0; j < 8; ++j)
        for (int i = 0; i < 8; ++i) {
          uint8_t& px = dst[(y0 + j * step) * ds + x0 + i];
          px = uint8_t(std::clamp(int(px) + res[b][j * 8 + i], 0, 255));
        }
    }
    put_mb(py, pu, pv, mbx, mby);
  }

  void run(const uint8_t* d, size_t n, size_t seq_off, size_t start, int base, const Sink& s) {
    sink = &s;
    stop = false;
    disp = base;
    cur.reset();
    fwd.reset();
    bwd.reset();
    held.reset();
    cur_fields = 0;
    pic_started = in_picture = false;
    broken_link = false;
    bool have_seq = false;
    if (seq_off < start && seq_off + 4 < n && d[seq_off] == 0 && d[seq_off + 1] == 0 && d[seq_off + 2] == 1 &&
        d[seq_off + 3] == 0xB3) {
      Reader r(d, n, seq_off + 4);
      parse_seq_header(r, seq);
      have_seq = true;
      for (size_t q = next_start_code(d, n, seq_off + 4); q < n && q < start; q = next_start_code(d, n, q + 4)) {
        if (d[q + 3] != 0xB5) break;
        Reader x(d, n, q + 4);
        parse_extension(x, seq, nullptr);
      }
    }
    for (size_t p = next_start_code(d, n, start); p < n && !stop; p = next_start_code(d, n, p + 4)) {
      const uint8_t c = d[p + 3];
      if (c >= 0x01 && c <= 0xAF) {
        if (!in_picture) continue;
        if (!pic_started) begin_picture();
        try {
          decode_slice(d, n, p);
        } catch (const std::runtime_error&) {  // a damaged slice: conceal it, keep decoding
          ++st[17];
          if (!cur) throw;
        }
        continue;
      }
      end_picture();
      try {
        if (c == 0xB3) {
          Reader r(d, n, p + 4);
          SeqHeader sh = seq;
          parse_seq_header(r, sh);
          seq = sh;
          have_seq = true;
        } else if (c == 0xB5) {
          Reader r(d, n, p + 4);
          SeqHeader sh = seq;
          PicInfo pc = pi;
          parse_extension(r, sh, in_picture ? &pc : nullptr);
          seq = sh;
          pi = pc;
        } else if (c == 0x00 && have_seq) {
          Reader r(d, n, p + 4);
          parse_picture_header(r, pi);
          in_picture = true;
        }
      } catch (const std::runtime_error&) {  // a damaged header: skip it (and a picture's slices)
        ++st[17];
        if (c == 0x00) in_picture = false;
        continue;
      }
      if (c == 0xB8) {
        Reader r(d, n, p + 4);
        r.skip(25);
        gop_closed = r.get(1);
        broken_link = r.get(1);
      } else if (c == 0xB7) {
        in_picture = false;
      }
    }
    end_picture();
    if (!stop) flush();
  }
};

Decoder::Decoder() : p_(new Impl) {}
const int64_t* Decoder::stats() const { return p_->st; }
Decoder::~Decoder() = default;
void Decoder::decode(const uint8_t* d, size_t n, size_t seq_off, size_t start, int base, const Sink& sink) {
  p_->run(d, n, seq_off, start, base, sink);
}

// ================================================================= writer ================
namespace {

struct Lcg {
  uint32_t s;
  uint32_t next() {
    s = s * 1664525u + 1013904223u;
    return s >> 8;
  }
  int below(int n) { return int(next() % uint32_t(n)); }
};

// quantiser_scale from quantiser_scale_code with the writer's copy of Table 7-6
inline int w_quant_scale(int code, int qst) { return qst ? wtab::get().nonlinear_q[code] : 2 * code; }

class Encoder {
 public:
  Encoder(const EncConfig& c, std::vector<uint8_t>& es) : c_(c), w_(es), es_(es), rng_{c.seed * 2654435761u + 7} {
    if (c.width % 16 || c.height % (c.interlaced ? 32 : 16)) fail("writer: size must be a multiple of 16 (32 interlaced)");
    if (c.field_pictures && !c.interlaced) fail("writer: field pictures need an interlaced sequence");
    seq_.width = c.width;
    seq_.height = c.height;
    seq_.progressive_seq = c.interlaced ? 0 : 1;
    if (c.custom_matrices) {
      for (int i = 0; i < 64; ++i) {
        seq_.intra_q[i] = uint8_t(std::min(255, 8 + 2 * ((i >> 3) + (i & 7)) + (i % 5)));  // any custom matrix
        seq_.inter_q[i] = uint8_t(14 + (i * 7) % 9);
      }
      seq_.intra_q[0] = 8;
      std::memcpy(seq_.cintra_q, seq_.intra_q, 64);
      std::memcpy(seq_.cinter_q, seq_.inter_q, 64);
    }
  }

  void write_sequence_header() {
    w_.start_code(0xB3);
    w_.put(c_.width & 0xfff, 12);
    w_.put(c_.height & 0xfff, 12);
    w_.put(2, 4);  // 4:3
    w_.put(c_.frame_rate_code, 4);
    w_.put(24500, 18);  // 9.8 Mbit/s
    w_.put(1, 1);
    w_.put(112, 10);
    w_.put(0, 1);
    w_.put(c_.custom_matrices, 1);
    if (c_.custom_matrices)
      for (int i = 0; i < 64; ++i) w_.put(seq_.intra_q[wt_.scan[0][i]], 8);
    w_.put(c_.custom_matrices, 1);
    if (c_.custom_matrices)
      for (int i = 0; i < 64; ++i) w_.put(seq_.inter_q[wt_.scan[0][i]], 8);
    w_.start_code(0xB5);  // sequence_extension
    w_.put(1, 4);
    w_.put(0x48, 8);  // Main Profile @ Main Level
    w_.put(seq_.progressive_seq, 1);
    w_.put(1, 2);  // 4:2:0
    w_.put(0, 2);
    w_.put(0, 2);
    w_.put(0, 12);
    w_.put(1, 1);
    w_.put(0, 8);
    w_.put(0, 1);  // low_delay
    w_.put(0, 2);
    w_.put(0, 5);
  }

  void write_gop(int frame_no, bool closed) {
    w_.start_code(0xB8);
    int num, den;
    seq_.fps(num, den);
    const int fps = (num + den - 1) / den;
    const int f = frame_no % fps, s = (frame_no / fps) % 60, m = (frame_no / fps / 60) % 60, h = (frame_no / fps / 3600) % 24;
    w_.put(0, 1);  // drop_frame_flag
    w_.put(h, 5);
    w_.put(m, 6);
    w_.put(1, 1);
    w_.put(s, 6);
    w_.put(f, 6);
    w_.put(closed, 1);
    w_.put(0, 1);
  }

  void write_picture_header(const PicInfo& pi) {
    w_.start_code(0x00);
    w_.put(pi.temporal_ref & 1023, 10);
    w_.put(pi.type, 3);
    w_.put(0xffff, 16);
    if (pi.type >= 2) {
      w_.put(0, 1);
      w_.put(7, 3);
    }
    if (pi.type == 3) {
      w_.put(0, 1);
      w_.put(7, 3);
    }
    w_.put(0, 1);  // extra_bit_picture
    w_.start_code(0xB5);
    w_.put(8, 4);
    for (int s = 0; s < 2; ++s)
      for (int t = 0; t < 2; ++t) w_.put(pi.fcode[s][t], 4);
    w_.put(pi.dc_prec, 2);
    w_.put(pi.structure, 2);
    w_.put(pi.tff, 1);
    w_.put(pi.fpfd, 1);
    w_.put(0, 1);  // concealment_motion_vectors
    w_.put(pi.qst, 1);
    w_.put(pi.ivlc, 1);
    w_.put(pi.alt, 1);
    w_.put(0, 1);  // repeat_first_field
    w_.put(pi.progressive, 1);  // chroma_420_type
    w_.put(pi.progressive, 1);
    w_.put(0, 1);  // composite_display_flag
  }

  // ---------------------------------------------------------------- motion search ----
  struct Cand {
    Motion m;
    bool intra = false, zero = false, skip = false;
    int cost = 0;
    uint8_t py[256] = {}, pu[64] = {}, pv[64] = {};
  };

  int sad_rows(const uint8_t* a, const uint8_t* b, int w, int h) {
    int s = 0;
    for (int i = 0; i < w * h; ++i) s += std::abs(int(a[i]) - int(b[i]));
    return s;
  }

  // best half-pel vector of a w x h block (source rows `src`) at picture position (x, y) in view v
  void search(const View& v, const uint8_t* src, int x, int y, int w, int h, int& bx, int& by) {
    const int R = c_.search;
    const int lim = 16 * (1 << (c_.f_code - 1)) - 1;
    uint8_t blk[256];
    int best = INT32_MAX;
    bx = by = 0;
    auto legal = [&](int mx, int my) {
      const int ix = x + (mx >> 1), iy = y + (my >> 1);
      return std::abs(mx) <= lim && std::abs(my) <= lim && ix >= 0 && iy >= 0 && ix + w + (mx & 1) <= v.w &&
             iy + h + (my & 1) <= v.h;
    };
    auto eval = [&](int mx, int my) {
      if (!legal(mx, my)) return;
      mc(v, x + (mx >> 1), y + (my >> 1), mx & 1, my & 1, w, h, blk, w);
      const int s = sad_rows(src, blk, w, h) + (std::abs(mx) + std::abs(my)) * 2;
      if (s < best) {
        best = s;
        bx = mx;
        by = my;
      }
    };
    for (int dy = -R; dy <= R; dy += 2)
      for (int dx = -R; dx <= R; dx += 2) eval(2 * dx, 2 * dy);
    const int cx = bx, cy = by;  // the full-pel grid is 2 pels apart: refine +-1 pel, then half
    for (int dy = -2; dy <= 2; dy += 2)
      for (int dx = -2; dx <= 2; dx += 2) eval(cx + dx, cy + dy);
    const int hx = bx, hy = by;
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) eval(hx + dx, hy + dy);
  }

  // source rows of the MB as the prediction layout (frame lines / field lines)
  void source_mb(const uint8_t* frame, int mbx, int mby, uint8_t* sy, uint8_t* su, uint8_t* sv) {
    const int W = c_.width, H = c_.height;
    const uint8_t* Y = frame;
    const uint8_t* U = frame + (size_t)W * H;
    const uint8_t* V = U + (size_t)W * H / 4;
    const int par = pi_.structure == 2 ? 1 : 0, f = pi_.structure == 3 ? 1 : 2;
    for (int j = 0; j < 16; ++j) std::memcpy(sy + j * 16, Y + (size_t)(par + (mby * 16 + j) * f) * W + mbx * 16, 16);
    for (int j = 0; j < 8; ++j) {
      std::memcpy(su + j * 8, U + (size_t)(par + (mby * 8 + j) * f) * (W / 2) + mbx * 8, 8);
      std::memcpy(sv + j * 8, V + (size_t)(par + (mby * 8 + j) * f) * (W / 2) + mbx * 8, 8);
    }
  }

  void finish_cand(Cand& k, const uint8_t* sy, int mbx, int mby, const Refs& rf) {
    predict(pi_, rf, k.m, mbx, mby, k.py, k.pu, k.pv);
    k.cost = sad_rows(sy, k.py, 16, 16);
  }

  std::vector<Cand> candidates(const uint8_t* sy, int mbx, int mby, const Refs& rf) {
    std::vector<Cand> cs;
    const bool frame_pic = pi_.structure == 3;
    const int cur_par = pi_.structure == 2 ? 1 : 0;
    {  // intra
      Cand k;
      k.intra = true;
      int mean = 0;
      for (int i = 0; i < 256; ++i) mean += sy[i];
      mean /= 256;
      for (int i = 0; i < 256; ++i) k.cost += std::abs(sy[i] - mean);
      k.cost += 500;
      cs.push_back(k);
    }
    if (pi_.type == 1) return cs;
    auto ref_view = [&](int s, int parity) -> View {
      const Image* im = s == 0 ? rf.fwd : rf.bwd;
      if (!frame_pic && pi_.type == 2 && pi_.second_field && s == 0 && parity != cur_par) im = rf.cur;
      return plane_view(*im, 0, parity);
    };
    // per direction: the best single-vector prediction (frame MC / field MC of the picture)
    Motion best[2];
    for (int s = 0; s < (pi_.type == 3 ? 2 : 1); ++s) {
      Motion m;
      m.dirs = 1 << s;
      if (frame_pic) {
        m.mtype = 2;
        search(ref_view(s, -1), sy, mbx * 16, mby * 16, 16, 16, m.mv[0][s][0], m.mv[0][s][1]);
      } else {
        m.mtype = 1;
        int bc = INT32_MAX;
        for (int par = 0; par < 2; ++par) {
          if (ipfield_ && par == cur_par) continue;  // P field of an I frame: its first field only
          int mx, my;
          search(ref_view(s, par), sy, mbx * 16, mby * 16, 16, 16, mx, my);
          Cand t;
          t.m = m;
          t.m.sel[0][s] = par;
          t.m.mv[0][s][0] = mx;
          t.m.mv[0][s][1] = my;
          finish_cand(t, sy, mbx, mby, rf);
          if (t.cost < bc) {
            bc = t.cost;
            m = t.m;
          }
        }
      }
      best[s] = m;
      Cand k;
      k.m = m;
      finish_cand(k, sy, mbx, mby, rf);
      cs.push_back(k);
      // two-vector variants: field MC in interlaced frame pictures, 16x8 in field pictures
      if (!frame_pic || !pi_.fpfd) {
        Cand f;
        f.m.dirs = 1 << s;
        f.m.mtype = frame_pic ? 1 : 2;
        for (int r = 0; r < 2; ++r) {
          uint8_t half[128];
          int par = frame_pic ? (rng_.below(2) ? r : 1 - r) : (rng_.below(3) ? cur_par : 1 - cur_par);
          if (ipfield_) par = 1 - cur_par;
          f.m.sel[r][s] = par;
          int mx, my;
          if (frame_pic) {
            for (int j = 0; j < 8; ++j) std::memcpy(half + j * 16, sy + (2 * j + r) * 16, 16);
            search(ref_view(s, par), half, mbx * 16, mby * 8, 16, 8, mx, my);
          } else {
            std::memcpy(half, sy + r * 128, 128);
            search(ref_view(s, par), half, mbx * 16, mby * 16 + 8 * r, 16, 8, mx, my);
          }
          f.m.mv[r][s][0] = mx;
          f.m.mv[r][s][1] = my;
        }
        finish_cand(f, sy, mbx, mby, rf);
        cs.push_back(f);
      }
    }
    if (pi_.type == 3) {  // bi-prediction from the two best
      Cand k;
      k.m = best[0];
      k.m.dirs = 3;
      if (best[1].mtype != k.m.mtype) k.m.mtype = frame_pic ? 2 : 1;
      for (int r = 0; r < 2; ++r) {
        k.m.mv[r][1][0] = best[1].mv[r][1][0];
        k.m.mv[r][1][1] = best[1].mv[r][1][1];
        k.m.sel[r][1] = best[1].sel[r][1];
      }
      finish_cand(k, sy, mbx, mby, rf);
      cs.push_back(k);
    }
    if (pi_.type == 2 && !ipfield_) {  // zero vector (skip / "no MC")
      Cand k;
      k.zero = true;
      k.m.dirs = 1;
      k.m.mtype = frame_pic ? 2 : 1;
      k.m.sel[0][0] = cur_par;
      finish_cand(k, sy, mbx, mby, rf);
      k.cost -= 64;
      cs.push_back(k);
    } else if (pi_.type == 3 && !prev_intra_ && prev_.dirs) {  // B skip: the previous directions at the PMVs
      Cand k;
      k.skip = true;
      k.m.dirs = prev_.dirs;
      k.m.mtype = frame_pic ? 2 : 1;
      bool ok = true;
      for (int s = 0; s < 2; ++s) {
        k.m.mv[0][s][0] = pmv_[0][s][0];
        k.m.mv[0][s][1] = pmv_[0][s][1];
        k.m.sel[0][s] = cur_par;
        if (!(k.m.dirs & (1 << s))) continue;
        const View v = ref_view(s, frame_pic ? -1 : cur_par);
        const int mx = pmv_[0][s][0], my = pmv_[0][s][1];
        const int ix = mbx * 16 + (mx >> 1), iy = mby * 16 + (my >> 1);
        ok &= ix >= 0 && iy >= 0 && ix + 16 + (mx & 1) <= v.w && iy + 16 + (my & 1) <= v.h;
        // the chroma block of the skip vector stays inside too (vectors derived by /2)
      }
      if (ok) {
        finish_cand(k, sy, mbx, mby, rf);
        k.cost -= 64;
        cs.push_back(k);
      }
    }
    return cs;
  }

  // ---------------------------------------------------------------- syntax writing ---
  void put_mba(int inc) {
    while (inc > 33) {
      w_.put(wt_.mba_escape);
      inc -= 33;
    }
    w_.put(wt_.mba[inc]);
  }

  void put_type(int flags) {
    const wtab::TypeEntry* t;
    int n;
    if (pi_.type == 1) {
      t = wt_.type_i;
      n = 2;
    } else if (pi_.type == 2) {
      t = wt_.type_p;
      n = 7;
    } else {
      t = wt_.type_b;
      n = 11;
    }
    // the writer's flag bits are its own (wtab) and mean the same columns of B.2-B.4
    const int wf = (flags & MQ ? wtab::kQuant : 0) | (flags & MF ? wtab::kFwd : 0) | (flags & MB ? wtab::kBwd : 0) |
                   (flags & MP ? wtab::kPattern : 0) | (flags & MI ? wtab::kIntra : 0);
    for (int i = 0; i < n; ++i)
      if (t[i].flags == wf) {
        w_.put(wtab::detail::bits(t[i].bits));
        return;
      }
    fail("writer: no macroblock_type for these flags");
  }

  void put_motion_code(int delta, int s, int t) {
    const int rsize = pi_.fcode[s][t] - 1, f = 1 << rsize;
    int mc, resid = 0;
    if (f == 1 || delta == 0) {
      mc = delta;
    } else {
      const int a = std::abs(delta);
      mc = (a - 1) / f + 1;
      resid = (a - 1) % f;
      if (delta < 0) mc = -mc;
    }
    if (std::abs(mc) > 16) fail("writer: motion vector out of the f_code range");
    w_.put(wt_.motion[std::abs(mc)]);
    if (mc) w_.put(mc < 0, 1);
    if (f != 1 && mc) w_.put(resid, rsize);
  }

  void put_vector(const Motion& m, int r, int s, bool field_in_frame) {
    for (int t = 0; t < 2; ++t) {
      const int f = 1 << (pi_.fcode[s][t] - 1);
      const int high = 16 * f - 1, low = -16 * f, range = 32 * f;
      int pred = pmv_[r][s][t];
      if (field_in_frame && t == 1) pred >>= 1;
      const int v = m.mv[r][s][t];
      int delta = v - pred;
      if (delta < low) delta += range;
      if (delta > high) delta -= range;
      put_motion_code(delta, s, t);
      pmv_[r][s][t] = (field_in_frame && t == 1) ? v * 2 : v;
    }
  }

  void put_vectors(const Motion& m, int s) {
    const bool frame_pic = pi_.structure == 3;
    const bool two = frame_pic ? m.mtype == 1 : m.mtype == 2;
    if (!two) {
      if (!frame_pic) w_.put(m.sel[0][s], 1);
      put_vector(m, 0, s, false);
      pmv_[1][s][0] = pmv_[0][s][0];
      pmv_[1][s][1] = pmv_[0][s][1];
    } else {
      for (int r = 0; r < 2; ++r) {
        w_.put(m.sel[r][s], 1);
        put_vector(m, r, s, frame_pic);
      }
    }
  }

  void put_block(const int32_t* qf, bool intra, int b) {
    const uint8_t* scan = wt_.scan[pi_.alt];
    int start = 0;
    const int vlc = intra && pi_.ivlc ? 1 : 0;
    if (intra) {
      const int cc = b < 4 ? 0 : b - 3;
      const int diff = qf[0] - dc_pred_[cc];
      dc_pred_[cc] = qf[0];
      const int a = std::abs(diff);
      int size = 0;
      while ((1 << size) <= a) ++size;
      w_.put(cc == 0 ? wt_.dc_luma[size] : wt_.dc_chroma[size]);
      if (size) w_.put(diff > 0 ? diff : diff + (1 << size) - 1, size);
      start = 1;
    }
    int run = 0;
    bool first = !intra;
    for (int n = start; n < 64; ++n) {
      const int v = qf[scan[n]];
      if (!v) {
        ++run;
        continue;
      }
      const int a = std::abs(v);
      if (first && run == 0 && a == 1) {
        w_.put(1, 1);
        w_.put(v < 0, 1);
      } else if (run < 32 && a <= 40 && wt_.coef[vlc][run][a].len) {
        w_.put(wt_.coef[vlc][run][a]);
        w_.put(v < 0, 1);
      } else {
        w_.put(wt_.escape);
        w_.put(run, 6);
        w_.put(v & 0xfff, 12);
      }
      first = false;
      run = 0;
    }
    w_.put(wt_.eob[vlc]);
  }

  // ---------------------------------------------------------------- residual ---------
  // forward transform + quantisation of block b of (src - pred) in the MB layout; returns
  // whether any level is non-zero and reconstructs the block into `rec`
  bool code_block(const uint8_t* src, const uint8_t* pred, int b, int dct_type, bool intra, int qs, int32_t* qf,
                  uint8_t* rec) {
    int x0, y0, step;
    block_geom(b, dct_type, x0, y0, step);
    const int ds = b < 4 ? 16 : 8;
    int16_t diff[64];
    for (int j = 0; j < 8; ++j)
      for (int i = 0; i < 8; ++i) {
        const int o = (y0 + j * step) * ds + x0 + i;
        diff[j * 8 + i] = int16_t(int(src[o]) - (intra ? 0 : int(pred[o])));
      }
    double F[64];
    fdct(diff, F);
    const uint8_t* W = intra ? (b < 4 ? seq_.intra_q : seq_.cintra_q) : (b < 4 ? seq_.inter_q : seq_.cinter_q);
    bool any = false;
    const int dc_mult = 8 >> pi_.dc_prec;
    for (int i = 0; i < 64; ++i) {
      int q;
      if (intra && i == 0) {
        q = std::clamp((int)std::lround(F[0] / dc_mult), 0, (1 << (8 + pi_.dc_prec)) - 1);
      } else {
        const double t = std::fabs(F[i]) * 16.0 / (double(W[i]) * qs);
        q = intra ? (int)std::floor(t + 0.5) : (int)std::floor(t + 0.1);
        q = std::min(q, 2047);
        if (F[i] < 0) q = -q;
      }
      qf[i] = q;
      any |= q != 0 && !(intra && i == 0);
    }
    // the decoder's reconstruction
    int32_t deq[64];
    std::memcpy(deq, qf, sizeof(deq));
    dequant(deq, intra, W, qs, dc_mult);
    int16_t res[64];
    idct(deq, res);
    for (int j = 0; j < 8; ++j)
      for (int i = 0; i < 8; ++i) {
        const int o = (y0 + j * step) * ds + x0 + i;
        rec[o] = uint8_t(std::clamp((intra ? 0 : int(pred[o])) + res[j * 8 + i], 0, 255));
      }
    return intra || any;
  }

  // all six blocks of the candidate at scale qs: levels, coded_block_pattern, reconstruction
  int code_mb(const uint8_t* sy, const uint8_t* su, const uint8_t* sv, const Cand& k, int dct_type, int qs,
              int32_t (*qf)[64], uint8_t* ry, uint8_t* ru, uint8_t* rv) {
    std::memcpy(ry, k.py, 256);
    std::memcpy(ru, k.pu, 64);
    std::memcpy(rv, k.pv, 64);
    int cbp = 0;
    for (int b = 0; b < 6; ++b) {
      const uint8_t* s = b < 4 ? sy : b == 4 ? su : sv;
      const uint8_t* p = b < 4 ? k.py : b == 4 ? k.pu : k.pv;
      uint8_t* rr = b < 4 ? ry : b == 4 ? ru : rv;
      uint8_t tmp[256];
      std::memcpy(tmp, rr, b < 4 ? 256 : 64);
      if (code_block(s, p, b, dct_type, k.intra, qs, qf[b], tmp)) {
        cbp |= 32 >> b;
        std::memcpy(rr, tmp, b < 4 ? 256 : 64);
      }
    }
    return cbp;
  }

  // ---------------------------------------------------------------- pictures ---------
  void encode_picture(const uint8_t* src, Image& cur, const Image* fwd, const Image* bwd, const PicInfo& pi) {
    pi_ = pi;
    write_picture_header(pi_);
    const int mbw = c_.width / 16;
    const int mbh = pi_.structure == 3 ? c_.height / 16 : c_.height / 32;
    Refs rf;
    if (pi_.type == 2) {
      rf.fwd = fwd;
    } else {
      rf.fwd = fwd;
      rf.bwd = bwd;
    }
    rf.cur = &cur;
    const bool frame_pic = pi_.structure == 3;
    const int S = std::max(1, std::min(c_.slices_per_row, mbw));
    for (int row = 0; row < mbh; ++row)
      for (int sl = 0; sl < S; ++sl) {
        const int x0 = sl * mbw / S, x1 = (sl + 1) * mbw / S;
        w_.start_code(uint8_t(row + 1));
        qcode_ = c_.qscale_code;
        w_.put(qcode_, 5);
        w_.put(0, 1);  // extra_bit_slice
        dc_reset();
        std::memset(pmv_, 0, sizeof(pmv_));
        prev_ = Motion{};
        prev_intra_ = false;
        int last = row * mbw - 1;  // macroblock_address_increment base of the slice
        for (int mbx = x0; mbx < x1; ++mbx) {
          uint8_t sy[256], su[64], sv[64];
          source_mb(src, mbx, row, sy, su, sv);
          std::vector<Cand> cs = candidates(sy, mbx, row, rf);
          int pick = 0;
          for (int k = 1; k < (int)cs.size(); ++k)
            if (cs[k].cost < cs[pick].cost) pick = k;
          if (rng_.below(4) == 0) pick = rng_.below((int)cs.size());  // visit every path
          Cand& k = cs[pick];
          // quantiser change (only with levels: a macroblock without any keeps the scale)
          int flags = 0, qc = qcode_;
          if (c_.vary_quant && rng_.below(6) == 0) {
            qc = 2 + rng_.below(20);
            if (qc != qcode_) flags |= MQ;
          }
          const int dct_type = (frame_pic && !pi_.fpfd) ? rng_.below(2) : 0;
          int32_t qf[6][64];
          uint8_t ry[256], ru[64], rv[64];
          int cbp = code_mb(sy, su, sv, k, dct_type, w_quant_scale(qc, pi_.qst), qf, ry, ru, rv);
          if ((flags & MQ) && cbp == 0 && !k.intra) {
            flags &= ~MQ;
            qc = qcode_;
            cbp = code_mb(sy, su, sv, k, dct_type, w_quant_scale(qc, pi_.qst), qf, ry, ru, rv);
          }
          qcode_ = qc;
          const bool edge = mbx == x0 || mbx == x1 - 1;
          const bool can_skip = !edge && !(flags & MQ) && cbp == 0 && !k.intra && (k.zero || k.skip);
          if (can_skip) {  // skipped: the decoder forms exactly this prediction
            if (pi_.type == 2) std::memset(pmv_, 0, sizeof(pmv_));
            dc_reset();
            put_rec(cur, ry, ru, rv, mbx, row);
            continue;
          }
          const int addr = row * mbw + mbx;
          put_mba(addr - last);
          last = addr;
          if (k.intra) {
            flags |= MI;
          } else if (k.zero && pi_.type == 2) {
            flags |= cbp ? MP : MF;  // "no MC" (PMV reset) / MC not coded with a zero vector
          } else {
            if (k.m.dirs & 1) flags |= MF;
            if (k.m.dirs & 2) flags |= MB;
            if (cbp) flags |= MP;
          }
          put_type(flags);
          if (frame_pic) {
            if ((flags & (MF | MB)) && !pi_.fpfd) w_.put(k.m.mtype, 2);
            if (!pi_.fpfd && (flags & (MI | MP))) w_.put(dct_type, 1);
          } else if (flags & (MF | MB)) {
            w_.put(k.m.mtype, 2);
          }
          if (flags & MQ) w_.put(qcode_, 5);
          if (flags & MF) put_vectors(k.m, 0);
          if (flags & MB) put_vectors(k.m, 1);
          if (flags & MP) w_.put(wt_.cbp[cbp]);
          for (int b = 0; b < 6; ++b)
            if (cbp & (32 >> b)) put_block(qf[b], k.intra, b);
          if (k.intra) {
            std::memset(pmv_, 0, sizeof(pmv_));
          } else {
            dc_reset();
            if (pi_.type == 2 && !(flags & MF)) std::memset(pmv_, 0, sizeof(pmv_));
          }
          prev_ = k.m;
          prev_intra_ = k.intra;
          put_rec(cur, ry, ru, rv, mbx, row);
        }
      }
  }

  void put_rec(Image& cur, const uint8_t* ry, const uint8_t* ru, const uint8_t* rv, int mbx, int mby) {
    Dest dd = mb_dest(cur, pi_, mbx, mby);
    for (int j = 0; j < 16; ++j) std::memcpy(dd.y + (size_t)j * dd.ys, ry + j * 16, 16);
    for (int j = 0; j < 8; ++j) {
      std::memcpy(dd.u + (size_t)j * dd.cs, ru + j * 8, 8);
      std::memcpy(dd.v + (size_t)j * dd.cs, rv + j * 8, 8);
    }
  }

  void dc_reset() { dc_pred_[0] = dc_pred_[1] = dc_pred_[2] = 128 << pi_.dc_prec; }

  PicInfo base_pic(int type, int structure, int tref) const {
    PicInfo pi;
    pi.type = type;
    pi.structure = structure;
    pi.temporal_ref = tref;
    const int fc = c_.f_code;
    pi.fcode[0][0] = pi.fcode[0][1] = type >= 2 ? fc : 15;
    pi.fcode[1][0] = pi.fcode[1][1] = type == 3 ? fc : 15;
    pi.dc_prec = c_.intra_dc_precision;
    pi.tff = structure == 3 && c_.interlaced ? c_.top_field_first : 0;
    pi.fpfd = c_.interlaced ? 0 : 1;
    if (structure != 3) pi.fpfd = 0;
    pi.qst = c_.q_scale_type;
    pi.ivlc = c_.intra_vlc;
    pi.alt = c_.alternate_scan;
    pi.progressive = c_.interlaced ? 0 : 1;
    return pi;
  }

  void encode_frame(const uint8_t* src, Image& cur, const Image* fwd, const Image* bwd, int type, int tref) {
    if (!c_.field_pictures) {
      encode_picture(src, cur, fwd, bwd, base_pic(type, 3, tref));
      return;
    }
    const int first = c_.top_field_first ? 1 : 2;
    PicInfo a = base_pic(type, first, tref);
    encode_picture(src, cur, fwd, bwd, a);
    PicInfo b = base_pic(type == 1 ? 2 : type, 3 - first, tref);  // I frames: I + P field
    b.second_field = true;
    if (type == 1) {  // the P field predicts from the first field only (random access stays clean)
      b.fcode[0][0] = b.fcode[0][1] = c_.f_code;
      ipfield_ = true;
      encode_picture(src, cur, nullptr, nullptr, b);
      ipfield_ = false;
    } else {
      encode_picture(src, cur, fwd, bwd, b);
    }
  }

  void run(const std::vector<const uint8_t*>& frames, std::vector<size_t>* units, std::vector<int>* udisp,
           std::vector<Image>* recon) {
    const int N = (int)frames.size();
    const int M = c_.bframes + 1, G = std::max(1, c_.gop);
    std::vector<int> type(N);
    for (int i = 0; i < N; ++i) {
      const int g = i % G;
      if (g == 0)
        type[i] = 1;
      else if (c_.closed_gop && g == G - 1)
        type[i] = 2;
      else
        type[i] = (g % M == 0) ? 2 : 3;
    }
    if (N && type[N - 1] == 3) type[N - 1] = 2;
    // decoding order: each reference, then the B pictures before it
    std::vector<int> order;
    int prev_ref = -1;
    for (int i = 0; i < N; ++i) {
      if (type[i] == 3) continue;
      order.push_back(i);
      for (int b = prev_ref + 1; b < i; ++b) order.push_back(b);
      prev_ref = i;
    }
    std::vector<Image> rec(N);
    int last_ref = -1, older_ref = -1;
    int gop_first_disp = 0;
    for (size_t k = 0; k < order.size(); ++k) {
      const int i = order[k];
      const size_t unit_start = w_.size();
      if (type[i] == 1) {
        write_sequence_header();
        // the GOP's first displayed frame: leading B pictures (open GOP) come first
        int first = i;
        while (first > 0 && type[first - 1] == 3) --first;
        gop_first_disp = first;
        write_gop(first, c_.closed_gop || i == 0);
      }
      rec[i].alloc(c_.width, c_.height);
      const Image* fwd = nullptr;
      const Image* bwd = nullptr;
      if (type[i] == 2) {
        fwd = &rec[last_ref];
      } else if (type[i] == 3) {
        fwd = older_ref >= 0 ? &rec[older_ref] : nullptr;
        bwd = &rec[last_ref];
        // closed GOP leading pictures never occur (the GOP ends on a P picture)
        if (!fwd) fail("writer: B picture without a forward reference");
      }
      encode_frame(frames[i], rec[i], fwd, bwd, type[i], i - gop_first_disp);
      w_.align();  // the frame's last byte belongs to its unit
      if (type[i] != 3) {
        older_ref = last_ref;
        last_ref = i;
      }
      if (units) units->push_back(w_.size() - unit_start);
      if (udisp) udisp->push_back(i);
    }
    w_.start_code(0xB7);
    if (units && !units->empty()) units->back() += 4;
    if (recon) *recon = std::move(rec);
  }

 private:
  EncConfig c_;
  Writer w_;
  std::vector<uint8_t>& es_;
  const wtab::Tables& wt_ = wtab::get();  // the writer's own Annex B transcription
  SeqHeader seq_;
  PicInfo pi_;
  Lcg rng_;
  int qcode_ = 0;
  int dc_pred_[3] = {};
  int pmv_[2][2][2] = {};
  Motion prev_{};
  bool prev_intra_ = false;
  bool ipfield_ = false;
};

}  // namespace

std::vector<uint8_t> encode(const EncConfig& cfg, const std::vector<const uint8_t*>& frames,
                            std::vector<size_t>* units, std::vector<int>* unit_display, std::vector<Image>* recon) {
  std::vector<uint8_t> es;
  Encoder e(cfg, es);
  e.run(frames, units, unit_display, recon);
  return es;
}

}  // namespace tv::mpeg2

// ================================================================= C API =================
namespace {
thread_local std::string g_m2err;
template <class F>
int m2guard(F&& f) {
  try {
    f();
    return 0;
  } catch (const std::exception& e) {
    g_m2err = e.what();
    return -1;
  }
}
}  // namespace

extern "C" {
using namespace tv::mpeg2;

const char* tv_mpeg2_last_error() { return g_m2err.c_str(); }

// cfg (int32, any prefix): width, height, frame_rate_code, gop, bframes, qscale_code, interlaced,
// field_pictures, top_field_first, alternate_scan, intra_vlc, q_scale_type, intra_dc_precision,
// custom_matrices, closed_gop, vary_quant, slices_per_row, f_code, search, seed.
// n display-order I420 frames (width x height) -> `out` (a tv_bytes buffer); unit_sizes[n] /
// unit_disp[n]: the decoding-order frame units; recon: n I420 frames in display order.
int tv_mpeg2_encode(const int32_t* cfg, int ncfg, int n, const uint8_t* yuv, void* out, int64_t* unit_sizes,
                    int32_t* unit_disp, uint8_t* recon) {
  return m2guard([&] {
    EncConfig c;
    int* f[] = {&c.width, &c.height, &c.frame_rate_code, &c.gop, &c.bframes, &c.qscale_code};
    const int nf = int(sizeof(f) / sizeof(f[0]));
    for (int i = 0; i < nf && i < ncfg; ++i) *f[i] = cfg[i];
    bool* b[] = {&c.interlaced, &c.field_pictures, &c.top_field_first, &c.alternate_scan, &c.intra_vlc,
                 &c.q_scale_type};
    for (int i = 0; i < 6 && nf + i < ncfg; ++i) *b[i] = cfg[nf + i] != 0;
    if (ncfg > 12) c.intra_dc_precision = cfg[12];
    if (ncfg > 13) c.custom_matrices = cfg[13] != 0;
    if (ncfg > 14) c.closed_gop = cfg[14] != 0;
    if (ncfg > 15) c.vary_quant = cfg[15] != 0;
    if (ncfg > 16) c.slices_per_row = cfg[16];
    if (ncfg > 17) c.f_code = cfg[17];
    if (ncfg > 18) c.search = cfg[18];
    if (ncfg > 19) c.seed = uint32_t(cfg[19]);
    if (c.intra_dc_precision < 0 || c.intra_dc_precision > 2 || c.f_code < 1 || c.f_code > 9)
      throw std::runtime_error("mpeg2: writer configuration out of range");
    const size_t fsz = (size_t)c.width * c.height * 3 / 2;
    std::vector<const uint8_t*> frames(n);
    for (int i = 0; i < n; ++i) frames[i] = yuv + i * fsz;
    std::vector<size_t> units;
    std::vector<int> disp;
    std::vector<Image> rec;
    *static_cast<std::vector<uint8_t>*>(out) = encode(c, frames, &units, &disp, &rec);
    for (int i = 0; i < n; ++i) {
      unit_sizes[i] = (int64_t)units[i];
      unit_disp[i] = disp[i];
      if (recon) {
        uint8_t* o = recon + i * fsz;
        std::memcpy(o, rec[i].y.data(), (size_t)c.width * c.height);
        std::memcpy(o + (size_t)c.width * c.height, rec[i].u.data(), (size_t)c.width * c.height / 4);
        std::memcpy(o + (size_t)c.width * c.height * 5 / 4, rec[i].v.data(), (size_t)c.width * c.height / 4);
      }
    }
  });
}

// info[16]: width, height, frames, fps_num, fps_den, interlaced, top_field_first, field_pictures,
// progressive_sequence, aspect_ratio_information, profile_and_level, random-access points,
// mb_width, mb_height, mpeg2 (0: MPEG-1 stream)
int tv_mpeg2_probe(const uint8_t* d, size_t n, int32_t* info) {
  return m2guard([&] {
    const StreamIndex ix = index_stream(d, n);
    int num, den;
    ix.seq.fps(num, den);
    const int32_t v[16] = {ix.seq.width, ix.seq.height, ix.frames, num, den, ix.interlaced, ix.top_field_first,
                           ix.field_pictures, ix.seq.progressive_seq, ix.seq.aspect, ix.seq.profile_level,
                           (int32_t)ix.raps.size(), ix.seq.mb_width(), ix.seq.mb_height(), ix.seq.mpeg2, 0};
    std::memcpy(info, v, sizeof(v));
  });
}

int tv_mpeg2_raps(const uint8_t* d, size_t n, int64_t* off, int64_t* seq_off, int32_t* frames_before, int32_t* closed,
                  int cap) {
  int got = 0;
  const int rc = m2guard([&] {
    const StreamIndex ix = index_stream(d, n);
    for (const Rap& r : ix.raps) {
      if (got < cap) {
        off[got] = (int64_t)r.offset;
        seq_off[got] = (int64_t)r.seq_offset;
        frames_before[got] = r.frames_before;
        closed[got] = r.closed;
      }
      ++got;
    }
  });
  return rc ? rc : got;
}

// display frames [first, first + count) of the pictures from d[start] (sequence header at
// seq_off, frames numbered from base) -> out: count I420 frames at the display size (chroma
// (w+1)/2 x (h+1)/2); got[k] = 1 for every frame delivered
int tv_mpeg2_decode(const uint8_t* d, size_t n, int64_t seq_off, int64_t start, int32_t base, int32_t first,
                    int32_t count, uint8_t* out, int32_t* got, int64_t* stats) {
  return m2guard([&] {
    Decoder dec;
    std::memset(got, 0, sizeof(int32_t) * count);
    int w = 0, h = 0;
    {
      const StreamIndex ix = index_stream(d + seq_off, std::min(n - (size_t)seq_off, (size_t)1 << 20));
      w = ix.seq.width;
      h = ix.seq.height;
    }
    const int cw = (w + 1) / 2, ch = (h + 1) / 2;
    const size_t fsz = (size_t)w * h + 2 * (size_t)cw * ch;
    dec.decode(d, n, (size_t)seq_off, (size_t)start, base, [&](int k, const Image& im) {
      if (k >= first && k < first + count) {
        uint8_t* o = out + (size_t)(k - first) * fsz;
        for (int y = 0; y < h; ++y) std::memcpy(o + (size_t)y * w, im.y.data() + (size_t)y * im.w, w);
        uint8_t* ou = o + (size_t)w * h;
        uint8_t* ov = ou + (size_t)cw * ch;
        for (int y = 0; y < ch; ++y) {
          std::memcpy(ou + (size_t)y * cw, im.u.data() + (size_t)y * (im.w / 2), cw);
          std::memcpy(ov + (size_t)y * cw, im.v.data() + (size_t)y * (im.w / 2), cw);
        }
        got[k - first] = 1;
      }
      return k < first + count - 1;
    });
    if (stats) std::memcpy(stats, dec.stats(), sizeof(int64_t) * kNumStats);
  });
}

// the decoder's VLC tables (see models/mpeg2.py table()); which + 100: the fixture writer's
// own transcription (mpeg2_wtab.h) in the same layout, so the two can be compared entry by
// entry.  7 / 8 / 9: macroblock_type of I / P / B pictures (value = the flag bits MQ 1, MF 2,
// MB 4, MP 8, MI 16).
int tv_mpeg2_table(int which, int32_t* code, int32_t* len, int32_t* value, int cap) {
  std::vector<std::array<int32_t, 3>> t;
  auto add = [&](Vc c, int v) { t.push_back({c.code, c.len, v}); };
  auto addw = [&](wtab::Code c, int v) { t.push_back({c.code, c.len, v}); };
  const bool wr = which >= 100;
  which %= 100;
  const wtab::Tables& W = wtab::get();
  if (which == 0 || which == 1) {
    const CoefLut& l = tabs().coef[which];
    for (int r = 0; r < 32; ++r)
      for (int lv = 1; lv <= 40; ++lv) {
        if (wr && W.coef[which][r][lv].len) addw(W.coef[which][r][lv], r << 8 | lv);
        if (!wr && l.enc[r][lv].len) add(l.enc[r][lv], r << 8 | lv);
      }
    if (wr) {
      addw(W.eob[which], -1);
      addw(W.escape, -2);
    } else {
      add(l.eob, -1);
      add(kEsc, -2);
    }
  } else if (which == 2) {
    for (int i = 0; i < 64; ++i) wr ? addw(W.cbp[i], i) : add(kCbp[i], i);
  } else if (which == 3) {
    for (int i = 0; i <= 16; ++i) wr ? addw(W.motion[i], i) : add(kMotion[i], i);
  } else if (which == 4 || which == 5) {
    for (int i = 0; i < 12; ++i)
      wr ? addw(which == 4 ? W.dc_luma[i] : W.dc_chroma[i], i) : add(which == 4 ? kDcLuma[i] : kDcChroma[i], i);
  } else if (which == 6) {
    for (int i = 1; i <= 33; ++i) wr ? addw(W.mba[i], i) : add(kMba[i], i);
    wr ? addw(W.mba_escape, 0) : add(kMbaEscape, 0);
  } else if (which >= 7 && which <= 9) {
    const int n = which == 7 ? 2 : (which == 8 ? 7 : 11);
    for (int i = 0; i < n; ++i) {
      if (wr) {
        const wtab::TypeEntry& e = (which == 7 ? W.type_i : which == 8 ? W.type_p : W.type_b)[i];
        const int f = (e.flags & wtab::kQuant ? MQ : 0) | (e.flags & wtab::kFwd ? MF : 0) |
                      (e.flags & wtab::kBwd ? MB : 0) | (e.flags & wtab::kPattern ? MP : 0) |
                      (e.flags & wtab::kIntra ? MI : 0);
        addw(wtab::detail::bits(e.bits), f);
      } else {
        const TypeCode& e = (which == 7 ? kTypeI : which == 8 ? kTypeP : kTypeB)[i];
        add(e.c, e.flags);
      }
    }
  } else if (which == 10 || which == 11) {  // scans (code = position, len 0)
    for (int i = 0; i < 64; ++i) t.push_back({wr ? W.scan[which - 10][i] : kScan[which - 10][i], 0, i});
  } else if (which == 12) {  // non-linear quantiser_scale
    for (int i = 0; i < 32; ++i) t.push_back({wr ? W.nonlinear_q[i] : kNonLinearQ[i], 0, i});
  }
  for (int i = 0; i < (int)t.size() && i < cap; ++i) {
    code[i] = t[i][0];
    len[i] = t[i][1];
    value[i] = t[i][2];
  }
  return (int)t.size();
}

const char* tv_mpeg2_stat_name(int i) { return i >= 0 && i < kNumStats ? kStatNames[i] : ""; }
int tv_mpeg2_num_stats() { return kNumStats; }

}  // extern "C"
