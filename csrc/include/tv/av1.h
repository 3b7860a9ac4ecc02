// av1.h — AV1 coding tools of the C++ golden model: CDEF, loop
// restoration (Wiener, self-guided) with their encoder-side searches, and the AV1
// multi-symbol range coder with adaptive 15-bit CDFs.  The gfx950 kernels in
// csrc/gpu/k_av1.hip implement the same filters/statistics bit-exactly (av1_defs.h).
#pragma once
#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <vector>

namespace tv {
namespace av1 {

// ---- CDEF ----------------------------------------------------------------------------
// Direction + variance of every 8x8 block of a w x h luma plane (w, h multiples of 8).
void cdef_find_dirs(const uint8_t* Y, int w, int h, uint8_t* dir, int* var);
// Per-(64x64 filter block, preset) SSE after filtering plane `rec` against `src`.
// chroma: 4:2:0 plane (4x4 blocks take the co-located luma direction, no variance
// adjustment, damping - 1).  sse: [nfb][64] with nfb = ceil(w/fbs) * ceil(h/fbs).
// pmask: presets to evaluate (bit p); the others get kCdefSkipped (an SSE no evaluated
// preset reaches, small enough that sums over every filter block cannot overflow).
void cdef_search(const uint8_t* src, const uint8_t* rec, int w, int h, bool chroma, const uint8_t* dir,
                 const int* var, int luma_w8, int damping, uint64_t* sse, uint64_t pmask = ~0ull,
                 bool checker = false);  // checker: only blocks with (bx + by) even (encoder search)
// Filter a plane with a per-filter-block preset index (-1 = off) into `out`.
void cdef_apply(const uint8_t* rec, int w, int h, bool chroma, const uint8_t* dir, const int* var, int luma_w8,
                int damping, const int8_t* fb_preset, uint8_t* out);

// ---- loop restoration (64x64 restoration units) -----------------------------------------
constexpr int kRu = 64;
// Wiener filter with per-unit coefficients coef[unit][6] = (h0,h1,h2, v0,v1,v2); a unit
// with all six == 0 keeps the identity filter.
void wiener_apply(const uint8_t* rec, int w, int h, const int* coef, uint8_t* out);
// Normal-equation statistics for one separable pass: `dir` 0 estimates the horizontal
// taps given the vertical taps `other` (per unit, 3 ints), 1 the reverse.  stats[unit][9]
// = A00 A01 A02 A11 A12 A22 b0 b1 b2 (int64).
void wiener_stats(const uint8_t* src, const uint8_t* rec, int w, int h, int dir, const int* other, int64_t* stats);
// Self-guided filter: per-unit (set, w0, w1) (set < 0 = off).
void sgr_apply(const uint8_t* rec, int w, int h, const int* params, uint8_t* out);
// Projection statistics of parameter set `set` for every unit: stats[unit][5] =
// H00 H01 H11 c0 c1 (int64) of the least-squares problem for (w0, w1).
void sgr_stats(const uint8_t* src, const uint8_t* rec, int w, int h, int set, int64_t* stats);
// The two guided-filter outputs (RST domain) of one plane, for tests / the GPU check.
void sgr_filter_planes(const uint8_t* rec, int w, int h, int set, int32_t* f0, int32_t* f1);

// ---- normative self-guided restoration (AV1 7.17; 64x64 units, 4:2:0) ----------------------
// One plane w x h (ss: 0 luma, 1 chroma): cdef = CDEF output, dbk = deblocked pre-CDEF
// plane (the rows beyond a stripe come from it).  Units follow av1_defs.h lr_count_units.
// F0 / F1 (RST domain) of parameter set `set` for every pixel.
void sgr_flt(const uint8_t* cdef, const uint8_t* dbk, int w, int h, int ss, int set, int32_t* f0, int32_t* f1);
// restore with per-unit (set | -1, xqd0, xqd1), units row-major
void lr_apply(const uint8_t* cdef, const uint8_t* dbk, int w, int h, int ss, const int* params, uint8_t* out);
// per-unit normal equations [units][5] = H00 H01 H11 c0 c1 of parameter set `set`
void lr_stats(const uint8_t* src, const uint8_t* cdef, const uint8_t* dbk, int w, int h, int ss, int set,
              int64_t* stats);

// ---- deblocking loop filter (AV1 7.14) -------------------------------------------------
// Filter every tx edge of a plane: `info` holds one word per 4x4 unit (layout in
// av1_defs.h: tx / block log2 sizes, per-direction levels, skip && inter); sharp 0..7.
void deblock(const uint8_t* in, int w, int h, bool chroma, const uint32_t* info, int sharp, uint8_t* out);

// ---- multi-symbol range coder -------------------------------------------------------------
// Probabilities are AV1 inverse CDFs: icdf[i] = 32768 * P(X > i), icdf[n-1] = 0, plus one
// adaptation counter at icdf[n] (n <= 16).
void cdf_init_uniform(uint16_t* icdf, int n);
// CDF adaptation after coding `sym` (inline: the syntax writer / reader call it per symbol)
inline void cdf_adapt(uint16_t* icdf, int n, int sym) {
  const int cnt = icdf[n];
  const int lg = 31 - __builtin_clz((unsigned)n);
  const int rate = 3 + (cnt > 15) + (cnt > 31) + (lg < 2 ? lg : 2);
  for (int i = 0; i < n - 1; ++i) {
    if (i < sym) icdf[i] = (uint16_t)(icdf[i] + ((32768 - icdf[i]) >> rate));
    else icdf[i] = (uint16_t)(icdf[i] - (icdf[i] >> rate));
  }
  icdf[n] = (uint16_t)(cnt + (cnt < 32));
}

// Multi-symbol range encoder (the per-symbol paths are inline: the OBU writer codes ~10^5
// symbols per frame)
class RangeEncoder {
 public:
  // The pre-carry buffer is thread-local and reused (cleared, capacity kept): a writer per
  // frame would otherwise map and fault fresh pages for it on every call.
  RangeEncoder() : pre_(tl_buffer()) { pre_.clear(); }
  __attribute__((always_inline)) void encode(int sym, uint16_t* icdf, int n, bool adapt = true) {
    if (__builtin_expect(sym < 0 || sym >= n, 0)) throw std::runtime_error("range coder: symbol out of range");
    const uint32_t r = rng_;
    uint32_t nr;
    if (sym > 0) {
      const uint32_t u = bound(r, icdf[sym - 1], n, sym - 1), v = bound(r, icdf[sym], n, sym);
      low_ += r - u;
      nr = u - v;
    } else {
      nr = r - bound(r, icdf[0], n, 0);
    }
    emit(nr);
    if (adapt) cdf_adapt(icdf, n, sym);
  }
  void encode_bool(int bit, int p0_q15) {  // p0 = P(bit == 0) in 1/32768
    const int p = p0_q15 < 1 ? 1 : (p0_q15 > 32767 ? 32767 : p0_q15);
    uint16_t icdf[3] = {(uint16_t)(32768 - p), 0, 0};
    encode(bit ? 1 : 0, icdf, 2, false);
  }
  void encode_literal(uint32_t v, int bits) {
    for (int b = bits - 1; b >= 0; --b) encode_bool((v >> b) & 1, 16384);
  }
  std::vector<uint8_t> finish();
  size_t bits_written() const;

 private:
  static constexpr int kProbShift = 6, kMinProb = 4;
  static uint32_t bound(uint32_t r, int icdf_v, int n, int k) {
    return ((r >> 8) * (uint32_t)(icdf_v >> kProbShift) >> (7 - kProbShift)) + kMinProb * (n - 1 - k);
  }
  // low_ already holds the new low; normalise the range back to [2^15, 2^16)
  __attribute__((always_inline)) void emit(uint32_t r) {
    const int d = 16 - (32 - __builtin_clz(r));
    int c = cnt_, s = c + d;
    uint64_t l = low_;
    if (s >= 0) {
      c += 16;
      uint64_t m = (1ull << c) - 1;
      if (s >= 8) {
        pre_.push_back((uint16_t)(l >> c));
        l &= m;
        c -= 8;
        m >>= 8;
      }
      pre_.push_back((uint16_t)(l >> c));
      s = c + d - 24;
      l &= m;
    }
    low_ = l << d;
    rng_ = r << d;
    cnt_ = s;
  }
  uint64_t low_ = 0;
  uint32_t rng_ = 0x8000;
  int cnt_ = -9;
  static std::vector<uint16_t>& tl_buffer() {
    thread_local std::vector<uint16_t> b;
    return b;
  }
  std::vector<uint16_t>& pre_;  // pre-carry bytes (one live encoder per thread)
};

class RangeDecoder {
 public:
  RangeDecoder(const uint8_t* data, size_t size);
  int decode(uint16_t* icdf, int n, bool adapt = true);
  int decode_bool(int p0_q15);
  uint32_t decode_literal(int bits);

 private:
  void refill();
  void normalize(uint32_t rng_new);
  const uint8_t *p_, *end_;
  uint64_t dif_ = 0;
  uint32_t rng_ = 0x8000;
  int cnt_ = 0;
};

}  // namespace av1
}  // namespace tv
