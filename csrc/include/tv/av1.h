// av1.h — AV1 coding tools of the C++ golden model: CDEF, loop
// restoration (Wiener, self-guided) with their encoder-side searches, and the AV1
// multi-symbol range coder with adaptive 15-bit CDFs.  The gfx950 kernels in
// csrc/gpu/k_av1.hip implement the same filters/statistics bit-exactly (av1_defs.h).
#pragma once
#include <cstddef>
#include <cstdint>
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

// ---- deblocking loop filter (AV1 7.14) -------------------------------------------------
// Filter every tx edge of a plane: `info` holds one word per 4x4 unit (layout in
// av1_defs.h: tx / block log2 sizes, per-direction levels, skip && inter); sharp 0..7.
void deblock(const uint8_t* in, int w, int h, bool chroma, const uint32_t* info, int sharp, uint8_t* out);

// ---- multi-symbol range coder -------------------------------------------------------------
// Probabilities are AV1 inverse CDFs: icdf[i] = 32768 * P(X > i), icdf[n-1] = 0, plus one
// adaptation counter at icdf[n] (n <= 16).
void cdf_init_uniform(uint16_t* icdf, int n);
void cdf_adapt(uint16_t* icdf, int n, int sym);

class RangeEncoder {
 public:
  void encode(int sym, uint16_t* icdf, int n, bool adapt = true);
  void encode_bool(int bit, int p0_q15);  // p0 = P(bit == 0) in 1/32768
  void encode_literal(uint32_t v, int bits);
  std::vector<uint8_t> finish();
  size_t bits_written() const;

 private:
  void emit(uint32_t low_new, uint32_t rng_new);
  uint64_t low_ = 0;
  uint32_t rng_ = 0x8000;
  int cnt_ = -9;
  std::vector<uint16_t> pre_;  // pre-carry bytes
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
