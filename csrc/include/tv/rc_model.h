// rc_model.h — in-engine CRF rate control shared by the CPU golden model and the gfx950
// kernels (integer-only, so both pick identical per-frame QPs).
//
// The lookahead of the hierarchical motion search gives every frame a complexity before it
// is coded: a P frame's quarter-resolution coarse-search cost summed over CTBs, an IDR
// frame's quarter-resolution activity (sum of |q - mean| per 8x8 quarter block).  x264's
// CRF curve (qcomp = 0.6: qscale ~ complexity^0.4, i.e. QP = crf + 2.4 log2(c / c_ref)),
// I frames at -3 (ipratio 1.4), clamped to crf +- 8.
#pragma once
#include "hevc_defs.h"

namespace tv {

// floor(256 * log2(x)) for x >= 1, integer only (8 fraction bits by repeated squaring)
TV_HD int rc_log2_q8(uint32_t x) {
  if (x < 1) x = 1;
  int e = 31;
  while (!(x >> e)) --e;
  uint64_t y = (uint64_t)x << (31 - e);  // Q31 mantissa in [2^31, 2^32)
  int r = e << 8;
  for (int b = 7; b >= 0; --b) {
    y = (y * y) >> 31;
    if (y >= (1ull << 32)) {
      r |= 1 << b;
      y >>= 1;
    }
  }
  return r;
}

// reference complexities per CTB (quarter-res units): the QP offset is 0 at these
constexpr uint32_t kRcRefInter = 640;   // coarse SAD + rate per 8x8 quarter block
constexpr uint32_t kRcRefIntra = 1024;  // activity per 8x8 quarter block

// frame QP from its summed complexity over `nctb` CTBs
TV_HD int rc_crf_qp(int crf, bool intra, uint64_t sum, int nctb) {
  const uint32_t per = (uint32_t)((sum + (uint64_t)nctb / 2) / (uint64_t)(nctb > 0 ? nctb : 1));
  const int d = rc_log2_q8(per > 0 ? per : 1) - rc_log2_q8(intra ? kRcRefIntra : kRcRefInter);
  // round(2.4 * d / 256) = round(24 d / 2560)
  const int off = d >= 0 ? (24 * d + 1280) / 2560 : -((-24 * d + 1280) / 2560);
  const int q = crf + (intra ? -3 : 0) + clip3(-8, 8, off);
  return clip3(0, 51, q);
}

// activity of one 8x8 quarter-res block: sum |q - round(mean)|
TV_HD uint32_t rc_block_activity(const uint8_t* q, int stride) {
  int s = 0;
  for (int j = 0; j < 8; ++j)
    for (int i = 0; i < 8; ++i) s += q[j * stride + i];
  const int m = (s + 32) >> 6;
  uint32_t a = 0;
  for (int j = 0; j < 8; ++j)
    for (int i = 0; i < 8; ++i) a += (uint32_t)tv_abs(q[j * stride + i] - m);
  return a;
}

}  // namespace tv
