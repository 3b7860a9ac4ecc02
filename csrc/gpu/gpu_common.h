// gpu_common.h — device-side helpers shared by the gfx950 encoder kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "tv/hevc_defs.h"

namespace tv {
namespace gpu {

constexpr int kWave = 64;  // CDNA wavefront

// Geometry of one coded picture (all planes tightly packed, pitch == width).
struct Geo {
  int W, H;        // coded luma size (multiples of 32)
  int dw, dh;      // display size
  int w8, h8;      // 8x8 units
  int wc, hc;      // CTBs
  long ysz, csz;   // plane sizes (bytes / elements)
  long usz;        // units
  int pw16;        // phase-plane pitch (W + 16: 8-sample pad each side)
  long psz;        // phase-plane size ((W + 16) * (H + 16))
};

inline Geo make_geo(int dw, int dh) {
  Geo g;
  g.dw = dw;
  g.dh = dh;
  g.W = (dw + kCtb - 1) / kCtb * kCtb;
  g.H = (dh + kCtb - 1) / kCtb * kCtb;
  g.w8 = g.W / 8;
  g.h8 = g.H / 8;
  g.wc = g.W / kCtb;
  g.hc = g.H / kCtb;
  g.ysz = (long)g.W * g.H;
  g.csz = g.ysz / 4;
  g.usz = (long)g.w8 * g.h8;
  g.pw16 = g.W + 16;
  g.psz = (long)(g.W + 16) * (g.H + 16);
  return g;
}

// Per-batch frame buffers: element b of a plane array lives at base + b * size.
struct FrameSet {
  uint8_t* y;
  uint8_t* u;
  uint8_t* v;
  __device__ __host__ uint8_t* plane(int c, int b, const Geo& g) const {
    return c == 0 ? y + b * g.ysz : (c == 1 ? u + b * g.csz : v + b * g.csz);
  }
};

struct DecisionSet {
  uint8_t* cu_log2;
  uint8_t* intra;
  uint8_t* ipm;
  int16_t* mv;
  uint8_t* cbf;
  int16_t* coef_y;
  int16_t* coef_u;
  int16_t* coef_v;
};

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ unsigned wave_min_u32(unsigned v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    unsigned w = __shfl_xor(v, o, 64);
    v = w < v ? w : v;
  }
  return v;
}
__device__ __forceinline__ unsigned long long wave_min_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    unsigned long long w = __shfl_xor(v, o, 64);
    v = w < v ? w : v;
  }
  return v;
}

// 8x8 SATD computed by one wavefront, lane l holds difference d at (x = l&7, y = l>>3).
// Matches tv satd8x8 on the CPU: (sum |H d H| + 2) >> 2.
__device__ __forceinline__ int wave_satd8x8(int d) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) {
    const int p = __shfl_xor(d, s, 64);
    d = (lane & s) ? (p - d) : (d + p);
  }
  return (wave_sum(tv_abs(d)) + 2) >> 2;
}

}  // namespace gpu
}  // namespace tv
