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
  int rdoq = 0;    // k_inter_recon RDOQ-lite mode (hevc_defs.h kRdoqMode; 0 off): SeqConfig::rdoq
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
  int8_t* qp;  // [B] slice QP of this frame per segment (rate control)
  uint8_t* cu_log2;
  uint8_t* intra;
  uint8_t* ipm;
  int16_t* mv;
  uint8_t* cbf;
  int16_t* coef_y;
  int16_t* coef_u;
  int16_t* coef_v;
  // B pictures only (nullptr otherwise): per-unit direction (1 L0, 2 L1, 3 bi), list-1 MVs
  uint8_t* dir = nullptr;
  int16_t* mv1 = nullptr;
  // P pictures with RQT (hevc_defs.h rqt_split): 1 = the unit's 32x32 inter CU codes four
  // 16x16 TBs; written by k_inter_recon for every unit (nullptr: no splits)
  uint8_t* tu = nullptr;
};

// ---- wave-level data movement on the VALU (DPP) instead of LDS (ds_bpermute) ----------
// A __shfl_xor is a ds_bpermute: an LDS round trip (~100+ cycles) per step, and reduction
// chains of them serialise.  Within a 16-lane row DPP permutes are free operand modifiers;
// the four row results are then combined with v_readlane (scalar).  Requires a full wave.
namespace dpp {
constexpr int kQuadXor1 = 0xB1;       // quad_perm [1,0,3,2]
constexpr int kQuadXor2 = 0x4E;       // quad_perm [2,3,0,1]
constexpr int kRowShl4 = 0x104, kRowShr4 = 0x114, kRowShl8 = 0x108, kRowShr8 = 0x118;
constexpr int kRowRor8 = 0x128;      // lane i <- i ^ 8 within 16 (rotate by 8)
constexpr int kRowRor4 = 0x124;      // lane i <- (i - 4) mod 16 within the row
constexpr int kRowHalfMirror = 0x141;  // lane i <- 7 - i within 8
constexpr int kRowMirror = 0x140;      // lane i <- 15 - i within 16
template <int CTRL> __device__ __forceinline__ int mov(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
}  // namespace dpp

// ---- XCD-aware workgroup placement (guide T1) -------------------------------------------
// Workgroups are dealt round-robin to the 8 XCDs, each with a private 4 MB L2.  Neighbouring
// CTBs read overlapping reference windows / phase-plane rows (four CTBs share a 128-byte
// line), so the default placement makes every XCD fetch the same lines.  Remap the linear
// workgroup id so each XCD walks one contiguous run of the logical grid.  Bijective for any
// grid size; placement only changes speed, never results.
__device__ __forceinline__ int xcd_remap(int id, int n) {
  const int per = (n + 7) >> 3, r = n & 7;  // r == 0: every XCD owns `per` workgroups
  const int x = id & 7, s = id >> 3;
  return x * per - (r && x > r ? x - r : 0) + s;
}
// (CTB, segment) of this workgroup in a gridDim = (CTBs, segments) launch
__device__ __forceinline__ void xcd_ctb(int& ctu, int& b) {
  const int L = xcd_remap(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y);
  ctu = L % gridDim.x;
  b = L / gridDim.x;
}

#ifdef TV_NO_DPP  // ds_bpermute reference implementations (debug builds)
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
#else
__device__ __forceinline__ int wave_sum(int v) {
  v += dpp::mov<dpp::kQuadXor1>(v);
  v += dpp::mov<dpp::kQuadXor2>(v);
  v += dpp::mov<dpp::kRowHalfMirror>(v);
  v += dpp::mov<dpp::kRowMirror>(v);  // every lane: its 16-lane row sum
  return __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16) + __builtin_amdgcn_readlane(v, 32) +
         __builtin_amdgcn_readlane(v, 48);
}
__device__ __forceinline__ unsigned umin2(unsigned a, unsigned b) { return a < b ? a : b; }
__device__ __forceinline__ unsigned wave_min_u32(unsigned v) {
  v = umin2(v, (unsigned)dpp::mov<dpp::kQuadXor1>((int)v));
  v = umin2(v, (unsigned)dpp::mov<dpp::kQuadXor2>((int)v));
  v = umin2(v, (unsigned)dpp::mov<dpp::kRowHalfMirror>((int)v));
  v = umin2(v, (unsigned)dpp::mov<dpp::kRowMirror>((int)v));
  const unsigned a = (unsigned)__builtin_amdgcn_readlane((int)v, 0), b = (unsigned)__builtin_amdgcn_readlane((int)v, 16);
  const unsigned c = (unsigned)__builtin_amdgcn_readlane((int)v, 32), d = (unsigned)__builtin_amdgcn_readlane((int)v, 48);
  return umin2(umin2(a, b), umin2(c, d));
}
#endif
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
#ifdef TV_NO_DPP
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) {
    const int p = __shfl_xor(d, s, 64);
    d = (lane & s) ? (p - d) : (d + p);
  }
  return (wave_sum(tv_abs(d)) + 2) >> 2;
#endif
  // butterflies over x (lane bits 0..2) and the first y bit (lane bit 3) stay inside a
  // 16-lane row: DPP.  Only the two cross-row stages (y bits 1, 2) use ds_bpermute.
  int p = dpp::mov<dpp::kQuadXor1>(d);
  d = (lane & 1) ? (p - d) : (d + p);
  p = dpp::mov<dpp::kQuadXor2>(d);
  d = (lane & 2) ? (p - d) : (d + p);
  // Both shifts are evaluated by the whole wave: a DPP op inside a divergent branch (which
  // `c ? dpp_a : dpp_b` is, since the intrinsic is convergent) reads disabled lanes.
  int pr = dpp::mov<dpp::kRowShr4>(d), pl = dpp::mov<dpp::kRowShl4>(d);
  d = (lane & 4) ? (pr - d) : (d + pl);
  pr = dpp::mov<dpp::kRowShr8>(d);
  pl = dpp::mov<dpp::kRowShl8>(d);
  d = (lane & 8) ? (pr - d) : (d + pl);
#pragma unroll
  for (int s = 16; s < 64; s <<= 1) {
    p = __shfl_xor(d, s, 64);
    d = (lane & s) ? (p - d) : (d + p);
  }
  return (wave_sum(tv_abs(d)) + 2) >> 2;
}

}  // namespace gpu
}  // namespace tv
