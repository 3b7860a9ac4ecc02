// tb_coder.h — workgroup-cooperative transform-block coding on gfx950 matrix cores.
//
// Forward DCT, deadzone quantisation, dequantisation and the normative inverse DCT of one
// N x N TB.  The 16- and 32-point 2-D transforms run as 16x16 output tiles of
// v_mfma_f32_16x16x4_f32 (exact f32 MFMA, one wave per tile).  Every MFMA product stays an
// exact integer: operands that can exceed 8 bits (intermediate rows, dequantised levels)
// are split as v = 256*hi + lo and accumulated in two chains, so each chain's partial sums
// are < 2^24 and the int32 recombination is bit-identical to the scalar golden model
// (tv::forward_transform / tv::inverse_transform).  4- and 8-point TBs use the VALU.
#pragma once
#include "gpu_common.h"

namespace tv {
namespace gpu {

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int tbT(const int (*T)[33], int log2N, int k, int n) {
  return T[k << (5 - log2N)][n];
}
__device__ inline void tb_load_matrix(int (*T)[33]) {
  for (int i = threadIdx.x; i < 1024; i += blockDim.x) T[i >> 5][i & 31] = kDct32.m[i >> 5][i & 31];
}

// One 16x16 output tile P = X * Y (K = 16 or 32) on the calling wave.  X(i,k), Y(k,j) are
// callables returning ints (exactly representable in f32).  When `split`, the operand
// selected by `split_x` is decomposed into 8-bit halves and the tile recombined in int32.
//
// gfx950 path: the whole K = 32 (16) reduction is ONE v_mfma_f32_16x16x32_f16
// (16x16x16f16) per split half.  Every operand is an integer of at most 9 bits (DCT basis
// <= 90, residual / split halves within +-256), so it is exact in f16, every product is
// exact in f32 and all partial sums stay below 2^24: bit-identical to the scalar model,
// with 4-8x fewer matrix instructions than the f32 16x16x4 chain (TV_MFMA_F32 keeps that).
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));

template <class FX, class FY>
__device__ __forceinline__ void mfma_tile(FX X, FY Y, int ti, int tj, int K, bool split, bool split_x,
                                          int out[4]) {
  const int lane = threadIdx.x & 63, i = lane & 15, kq = lane >> 4;
  f32x4 hi = {0.f, 0.f, 0.f, 0.f}, lo = {0.f, 0.f, 0.f, 0.f};
#ifndef TV_MFMA_F32
  if (K == 32) {
    h8 a, b, a2, b2;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int k = 8 * kq + e;
      const int xv = X(16 * ti + i, k), yv = Y(k, 16 * tj + i);
      const bool sx = split && split_x, sy = split && !split_x;
      a[e] = (_Float16)(sx ? (xv >> 8) : xv);
      a2[e] = (_Float16)(xv & 255);
      b[e] = (_Float16)(sy ? (yv >> 8) : yv);
      b2[e] = (_Float16)(yv & 255);
    }
    hi = __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, hi, 0, 0, 0);
    if (split) lo = split_x ? __builtin_amdgcn_mfma_f32_16x16x32_f16(a2, b, lo, 0, 0, 0)
                            : __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b2, lo, 0, 0, 0);
  } else {
    h4 a, b, a2, b2;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = 4 * kq + e;
      const int xv = X(16 * ti + i, k), yv = Y(k, 16 * tj + i);
      const bool sx = split && split_x, sy = split && !split_x;
      a[e] = (_Float16)(sx ? (xv >> 8) : xv);
      a2[e] = (_Float16)(xv & 255);
      b[e] = (_Float16)(sy ? (yv >> 8) : yv);
      b2[e] = (_Float16)(yv & 255);
    }
    hi = __builtin_amdgcn_mfma_f32_16x16x16f16(a, b, hi, 0, 0, 0);
    if (split) lo = split_x ? __builtin_amdgcn_mfma_f32_16x16x16f16(a2, b, lo, 0, 0, 0)
                            : __builtin_amdgcn_mfma_f32_16x16x16f16(a, b2, lo, 0, 0, 0);
  }
#else
  for (int kk = 0; kk < K; kk += 4) {
    const int xv = X(16 * ti + i, kk + kq), yv = Y(kk + kq, 16 * tj + i);
    if (!split) {
      hi = __builtin_amdgcn_mfma_f32_16x16x4f32((float)xv, (float)yv, hi, 0, 0, 0);
    } else if (split_x) {
      hi = __builtin_amdgcn_mfma_f32_16x16x4f32((float)(xv >> 8), (float)yv, hi, 0, 0, 0);
      lo = __builtin_amdgcn_mfma_f32_16x16x4f32((float)(xv & 255), (float)yv, lo, 0, 0, 0);
    } else {
      hi = __builtin_amdgcn_mfma_f32_16x16x4f32((float)xv, (float)(yv >> 8), hi, 0, 0, 0);
      lo = __builtin_amdgcn_mfma_f32_16x16x4f32((float)xv, (float)(yv & 255), lo, 0, 0, 0);
    }
  }
#endif
#pragma unroll
  for (int r = 0; r < 4; ++r) out[r] = split ? (int)hi[r] * 256 + (int)lo[r] : (int)hi[r];
}

// Run a stage over the whole N x N output: each wave owns 16x16 tiles; N <= 8 uses VALU.
// `emit(row, col, value)` stores the stage output.  All threads must call (no barrier here).
template <class FX, class FY, class EMIT>
__device__ __forceinline__ void tb_stage(int log2N, FX X, FY Y, bool split, bool split_x, EMIT emit) {
  const int N = 1 << log2N;
  if (N >= 16) {
    const int tiles = (N >> 4) * (N >> 4);
    const int wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    for (int t = wave; t < tiles; t += nw) {
      const int ti = t / (N >> 4), tj = t % (N >> 4);
      int o[4];
      mfma_tile(X, Y, ti, tj, N, split, split_x, o);
      const int lane = threadIdx.x & 63;
#pragma unroll
      for (int r = 0; r < 4; ++r) emit(16 * ti + (lane >> 4) * 4 + r, 16 * tj + (lane & 15), o[r]);
    }
  } else {
    for (int e = threadIdx.x; e < N * N; e += blockDim.x) {
      const int r = e >> log2N, c = e & (N - 1);
      int acc = 0;
      for (int k = 0; k < N; ++k) acc += X(r, k) * Y(k, c);
      emit(r, c, acc);
    }
  }
}

// Code one TB with the whole workgroup (each wave owns 16x16 output tiles of a stage;
// workgroup barriers between stages).  resid/pred are LDS arrays (N*N row-major), tbm the
// DCT matrix in LDS, `tmp`/`coef` LDS scratch, `red` 4 LDS ints.  Writes levels to `lev`
// (stride ls) and reconstructed pixels to `rec` (stride rs).  Returns cbf (uniform).
// Same arithmetic as wave_code_tb (wave_tb.h) and tv::forward/inverse_transform.
template <class PredT, class RecT>
__device__ int wg_code_tb(const int16_t* resid, const PredT* pred, int log2N, int qp, bool intra, int16_t* lev,
                          int ls, RecT* rec, int rs, const int (*tbm)[33], int* tmp, int* coef, int* red) {
  const int N = 1 << log2N, n2 = N * N, tid = threadIdx.x, nt = blockDim.x;
  const int sh1 = log2N - 1, sh2 = log2N + 6;
  if (tid < 4) red[tid] = 0;
  // forward stage 1: tmp[k][x] = (sum_y T[k][y] r[y][x] + rnd) >> sh1     (operands <= 9 bit)
  tb_stage(
      log2N, [&](int k, int y) { return tbT(tbm, log2N, k, y); }, [&](int y, int x) { return (int)resid[y * N + x]; },
      false, false, [&](int r, int c, int v) { tmp[r * 33 + c] = (v + (1 << (sh1 - 1))) >> sh1; });
  __syncthreads();
  // forward stage 2 + quantisation: coef[k][j] = (sum_x tmp[k][x] T[j][x] + rnd) >> sh2
  tb_stage(
      log2N, [&](int k, int x) { return tmp[k * 33 + x]; }, [&](int x, int j) { return tbT(tbm, log2N, j, x); },
      true, true, [&](int r, int c, int v) {
        coef[r * N + c] = quant_level((v + (1 << (sh2 - 1))) >> sh2, qp, log2N, intra);
      });
  __syncthreads();
  int nz = 0, sa = 0;
  for (int i = tid; i < n2; i += nt) {
    nz += coef[i] != 0;
    sa += tv_abs(coef[i]);
  }
  nz = wave_sum(nz);
  sa = wave_sum(sa);
  if ((tid & 63) == 0) {
    atomicAdd(&red[0], nz);
    atomicAdd(&red[1], sa);
  }
  __syncthreads();
  const int NZ = (!intra && red[0] == 1 && red[1] == 1 && coef[0] == 0) ? 0 : red[0];
  for (int i = tid; i < n2; i += nt) {
    const int l = NZ ? coef[i] : 0;
    lev[(i >> log2N) * ls + (i & (N - 1))] = (int16_t)l;
    if (!NZ) rec[(i >> log2N) * rs + (i & (N - 1))] = (RecT)clip_pixel((int)pred[i]);
    else coef[i] = dequant_level(l, qp, log2N);
  }
  __syncthreads();
  if (!NZ) return 0;
  // inverse stage 1: tmp[y][x] = clip16((sum_k T[k][y] d[k][x] + 64) >> 7)   (split d)
  tb_stage(
      log2N, [&](int y, int k) { return tbT(tbm, log2N, k, y); }, [&](int k, int x) { return coef[k * N + x]; },
      true, false, [&](int r, int c, int v) { tmp[r * 33 + c] = clip3(-32768, 32767, (v + 64) >> 7); });
  __syncthreads();
  // inverse stage 2: res[y][x] = (sum_k g[y][k] T[k][x] + 2048) >> 12            (split g)
  tb_stage(
      log2N, [&](int y, int k) { return tmp[y * 33 + k]; }, [&](int k, int x) { return tbT(tbm, log2N, k, x); },
      true, true, [&](int r, int c, int v) {
        rec[r * rs + c] = (RecT)clip_pixel((int)pred[r * N + c] + ((v + 2048) >> 12));
      });
  __syncthreads();
  return 1;
}

}  // namespace gpu
}  // namespace tv
