// mfma_exact.h — exact integer 16x16 tile products on the gfx950 matrix cores, shared by
// the AV1 transform kernels (k_av1_txfm.hip) and the AV1 encoder's block transforms
// (k_av1_enc.hip).  Operands are integers within int16; each is split as v = 256*hi + lo
// with |hi| <= 128 and 0 <= lo <= 255 (exact in f16) and the tile is accumulated in three
// f32 accumulators (hi*hi, hi*lo + lo*hi, lo*lo) whose partial sums stay below 2^24 for
// K <= 64, then recombined exactly in int64.
#pragma once
#include <hip/hip_runtime.h>

namespace tv {
namespace gpu {
namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int rshift_round(long long v, int s) { return (int)((v + (1LL << (s - 1))) >> s); }
__device__ __forceinline__ int clamp16(int v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }

// P[i][j] = sum_k A(i, k) * B(k, j) for the 16x16 tile (ti, tj) over K (multiple of 16);
// lane l receives rows 16*ti + (l >> 4) * 4 + r (r = 0..3) of column 16*tj + (l & 15).
template <class FA, class FB>
__device__ __forceinline__ void exact_tile(FA A, FB B, int ti, int tj, int K, long long out[4]) {
  const int lane = threadIdx.x & 63, i = lane & 15, kq = lane >> 4;
  f4 hh = {0.f, 0.f, 0.f, 0.f}, mid = hh, ll = hh;
  for (int kk = 0; kk < K; kk += 16) {
    h4 ah, al, bh, bl;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = kk + 4 * kq + e;
      const int a = A(16 * ti + i, k), b = B(k, 16 * tj + i);
      ah[e] = (_Float16)(a >> 8);
      al[e] = (_Float16)(a & 255);
      bh[e] = (_Float16)(b >> 8);
      bl[e] = (_Float16)(b & 255);
    }
    hh = __builtin_amdgcn_mfma_f32_16x16x16f16(ah, bh, hh, 0, 0, 0);
    mid = __builtin_amdgcn_mfma_f32_16x16x16f16(ah, bl, mid, 0, 0, 0);
    mid = __builtin_amdgcn_mfma_f32_16x16x16f16(al, bh, mid, 0, 0, 0);
    ll = __builtin_amdgcn_mfma_f32_16x16x16f16(al, bl, ll, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) out[r] = (long long)hh[r] * 65536 + (long long)mid[r] * 256 + (long long)ll[r];
}


}  // namespace
}  // namespace gpu
}  // namespace tv
