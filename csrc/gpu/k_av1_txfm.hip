// k_av1_txfm.hip — AV1 2-D transforms (DCT / ADST / FLIPADST / IDTX, 4..64) on gfx950
// matrix cores.  Bit-exact with tv::av1::txfm2d_ref (av1_tools.cpp).
//
// One wavefront owns one N x N block (N >= 16): the block lives in LDS, each stage is a
// set of 16x16 output tiles of v_mfma_f32_16x16x16f16.  Stage operands are integers within
// int16 (basis <= 23170, data clamped to int16); each is split as v = 256*hi + lo with
// |hi| <= 128 and 0 <= lo <= 255 — exact in f16 — and the tile is accumulated in three
// f32 accumulators (hi*hi, hi*lo + lo*hi, lo*lo) whose partial sums stay below 2^24, then
// recombined exactly in int64.  4x4 and 8x8 blocks use one lane per coefficient (VALU).
#include <hip/hip_runtime.h>

#include <string>

#include "gpu_common.h"
#include "mfma_exact.h"
#include "tv/av1_txfm.h"

namespace tv {
namespace gpu {
namespace {

// one stage over the whole N x N block on the calling wave
template <class FA, class FB, class EMIT>
__device__ __forceinline__ void wave_mm(int N, FA A, FB B, EMIT emit) {
  const int lane = threadIdx.x & 63, nt = N >> 4;
  for (int t = 0; t < nt * nt; ++t) {
    const int ti = t / nt, tj = t - ti * nt;
    long long o[4];
    exact_tile(A, B, ti, tj, N, o);
#pragma unroll
    for (int r = 0; r < 4; ++r) emit(16 * ti + (lane >> 4) * 4 + r, 16 * tj + (lane & 15), o[r]);
  }
}

constexpr int kMaxN = 64;

// Large blocks: one wave per block, LDS = block + intermediate (int, padded rows).
__global__ void __launch_bounds__(64) k_av1_txfm_mfma(const int16_t* __restrict__ in, int16_t* __restrict__ out,
                                                      int nblk, int log2N, int inverse, const int* __restrict__ Bc,
                                                      const int* __restrict__ Br, int s1, int s2) {
  const int blk = blockIdx.x, N = 1 << log2N, n2 = N * N, lane = threadIdx.x;
  if (blk >= nblk) return;
  __shared__ int X[kMaxN * (kMaxN + 1)];
  __shared__ int T[kMaxN * (kMaxN + 1)];
  const int P = N + 1;
  for (int i = lane; i < n2; i += 64) X[(i >> log2N) * P + (i & (N - 1))] = in[(long)blk * n2 + i];
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (!inverse) {
    wave_mm(N, [&](int r, int k) { return Bc[r * N + k]; }, [&](int k, int c) { return X[k * P + c]; },
            [&](int r, int c, long long v) { T[r * P + c] = clamp16(rshift_round(v, s1)); });
  } else {
    wave_mm(N, [&](int r, int k) { return X[r * P + k]; }, [&](int k, int c) { return Br[k * N + c]; },
            [&](int r, int c, long long v) { T[r * P + c] = clamp16(rshift_round(v, s1)); });
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  int16_t* o = out + (long)blk * n2;
  if (!inverse) {
    wave_mm(N, [&](int r, int k) { return T[r * P + k]; }, [&](int k, int c) { return Br[c * N + k]; },
            [&](int r, int c, long long v) { o[r * N + c] = (int16_t)clamp16(rshift_round(v, s2)); });
  } else {
    wave_mm(N, [&](int r, int k) { return Bc[k * N + r]; }, [&](int k, int c) { return T[k * P + c]; },
            [&](int r, int c, long long v) { o[r * N + c] = (int16_t)clamp16(rshift_round(v, s2)); });
  }
}

// Small blocks (4x4, 8x8): one lane per output coefficient, 64 / N^2 blocks per wave.
__global__ void __launch_bounds__(256) k_av1_txfm_small(const int16_t* __restrict__ in, int16_t* __restrict__ out,
                                                        int nblk, int log2N, int inverse, const int* __restrict__ Bc,
                                                        const int* __restrict__ Br, int s1, int s2) {
  const int N = 1 << log2N, n2 = N * N;
  const int per = 256 / n2;  // blocks per workgroup
  const int lb = threadIdx.x / n2, e = threadIdx.x % n2, r = e >> log2N, c = e & (N - 1);
  const int blk = blockIdx.x * per + lb;
  __shared__ int X[256], T[256];
  const bool ok = blk < nblk;
  X[threadIdx.x] = ok ? in[(long)blk * n2 + e] : 0;
  __syncthreads();
  const int* x = X + lb * n2;
  long long s = 0;
  for (int k = 0; k < N; ++k)
    s += inverse ? (long long)x[r * N + k] * Br[k * N + c] : (long long)Bc[r * N + k] * x[k * N + c];
  T[threadIdx.x] = clamp16(rshift_round(s, s1));
  __syncthreads();
  const int* t = T + lb * n2;
  s = 0;
  for (int k = 0; k < N; ++k)
    s += inverse ? (long long)Bc[k * N + r] * t[k * N + c] : (long long)t[r * N + k] * Br[c * N + k];
  if (ok) out[(long)blk * n2 + e] = (int16_t)clamp16(rshift_round(s, s2));
}

thread_local std::string g_txfm_err;

}  // namespace
}  // namespace gpu
}  // namespace tv

extern "C" {
const char* tv_av1_txfm_last_error() { return tv::gpu::g_txfm_err.c_str(); }

// nblk N x N int16 blocks (row-major, back to back); Bc / Br: device N x N int32 bases of
// the column / row 1-D transforms (tv_av1_txfm_basis).  inverse: rows then columns.
int tv_gpu_av1_txfm(const int16_t* in, int16_t* out, int nblk, int log2N, int inverse, const int* Bc, const int* Br,
                    void* stream) {
  using namespace tv::gpu;
  if (log2N < 2 || log2N > 6 || nblk < 1) {
    g_txfm_err = "av1_txfm: bad size";
    return -1;
  }
  int f1, f2, i1, i2;
  tv::av1::txfm_shifts(log2N, f1, f2, i1, i2);
  const int s1 = inverse ? i1 : f1, s2 = inverse ? i2 : f2;
  auto st = static_cast<hipStream_t>(stream);
  if (log2N >= 4) {
    k_av1_txfm_mfma<<<nblk, 64, 0, st>>>(in, out, nblk, log2N, inverse, Bc, Br, s1, s2);
  } else {
    const int per = 256 >> (2 * log2N);
    k_av1_txfm_small<<<(nblk + per - 1) / per, 256, 0, st>>>(in, out, nblk, log2N, inverse, Bc, Br, s1, s2);
  }
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_txfm_err = hipGetErrorString(e);
    return -1;
  }
  return 0;
}
}
