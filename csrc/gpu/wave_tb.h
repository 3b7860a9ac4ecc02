// wave_tb.h — wave-synchronous (one 64-lane wavefront, no workgroup barriers) coding of
// one transform block: forward DCT + quantisation + dequantisation + exact inverse DCT +
// reconstruction.  16/32-point stages run on v_mfma_f32_16x16x4_f32 with the 8-bit split
// that keeps every partial sum exact (see tb_coder.h); 4/8-point stages use one lane per
// output.  Used where a whole CTU is owned by one wave (wavefront intra reconstruction),
// so a TB costs no __syncthreads at all — only LDS ordering within the wave.
#pragma once
#include "gpu_common.h"
#include "tb_coder.h"

namespace tv {
namespace gpu {

// Order LDS accesses between the lanes of this wave.  A wave's DS instructions execute in
// issue order, so only the compiler has to be stopped from moving memory operations across;
// a wavefront-scope fence emits no wait at all (a workgroup-scope fence would also wait for
// every outstanding global store, vmcnt(0), which dominated the wavefront latency).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// scratch of TBs up to N_MAX x N_MAX (stage outputs at pitch 33, coefficients at pitch N)
template <int N_MAX>
struct WaveTbScratchT {
  int tmp[N_MAX * 33];
  int coef[N_MAX * N_MAX];
};
using WaveTbScratch = WaveTbScratchT<32>;

template <class FX, class FY, class EMIT>
__device__ __forceinline__ void wave_stage(int log2N, FX X, FY Y, bool split, bool split_x, EMIT emit) {
  const int N = 1 << log2N, lane = threadIdx.x & 63;
  if (N >= 16) {
    const int nt = N >> 4;
    for (int t = 0; t < nt * nt; ++t) {
      const int ti = t / nt, tj = t - ti * nt;
      int o[4];
      mfma_tile(X, Y, ti, tj, N, split, split_x, o);
#pragma unroll
      for (int r = 0; r < 4; ++r) emit(16 * ti + (lane >> 4) * 4 + r, 16 * tj + (lane & 15), o[r]);
    }
  } else {
    for (int e = lane; e < N * N; e += 64) {
      const int r = e >> log2N, c = e & (N - 1);
      int acc = 0;
      for (int k = 0; k < N; ++k) acc += X(r, k) * Y(k, c);
      emit(r, c, acc);
    }
  }
}

// resid/pred: LDS N*N (pred may be uint8).  Levels -> `lev` (global, stride ls);
// reconstruction -> `rec` (LDS or global, stride rs).  Returns cbf (wave-uniform).
template <class PredT, class RecT, class Scratch>
__device__ __forceinline__ int wave_code_tb(const int16_t* resid, const PredT* pred, int log2N, int qp, bool intra,
                            int16_t* lev, int ls, RecT* rec, int rs, const int (*tbm)[33], Scratch& s) {
  const int N = 1 << log2N, n2 = N * N, lane = threadIdx.x & 63;
  const int sh1 = log2N - 1, sh2 = log2N + 6;
  wave_stage(
      log2N, [&](int k, int y) { return tbT(tbm, log2N, k, y); }, [&](int y, int x) { return (int)resid[y * N + x]; },
      false, false, [&](int r, int c, int v) { s.tmp[r * 33 + c] = (v + (1 << (sh1 - 1))) >> sh1; });
  wave_sync();
  wave_stage(
      log2N, [&](int k, int x) { return s.tmp[k * 33 + x]; }, [&](int x, int j) { return tbT(tbm, log2N, j, x); },
      true, true, [&](int r, int c, int v) {
        s.coef[r * N + c] = quant_level((v + (1 << (sh2 - 1))) >> sh2, qp, log2N, intra);
      });
  wave_sync();
  int nz = 0, sa = 0;
  for (int i = lane; i < n2; i += 64) {
    nz += s.coef[i] != 0;
    sa += tv_abs(s.coef[i]);
  }
  nz = wave_sum(nz);
  sa = wave_sum(sa);
  const int NZ = (!intra && nz == 1 && sa == 1 && s.coef[0] == 0) ? 0 : nz;
  for (int i = lane; i < n2; i += 64) {
    const int l = NZ ? s.coef[i] : 0;
    lev[(i >> log2N) * ls + (i & (N - 1))] = (int16_t)l;
    if (!NZ) rec[(i >> log2N) * rs + (i & (N - 1))] = (RecT)clip_pixel((int)pred[i]);
  }
  wave_sync();
  if (!NZ) return 0;
  for (int i = lane; i < n2; i += 64) s.coef[i] = dequant_level(s.coef[i], qp, log2N);
  wave_sync();
  wave_stage(
      log2N, [&](int y, int k) { return tbT(tbm, log2N, k, y); }, [&](int k, int x) { return s.coef[k * N + x]; },
      true, false, [&](int r, int c, int v) { s.tmp[r * 33 + c] = clip3(-32768, 32767, (v + 64) >> 7); });
  wave_sync();
  wave_stage(
      log2N, [&](int y, int k) { return s.tmp[y * 33 + k]; }, [&](int k, int x) { return tbT(tbm, log2N, k, x); },
      true, true, [&](int r, int c, int v) {
        rec[r * rs + c] = (RecT)clip_pixel((int)pred[r * N + c] + ((v + 2048) >> 12));
      });
  wave_sync();
  return 1;
}

}  // namespace gpu
}  // namespace tv
