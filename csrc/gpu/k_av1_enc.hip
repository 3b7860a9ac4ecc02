// k_av1_enc.hip — gfx950 kernels of the AV1 encode engine (BASELINE
// config #4).  Every decision and reconstruction equals the C++ golden encoder
// (csrc/core/av1_codec.cpp golden_encode) bit for bit; the shared arithmetic lives in
// tv/av1_enc.h (TV_HD) and the integer transform stages follow av1_txfm.h exactly.
//
//   k_av1e_inter   one wave per 16x16 block (P frames): reference window staged in LDS
//                  (57 x 57 bytes, clamped), full-pel +-16 search on packed v_sad_u8 with
//                  alignbyte-unaligned LDS rows, half- then quarter-pel refinement (4
//                  candidates x 16 4x4-SATD lanes per pass, 16-lane DPP reductions),
//                  luma / chroma prediction, forward transform, quantisation,
//                  dequantisation, the specification's inverse transform, reconstruction.
//   k_av1e_intra   one wave per 16x16 block of an anti-diagonal (key frames): the seven
//                  candidate modes read no above-right samples, so the frame is a plain
//                  (rows + cols - 1)-step wavefront; 4 luma modes x 16 lanes per pass, all
//                  7 chroma modes x 8 lanes (U + V 4x4 SATDs) in one pass.
//   k_av1e_lfinfo  deblocking info words (tx / block sizes, levels, skip && inter).
//   k_av1e_cdef_choose  one workgroup per segment: greedy 8-preset CDEF table from the
//                  k_cdef_search SSEs of the active 64x64 blocks (identical to cdef_choose).
// Grids are (blocks, segments): one launch covers the same frame of every segment.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include <cstdlib>

#include "gpu_common.h"
#include "mfma_exact.h"
#include "tv/av1_defs.h"
#include "tv/av1_enc.h"
#include "tv/av1_itx.h"
#include "tv/av1_txfm.h"

namespace tv {
namespace gpu {
namespace {

using namespace tv::av1;

__constant__ int32_t c_dct16[256];
__constant__ int32_t c_dct8[64];
__constant__ int32_t c_adst8[64];

constexpr int R = kMeRange;
constexpr int kWinP = 60;              // window pitch (bytes, multiple of 4)
constexpr int kWinN = 16 + 2 * R + 9;  // 57 rows: [-R-4, R+20] around the block
constexpr int kWinOff = R + 4;         // block origin inside the window
// chroma window: block-relative x in [-12, 19] (integer MV part [-9, 8] + 8-tap reach)
constexpr int kCWin = 32, kCWinOff = 12;

__device__ __forceinline__ int rsr(long long v, int s) { return (int)((v + (1LL << (s - 1))) >> s); }
__device__ __forceinline__ int c16(int v) { return v < -32768 ? -32768 : (v > 32767 ? 32767 : v); }

// sum over a 16-lane row (every lane gets its row's sum)
__device__ __forceinline__ int row16_sum(int v) {
  v += dpp::mov<dpp::kQuadXor1>(v);
  v += dpp::mov<dpp::kQuadXor2>(v);
  v += dpp::mov<dpp::kRowHalfMirror>(v);
  v += dpp::mov<dpp::kRowMirror>(v);
  return v;
}
// sum over an 8-lane half row
__device__ __forceinline__ int row8_sum(int v) {
  v += dpp::mov<dpp::kQuadXor1>(v);
  v += dpp::mov<dpp::kQuadXor2>(v);
  v += dpp::mov<dpp::kRowHalfMirror>(v);
  return v;
}

// basis of 1-D type (0 DCT, 1 ADST) for N = 8 / 16
__device__ __forceinline__ const int32_t* basis(int lg, int type) {
  return lg == 4 ? c_dct16 : (type ? c_adst8 : c_dct8);
}

// One N x N 2-D transform on the calling wave (LDS in -> LDS out), the stages of
// txfm2d_ref: forward tmp = Bc X (round f1), C = tmp Br^T (round f2); inverse
// g = X Br (round i1), out = Bc^T g (round i2); int16 clamps after each stage.
template <int LG>
__device__ void wave_txfm(const int16_t* in, int16_t* tmp, int16_t* out, int tcol, int trow, bool inverse);

// 16x16 on the matrix cores: each stage is one exact 16x16x16 tile (mfma_exact.h, four
// v_mfma_f32_16x16x16f16 per stage), same integers as the VALU form below.
template <>
__device__ void wave_txfm<4>(const int16_t* in, int16_t* tmp, int16_t* out, int tcol, int trow, bool inverse) {
  const int lane = threadIdx.x & 63, row0 = (lane >> 4) * 4, col = lane & 15;
  const int32_t* Bc = basis(4, tcol);
  const int32_t* Br = basis(4, trow);
  constexpr int f1 = 12 + (4 - 1) / 2 - 2, f2 = 12 + 4 / 2 - 1, i1 = 13 + 4 / 2, i2 = 14 + (4 - 1) / 2;
  long long o[4];
  if (!inverse) exact_tile([&](int r, int k) { return (int)Bc[r * 16 + k]; }, [&](int k, int c) { return (int)in[k * 16 + c]; }, 0, 0, 16, o);
  else exact_tile([&](int r, int k) { return (int)in[r * 16 + k]; }, [&](int k, int c) { return (int)Br[k * 16 + c]; }, 0, 0, 16, o);
#pragma unroll
  for (int r = 0; r < 4; ++r) tmp[(row0 + r) * 16 + col] = (int16_t)c16(rsr(o[r], inverse ? i1 : f1));
  __syncthreads();
  if (!inverse) exact_tile([&](int r, int k) { return (int)tmp[r * 16 + k]; }, [&](int k, int c) { return (int)Br[c * 16 + k]; }, 0, 0, 16, o);
  else exact_tile([&](int r, int k) { return (int)Bc[k * 16 + r]; }, [&](int k, int c) { return (int)tmp[k * 16 + c]; }, 0, 0, 16, o);
#pragma unroll
  for (int r = 0; r < 4; ++r) out[(row0 + r) * 16 + col] = (int16_t)c16(rsr(o[r], inverse ? i2 : f2));
  __syncthreads();
}

// 8x8 (chroma): one lane per output, VALU
template <int LG>
__device__ void wave_txfm(const int16_t* in, int16_t* tmp, int16_t* out, int tcol, int trow, bool inverse) {
  constexpr int N = 1 << LG;
  const int lane = threadIdx.x & 63;
  const int32_t* Bc = basis(LG, tcol);
  const int32_t* Br = basis(LG, trow);
  const int f1 = 12 + (LG - 1) / 2 - 2, f2 = 12 + LG / 2 - 1, i1 = 13 + LG / 2, i2 = 14 + (LG - 1) / 2;
  for (int idx = lane; idx < N * N; idx += 64) {
    const int r = idx >> LG, c = idx & (N - 1);
    long long s = 0;
#pragma unroll
    for (int k = 0; k < N; ++k)
      s += inverse ? (long long)in[r * N + k] * Br[k * N + c] : (long long)Bc[r * N + k] * in[k * N + c];
    tmp[idx] = (int16_t)c16(rsr(s, inverse ? i1 : f1));
  }
  __syncthreads();
  for (int idx = lane; idx < N * N; idx += 64) {
    const int r = idx >> LG, c = idx & (N - 1);
    long long s = 0;
#pragma unroll
    for (int k = 0; k < N; ++k)
      s += inverse ? (long long)Bc[k * N + r] * tmp[k * N + c] : (long long)tmp[r * N + k] * Br[c * N + k];
    out[idx] = (int16_t)c16(rsr(s, inverse ? i2 : f2));
  }
  __syncthreads();
}

// Residual coding of one TB held in LDS: res (int16, src - pred) -> levels (global),
// reconstruction added onto pred (int, LDS) -> returns 1 if any level is nonzero.
// Scratch a/b: LDS int16 [N*N] each; ti: LDS int32 [N*N].  Forward: the basis-matrix
// transform (MFMA for 16x16); inverse: the specification's 2-D process (tv/av1_itx.h), one
// lane per row, then one lane per column.  Force-inlined: called, its LDS pointers were flat
// (generic) accesses.
template <int LG>
__device__ __forceinline__ int code_tb(int16_t* res, int16_t* a, int16_t* b, int32_t* ti, int tcol, int trow, int qidx, int rnd,
                       int16_t* __restrict__ lev_out) {
  constexpr int N = 1 << LG;
  const int lane = threadIdx.x & 63;
  wave_txfm<LG>(res, a, b, tcol, trow, false);  // coefficients in b
  const int qd = dc_q(qidx), qa = ac_q(qidx);
  int nz = 0;
  for (int i = lane; i < N * N; i += 64) {
    const int l = quant(b[i], i ? qa : qd, rnd);
    lev_out[i] = (int16_t)l;
    a[i] = (int16_t)dequant(l, i ? qa : qd);
    nz |= l != 0;
  }
  const bool any = __any(nz);
  __syncthreads();
  if (any) {
    if (lane < N) {
      int32_t in[N];
#pragma unroll
      for (int j = 0; j < N; ++j) in[j] = a[lane * N + j];
      inv_row<LG>(in, trow, ti + lane * N);
    }
    __syncthreads();
    if (lane < N) {
      int32_t t[N];
#pragma unroll
      for (int i = 0; i < N; ++i) t[i] = ti[i * N + lane];
      inv_col<LG>(t, tcol);
#pragma unroll
      for (int i = 0; i < N; ++i) res[i * N + lane] = (int16_t)t[i];
    }
    __syncthreads();
  } else {
    for (int i = lane; i < N * N; i += 64) res[i] = 0;
    __syncthreads();
  }
  return any ? 1 : 0;
}

struct Planes3 {
  const uint8_t *y, *u, *v;
};
struct Planes3W {
  uint8_t *y, *u, *v;
};

// ================================================================= inter ================
// STAGE 0: the motion search only (mvout = the block's MV).  STAGE 1: prediction at mvin
// (the refined field) + residual coding + reconstruction (mvout = mvin).
// WPE: minimum waves per SIMD for the register allocation (stage 0: 6 -> <= 80 VGPRs, no
// scratch, against the compiler's 84 / 5 waves; stage 1 is LDS-limited, left alone)
template <int STAGE, int WPE>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(WPE))) k_av1e_inter(Planes3 src, Planes3 ref, Planes3W rec, uint32_t* __restrict__ mode,
                                                   const uint32_t* __restrict__ mvin, uint32_t* __restrict__ mvout,
                                                   int16_t* __restrict__ ly, int16_t* __restrict__ lu,
                                                   int16_t* __restrict__ lv, int W, int H, const int* __restrict__ qarr,
                                                   const unsigned long long* __restrict__ satd_acc) {
  __shared__ __attribute__((aligned(16))) uint8_t win[kWinN * kWinP + 8];
  __shared__ __attribute__((aligned(16))) uint8_t sblk[256];
  __shared__ __attribute__((aligned(16))) uint8_t cwin[2][kCWin * kCWin];
  __shared__ int16_t hpl[3][25][16];  // horizontally filtered planes of a sub-pel step
  __shared__ int cost[9];
  int lastk = 1;
  __shared__ int16_t res[256], ta[256], tb[256];
  __shared__ int32_t ti[256];
  __shared__ int predc[256];
  int blk, b;
  xcd_ctb(blk, b);
  const int lane = threadIdx.x, qidx = qarr[b];
  const int bw = W >> 4, bx = blk % bw, by = blk / bw, x0 = bx * 16, y0 = by * 16;
  const long ysz = (long)W * H, csz = ysz >> 2;
  const uint8_t* S = src.y + b * ysz;
  const uint8_t* Rf = ref.y + b * ysz;
  const int lam = lambda16(qidx);
  // stage the clamped reference windows (luma 57 x 57, chroma 32 x 32 per plane) and the
  // source block; windows fully inside the frame take dword loads (their origins are
  // 4-byte aligned: x0 - 20 and cx0 - 12 with x0 % 16 == 0, cx0 % 8 == 0)
  const int wx0 = x0 - kWinOff, wy0 = y0 - kWinOff;
  if (STAGE == 1) {
    // the recon reads only the 23 x 23 reference samples of its MV's 8-tap footprint: stage
    // just those (clamped) into their window positions
    const uint32_t m = mvin[(long)b * (bw * (H >> 4)) + blk];
    const int ix = mv_int(mv_col(m), false) - 3, iy = mv_int(mv_row(m), false) - 3;
    for (int i = lane; i < 23 * 23; i += 64) {
      const int wy = i / 23, wx = i - wy * 23;
      const int yy = clip3(0, H - 1, y0 + iy + wy), xx = clip3(0, W - 1, x0 + ix + wx);
      win[(kWinOff + iy + wy) * kWinP + kWinOff + ix + wx] = Rf[(long)yy * W + xx];
    }
  } else if (wx0 >= 0 && wy0 >= 0 && wx0 + kWinP <= W && wy0 + kWinN <= H) {
    for (int i = lane; i < kWinN * (kWinP / 4); i += 64) {
      const int wy = i / (kWinP / 4), wq = i - wy * (kWinP / 4);
      reinterpret_cast<uint32_t*>(win + wy * kWinP)[wq] =
          *reinterpret_cast<const uint32_t*>(Rf + (long)(wy0 + wy) * W + wx0 + 4 * wq);
    }
  } else {
    for (int i = lane; i < kWinN * kWinN; i += 64) {
      const int wy = i / kWinN, wx = i - wy * kWinN;
      const int yy = clip3(0, H - 1, wy0 + wy), xx = clip3(0, W - 1, wx0 + wx);
      win[wy * kWinP + wx] = Rf[(long)yy * W + xx];
    }
  }
  if (STAGE == 1) {
    const int Wc = W >> 1, Hc = H >> 1, cwx = bx * 8 - kCWinOff, cwy = by * 8 - kCWinOff;
    const bool in = cwx >= 0 && cwy >= 0 && cwx + kCWin <= Wc && cwy + kCWin <= Hc;
    for (int pl = 0; pl < 2; ++pl) {
      const uint8_t* Rc = (pl ? ref.v : ref.u) + b * csz;
      if (in) {
        for (int i = lane; i < kCWin * (kCWin / 4); i += 64) {
          const int wy = i / (kCWin / 4), wq = i - wy * (kCWin / 4);
          reinterpret_cast<uint32_t*>(cwin[pl] + wy * kCWin)[wq] =
              *reinterpret_cast<const uint32_t*>(Rc + (long)(cwy + wy) * Wc + cwx + 4 * wq);
        }
      } else {
        for (int i = lane; i < kCWin * kCWin; i += 64) {
          const int wy = i / kCWin, wx = i - wy * kCWin;
          cwin[pl][i] = Rc[(long)clip3(0, Hc - 1, cwy + wy) * Wc + clip3(0, Wc - 1, cwx + wx)];
        }
      }
    }
  }
  for (int i = lane; i < 256; i += 64) sblk[i] = S[(long)(y0 + (i >> 4)) * W + x0 + (i & 15)];
  __syncthreads();
  const int nb = bw * (H >> 4);
  const long bo = (long)b * nb + blk;
  auto wget = [&](int x, int y) -> int {  // window sample at block-relative (x, y)
    return win[(kWinOff + y) * kWinP + kWinOff + x];
  };
  int mr = 0, mc = 0, yb = 0;
  if (STAGE == 1) {
    // the refined MV: its horizontal plane (column offset 0) for the luma prediction below
    mr = mv_row(mvin[bo]);
    mc = mv_col(mvin[bo]);
    yb = (mr >> 3) - 3;
    const int ix = mv_int(mc, false), fx = mv_frac(mc, false);
    for (int idx = lane; idx < 23 * 16; idx += 64) {
      const int yy = idx >> 4, x = idx & 15;
      int sum = 0;
#pragma unroll
      for (int t = 0; t < 8; ++t) sum += subpel_tap(fx, t) * wget(x + ix + t - 3, yb + yy);
      hpl[1][yy][x] = (int16_t)((sum + (1 << (kInterRound0 - 1))) >> kInterRound0);
    }
    lastk = 1;
    __syncthreads();
  } else {
  // ---- full-pel search: packed SAD, first minimum of (cost, index)
  uint32_t sv[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) sv[i] = reinterpret_cast<const uint32_t*>(sblk)[i];
  // packed SAD of rows [i0, i0 + n) at full-pel offset (dx, dy)
  auto sad_rows = [&](int dx, int dy, int i0, int n) -> unsigned {
    unsigned sad = 0;
    const int ox = kWinOff + dx, sh = ox & 3;
    for (int i = i0; i < i0 + n; ++i) {
      const uint32_t* row = reinterpret_cast<const uint32_t*>(win + (kWinOff + dy + i) * kWinP + (ox & ~3));
      const uint32_t* sr = reinterpret_cast<const uint32_t*>(sblk) + i * 4;
      const uint32_t w0 = row[0], w1 = row[1], w2 = row[2], w3 = row[3], w4 = row[4];
      sad = __builtin_amdgcn_sad_u8(sr[0], __builtin_amdgcn_alignbyte(w1, w0, sh), sad);
      sad = __builtin_amdgcn_sad_u8(sr[1], __builtin_amdgcn_alignbyte(w2, w1, sh), sad);
      sad = __builtin_amdgcn_sad_u8(sr[2], __builtin_amdgcn_alignbyte(w3, w2, sh), sad);
      sad = __builtin_amdgcn_sad_u8(sr[3], __builtin_amdgcn_alignbyte(w4, w3, sh), sad);
    }
    return sad;
  };
  unsigned best = 0xFFFFFFFFu;
  for (int k = lane; k < kMeGrid * kMeGrid; k += 64) {  // 2-pel grid, one candidate per lane
    const int dx = me_cand_dx(k), dy = me_cand_dy(k);
    unsigned sad = 0;
    const int ox = kWinOff + dx, sh = ox & 3;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t* row = reinterpret_cast<const uint32_t*>(win + (kWinOff + dy + i) * kWinP + (ox & ~3));
      const uint32_t w0 = row[0], w1 = row[1], w2 = row[2], w3 = row[3], w4 = row[4];
      sad = __builtin_amdgcn_sad_u8(sv[i * 4 + 0], __builtin_amdgcn_alignbyte(w1, w0, sh), sad);
      sad = __builtin_amdgcn_sad_u8(sv[i * 4 + 1], __builtin_amdgcn_alignbyte(w2, w1, sh), sad);
      sad = __builtin_amdgcn_sad_u8(sv[i * 4 + 2], __builtin_amdgcn_alignbyte(w3, w2, sh), sad);
      sad = __builtin_amdgcn_sad_u8(sv[i * 4 + 3], __builtin_amdgcn_alignbyte(w4, w3, sh), sad);
    }
    const unsigned c = sad + ((lam * (mv_comp_bits(dy * 8) + mv_comp_bits(dx * 8))) >> 4);
    const unsigned key = (c << 12) | (unsigned)k;
    best = key < best ? key : best;
  }
  best = wave_min_u32(best);
  const int bk = best & 4095;
  int gx = me_cand_dx(bk), gy = me_cand_dy(bk);
  {  // full-pel neighbours of the best grid point: 8 candidates x 8 lanes (2 rows each)
    const int ci = lane >> 3, r2 = (lane & 7) * 2;
    const int dx = gx + me_ring_dx(ci), dy = gy + me_ring_dy(ci);
    const bool ok = dx >= -kMeRange && dx <= kMeRange && dy >= -kMeRange && dy <= kMeRange;
    const int part = ok ? (int)sad_rows(dx, dy, r2, 2) : 0;
    const int sad = row8_sum(part);
    if ((lane & 7) == 0) cost[ci] = ok ? sad + ((lam * (mv_comp_bits(dy * 8) + mv_comp_bits(dx * 8))) >> 4) : -1;
    __syncthreads();
    int bc = (int)(best >> 12), bi = -1;
    for (int k = 0; k < 8; ++k)
      if (cost[k] >= 0 && cost[k] < bc) bc = cost[k], bi = k;
    if (bi >= 0) gx += me_ring_dx(bi), gy += me_ring_dy(bi);
    __syncthreads();
  }
  mr = gy * 8, mc = gx * 8;
  // ---- sub-pel refinement: center + 8 ring candidates at step 4 (half) then 2 (quarter)
  // Separable and shared: per step, the three horizontally filtered planes (column offsets
  // -step, 0, +step) are computed once into LDS (int16, Round0), then each of the 9
  // candidates only runs the vertical 8-tap pass (the same integers as inter_pred_px).
  const int grp = lane >> 4, b4 = lane & 15, px = (b4 & 3) * 4, py = (b4 >> 2) * 4;
  for (int step = 4; step >= 2; step >>= 1) {
    yb = ((mr - step) >> 3) - 3;
    const int nrows = ((mr + step) >> 3) + 19 - yb + 1;  // <= 25
    for (int idx = lane; idx < 3 * nrows * 16; idx += 64) {
      const int k = idx / (nrows * 16), rem = idx - k * nrows * 16, yy = rem >> 4, x = rem & 15;
      const int c = mc + (k - 1) * step, ix = mv_int(c, false), fx = mv_frac(c, false);
      int sum = 0;
#pragma unroll
      for (int t = 0; t < 8; ++t) sum += subpel_tap(fx, t) * wget(x + ix + t - 3, yb + yy);
      hpl[k][yy][x] = (int16_t)((sum + (1 << (kInterRound0 - 1))) >> kInterRound0);
    }
    __syncthreads();
    for (int pass = 0; pass < 3; ++pass) {
      const int ci = pass * 4 + grp;  // 0 = center, 1..8 = ring
      int dr = 0, dc = 0;
      if (ci >= 1 && ci <= 8) {
        dr = me_ring_dy(ci - 1) * step;
        dc = me_ring_dx(ci - 1) * step;
      }
      const int r = mr + dr, c = mc + dc, k = dc / step + 1;
      const int iy = mv_int(r, false), fy = mv_frac(r, false), r0 = py + iy - 3 - yb;
      int d[16];
      int col[11][4];
#pragma unroll
      for (int rr = 0; rr < 11; ++rr)
#pragma unroll
        for (int j = 0; j < 4; ++j) col[rr][j] = hpl[k][r0 + rr][px + j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          int sum = 0;
#pragma unroll
          for (int t = 0; t < 8; ++t) sum += subpel_tap(fy, t) * col[i + t][j];
          const int p = clip_pixel((sum + (1 << (kInterRound1 - 1))) >> kInterRound1);
          d[i * 4 + j] = (int)sblk[(py + i) * 16 + px + j] - p;
        }
      const int sat = row16_sum(satd4(d));
      if (b4 == 0 && ci <= 8) cost[ci] = sat + ((lam * (mv_comp_bits(r) + mv_comp_bits(c))) >> 4);
    }
    __syncthreads();
    int bc = cost[0], bi = 0;
    for (int k = 1; k <= 8; ++k)
      if (cost[k] < bc) bc = cost[k], bi = k;
    if (bi) {
      mr += me_ring_dy(bi - 1) * step;
      mc += me_ring_dx(bi - 1) * step;
      lastk = me_ring_dx(bi - 1) + 1;
    } else {
      lastk = 1;
    }
    __syncthreads();
  }
  if (lane == 0) mvout[bo] = pack_mv(mr, mc);
  return;
  }  // STAGE 0
  // ---- luma prediction + residual: vertical pass of the chosen candidate over the
  // horizontal plane
  {
    const int iy = mv_int(mr, false), fy = mv_frac(mr, false);
    for (int i = lane; i < 256; i += 64) {
      const int yy = i >> 4, xx = i & 15, r0 = yy + iy - 3 - yb;
      int sum = 0;
#pragma unroll
      for (int t = 0; t < 8; ++t) sum += subpel_tap(fy, t) * hpl[lastk][r0 + t][xx];
      const int p = clip_pixel((sum + (1 << (kInterRound1 - 1))) >> kInterRound1);
      predc[i] = p;
      res[i] = (int16_t)((int)sblk[i] - p);
    }
  }
  __syncthreads();
  const int rnd = inter_rounding((long long)satd_acc[b], W, H);
  int nz = code_tb<4>(res, ta, tb, ti, 0, 0, qidx, rnd, ly + bo * 256);
  for (int i = lane; i < 256; i += 64)
    rec.y[b * ysz + (long)(y0 + (i >> 4)) * W + x0 + (i & 15)] = (uint8_t)clip_pixel(predc[i] + res[i]);
  __syncthreads();
  // ---- chroma (8x8 per plane) from the staged chroma windows
  const int Wc = W >> 1, cx0 = bx * 8, cy0 = by * 8;
  const int ix = mv_int(mc, true), iy = mv_int(mr, true), fx = mv_frac(mc, true), fy = mv_frac(mr, true);
  for (int pl = 1; pl <= 2; ++pl) {
    const uint8_t* Sc = (pl == 1 ? src.u : src.v) + b * csz;
    const uint8_t* cw = cwin[pl - 1];
    auto cget = [&](int x, int y) -> int { return cw[(kCWinOff + y) * kCWin + kCWinOff + x]; };
    {
      const int yy = lane >> 3, xx = lane & 7;
      const int p = inter_pred_px(cget, xx + ix, yy + iy, fx, fy);
      predc[lane] = p;
      res[lane] = (int16_t)((int)Sc[(long)(cy0 + yy) * Wc + cx0 + xx] - p);
    }
    __syncthreads();
    int16_t* lo = (pl == 1 ? lu : lv) + bo * 64;
    if (code_tb<3>(res, ta, tb, ti, 0, 0, qidx, rnd, lo)) nz |= 1 << pl;
    uint8_t* Rw = (pl == 1 ? rec.u : rec.v) + b * csz;
    Rw[(long)(cy0 + (lane >> 3)) * Wc + cx0 + (lane & 7)] = (uint8_t)clip_pixel(predc[lane] + res[lane]);
    __syncthreads();
  }
  if (lane == 0) {
    mode[bo] = pack_mode(1, 0, 0, nz == 0, nz);
    mvout[bo] = pack_mv(mr, mc);
  }
}

// MV unification (tv/av1_enc.h quad_unify / sb_unify): one 256-thread workgroup per 64x64
// superblock.  The superblock's reference window (104 x 104, clamped) and source are staged
// in LDS; (block, candidate MV) pairs are scored 16 per pass, 16 lanes per pair (one 4x4
// SATD each).  The quads of the superblock first, then the superblock itself; only the
// superblock's own 16 MV words are read and written.
constexpr int kSbWin = 104, kSbWinOff = 20;

// Stage a superblock's clamped reference window and its source (zero outside the frame).
__device__ void stage_sb(const uint8_t* S, const uint8_t* Rf, int W, int H, int X0, int Y0, uint8_t* win, uint8_t* sb) {
  const int t = threadIdx.x;
  for (int i = t; i < kSbWin * kSbWin; i += 256) {
    const int wy = i / kSbWin, wx = i - wy * kSbWin;
    win[i] = Rf[(long)clip3(0, H - 1, Y0 - kSbWinOff + wy) * W + clip3(0, W - 1, X0 - kSbWinOff + wx)];
  }
  for (int i = t; i < 64 * 64; i += 256) {
    const int yy = Y0 + (i >> 6), xx = X0 + (i & 63);
    sb[i] = (yy < H && xx < W) ? S[(long)yy * W + xx] : 0;
  }
}

// Luma SATD of superblock-local block k (4 x 4 raster of 16x16) at MV m, from the staged
// window / source: the calling lane's 4x4 (b4 = lane & 15) predicted with the 8-tap
// separable filter of inter_pred_px, summed over its 16-lane row.
__device__ __forceinline__ int sb_pair_satd(const uint8_t* win, const uint8_t* sb, int k, uint32_t m, int b4) {
  const int px = (b4 & 3) * 4, py = (b4 >> 2) * 4;
  const int ox = (k & 3) * 16 + px, oy = (k >> 2) * 16 + py;
  const int r = mv_row(m), c = mv_col(m);
  const int ix = mv_int(c, false), iy = mv_int(r, false), fx = mv_frac(c, false), fy = mv_frac(r, false);
  auto wget = [&](int x, int y) -> int { return win[(kSbWinOff + y) * kSbWin + kSbWinOff + x]; };
  int d[16];
  if (!fx && !fy) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) d[i * 4 + j] = (int)sb[(oy + i) * 64 + ox + j] - wget(ox + j + ix, oy + i + iy);
  } else {
    int col[11][4];
#pragma unroll
    for (int rr = 0; rr < 11; ++rr)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        int sum = 0;
#pragma unroll
        for (int tp = 0; tp < 8; ++tp) sum += subpel_tap(fx, tp) * wget(ox + j + ix + tp - 3, oy + rr + iy - 3);
        col[rr][j] = (sum + (1 << (kInterRound0 - 1))) >> kInterRound0;
      }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        int sum = 0;
#pragma unroll
        for (int tp = 0; tp < 8; ++tp) sum += subpel_tap(fy, tp) * col[i + tp][j];
        d[i * 4 + j] = (int)sb[(oy + i) * 64 + ox + j] - clip_pixel((sum + (1 << (kInterRound1 - 1))) >> kInterRound1);
      }
  }
  return row16_sum(satd4(d));
}

// One Jacobi round of the motion-field refinement (tv/av1_enc.h mv_refine_cands), one
// 256-thread workgroup per superblock: each of its 16x16 blocks re-chooses among its
// neighbours' current MVs (read from `cur`, across superblock edges too) by luma SATD
// (first minimum, own MV first) and writes `nxt`.  (block, candidate) pairs 16 per pass
// on the staged superblock window.
// Memo: each round records, per block, the (MV, SATD) pairs it scored ([B][nb] records of
// kMvRefineMaxCand + a count); the next round takes the SATD of a candidate it already scored
// from there (its own MV always, most neighbours' MVs too) instead of recomputing it.
struct MvMemo {
  uint32_t* mv;   // [B][nb][kMvRefineMaxCand]
  int* sat;       // [B][nb][kMvRefineMaxCand]
  uint8_t* n;     // [B][nb]
};
__global__ void __launch_bounds__(256) k_av1e_mv_refine(const uint8_t* __restrict__ srcy, const uint8_t* __restrict__ refy,
                                                        const uint32_t* __restrict__ cur, uint32_t* __restrict__ nxt,
                                                        int W, int H, MvMemo prev, MvMemo next, int use_prev) {
  __shared__ __attribute__((aligned(16))) uint8_t win[kSbWin * kSbWin];
  __shared__ __attribute__((aligned(16))) uint8_t sb[64 * 64];
  __shared__ uint32_t cand[16][kMvRefineMaxCand];
  __shared__ int ncand[16];
  __shared__ int sat[16][kMvRefineMaxCand];
  __shared__ int pk[16 * kMvRefineMaxCand];  // pair -> (block << 8) | candidate
  __shared__ int npairs;
  const int sbi = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  const int bw = W >> 4, bh = H >> 4, sbw = (W + 63) >> 6, sx = sbi % sbw, sy = sbi / sbw;
  const long ysz = (long)W * H, nb = (long)bw * bh;
  const uint32_t* C = cur + b * nb;
  // round 0 (nothing memoised) stages up front, its loads overlapping the candidate lists;
  // later rounds stage only superblocks with a pair left to score (below)
  if (!use_prev) stage_sb(srcy + b * ysz, refy + b * ysz, W, H, sx * 64, sy * 64, win, sb);
  constexpr int kM = kMvRefineMaxCand;
  __shared__ uint32_t pmv[16][kM];
  __shared__ int psat[16][kM], pn[16];
  // lanes (k, j) = (t / kM, t % kM) of the first 16 * kM: block k's record j of the previous round
  const int mk = t / kM, mj = t - mk * kM;
  const int mbx = sx * 4 + (mk & 3), mby = sy * 4 + (mk >> 2);
  const bool mlane = t < 16 * kM && mbx < bw && mby < bh;
  const long mr = b * nb + (long)mby * bw + mbx;
  if (t < 16) {
    const int bx = sx * 4 + (t & 3), by = sy * 4 + (t >> 2);
    const bool in = bx < bw && by < bh;
    ncand[t] = in ? mv_refine_cands(C, bw, bh, bx, by, cand[t]) : 0;
    pn[t] = (in && use_prev) ? prev.n[b * nb + (long)by * bw + bx] : 0;
  }
  if (mlane && use_prev) {
    pmv[mk][mj] = prev.mv[mr * kM + mj];
    psat[mk][mj] = prev.sat[mr * kM + mj];
  }
  __syncthreads();
  if (mlane && mj < ncand[mk]) {  // memo lookup of pair (mk, mj)
    int v = -1;
    for (int j = 0; j < pn[mk]; ++j)
      if (pmv[mk][j] == cand[mk][mj]) v = psat[mk][j];
    sat[mk][mj] = v;
  }
  __syncthreads();
  if (t == 0) {
    int n = 0;
    for (int k = 0; k < 16; ++k)
      for (int c = 0; c < ncand[k]; ++c)
        if (sat[k][c] < 0) pk[n++] = (k << 8) | c;
    npairs = n;
  }
  __syncthreads();
  const int grp = t >> 4, b4 = t & 15, n = npairs;
  if (n && use_prev) {  // a converged superblock (every candidate memoised) skips the staging
    stage_sb(srcy + b * ysz, refy + b * ysz, W, H, sx * 64, sy * 64, win, sb);
    __syncthreads();
  }
  for (int p0 = 0; p0 < n; p0 += 16) {
    const int p = p0 + grp;
    if (p < n) {  // uniform over each 16-lane row (the row16_sum DPP stays inside it)
      const int k = pk[p] >> 8, c = pk[p] & 255;
      const int v = sb_pair_satd(win, sb, k, cand[k][c], b4);
      if (b4 == 0) sat[k][c] = v;
    }
  }
  __syncthreads();
  if (t < 16 && ncand[t]) {
    int bc = sat[t][0], bi = 0;
    for (int c = 1; c < ncand[t]; ++c)
      if (sat[t][c] < bc) bc = sat[t][c], bi = c;
    const int bx = sx * 4 + (t & 3), by = sy * 4 + (t >> 2);
    const long r = b * nb + (long)by * bw + bx;
    nxt[r] = cand[t][bi];
    if (next.n) next.n[r] = (uint8_t)ncand[t];
  }
  if (next.n && mlane && mj < ncand[mk]) {
    next.mv[mr * kM + mj] = cand[mk][mj];
    next.sat[mr * kM + mj] = sat[mk][mj];
  }
}

__global__ void __launch_bounds__(256) k_av1e_mv_unify(const uint8_t* __restrict__ srcy, const uint8_t* __restrict__ refy,
                                                       uint32_t* __restrict__ mv, int W, int H, const int* __restrict__ qarr,
                                                       unsigned long long* __restrict__ satd_acc) {
  __shared__ __attribute__((aligned(16))) uint8_t win[kSbWin * kSbWin];
  __shared__ __attribute__((aligned(16))) uint8_t sb[64 * 64];
  __shared__ uint32_t mvl[16];
  __shared__ int sat[80];
  const int sbi = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  const int bw = W >> 4, bh = H >> 4, sbw = (W + 63) >> 6, sx = sbi % sbw, sy = sbi / sbw;
  const int X0 = sx * 64, Y0 = sy * 64;
  const long ysz = (long)W * H, nb = (long)bw * bh;
  const uint8_t* S = srcy + b * ysz;
  const uint8_t* Rf = refy + b * ysz;
  uint32_t* M = mv + b * nb;
  const int lam = lambda16(qarr[b]);
  stage_sb(S, Rf, W, H, X0, Y0, win, sb);
  if (t < 16) {
    const int bx = sx * 4 + (t & 3), by = sy * 4 + (t >> 2);
    mvl[t] = (bx < bw && by < bh) ? M[by * bw + bx] : 0u;
  }
  __syncthreads();
  const int grp = t >> 4, b4 = t & 15;
  auto pair_satd = [&](int k, uint32_t m) -> int { return sb_pair_satd(win, sb, k, m, b4); };
  // ---- quads: pair p = q * 16 + k * 4 + c (block k of quad q at member c's MV)
  auto quad_ok = [&](int q) {
    const int qx = sx * 2 + (q & 1), qy = sy * 2 + (q >> 1);
    return 2 * qx + 1 < bw && 2 * qy + 1 < bh;
  };
  auto qblk = [&](int q, int k) { return ((q >> 1) * 2 + (k >> 1)) * 4 + (q & 1) * 2 + (k & 1); };
  for (int p0 = 0; p0 < 64; p0 += 16) {
    const int p = p0 + grp, q = p >> 4, k = (p >> 2) & 3, c = p & 3;
    int v = 0;
    if (quad_ok(q)) v = pair_satd(qblk(q, k), mvl[qblk(q, c)]);
    if (b4 == 0) sat[p] = v;  // (80-entry scratch: quads use 64)
  }
  __syncthreads();
  if (t < 4 && quad_ok(t)) {
    int q4[4][4];
    for (int k = 0; k < 4; ++k)
      for (int c = 0; c < 4; ++c) q4[k][c] = sat[t * 16 + k * 4 + c];
    const int c = quad_unify(q4, lam);
    if (c >= 0) {
      const uint32_t m = mvl[qblk(t, c)];
      for (int k = 0; k < 4; ++k) mvl[qblk(t, k)] = m;  // each thread writes its own quad
    }
  }
  __syncthreads();
  // ---- the superblock: pair p < 16: block p at its MV; p >= 16: block (p-16)>>2 at quad (p-16)&3's
  if (sx * 4 + 3 < bw && sy * 4 + 3 < bh) {
    for (int p0 = 0; p0 < 80; p0 += 16) {
      const int p = p0 + grp;
      const uint32_t m = p < 16 ? mvl[p] : mvl[qblk((p - 16) & 3, 0)];
      const int v = pair_satd(p < 16 ? p : (p - 16) >> 2, m);
      if (b4 == 0) sat[p] = v;
    }
    __syncthreads();
    if (t == 0) {
      int own = 0, tot[4] = {0, 0, 0, 0};
      for (int k = 0; k < 16; ++k) {
        own += sat[k];
        for (int c = 0; c < 4; ++c) tot[c] += sat[16 + k * 4 + c];
      }
      const int c = sb_unify(own, tot, lam);
      if (c >= 0) {
        const uint32_t m = mvl[qblk(c, 0)];
        for (int k = 0; k < 16; ++k) mvl[k] = m;
      }
    }
    __syncthreads();
  }
  if (t < 16) {
    const int bx = sx * 4 + (t & 3), by = sy * 4 + (t >> 2);
    if (bx < bw && by < bh) M[by * bw + bx] = mvl[t];
  }
  // the frame's luma SATD at the final MVs (tv/av1_enc.h inter_rounding): this superblock's
  // blocks, one pass of 16 pairs, summed into the segment's accumulator
  {
    const int bx = sx * 4 + (grp & 3), by = sy * 4 + (grp >> 2);
    const bool in = bx < bw && by < bh;
    const int v = in ? pair_satd(grp, mvl[grp]) : 0;
    __shared__ int part[16];
    if (b4 == 0) part[grp] = v;
    __syncthreads();
    if (t == 0) {
      long long sum = 0;
      for (int k = 0; k < 16; ++k) sum += part[k];
      atomicAdd(satd_acc + b, (unsigned long long)sum);
    }
  }
}

// ================================================================= intra ================
struct EdgeLds {
  IntraEdge e;
  int dc;
};

// edges of an N x N block of plane P (pitch w) at (x, y) into LDS (lanes 0..2N)
__device__ void load_edges(const uint8_t* P, int w, int x, int y, int N, EdgeLds& E) {
  const int lane = threadIdx.x & 63;
  auto get = [&](int xx, int yy) -> int { return P[(long)yy * w + xx]; };
  if (lane == 0) {
    E.e.have_a = y > 0;
    E.e.have_l = x > 0;
    if (E.e.have_a && E.e.have_l) E.e.tl = get(x - 1, y - 1);
    else if (E.e.have_a) E.e.tl = get(x, y - 1);
    else if (E.e.have_l) E.e.tl = get(x - 1, y);
    else E.e.tl = 128;
  }
  if (lane < N) {
    const int i = lane;
    int a, l;
    if (y > 0) a = get(x + i, y - 1);
    else if (x > 0) a = get(x - 1, y);
    else a = 127;
    if (x > 0) l = get(x - 1, y + i);
    else if (y > 0) l = get(x, y - 1);
    else l = 129;
    E.e.above[i] = a;
    E.e.left[i] = l;
  }
  __syncthreads();
  if (lane == 0) E.dc = intra_dc(E.e, N);
  __syncthreads();
}

__global__ void __launch_bounds__(64) k_av1e_intra(Planes3 src, Planes3W rec, uint32_t* __restrict__ mode,
                                                   uint32_t* __restrict__ mvout, int16_t* __restrict__ ly,
                                                   int16_t* __restrict__ lu, int16_t* __restrict__ lv, int W, int H,
                                                   const int* __restrict__ qarr, int diag, int bx_lo) {
  __shared__ EdgeLds E[2];
  __shared__ uint8_t sblk[256];
  __shared__ uint8_t sc[2][64];
  __shared__ int cost[16];
  __shared__ int16_t res[256], ta[256], tb[256];
  __shared__ int32_t ti[256];
  __shared__ int predc[256];
  const int lane = threadIdx.x, b = blockIdx.y, qidx = qarr[b];
  const int bw = W >> 4, bx = bx_lo + blockIdx.x, by = diag - bx, x0 = bx * 16, y0 = by * 16;
  const long ysz = (long)W * H, csz = ysz >> 2;
  const int lam = lambda16(qidx), Wc = W >> 1, cx0 = bx * 8, cy0 = by * 8;
  const uint8_t* S = src.y + b * ysz;
  uint8_t* RY = rec.y + b * ysz;
  for (int i = lane; i < 256; i += 64) sblk[i] = S[(long)(y0 + (i >> 4)) * W + x0 + (i & 15)];
  sc[0][lane] = (src.u + b * csz)[(long)(cy0 + (lane >> 3)) * Wc + cx0 + (lane & 7)];
  sc[1][lane] = (src.v + b * csz)[(long)(cy0 + (lane >> 3)) * Wc + cx0 + (lane & 7)];
  load_edges(RY, W, x0, y0, 16, E[0]);
  // ---- luma: kNumIntraCand candidates, 4 per pass (16 lanes = 16 4x4 SATDs each)
  const int grp = lane >> 4, b4 = lane & 15, px = (b4 & 3) * 4, py = (b4 >> 2) * 4;
  for (int pass = 0; pass < (kNumIntraCand + 3) / 4; ++pass) {
    const int ci = pass * 4 + grp;
    const int m = intra_cand(ci < kNumIntraCand ? ci : 0);
    int d[16];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        d[i * 4 + j] = (int)sblk[(py + i) * 16 + px + j] - intra_pred_px(m, E[0].e, 16, py + i, px + j, E[0].dc);
    const int sat = row16_sum(satd4(d));
    if (b4 == 0 && ci < kNumIntraCand) cost[ci] = sat + ((lam * intra_mode_bits16(m)) >> 8);
  }
  __syncthreads();
  int ym = intra_cand(0);
  {
    int bc = cost[0];
    for (int k = 1; k < kNumIntraCand; ++k)
      if (cost[k] < bc) bc = cost[k], ym = intra_cand(k);
  }
  __syncthreads();
  for (int i = lane; i < 256; i += 64) {
    const int p = intra_pred_px(ym, E[0].e, 16, i >> 4, i & 15, E[0].dc);
    predc[i] = p;
    res[i] = (int16_t)((int)sblk[i] - p);
  }
  __syncthreads();
  const int nb = bw * (H >> 4), blk = by * bw + bx;
  const long bo = (long)b * nb + blk;
  int nz = code_tb<4>(res, ta, tb, ti, 0, 0, qidx, kRndIntra, ly + bo * 256);
  for (int i = lane; i < 256; i += 64)
    RY[(long)(y0 + (i >> 4)) * W + x0 + (i & 15)] = (uint8_t)clip_pixel(predc[i] + res[i]);
  __syncthreads();
  // ---- chroma: kNumIntraCand candidates x 8 lanes (U: 4 blocks, V: 4 blocks), 8 per pass
  uint8_t* RU = rec.u + b * csz;
  uint8_t* RV = rec.v + b * csz;
  load_edges(RU, Wc, cx0, cy0, 8, E[0]);
  load_edges(RV, Wc, cx0, cy0, 8, E[1]);
  for (int pass = 0; pass < (kNumIntraCand + 7) / 8; ++pass) {
    const int ci = pass * 8 + (lane >> 3), q = lane & 7, pl = q >> 2, qb = q & 3, qx = (qb & 1) * 4, qy = (qb >> 1) * 4;
    const int m = intra_cand(ci < kNumIntraCand ? ci : 0);
    int d[16];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        d[i * 4 + j] = (int)sc[pl][(qy + i) * 8 + qx + j] - intra_pred_px(m, E[pl].e, 8, qy + i, qx + j, E[pl].dc);
    const int sat = row8_sum(satd4(d));
    if (q == 0 && ci < kNumIntraCand) cost[ci] = sat + ((lam * intra_mode_bits16(m)) >> 8);
  }
  __syncthreads();
  int uvm = intra_cand(0);
  {
    int bc = cost[0];
    for (int k = 1; k < kNumIntraCand; ++k)
      if (cost[k] < bc) bc = cost[k], uvm = intra_cand(k);
  }
  const int txt = uv_txtype(uvm);
  for (int pl = 0; pl < 2; ++pl) {
    __syncthreads();
    const int p = intra_pred_px(uvm, E[pl].e, 8, lane >> 3, lane & 7, E[pl].dc);
    predc[lane] = p;
    res[lane] = (int16_t)((int)sc[pl][lane] - p);
    __syncthreads();
    int16_t* lo = (pl == 0 ? lu : lv) + bo * 64;
    if (code_tb<3>(res, ta, tb, ti, txt & 1, (txt >> 1) & 1, qidx, kRndIntra, lo)) nz |= 2 << pl;
    uint8_t* Rw = pl == 0 ? RU : RV;
    Rw[(long)(cy0 + (lane >> 3)) * Wc + cx0 + (lane & 7)] = (uint8_t)clip_pixel(predc[lane] + res[lane]);
  }
  if (lane == 0) {
    mode[bo] = pack_mode(0, ym, uvm, nz == 0, nz);
    mvout[bo] = 0;
  }
}

// ================================================================= loop-filter info ======
__global__ void k_av1e_lfinfo(const uint32_t* __restrict__ mode, int W, int H, const int* __restrict__ lvl,
                              uint32_t* __restrict__ iy, uint32_t* __restrict__ iu, uint32_t* __restrict__ iv) {
  const int b = blockIdx.y, lv0 = lvl[4 * b], lv1 = lvl[4 * b + 1], lv2 = lvl[4 * b + 2], lv3 = lvl[4 * b + 3], w4 = W >> 2, h4 = H >> 2, bw = W >> 4, nb = bw * (H >> 4);
  const int u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= w4 * h4) return;
  const int x = u % w4, y = u / w4;
  const uint32_t m = mode[(long)b * nb + (y >> 2) * bw + (x >> 2)];
  const bool si = mode_skip(m) && mode_inter(m);
  const int bz = mode_bsz(m);
  iy[(long)b * w4 * h4 + u] = lf_word(false, lv0, lv1, si, bz);
  if (!(x & 1) && !(y & 1)) {
    const long cu = (long)b * (w4 / 2) * (h4 / 2) + (y >> 1) * (w4 / 2) + (x >> 1);
    iu[cu] = lf_word(true, lv2, lv2, si, bz);
    iv[cu] = lf_word(true, lv3, lv3, si, bz);
  }
}

// ================================================================= CDEF skip flags =======
// one thread per 8x8 luma block: flag the blocks of skip blocks in the direction array
// (kCdefSkipBlock: 7.15 cdef_block filters no 8x8 whose 4x4 units are all skip)
__global__ void k_av1e_cdef_skip(const uint32_t* __restrict__ mode, uint8_t* __restrict__ dir, int W, int H) {
  const int b = blockIdx.y, w8 = W >> 3, n8 = w8 * (H >> 3), bw = W >> 4, nb = bw * (H >> 4);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n8) return;
  const int y = i / w8, x = i - y * w8;
  if (mode_skip(mode[(long)b * nb + (y >> 1) * bw + (x >> 1)])) dir[(long)b * n8 + i] |= (uint8_t)kCdefSkipBlock;
}

// ================================================================= skip-block merging ===
// one thread per (superblock, segment): merge_sb (tv/av1_enc.h), same rule as the golden
__global__ void k_av1e_merge(uint32_t* __restrict__ mode, const uint32_t* __restrict__ mv, int W, int H, int B) {
  const int bw = W >> 4, bh = H >> 4, sbw = (W + 63) >> 6, sbh = (H + 63) >> 6, nsb = sbw * sbh;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nsb * B) return;
  const int b = i / nsb, s = i - b * nsb;
  merge_sb(mode + (long)b * bw * bh, mv + (long)b * bw * bh, bw, bh, s % sbw, s / sbw);
}

// ================================================================= CDEF preset choice ====
constexpr int kMaxFb = 4096;
// One workgroup per segment (a sequential greedy), so the 64 presets x nfb SSE sweeps are
// latency-bound: 16 waves (each a slice of the 64x64 blocks, lanes = presets) keep 4x more
// loads in flight than 4 did.  Column sums and the first-minimum pick are shared helpers.
constexpr int kCcT = 1024, kCcW = kCcT / 64;
__global__ void __launch_bounds__(kCcT) k_av1e_cdef_choose(const unsigned long long* __restrict__ sy,
                                                          const unsigned long long* __restrict__ su,
                                                          const unsigned long long* __restrict__ sv,
                                                          const uint32_t* __restrict__ mode, int W, int H,
                                                          uint8_t* __restrict__ tabs, int8_t* __restrict__ fbidx,
                                                          int8_t* __restrict__ py, int8_t* __restrict__ puv) {
  __shared__ unsigned long long best[kMaxFb];
  __shared__ uint8_t active[kMaxFb], asg[kMaxFb];
  __shared__ unsigned long long part[kCcW][64];
  __shared__ unsigned long long tot[64];
  __shared__ uint8_t ytab[8], uvtab[8];
  const int b = blockIdx.x, t = threadIdx.x;
  const int bw = W >> 4, bh = H >> 4, nb = bw * bh, sbw = (W + 63) >> 6, sbh = (H + 63) >> 6, nfb = sbw * sbh;
  const long so = (long)b * nfb * 64;
  for (int f = t; f < nfb; f += kCcT) {
    const int sx = f % sbw, sy0 = f / sbw;
    int act = 0;
    for (int yy = sy0 * 4; yy < min(bh, sy0 * 4 + 4); ++yy)
      for (int xx = sx * 4; xx < min(bw, sx * 4 + 4); ++xx) act |= !mode_skip(mode[(long)b * nb + yy * bw + xx]);
    active[f] = (uint8_t)act;
    best[f] = ~0ull;
  }
  __syncthreads();
  const int p = t & 63, pq = t >> 6;
  for (int k = 0; k < kMaxPresets; ++k) {
    unsigned long long acc = 0;
    for (int f = pq; f < nfb; f += kCcW)
      if (active[f]) {
        const unsigned long long v = sy[so + f * 64 + p];
        acc += v < best[f] ? v : best[f];
      }
    part[pq][p] = acc;
    __syncthreads();
    if (t < 64) {
      unsigned long long s = 0;
      for (int q = 0; q < kCcW; ++q) s += part[q][t];
      tot[t] = s;
    }
    __syncthreads();
    if (t == 0) {
      int bp = 0;
      unsigned long long bt = ~0ull;
      for (int q = 0; q < 64; ++q)
        if (tot[q] < bt) bt = tot[q], bp = q;
      ytab[k] = (uint8_t)bp;
    }
    __syncthreads();
    for (int f = t; f < nfb; f += kCcT) {
      const unsigned long long v = sy[so + f * 64 + ytab[k]];
      if (v < best[f]) best[f] = v;
    }
    __syncthreads();
  }
  for (int f = t; f < nfb; f += kCcT) {
    unsigned long long bv = ~0ull;
    int a = 0;
    for (int k = 0; k < kMaxPresets; ++k) {
      const unsigned long long v = sy[so + f * 64 + ytab[k]];
      if (v < bv) bv = v, a = k;
    }
    asg[f] = (uint8_t)a;
  }
  __syncthreads();
  for (int k = 0; k < kMaxPresets; ++k) {
    unsigned long long acc = 0;
    for (int f = pq; f < nfb; f += kCcW)
      if (active[f] && asg[f] == k) acc += su[so + f * 64 + p] + sv[so + f * 64 + p];
    part[pq][p] = acc;
    __syncthreads();
    if (t < 64) {
      unsigned long long s = 0;
      for (int q = 0; q < kCcW; ++q) s += part[q][t];
      tot[t] = s;
    }
    __syncthreads();
    if (t == 0) {
      int bp = 0;
      unsigned long long bt = ~0ull;
      for (int q = 0; q < 64; ++q)
        if (tot[q] < bt) bt = tot[q], bp = q;
      uvtab[k] = (uint8_t)bp;
    }
    __syncthreads();
  }
  for (int f = t; f < nfb; f += kCcT) {
    int bk = -1;
    if (active[f]) {
      unsigned long long bv = ~0ull;
      for (int k = 0; k < kMaxPresets; ++k) {
        const unsigned long long v = sy[so + f * 64 + ytab[k]] + su[so + f * 64 + uvtab[k]] + sv[so + f * 64 + uvtab[k]];
        if (v < bv) bv = v, bk = k;
      }
    }
    fbidx[(long)b * nfb + f] = (int8_t)bk;
    py[(long)b * nfb + f] = bk < 0 ? (int8_t)-1 : (int8_t)ytab[bk];
    puv[(long)b * nfb + f] = bk < 0 ? (int8_t)-1 : (int8_t)uvtab[bk];
  }
  if (t < 8) {
    tabs[b * 16 + t] = ytab[t];
    tabs[b * 16 + 8 + t] = uvtab[t];
  }
}

// ================================================================= loop restoration =====
// per (segment, unit): projection weights of parameter set `set` from sgr_stats
__global__ void k_av1e_lr_solve(const long long* __restrict__ st, int nu, int B, int set, int* __restrict__ prm) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nu * B) return;
  int x0, x1;
  sgr_solve(st + 5L * i, sgr_param(set, 0), sgr_param(set, 2), &x0, &x1);
  prm[3L * i] = set;
  prm[3L * i + 1] = x0;
  prm[3L * i + 2] = x1;
}

// per (64x64 unit, segment): SSE of two planes over the valid region [0, vw) x [0, vh)
__global__ void __launch_bounds__(256) k_av1e_unit_sse(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b,
                                                       int w, int h, int vw, int vh, long long* __restrict__ out) {
  const int u = blockIdx.x, s = blockIdx.y, ux = (w + 63) >> 6;
  const int x0 = (u % ux) * 64, y0 = (u / ux) * 64;
  const long po = (long)s * w * h;
  unsigned acc = 0;  // <= 4096 * 255^2 < 2^32
  for (int i = threadIdx.x; i < 4096; i += 256) {
    const int x = x0 + (i & 63), y = y0 + (i >> 6);
    if (x < vw && y < vh) {
      const int d = (int)a[po + (long)y * w + x] - (int)b[po + (long)y * w + x];
      acc += (unsigned)(d * d);
    }
  }
  __shared__ long long tot[4];
  const int v = wave_sum((int)acc);  // 1024 pixels x 255^2 per wave < 2^31
  if ((threadIdx.x & 63) == 0) tot[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) out[(long)s * gridDim.x + u] = tot[0] + tot[1] + tot[2] + tot[3];
}

// ================================================================= host helpers =========
thread_local std::string g_err;
int status(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_err = std::string(what) + ": " + hipGetErrorString(e);
    return -1;
  }
  return 0;
}
int ensure_tables() {
  static bool done[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
    g_err = "av1e: no device";
    return -1;
  }
  if (done[dev]) return 0;
  int32_t d16[256], d8[64], a8[64];
  for (int k = 0; k < 16; ++k)
    for (int n = 0; n < 16; ++n) d16[k * 16 + n] = tv::av1::txfm_basis(tv::av1::TX_DCT, 16, k, n);
  for (int k = 0; k < 8; ++k)
    for (int n = 0; n < 8; ++n) {
      d8[k * 8 + n] = tv::av1::txfm_basis(tv::av1::TX_DCT, 8, k, n);
      a8[k * 8 + n] = tv::av1::txfm_basis(tv::av1::TX_ADST, 8, k, n);
    }
  if (hipMemcpyToSymbol(HIP_SYMBOL(c_dct16), d16, sizeof(d16)) != hipSuccess ||
      hipMemcpyToSymbol(HIP_SYMBOL(c_dct8), d8, sizeof(d8)) != hipSuccess ||
      hipMemcpyToSymbol(HIP_SYMBOL(c_adst8), a8, sizeof(a8)) != hipSuccess) {
    g_err = "av1e: basis upload failed";
    return -1;
  }
  done[dev] = true;
  return 0;
}
bool bad(int W, int H, int B, int qidx, const char* what) {
  if (W < 16 || H < 16 || (W & 15) || (H & 15) || B < 1 || B > 65535 || qidx < 1 || qidx > 255 || W > 8192 ||
      H > 8192) {
    g_err = std::string(what) + ": bad geometry / q-index";
    return true;
  }
  return false;
}

// ================================================================= level packing ========
// Device->host layout of a GOP's levels (FrameDecisions::scan_packed): every TB whose plane
// bit is set in its mode word becomes [eob, eob levels in zigzag_scan order], TBs back to
// back in (frame, segment, block) order; the syntax writer expands them.  Past the eob a TB
// is all zero, so the copy moves a fraction of whole-TB bytes.  One wave per TB: length
// pass -> inclusive scan (torch.cumsum) -> pack.  Levels / modes are [F][Bmax][nb] slots
// of which the first `nseg` segments are used.
__device__ __forceinline__ long tb_index(long tb, int nb, int nseg, int Bmax) {
  const long fs = tb / nb;
  return ((fs / nseg) * Bmax + fs % nseg) * nb + (tb - fs * nb);
}
__global__ void __launch_bounds__(256) k_av1e_tb_len(const int16_t* __restrict__ lev,
                                                     const uint32_t* __restrict__ mode, long ntb, int nb, int nseg,
                                                     int Bmax, int p, int* __restrict__ len) {
  __shared__ int16_t sc[256];
  const int N2 = p ? 64 : 256, lane = threadIdx.x & 63;
  if (threadIdx.x == 0) zigzag_scan(p ? 8 : 16, sc);
  __syncthreads();
  for (long tb = (long)blockIdx.x * 4 + (threadIdx.x >> 6); tb < ntb; tb += (long)gridDim.x * 4) {
    const long mi = tb_index(tb, nb, nseg, Bmax);
    const bool nz = (mode[mi] >> (10 + p)) & 1;  // wave-uniform
    int last = 0;                                  // scan index + 1 of the lane's last nonzero
    if (nz)
      for (int k = lane; k < N2; k += 64)
        if (lev[mi * N2 + sc[k]]) last = k + 1;
    const unsigned eob = ~wave_min_u32(~(unsigned)last);
    if (lane == 0) len[tb] = nz ? 1 + (int)eob : 0;
  }
}
__global__ void __launch_bounds__(256) k_av1e_tb_pack(const int16_t* __restrict__ lev, const int* __restrict__ len,
                                                      const long long* __restrict__ end, long ntb, int nb, int nseg,
                                                      int Bmax, int p, int16_t* __restrict__ out) {
  __shared__ int16_t sc[256];
  const int N2 = p ? 64 : 256, lane = threadIdx.x & 63;
  if (threadIdx.x == 0) zigzag_scan(p ? 8 : 16, sc);
  __syncthreads();
  for (long tb = (long)blockIdx.x * 4 + (threadIdx.x >> 6); tb < ntb; tb += (long)gridDim.x * 4) {
    const int L = len[tb];
    if (!L) continue;
    const long mi = tb_index(tb, nb, nseg, Bmax), o = end[tb] - L;
    if (lane == 0) out[o] = (int16_t)(L - 1);
    for (int k = lane; k < L - 1; k += 64) out[o + 1 + k] = lev[mi * N2 + sc[k]];
  }
}

// TV_AV1_INTER_WPE=5: the stage-0 search at the compiler's own allocation (same-box A/B)
using Av1InterKernel = decltype(&k_av1e_inter<0, 6>);
static Av1InterKernel av1_inter0_kernel() {
  static const Av1InterKernel k = [] {
    const char* e = std::getenv("TV_AV1_INTER_WPE");
    return (e && std::atoi(e) == 5) ? &k_av1e_inter<0, 1> : &k_av1e_inter<0, 6>;
  }();
  return k;
}

}  // namespace
}  // namespace gpu
}  // namespace tv

using namespace tv::gpu;

extern "C" {
const char* tv_av1e_last_error() { return g_err.c_str(); }

// P frame of B segments: src / ref / rec planes [B][H][W] (+ chroma [B][H/2][W/2]); qarr:
// device q-index per segment (1..255, range-checked by the host engine).  The motion field
// goes through `tmp` ([B][nb] words): search -> tmp, kMvRefineRounds refinement rounds
// ping-ponging between tmp and mv (ending in mv), then the recon at mv.
int tv_av1e_inter(const uint8_t* sy, const uint8_t* su, const uint8_t* sv, const uint8_t* ry, const uint8_t* ru,
                  const uint8_t* rv, uint8_t* oy, uint8_t* ou, uint8_t* ov, uint32_t* mode, uint32_t* mv, uint32_t* tmp,
                  unsigned long long* satd_acc, uint8_t* memo, int16_t* ly, int16_t* lu, int16_t* lv, int W, int H,
                  int B, const int* qarr, void* stream) {
  if (bad(W, H, B, 1, "av1e_inter") || ensure_tables()) return -1;
  static_assert(kMvRefineRounds % 2 == 1, "an odd round count ends the field in `mv`");
  const int nb = (W >> 4) * (H >> 4), nsb = ((W + 63) >> 6) * ((H + 63) >> 6);
  hipStream_t st = (hipStream_t)stream;
  av1_inter0_kernel()<<<dim3(nb, B), 64, 0, st>>>(Planes3{sy, su, sv}, Planes3{ry, ru, rv}, Planes3W{oy, ou, ov}, mode,
                                               nullptr, tmp, ly, lu, lv, W, H, qarr, satd_acc);
  // memo: two [B][nb] record sets (mv words, SATDs, counts), ping-ponged across the rounds
  const long nrec = (long)B * nb;
  MvMemo mm[2];
  for (int k = 0; k < 2; ++k) {
    uint8_t* base = memo + k * nrec * (kMvRefineMaxCand * 8 + 1);
    mm[k].mv = reinterpret_cast<uint32_t*>(base);
    mm[k].sat = reinterpret_cast<int*>(base + nrec * kMvRefineMaxCand * 4);
    mm[k].n = base + nrec * kMvRefineMaxCand * 8;
  }
  for (int r = 0; r < kMvRefineRounds; ++r) {
    const MvMemo none{nullptr, nullptr, nullptr};
    k_av1e_mv_refine<<<dim3(nsb, B), 256, 0, st>>>(sy, ry, (r & 1) ? mv : tmp, (r & 1) ? tmp : mv, W, H,
                                                    r ? mm[(r - 1) & 1] : none, r + 1 < kMvRefineRounds ? mm[r & 1] : none,
                                                    r > 0);
  }
  if (hipMemsetAsync(satd_acc, 0, (size_t)B * sizeof(unsigned long long), st) != hipSuccess) return status("av1e_inter");
  k_av1e_mv_unify<<<dim3(nsb, B), 256, 0, st>>>(sy, ry, mv, W, H, qarr, satd_acc);
  k_av1e_inter<1, 1><<<dim3(nb, B), 64, 0, st>>>(Planes3{sy, su, sv}, Planes3{ry, ru, rv}, Planes3W{oy, ou, ov}, mode,
                                               mv, mv, ly, lu, lv, W, H, qarr, satd_acc);
  return status("av1e_inter");
}

// Key frame of B segments: one launch per anti-diagonal of the 16x16 block grid.
int tv_av1e_intra(const uint8_t* sy, const uint8_t* su, const uint8_t* sv, uint8_t* oy, uint8_t* ou, uint8_t* ov,
                  uint32_t* mode, uint32_t* mv, int16_t* ly, int16_t* lu, int16_t* lv, int W, int H, int B,
                  const int* qarr, void* stream) {
  if (bad(W, H, B, 1, "av1e_intra") || ensure_tables()) return -1;
  const int bw = W >> 4, bh = H >> 4;
  for (int d = 0; d < bw + bh - 1; ++d) {
    const int lo = d - (bh - 1) > 0 ? d - (bh - 1) : 0, hi = d < bw - 1 ? d : bw - 1;
    k_av1e_intra<<<dim3(hi - lo + 1, B), 64, 0, (hipStream_t)stream>>>(Planes3{sy, su, sv}, Planes3W{oy, ou, ov},
                                                                       mode, mv, ly, lu, lv, W, H, qarr, d, lo);
  }
  return status("av1e_intra");
}

// flag the 8x8 blocks of skip blocks in dir [B][n8] (after tv_gpu_cdef_dirs)
int tv_av1e_cdef_skip(const uint32_t* mode, uint8_t* dir, int W, int H, int B, void* stream) {
  if (bad(W, H, B, 1, "av1e_cdef_skip")) return -1;
  const int n8 = (W >> 3) * (H >> 3);
  k_av1e_cdef_skip<<<dim3((n8 + 255) / 256, B), 256, 0, (hipStream_t)stream>>>(mode, dir, W, H);
  return status("av1e_cdef_skip");
}

// skip-block merging of a P frame's decisions (before lfinfo / deblocking)
int tv_av1e_merge(uint32_t* mode, const uint32_t* mv, int W, int H, int B, void* stream) {
  if (bad(W, H, B, 1, "av1e_merge")) return -1;
  const int n = ((W + 63) >> 6) * ((H + 63) >> 6) * B;
  k_av1e_merge<<<(n + 127) / 128, 128, 0, (hipStream_t)stream>>>(mode, mv, W, H, B);
  return status("av1e_merge");
}

// eob-truncated level packing of `ntb` = F * nseg * nb TBs of plane p (0 luma, 1/2 chroma)
int tv_av1e_tb_len(const int16_t* lev, const uint32_t* mode, long ntb, int nb, int nseg, int Bmax, int p, int* len,
                   void* stream) {
  if (ntb < 0 || nb <= 0 || nseg <= 0 || nseg > Bmax || p < 0 || p > 2 || ntb % ((long)nb * nseg)) {
    g_err = "av1e_tb_len: bad geometry";
    return -1;
  }
  if (!ntb) return 0;
  const long g = std::min((ntb + 3) / 4, 1L << 18);
  k_av1e_tb_len<<<(unsigned)g, 256, 0, (hipStream_t)stream>>>(lev, mode, ntb, nb, nseg, Bmax, p, len);
  return status("av1e_tb_len");
}
// end: inclusive prefix sum of len (int64); out sized end[ntb - 1]
int tv_av1e_tb_pack(const int16_t* lev, const int* len, const long long* end, long ntb, int nb, int nseg, int Bmax,
                    int p, int16_t* out, void* stream) {
  if (ntb < 0 || nb <= 0 || nseg <= 0 || nseg > Bmax || p < 0 || p > 2 || ntb % ((long)nb * nseg)) {
    g_err = "av1e_tb_pack: bad geometry";
    return -1;
  }
  if (!ntb) return 0;
  const long g = std::min((ntb + 3) / 4, 1L << 18);
  k_av1e_tb_pack<<<(unsigned)g, 256, 0, (hipStream_t)stream>>>(lev, len, end, ntb, nb, nseg, Bmax, p, out);
  return status("av1e_tb_pack");
}

// lvl: [B][4] loop_filter_level[0..3] per segment
int tv_av1e_lfinfo(const uint32_t* mode, int W, int H, int B, const int* lvl, uint32_t* iy, uint32_t* iu,
                   uint32_t* iv, void* stream) {
  if (bad(W, H, B, 1, "av1e_lfinfo")) return -1;
  const int n = (W >> 2) * (H >> 2);
  k_av1e_lfinfo<<<dim3((n + 255) / 256, B), 256, 0, (hipStream_t)stream>>>(mode, W, H, lvl, iy, iu, iv);
  return status("av1e_lfinfo");
}

// st [B][nu][5] (tv_gpu_sgr_stats) -> prm [B][nu][3] = (set, xqd0, xqd1)
int tv_av1e_lr_solve(const long long* st, int nu, int B, int set, int* prm, void* stream) {
  if (nu < 1 || B < 1 || set < 0 || set > 15) {
    g_err = "av1e_lr_solve: bad arguments";
    return -1;
  }
  k_av1e_lr_solve<<<(nu * B + 255) / 256, 256, 0, (hipStream_t)stream>>>(st, nu, B, set, prm);
  return status("av1e_lr_solve");
}

// out [B][units]: per-64x64-unit SSE of a / b ([B][h][w]) over the valid region vw x vh
int tv_av1e_unit_sse(const uint8_t* a, const uint8_t* b, int w, int h, int vw, int vh, int B, long long* out,
                     void* stream) {
  if (w < 1 || h < 1 || B < 1 || vw > w || vh > h) {
    g_err = "av1e_unit_sse: bad geometry";
    return -1;
  }
  const int nu = ((w + 63) >> 6) * ((h + 63) >> 6);
  k_av1e_unit_sse<<<dim3(nu, B), 256, 0, (hipStream_t)stream>>>(a, b, w, h, vw, vh, out);
  return status("av1e_unit_sse");
}

// sse_* [B][nfb][64]; tabs [B][16] (8 luma + 8 chroma presets); fbidx / py / puv [B][nfb]
int tv_av1e_cdef_choose(const unsigned long long* sy, const unsigned long long* su, const unsigned long long* sv,
                        const uint32_t* mode, int W, int H, int B, uint8_t* tabs, int8_t* fbidx, int8_t* py,
                        int8_t* puv, void* stream) {
  if (bad(W, H, B, 1, "av1e_cdef_choose")) return -1;
  if (((W + 63) >> 6) * ((H + 63) >> 6) > kMaxFb) {
    g_err = "av1e_cdef_choose: frame too large";
    return -1;
  }
  k_av1e_cdef_choose<<<B, kCcT, 0, (hipStream_t)stream>>>(sy, su, sv, mode, W, H, tabs, fbidx, py, puv);
  return status("av1e_cdef_choose");
}
}

