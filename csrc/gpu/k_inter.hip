// k_inter.hip — P-frame kernels.
//
//  k_inter_me     pass A per CTB (320 threads = 5 waves):
//                   * the source CTB and a 72x72 reference window are staged in LDS as
//                     32-bit words;
//                   * integer full search over [-R, R]^2: each thread owns 4 horizontally
//                     adjacent candidates, loads 3 window words per row and derives the 4
//                     shifted rows with v_alignbyte, accumulating 16 8x8 SADs per candidate
//                     with v_sad_u8 (4 pixels / instruction); 16x16 and 32x32 costs are sums
//                     of 8x8 SADs (SAD reuse);
//                   * half- then quarter-pel refinement of all 21 blocks at once, reading
//                     the precomputed phase planes (no per-block barriers);
//                   * bottom-up CU split decision.
//  k_inter_recon  pass B per CTB: luma prediction = phase-plane loads, chroma 4-tap MC,
//                 residual, MFMA transform/quant, exact inverse, reconstruction.
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "gpu_common.h"
#include "k_encode.h"
#include "tb_coder.h"
#include "wave_tb.h"
#include "tv/me_model.h"
#include "tv/rc_model.h"

namespace tv {
namespace gpu {

// ---------------------------------------------------------------------------------------
// Hierarchical motion search (tv/me_model.h; the CPU golden model is tv::analyze_inter).
//
//  k_quarter     quarter-resolution luma of the source: (sum of a 4x4 block + 8) >> 4,
//                one v_sad_u8 against zero per source row word.
//  k_coarse_me   one wave per CTB: the 8x8 quarter-res block vs the previous quarter-res
//                SOURCE frame, full search over [-Rq, Rq]^2 (Rq = range/4) from an LDS
//                window, 4 horizontally adjacent candidates per lane via v_alignbyte +
//                v_sad_u8.  No recon dependency: the coarse field is a lookahead.
//  k_inter_me    two waves per CTB: up to 7 candidate centres (zero, coarse, 4 coarse
//                neighbours, temporal), an [-4,+3] x [-3,+3] integer window each staged in
//                LDS pre-aligned to the window origin; every lane owns 4 adjacent positions
//                of one (candidate, row) and accumulates all 16 8x8 SADs (16x16 / 32x32 are
//                sums: SAD reuse); then half/quarter-pel refinement of the 21 blocks from
//                the phase planes and the bottom-up CU split decision.  Rate = MVD bits
//                against the CTB predictor.
// ---------------------------------------------------------------------------------------
#ifndef TV_ME_THREADS
#define TV_ME_THREADS 256
#endif
constexpr int kMeThreads = TV_ME_THREADS;  // a multiple of 64 (the DPP group sums assume it)
static_assert(kMeThreads % 64 == 0 && kMeThreads >= 256, "k_inter_me block size");
constexpr int kFRows = kCtb + kMeWinH - 1;  // 38 window rows per candidate
constexpr int kFWords = 12;                 // 48 bytes staged (40 used: 32 + 7 offsets + 1)
constexpr int kFChunks = kFWords / 4;       // 16-byte chunks per staged row
// Window layout: pitch 12 words, rows >= 16 kWinSkew words further (per candidate).  A
// half-wave of the integer search reads 8 (row, 4-position group) items x 4 quadrants,
// rows r and r + 16 together; brute force over pitch / skew (ds_read_b32 banks (a/4) % 32)
// gives 1344 extra LDS cycles over all item phases for 12 / +2 against 2016 for the former
// odd pitch 13, in less LDS.
constexpr int kFPitch = kFWords, kWinSkew = 2, kWinCand = kFRows * kFPitch + kWinSkew;
__device__ __forceinline__ int win_word(int k, int r, int w) { return k * kWinCand + r * kFPitch + (r >= 16 ? kWinSkew : 0) + w; }
// LDS pitch (words) of a source-CTB row (uniform s0/s1 reads stay one aligned 8-byte read).
// Every 8-row band sits kSrcSkew (8) words further, so rows 8 apart land 8 banks apart: the
// sub-pel SAD lanes of one candidate read rows by + j of blocks 8 / 16 rows apart at the same
// time (with a flat 8-word pitch 64 words apart -- one bank, 4-way conflicts: 18.6 % of the
// kernel's LDS cycles, r6_prof), and the four quadrant lanes of an integer-search item read
// rows r and r + 16 (16 banks apart) at word offsets 0 / 4: 32 distinct banks either way.
constexpr int kSrcP = 8, kSrcSkew = 8;
__device__ __forceinline__ int src_word(int row, int w) { return row * kSrcP + w + (row >> 3) * kSrcSkew; }

__device__ __forceinline__ void me_blk_geom(int bi, int& bx, int& by, int& l2) {
  if (bi < 16) {
    bx = (bi & 3) * 8;
    by = (bi >> 2) * 8;
    l2 = 3;
  } else if (bi < 20) {
    bx = ((bi - 16) & 1) * 16;
    by = ((bi - 16) >> 1) * 16;
    l2 = 4;
  } else {
    bx = by = 0;
    l2 = 5;
  }
}
__device__ __forceinline__ int me_blk8_of(int q, int r) {
  return (((q >> 1) * 2 + (r >> 1)) << 2) + (q & 1) * 2 + (r & 1);
}
// tv::dequant_level in 32-bit arithmetic: with m = 16 * levelScale << (qp / 6) and the level
// clamped to +-thr, where thr * m just exceeds (32768 + 1) << bdShift, a clamped level still
// saturates to the same int16 bound and every unclamped product fits in 32 bits -- the same
// result as the 64-bit golden form, with a med3 + mad + shift + med3 per level.
struct DeqParams {
  int m, thr, sh, rnd;
};
__device__ __forceinline__ DeqParams deq_params(int qp, int log2N) {
  DeqParams d;
  d.sh = 8 + log2N - 5;
  d.rnd = 1 << (d.sh - 1);
  d.m = (16 * level_scale(qp)) << (qp / 6);
  d.thr = (((32768 + 1) << d.sh) + d.m - 1) / d.m;
  return d;
}
__device__ __forceinline__ int deq_fast(int level, const DeqParams& d) {
  const int t = clip3(-d.thr, d.thr, level);
  return clip3(-32768, 32767, (t * d.m + d.rnd) >> d.sh);
}

// the 4 byte differences a - b as two dwords of int16 pairs (residual = source - prediction)
__device__ __forceinline__ uint2 bytes_minus(uint32_t a, uint32_t b) {
  typedef short s2 __attribute__((ext_vector_type(2)));
  const s2 lo = __builtin_bit_cast(s2, __builtin_amdgcn_perm(0u, a, 0x0c010c00u)) -
                __builtin_bit_cast(s2, __builtin_amdgcn_perm(0u, b, 0x0c010c00u));
  const s2 hi = __builtin_bit_cast(s2, __builtin_amdgcn_perm(0u, a, 0x0c030c02u)) -
                __builtin_bit_cast(s2, __builtin_amdgcn_perm(0u, b, 0x0c030c02u));
  return make_uint2(__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi));
}
__device__ __forceinline__ int phase_at(const uint8_t* P, const Geo& g, int x, int y) {
  x = clip3(-8, g.W + 7, x);
  y = clip3(-8, g.H + 7, y);
  return P[(long)(y + 8) * g.pw16 + x + 8];
}
// 4 bytes of row `row` starting at byte x (any alignment), clamped horizontally to [0, w-1]
__device__ __forceinline__ uint32_t load4_clamped(const uint8_t* row, int x, int w) {
  const int a = x & ~3, sh = x & 3;
  if (x >= 0 && a + 7 < w) {
    const uint32_t w0 = *reinterpret_cast<const uint32_t*>(row + a);
    if (!sh) return w0;
    const uint32_t w1 = *reinterpret_cast<const uint32_t*>(row + a + 4);
    return __builtin_amdgcn_alignbyte(w1, w0, sh);
  }
  uint32_t v = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) v |= (uint32_t)row[clip3(0, w - 1, x + k)] << (8 * k);
  return v;
}

__global__ void __launch_bounds__(256) k_quarter(FrameSet src, uint8_t* q, Geo g) {
  const int b = blockIdx.y, qw = g.W >> 2, qh = g.H >> 2;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= qw * qh) return;
  const int x = i % qw, y = i / qw;
  const uint8_t* S = src.plane(0, b, g) + (long)(4 * y) * g.W + 4 * x;
  unsigned s = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) s = __builtin_amdgcn_sad_u8(*reinterpret_cast<const uint32_t*>(S + (long)j * g.W), 0u, s);
  q[(long)b * qw * qh + i] = (uint8_t)((s + 8) >> 4);
}

constexpr int kCoarseMaxRq = 32;
constexpr int kCoarseRows = 8 + 2 * kCoarseMaxRq;
constexpr int kCoarseWords = kCoarseMaxRq / 2 + 3;

__global__ void __launch_bounds__(64) k_coarse_me(const uint8_t* qcur, const uint8_t* qprev, Geo g, const RcTables* rc,
                                                  int seq_qp, int rq, int16_t* cmv, int* ccost) {
  const int lane = threadIdx.x;
  int ctu, b;
  xcd_ctb(ctu, b);
  const Penalties& pen = rc->pen[seq_qp];  // lookahead: the frame QP may depend on its result
  const int qw = g.W >> 2, qh = g.H >> 2;
  const int x0 = 8 * (ctu % g.wc), y0 = 8 * (ctu / g.wc);
  const uint8_t* C = qcur + (long)b * qw * qh;
  const uint8_t* P = qprev + (long)b * qw * qh;
  __shared__ uint32_t s32[16];
  extern __shared__ uint32_t win[];  // (8 + 2 rq) rows x ((rq / 2 + 3) | 1) words: sized per launch
  __shared__ int penL[64];  // the MV-rate table: read per candidate (a global load chain before)
  const int side = 2 * rq + 1, rows = 8 + 2 * rq, wpr = rq / 2 + 3, pitch = wpr | 1;
  penL[lane] = pen.mv[lane];
  if (lane < 16) s32[lane] = *reinterpret_cast<const uint32_t*>(C + (long)(y0 + (lane >> 1)) * qw + x0 + 4 * (lane & 1));
  for (int w = lane; w < rows * wpr; w += 64) {
    const int r = w / wpr, c = w - r * wpr;
    const uint8_t* row = P + (long)clip3(0, qh - 1, y0 - rq + r) * qw;
    win[r * pitch + c] = load4_clamped(row, x0 - rq + 4 * c, qw);
  }
  __syncthreads();
  unsigned best = 0xffffffffu;
  const int groups = rq / 2 + 1;
  uint32_t sv[16];  // the source block in registers (loop-invariant)
#pragma unroll
  for (int k = 0; k < 16; ++k) sv[k] = s32[k];
  // item = gi * side + dyi, advanced by 64 per pass without a division
  const int step_g = 64 / side, step_d = 64 - step_g * side;
  int gi = lane / side, dyi = lane - gi * side;
  for (int item = lane; item < groups * side; item += 64) {
    const int dy = dyi - rq, dx0 = 4 * gi - rq;
    unsigned acc[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t s0 = sv[2 * j], s1 = sv[2 * j + 1];
      const int wr = (dyi + j) * pitch + gi;
      const uint32_t w0 = win[wr], w1 = win[wr + 1], w2 = win[wr + 2];
      acc[0] = __builtin_amdgcn_sad_u8(w1, s1, __builtin_amdgcn_sad_u8(w0, s0, acc[0]));
#pragma unroll
      for (int sft = 1; sft < 4; ++sft) {
        const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sft);
        const uint32_t hi = __builtin_amdgcn_alignbyte(w2, w1, sft);
        acc[sft] = __builtin_amdgcn_sad_u8(hi, s1, __builtin_amdgcn_sad_u8(lo, s0, acc[sft]));
      }
    }
#pragma unroll
    for (int sft = 0; sft < 4; ++sft) {
      const int dx = dx0 + sft;
      if (dx > rq) continue;
      const unsigned v = ((acc[sft] + (unsigned)me_coarse_pen(penL, dx, dy)) << 13) | (unsigned)(dyi * side + dx + rq);
      best = v < best ? v : best;
    }
    gi += step_g;
    dyi += step_d;
    if (dyi >= side) {
      dyi -= side;
      ++gi;
    }
  }
  best = wave_min_u32(best);
  if (lane == 0) {
    const int idx = (int)(best & 8191), o = b * g.wc * g.hc + ctu;
    cmv[2 * o] = (int16_t)(4 * (idx % side - rq));
    cmv[2 * o + 1] = (int16_t)(4 * (idx / side - rq));
    ccost[o] = (int)(best >> 13);
  }
}

// ROWS: rows per sub-pel SAD group, 8 (384 groups) or 4 (768 groups, 3 per thread: measured
// 10 % slower -- a third pass exposes its load latency once more).  PEN_LDS: the MV-rate table
// (Penalties::mv, 64 ints) staged in LDS -- the integer search and the sub-pel argmin read it
// per candidate, which from global memory put a dependent load chain between the barriers.
// WPE: waves per SIMD the register allocation must allow (8: <= 64 VGPRs, 8 CTBs per CU --
// with the 7.8 KB quadrant table gone the LDS fits 8 as well; 7 = the compiler's own 70 VGPRs).
template <int ROWS, bool PEN_LDS, int WPE>
__global__ void __launch_bounds__(kMeThreads) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) k_inter_me(FrameSet src, FrameSet ref, const uint8_t* phase,
                                                         DecisionSet dec, const int16_t* prev_mv, const int16_t* cmv,
                                                         Geo g, const RcTables* rc, int range, int diag_stop,
                                                         CtbMeOut* bout, PIntraBuffers pi) {
  const int tid = threadIdx.x;
  int ctu, b;
  xcd_ctb(ctu, b);
  const Penalties& pen = rc->pen[dec.qp[b]];
  __shared__ int penL[64];
  if (PEN_LDS && tid < 64) penL[tid] = pen.mv[tid];
  const int* penmv = PEN_LDS ? penL : pen.mv;  // visible after the first barrier below
  const int cxi = ctu % g.wc, cyi = ctu / g.wc, cx = cxi * 32, cy = cyi * 32;
  const uint8_t* S = src.plane(0, b, g);
  const uint8_t* R = ref.plane(0, b, g);
  __shared__ uint32_t s32[32 * kSrcP + 3 * kSrcSkew];
  __shared__ uint32_t win[kMeMaxCand * kWinCand];
  __shared__ int cand[kMeMaxCand][2];
  __shared__ int pmv[2], ncand;
  __shared__ unsigned best[21];
  __shared__ int bcost[21], bmv[21][2];
  __shared__ int subsad[21][8];
  for (int t = tid; t < 256; t += kMeThreads)
    s32[src_word(t >> 3, t & 7)] = *reinterpret_cast<const uint32_t*>(S + (long)(cy + (t >> 3)) * g.W + cx + 4 * (t & 7));
  // candidate sources: the coarse vectors of the CTB's 3x3 neighbourhood (clipped to the
  // picture) and the co-located previous vector, gathered by 10 lanes at once into LDS; thread
  // 0 then runs me_candidates on that local window (same bounds, so the same candidates)
  // instead of a chain of dependent global loads ahead of the window staging
  __shared__ int16_t nbmv[18], tmv[2];
  const int lx0 = cxi > 0 ? cxi - 1 : 0, ly0 = cyi > 0 ? cyi - 1 : 0;
  const int lw = (cxi + 1 < g.wc ? cxi + 1 : g.wc - 1) - lx0 + 1, lh = (cyi + 1 < g.hc ? cyi + 1 : g.hc - 1) - ly0 + 1;
  if (tid < 9) {
    const int i = tid % 3, j = tid / 3;
    if (i < lw && j < lh) {
      const int16_t* c = cmv + (long)b * g.wc * g.hc * 2 + 2 * ((long)(ly0 + j) * g.wc + lx0 + i);
      nbmv[2 * (j * lw + i)] = c[0];
      nbmv[2 * (j * lw + i) + 1] = c[1];
    }
  } else if (tid == 9) {
    const long u0 = b * g.usz + (long)(cy >> 3) * g.w8 + (cx >> 3);
    tmv[0] = prev_mv[2 * u0];
    tmv[1] = prev_mv[2 * u0 + 1];
  }
  if (tid < 21) best[tid] = 0xffffffffu;
  __syncthreads();
  if (tid == 0) {
    if (diag_stop & 16)  // TV_ME_CAND=global (A/B reference): the former global-memory path
      ncand = me_candidates(cmv + (long)b * g.wc * g.hc * 2, g.wc, g.hc, cxi, cyi, tmv[0], tmv[1], range - 4, cand, pmv);
    else
      ncand = me_candidates(nbmv, lw, lh, cxi - lx0, cyi - ly0, tmv[0], tmv[1], range - 4, cand, pmv);
  }
  __syncthreads();
  diag_stop &= 15;
  const int nc = ncand;
  // candidate windows, each pre-aligned so byte 0 of a row is x = cx + cand_x + kMeWinX0
  // one lane per 16-byte chunk: a dwordx4 + dword load from the dword-aligned address, then
  // v_alignbyte to the candidate's byte offset (the clamped per-byte path only at the edges)
  // All of a thread's chunks (<= 4) are loaded before any is stored, so their global
  // latencies overlap instead of one round trip per loop pass.
  constexpr int kWinPer = (kMeMaxCand * kFRows * kFChunks + kMeThreads - 1) / kMeThreads;
  {
    const int ntot = nc * kFRows * kFChunks;
    uint4 u[kWinPer];
    uint32_t u4[kWinPer];
#pragma unroll
    for (int n = 0; n < kWinPer; ++n) {
      const int e = tid + n * kMeThreads;
      u[n] = make_uint4(0, 0, 0, 0);
      u4[n] = 0;
      if (e < ntot) {
        const int k = e / (kFRows * kFChunks), rem = e - k * (kFRows * kFChunks);
        const int r = rem / kFChunks, ch = rem - r * kFChunks;
        const uint8_t* row = R + (long)clip3(0, g.H - 1, cy + cand[k][1] + kMeWinY0 + r) * g.W;
        const int x = cx + cand[k][0] + kMeWinX0 + 16 * ch, a = x & ~3;
        if (x >= 0 && a + 20 <= g.W) {
          u[n] = *reinterpret_cast<const uint4*>(row + a);
          u4[n] = *reinterpret_cast<const uint32_t*>(row + a + 16);
        }
      }
    }
#pragma unroll
    for (int n = 0; n < kWinPer; ++n) {
      const int e = tid + n * kMeThreads;
      if (e >= ntot) break;
      const int k = e / (kFRows * kFChunks), rem = e - k * (kFRows * kFChunks);
      const int r = rem / kFChunks, ch = rem - r * kFChunks;
      const int x = cx + cand[k][0] + kMeWinX0 + 16 * ch, a = x & ~3, sh = x & 3;
      uint32_t* dst = win + win_word(k, r, 4 * ch);
      if (x >= 0 && a + 20 <= g.W) {
        dst[0] = __builtin_amdgcn_alignbyte(u[n].y, u[n].x, sh);
        dst[1] = __builtin_amdgcn_alignbyte(u[n].z, u[n].y, sh);
        dst[2] = __builtin_amdgcn_alignbyte(u[n].w, u[n].z, sh);
        dst[3] = __builtin_amdgcn_alignbyte(u4[n], u[n].w, sh);
      } else {  // the clamped per-byte path at the picture edges
        const uint8_t* row = R + (long)clip3(0, g.H - 1, cy + cand[k][1] + kMeWinY0 + r) * g.W;
#pragma unroll
        for (int j = 0; j < 4; ++j) dst[j] = load4_clamped(row, x + 4 * j, g.W);
      }
    }
  }
  __syncthreads();
  // timing diagnostics only (TV_DIAG_ME_STOP=1/2/3): later search phases are skipped and the
  // decisions degrade (still well-formed); never set in production
  const bool skip_int = diag_stop == 1, skip_sub = diag_stop == 1 || diag_stop == 2;

  // ------------------------------- integer refinement -----------------------------------
  // item = (candidate, window row, 4-position group, 16x16 quadrant): a lane accumulates
  // the 4 8x8 SADs of its quadrant for 4 adjacent positions (their sum is the quadrant's
  // 16x16 SAD); the 32x32 SADs are the sums of the 4 quadrants, which are the 4 lanes of a
  // quad (items 4j..4j+3): a DPP quad sum, no LDS round trip (a [position][quadrant] LDS
  // table cost 7.8 KB -- a CTB per CU of occupancy -- and a barrier).
  // Splitting by quadrant keeps every lane busy when few distinct candidates remain.
  unsigned lb[5];  // 4 8x8 blocks of my quadrant, then its 16x16
#pragma unroll
  for (int k = 0; k < 5; ++k) lb[k] = 0xffffffffu;
  unsigned lb32 = 0xffffffffu;  // the 32x32 minimum (quadrant-0 lanes)
  int qd = 0;
  for (int item = skip_int ? kMeThreads * 64 : tid; item < nc * kMeWinH * 2 * 4; item += kMeThreads) {
    qd = item & 3;
    const int it = item >> 2;
    const int k = it / (kMeWinH * 2), rr = it - k * (kMeWinH * 2);
    const int dyi = rr >> 1, gs = rr & 1;
    const int pos0 = k * kMePosPerCand + dyi * kMeWinW + 4 * gs;
    const int my = cand[k][1] + kMeWinY0 + dyi;
    unsigned mvc[4];
#pragma unroll
    for (int sft = 0; sft < 4; ++sft) {
      const int mx = cand[k][0] + kMeWinX0 + 4 * gs + sft;
      mvc[sft] = (unsigned)penmv[me_pen_index(4 * mx - pmv[0], 4 * my - pmv[1])];
    }
    const int qx = (qd & 1) * 16, qy = (qd >> 1) * 16;

    unsigned q16[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j8 = 0; j8 < 4; ++j8) {
      const int bx = qx + (j8 & 1) * 8, by = qy + (j8 >> 1) * 8;
      unsigned acc[4] = {0, 0, 0, 0};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int srow = src_word(by + j, bx >> 2);
        const uint32_t s0 = s32[srow], s1 = s32[srow + 1];
        const uint32_t* wp = win + win_word(k, dyi + by + j, gs + (bx >> 2));
        const uint32_t w0 = wp[0], w1 = wp[1], w2 = wp[2];
        acc[0] = __builtin_amdgcn_sad_u8(w1, s1, __builtin_amdgcn_sad_u8(w0, s0, acc[0]));
#pragma unroll
        for (int sft = 1; sft < 4; ++sft) {
          const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sft);
          const uint32_t hi = __builtin_amdgcn_alignbyte(w2, w1, sft);
          acc[sft] = __builtin_amdgcn_sad_u8(hi, s1, __builtin_amdgcn_sad_u8(lo, s0, acc[sft]));
        }
      }
#pragma unroll
      for (int sft = 0; sft < 4; ++sft) {
        const unsigned v = ((acc[sft] + mvc[sft]) << 11) | (unsigned)(pos0 + sft);
        lb[j8] = v < lb[j8] ? v : lb[j8];
        q16[sft] += acc[sft];
      }
      __builtin_amdgcn_sched_barrier(0);  // bound live ranges: no hoisting across 8x8 blocks
    }
#pragma unroll
    for (int sft = 0; sft < 4; ++sft) {
      const unsigned v = ((q16[sft] + mvc[sft]) << 11) | (unsigned)(pos0 + sft);
      lb[4] = v < lb[4] ? v : lb[4];
      // the quad's lanes are one position's 4 quadrants (a quad is always wholly in range)
      int t = (int)q16[sft];
      t += dpp::mov<dpp::kQuadXor1>(t);
      t += dpp::mov<dpp::kQuadXor2>(t);
      const unsigned v32 = ((unsigned)(t + (int)mvc[sft]) << 11) | (unsigned)(pos0 + sft);
      lb32 = (qd == 0 && v32 < lb32) ? v32 : lb32;
    }
  }
  // a lane's quadrant is fixed (item stride is a multiple of 4: quadrant = lane & 3), so lb[]
  // maps to static slots.  Each slot is reduced over the 16 lanes of its quadrant class:
  // rotations by 4 and 8 inside a DPP row, then the row pairs and halves exchanged with
  // v_permlane16_swap / v_permlane32_swap (gfx950) -- lanes 0..3 end with quadrant 0..3's
  // minima and post them (5 x ~6 VALU instead of 20 full wave reductions)
  {
    auto umin = [](unsigned x, unsigned y) { return x < y ? x : y; };
    const int lane = tid & 63;
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      unsigned v = lb[j];
      v = umin(v, (unsigned)dpp::mov<dpp::kRowRor4>((int)v));
      v = umin(v, (unsigned)dpp::mov<dpp::kRowRor8>((int)v));
      const auto r16 = __builtin_amdgcn_permlane16_swap(v, v, false, false);
      v = umin(r16[0], r16[1]);
      const auto r32 = __builtin_amdgcn_permlane32_swap(v, v, false, false);
      v = umin(r32[0], r32[1]);
      if (lane < 4) {  // quadrant q = lane: 8x8 block (q, j) in raster order, or its 16x16
        const int k = j < 4 ? ((lane >> 1) << 3) | ((j >> 1) << 2) | ((lane & 1) << 1) | (j & 1) : 16 + lane;
        atomicMin(&best[k], v);
      }
    }
  }
  {
    const unsigned m = wave_min_u32(lb32);
    if ((tid & 63) == 0) atomicMin(&best[20], m);
  }
  __syncthreads();
  if (tid < 21) {
    int mx = 0, my = 0;
    if (!skip_int) me_pos_to_mv((int)(best[tid] & 2047), cand, mx, my);
    bcost[tid] = skip_int ? 0 : (int)(best[tid] >> 11);
    bmv[tid][0] = 4 * mx;
    bmv[tid][1] = 4 * my;
  }

  // ------------------------ half- then quarter-pel refinement ---------------------------
  const uint8_t* sb = reinterpret_cast<const uint8_t*>(s32);
  const uint8_t* ph = phase + (long)b * 16 * g.psz;
  const int last_step = skip_sub ? 4 : (diag_stop == 3 ? 2 : 1);
  for (int step = 2; step >= last_step; step >>= 1) {
    __syncthreads();  // bmv of the previous step / the integer search
    // A thread owns a group of ROWS rows x 8 pixels of one (block, candidate): per row it
    // loads 3 aligned dwords of the phase plane, forms the 2 shifted dwords with v_alignbyte
    // and accumulates with v_sad_u8.  ROWS = 4: 32 (8x8) + 32 (16x16) + 32 (32x32) groups per
    // candidate, 768 in all = exactly 3 per thread; ROWS = 8: 384 = 1.5 per thread (half the
    // threads run a second pass while the others wait at the barrier).
    constexpr int G8 = 8 / ROWS, N8 = 16 * G8, NC = 3 * N8;  // groups per 8x8 block / class / candidate
    for (int grp = tid; grp < 8 * NC; grp += kMeThreads) {
      const int k = grp / NC, r = grp - k * NC;
      int bi, row0, col0;
      if (r < N8) {
        bi = r / G8;
        row0 = ROWS * (r % G8);
        col0 = 0;
      } else if (r < 2 * N8) {
        const int q = (r - N8) % (4 * G8);
        bi = 16 + (r - N8) / (4 * G8);
        row0 = ROWS * (q >> 1);
        col0 = 8 * (q & 1);
      } else {
        const int q = r - 2 * N8;
        bi = 20;
        row0 = ROWS * (q >> 2);
        col0 = 8 * (q & 3);
      }
      int bx, by, l2b;
      me_blk_geom(bi, bx, by, l2b);
      int ox, oy;
      me_cand_offset(k, ox, oy);
      const int mx = bmv[bi][0] + ox * step, my = bmv[bi][1] + oy * step;
      const uint8_t* P = ph + (long)((mx & 3) + 4 * (my & 3)) * g.psz;
      const int gx0 = cx + bx + col0 + (mx >> 2);
      const int gy0 = cy + by + row0 + (my >> 2);
      const int sr0 = by + row0, sw0 = (bx + col0) >> 2;  // source row / word of row 0
      unsigned sad = 0;
      if (gx0 >= -8 && gx0 + 11 <= g.W + 7 && gy0 >= -8 && gy0 + ROWS - 1 <= g.H + 7) {
        const int a = gx0 & ~3, sh = gx0 & 3;
        const uint8_t* rowp = P + (long)(gy0 + 8) * g.pw16 + a + 8;
#pragma unroll
        for (int j = 0; j < ROWS; ++j) {
          const uint32_t* wp = reinterpret_cast<const uint32_t*>(rowp + (long)j * g.pw16);
          const uint32_t w0 = wp[0], w1 = wp[1], w2 = wp[2];
          const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sh);
          const uint32_t hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
          const int sw = src_word(sr0 + j, sw0);
          sad = __builtin_amdgcn_sad_u8(hi, s32[sw + 1], __builtin_amdgcn_sad_u8(lo, s32[sw], sad));
        }
      } else {  // touches the clamped border: per-pixel path
        for (int j = 0; j < ROWS; ++j) {
          const int gy = clip3(-8, g.H + 7, gy0 + j);
          for (int i = 0; i < 8; ++i) {
            const int gx = clip3(-8, g.W + 7, gx0 + i);
            sad += tv_abs((int)sb[4 * src_word(sr0 + j, 0) + bx + col0 + i] - (int)P[(long)(gy + 8) * g.pw16 + gx + 8]);
          }
        }
      }
      // group sums on the VALU (a wave's lanes all run the same passes): aligned groups of G8
      // lanes = an 8x8 block, 4 G8 = a 16x16 block, 16 G8 = the 32x32 block -- every
      // (block, candidate) cell is written exactly once, by a plain store
      int s1 = (int)sad;
      if (G8 == 2) s1 += dpp::mov<dpp::kQuadXor1>(s1);
      int s4 = s1 + dpp::mov<G8 == 2 ? dpp::kQuadXor2 : dpp::kQuadXor1>(s1);
      if (G8 == 1) s4 += dpp::mov<dpp::kQuadXor2>(s4);
      else s4 += dpp::mov<dpp::kRowHalfMirror>(s4);  // G8 = 2: 8 lanes
      int s16 = s4;
      if (G8 == 1) s16 += dpp::mov<dpp::kRowHalfMirror>(s16);
      s16 += dpp::mov<dpp::kRowMirror>(s16);
      if (G8 == 2) s16 += __shfl_xor(s16, 16, 64);
      if (r < N8) {
        if (r % G8 == 0) subsad[bi][k] = s1;
      } else if (r < 2 * N8) {
        if ((r - N8) % (4 * G8) == 0) subsad[bi][k] = s4;
      } else if (r == 2 * N8) {
        subsad[bi][k] = s16;
      }
    }
    __syncthreads();
    if (tid < 21) {
      unsigned bestv = (unsigned)bcost[tid] << 4;
      for (int k = 0; k < 8; ++k) {
        int ox, oy;
        me_cand_offset(k, ox, oy);
        const int mx = bmv[tid][0] + ox * step, my = bmv[tid][1] + oy * step;
        const unsigned v =
            ((unsigned)(subsad[tid][k] + penmv[me_pen_index(mx - pmv[0], my - pmv[1])]) << 4) | (unsigned)(k + 1);
        bestv = v < bestv ? v : bestv;
      }
      const int kk = (int)(bestv & 15);
      bcost[tid] = (int)(bestv >> 4);
      if (kk) {
        int ox, oy;
        me_cand_offset(kk - 1, ox, oy);
        bmv[tid][0] += ox * step;
        bmv[tid][1] += oy * step;
      }
    }
    __syncthreads();
  }

  // B picture: hand this list's 21 block results to k_bi_decide
  if (bout) {
    if (tid < 21) {
      CtbMeOut& o = bout[(long)b * g.wc * g.hc + ctu];
      o.cost[tid] = bcost[tid];
      o.mv[tid][0] = bmv[tid][0];
      o.mv[tid][1] = bmv[tid][1];
      o.pen[tid] = penmv[me_pen_index(bmv[tid][0] - pmv[0], bmv[tid][1] - pmv[1])];
    }
    return;
  }
  // ------------------------------- CU split decision ------------------------------------
  // one lane per 8x8 unit k (raster): every lane forms the same quadrant / CTB sums from the
  // 21 block costs (the same order of additions as the serial form), then writes its unit
  if (tid < 16) {
    const int ps = pen.split_inter, k = tid, ux = k & 3, uy = k >> 2;
    int sum16 = 0, qsplit = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      int sum8 = 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) sum8 += bcost[me_blk8_of(q, r)] + ps;
      const bool split = sum8 < bcost[16 + q] + ps;
      sum16 += split ? sum8 : bcost[16 + q] + ps;
      qsplit |= split ? 1 << q : 0;
    }
    const bool whole = bcost[20] + ps <= sum16;
    const int q = (uy >> 1) * 2 + (ux >> 1), r = (uy & 1) * 2 + (ux & 1);
    const bool split = (qsplit >> q) & 1;
    const int sbi = whole ? 20 : (split ? me_blk8_of(q, r) : 16 + q);
    const long u = b * g.usz + (long)((cy >> 3) + uy) * g.w8 + (cx >> 3) + ux;
    dec.cu_log2[u] = whole ? 5 : (split ? 3 : 4);
    dec.mv[2 * u] = (int16_t)bmv[sbi][0];
    dec.mv[2 * u + 1] = (int16_t)bmv[sbi][1];
    dec.intra[u] = 0;
    dec.ipm[u] = 1;
    if (pi.qcost && k < 4) {  // intra-in-P: quadrants past the gate go on k_pintra_analysis' list
      const long qi = ((long)b * g.wc * g.hc + ctu) * 4 + k;
      pi.qcost[qi] = bcost[16 + k];
      pi.cand[qi] = 0;
      if (bcost[16 + k] > kPIntraGate * 256) pi.gate[atomicAdd(&pi.count[0], 1)] = (int)qi;
    }
  }
}

// ---------------------------------------------------------------------------------------
// B picture pass A, second half (golden: tv::analyze_inter_b): the SAD of the 8-bit average
// of both lists' predictions for all 21 ME blocks (one wave covers one 8x8 block or a 64-
// sample quarter of a larger one: a wave sum, one LDS atomic), then per block the cheapest of
// list 0, list 1 and bi (ties keep the earlier), then the bottom-up CU split.
// ---------------------------------------------------------------------------------------
// 4 phase-plane samples at (x .. x+3, y), any alignment: two dword loads + v_alignbyte
// inside the padded plane, per-byte clamped loads at the border
__device__ __forceinline__ uint32_t phase4(const uint8_t* P, const Geo& g, int x, int y) {
  const int a = x & ~3;
  if (x >= -8 && a + 7 <= g.W + 7 && y >= -8 && y <= g.H + 7) {
    const uint8_t* row = P + (long)(y + 8) * g.pw16 + a + 8;
    const uint32_t w0 = *reinterpret_cast<const uint32_t*>(row), w1 = *reinterpret_cast<const uint32_t*>(row + 4);
    return __builtin_amdgcn_alignbyte(w1, w0, x & 3);
  }
  uint32_t v = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) v |= (uint32_t)phase_at(P, g, x + k, y) << (8 * k);
  return v;
}

__global__ void __launch_bounds__(256) k_bi_decide(FrameSet src, const uint8_t* phase0, const uint8_t* phase1,
                                                    const CtbMeOut* me0, const CtbMeOut* me1, DecisionSet dec, Geo g,
                                                    const RcTables* rc) {
  const int tid = threadIdx.x;
  int ctu, b;
  xcd_ctb(ctu, b);
  const long o = (long)b * g.wc * g.hc + ctu;
  const CtbMeOut& A = me0[o];
  const CtbMeOut& Bm = me1[o];
  const int cx = (ctu % g.wc) * 32, cy = (ctu / g.wc) * 32;
  __shared__ uint32_t s32[256];  // the source CTB, 8 words per row
  __shared__ int sad[21];
  __shared__ int mvs[2][21][2];
  const uint8_t* S = src.plane(0, b, g);
  s32[tid] = *reinterpret_cast<const uint32_t*>(S + (long)(cy + (tid >> 3)) * g.W + cx + 4 * (tid & 7));
  if (tid < 21) sad[tid] = 0;
  if (tid < 84) {
    const int l = tid / 42, r = tid - l * 42;
    mvs[l][r >> 1][r & 1] = (l ? Bm : A).mv[r >> 1][r & 1];
  }
  __syncthreads();
  const uint8_t* p0b = phase0 + (long)b * 16 * g.psz;
  const uint8_t* p1b = phase1 + (long)b * 16 * g.psz;
  // item = 4 horizontally adjacent samples of one block: 256 for the 16 8x8 blocks, 256 for
  // the 4 16x16, 256 for the 32x32; the 8-bit average of both predictions is one
  // (a | c) - ((a ^ c) >> 1) per dword and its SAD one v_sad_u8
  for (int item = tid; item < 768; item += 256) {
    int bi, x, y;
    if (item < 256) {
      bi = item >> 4;
      const int r = item & 15;
      x = (bi & 3) * 8 + (r & 1) * 4;
      y = (bi >> 2) * 8 + (r >> 1);
    } else if (item < 512) {
      const int j = item - 256;
      bi = 16 + (j >> 6);
      const int r = j & 63;
      x = ((bi - 16) & 1) * 16 + (r & 3) * 4;
      y = ((bi - 16) >> 1) * 16 + (r >> 2);
    } else {
      const int j = item - 512;
      bi = 20;
      x = (j & 7) * 4;
      y = j >> 3;
    }
    const int m0x = mvs[0][bi][0], m0y = mvs[0][bi][1], m1x = mvs[1][bi][0], m1y = mvs[1][bi][1];
    const uint32_t a = phase4(p0b + (long)((m0x & 3) + 4 * (m0y & 3)) * g.psz, g, cx + x + (m0x >> 2), cy + y + (m0y >> 2));
    const uint32_t c = phase4(p1b + (long)((m1x & 3) + 4 * (m1y & 3)) * g.psz, g, cx + x + (m1x >> 2), cy + y + (m1y >> 2));
    const uint32_t avg = (a | c) - (((a ^ c) >> 1) & 0x7f7f7f7fu);
    atomicAdd(&sad[bi], (int)__builtin_amdgcn_sad_u8(avg, s32[y * 8 + (x >> 2)], 0u));
  }
  __syncthreads();
  // per block: the cheapest of list 0, list 1 and bi (ties keep the earlier); then the
  // quadrant splits, the whole-CTB choice and each unit's motion, one lane each
  __shared__ int cost[21], dirb[21], qsum[4], qsplit[4], whole;
  const Penalties& pen = rc->pen[dec.qp[b]];
  const int ps = pen.split_inter;
  if (tid < 21) {
    const int cb = sad[tid] + A.pen[tid] + Bm.pen[tid];
    int c = A.cost[tid], d = 1;
    if (Bm.cost[tid] < c) {
      c = Bm.cost[tid];
      d = 2;
    }
    if (cb < c) {
      c = cb;
      d = 3;
    }
    cost[tid] = c;
    dirb[tid] = d;
  }
  __syncthreads();
  if (tid < 4) {
    int sum8 = 0;
    for (int r = 0; r < 4; ++r) sum8 += cost[me_blk8_of(tid, r)] + ps;
    const bool split = sum8 < cost[16 + tid] + ps;
    qsplit[tid] = split;
    qsum[tid] = split ? sum8 : cost[16 + tid] + ps;
  }
  __syncthreads();
  if (tid == 0) whole = cost[20] + ps <= qsum[0] + qsum[1] + qsum[2] + qsum[3];
  __syncthreads();
  if (tid < 16) {
    const int k = tid, q = ((k >> 3) << 1) | ((k >> 1) & 1), r = ((k >> 2) & 1) * 2 + (k & 1);
    const int s = whole ? 20 : (qsplit[q] ? me_blk8_of(q, r) : 16 + q), d = dirb[s];
    const long u = b * g.usz + (long)((cy >> 3) + (k >> 2)) * g.w8 + (cx >> 3) + (k & 3);
    dec.cu_log2[u] = (uint8_t)(whole ? 5 : (qsplit[q] ? 3 : 4));
    dec.dir[u] = (uint8_t)d;
    dec.mv[2 * u] = (int16_t)(d & 1 ? mvs[0][s][0] : 0);
    dec.mv[2 * u + 1] = (int16_t)(d & 1 ? mvs[0][s][1] : 0);
    dec.mv1[2 * u] = (int16_t)(d & 2 ? mvs[1][s][0] : 0);
    dec.mv1[2 * u + 1] = (int16_t)(d & 2 ? mvs[1][s][1] : 0);
    dec.intra[u] = 0;
    dec.ipm[u] = 1;
  }
}

// ---------------------------------------------------------------------------------------
// P-frame pass B on matrix cores: every TB of the CTB is coded by 16x16 MFMA tiles.
//
// A P frame has only inter CUs, so all predictions and residuals of the CTB exist up front
// and every transform stage is a batch of small GEMMs.  TBs smaller than 16 are packed
// block-diagonally into one v_mfma 16x16x16 tile: a 16x16 luma quadrant of four 8x8 TBs is
// diag(T8, T8) * R (stage 1) / A * diag(T8, T8)^T (stage 2) — the shared DCT matrix makes the
// four products one MFMA; the Cb and Cr 8x8 regions of a quadrant (one 8x8 TB each, or four
// 4x4 TBs each) form the two diagonal blocks of one tile, diag(Rcb, Rcr).  So a CTB is 8
// tiles per stage (4 luma quadrants + 4 chroma pairs; a single 32x32 CU: 4 K=32 luma tiles +
// 2 chroma tiles) with no VALU dot products at all.  Every operand is an integer of <= 9
// bits (8-bit split halves where needed) so every product and partial sum is exact in f32:
// bit-identical to tv::forward_transform / tv::inverse_transform (see tb_coder.h).
// ---------------------------------------------------------------------------------------
struct PReconLds {
  int16_t T[32][34];          // DCT-32 (every smaller DCT is a row subsample); rows padded to
                              // 17 dwords: column reads across lanes hit distinct banks
  int tmpY[32 * 33];          // stage 1 / stage 3 outputs (luma)
  int tmpC[2][16 * 17];       // stage 1 / stage 3 outputs (Cb, Cr), rows of 17 (bank spread)
  int16_t resY[32 * 32];      // residual, later levels (luma)
  int16_t resC[2][16 * 16];   // residual, later levels (chroma)
  uint8_t predY[32 * 32];
  uint8_t predC[2][16 * 16];
  int mv[16][2];              // per 8x8 unit (raster within the CTB)
  int mv1[16][2];             // B pictures: list-1 vectors and directions
  int dir[16];
  uint8_t bwin[4][15 * 16];   // per wave: 15x15 luma reference window of a bi unit
  int16_t bh[4][15 * 8];      // per wave: horizontal filter pass (15 rows x 8)
  int nz[48], sa[48], dc[48];  // per-TB statistics: luma 0..15, Cb 16..31, Cr 32..47
  int qtype[4];               // luma quadrant: 0 part of a 32x32 CU, 1 16x16 CU, 2 four 8x8 CUs
  int tzero[8];               // stage-3/4 tile t has no surviving level: reconstruction = prediction
  int qsad[4], split;         // RQT: luma residual SAD per quadrant of a 32x32 CU, the decision
  int qsplit[4];              // RQT of the 16x16 CU in quadrant q (four 8x8 TBs)
  int qintra[4];              // quadrant q is an intra CU of a P picture (k_pintra_recon codes it)
  uint32_t ctap[8];           // chroma filter of fraction f as 4 signed bytes
  int cgmax[48];              // RDOQ-lite: highest scan key of a TB's groups that are kept
  int multi;                  // some TB has >= 2 non-zero levels (else RDOQ-lite changes nothing)
};

// block size (log2) of the TB owning luma sample (x, y) / chroma sample (x, y) of the CTB
__device__ __forceinline__ int pr_l2_luma(const PReconLds& L, int x, int y) {
  const int t = L.qtype[(y >> 4) * 2 + (x >> 4)];
  return t == 0 ? 5 : (t == 1 ? 4 : 3);
}
__device__ __forceinline__ int pr_tb_luma(const PReconLds& L, int x, int y) {
  const int q = (y >> 4) * 2 + (x >> 4), t = L.qtype[q];
  return t == 0 ? 0 : (t == 1 ? 4 * q : 4 * q + ((y >> 3) & 1) * 2 + ((x >> 3) & 1));
}
__device__ __forceinline__ int pr_tb_chroma(const PReconLds& L, int p, int x, int y) {
  const int q = (y >> 3) * 2 + (x >> 3), t = L.qtype[q];
  const int base = 16 + 16 * p;
  return t == 0 ? base : (t == 1 ? base + 4 * q : base + 4 * q + ((y >> 2) & 1) * 2 + ((x >> 2) & 1));
}
// block-diagonal composite of DCT blocks of size 2^l2 inside a 16x16 tile: C(r, k)
__device__ __forceinline__ int pr_comp(const PReconLds& L, int l2, int r, int k) {
  return (r >> l2) == (k >> l2) ? (int)L.T[(r & ((1 << l2) - 1)) << (5 - l2)][k & ((1 << l2) - 1)] : 0;
}
// a TB whose only non-zero level is a lone +-1 outside DC is dropped (tv code_tb, inter)
__device__ __forceinline__ bool pr_zeroed(const PReconLds& L, int id) {
  return L.nz[id] == 0 || (L.nz[id] == 1 && L.sa[id] == 1 && L.dc[id] == 0);
}

// WPE: waves per SIMD the register allocation must allow (6: 80 VGPRs; 7: 72, no scratch;
// 8: 64 + a 36-byte spill since the packed prediction) -- TV_RECON_WPE for same-box A/B,
// default 7 (+1.9 % over 8 at 1080p, profiles/r6_recon/).
template <int WPE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) k_inter_recon(FrameSet src, FrameSet ref, const uint8_t* phase,
                                                     FrameSet rec, DecisionSet dec, Geo g, int tile_skip,
                                                     FrameSet ref1, const uint8_t* phase1) {
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int diag = (tile_skip >> 8) & 255;  // TV_DIAG_RECON_STOP (timing only)
  const int rdoq = g.rdoq;                  // RDOQ-lite mode (tv code_tb), 0 off
  tile_skip &= 255;
  int ctu, b;
  xcd_ctb(ctu, b);
  const int qp = dec.qp[b];
  const int cx = (ctu % g.wc) * 32, cy = (ctu / g.wc) * 32;
  const long ub = b * g.usz;
  const int qpc = chroma_qp(qp, 0), Wc = g.W >> 1, Hc = g.H >> 1;
  __shared__ PReconLds L;
  for (int i = tid; i < 1024; i += 256) L.T[i >> 5][i & 31] = (int16_t)kDct32.m[i >> 5][i & 31];
  if (tid < 16) {
    const long u = ub + (long)((cy >> 3) + (tid >> 2)) * g.w8 + (cx >> 3) + (tid & 3);
    L.mv[tid][0] = dec.mv[2 * u];
    L.mv[tid][1] = dec.mv[2 * u + 1];
    L.dir[tid] = dec.dir ? dec.dir[u] : 1;
    L.mv1[tid][0] = dec.mv1 ? dec.mv1[2 * u] : 0;
    L.mv1[tid][1] = dec.mv1 ? dec.mv1[2 * u + 1] : 0;
  }
  if (tid < 48) {
    L.nz[tid] = L.sa[tid] = L.dc[tid] = 0;
    L.cgmax[tid] = -1;
  }
  if (tid < 8)
    L.ctap[tid] = (uint32_t)(uint8_t)kChromaFilter[tid][0] | (uint32_t)(uint8_t)kChromaFilter[tid][1] << 8 |
                  (uint32_t)(uint8_t)kChromaFilter[tid][2] << 16 | (uint32_t)(uint8_t)kChromaFilter[tid][3] << 24;
  if (tid == 0) L.split = 0, L.multi = 0;
  if (tid < 4) {
    L.qsplit[tid] = 0;
    L.qintra[tid] = dec.intra[ub + (long)((cy >> 3) + (tid >> 1) * 2) * g.w8 + (cx >> 3) + (tid & 1) * 2];
  }
  if (tid < 4) {
    const int l2 = dec.cu_log2[ub + (long)((cy >> 3) + (tid >> 1) * 2) * g.w8 + (cx >> 3) + (tid & 1) * 2];
    L.qtype[tid] = l2 == 5 ? 0 : (l2 == 4 ? 1 : 2);
  }
  __syncthreads();
  // ---- prediction + residual of all three planes
  {
    const uint8_t* S = src.plane(0, b, g);
    const uint8_t* ph = phase + (long)b * 16 * g.psz;
    const uint8_t* ph1 = phase1 ? phase1 + (long)b * 16 * g.psz : nullptr;
    {  // uni-prediction: the reference's phase plane holds the final samples; one item = 4
       // samples of a row of one 8x8 unit (a dword of prediction, two int16 residual pairs)
      const int x = (tid & 7) * 4, y = tid >> 3, un = (y >> 3) * 4 + (x >> 3);
      const int d = L.dir[un];
      if (d != 3) {  // bi units: below, one wave per unit
        const int mvx = d == 1 ? L.mv[un][0] : L.mv1[un][0], mvy = d == 1 ? L.mv[un][1] : L.mv1[un][1];
        const uint8_t* P = (d == 1 ? ph : ph1) + (long)((mvx & 3) + 4 * (mvy & 3)) * g.psz;
        const int px = cx + x + (mvx >> 2), py = clip3(-8, g.H + 7, cy + y + (mvy >> 2));
        const uint8_t* row = P + (long)(py + 8) * g.pw16;
        const int bx = px + 8, a4 = bx & ~3;
        uint32_t pw;
        if (bx >= 0 && a4 + 7 < g.pw16) {  // in the padded row: two aligned dwords
          const uint32_t d0 = *reinterpret_cast<const uint32_t*>(row + a4);
          const uint32_t d1 = *reinterpret_cast<const uint32_t*>(row + a4 + 4);
          pw = __builtin_amdgcn_alignbyte(d1, d0, bx & 3);
        } else {
          pw = 0;
#pragma unroll
          for (int k = 0; k < 4; ++k) pw |= (uint32_t)phase_at(P, g, px + k, cy + y + (mvy >> 2)) << (8 * k);
        }
        const uint32_t sw = *reinterpret_cast<const uint32_t*>(S + (long)(cy + y) * g.W + cx + x);
        *reinterpret_cast<uint32_t*>(&L.predY[y * 32 + x]) = pw;
        *reinterpret_cast<uint2*>(&L.resY[y * 32 + x]) = bytes_minus(sw, pw);
      }
    }
    // bi-predicted 8x8 units (8.5.3.3.4.2): per list the 15x15 reference window is staged
    // in this wave's LDS, the 8-tap horizontal pass gives 15 x 8 intermediates, the vertical
    // pass one 14-bit sample per lane; then (p0 + p1 + 64) >> 7.  Wave-local: no barrier.
    for (int un = wave; un < 16; un += 4) {
      if (L.dir[un] != 3) continue;  // wave-uniform
      const int x0 = cx + (un & 3) * 8, y0 = cy + (un >> 2) * 8;
      int pl[2];
      for (int l = 0; l < 2; ++l) {
        const int mvx = l ? L.mv1[un][0] : L.mv[un][0], mvy = l ? L.mv1[un][1] : L.mv[un][1];
        const int fx = mvx & 3, fy = mvy & 3, bx = x0 + (mvx >> 2) - 3, by = y0 + (mvy >> 2) - 3;
        const uint8_t* R = (l ? ref1 : ref).plane(0, b, g);
        uint8_t* win = L.bwin[wave];
        for (int k = lane; k < 225; k += 64) {
          const int r = k / 15, c = k - r * 15;
          win[r * 16 + c] = R[(long)clip3(0, g.H - 1, by + r) * g.W + clip3(0, g.W - 1, bx + c)];
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        int16_t* hb = L.bh[wave];
        for (int k = lane; k < 120; k += 64) {
          const int r = k >> 3, c = k & 7;
          int h;
          if (fx) {
            h = 0;
#pragma unroll
            for (int t = 0; t < 8; ++t) h += kLumaFilter[fx][t] * win[r * 16 + c + t];
          } else {
            h = win[r * 16 + c + 3] << 6;
          }
          hb[k] = (int16_t)h;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int xo = lane & 7, yo = lane >> 3;
        if (fy) {
          int v = 0;
#pragma unroll
          for (int t = 0; t < 8; ++t) v += kLumaFilter[fy][t] * hb[(yo + t) * 8 + xo];
          pl[l] = v >> 6;
        } else {
          pl[l] = hb[(yo + 3) * 8 + xo];
        }
        __builtin_amdgcn_wave_barrier();  // the window / pass buffers are reused by list 1
      }
      const int x = (un & 3) * 8 + (lane & 7), y = (un >> 2) * 8 + (lane >> 3);
      const int p = bipred_sample(pl[0], pl[1]);
      L.predY[y * 32 + x] = (uint8_t)p;
      L.resY[y * 32 + x] = (int16_t)((int)S[(long)(cy + y) * g.W + cx + x] - p);
    }
    // chroma: one item = 4 samples of a row of one 4x4 unit (128 items), the separable 4-tap
    // filter on packed bytes: per reference row the 7 samples are two dwords, each output a
    // v_dot4 of a v_alignbyte window against the biased taps (samples ^ 0x80 as int8: the
    // bias is 128 * 64 = 8192), then the vertical taps.  The 0-fraction filter {0, 64, 0, 0}
    // makes the one 2-D formula exact for every fraction (8.5.3.3.3.2, as mc_chroma_inter).
    if (tid < 128) {
      const int pl = tid >> 6, y = (tid >> 2) & 15, x = (tid & 3) * 4, un = (y >> 2) * 4 + (x >> 2);
      const int d = L.dir[un];
      const int gx = (cx >> 1) + x, gy = (cy >> 1) + y;
      int prev[4] = {0, 0, 0, 0};  // bi: the list-0 intermediates
      uint32_t pw = 0;
#pragma unroll 1
      for (int l = 0; l < 2; ++l) {
        if (!(d & (1 << l))) continue;
        const int mvx = l ? L.mv1[un][0] : L.mv[un][0], mvy = l ? L.mv1[un][1] : L.mv[un][1];
        const uint8_t* Rf = (l ? ref1 : ref).plane(1 + pl, b, g);
        const uint32_t tx = L.ctap[mvx & 7], ty = L.ctap[mvy & 7];
        const int x0 = gx + (mvx >> 3) - 1, y0 = gy + (mvy >> 3) - 1;
        int acc[4] = {0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint8_t* row = Rf + (long)clip3(0, Hc - 1, y0 + j) * Wc;
          const int a4 = x0 & ~3;
          uint32_t w0, w1;
          if (x0 >= 0 && a4 + 11 < Wc) {
            const uint32_t d0 = *reinterpret_cast<const uint32_t*>(row + a4);
            const uint32_t d1 = *reinterpret_cast<const uint32_t*>(row + a4 + 4);
            const uint32_t d2 = *reinterpret_cast<const uint32_t*>(row + a4 + 8);
            w0 = __builtin_amdgcn_alignbyte(d1, d0, x0 & 3);
            w1 = __builtin_amdgcn_alignbyte(d2, d1, x0 & 3);
          } else {
            w0 = w1 = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              w0 |= (uint32_t)row[clip3(0, Wc - 1, x0 + k)] << (8 * k);
              w1 |= (uint32_t)row[clip3(0, Wc - 1, x0 + 4 + k)] << (8 * k);
            }
          }
          w0 ^= 0x80808080u;
          w1 ^= 0x80808080u;
          const int fyj = (int)(int8_t)(ty >> (8 * j));
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const uint32_t win = k == 0 ? w0 : __builtin_amdgcn_alignbyte(w1, w0, k);
            acc[k] += fyj * __builtin_amdgcn_sdot4((int)win, (int)tx, 8192, false);
          }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int v = acc[k] >> 6;  // the 14-bit intermediate
          if (d == 3 && l == 0) {
            prev[k] = v;
          } else {
            const int p = d == 3 ? bipred_sample(prev[k], v) : clip_pixel((v + 32) >> 6);
            pw |= (uint32_t)p << (8 * k);
          }
        }
      }
      const uint32_t sw = *reinterpret_cast<const uint32_t*>(src.plane(1 + pl, b, g) + (long)gy * Wc + gx);
      *reinterpret_cast<uint32_t*>(&L.predC[pl][y * 16 + x]) = pw;
      *reinterpret_cast<uint2*>(&L.resC[pl][y * 16 + x]) = bytes_minus(sw, pw);
    }
  }
  __syncthreads();
  if (dec.tu) {  // RQT (P pictures): a 32x32 CU may code four 16x16 TBs (hevc_defs.h rqt_split)
    if (L.qtype[0] == 0) {  // workgroup-uniform
      const int qx = (wave & 1) * 16, qy = (wave >> 1) * 16;
      int d = 0;
      for (int k = lane; k < 256; k += 64) d += tv_abs((int)L.resY[(qy + (k >> 4)) * 32 + qx + (k & 15)]);
      d = wave_sum(d);
      if (lane == 0) L.qsad[wave] = d;
      __syncthreads();
      if (tid == 0 && rqt_split(L.qsad)) {
        L.split = 1;
        L.qtype[0] = L.qtype[1] = L.qtype[2] = L.qtype[3] = 1;  // the 16x16-CU tile layout
      }
      __syncthreads();
    } else if (kRqtMinLog2 <= 4) {  // 16x16 CUs: quadrant `wave`'s four 8x8 SADs, four 8x8 TBs on a split
      if (L.qtype[wave] == 1 && !L.qintra[wave]) {  // wave-uniform
        const int qx = (wave & 1) * 16, qy = (wave >> 1) * 16;
        int s4[4];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          s4[k] = wave_sum(tv_abs((int)L.resY[(qy + (k >> 1) * 8 + (lane >> 3)) * 32 + qx + (k & 1) * 8 + (lane & 7)]));
        if (lane == 0 && rqt_split(s4, 64)) L.qsplit[wave] = 1;
      }
      __syncthreads();
      if (tid < 4 && L.qsplit[tid]) L.qtype[tid] = 2;  // the 8x8-CU tile layout
      __syncthreads();
    }
    if (tid < 16)
      dec.tu[ub + (long)((cy >> 3) + (tid >> 2)) * g.w8 + (cx >> 3) + (tid & 3)] =
          (uint8_t)(L.split | L.qsplit[((tid >> 3) << 1) | ((tid >> 1) & 1)]);
  }
  const bool whole = L.qtype[0] == 0;
  const int ntiles = whole ? 6 : 8;
  // tile t: luma (whole: 32x32 tile ti,tj = t>>1, t&1; else quadrant t) for t < 4, chroma
  // (whole: plane t-4 as one 16x16 TB; else the Cb|Cr pair of quadrant t-4) for t >= 4.
  // ---------------------------------------------------------------- stage 1: T * R
  // (diag 1: no forward transform -- every TB counts as empty, the stream stays consistent)
  for (int t = wave; t < (diag == 1 ? 0 : ntiles); t += 4) {
    int o[4];
    if (t < 4) {
      if (whole) {
        mfma_tile([&](int r, int k) { return (int)L.T[r][k]; }, [&](int k, int c) { return (int)L.resY[k * 32 + c]; },
                  t >> 1, t & 1, 32, false, false, o);
      } else {
        const int ox = (t & 1) * 16, oy = (t >> 1) * 16, l2 = L.qtype[t] == 1 ? 4 : 3;
        mfma_tile([&](int r, int k) { return pr_comp(L, l2, r, k); },
                  [&](int k, int c) { return (int)L.resY[(oy + k) * 32 + ox + c]; }, 0, 0, 16, false, false, o);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = (lane >> 4) * 4 + r, cc = lane & 15;
        const int y = whole ? 16 * (t >> 1) + rr : (t >> 1) * 16 + rr, x = whole ? 16 * (t & 1) + cc : (t & 1) * 16 + cc;
        const int sh1 = pr_l2_luma(L, x, y) - 1;
        L.tmpY[y * 33 + x] = (o[r] + (1 << (sh1 - 1))) >> sh1;
      }
    } else if (whole) {
      const int pl = t - 4;
      mfma_tile([&](int r, int k) { return pr_comp(L, 4, r, k); }, [&](int k, int c) { return (int)L.resC[pl][k * 16 + c]; },
                0, 0, 16, false, false, o);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = (lane >> 4) * 4 + r, cc = lane & 15;
        L.tmpC[pl][rr * 17 + cc] = (o[r] + 4) >> 3;  // 16-point: sh1 = 3
      }
    } else {
      const int q = t - 4, ox = (q & 1) * 8, oy = (q >> 1) * 8, l2 = L.qtype[q] == 1 ? 3 : 2;
      mfma_tile([&](int r, int k) { return pr_comp(L, l2, r, k); },
                [&](int k, int c) {
                  return (k >> 3) == (c >> 3) ? (int)L.resC[k >> 3][(oy + (k & 7)) * 16 + ox + (c & 7)] : 0;
                },
                0, 0, 16, false, false, o);
      const int sh1 = l2 - 1;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = (lane >> 4) * 4 + r, cc = lane & 15;
        if ((rr >> 3) == (cc >> 3)) L.tmpC[rr >> 3][(oy + (rr & 7)) * 17 + ox + (cc & 7)] = (o[r] + (1 << (sh1 - 1))) >> sh1;
      }
    }
  }
  __syncthreads();
  // ------------------------------------------------- stage 2: A * T^T + quantisation
  auto emit_level = [&](int16_t* dst, int id, int l2, int q, int v, bool origin) {
    const int sh2 = l2 + 6;
    const int lev = quant_level((v + (1 << (sh2 - 1))) >> sh2, q, l2, false);
    *dst = (int16_t)lev;
    if (lev) {
      if (atomicAdd(&L.nz[id], 1)) L.multi = 1;
      atomicAdd(&L.sa[id], tv_abs(lev));
    }
    if (origin) L.dc[id] = lev;
  };
  for (int t = wave; t < (diag == 1 ? 0 : ntiles); t += 4) {
    int o[4];
    if (t < 4) {
      if (whole) {
        mfma_tile([&](int r, int k) { return L.tmpY[r * 33 + k]; }, [&](int k, int c) { return (int)L.T[c][k]; },
                  t >> 1, t & 1, 32, true, true, o);
      } else {
        const int ox = (t & 1) * 16, oy = (t >> 1) * 16, l2 = L.qtype[t] == 1 ? 4 : 3;
        mfma_tile([&](int r, int k) { return L.tmpY[(oy + r) * 33 + ox + k]; },
                  [&](int k, int c) { return pr_comp(L, l2, c, k); }, 0, 0, 16, true, true, o);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = (lane >> 4) * 4 + r, cc = lane & 15;
        const int y = (t >> 1) * 16 + rr, x = (t & 1) * 16 + cc;
        const int l2 = pr_l2_luma(L, x, y), m = (1 << l2) - 1;
        emit_level(&L.resY[y * 32 + x], pr_tb_luma(L, x, y), l2, qp, o[r], (x & m) == 0 && (y & m) == 0);
      }
    } else if (whole) {
      const int pl = t - 4;
      mfma_tile([&](int r, int k) { return L.tmpC[pl][r * 17 + k]; }, [&](int k, int c) { return pr_comp(L, 4, c, k); },
                0, 0, 16, true, true, o);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = (lane >> 4) * 4 + r, cc = lane & 15;
        emit_level(&L.resC[pl][rr * 16 + cc], 16 + 16 * pl, 4, qpc, o[r], rr == 0 && cc == 0);
      }
    } else {
      const int q = t - 4, ox = (q & 1) * 8, oy = (q >> 1) * 8, l2 = L.qtype[q] == 1 ? 3 : 2;
      mfma_tile([&](int r, int k) {
                  return (r >> 3) == (k >> 3) ? L.tmpC[r >> 3][(oy + (r & 7)) * 17 + ox + (k & 7)] : 0;
                },
                [&](int k, int c) { return pr_comp(L, l2, c, k); }, 0, 0, 16, true, true, o);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = (lane >> 4) * 4 + r, cc = lane & 15;
        if ((rr >> 3) != (cc >> 3)) continue;
        const int pl = rr >> 3, x = ox + (cc & 7), y = oy + (rr & 7), m = (1 << l2) - 1;
        emit_level(&L.resC[pl][y * 16 + x], pr_tb_chroma(L, pl, x, y), l2, qpc, o[r], (x & m) == 0 && (y & m) == 0);
      }
    }
  }
  __syncthreads();
  // ---- RDOQ-lite (tv code_tb, inter TBs of 8x8 and up): trailing coefficient groups whose
  // only level is a lone +-1 are dropped -- tv walks the TB's groups in reverse up-right
  // diagonal scan to the first group holding anything else, down to diagonal rdoq_dmin.  In
  // parallel that is: a lone group is dropped iff its scan key (diagonal major, then rows
  // from the bottom) is above every other non-empty-non-lone group's of its TB (one LDS max
  // per TB) and its diagonal is >= rdoq_dmin.  One thread per 4x4 group (luma 64, Cb / Cr 16).
  // A CTB whose TBs hold at most one level each skips it (workgroup-uniform): a lone level
  // the pass could drop is dropped by the whole-TB rule (pr_zeroed) anyway.
  if (diag != 1 && rdoq && L.multi) {
    int code = 0, key = 0, id = 0, dmin = 1 << 20;
    int16_t* p = nullptr;
    int st = 32;
    if (tid < 96) {
      int x, y, l2, pl = -1;
      if (tid < 64) {
        x = (tid & 7) * 4, y = (tid >> 3) * 4;
        l2 = pr_l2_luma(L, x, y);
        id = pr_tb_luma(L, x, y);
        p = &L.resY[y * 32 + x];
      } else {
        const int c = tid - 64;
        pl = c >> 4, x = (c & 3) * 4, y = ((c & 15) >> 2) * 4;
        l2 = pr_l2_luma(L, 2 * x, 2 * y) - 1;
        id = pr_tb_chroma(L, pl, x, y);
        p = &L.resC[pl][y * 16 + x];
        st = 16;
      }
      int t = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint2 w = *reinterpret_cast<const uint2*>(p + j * st);
        t += tv_abs((int)(int16_t)(w.x & 0xffff)) + tv_abs((int)(int16_t)(w.x >> 16)) + tv_abs((int)(int16_t)(w.y & 0xffff)) +
             tv_abs((int)(int16_t)(w.y >> 16));
      }
      const int m = (1 << l2) - 1, gx = (x & m) >> 2, gy = (y & m) >> 2;
      code = tv_min(t, 2);
      key = (gx + gy) * 16 + 15 - gy;
      const int q = pl < 0 ? (y >> 4) * 2 + (x >> 4) : (y >> 3) * 2 + (x >> 3);
      if (l2 >= 3 && !L.qintra[L.qtype[0] == 0 ? 0 : q]) dmin = rdoq_dmin(rdoq, 1 << (l2 - 2));
      if (code == 2) atomicMax(&L.cgmax[id], key);
      if (gx + gy < dmin) code = 0;  // groups this TB keeps whatever they hold
    }
    // all groups of a TB are in one wave (luma wave 0, chroma wave 1) and one wave's LDS
    // operations execute in order: the max needs no workgroup barrier before it is read
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (code == 1 && key > L.cgmax[id]) {
#pragma unroll
      for (int j = 0; j < 4; ++j) *reinterpret_cast<uint2*>(p + j * st) = make_uint2(0u, 0u);
      atomicSub(&L.nz[id], 1);
      atomicSub(&L.sa[id], 1);
    }
    __syncthreads();
  }
  // ---- final levels (dropped TBs zeroed) -> the level planes; cbf per CU
  {
    // 4 levels (one TB: TBs are >= 4 wide and 4-aligned) per item, one 8-byte store
    int16_t* LY = dec.coef_y + b * g.ysz + (long)cy * g.W + cx;
    {
      const int x = (tid & 7) * 4, y = tid >> 3;
      uint2* r = reinterpret_cast<uint2*>(&L.resY[y * 32 + x]);
      if (pr_zeroed(L, pr_tb_luma(L, x, y))) *r = make_uint2(0u, 0u);
      *reinterpret_cast<uint2*>(LY + (long)y * g.W + x) = *r;
    }
    if (tid < 128) {
      const int pl = tid >> 6, y = (tid >> 2) & 15, x = (tid & 3) * 4;
      uint2* r = reinterpret_cast<uint2*>(&L.resC[pl][y * 16 + x]);
      if (pr_zeroed(L, pr_tb_chroma(L, pl, x, y))) *r = make_uint2(0u, 0u);
      *reinterpret_cast<uint2*>((pl ? dec.coef_v : dec.coef_u) + b * g.csz + (long)((cy >> 1) + y) * Wc + (cx >> 1) + x) = *r;
    }
    if (tid < 8) {  // tiles whose TBs all dropped out skip the inverse transform
      bool z = true;
      if (tid < 4) {
        if (L.qtype[0] == 0) z = pr_zeroed(L, 0);
        else for (int k = 0; k < 4; ++k) z = z && pr_zeroed(L, pr_tb_luma(L, (tid & 1) * 16 + (k & 1) * 8, (tid >> 1) * 16 + (k >> 1) * 8));
      } else if (L.qtype[0] == 0) {
        z = pr_zeroed(L, 16 + 16 * (tid - 4));
      } else {
        const int q = tid - 4;  // Cb | Cr pair of quadrant q (Cb and Cr 8x8 regions)
        for (int pl = 0; pl < 2; ++pl)
          for (int k = 0; k < 4; ++k) z = z && pr_zeroed(L, pr_tb_chroma(L, pl, (q & 1) * 8 + (k & 1) * 4, (q >> 1) * 8 + (k >> 1) * 4));
      }
      L.tzero[tid] = z && tile_skip;
    }
    if (tid < 16) {
      const int x = (tid & 3) * 8, y = (tid >> 2) * 8;  // this unit's CU = its TBs
      const int cb = (pr_zeroed(L, pr_tb_luma(L, x, y)) ? 0 : 1) | (pr_zeroed(L, pr_tb_chroma(L, 0, x >> 1, y >> 1)) ? 0 : 2) |
                     (pr_zeroed(L, pr_tb_chroma(L, 1, x >> 1, y >> 1)) ? 0 : 4);
      dec.cbf[ub + (long)((cy >> 3) + (tid >> 2)) * g.w8 + (cx >> 3) + (tid & 3)] = (uint8_t)cb;
    }
  }
  __syncthreads();
  if (diag == 3) return;
  // --------------------------------------- stage 3: T^T * dequant(levels)  (split d)
  const DeqParams dq5 = deq_params(qp, 5), dqc4 = deq_params(qpc, 4);
  for (int t = wave; t < ntiles; t += 4) {
    if (L.tzero[t]) continue;  // wave-uniform: an all-zero tile reconstructs to the prediction
    int o[4];
    if (t < 4) {
      if (whole) {
        mfma_tile([&](int r, int k) { return (int)L.T[k][r]; },
                  [&](int k, int c) { return deq_fast(L.resY[k * 32 + c], dq5); }, t >> 1, t & 1, 32, true, false, o);
      } else {
        const int ox = (t & 1) * 16, oy = (t >> 1) * 16, l2 = L.qtype[t] == 1 ? 4 : 3;
        const DeqParams dql = deq_params(qp, l2);
        mfma_tile([&](int r, int k) { return pr_comp(L, l2, k, r); },
                  [&](int k, int c) { return deq_fast(L.resY[(oy + k) * 32 + ox + c], dql); }, 0, 0, 16, true, false, o);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int y = (t >> 1) * 16 + (lane >> 4) * 4 + r, x = (t & 1) * 16 + (lane & 15);
        L.tmpY[y * 33 + x] = clip3(-32768, 32767, (o[r] + 64) >> 7);
      }
    } else if (whole) {
      const int pl = t - 4;
      mfma_tile([&](int r, int k) { return pr_comp(L, 4, k, r); },
                [&](int k, int c) { return deq_fast(L.resC[pl][k * 16 + c], dqc4); }, 0, 0, 16, true, false, o);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        L.tmpC[pl][((lane >> 4) * 4 + r) * 17 + (lane & 15)] = clip3(-32768, 32767, (o[r] + 64) >> 7);
    } else {
      const int q = t - 4, ox = (q & 1) * 8, oy = (q >> 1) * 8, l2 = L.qtype[q] == 1 ? 3 : 2;
      const DeqParams dqcl = deq_params(qpc, l2);
      mfma_tile([&](int r, int k) { return pr_comp(L, l2, k, r); },
                [&](int k, int c) {
                  return (k >> 3) == (c >> 3) ? deq_fast(L.resC[k >> 3][(oy + (k & 7)) * 16 + ox + (c & 7)], dqcl) : 0;
                },
                0, 0, 16, true, false, o);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = (lane >> 4) * 4 + r, cc = lane & 15;
        if ((rr >> 3) == (cc >> 3))
          L.tmpC[rr >> 3][(oy + (rr & 7)) * 17 + ox + (cc & 7)] = clip3(-32768, 32767, (o[r] + 64) >> 7);
      }
    }
  }
  __syncthreads();
  if (diag == 4) return;
  // ------------------------------------- stage 4: G * T + prediction -> reconstruction
  for (int t = wave; t < ntiles; t += 4) {
    int o[4];
    const bool tz = L.tzero[t];
    if (tz) {  // copy the prediction (what clip(pred + 0) gives)
      o[0] = o[1] = o[2] = o[3] = 0;
    }
    if (t < 4) {
      if (whole) {
        if (!tz) mfma_tile([&](int r, int k) { return L.tmpY[r * 33 + k]; }, [&](int k, int c) { return (int)L.T[k][c]; },
                  t >> 1, t & 1, 32, true, true, o);
      } else {
        const int ox = (t & 1) * 16, oy = (t >> 1) * 16, l2 = L.qtype[t] == 1 ? 4 : 3;
        if (!tz) mfma_tile([&](int r, int k) { return L.tmpY[(oy + r) * 33 + ox + k]; },
                  [&](int k, int c) { return pr_comp(L, l2, k, c); }, 0, 0, 16, true, true, o);
      }
      uint8_t* R = rec.plane(0, b, g) + (long)cy * g.W + cx;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int y = (t >> 1) * 16 + (lane >> 4) * 4 + r, x = (t & 1) * 16 + (lane & 15);
        R[(long)y * g.W + x] = (uint8_t)clip_pixel((int)L.predY[y * 32 + x] + ((o[r] + 2048) >> 12));
      }
    } else if (whole) {
      const int pl = t - 4;
      if (!tz) mfma_tile([&](int r, int k) { return L.tmpC[pl][r * 17 + k]; }, [&](int k, int c) { return pr_comp(L, 4, k, c); },
                0, 0, 16, true, true, o);
      uint8_t* R = rec.plane(1 + pl, b, g) + (long)(cy >> 1) * Wc + (cx >> 1);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int y = (lane >> 4) * 4 + r, x = lane & 15;
        R[(long)y * Wc + x] = (uint8_t)clip_pixel((int)L.predC[pl][y * 16 + x] + ((o[r] + 2048) >> 12));
      }
    } else {
      const int q = t - 4, ox = (q & 1) * 8, oy = (q >> 1) * 8, l2 = L.qtype[q] == 1 ? 3 : 2;
      if (!tz) mfma_tile([&](int r, int k) {
                  return (r >> 3) == (k >> 3) ? L.tmpC[r >> 3][(oy + (r & 7)) * 17 + ox + (k & 7)] : 0;
                },
                [&](int k, int c) { return pr_comp(L, l2, k, c); }, 0, 0, 16, true, true, o);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int rr = (lane >> 4) * 4 + r, cc = lane & 15;
        if ((rr >> 3) != (cc >> 3)) continue;
        const int pl = rr >> 3, x = ox + (cc & 7), y = oy + (rr & 7);
        rec.plane(1 + pl, b, g)[(long)((cy >> 1) + y) * Wc + (cx >> 1) + x] =
            (uint8_t)clip_pixel((int)L.predC[pl][y * 16 + x] + ((o[r] + 2048) >> 12));
      }
    }
  }
}

void launch_quarter(FrameSet src, uint8_t* q, const Geo& g, int B, hipStream_t s) {
  const int n = (g.W >> 2) * (g.H >> 2);
  k_quarter<<<dim3((n + 255) / 256, B), 256, 0, s>>>(src, q, g);
}

void launch_coarse_me(const MeBuffers& me, const Geo& g, const RcTables* rc, int seq_qp, int range, int B,
                      hipStream_t s) {
  const int rq = range / 4;
  if (rq > kCoarseMaxRq) throw std::runtime_error("coarse search range too large");
  const size_t lds = sizeof(uint32_t) * (size_t)(8 + 2 * rq) * (size_t)((rq / 2 + 3) | 1);  // the window only
  k_coarse_me<<<dim3(g.wc * g.hc, B), 64, lds, s>>>(me.qcur, me.qprev, g, rc, seq_qp, rq, me.cmv, me.ccost);
}

// CRF (tv/rc_model.h): the frame QP of every segment from its lookahead complexity — the
// summed coarse-search cost (P) or the quarter-res activity (IDR) — written into dec.qp
__global__ void __launch_bounds__(256) k_rc_crf(const uint8_t* q, const int* ccost, int8_t* qp, Geo g, int crf,
                                                int intra) {
  const int b = blockIdx.x, nctu = g.wc * g.hc, qw = g.W >> 2;
  __shared__ unsigned long long sum;
  if (threadIdx.x == 0) sum = 0;
  __syncthreads();
  unsigned long long acc = 0;
  for (int c = threadIdx.x; c < nctu; c += 256) {
    if (intra) {
      const uint8_t* Q = q + (long)b * qw * (g.H >> 2) + (long)(8 * (c / g.wc)) * qw + 8 * (c % g.wc);
      acc += rc_block_activity(Q, qw);
    } else {
      acc += (unsigned long long)ccost[(long)b * nctu + c];
    }
  }
  atomicAdd(&sum, acc);
  __syncthreads();
  if (threadIdx.x == 0) qp[b] = (int8_t)rc_crf_qp(crf, intra != 0, sum, nctu);
}

void launch_rc_crf(const uint8_t* q, const int* ccost, int8_t* qp, const Geo& g, int crf, bool intra, int B,
                   hipStream_t s) {
  k_rc_crf<<<B, 256, 0, s>>>(q, ccost, qp, g, crf, intra ? 1 : 0);
}

// TV_RECON_TILE_SKIP=0 runs the inverse transform on all-zero tiles too (same output; kept
// as a same-box A/B switch for the skip)
static int recon_tile_skip() {
  static const int v = [] {
    const char* e = std::getenv("TV_RECON_TILE_SKIP");
    // timing diagnostics only (TV_DIAG_RECON_STOP=1: no forward transform (all TBs empty), 3:
    // stop after the level write, 4: after inverse stage 1; the reconstruction is then
    // incomplete) -- never in production
    const char* d = std::getenv("TV_DIAG_RECON_STOP");
    return (e ? std::atoi(e) : 1) | (d ? (std::atoi(d) & 15) << 8 : 0);
  }();
  return v;
}

using ReconKernel = decltype(&k_inter_recon<7>);
static ReconKernel recon_kernel() {
  static const ReconKernel k = [] {
    const char* e = std::getenv("TV_RECON_WPE");
    const int w = e ? std::atoi(e) : 7;
    return w == 6 ? &k_inter_recon<6> : (w == 8 ? &k_inter_recon<8> : &k_inter_recon<7>);
  }();
  return k;
}

// Variants for same-box A/B measurements (same decisions): TV_ME_SUBPEL_ROWS=4 (768 sub-pel
// groups), TV_ME_PEN=global (MV-rate table read from global memory), TV_ME_WPE=7 (the
// compiler's register allocation: 7 CTBs per CU).
using MeKernel = decltype(&k_inter_me<8, true, 8>);
static MeKernel me_kernel() {
  static const MeKernel k = [] {
    const char* r = std::getenv("TV_ME_SUBPEL_ROWS");
    const char* p = std::getenv("TV_ME_PEN");
    const char* w = std::getenv("TV_ME_WPE");
    const bool rows4 = r && std::atoi(r) == 4, glob = p && std::string(p) == "global", w7 = w && std::atoi(w) == 7;
    if (rows4) return glob ? &k_inter_me<4, false, 8> : &k_inter_me<4, true, 8>;
    if (w7) return glob ? &k_inter_me<8, false, 7> : &k_inter_me<8, true, 7>;
    return glob ? &k_inter_me<8, false, 8> : &k_inter_me<8, true, 8>;
  }();
  return k;
}

void launch_inter_frame(FrameSet src, FrameSet ref, const uint8_t* phase, FrameSet rec, DecisionSet dec,
                        const Geo& g, const RcTables* rc, int range, const MeBuffers& me, int B, hipStream_t s,
                        const PIntraBuffers* pi) {
  static const int diag_stop = [] {
    const char* e = std::getenv("TV_DIAG_ME_STOP");
    const char* c = std::getenv("TV_ME_CAND");
    return (e ? std::atoi(e) : 0) | (c && std::string(c) == "global" ? 16 : 0);
  }();
  const PIntraBuffers none{};
  if (pi && hipMemsetAsync(pi->count, 0, 6 * sizeof(int), s) != hipSuccess) return;
  me_kernel()<<<dim3(g.wc * g.hc, B), kMeThreads, 0, s>>>(src, ref, phase, dec, me.prev_mv, me.cmv, g, rc, range,
                                                         diag_stop, nullptr, pi ? *pi : none);
  if (pi) launch_pintra_decide(src, dec, g, rc, *pi, B, s);
  recon_kernel()<<<dim3(g.wc * g.hc, B), 256, 0, s>>>(src, ref, phase, rec, dec, g, recon_tile_skip(), FrameSet{},
                                                     nullptr);
  if (pi) launch_pintra_recon(src, rec, dec, g, *pi, B, s);
}

void launch_inter_frame_b(FrameSet src, FrameSet ref0, const uint8_t* phase0, FrameSet ref1, const uint8_t* phase1,
                          FrameSet rec, DecisionSet dec, const Geo& g, const RcTables* rc, const int* range,
                          const MeBuffers& me0, const MeBuffers& me1, CtbMeOut* meout, int B, hipStream_t s) {
  const dim3 grid(g.wc * g.hc, B);
  CtbMeOut* o1 = meout + (long)B * g.wc * g.hc;
  const PIntraBuffers none{};
  me_kernel()<<<grid, kMeThreads, 0, s>>>(src, ref0, phase0, dec, me0.prev_mv, me0.cmv, g, rc, range[0], 0, meout, none);
  me_kernel()<<<grid, kMeThreads, 0, s>>>(src, ref1, phase1, dec, me1.prev_mv, me1.cmv, g, rc, range[1], 0, o1, none);
  k_bi_decide<<<grid, 256, 0, s>>>(src, phase0, phase1, meout, o1, dec, g, rc);
  recon_kernel()<<<grid, 256, 0, s>>>(src, ref0, phase0, rec, dec, g, recon_tile_skip(), ref1, phase1);
}

}  // namespace gpu
}  // namespace tv
