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
#include "gpu_common.h"
#include "k_encode.h"
#include "tb_coder.h"
#include "wave_tb.h"
#include "tv/me_model.h"

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
constexpr int kMeThreads = 128;
constexpr int kFRows = kCtb + kMeWinH - 1;  // 38 window rows per candidate
constexpr int kFWords = 10;                 // 40 bytes: 32 + 7 offsets + 1 spare word
constexpr int kFPitch = kFWords + 1;        // odd pitch: lanes walking rows hit distinct banks
// LDS pitch (words) of a source-CTB row (uniform s0/s1 reads stay one aligned 8-byte read)
constexpr int kSrcP = 8;

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

__global__ void __launch_bounds__(64) k_coarse_me(const uint8_t* qcur, const uint8_t* qprev, Geo g, Penalties pen,
                                                  int rq, int16_t* cmv, int* ccost) {
  const int ctu = blockIdx.x, b = blockIdx.y, lane = threadIdx.x;
  const int qw = g.W >> 2, qh = g.H >> 2;
  const int x0 = 8 * (ctu % g.wc), y0 = 8 * (ctu / g.wc);
  const uint8_t* C = qcur + (long)b * qw * qh;
  const uint8_t* P = qprev + (long)b * qw * qh;
  __shared__ uint32_t s32[16];
  __shared__ uint32_t win[kCoarseRows * (kCoarseWords | 1)];
  const int side = 2 * rq + 1, rows = 8 + 2 * rq, wpr = rq / 2 + 3, pitch = wpr | 1;
  if (lane < 16) s32[lane] = *reinterpret_cast<const uint32_t*>(C + (long)(y0 + (lane >> 1)) * qw + x0 + 4 * (lane & 1));
  for (int w = lane; w < rows * wpr; w += 64) {
    const int r = w / wpr, c = w - r * wpr;
    const uint8_t* row = P + (long)clip3(0, qh - 1, y0 - rq + r) * qw;
    win[r * pitch + c] = load4_clamped(row, x0 - rq + 4 * c, qw);
  }
  __syncthreads();
  unsigned best = 0xffffffffu;
  const int groups = rq / 2 + 1;
  for (int item = lane; item < groups * side; item += 64) {
    const int gi = item / side, dyi = item - gi * side;
    const int dy = dyi - rq, dx0 = 4 * gi - rq;
    unsigned acc[4] = {0, 0, 0, 0};
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t s0 = s32[2 * j], s1 = s32[2 * j + 1];
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
      const unsigned v = ((acc[sft] + (unsigned)me_coarse_pen(pen.mv, dx, dy)) << 13) | (unsigned)(dyi * side + dx + rq);
      best = v < best ? v : best;
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

__global__ void __launch_bounds__(kMeThreads) k_inter_me(FrameSet src, FrameSet ref, const uint8_t* phase,
                                                         DecisionSet dec, const int16_t* prev_mv, const int16_t* cmv,
                                                         Geo g, Penalties pen, int range) {
  const int ctu = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int cxi = ctu % g.wc, cyi = ctu / g.wc, cx = cxi * 32, cy = cyi * 32;
  const uint8_t* S = src.plane(0, b, g);
  const uint8_t* R = ref.plane(0, b, g);
  __shared__ uint32_t s32[32 * kSrcP];
  __shared__ uint32_t win[kMeMaxCand * kFRows * kFPitch];
  __shared__ int cand[kMeMaxCand][2];
  __shared__ int pmv[2], ncand;
  __shared__ unsigned best[21];
  __shared__ int bcost[21], bmv[21][2];
  __shared__ int subsad[21][8];
  for (int t = tid; t < 256; t += kMeThreads)
    s32[(t >> 3) * kSrcP + (t & 7)] = *reinterpret_cast<const uint32_t*>(S + (long)(cy + (t >> 3)) * g.W + cx + 4 * (t & 7));
  if (tid == 0) {
    const long u0 = b * g.usz + (long)(cy >> 3) * g.w8 + (cx >> 3);
    ncand = me_candidates(cmv + (long)b * g.wc * g.hc * 2, g.wc, g.hc, cxi, cyi, prev_mv[2 * u0], prev_mv[2 * u0 + 1],
                          range - 4, cand, pmv);
  }
  if (tid < 21) best[tid] = 0xffffffffu;
  __syncthreads();
  const int nc = ncand;
  // candidate windows, each pre-aligned so byte 0 of a row is x = cx + cand_x + kMeWinX0
  for (int e = tid; e < nc * kFRows * kFWords; e += kMeThreads) {
    const int k = e / (kFRows * kFWords), rem = e - k * (kFRows * kFWords);
    const int r = rem / kFWords, w = rem - r * kFWords;
    const uint8_t* row = R + (long)clip3(0, g.H - 1, cy + cand[k][1] + kMeWinY0 + r) * g.W;
    win[(k * kFRows + r) * kFPitch + w] = load4_clamped(row, cx + cand[k][0] + kMeWinX0 + 4 * w, g.W);
  }
  __syncthreads();

  // ------------------------------- integer refinement -----------------------------------
  unsigned lb[21];
#pragma unroll
  for (int k = 0; k < 21; ++k) lb[k] = 0xffffffffu;
  for (int item = tid; item < nc * kMeWinH * 2; item += kMeThreads) {
    const int k = item / (kMeWinH * 2), rr = item - k * (kMeWinH * 2);
    const int dyi = rr >> 1, gs = rr & 1;
    const int pos0 = k * kMePosPerCand + dyi * kMeWinW + 4 * gs;
    const int my = cand[k][1] + kMeWinY0 + dyi;
    unsigned mvc[4];
#pragma unroll
    for (int sft = 0; sft < 4; ++sft) {
      const int mx = cand[k][0] + kMeWinX0 + 4 * gs + sft;
      mvc[sft] = (unsigned)pen.mv[me_pen_index(4 * mx - pmv[0], 4 * my - pmv[1])];
    }
    const uint32_t* W0 = win + (k * kFRows + dyi) * kFPitch + gs;
    unsigned q16[4][4], t32[4];
#pragma unroll
    for (int sft = 0; sft < 4; ++sft) {
      t32[sft] = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) q16[q][sft] = 0;
    }
#pragma unroll
    for (int kb = 0; kb < 16; ++kb) {
      const int bx = (kb & 3) * 8, by = (kb >> 2) * 8;
      const int q = ((kb >> 3) << 1) | ((kb >> 1) & 1);
      unsigned acc[4] = {0, 0, 0, 0};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int srow = (by + j) * kSrcP + (bx >> 2);
        const uint32_t s0 = s32[srow], s1 = s32[srow + 1];
        const uint32_t* wp = W0 + (by + j) * kFPitch + (bx >> 2);
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
        lb[kb] = v < lb[kb] ? v : lb[kb];
        q16[q][sft] += acc[sft];
        t32[sft] += acc[sft];
      }
      __builtin_amdgcn_sched_barrier(0);  // bound live ranges: no hoisting across 8x8 blocks
    }
#pragma unroll
    for (int sft = 0; sft < 4; ++sft) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const unsigned v = ((q16[q][sft] + mvc[sft]) << 11) | (unsigned)(pos0 + sft);
        lb[16 + q] = v < lb[16 + q] ? v : lb[16 + q];
      }
      const unsigned v = ((t32[sft] + mvc[sft]) << 11) | (unsigned)(pos0 + sft);
      lb[20] = v < lb[20] ? v : lb[20];
    }
  }
#pragma unroll
  for (int k = 0; k < 21; ++k) {
    const unsigned m = wave_min_u32(lb[k]);
    if ((tid & 63) == 0) atomicMin(&best[k], m);
  }
  __syncthreads();
  if (tid < 21) {
    int mx, my;
    me_pos_to_mv((int)(best[tid] & 2047), cand, mx, my);
    bcost[tid] = (int)(best[tid] >> 11);
    bmv[tid][0] = 4 * mx;
    bmv[tid][1] = 4 * my;
  }

  // ------------------------ half- then quarter-pel refinement ---------------------------
  const uint8_t* sb = reinterpret_cast<const uint8_t*>(s32);
  const uint8_t* ph = phase + (long)b * 16 * g.psz;
  for (int step = 2; step >= 1; step >>= 1) {
    for (int t = tid; t < 168; t += kMeThreads) subsad[t >> 3][t & 7] = 0;
    __syncthreads();
    // A thread owns a group of 8 rows x 8 pixels of one (block, candidate): per row it loads
    // 3 aligned dwords of the phase plane, forms the 2 shifted dwords with v_alignbyte and
    // accumulates with v_sad_u8.  Groups per candidate: 16 (8x8) + 16 (16x16) + 16 (32x32).
    for (int grp = tid; grp < 8 * 48; grp += kMeThreads) {
      const int k = grp / 48, r = grp - k * 48;
      int bi, row0, col0;
      if (r < 16) {
        bi = r;
        row0 = col0 = 0;
      } else if (r < 32) {
        const int q = (r - 16) & 3;
        bi = 16 + ((r - 16) >> 2);
        row0 = 8 * (q >> 1);
        col0 = 8 * (q & 1);
      } else {
        const int q = r - 32;
        bi = 20;
        row0 = 8 * (q >> 2);
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
      const int sw = (by + row0) * kSrcP + ((bx + col0) >> 2);  // source word index of row 0
      unsigned sad = 0;
      if (gx0 >= -8 && gx0 + 11 <= g.W + 7 && gy0 >= -8 && gy0 + 7 <= g.H + 7) {
        const int a = gx0 & ~3, sh = gx0 & 3;
        const uint8_t* rowp = P + (long)(gy0 + 8) * g.pw16 + a + 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const uint32_t* wp = reinterpret_cast<const uint32_t*>(rowp + (long)j * g.pw16);
          const uint32_t w0 = wp[0], w1 = wp[1], w2 = wp[2];
          const uint32_t lo = __builtin_amdgcn_alignbyte(w1, w0, sh);
          const uint32_t hi = __builtin_amdgcn_alignbyte(w2, w1, sh);
          sad = __builtin_amdgcn_sad_u8(hi, s32[sw + kSrcP * j + 1], __builtin_amdgcn_sad_u8(lo, s32[sw + kSrcP * j], sad));
        }
      } else {  // touches the clamped border: per-pixel path
        for (int j = 0; j < 8; ++j) {
          const int gy = clip3(-8, g.H + 7, gy0 + j);
          for (int i = 0; i < 8; ++i) {
            const int gx = clip3(-8, g.W + 7, gx0 + i);
            sad += tv_abs((int)sb[(by + row0 + j) * 4 * kSrcP + bx + col0 + i] - (int)P[(long)(gy + 8) * g.pw16 + gx + 8]);
          }
        }
      }
      atomicAdd(&subsad[bi][k], (int)sad);
    }
    __syncthreads();
    if (tid < 21) {
      unsigned bestv = (unsigned)bcost[tid] << 4;
      for (int k = 0; k < 8; ++k) {
        int ox, oy;
        me_cand_offset(k, ox, oy);
        const int mx = bmv[tid][0] + ox * step, my = bmv[tid][1] + oy * step;
        const unsigned v =
            ((unsigned)(subsad[tid][k] + pen.mv[me_pen_index(mx - pmv[0], my - pmv[1])]) << 4) | (unsigned)(k + 1);
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

  // ------------------------------- CU split decision ------------------------------------
  if (tid == 0) {
    const int ps = pen.split_inter;
    int sum16 = 0;
    uint8_t l2u[16];
    int mvu[16][2];
    for (int q = 0; q < 4; ++q) {
      int sum8 = 0;
      for (int r = 0; r < 4; ++r) sum8 += bcost[me_blk8_of(q, r)] + ps;
      const bool split = sum8 < bcost[16 + q] + ps;
      sum16 += split ? sum8 : bcost[16 + q] + ps;
      for (int r = 0; r < 4; ++r) {
        const int ux = (q & 1) * 2 + (r & 1), uy = (q >> 1) * 2 + (r >> 1);
        const int sbi = split ? me_blk8_of(q, r) : 16 + q;
        l2u[uy * 4 + ux] = split ? 3 : 4;
        mvu[uy * 4 + ux][0] = bmv[sbi][0];
        mvu[uy * 4 + ux][1] = bmv[sbi][1];
      }
    }
    const bool whole = bcost[20] + ps <= sum16;
    for (int k = 0; k < 16; ++k) {
      const long u = b * g.usz + (long)((cy >> 3) + (k >> 2)) * g.w8 + (cx >> 3) + (k & 3);
      dec.cu_log2[u] = whole ? 5 : l2u[k];
      dec.mv[2 * u] = (int16_t)(whole ? bmv[20][0] : mvu[k][0]);
      dec.mv[2 * u + 1] = (int16_t)(whole ? bmv[20][1] : mvu[k][1]);
      dec.intra[u] = 0;
      dec.ipm[u] = 1;
    }
  }
}

// P-frame pass B: all TBs of a P-frame are independent (inter-only), so the (CU, component)
// TBs of a CTB are dealt round-robin to the 4 waves and coded wave-synchronously.
struct TbLds {
  uint8_t pred[1024];
  int16_t resid[1024];
  WaveTbScratch tb;
};

__global__ void __launch_bounds__(256) k_inter_recon(FrameSet src, FrameSet ref, const uint8_t* phase,
                                                     FrameSet rec, DecisionSet dec, Geo g, int qp) {
  const int ctu = blockIdx.x, b = blockIdx.y, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int cx = (ctu % g.wc) * 32, cy = (ctu / g.wc) * 32;
  __shared__ int Tm[32][33];
  __shared__ TbLds W[4];
  __shared__ int cus[16][4];  // x0, y0, log2, unit
  __shared__ int ncu;
  __shared__ unsigned cbfs[16];
  const long ub = b * g.usz;
  const uint8_t* ph = phase + (long)b * 16 * g.psz;
  tb_load_matrix(Tm);
  if (threadIdx.x == 0) {
    int n = 0;
    for (int k8 = 0; k8 < 16; ++k8) {
      const int x0 = cx + (k8 & 3) * 8, y0 = cy + (k8 >> 2) * 8;
      const int u = (y0 >> 3) * g.w8 + (x0 >> 3);
      const int log2 = dec.cu_log2[ub + u];
      if ((x0 & ((1 << log2) - 1)) || (y0 & ((1 << log2) - 1))) continue;  // not a CU origin
      cus[n][0] = x0;
      cus[n][1] = y0;
      cus[n][2] = log2;
      cus[n][3] = u;
      ++n;
    }
    ncu = n;
  }
  if (threadIdx.x < 16) cbfs[threadIdx.x] = 0;
  __syncthreads();
  // A CTB coded as one 32x32 CU: its luma TB would keep one wave busy for the whole
  // kernel while the others idle after chroma, so all four waves code it together (one
  // 16x16 MFMA tile each per stage), then two waves take the chroma TBs.
  const bool whole = ncu == 1 && cus[0][2] == 5;
  if (whole) {
    const long u = ub + cus[0][3];
    const int mvx = dec.mv[2 * u], mvy = dec.mv[2 * u + 1];
    const uint8_t* P = ph + (long)((mvx & 3) + 4 * (mvy & 3)) * g.psz;
    const uint8_t* S = src.plane(0, b, g);
    uint8_t* pred = W[0].pred;
    int16_t* resid = W[0].resid;
    for (int i = threadIdx.x; i < 1024; i += blockDim.x) {
      const int px = i & 31, py = i >> 5;
      const int p = phase_at(P, g, cx + px + (mvx >> 2), cy + py + (mvy >> 2));
      pred[i] = (uint8_t)p;
      resid[i] = (int16_t)((int)S[(cy + py) * g.W + cx + px] - p);
    }
    __syncthreads();
    const int cb = wg_code_tb(resid, pred, 5, qp, false, dec.coef_y + b * g.ysz + (long)cy * g.W + cx, g.W,
                              rec.plane(0, b, g) + (long)cy * g.W + cx, g.W, Tm, W[1].tb.tmp, W[1].tb.coef,
                              reinterpret_cast<int*>(W[2].resid));
    if (threadIdx.x == 0 && cb) atomicOr(&cbfs[0], 1u);
  }
  TbLds& Ld = W[wave];
  for (int t = whole ? wave + 1 : wave; t < 3 * ncu; t += whole ? 8 : 4) {
    const int k = t / 3, c = t - 3 * k;
    const int x0 = cus[k][0], y0 = cus[k][1], log2 = cus[k][2];
    const long u = ub + cus[k][3];
    const int mvx = dec.mv[2 * u], mvy = dec.mv[2 * u + 1];
    const int l2 = c ? log2 - 1 : log2, N = 1 << l2;
    const int x = c ? x0 >> 1 : x0, y = c ? y0 >> 1 : y0;
    const int pw = c ? g.W / 2 : g.W, phh = c ? g.H / 2 : g.H;
    const uint8_t* S = src.plane(c, b, g);
    if (c == 0) {
      const uint8_t* P = ph + (long)((mvx & 3) + 4 * (mvy & 3)) * g.psz;
      for (int i = lane; i < N * N; i += 64) {
        const int px = i & (N - 1), py = i >> l2;
        const int p = phase_at(P, g, x + px + (mvx >> 2), y + py + (mvy >> 2));
        Ld.pred[i] = (uint8_t)p;
        Ld.resid[i] = (int16_t)((int)S[(y + py) * pw + x + px] - p);
      }
    } else {
      const uint8_t* Rf = ref.plane(c, b, g);
      for (int i = lane; i < N * N; i += 64) {
        const int px = i & (N - 1), py = i >> l2;
        const int p = mc_chroma_sample(Rf, pw, pw, phh, x + px + (mvx >> 3), y + py + (mvy >> 3), mvx & 7, mvy & 7);
        Ld.pred[i] = (uint8_t)p;
        Ld.resid[i] = (int16_t)((int)S[(y + py) * pw + x + px] - p);
      }
    }
    wave_sync();
    int16_t* lev = (c == 0 ? dec.coef_y + b * g.ysz : (c == 1 ? dec.coef_u : dec.coef_v) + b * g.csz) +
                   (long)y * pw + x;
    const int cb = wave_code_tb(Ld.resid, Ld.pred, l2, c ? chroma_qp(qp, 0) : qp, false, lev, pw,
                                rec.plane(c, b, g) + (long)y * pw + x, pw, Tm, Ld.tb);
    if (lane == 0 && cb) atomicOr(&cbfs[k], 1u << c);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < ncu * 16; k += blockDim.x) {
    const int cu = k >> 4, j = k & 15, n8 = 1 << (cus[cu][2] - 3);
    if (j < n8 * n8) dec.cbf[ub + cus[cu][3] + (j / n8) * g.w8 + j % n8] = (uint8_t)cbfs[cu];
  }
}

void launch_quarter(FrameSet src, uint8_t* q, const Geo& g, int B, hipStream_t s) {
  const int n = (g.W >> 2) * (g.H >> 2);
  k_quarter<<<dim3((n + 255) / 256, B), 256, 0, s>>>(src, q, g);
}

void launch_inter_frame(FrameSet src, FrameSet ref, const uint8_t* phase, FrameSet rec, DecisionSet dec,
                        const Geo& g, int qp, const Penalties& pen, int range, const MeBuffers& me, int B,
                        hipStream_t s) {
  k_coarse_me<<<dim3(g.wc * g.hc, B), 64, 0, s>>>(me.qcur, me.qprev, g, pen, range / 4, me.cmv, me.ccost);
  k_inter_me<<<dim3(g.wc * g.hc, B), kMeThreads, 0, s>>>(src, ref, phase, dec, me.prev_mv, me.cmv, g, pen, range);
  k_inter_recon<<<dim3(g.wc * g.hc, B), 256, 0, s>>>(src, ref, phase, rec, dec, g, qp);
}

}  // namespace gpu
}  // namespace tv
