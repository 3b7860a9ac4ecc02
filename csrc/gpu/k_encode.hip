// k_encode.hip — gfx950 kernels of the HEVC encode pipeline (SURVEY.md §2.3 K5a–K5h).
//
// Every kernel processes a BATCH of independent segments (blockIdx.y = segment) so one
// launch covers B x CTUs workgroups: a single 1080p frame is only 510 CTUs, far too few
// for 256 CUs; batching GOP-aligned segments (the reference's unit of parallelism,
// worker/tasks.py:1146-1162) fills the chip.
//
//  k_synth            synthetic source frame generation (direct-source mode, P5)
//  k_sse              per-plane SSE for PSNR (K5h)
//  k_intra_analysis   I-frame pass A: 35-mode SATD search on 8/16/32 blocks + CU split
//  k_intra_recon      I-frame pass B: CTU-diagonal wavefront reconstruction
//  k_inter_me         P-frame pass A: LDS-windowed full search + quarter-pel refine + split
//  k_inter_recon      P-frame pass B: motion compensation + transform/quant + recon
//  k_deblock_*        in-loop deblocking (vertical then horizontal edges)
//
// All integer arithmetic mirrors the scalar golden model in tv/hevc_defs.h, so the GPU
// pipeline's decisions, levels and reconstruction are bit-identical to the CPU encoder.
#include "gpu_common.h"
#include "k_encode.h"
#include "tv/synth.h"

namespace tv {
namespace gpu {

// ------------------------------------ synth / sse ---------------------------------------
__global__ void k_synth(FrameSet src, Geo g, uint32_t seed, FrameIdx fi) {
  const int c = blockIdx.y, b = blockIdx.z;
  const int pw = c ? g.W / 2 : g.W, ph = c ? g.H / 2 : g.H;
  const int dw = c ? g.dw / 2 : g.dw, dh = c ? g.dh / 2 : g.dh;
  uint8_t* P = src.plane(c, b, g);
  const int t = fi.t[b];
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < pw * ph; i += gridDim.x * blockDim.x) {
    const int x = i % pw, y = i / pw;
    P[i] = (uint8_t)synth_sample(seed, t, c, tv_min(x, dw - 1), tv_min(y, dh - 1), g.dw, g.dh);
  }
}

__global__ void k_sse(FrameSet a, FrameSet r, Geo g, unsigned long long* sse /*[B][3]*/) {
  const int c = blockIdx.y, b = blockIdx.z;
  const int pw = c ? g.W / 2 : g.W;
  const int dw = c ? g.dw / 2 : g.dw, dh = c ? g.dh / 2 : g.dh;
  const uint8_t* A = a.plane(c, b, g);
  const uint8_t* R = r.plane(c, b, g);
  unsigned long long s = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < dw * dh; i += gridDim.x * blockDim.x) {
    const int x = i % dw, y = i / dw;
    const int d = (int)A[y * pw + x] - (int)R[y * pw + x];
    s += (unsigned long long)(d * d);
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(sse + b * 3 + c, s);
}

// -------------------------------- shared TB coding --------------------------------------
// Workgroup-cooperative: forward transform, quantisation, (inter) lone-coefficient zeroing,
// dequantisation, exact inverse transform and reconstruction of one N x N TB.
//   resid/pred: LDS, N*N, row-major.  Levels -> `lev` (stride ls), pixels -> `rec` (stride rs).
// Returns cbf (uniform across the workgroup).
struct TbScratch {
  int tmp[1024];
  int coef[1024];
  int red[4];
};

__device__ int wg_code_tb(const int* resid, const int* pred, int log2N, int qp, bool intra,
                          int16_t* lev, int ls, uint8_t* rec, int rs, TbScratch& s) {
  const int N = 1 << log2N, n2 = N * N, tid = threadIdx.x, nt = blockDim.x;
  const int sh1 = log2N - 1, sh2 = log2N + 6;
  if (tid < 4) s.red[tid] = 0;
  for (int i = tid; i < n2; i += nt) {
    const int k = i >> log2N, x = i & (N - 1);
    int acc = 0;
    for (int y = 0; y < N; ++y) acc += dct_coef(log2N, k, y) * resid[y * N + x];
    s.tmp[i] = (acc + (1 << (sh1 - 1))) >> sh1;
  }
  __syncthreads();
  int nz = 0, sa = 0;
  for (int i = tid; i < n2; i += nt) {
    const int k = i >> log2N, j = i & (N - 1);
    int acc = 0;
    for (int x = 0; x < N; ++x) acc += dct_coef(log2N, j, x) * s.tmp[k * N + x];
    const int c = (acc + (1 << (sh2 - 1))) >> sh2;
    const int l = quant_level(c, qp, log2N, intra);
    s.coef[i] = l;
    nz += l != 0;
    sa += tv_abs(l);
  }
  nz = wave_sum(nz);
  sa = wave_sum(sa);
  if ((tid & 63) == 0) {
    atomicAdd(&s.red[0], nz);
    atomicAdd(&s.red[1], sa);
  }
  __syncthreads();
  if (tid == 0) s.red[2] = (!intra && s.red[0] == 1 && s.red[1] == 1 && s.coef[0] == 0) ? 0 : s.red[0];
  __syncthreads();
  const int NZ = s.red[2];
  for (int i = tid; i < n2; i += nt) {
    const int l = NZ ? s.coef[i] : 0;
    lev[(i >> log2N) * ls + (i & (N - 1))] = (int16_t)l;
    if (!NZ) rec[(i >> log2N) * rs + (i & (N - 1))] = (uint8_t)clip_pixel(pred[i]);
    else s.coef[i] = dequant_level(l, qp, log2N);
  }
  if (!NZ) {
    __syncthreads();
    return 0;
  }
  __syncthreads();
  for (int i = tid; i < n2; i += nt) {
    const int y = i >> log2N, x = i & (N - 1);
    int acc = 0;
    for (int k = 0; k < N; ++k) acc += dct_coef(log2N, k, y) * s.coef[k * N + x];
    s.tmp[i] = clip3(-32768, 32767, (acc + 64) >> 7);
  }
  __syncthreads();
  for (int i = tid; i < n2; i += nt) {
    const int y = i >> log2N, x = i & (N - 1);
    int acc = 0;
    for (int k = 0; k < N; ++k) acc += dct_coef(log2N, k, x) * s.tmp[y * N + k];
    const int r = (acc + 2048) >> 12;
    rec[y * rs + x] = (uint8_t)clip_pixel(pred[i] + r);
  }
  __syncthreads();
  return 1;
}

// Build intra reference samples of a TB from a plane into LDS (all threads must call:
// contains barriers).  Lanes of wave 0 gather, thread 0 substitutes and smooths.
__device__ void wg_build_refs(const uint8_t* P, int pw, int cIdx, int x, int y, int log2N, int mode,
                              const Geo& g, int* L, int* T, bool* la, bool* ta) {
  const int N = 1 << log2N, s = cIdx ? 1 : 0, tid = threadIdx.x;
  const int xL = x << s, yL = y << s;
  for (int i = tid; i <= 2 * N; i += blockDim.x) {
    if (i == 0) {
      const bool a = zscan_available(xL, yL, (x - 1) << s, (y - 1) << s, g.W, g.H);
      la[0] = ta[0] = a;
      L[0] = T[0] = a ? P[(y - 1) * pw + (x - 1)] : 0;
    } else {
      const bool al = zscan_available(xL, yL, (x - 1) << s, (y + i - 1) << s, g.W, g.H);
      la[i] = al;
      L[i] = al ? P[(y + i - 1) * pw + (x - 1)] : 0;
      const bool at = zscan_available(xL, yL, (x + i - 1) << s, (y - 1) << s, g.W, g.H);
      ta[i] = at;
      T[i] = at ? P[(y - 1) * pw + (x + i - 1)] : 0;
    }
  }
  __syncthreads();
  if (tid == 0) {
    intra_substitute(L, T, la, ta, N);
    if (cIdx == 0 && intra_filter_refs(log2N, mode)) intra_smooth_refs(L, T, N);
  }
  __syncthreads();
}

// ------------------------------- I-frame: analysis --------------------------------------
__device__ __forceinline__ void blk_geom(int bi, int& bx, int& by, int& l2) {
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
__device__ __forceinline__ int blk8_of(int q, int r) {
  return (((q >> 1) * 2 + (r >> 1)) << 2) + (q & 1) * 2 + (r & 1);
}

__global__ void __launch_bounds__(256) k_intra_analysis(FrameSet src, DecisionSet dec, Geo g,
                                                        Penalties pen) {
  const int ctu = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int cx = (ctu % g.wc) * 32, cy = (ctu / g.wc) * 32;
  const uint8_t* S = src.plane(0, b, g);
  __shared__ uint8_t sblk[32 * 32];
  __shared__ int refs[21][4][65];  // left, top, filtered left, filtered top
  __shared__ bool avl[21][2][65];
  __shared__ int dcv[21];
  __shared__ unsigned best[21];
  for (int i = tid; i < 1024; i += 256) sblk[i] = S[(cy + (i >> 5)) * g.W + cx + (i & 31)];
  if (tid < 21) best[tid] = 0xffffffffu;
  // reference samples from the SOURCE picture (analysis): one thread per block
  if (tid < 21) {
    int bx, by, l2;
    blk_geom(tid, bx, by, l2);
    const int N = 1 << l2, x = cx + bx, y = cy + by;
    int* L = refs[tid][0];
    int* T = refs[tid][1];
    bool* la = avl[tid][0];
    bool* ta = avl[tid][1];
    {
      const bool a = zscan_available(x, y, x - 1, y - 1, g.W, g.H);
      la[0] = ta[0] = a;
      L[0] = T[0] = a ? S[(y - 1) * g.W + x - 1] : 0;
    }
    for (int i = 0; i < 2 * N; ++i) {
      const bool al = zscan_available(x, y, x - 1, y + i, g.W, g.H);
      la[i + 1] = al;
      L[i + 1] = al ? S[(y + i) * g.W + x - 1] : 0;
      const bool at = zscan_available(x, y, x + i, y - 1, g.W, g.H);
      ta[i + 1] = at;
      T[i + 1] = at ? S[(y - 1) * g.W + x + i] : 0;
    }
    intra_substitute(L, T, la, ta, N);
    int* FL = refs[tid][2];
    int* FT = refs[tid][3];
    for (int i = 0; i <= 2 * N; ++i) {
      FL[i] = L[i];
      FT[i] = T[i];
    }
    intra_smooth_refs(FL, FT, N);
    dcv[tid] = intra_dc_value(L, T, l2);
  }
  __syncthreads();
  const int wave = tid >> 6, lane = tid & 63;
  for (int t = wave; t < 735; t += 4) {
    int bi, mode;
    if (t < 560) {
      bi = t / 35;
      mode = t % 35;
    } else if (t < 700) {
      bi = 16 + (t - 560) / 35;
      mode = (t - 560) % 35;
    } else {
      bi = 20;
      mode = t - 700;
    }
    int bx, by, l2;
    blk_geom(bi, bx, by, l2);
    const int N = 1 << l2, nq = N >> 3;
    const bool filt = intra_filter_refs(l2, mode);
    const int* L = refs[bi][filt ? 2 : 0];
    const int* T = refs[bi][filt ? 3 : 1];
    int sum = 0;
    for (int q = 0; q < nq * nq; ++q) {
      const int qx = (q % nq) * 8 + (lane & 7), qy = (q / nq) * 8 + (lane >> 3);
      const int p = intra_pred_pixel(L, T, l2, mode, N < 32, dcv[bi], qx, qy);
      sum += wave_satd8x8((int)sblk[(by + qy) * 32 + bx + qx] - p);
    }
    const unsigned cost = (unsigned)(sum + (mode <= 1 ? pen.mode_dcpl : pen.mode_ang));
    if (lane == 0) atomicMin(&best[bi], (cost << 6) | (unsigned)mode);
  }
  __syncthreads();
  if (tid == 0) {
    const int ps = pen.split_intra;
    const int c32 = (int)(best[20] >> 6);
    int sum16 = 0;
    uint8_t l2u[16], mu[16];
    for (int q = 0; q < 4; ++q) {
      const int c16 = (int)(best[16 + q] >> 6);
      int sum8 = 0;
      for (int r = 0; r < 4; ++r) sum8 += (int)(best[blk8_of(q, r)] >> 6) + ps;
      const bool split = sum8 < c16 + ps;
      sum16 += split ? sum8 : c16 + ps;
      for (int r = 0; r < 4; ++r) {
        const int ux = (q & 1) * 2 + (r & 1), uy = (q >> 1) * 2 + (r >> 1);
        l2u[uy * 4 + ux] = split ? 3 : 4;
        mu[uy * 4 + ux] = (uint8_t)(split ? (best[blk8_of(q, r)] & 63) : (best[16 + q] & 63));
      }
    }
    const bool whole = c32 + ps <= sum16;
    for (int k = 0; k < 16; ++k) {
      const long u = b * g.usz + (long)((cy >> 3) + (k >> 2)) * g.w8 + (cx >> 3) + (k & 3);
      dec.cu_log2[u] = whole ? 5 : l2u[k];
      dec.ipm[u] = whole ? (uint8_t)(best[20] & 63) : mu[k];
      dec.intra[u] = 1;
      dec.mv[2 * u] = dec.mv[2 * u + 1] = 0;
    }
  }
}

// -------------------------- I-frame: wavefront reconstruction ---------------------------
// One workgroup per CTU on anti-diagonal `diag` (cx + 2*cy == diag): all of its left,
// above and above-right neighbours were reconstructed by earlier launches.
__global__ void __launch_bounds__(256) k_intra_recon(FrameSet src, FrameSet rec, DecisionSet dec,
                                                     Geo g, int qp, int diag, int cy0) {
  const int b = blockIdx.y, tid = threadIdx.x;
  const int cyi = cy0 + blockIdx.x, cxi = diag - 2 * cyi;
  const int cx = cxi * 32, cy = cyi * 32;
  __shared__ int pred[1024], resid[1024];
  __shared__ int L[65], T[65];
  __shared__ bool la[65], ta[65];
  __shared__ TbScratch scr;
  const long ub = b * g.usz;
  const int qpc = chroma_qp(qp, 0);
  // enumerate CUs of this CTU in z-order
  int cus[16][3];
  int ncu = 0;
  {
    const int l32 = dec.cu_log2[ub + (cy >> 3) * g.w8 + (cx >> 3)];
    if (l32 == 5) {
      cus[ncu][0] = cx;
      cus[ncu][1] = cy;
      cus[ncu][2] = 5;
      ++ncu;
    } else {
      for (int q = 0; q < 4; ++q) {
        const int x16 = cx + (q & 1) * 16, y16 = cy + (q >> 1) * 16;
        if (dec.cu_log2[ub + (y16 >> 3) * g.w8 + (x16 >> 3)] == 4) {
          cus[ncu][0] = x16;
          cus[ncu][1] = y16;
          cus[ncu][2] = 4;
          ++ncu;
        } else {
          for (int r = 0; r < 4; ++r) {
            cus[ncu][0] = x16 + (r & 1) * 8;
            cus[ncu][1] = y16 + (r >> 1) * 8;
            cus[ncu][2] = 3;
            ++ncu;
          }
        }
      }
    }
  }
  for (int k = 0; k < ncu; ++k) {
    const int x0 = cus[k][0], y0 = cus[k][1], log2 = cus[k][2];
    const long u = ub + (y0 >> 3) * g.w8 + (x0 >> 3);
    const int mode = dec.ipm[u];
    int cbf = 0;
    for (int c = 0; c < 3; ++c) {
      const int l2 = c ? log2 - 1 : log2, N = 1 << l2;
      const int x = c ? x0 >> 1 : x0, y = c ? y0 >> 1 : y0;
      const int pw = c ? g.W / 2 : g.W;
      uint8_t* R = rec.plane(c, b, g);
      const uint8_t* S = src.plane(c, b, g);
      wg_build_refs(R, pw, c, x, y, l2, mode, g, L, T, la, ta);
      const int dc = mode == 1 ? intra_dc_value(L, T, l2) : 0;
      for (int i = tid; i < N * N; i += 256) {
        const int px = i & (N - 1), py = i >> l2;
        const int p = intra_pred_pixel(L, T, l2, mode, c == 0 && N < 32, dc, px, py);
        pred[i] = p;
        resid[i] = (int)S[(y + py) * pw + x + px] - p;
      }
      __syncthreads();
      int16_t* lev = (c == 0 ? dec.coef_y + b * g.ysz : (c == 1 ? dec.coef_u : dec.coef_v) + b * g.csz) +
                     (long)y * pw + x;
      const int cb = wg_code_tb(resid, pred, l2, c ? qpc : qp, true, lev, pw, R + (long)y * pw + x, pw, scr);
      cbf |= cb << c;
      __syncthreads();
    }
    if (tid < (1 << (2 * (log2 - 3)))) {
      const int n8 = 1 << (log2 - 3);
      dec.cbf[u + (tid / n8) * g.w8 + (tid % n8)] = (uint8_t)cbf;
    }
  }
}

// -------------------------------- P-frame: analysis -------------------------------------
constexpr int kWin = 72;   // reference window side (32 + 2*16 search + 8 filter taps)
constexpr int kWinOff = 20;  // window origin = CTU origin - 20

__global__ void __launch_bounds__(256) k_inter_me(FrameSet src, FrameSet ref, DecisionSet dec, Geo g,
                                                  Penalties pen, int range) {
  const int ctu = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int cx = (ctu % g.wc) * 32, cy = (ctu / g.wc) * 32;
  const uint8_t* S = src.plane(0, b, g);
  const uint8_t* R = ref.plane(0, b, g);
  __shared__ uint8_t sblk[32 * 32];
  __shared__ uint8_t win[kWin * kWin];
  __shared__ unsigned best[21];
  __shared__ int bcost[21];
  __shared__ int bmv[21][2];
  for (int i = tid; i < 1024; i += 256) sblk[i] = S[(cy + (i >> 5)) * g.W + cx + (i & 31)];
  for (int i = tid; i < kWin * kWin; i += 256) {
    const int wx = i % kWin, wy = i / kWin;
    const int gx = clip3(0, g.W - 1, cx - kWinOff + wx), gy = clip3(0, g.H - 1, cy - kWinOff + wy);
    win[i] = R[gy * g.W + gx];
  }
  if (tid < 21) best[tid] = 0xffffffffu;
  __syncthreads();
  // ---- integer full search
  const int side = 2 * range + 1, ncand = side * side;
  unsigned lb[21];
#pragma unroll
  for (int k = 0; k < 21; ++k) lb[k] = 0xffffffffu;
  for (int c = tid; c < ncand; c += 256) {
    const int dx = c % side - range, dy = c / side - range;
    const int mvc = pen.mv[mv_bits_est(4 * dx, 4 * dy)];
    int s8[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int bx = (k & 3) * 8, by = (k >> 2) * 8;
      int s = 0;
      const uint8_t* wp = win + (kWinOff + dy + by) * kWin + kWinOff + dx + bx;
      const uint8_t* sp = sblk + by * 32 + bx;
      for (int j = 0; j < 8; ++j)
#pragma unroll
        for (int i = 0; i < 8; ++i) s += tv_abs((int)sp[j * 32 + i] - (int)wp[j * kWin + i]);
      s8[k] = s;
    }
    int s32 = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const unsigned v = ((unsigned)(s8[k] + mvc) << 11) | (unsigned)c;
      lb[k] = v < lb[k] ? v : lb[k];
      s32 += s8[k];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int s16 = s8[blk8_of(q, 0)] + s8[blk8_of(q, 1)] + s8[blk8_of(q, 2)] + s8[blk8_of(q, 3)];
      const unsigned v = ((unsigned)(s16 + mvc) << 11) | (unsigned)c;
      lb[16 + q] = v < lb[16 + q] ? v : lb[16 + q];
    }
    const unsigned v = ((unsigned)(s32 + mvc) << 11) | (unsigned)c;
    lb[20] = v < lb[20] ? v : lb[20];
  }
#pragma unroll
  for (int k = 0; k < 21; ++k) {
    const unsigned m = wave_min_u32(lb[k]);
    if ((tid & 63) == 0) atomicMin(&best[k], m);
  }
  __syncthreads();
  if (tid < 21) {
    const int c = (int)(best[tid] & 2047);
    bcost[tid] = (int)(best[tid] >> 11);
    bmv[tid][0] = 4 * (c % side - range);
    bmv[tid][1] = 4 * (c / side - range);
  }
  __syncthreads();
  // ---- half- then quarter-pel refinement, one block at a time, 8 candidates in parallel
  __shared__ unsigned sub[21];
  for (int bi = 0; bi < 21; ++bi) {
    int bx, by, l2;
    blk_geom(bi, bx, by, l2);
    const int N = 1 << l2, n2 = N * N;
    for (int step = 2; step >= 1; step >>= 1) {
      if (tid == 0) sub[bi] = ((unsigned)bcost[bi] << 4);  // center = candidate 0
      __syncthreads();
      const int k = tid >> 5, lane32 = tid & 31;
      const int ox = (k == 0 || k == 3 || k == 5) ? -1 : ((k == 1 || k == 6) ? 0 : 1);
      const int oy = k < 3 ? -1 : (k < 5 ? 0 : 1);
      const int mx = bmv[bi][0] + ox * step, my = bmv[bi][1] + oy * step;
      const int fx = mx & 3, fy = my & 3;
      const int ix = kWinOff + bx + (mx >> 2), iy = kWinOff + by + (my >> 2);
      int s = 0;
      for (int p = lane32; p < n2; p += 32) {
        const int px = p & (N - 1), py = p >> l2;
        const int pv = mc_luma_sample(win, kWin, kWin, kWin, ix + px, iy + py, fx, fy);
        s += tv_abs((int)sblk[(by + py) * 32 + bx + px] - pv);
      }
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      if (lane32 == 0) {
        const unsigned v = ((unsigned)(s + pen.mv[mv_bits_est(mx, my)]) << 4) | (unsigned)(k + 1);
        atomicMin(&sub[bi], v);
      }
      __syncthreads();
      if (tid == 0) {
        const unsigned v = sub[bi];
        const int kk = (int)(v & 15);
        bcost[bi] = (int)(v >> 4);
        if (kk) {
          const int j = kk - 1;
          const int jx = (j == 0 || j == 3 || j == 5) ? -1 : ((j == 1 || j == 6) ? 0 : 1);
          const int jy = j < 3 ? -1 : (j < 5 ? 0 : 1);
          bmv[bi][0] += jx * step;
          bmv[bi][1] += jy * step;
        }
      }
      __syncthreads();
    }
  }
  // ---- CU split decision (same rule as the CPU reference)
  if (tid == 0) {
    const int ps = pen.split_inter;
    int sum16 = 0;
    uint8_t l2u[16];
    int mvu[16][2];
    for (int q = 0; q < 4; ++q) {
      int sum8 = 0;
      for (int r = 0; r < 4; ++r) sum8 += bcost[blk8_of(q, r)] + ps;
      const bool split = sum8 < bcost[16 + q] + ps;
      sum16 += split ? sum8 : bcost[16 + q] + ps;
      for (int r = 0; r < 4; ++r) {
        const int ux = (q & 1) * 2 + (r & 1), uy = (q >> 1) * 2 + (r >> 1);
        const int src_b = split ? blk8_of(q, r) : 16 + q;
        l2u[uy * 4 + ux] = split ? 3 : 4;
        mvu[uy * 4 + ux][0] = bmv[src_b][0];
        mvu[uy * 4 + ux][1] = bmv[src_b][1];
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

// ------------------------------ P-frame: reconstruction ---------------------------------
__global__ void __launch_bounds__(256) k_inter_recon(FrameSet src, FrameSet ref, FrameSet rec,
                                                     DecisionSet dec, Geo g, int qp) {
  const int ctu = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const int cx = (ctu % g.wc) * 32, cy = (ctu / g.wc) * 32;
  __shared__ int pred[1024], resid[1024];
  __shared__ TbScratch scr;
  const long ub = b * g.usz;
  const int qpc = chroma_qp(qp, 0);
  for (int k8 = 0; k8 < 16; ++k8) {
    // visit each CU once, at its top-left 8x8 unit (z-order irrelevant for inter)
    const int x0 = cx + (k8 & 3) * 8, y0 = cy + (k8 >> 2) * 8;
    const long u = ub + (y0 >> 3) * g.w8 + (x0 >> 3);
    const int log2 = dec.cu_log2[u];
    if ((x0 & ((1 << log2) - 1)) || (y0 & ((1 << log2) - 1))) continue;
    const int mvx = dec.mv[2 * u], mvy = dec.mv[2 * u + 1];
    int cbf = 0;
    for (int c = 0; c < 3; ++c) {
      const int l2 = c ? log2 - 1 : log2, N = 1 << l2;
      const int x = c ? x0 >> 1 : x0, y = c ? y0 >> 1 : y0;
      const int pw = c ? g.W / 2 : g.W, ph = c ? g.H / 2 : g.H;
      const uint8_t* Rf = ref.plane(c, b, g);
      const uint8_t* S = src.plane(c, b, g);
      for (int i = tid; i < N * N; i += 256) {
        const int px = i & (N - 1), py = i >> l2;
        int p;
        if (c == 0) p = mc_luma_sample(Rf, pw, pw, ph, x + px + (mvx >> 2), y + py + (mvy >> 2), mvx & 3, mvy & 3);
        else p = mc_chroma_sample(Rf, pw, pw, ph, x + px + (mvx >> 3), y + py + (mvy >> 3), mvx & 7, mvy & 7);
        pred[i] = p;
        resid[i] = (int)S[(y + py) * pw + x + px] - p;
      }
      __syncthreads();
      int16_t* lev = (c == 0 ? dec.coef_y + b * g.ysz : (c == 1 ? dec.coef_u : dec.coef_v) + b * g.csz) +
                     (long)y * pw + x;
      const int cb = wg_code_tb(resid, pred, l2, c ? qpc : qp, false, lev, pw,
                                rec.plane(c, b, g) + (long)y * pw + x, pw, scr);
      cbf |= cb << c;
    }
    const int n8 = 1 << (log2 - 3);
    if (tid < n8 * n8) dec.cbf[u + (tid / n8) * g.w8 + (tid % n8)] = (uint8_t)cbf;
    __syncthreads();
  }
}

// ------------------------------------ deblocking ----------------------------------------
__global__ void k_deblock(FrameSet rec, DecisionSet dec, Geo g, int qp, int horizontal) {
  const int b = blockIdx.y;
  const long ub = b * g.usz;
  const uint8_t* cl = dec.cu_log2 + ub;
  const uint8_t* in = dec.intra + ub;
  const uint8_t* cb = dec.cbf + ub;
  const int16_t* mv = dec.mv + 2 * ub;
  uint8_t* Y = rec.plane(0, b, g);
  uint8_t* U = rec.plane(1, b, g);
  uint8_t* V = rec.plane(2, b, g);
  const int W = g.W, H = g.H, Wc = W / 2;
  const int qpc = chroma_qp(qp, 0);
  // luma segments: vertical edges -> (W/8 - 1) x (H/4); horizontal -> (H/8 - 1) x (W/4)
  const int nl = horizontal ? (H / 8 - 1) * (W / 4) : (W / 8 - 1) * (H / 4);
  const int nc = horizontal ? (H / 16 - 1) * (Wc / 4) : (W / 16 - 1) * (H / 8);
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nl + nc; i += gridDim.x * blockDim.x) {
    if (i < nl) {
      if (!horizontal) {
        const int x = 8 * (1 + i % (W / 8 - 1)), y = 4 * (i / (W / 8 - 1));
        const int bs = deblock_edge_bs(cl, in, cb, mv, g.w8, x - 1, y, x, y);
        if (bs) deblock_luma_edge4(Y + (long)y * W + x, 1, W, bs, qp);
      } else {
        const int y = 8 * (1 + i % (H / 8 - 1)), x = 4 * (i / (H / 8 - 1));
        const int bs = deblock_edge_bs(cl, in, cb, mv, g.w8, x, y - 1, x, y);
        if (bs) deblock_luma_edge4(Y + (long)y * W + x, W, 1, bs, qp);
      }
    } else {
      const int j = i - nl;
      if (!horizontal) {
        const int xc = 8 * (1 + j % (W / 16 - 1)), yc = 4 * (j / (W / 16 - 1));
        const int bs = deblock_edge_bs(cl, in, cb, mv, g.w8, 2 * xc - 1, 2 * yc, 2 * xc, 2 * yc);
        if (bs == 2) {
          deblock_chroma_edge(U + (long)yc * Wc + xc, 1, Wc, 4, qpc);
          deblock_chroma_edge(V + (long)yc * Wc + xc, 1, Wc, 4, qpc);
        }
      } else {
        const int yc = 8 * (1 + j % (H / 16 - 1)), xc = 4 * (j / (H / 16 - 1));
        const int bs = deblock_edge_bs(cl, in, cb, mv, g.w8, 2 * xc, 2 * yc - 1, 2 * xc, 2 * yc);
        if (bs == 2) {
          deblock_chroma_edge(U + (long)yc * Wc + xc, Wc, 1, 4, qpc);
          deblock_chroma_edge(V + (long)yc * Wc + xc, Wc, 1, 4, qpc);
        }
      }
    }
  }
}

// ------------------------------------ launchers -----------------------------------------
void launch_synth(FrameSet src, const Geo& g, uint32_t seed, const FrameIdx& fi, int B, hipStream_t s) {
  dim3 grid((unsigned)tv_min(1024, (int)((g.ysz + 255) / 256)), 3, B);
  k_synth<<<grid, 256, 0, s>>>(src, g, seed, fi);
}
void launch_sse(FrameSet a, FrameSet r, const Geo& g, unsigned long long* sse, int B, hipStream_t s) {
  dim3 grid((unsigned)tv_min(512, (int)((g.ysz + 255) / 256)), 3, B);
  k_sse<<<grid, 256, 0, s>>>(a, r, g, sse);
}
void launch_intra_frame(FrameSet src, FrameSet rec, DecisionSet dec, const Geo& g, int qp,
                        const Penalties& pen, int B, hipStream_t s) {
  k_intra_analysis<<<dim3(g.wc * g.hc, B), 256, 0, s>>>(src, dec, g, pen);
  const int ndiag = (g.wc - 1) + 2 * (g.hc - 1) + 1;
  for (int d = 0; d < ndiag; ++d) {
    const int cy0 = tv_max(0, (d - (g.wc - 1) + 1) / 2);
    const int cy1 = tv_min(g.hc - 1, d / 2);
    if (cy1 < cy0) continue;
    k_intra_recon<<<dim3(cy1 - cy0 + 1, B), 256, 0, s>>>(src, rec, dec, g, qp, d, cy0);
  }
}
void launch_inter_frame(FrameSet src, FrameSet ref, FrameSet rec, DecisionSet dec, const Geo& g,
                        int qp, const Penalties& pen, int range, int B, hipStream_t s) {
  k_inter_me<<<dim3(g.wc * g.hc, B), 256, 0, s>>>(src, ref, dec, g, pen, range);
  k_inter_recon<<<dim3(g.wc * g.hc, B), 256, 0, s>>>(src, ref, rec, dec, g, qp);
}
void launch_deblock(FrameSet rec, DecisionSet dec, const Geo& g, int qp, int B, hipStream_t s) {
  dim3 grid((unsigned)tv_min(1024, (int)(g.ysz / 32 / 256 + 1)), B);
  k_deblock<<<grid, 256, 0, s>>>(rec, dec, g, qp, 0);
  k_deblock<<<grid, 256, 0, s>>>(rec, dec, g, qp, 1);
}

}  // namespace gpu
}  // namespace tv
