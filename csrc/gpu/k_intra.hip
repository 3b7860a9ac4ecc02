// k_intra.hip — I-frame kernels.
//
//  k_intra_analysis  pass A, fully parallel over CTUs: for all 21 blocks of a CTB
//                    (16 x 8x8, 4 x 16x16, 1 x 32x32) and all 35 HEVC intra modes, predict
//                    from SOURCE neighbours and compute the 8x8-Hadamard SATD with one wave
//                    per (block, mode): lane = pixel, butterflies via cross-lane shuffles.
//                    Then the bottom-up CU split decision.
//  k_intra_recon     pass B, CTB anti-diagonal wavefront (cx + 2*cy = d per launch): the
//                    normative prediction from reconstructed neighbours + MFMA TB coding.
#include <cstdio>
#include <cstdlib>

#include "gpu_common.h"
#include "k_encode.h"
#include "tb_coder.h"
#include "wave_tb.h"
#include "tv/me_model.h"

namespace tv {
namespace gpu {

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
// flattened reference-sample entry e (0..468) -> (block, index within 2N+1)
__device__ __forceinline__ void ref_entry(int e, int& bi, int& i) {
  if (e < 272) {
    bi = e / 17;
    i = e % 17;
  } else if (e < 404) {
    bi = 16 + (e - 272) / 33;
    i = (e - 272) % 33;
  } else {
    bi = 20;
    i = e - 404;
  }
}

// the angular-mode tables in LDS (indexed constexpr tables become global loads on the GPU)
struct AngleLds {
  int8_t angle[35];
  int16_t inv[35];
  __device__ void load(int tid, int nthreads) {
    for (int m = tid; m < 35; m += nthreads) {
      angle[m] = m >= 2 ? (int8_t)intra_angle(m) : 0;
      inv[m] = m >= 2 ? (int16_t)intra_inv_angle(m) : 0;
    }
  }
};

__global__ void __launch_bounds__(256) k_intra_analysis(FrameSet src, DecisionSet dec, Geo g, const RcTables* rc) {
  const int ctu = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const Penalties& pen = rc->pen[dec.qp[b]];
  const int cx = (ctu % g.wc) * 32, cy = (ctu / g.wc) * 32;
  const uint8_t* S = src.plane(0, b, g);
  __shared__ uint8_t sblk[32 * 32];
  __shared__ int16_t refs[21][4][65];  // left, top, smoothed left, smoothed top
  __shared__ bool avl[21][2][65];
  __shared__ int dcv[21];
  __shared__ unsigned best[21], best_ang[21];
  __shared__ AngleLds ang;
  ang.load(tid, 256);
  for (int i = tid; i < 1024; i += 256) sblk[i] = S[(cy + (i >> 5)) * g.W + cx + (i & 31)];
  if (tid < 21) best[tid] = best_ang[tid] = 0xffffffffu;
  for (int e = tid; e < 469; e += 256) {
    int bi, i, bx, by, l2;
    ref_entry(e, bi, i);
    blk_geom(bi, bx, by, l2);
    const int x = cx + bx, y = cy + by;
    if (i == 0) {
      const bool a = zscan_available(x, y, x - 1, y - 1, g.W, g.H);
      avl[bi][0][0] = avl[bi][1][0] = a;
      refs[bi][0][0] = refs[bi][1][0] = a ? S[(y - 1) * g.W + x - 1] : 0;
    } else {
      const bool al = zscan_available(x, y, x - 1, y + i - 1, g.W, g.H);
      avl[bi][0][i] = al;
      refs[bi][0][i] = al ? S[(y + i - 1) * g.W + x - 1] : 0;
      const bool at = zscan_available(x, y, x + i - 1, y - 1, g.W, g.H);
      avl[bi][1][i] = at;
      refs[bi][1][i] = at ? S[(y - 1) * g.W + x + i - 1] : 0;
    }
  }
  __syncthreads();
  if (tid < 21) {
    int bx, by, l2;
    blk_geom(tid, bx, by, l2);
    intra_substitute(refs[tid][0], refs[tid][1], avl[tid][0], avl[tid][1], 1 << l2);
    dcv[tid] = intra_dc_value(refs[tid][0], refs[tid][1], l2);
  }
  __syncthreads();
  for (int e = tid; e < 469; e += 256) {  // [1 2 1] smoothed copies
    int bi, i, bx, by, l2;
    ref_entry(e, bi, i);
    blk_geom(bi, bx, by, l2);
    const int N2 = 2 << l2;
    const int16_t* L = refs[bi][0];
    const int16_t* T = refs[bi][1];
    if (i == 0) {
      refs[bi][2][0] = refs[bi][3][0] = (int16_t)((L[1] + 2 * L[0] + T[1] + 2) >> 2);
    } else if (i == N2) {
      refs[bi][2][i] = L[i];
      refs[bi][3][i] = T[i];
    } else {
      refs[bi][2][i] = (int16_t)((L[i + 1] + 2 * L[i] + L[i - 1] + 2) >> 2);
      refs[bi][3][i] = (int16_t)((T[i + 1] + 2 * T[i] + T[i - 1] + 2) >> 2);
    }
  }
  __syncthreads();
  const int wave = tid >> 6, lane = tid & 63;
  // one wave per (block, mode); stage 1 = the 11 coarse modes of every block, stage 2 = the
  // +-1 / +-2 neighbours of each block's best stage-1 angular mode (tv/me_model.h)
  auto eval = [&](int bi, int mode, bool coarse) {
    int bx, by, l2;
    blk_geom(bi, bx, by, l2);
    const int N = 1 << l2, nq = N >> 3;
    const bool filt = intra_filter_refs(l2, mode);
    const int16_t* L = refs[bi][filt ? 2 : 0];
    const int16_t* T = refs[bi][filt ? 3 : 1];
    int sum = 0;
    for (int q = 0; q < nq * nq; ++q) {
      const int qx = (q % nq) * 8 + (lane & 7), qy = (q / nq) * 8 + (lane >> 3);
      const int p = intra_pred_pixel_ai(L, T, l2, mode, ang.angle[mode], ang.inv[mode], N < 32, dcv[bi], qx, qy);
      sum += wave_satd8x8((int)sblk[(by + qy) * 32 + bx + qx] - p);
    }
    const unsigned v = ((unsigned)(sum + (mode <= 1 ? pen.mode_dcpl : pen.mode_ang)) << 6) | (unsigned)mode;
    if (lane == 0) {
      atomicMin(&best[bi], v);
      // only stage 1 moves the refinement centre: stage-2 waves read it concurrently
      if (coarse && mode >= 2) atomicMin(&best_ang[bi], v);
    }
  };
  for (int t = wave; t < 21 * kIntraCoarseModes; t += 4) eval(t / kIntraCoarseModes, intra_coarse_mode(t % kIntraCoarseModes), true);
  __syncthreads();
  for (int t = wave; t < 21 * 4; t += 4) {
    const int bi = t >> 2, m = intra_refine_mode((int)(best_ang[bi] & 63), t & 3);
    if (m >= 2) eval(bi, m, false);
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

// ------------------- I-frame pass B: CTB wavefront, one wave per component ----------------
// Each workgroup (3 waves) owns one CTB of the current anti-diagonal.  Intra prediction of a
// component only reads that component's reconstruction, so Y, Cb and Cr are three
// independent chains: wave c codes every TB of component c in z-order.  The component's
// source, own reconstruction and the reconstructed borders of the left / above /
// above-right neighbours are staged in LDS once; each TB is then predicted, transformed and
// reconstructed wave-synchronously from LDS (no workgroup barrier per TB).
// one component's CTB state; S = 32 (luma) or 16 (chroma): the chroma waves' copies are a
// third of the luma one, so the workgroup's LDS (50 KB with three luma-sized copies) allows 5
// CTBs per CU instead of 3 on the short wavefront launches
template <int S>
struct CompLdsT {
  uint8_t src[S * S];
  uint8_t rec[S * S];
  uint8_t top[2 * S + 8];  // row y = cy-1, x = cx-1 .. cx+2S-1  (index 0 = corner)
  uint8_t left[S];         // column x = cx-1, y = cy .. cy+S-1
  uint8_t pred[S * S];
  int16_t resid[S * S];
  int V[4 * S + 4];
  int L[2 * S + 1], T[2 * S + 1], FL[2 * S + 1], FT[2 * S + 1];
  WaveTbScratchT<S> tb;
};
using CompLds = CompLdsT<32>;

// TV_DIAG_INTRA=1: lane 0 of every wave adds the clock cycles of each phase to
// g_intra_phase[c][phase] (c = component wave): timing only, printed at engine teardown.
__device__ unsigned long long g_intra_phase[3][8];

__global__ void __launch_bounds__(192) k_intra_recon(FrameSet src, FrameSet rec, DecisionSet dec, Geo g, int diag,
                                                     int cy0, int timing) {
  const int b = blockIdx.y, c = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int qp = dec.qp[b];
  __shared__ int Tm[32][33];
  __shared__ CompLdsT<32> WY;    // luma
  __shared__ CompLdsT<16> WC[2];  // Cb, Cr
  __shared__ int cus[16][4];
  __shared__ AngleLds ang;
  ang.load(threadIdx.x, 192);
  __shared__ int ncu;
  __shared__ unsigned cbfs[16];
  long long tph = timing ? (long long)clock64() : 0;
  auto mark = [&](int ph) {
    if (!timing) return;
    const long long t = (long long)clock64();
    if ((threadIdx.x & 63) == 0) atomicAdd(&g_intra_phase[threadIdx.x >> 6][ph], (unsigned long long)(t - tph));
    tph = t;
  };
  const int cyi = cy0 + blockIdx.x, cxi = diag - 2 * cyi;
  const int cx = cxi * 32, cy = cyi * 32;
  const long ub = b * g.usz;
  tb_load_matrix(Tm);
  // the CTB's 16 8x8-unit sizes and modes, loaded in parallel (one global round trip instead
  // of a dependent load per CU inside the sequential CU loop)
  __shared__ uint8_t ul2[16], uipm[16];
  if (threadIdx.x < 16) {
    const long u = ub + (long)((cy >> 3) + (threadIdx.x >> 2)) * g.w8 + (cx >> 3) + (threadIdx.x & 3);
    ul2[threadIdx.x] = dec.cu_log2[u];
    uipm[threadIdx.x] = dec.ipm[u];
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // CUs of this CTB in z-order: x, y, log2, mode
    int n = 0;
    auto add = [&](int ux, int uy, int l2) {
      cus[n][0] = cx + 8 * ux;
      cus[n][1] = cy + 8 * uy;
      cus[n][2] = l2;
      cus[n][3] = uipm[uy * 4 + ux];
      ++n;
    };
    if (ul2[0] == 5) {
      add(0, 0, 5);
    } else {
      for (int q = 0; q < 4; ++q) {
        const int qx = (q & 1) * 2, qy = (q >> 1) * 2;
        if (ul2[qy * 4 + qx] == 4) {
          add(qx, qy, 4);
        } else {
          for (int r = 0; r < 4; ++r) add(qx + (r & 1), qy + (r >> 1), 3);
        }
      }
    }
    ncu = n;
  }
  if (threadIdx.x < 16) cbfs[threadIdx.x] = 0;
  // the component's work, instantiated for the luma- and the chroma-sized state (each wave
  // runs one: the branch on c is wave-uniform; both run the same two barriers)
  auto comp = [&](auto& L) {
  const int sh = c ? 1 : 0, S = c ? 16 : 32;
  const int pw = g.W >> sh, ph = g.H >> sh, bx = cx >> sh, by = cy >> sh;
  {  // stage source + neighbour borders of this component
    const uint8_t* Sp = src.plane(c, b, g);
    const uint8_t* Rp = rec.plane(c, b, g);
    for (int i = lane; i < S * S; i += 64) L.src[i] = Sp[(long)(by + i / S) * pw + bx + i % S];
    for (int i = lane; i <= 2 * S; i += 64)
      L.top[i] = Rp[(long)tv_max(0, by - 1) * pw + tv_min(pw - 1, tv_max(0, bx - 1 + i))];
    for (int i = lane; i < S; i += 64) L.left[i] = Rp[(long)tv_min(ph - 1, by + i) * pw + tv_max(0, bx - 1)];
  }
  __syncthreads();
  mark(0);  // matrix + CU list + staging
  const int qpx = c ? chroma_qp(qp, 0) : qp;
  int16_t* coefp = (c == 0 ? dec.coef_y + b * g.ysz : (c == 1 ? dec.coef_u : dec.coef_v) + b * g.csz);
  for (int k = 0; k < ncu; ++k) {
    const int x0 = cus[k][0], y0 = cus[k][1], log2 = cus[k][2];
    const int mode = cus[k][3];
    const int l2 = log2 - sh, N = 1 << l2;
    const int x = x0 >> sh, y = y0 >> sh;  // TB position (component samples)
    // --- reference samples in canonical order (bottom-left .. corner .. top-right)
    const int total = 4 * N + 1;
    // one round = 64 reference positions; the common 8x8 / 4x4 TBs (4N+1 <= 64) need one
    auto round = [&](int r) -> unsigned long long {
      const int i = lane + 64 * r;
      bool av = false;
      if (i < total) {
        int xn, yn;
        if (i < 2 * N) {
          xn = x - 1;
          yn = y + 2 * N - 1 - i;
        } else {
          xn = x - 1 + (i - 2 * N);
          yn = y - 1;
        }
        av = zscan_available(x0, y0, xn << sh, yn << sh, g.W, g.H);
        int val = 0;
        if (av) {
          if (xn >= bx && yn >= by) val = L.rec[(yn - by) * S + (xn - bx)];
          else if (yn == by - 1) val = L.top[xn - (bx - 1)];
          else val = L.left[yn - by];
        }
        L.V[i] = val;
      }
      return __ballot(av);
    };
    unsigned long long m[3] = {round(0), 0, 0};
    if (total > 64) m[1] = round(1);
    if (total > 128) m[2] = round(2);
    wave_sync();
    mark(1);  // reference samples + availability
    // --- substitution (H.265 8.4.4.2.2) as a parallel nearest-available search
    for (int i = lane; i < total; i += 64) {
      int j = -1;
      for (int w = i >> 6; w >= 0 && j < 0; --w) {
        const unsigned long long mm =
            (w == (i >> 6)) ? (m[w] & (((i & 63) == 63) ? ~0ull : ((2ull << (i & 63)) - 1))) : m[w];
        if (mm) j = w * 64 + 63 - __clzll(mm);
      }
      if (j < 0)
        for (int w = 0; w < 3 && j < 0; ++w)
          if (m[w]) j = w * 64 + __ffsll(m[w]) - 1;
      const int v = j < 0 ? 128 : L.V[j];
      if (i < 2 * N) L.L[2 * N - i] = v;
      else if (i == 2 * N) L.L[0] = L.T[0] = v;
      else L.T[i - 2 * N] = v;
    }
    wave_sync();
    mark(2);  // substitution
    const bool filt = c == 0 && intra_filter_refs(l2, mode);
    if (filt) {
      for (int i = lane; i <= 2 * N; i += 64) {
        if (i == 0) {
          L.FL[0] = L.FT[0] = (L.L[1] + 2 * L.L[0] + L.T[1] + 2) >> 2;
        } else if (i == 2 * N) {
          L.FL[i] = L.L[i];
          L.FT[i] = L.T[i];
        } else {
          L.FL[i] = (L.L[i + 1] + 2 * L.L[i] + L.L[i - 1] + 2) >> 2;
          L.FT[i] = (L.T[i + 1] + 2 * L.T[i] + L.T[i - 1] + 2) >> 2;
        }
      }
      wave_sync();
    }
    const int* RL = filt ? L.FL : L.L;
    const int* RT = filt ? L.FT : L.T;
    const int dc = mode == 1 ? intra_dc_value(RL, RT, l2) : 0;
    const int ang_a = ang.angle[mode], ang_i = ang.inv[mode];
    for (int i = lane; i < N * N; i += 64) {
      const int px = i & (N - 1), py = i >> l2;
      const int p = intra_pred_pixel_ai(RL, RT, l2, mode, ang_a, ang_i, c == 0 && N < 32, dc, px, py);
      L.pred[i] = (uint8_t)p;
      L.resid[i] = (int16_t)((int)L.src[(y - by + py) * S + (x - bx + px)] - p);
    }
    wave_sync();
    mark(3);  // filter + prediction + residual
    const int cb = wave_code_tb(L.resid, L.pred, l2, qpx, true, coefp + (long)y * pw + x, pw,
                                &L.rec[(y - by) * S + (x - bx)], S, Tm, L.tb);
    if (lane == 0 && cb) atomicOr(&cbfs[k], 1u << c);
    mark(4);  // transform / quant / inverse / recon
  }
  __syncthreads();
  mark(5);  // waiting for the other component waves
  // write the CTB reconstruction and the per-CU cbf flags back
  uint8_t* Rp = rec.plane(c, b, g) + (long)by * pw + bx;
  for (int i = lane; i < S * S; i += 64) Rp[(long)(i / S) * pw + i % S] = L.rec[i];
  };
  if (c == 0) comp(WY);
  else comp(WC[c - 1]);
  for (int k = threadIdx.x; k < ncu * 16; k += blockDim.x) {
    const int cu = k >> 4, j = k & 15, log2 = cus[cu][2], n8 = 1 << (log2 - 3);
    if (j < n8 * n8)
      dec.cbf[ub + ((cus[cu][1] >> 3) + j / n8) * g.w8 + (cus[cu][0] >> 3) + j % n8] = (uint8_t)cbfs[cu];
  }
}

void launch_intra_frame(FrameSet src, FrameSet rec, DecisionSet dec, const Geo& g, const RcTables* rc, int B,
                        hipStream_t s) {
  k_intra_analysis<<<dim3(g.wc * g.hc, B), 256, 0, s>>>(src, dec, g, rc);
  const int ndiag = (g.wc - 1) + 2 * (g.hc - 1) + 1;
  for (int d = 0; d < ndiag; ++d) {
    const int cy0 = tv_max(0, (d - (g.wc - 1) + 1) / 2);
    const int cy1 = tv_min(g.hc - 1, d / 2);
    if (cy1 < cy0) continue;
    k_intra_recon<<<dim3(cy1 - cy0 + 1, B), 192, 0, s>>>(src, rec, dec, g, d, cy0, intra_timing() ? 1 : 0);
  }
}

// ----------------------- intra 16x16 CUs in P pictures (tv/me_model.h) --------------------
// k_pintra_analysis  one wave per gated quadrant (listed by k_inter_me): the I-frame
//                    analysis' 15-mode SATD search from SOURCE neighbours, then the SAD of
//                    the chosen mode -> candidate byte (golden: tv::pintra_candidate).
// k_pintra_select    per CTB: acceptance from the candidate bytes of its neighbourhood
//                    (tv::pintra_accepted), the CTB's decisions rewritten (tv::apply_pintra),
//                    each accepted quadrant listed for its reconstruction pass.
// k_pintra_recon     pass q over the listed CTBs after k_inter_recon: quadrant q's 16x16 CU
//                    with the normative intra prediction from the reconstruction and the TB
//                    coding of k_intra_recon (one wave per component), written over the inter
//                    result.  Acceptance guarantees every neighbour it reads is final.
__global__ void __launch_bounds__(256) k_pintra_analysis(FrameSet src, DecisionSet dec, Geo g, const RcTables* rc,
                                                         PIntraBuffers pi) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int n = pi.count[0], nctu = g.wc * g.hc;
  if ((int)blockIdx.x * 4 >= n) return;  // workgroup-uniform: nothing gated for this block
  __shared__ AngleLds ang;
  __shared__ int16_t R[4][4][33];  // per wave: left, top, smoothed left, smoothed top
  __shared__ bool av[4][2][33];
  __shared__ int dcv[4];
  ang.load(threadIdx.x, 256);
  __syncthreads();
  for (int it = blockIdx.x * 4 + w; it < n; it += gridDim.x * 4) {  // wave-uniform
    const int qi = pi.gate[it], q = qi & 3, cb = qi >> 2, b = cb / nctu, ctu = cb - b * nctu;
    const Penalties& pen = rc->pen[dec.qp[b]];
    const int x = (ctu % g.wc) * 32 + (q & 1) * 16, y = (ctu / g.wc) * 32 + (q >> 1) * 16;
    const uint8_t* S = src.plane(0, b, g);
    int16_t* L = R[w][0];
    int16_t* T = R[w][1];
    wave_sync();  // the previous item's reads of this wave's LDS are done
    if (lane == 0) {
      const bool a = zscan_available(x, y, x - 1, y - 1, g.W, g.H);
      av[w][0][0] = av[w][1][0] = a;
      L[0] = T[0] = a ? S[(long)(y - 1) * g.W + x - 1] : 0;
    } else if (lane < 33) {
      const bool al = zscan_available(x, y, x - 1, y + lane - 1, g.W, g.H);
      av[w][0][lane] = al;
      L[lane] = al ? S[(long)(y + lane - 1) * g.W + x - 1] : 0;
      const bool at = zscan_available(x, y, x + lane - 1, y - 1, g.W, g.H);
      av[w][1][lane] = at;
      T[lane] = at ? S[(long)(y - 1) * g.W + x + lane - 1] : 0;
    }
    wave_sync();
    if (lane == 0) {
      intra_substitute(L, T, av[w][0], av[w][1], 16);
      dcv[w] = intra_dc_value(L, T, 4);
    }
    wave_sync();
    if (lane <= 32) {  // [1 2 1] smoothed copies
      if (lane == 0) {
        R[w][2][0] = R[w][3][0] = (int16_t)((L[1] + 2 * L[0] + T[1] + 2) >> 2);
      } else if (lane == 32) {
        R[w][2][32] = L[32];
        R[w][3][32] = T[32];
      } else {
        R[w][2][lane] = (int16_t)((L[lane + 1] + 2 * L[lane] + L[lane - 1] + 2) >> 2);
        R[w][3][lane] = (int16_t)((T[lane + 1] + 2 * T[lane] + T[lane - 1] + 2) >> 2);
      }
    }
    wave_sync();
    int sv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      sv[k] = S[(long)(y + (k >> 1) * 8 + (lane >> 3)) * g.W + x + (k & 1) * 8 + (lane & 7)];
    auto pred = [&](int mode, int k) {
      const bool filt = intra_filter_refs(4, mode);
      return intra_pred_pixel_ai(R[w][filt ? 2 : 0], R[w][filt ? 3 : 1], 4, mode, ang.angle[mode], ang.inv[mode], true,
                                 dcv[w], (k & 1) * 8 + (lane & 7), (k >> 1) * 8 + (lane >> 3));
    };
    int d0 = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) d0 += tv_abs(sv[k] - pred(1, k));
    if (!pintra_worth_search(wave_sum(d0), pen.pintra, pi.qcost[qi])) continue;  // wave-uniform
    unsigned best = 0xffffffffu, best_ang = 0xffffffffu;
    auto eval = [&](int mode) {
      int sum = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) sum += wave_satd8x8(sv[k] - pred(mode, k));
      const unsigned v = ((unsigned)(sum + (mode <= 1 ? pen.mode_dcpl : pen.mode_ang)) << 6) | (unsigned)mode;
      best = v < best ? v : best;
      if (mode >= 2) best_ang = v < best_ang ? v : best_ang;
    };
    for (int i = 0; i < kIntraCoarseModes; ++i) eval(intra_coarse_mode(i));
    const int ma = (int)(best_ang & 63);
    for (int i = 0; i < 4; ++i) {
      const int m = intra_refine_mode(ma, i);
      if (m >= 2) eval(m);
    }
    const int mode = (int)(best & 63);
    int d = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) d += tv_abs(sv[k] - pred(mode, k));
    const int sad = wave_sum(d);
    if (lane == 0 && pintra_cost(sad, pen.pintra) < pi.qcost[qi]) {
      pi.cand[qi] = (uint8_t)(0x80 | mode);
      pi.clist[atomicAdd(&pi.count[5], 1)] = qi;  // k_pintra_select walks the candidates only
    }
  }
}

// One thread per candidate quadrant (k_pintra_analysis' list).  The CTB-wide 32x32 -> 16x16
// rewrite is idempotent: whichever candidate of a CTB reads its first unit still at 32x32
// rewrites all 16 units to 16x16, and every other write sets the same values.
__global__ void __launch_bounds__(256) k_pintra_select(DecisionSet dec, Geo g, PIntraBuffers pi, int B) {
  const int n = pi.count[5], nctu = g.wc * g.hc;
  for (int it = blockIdx.x * 256 + threadIdx.x; it < n; it += gridDim.x * 256) {
    const int qi = pi.clist[it], q = qi & 3, cb = qi >> 2, b = cb / nctu, ctu = cb - b * nctu;
    const int i = ctu % g.wc, j = ctu / g.wc;
    const uint8_t* C = pi.cand + (long)b * nctu * 4;
    if (!pintra_accepted(C, g.wc, g.hc, i, j, q)) continue;
    pi.pass[q * (long)B * nctu + atomicAdd(&pi.count[1 + q], 1)] = cb;
    const long u0 = b * g.usz + (long)(j * 4) * g.w8 + i * 4;
    if (dec.cu_log2[u0] == 5)
      for (int k = 0; k < 16; ++k) dec.cu_log2[u0 + (long)(k >> 2) * g.w8 + (k & 3)] = 4;
    for (int k = 0; k < 4; ++k) {
      const long u = u0 + (long)((q >> 1) * 2 + (k >> 1)) * g.w8 + (q & 1) * 2 + (k & 1);
      dec.cu_log2[u] = 4;
      dec.intra[u] = 1;
      dec.ipm[u] = (uint8_t)(C[(long)ctu * 4 + q] & 63);
      dec.mv[2 * u] = dec.mv[2 * u + 1] = 0;
    }
  }
}

struct PIntraLds {
  uint8_t pred[256];
  int16_t resid[256];
  int V[65];
  int L[33], T[33], FL[33], FT[33];
  WaveTbScratch tb;
};

__global__ void __launch_bounds__(192) k_pintra_recon(FrameSet src, FrameSet rec, DecisionSet dec, Geo g,
                                                      PIntraBuffers pi, int q, int B) {
  const int c = threadIdx.x >> 6, lane = threadIdx.x & 63, nctu = g.wc * g.hc;
  const int n = pi.count[1 + q];
  if ((int)blockIdx.x >= n) return;  // workgroup-uniform
  __shared__ int Tm[32][33];
  __shared__ AngleLds ang;
  __shared__ PIntraLds W[3];
  __shared__ unsigned cbfs;
  tb_load_matrix(Tm);
  ang.load(threadIdx.x, 192);
  __syncthreads();
  PIntraLds& L = W[c];
  const int sh = c ? 1 : 0, l2 = 4 - sh, N = 1 << l2, total = 4 * N + 1;
  const int pw = g.W >> sh;
  for (int it = blockIdx.x; it < n; it += gridDim.x) {  // workgroup-uniform
    const int cb = pi.pass[(long)q * B * nctu + it], b = cb / nctu, ctu = cb - b * nctu;
    const int x0 = (ctu % g.wc) * 32 + (q & 1) * 16, y0 = (ctu / g.wc) * 32 + (q >> 1) * 16;
    const int mode = pi.cand[(long)cb * 4 + q] & 63, qp = dec.qp[b];
    const int x = x0 >> sh, y = y0 >> sh;
    const uint8_t* Sp = src.plane(c, b, g);
    uint8_t* Rp = rec.plane(c, b, g);
    if (threadIdx.x == 0) cbfs = 0;
    // reference samples in canonical order (bottom-left .. corner .. top-right), final
    // reconstruction read straight from the plane
    unsigned long long m[2] = {0, 0};
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int i = lane + 64 * r;
      bool a = false;
      if (i < total) {
        const int xn = i < 2 * N ? x - 1 : x - 1 + (i - 2 * N), yn = i < 2 * N ? y + 2 * N - 1 - i : y - 1;
        a = zscan_available(x0, y0, xn << sh, yn << sh, g.W, g.H);
        L.V[i] = a ? Rp[(long)yn * pw + xn] : 0;
      }
      m[r] = __ballot(a);
    }
    wave_sync();
    for (int i = lane; i < total; i += 64) {  // substitution (H.265 8.4.4.2.2): nearest available below
      int jj = -1;
      for (int wv = i >> 6; wv >= 0 && jj < 0; --wv) {
        const unsigned long long mm =
            (wv == (i >> 6)) ? (m[wv] & (((i & 63) == 63) ? ~0ull : ((2ull << (i & 63)) - 1))) : m[wv];
        if (mm) jj = wv * 64 + 63 - __clzll(mm);
      }
      if (jj < 0)
        for (int wv = 0; wv < 2 && jj < 0; ++wv)
          if (m[wv]) jj = wv * 64 + __ffsll(m[wv]) - 1;
      const int v = jj < 0 ? 128 : L.V[jj];
      if (i < 2 * N) L.L[2 * N - i] = v;
      else if (i == 2 * N) L.L[0] = L.T[0] = v;
      else L.T[i - 2 * N] = v;
    }
    wave_sync();
    const bool filt = c == 0 && intra_filter_refs(l2, mode);
    if (filt) {
      for (int i = lane; i <= 2 * N; i += 64) {
        if (i == 0) {
          L.FL[0] = L.FT[0] = (L.L[1] + 2 * L.L[0] + L.T[1] + 2) >> 2;
        } else if (i == 2 * N) {
          L.FL[i] = L.L[i];
          L.FT[i] = L.T[i];
        } else {
          L.FL[i] = (L.L[i + 1] + 2 * L.L[i] + L.L[i - 1] + 2) >> 2;
          L.FT[i] = (L.T[i + 1] + 2 * L.T[i] + L.T[i - 1] + 2) >> 2;
        }
      }
      wave_sync();
    }
    const int* RL = filt ? L.FL : L.L;
    const int* RT = filt ? L.FT : L.T;
    const int dc = mode == 1 ? intra_dc_value(RL, RT, l2) : 0;
    for (int i = lane; i < N * N; i += 64) {
      const int px = i & (N - 1), py = i >> l2;
      const int p = intra_pred_pixel_ai(RL, RT, l2, mode, (int)ang.angle[mode], (int)ang.inv[mode], c == 0, dc, px, py);
      L.pred[i] = (uint8_t)p;
      L.resid[i] = (int16_t)((int)Sp[(long)(y + py) * pw + x + px] - p);
    }
    wave_sync();
    int16_t* coefp = (c == 0 ? dec.coef_y + b * g.ysz : (c == 1 ? dec.coef_u : dec.coef_v) + b * g.csz);
    const int cbit = wave_code_tb(L.resid, L.pred, l2, c ? chroma_qp(qp, 0) : qp, true, coefp + (long)y * pw + x, pw,
                                  Rp + (long)y * pw + x, pw, Tm, L.tb);
    if (lane == 0 && cbit) atomicOr(&cbfs, 1u << c);
    __syncthreads();
    if (threadIdx.x < 4)
      dec.cbf[b * g.usz + (long)((y0 >> 3) + (threadIdx.x >> 1)) * g.w8 + (x0 >> 3) + (threadIdx.x & 1)] = (uint8_t)cbfs;
    __syncthreads();  // cbfs and the LDS are reused by the next item
  }
}

void launch_pintra_decide(FrameSet src, DecisionSet dec, const Geo& g, const RcTables* rc, const PIntraBuffers& pi,
                          int B, hipStream_t s) {
  // list-driven: a fixed grid walks the gated quadrants (the count is on the device)
  k_pintra_analysis<<<512, 256, 0, s>>>(src, dec, g, rc, pi);
  k_pintra_select<<<64, 256, 0, s>>>(dec, g, pi, B);
}

void launch_pintra_recon(FrameSet src, FrameSet rec, DecisionSet dec, const Geo& g, const PIntraBuffers& pi, int B,
                         hipStream_t s) {
  for (int q = 0; q < 4; ++q) k_pintra_recon<<<128, 192, 0, s>>>(src, rec, dec, g, pi, q, B);
}

bool intra_timing() {
  static const bool on = [] {
    const char* e = std::getenv("TV_DIAG_INTRA");
    return e && *e == '1';
  }();
  return on;
}

void intra_timing_report() {
  if (!intra_timing()) return;
  unsigned long long h[3][8];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_intra_phase), sizeof(h)) != hipSuccess) return;
  const char* names[6] = {"staging", "refs", "substitution", "pred+resid", "tb coding", "join"};
  for (int c = 0; c < 3; ++c) {
    std::fprintf(stderr, "[TV_DIAG_INTRA] wave %d:", c);
    for (int k = 0; k < 6; ++k) std::fprintf(stderr, " %s %.1fM", names[k], h[c][k] / 1e6);
    std::fprintf(stderr, "\n");
  }
}

}  // namespace gpu
}  // namespace tv
