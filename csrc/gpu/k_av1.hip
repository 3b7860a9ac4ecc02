// k_av1.hip — AV1 in-loop filter kernels for gfx950 (BASELINE config #4):
//
//   k_cdef_dir     one wavefront per 8x8 luma block (lane = pixel): partial sums of the 8
//                  directions with LDS atomics, lanes 0..7 score one direction each;
//   k_cdef_search  one workgroup per 64x64 (chroma 32x32) filter block: the block + 2-pixel
//                  halo is staged in LDS once and every thread sweeps one of the 64
//                  (primary, secondary) strength presets over a quarter of the pixels —
//                  the encoder's CDEF strength search as one launch per plane batch;
//   k_cdef_apply   the filter with the chosen per-block preset (LDS tile, pixel per thread);
//   k_wiener_*     64x64 restoration units: LDS tile with a 3-pixel halo, horizontal 7-tap
//                  pass into an LDS intermediate, vertical pass to the output; the
//                  least-squares statistics of the separable tap estimation reduce per unit
//                  (wave DPP sums, int64 LDS atomics);
//   k_sgr_*        self-guided restoration: box sums from the LDS tile, (A, B) planes in LDS
//                  per radius, 3x3 weighted guide, projection / statistics per unit.
//
// All planes are batched (B planes of w x h, pitch w, back to back; grid.y = plane) and
// every per-pixel formula comes from tv/av1_defs.h, shared with the C++ golden model
// (csrc/core/av1_tools.cpp): GPU == CPU bit for bit.
#include <hip/hip_runtime.h>

#include <string>

#include "gpu_common.h"
#include "tv/av1_defs.h"
#include "tv/av1_enc.h"

namespace tv {
namespace gpu {
namespace {

using namespace tv::av1;
constexpr int kRu = 64;

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }

// 64-bit wave sum (DPP-free: 64-bit values are rare here, per-unit reductions only)
__device__ __forceinline__ long long wave_sum64(long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ------------------------------------------------------------------------------ CDEF ----
__global__ void __launch_bounds__(256) k_cdef_dir(const uint8_t* __restrict__ Y, int w, int h, uint8_t* dir,
                                                  int* var) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, b = blockIdx.y;
  const int w8 = w >> 3, n8 = w8 * (h >> 3);
  const int blk = blockIdx.x * 4 + wave;
  __shared__ int part[4][8][16];
  __shared__ int cost[4][8];
  for (int i = lane; i < 128; i += 64) part[wave][i >> 4][i & 15] = 0;
  __syncthreads();
  if (blk < n8) {
    const int by = blk / w8, bx = blk - by * w8, i = lane >> 3, j = lane & 7;
    const int x = (int)Y[(long)b * w * h + (long)(by * 8 + i) * w + bx * 8 + j] - 128;
#pragma unroll
    for (int d = 0; d < 8; ++d) atomicAdd(&part[wave][d][cdef_bin(d, i, j)], x);
  }
  __syncthreads();
  if (blk < n8 && lane < 8) cost[wave][lane] = cdef_cost(part[wave][lane], lane);
  __syncthreads();
  if (blk < n8 && lane == 0) {
    int v;
    dir[(long)b * n8 + blk] = (uint8_t)cdef_pick(cost[wave], &v);
    var[(long)b * n8 + blk] = v;
  }
}

constexpr int kFbMax = 64, kHalo = 2, kTile = kFbMax + 2 * kHalo;

// Stage filter block `fb` (+halo) of plane b in LDS as int16 (-1 = outside the frame).
__device__ __forceinline__ void cdef_stage(const uint8_t* P, int w, int h, int x0, int y0, int fbw, int fbh,
                                           int16_t (*T)[kTile]) {
  const int tw = fbw + 2 * kHalo, th = fbh + 2 * kHalo;
  for (int i = threadIdx.x; i < tw * th; i += blockDim.x) {
    const int ty = i / tw, tx = i - ty * tw, y = y0 + ty - kHalo, x = x0 + tx - kHalo;
    T[ty][tx] = (x >= 0 && x < w && y >= 0 && y < h) ? (int16_t)P[(long)y * w + x] : (int16_t)-1;
  }
}

// cdef_filter (av1_defs.h) on taps gathered into registers: P[k][sign] primary, S[k][sign][o]
// secondary (directions d -/+ 2); -1 = unavailable.  Same taps, same integer result.
__device__ __forceinline__ int cdef_eval(int c, const int (&P)[2][2], const int (&S)[2][2][2], int pri, int sec,
                                         int damping) {
  int sum = 0, mx = c, mn = c;
  const int pt = pri & 1;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int ptap = pt ? 3 : (k ? 2 : 4), stap = k ? 1 : 2;
#pragma unroll
    for (int sg = 0; sg < 2; ++sg) {
      if (pri) {
        const int v = P[k][sg];
        if (v >= 0) {
          sum += ptap * cdef_constrain(v - c, pri, damping);
          mx = v > mx ? v : mx;
          mn = v < mn ? v : mn;
        }
      }
      if (sec) {
#pragma unroll
        for (int o = 0; o < 2; ++o) {
          const int v = S[k][sg][o];
          if (v >= 0) {
            sum += stap * cdef_constrain(v - c, sec, damping);
            mx = v > mx ? v : mx;
            mn = v < mn ? v : mn;
          }
        }
      }
    }
  }
  const int y0 = c + ((8 + sum - (sum < 0)) >> 4);
  return clip3(mn, mx, y0);
}

__device__ __forceinline__ int cdef_tile_filter(const int16_t (*T)[kTile], int ty, int tx, int pri, int sec, int dmp,
                                                int d) {
  auto get = [&](int dy, int dx) -> int { return T[ty + dy][tx + dx]; };
  return cdef_filter(get, T[ty][tx], pri, sec, dmp, d);
}

__global__ void __launch_bounds__(256) k_cdef_search(const uint8_t* __restrict__ src, const uint8_t* __restrict__ rec,
                                                     int w, int h, int chroma, const uint8_t* __restrict__ dir,
                                                     const int* __restrict__ var, int luma_w8, int luma_n8,
                                                     int damping, unsigned long long* sse, unsigned long long pmask,
                                                     int checker) {
  const int b = blockIdx.y, fb = blockIdx.x;
  const int bs_l2 = chroma ? 2 : 3, fbs = chroma ? 32 : 64, nfx = (w + fbs - 1) / fbs;
  const int x0 = (fb % nfx) * fbs, y0 = (fb / nfx) * fbs;
  const int fbw = min(fbs, w - x0), fbh = min(fbs, h - y0);
  const int dmp = chroma ? damping - 1 : damping;
  __shared__ int16_t T[kTile][kTile];
  __shared__ unsigned long long acc[kCdefPresets];
  const long po = (long)b * w * h;
  cdef_stage(rec + po, w, h, x0, y0, fbw, fbh, T);
  if (threadIdx.x < kCdefPresets) acc[threadIdx.x] = 0;
  __syncthreads();
  // Pixel-major: each thread gathers a pixel's 12 CDEF taps from the tile once and
  // evaluates up to 16 presets of pmask from registers (cdef_eval = cdef_filter's
  // arithmetic on the gathered taps), so the LDS is read once per pixel and chunk.
  __shared__ int8_t plist[kCdefPresets];
  if (threadIdx.x == 0)
    for (int k = 0, n = 0; k < kCdefPresets; ++k)
      if (pmask >> k & 1) plist[n++] = (int8_t)k;
  __syncthreads();
  // measured blocks of this filter block (all, or the (bx + by)-even checkerboard), listed
  // so the threads stream only over their pixels
  __shared__ uint8_t blist[64];
  __shared__ int nbl;
  const int bsz = 1 << bs_l2, ppb = bsz * bsz;
  if (threadIdx.x == 0) {
    int n = 0;
    for (int by = 0; by < (fbh >> bs_l2); ++by)
      for (int bx = 0; bx < (fbw >> bs_l2); ++bx)
        if (!checker || !((bx + by) & 1)) blist[n++] = (uint8_t)(by * 8 + bx);
    nbl = n;
  }
  __syncthreads();
  const int np = __popcll(pmask), npx = nbl * ppb;
  for (int c0 = 0; c0 < np; c0 += 16) {
    const int nc = min(16, np - c0);
    unsigned a16[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) a16[k] = 0;
    for (int q = threadIdx.x; q < npx; q += 256) {
      const int bk = blist[q / ppb], pq = q - (q / ppb) * ppb;
      const int i = (bk >> 3) * bsz + pq / bsz, j = (bk & 7) * bsz + (pq & (bsz - 1)), x = x0 + j, y = y0 + i;
      const long kb = (long)b * luma_n8 + (y >> bs_l2) * luma_w8 + (x >> bs_l2);
      const int d0 = dir[kb], d = d0 & 7, vr = chroma ? 0 : var[kb];
      const bool skip = d0 & kCdefSkipBlock;
      const int ty = i + kHalo, tx = j + kHalo, c = T[ty][tx];
      // taps along the block direction, plus the secondary taps of direction 0 (presets
      // whose primary strength is 0 filter along directions 2 / 6: cdef_dir_used)
      int P[2][2], Sd[2][2][2], S0[2][2][2];
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int sg = 0; sg < 2; ++sg) {
          const int m = sg ? 1 : -1;
          P[k][sg] = T[ty + m * cdef_dir_dy(d, k)][tx + m * cdef_dir_dx(d, k)];
#pragma unroll
          for (int o = 0; o < 2; ++o) {
            const int d2 = (d + (o ? 2 : -2)) & 7, z2 = o ? 2 : 6;
            Sd[k][sg][o] = T[ty + m * cdef_dir_dy(d2, k)][tx + m * cdef_dir_dx(d2, k)];
            S0[k][sg][o] = T[ty + m * cdef_dir_dy(z2, k)][tx + m * cdef_dir_dx(z2, k)];
          }
        }
      const int e0 = (int)src[po + (long)y * w + x];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        if (k >= nc) break;
        const int pp = plist[c0 + k];
        const int psec = cdef_sec_value(pp & 3), ppri = pp >> 2;
        const int pri = chroma ? ppri : cdef_adjust_strength(ppri, vr);
        const int f = (!skip && (pri | psec)) ? cdef_eval(c, P, ppri ? Sd : S0, pri, psec, dmp) : c;
        const int e = f - e0;
        a16[k] += (unsigned)(e * e);
      }
    }
    for (int k = 0; k < nc; ++k) {
      const unsigned v = a16[k];
      if (v) atomicAdd(&acc[plist[c0 + k]], (unsigned long long)v);
    }
  }
  __syncthreads();
  const int nfb = nfx * ((h + fbs - 1) / fbs);
  if (threadIdx.x < kCdefPresets)
    sse[((long)b * nfb + fb) * kCdefPresets + threadIdx.x] =
        (pmask >> threadIdx.x & 1) ? acc[threadIdx.x] : (unsigned long long)kCdefSkipped;
}

__global__ void __launch_bounds__(256) k_cdef_apply(const uint8_t* __restrict__ rec, int w, int h, int chroma,
                                                    const uint8_t* __restrict__ dir, const int* __restrict__ var,
                                                    int luma_w8, int luma_n8, int damping,
                                                    const int8_t* __restrict__ fb_preset, uint8_t* out) {
  const int b = blockIdx.y, fb = blockIdx.x;
  const int bs_l2 = chroma ? 2 : 3, fbs = chroma ? 32 : 64, nfx = (w + fbs - 1) / fbs;
  const int nfb = nfx * ((h + fbs - 1) / fbs);
  const int x0 = (fb % nfx) * fbs, y0 = (fb / nfx) * fbs;
  const int fbw = min(fbs, w - x0), fbh = min(fbs, h - y0);
  const int dmp = chroma ? damping - 1 : damping;
  const int p = fb_preset[(long)b * nfb + fb];
  const long po = (long)b * w * h;
  __shared__ int16_t T[kTile][kTile];
  cdef_stage(rec + po, w, h, x0, y0, fbw, fbh, T);
  __syncthreads();
  for (int q = threadIdx.x; q < fbw * fbh; q += blockDim.x) {
    const int i = q / fbw, j = q - i * fbw, x = x0 + j, y = y0 + i;
    const long k = (long)b * luma_n8 + (y >> bs_l2) * luma_w8 + (x >> bs_l2);
    const int d0 = dir[k];
    int pri = 0, sec = 0;
    if (p >= 0 && !(d0 & kCdefSkipBlock)) {
      sec = cdef_sec_value(p & 3);
      pri = chroma ? (p >> 2) : cdef_adjust_strength(p >> 2, var[k]);
    }
    out[po + (long)y * w + x] = (uint8_t)((pri | sec) ? cdef_tile_filter(T, i + kHalo, j + kHalo, pri, sec, dmp,
                                                                         cdef_dir_used(p, d0))
                                                       : T[i + kHalo][j + kHalo]);
  }
}

// ---------------------------------------------------------------------- Wiener ----------
constexpr int kLrHalo = 3, kLrTile = kRu + 2 * kLrHalo;  // 70

// rec tile of unit (ux, uy) with edge-replicated 3-pixel halo
__device__ __forceinline__ void lr_stage(const uint8_t* P, int w, int h, int ux, int uy, int uw, int uh,
                                         uint8_t (*T)[kLrTile]) {
  const int tw = uw + 2 * kLrHalo, th = uh + 2 * kLrHalo;
  for (int i = threadIdx.x; i < tw * th; i += blockDim.x) {
    const int ty = i / tw, tx = i - ty * tw;
    T[ty][tx] = P[(long)clampi(uy + ty - kLrHalo, 0, h - 1) * w + clampi(ux + tx - kLrHalo, 0, w - 1)];
  }
}

__global__ void __launch_bounds__(256) k_wiener_apply(const uint8_t* __restrict__ rec, int w, int h,
                                                      const int* __restrict__ coef, uint8_t* out) {
  const int b = blockIdx.y, u = blockIdx.x, nux = (w + kRu - 1) / kRu, nu = nux * ((h + kRu - 1) / kRu);
  const int ux = (u % nux) * kRu, uy = (u / nux) * kRu, uw = min(kRu, w - ux), uh = min(kRu, h - uy);
  const long po = (long)b * w * h;
  __shared__ uint8_t T[kLrTile][kLrTile];
  __shared__ int mid[kLrTile][kRu];
  __shared__ int c[6];
  if (threadIdx.x < 6) c[threadIdx.x] = coef[((long)b * nu + u) * 6 + threadIdx.x];
  lr_stage(rec + po, w, h, ux, uy, uw, uh, T);
  __syncthreads();
  const bool id = !(c[0] | c[1] | c[2] | c[3] | c[4] | c[5]);
  if (id) {
    for (int q = threadIdx.x; q < uw * uh; q += blockDim.x) {
      const int i = q / uw, j = q - i * uw;
      out[po + (long)(uy + i) * w + ux + j] = T[i + kLrHalo][j + kLrHalo];
    }
    return;
  }
  for (int q = threadIdx.x; q < (uh + 6) * uw; q += blockDim.x) {
    const int r = q / uw, j = q - r * uw;
    mid[r][j] = wiener_h([&](int t) -> int { return T[r][j + t]; }, c);
  }
  __syncthreads();
  for (int q = threadIdx.x; q < uw * uh; q += blockDim.x) {
    const int i = q / uw, j = q - i * uw;
    out[po + (long)(uy + i) * w + ux + j] = (uint8_t)wiener_v(&mid[i][j], kRu, c + 3);
  }
}

__global__ void __launch_bounds__(256) k_wiener_stats(const uint8_t* __restrict__ src, const uint8_t* __restrict__ rec,
                                                      int w, int h, int dirn, const int* __restrict__ other,
                                                      long long* stats) {
  const int b = blockIdx.y, u = blockIdx.x, nux = (w + kRu - 1) / kRu, nu = nux * ((h + kRu - 1) / kRu);
  const int ux = (u % nux) * kRu, uy = (u / nux) * kRu, uw = min(kRu, w - ux), uh = min(kRu, h - uy);
  const long po = (long)b * w * h;
  __shared__ uint8_t T[kLrTile][kLrTile];
  __shared__ int Z[kLrTile][kLrTile];  // z on the unit extended by 3 along the estimation direction
  __shared__ int c[3];
  __shared__ unsigned long long red[9];
  if (threadIdx.x < 3) c[threadIdx.x] = other[((long)b * nu + u) * 3 + threadIdx.x];
  if (threadIdx.x < 9) red[threadIdx.x] = 0;
  lr_stage(rec + po, w, h, ux, uy, uw, uh, T);
  __syncthreads();
  // z at tile position (r, s): plane coordinate clamp(uy + r - 3), clamp(ux + s - 3)
  const int zw = dirn == 0 ? uw + 6 : uw, zh = dirn == 0 ? uh : uh + 6;
  for (int q = threadIdx.x; q < zw * zh; q += blockDim.x) {
    const int r = q / zw, s = q - r * zw;
    const int ty = dirn == 0 ? r + kLrHalo : r, tx = dirn == 0 ? s : s + kLrHalo;  // tile coords of the sample
    // the tile halo is edge-replicated, so tile neighbours == clamped plane neighbours
    Z[ty][tx] = dirn == 0 ? lr_tap_filter([&](int t) -> int { return T[ty + t - 3][tx]; }, c)
                          : lr_tap_filter([&](int t) -> int { return T[ty][tx + t - 3]; }, c);
  }
  __syncthreads();
  long long a[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (int q = threadIdx.x; q < uw * uh; q += blockDim.x) {
    const int i = q / uw, j = q - i * uw, ty = i + kLrHalo, tx = j + kLrHalo;
    // neighbour along the estimation direction, clamped at the frame border
    auto at = [&](int d) -> int {
      if (dirn == 0) {
        const int x = clampi(ux + j + d, 0, w - 1);
        return Z[ty][x - ux + kLrHalo];
      }
      const int y = clampi(uy + i + d, 0, h - 1);
      return Z[y - uy + kLrHalo][tx];
    };
    const int zc = at(0);
    const int f0 = at(-3) + at(3) - 2 * zc, f1 = at(-2) + at(2) - 2 * zc, f2 = at(-1) + at(1) - 2 * zc;
    const long long e = 128LL * ((int)src[po + (long)(uy + i) * w + ux + j] - zc);
    a[0] += f0 * f0;
    a[1] += f0 * f1;
    a[2] += f0 * f2;
    a[3] += f1 * f1;
    a[4] += f1 * f2;
    a[5] += f2 * f2;
    a[6] += f0 * e;
    a[7] += f1 * e;
    a[8] += f2 * e;
  }
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const long long v = wave_sum64(a[k]);
    if ((threadIdx.x & 63) == 0) atomicAdd(&red[k], (unsigned long long)v);
  }
  __syncthreads();
  if (threadIdx.x < 9) stats[((long)b * nu + u) * 9 + threadIdx.x] = (long long)red[threadIdx.x];
}

// ----------------------------------------------------------------- self-guided ----------
constexpr int kAb = kRu + 2;  // A/B planes cover the unit + 1

// guided output (RST domain) for the unit's pixels, radius r, into F (registers, 16/thread)
__device__ void sgr_guided(const uint8_t (*T)[kLrTile], int w, int h, int ux, int uy, int uw, int uh, int r, int eps,
                           uint16_t (*A)[kAb], uint16_t (*Bv)[kAb], const uint16_t* xt, int* F) {
  // A/B at plane positions clamp(uy - 1 + i), clamp(ux - 1 + j): box sums around the clamped
  // position over clamped coordinates (tile halo covers +-3 around the unit)
  for (int q = threadIdx.x; q < (uw + 2) * (uh + 2); q += blockDim.x) {
    const int i = q / (uw + 2), j = q - i * (uw + 2);
    const int cy = clampi(uy - 1 + i, 0, h - 1), cx = clampi(ux - 1 + j, 0, w - 1);
    int s = 0, sq = 0;
    for (int dy = -r; dy <= r; ++dy)
      for (int dx = -r; dx <= r; ++dx) {
        const int yy = clampi(cy + dy, 0, h - 1), xx = clampi(cx + dx, 0, w - 1);
        const int v = T[yy - uy + kLrHalo][xx - ux + kLrHalo];
        s += v;
        sq += v * v;
      }
    int a, bb;
    sgr_ab_x(s, sq, r, eps, [&](unsigned z) -> int { return xt[z < 255u ? z : 255u]; }, &a, &bb);
    A[i][j] = (uint16_t)a;
    Bv[i][j] = (uint16_t)bb;
  }
  __syncthreads();
  int n = 0;
  for (int q = threadIdx.x; q < uw * uh; q += blockDim.x, ++n) {
    const int i = q / uw, j = q - i * uw;
    int a = 0, bb = 0;
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        const int wt = (dx && dy) ? 3 : 4;
        // neighbour (clamped in the plane) -> A/B index
        const int yy = clampi(uy + i + dy, 0, h - 1) - uy + 1, xx = clampi(ux + j + dx, 0, w - 1) - ux + 1;
        a += wt * A[yy][xx];
        bb += wt * Bv[yy][xx];
      }
    const int sh = kSgrSgrBits + 5 - kSgrRstBits;
    F[n] = (a * (int)T[i + kLrHalo][j + kLrHalo] + bb + (1 << (sh - 1))) >> sh;
  }
  __syncthreads();
}

template <bool kStats>
__global__ void __launch_bounds__(256) k_sgr(const uint8_t* __restrict__ src, const uint8_t* __restrict__ rec, int w,
                                             int h, int set_all, const int* __restrict__ params, long long* stats,
                                             uint8_t* out) {
  const int b = blockIdx.y, u = blockIdx.x, nux = (w + kRu - 1) / kRu, nu = nux * ((h + kRu - 1) / kRu);
  const int ux = (u % nux) * kRu, uy = (u / nux) * kRu, uw = min(kRu, w - ux), uh = min(kRu, h - uy);
  const long po = (long)b * w * h;
  __shared__ uint8_t T[kLrTile][kLrTile];
  __shared__ uint16_t A[kAb][kAb], Bv[kAb][kAb], xt[256];
  __shared__ unsigned long long red[5];
  const int* pr = kStats ? nullptr : params + ((long)b * nu + u) * 3;
  const int set = kStats ? set_all : pr[0];
  if (!kStats && set < 0) {  // unit off: copy
    for (int q = threadIdx.x; q < uw * uh; q += blockDim.x) {
      const int i = q / uw, j = q - i * uw;
      out[po + (long)(uy + i) * w + ux + j] = rec[po + (long)(uy + i) * w + ux + j];
    }
    return;
  }
  lr_stage(rec + po, w, h, ux, uy, uw, uh, T);
  if (threadIdx.x < 256) xt[threadIdx.x] = (uint16_t)sgr_xbyx1(threadIdx.x);
  if (kStats && threadIdx.x < 5) red[threadIdx.x] = 0;
  __syncthreads();
  const int r0 = sgr_param(set, 0), r1 = sgr_param(set, 2);
  int f0[16], f1[16];
  int n = 0;
  for (int q = threadIdx.x; q < uw * uh; q += blockDim.x, ++n) {
    const int i = q / uw, j = q - i * uw;
    f0[n] = f1[n] = (int)T[i + kLrHalo][j + kLrHalo] << kSgrRstBits;
  }
  if (r0) sgr_guided(T, w, h, ux, uy, uw, uh, r0, sgr_param(set, 1), A, Bv, xt, f0);
  if (r1) sgr_guided(T, w, h, ux, uy, uw, uh, r1, sgr_param(set, 3), A, Bv, xt, f1);
  long long a[5] = {0, 0, 0, 0, 0};
  n = 0;
  for (int q = threadIdx.x; q < uw * uh; q += blockDim.x, ++n) {
    const int i = q / uw, j = q - i * uw;
    const int x = (int)T[i + kLrHalo][j + kLrHalo];
    if (kStats) {
      const int uu = x << kSgrRstBits;
      const long long da = f0[n] - uu, db = f1[n] - uu;
      const long long e = ((long long)(((int)src[po + (long)(uy + i) * w + ux + j]) << kSgrRstBits) - uu)
                          << kSgrPrjBits;
      a[0] += da * da;
      a[1] += da * db;
      a[2] += db * db;
      a[3] += da * e;
      a[4] += db * e;
    } else {
      out[po + (long)(uy + i) * w + ux + j] = (uint8_t)sgr_project(x, f0[n], f1[n], r0, r1, pr[1], pr[2]);
    }
  }
  if (kStats) {
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      const long long v = wave_sum64(a[k]);
      if ((threadIdx.x & 63) == 0) atomicAdd(&red[k], (unsigned long long)v);
    }
    __syncthreads();
    if (threadIdx.x < 5) stats[((long)b * nu + u) * 5 + threadIdx.x] = (long long)red[threadIdx.x];
  }
}

// Encoder restoration search for one parameter set, fused: guided filters once per unit,
// projection statistics -> integer solve (sgr_solve, shared with the golden encoder) ->
// projection + unit SSE vs the source, restored unit written to `out`.  Replaces the
// stats / solve / apply / SSE launch chain (one filter pass instead of two).
__global__ void __launch_bounds__(256) k_sgr_search(const uint8_t* __restrict__ src, const uint8_t* __restrict__ rec,
                                                    int w, int h, int set, int* __restrict__ prm,
                                                    long long* __restrict__ sse, uint8_t* __restrict__ out) {
  const int b = blockIdx.y, u = blockIdx.x, nux = (w + kRu - 1) / kRu, nu = nux * ((h + kRu - 1) / kRu);
  const int ux = (u % nux) * kRu, uy = (u / nux) * kRu, uw = min(kRu, w - ux), uh = min(kRu, h - uy);
  const long po = (long)b * w * h;
  __shared__ uint8_t T[kLrTile][kLrTile];
  __shared__ uint16_t A[kAb][kAb], Bv[kAb][kAb], xt[256];
  __shared__ unsigned long long red[6];
  __shared__ int xq[2];
  lr_stage(rec + po, w, h, ux, uy, uw, uh, T);
  if (threadIdx.x < 256) xt[threadIdx.x] = (uint16_t)sgr_xbyx1(threadIdx.x);
  if (threadIdx.x < 6) red[threadIdx.x] = 0;
  __syncthreads();
  const int r0 = sgr_param(set, 0), r1 = sgr_param(set, 2);
  int f0[16], f1[16];
  int n = 0;
  for (int q = threadIdx.x; q < uw * uh; q += blockDim.x, ++n) {
    const int i = q / uw, j = q - i * uw;
    f0[n] = f1[n] = (int)T[i + kLrHalo][j + kLrHalo] << kSgrRstBits;
  }
  if (r0) sgr_guided(T, w, h, ux, uy, uw, uh, r0, sgr_param(set, 1), A, Bv, xt, f0);
  if (r1) sgr_guided(T, w, h, ux, uy, uw, uh, r1, sgr_param(set, 3), A, Bv, xt, f1);
  long long a[5] = {0, 0, 0, 0, 0};
  n = 0;
  for (int q = threadIdx.x; q < uw * uh; q += blockDim.x, ++n) {
    const int i = q / uw, j = q - i * uw;
    const int uu = (int)T[i + kLrHalo][j + kLrHalo] << kSgrRstBits;
    const long long da = f0[n] - uu, db = f1[n] - uu;
    const long long e = ((long long)(((int)src[po + (long)(uy + i) * w + ux + j]) << kSgrRstBits) - uu) << kSgrPrjBits;
    a[0] += da * da;
    a[1] += da * db;
    a[2] += db * db;
    a[3] += da * e;
    a[4] += db * e;
  }
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const long long v = wave_sum64(a[k]);
    if ((threadIdx.x & 63) == 0) atomicAdd(&red[k], (unsigned long long)v);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    long long st[5];
    for (int k = 0; k < 5; ++k) st[k] = (long long)red[k];
    sgr_solve(st, r0, r1, &xq[0], &xq[1]);
    int* P = prm + ((long)b * nu + u) * 3;
    P[0] = set;
    P[1] = xq[0];
    P[2] = xq[1];
  }
  __syncthreads();
  const int w0 = xq[0], w1 = xq[1];
  long long e2 = 0;
  n = 0;
  for (int q = threadIdx.x; q < uw * uh; q += blockDim.x, ++n) {
    const int i = q / uw, j = q - i * uw;
    const int x = (int)T[i + kLrHalo][j + kLrHalo];
    const int o = sgr_project(x, f0[n], f1[n], r0, r1, w0, w1);
    out[po + (long)(uy + i) * w + ux + j] = (uint8_t)o;
    const int d = o - (int)src[po + (long)(uy + i) * w + ux + j];
    e2 += d * d;
  }
  const long long v = wave_sum64(e2);
  if ((threadIdx.x & 63) == 0) atomicAdd(&red[5], (unsigned long long)v);
  __syncthreads();
  if (threadIdx.x == 0) sse[(long)b * nu + u] = (long long)red[5];
}

// Encoder restoration choice per normative restoration unit (av1_defs.h lr_* geometry; 7.17
// stripes), fused over the candidate sets of lr_set(): the unit's SSE unrestored, then per
// set the guided filters -> projection statistics -> sgr_solve -> projection SSE; the first
// minimum of SSE + rate (rate[b] = lr_rate_cost of segment b's q-index, 0 when unrestored)
// wins and only the winner is written.  The golden encoder's decision (av1_codec.cpp) bit for
// bit.
//
// Layout: 512 threads own the unit's pixels (q = tid + 512 n, row-major) in registers: the
// CDEF | source samples and, per set, the packed guided outputs F0 | F1 << 16.  Per stripe
// chunk the source tile (CDEF output inside the stripe, up to 2 deblocked rows beyond it,
// clamped at the plane edges) is staged in LDS ONCE for every set (batched loads, all in
// flight together), the box sums of a pass are computed once and turned into the (A, B)
// planes of every set that uses the pass (the radius-1 sums serve sets 4 and 10 alike), and
// each thread filters its own pixels straight into registers (no F plane in LDS); A and B
// share one LDS word.  LDS ~60 KB.
constexpr int kLrCh = 64, kLrUw = 96;  // max stripe chunk height, max unit width (round layout)
constexpr int kLrTw = kLrUw + 6, kLrAw = kLrUw + 2;
constexpr int kLrThreads = 1024, kLrMaxPx = 104 * 96, kLrPer = (kLrMaxPx + kLrThreads - 1) / kLrThreads;  // unit <= 103 x 95
constexpr int kLrBatch = 5;  // tile loads per thread in flight together

// q / d for 0 <= q < 2^20, 1 <= d <= 128 by a float reciprocal: (q + 0.5) / d lies >= 0.5 / d
// away from an integer, far beyond the float error
__device__ __forceinline__ int lr_div(int q, float rd) { return (int)(((float)q + 0.5f) * rd); }
// a value the compiler must treat as unknown at this point: keeps it from hoisting the 20
// per-pixel (row, column) pairs out of the chunk loop into live registers
__device__ __forceinline__ float lr_opaque(float v) {
  asm volatile("" : "+v"(v));
  return v;
}

__global__ void __launch_bounds__(kLrThreads) k_sgr_select(const uint8_t* __restrict__ src, const uint8_t* __restrict__ cdef,
                                                       const uint8_t* __restrict__ dbk, int w, int h, int ss,
                                                       const long long* __restrict__ rate, int* __restrict__ prm,
                                                       uint8_t* __restrict__ out) {
  const int b = blockIdx.y, u = blockIdx.x, nux = lr_count_units(w);
  const int ur = u / nux, uc = u - ur * nux, nu = nux * lr_count_units(h);
  int x0, x1, y0, y1;
  lr_unit_cols(uc, w, &x0, &x1);
  lr_unit_rows(ur, h, ss, &y0, &y1);
  const int uw = x1 - x0, npx = (y1 - y0) * uw, S = 64 >> ss, aw = uw + 2, tw = uw + 6;
  const float ruw = 1.f / (float)uw, raw = 1.f / (float)aw, rtw = 1.f / (float)tw;
  const long po = (long)b * w * h;
  const uint8_t* C = cdef + po;
  const uint8_t* D = dbk + po;
  __shared__ uint8_t T[kLrCh + 6][kLrTw];
  __shared__ uint32_t AB[kNumLrSets][kLrCh + 2][kLrAw];  // A | B << 16
  __shared__ uint16_t xt[256];
  __shared__ unsigned long long red[1 + 6 * kNumLrSets];
  __shared__ int xq[kNumLrSets][2];
  if (threadIdx.x < 256) xt[threadIdx.x] = (uint16_t)sgr_xbyx1(threadIdx.x);
  if (threadIdx.x < 1 + 6 * kNumLrSets) red[threadIdx.x] = 0;
  auto block_add = [&](long long v, int slot) {
    v = wave_sum64(v);
    if ((threadIdx.x & 63) == 0) atomicAdd(&red[slot], (unsigned long long)v);
  };
  // xp: CDEF | source << 8 of pixel n in half-word n & 1 of xp[n >> 1]
  uint32_t xp[(kLrPer + 1) / 2], fv[kNumLrSets][kLrPer];
#define XS(n) ((xp[(n) >> 1] >> (((n) & 1) * 16)) & 0xFFFFu)
  long long e0 = 0;
#pragma unroll
  for (int n = 0; n < kLrPer; ++n) {
    const int q = threadIdx.x + kLrThreads * n;
    if (!(n & 1)) xp[n >> 1] = 0;
    if (n % 5 == 0) asm volatile("" ::: "memory");  // at most 5 pixels' loads in flight: bounds the address registers
    if (q < npx) {
      const int i = lr_div(q, ruw), j = q - i * uw;
      const long o = (long)(y0 + i) * w + x0 + j;
      const int c = C[o], sv = src[po + o];
      xp[n >> 1] |= ((uint32_t)c | ((uint32_t)sv << 8)) << ((n & 1) * 16);
      e0 += (c - sv) * (c - sv);
    }
    const uint32_t uu = (XS(n) & 255) << kSgrRstBits;  // a radius-0 pass outputs the sample itself
#pragma unroll
    for (int k = 0; k < kNumLrSets; ++k) fv[k][n] = uu | (uu << 16);
  }
  for (int s0 = lr_stripe_start(y0, ss); s0 < y1; s0 += S) {
    const int ya = s0 > y0 ? s0 : y0, yb = s0 + S < y1 ? s0 + S : y1, ntl = (yb - ya + 6) * tw;
    for (int q0 = threadIdx.x; q0 < ntl; q0 += kLrThreads * kLrBatch) {  // kLrBatch loads in flight
      uint8_t tv[kLrBatch];
#pragma unroll
      for (int n = 0; n < kLrBatch; ++n) {
        const int q = q0 + kLrThreads * n;
        if (q < ntl) {
          const int ty = lr_div(q, rtw), tx = q - ty * tw;
          bool db;
          const int yy = lr_src_row(ya - 3 + ty, h, s0, ss, &db), xx = clampi(x0 - 3 + tx, 0, w - 1);
          tv[n] = (db ? D : C)[(long)yy * w + xx];
        }
      }
#pragma unroll
      for (int n = 0; n < kLrBatch; ++n) {
        const int q = q0 + kLrThreads * n;
        if (q < ntl) {
          const int ty = lr_div(q, rtw);
          T[ty][q - ty * tw] = tv[n];
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      bool used = false;
#pragma unroll
      for (int k = 0; k < kNumLrSets; ++k) used |= sgr_param(lr_set(k), 2 * pass) != 0;
      if (!used) continue;
      // (A, B) rows y in [ya - 1, yb + 1) (pass 0: odd rows only) x columns [x0 - 1, x1 + 1)
      const int r = pass ? 1 : 2, step = pass ? 1 : 2, fy = pass ? ya - 1 : ((ya - 1) | 1);
      const int nr = pass ? yb - ya + 2 : (yb + 1 - fy + 1) >> 1;
      for (int q = threadIdx.x; q < nr * aw; q += kLrThreads) {
        const int ri = lr_div(q, raw), j = q - ri * aw, i = fy + step * ri - (ya - 1);
        int sum = 0, sq = 0;
        for (int dy = -r; dy <= r; ++dy)
          for (int dx = -r; dx <= r; ++dx) {
            const int v = T[i + 2 + dy][j + 2 + dx];
            sum += v;
            sq += v * v;
          }
#pragma unroll
        for (int k = 0; k < kNumLrSets; ++k) {
          if (!sgr_param(lr_set(k), 2 * pass)) continue;
          int a, bb;
          sgr_ab_x(sum, sq, r, sgr_param(lr_set(k), 2 * pass + 1),
                   [&](unsigned z) -> int { return xt[z < 255u ? z : 255u]; }, &a, &bb);
          AB[k][i][j] = (uint32_t)a | ((uint32_t)bb << 16);
        }
      }
      __syncthreads();
      const float ru = lr_opaque(ruw);
#pragma unroll
      for (int n = 0; n < kLrPer; ++n) {
        const int q = threadIdx.x + kLrThreads * n;
        const int i = lr_div(q, ru), j = q - i * uw, yy = y0 + i, ci = yy - ya;
        if (q >= npx || yy < ya || yy >= yb) continue;
        const int c = XS(n) & 255;
#pragma unroll
        for (int k = 0; k < kNumLrSets; ++k) {
          if (!sgr_param(lr_set(k), 2 * pass)) continue;
          uint32_t nb[3][3];  // one LDS read per neighbour for both coefficients
#pragma unroll
          for (int dy = 0; dy < 3; ++dy)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx)
              nb[dy][dx] = (pass || ((yy + dy - 1) & 1)) ? AB[k][ci + dy][j + dx] : 0u;
          const uint32_t f = (uint16_t)sgr_output(
              pass, yy, c, [&](int dy, int dx) -> int { return nb[dy + 1][dx + 1] & 0xFFFF; },
              [&](int dy, int dx) -> int { return nb[dy + 1][dx + 1] >> 16; });
          fv[k][n] = pass ? (fv[k][n] & 0xFFFFu) | (f << 16) : (fv[k][n] & 0xFFFF0000u) | f;
        }
      }
      __syncthreads();  // A / B (and T after pass 1) reused next
    }
  }
  // projection statistics of every set -> solve
  block_add(e0, 0);
#pragma unroll
  for (int k = 0; k < kNumLrSets; ++k) {
    // |F - u| < 2^12: the squares and cross term fit 32 bits per pixel and per thread (<= 20
    // pixels); the source correlation terms (<< kSgrPrjBits) need 64
    int q00 = 0, q01 = 0, q11 = 0;
    long long q0e = 0, q1e = 0;
#pragma unroll
    for (int n = 0; n < kLrPer; ++n) {
      if (threadIdx.x + kLrThreads * n >= npx) continue;
      const int uu = (int)(XS(n) & 255) << kSgrRstBits;
      const int da = (int)(int16_t)(fv[k][n] & 0xFFFF) - uu, db = (int)(int16_t)(fv[k][n] >> 16) - uu;
      const int e = ((int)(XS(n) >> 8) << kSgrRstBits) - uu;
      q00 += da * da;
      q01 += da * db;
      q11 += db * db;
      q0e += (long long)(da * e);
      q1e += (long long)(db * e);
    }
    const long long acc[5] = {q00, q01, q11, q0e << kSgrPrjBits, q1e << kSgrPrjBits};
#pragma unroll
    for (int c = 0; c < 5; ++c) block_add(acc[c], 1 + 6 * k + c);
  }
  __syncthreads();
  if (threadIdx.x < kNumLrSets) {
    const int k = threadIdx.x, set = lr_set(k);
    long long st[5];
    for (int c = 0; c < 5; ++c) st[c] = (long long)red[1 + 6 * k + c];
    sgr_solve(st, sgr_param(set, 0), sgr_param(set, 2), &xq[k][0], &xq[k][1]);
  }
  __syncthreads();
  // projection SSE of every set; the winner is written from the registers
#pragma unroll
  for (int k = 0; k < kNumLrSets; ++k) {
    const int set = lr_set(k), r0 = sgr_param(set, 0), r1 = sgr_param(set, 2), w0 = xq[k][0], w1 = xq[k][1];
    long long e2 = 0;
#pragma unroll
    for (int n = 0; n < kLrPer; ++n) {
      if (threadIdx.x + kLrThreads * n >= npx) continue;
      const int v = sgr_project_xqd(XS(n) & 255, (int16_t)(fv[k][n] & 0xFFFF), (int16_t)(fv[k][n] >> 16), r0, r1, w0, w1);
      const int d = v - (int)(XS(n) >> 8);
      e2 += d * d;
    }
    block_add(e2, 1 + 6 * k + 5);
  }
  __syncthreads();
  long long best = (long long)red[0];
  int bk = -1;
  const long long rt = rate[b];
  for (int k = 0; k < kNumLrSets; ++k)
    if ((long long)red[1 + 6 * k + 5] + rt < best) {  // block-uniform
      best = (long long)red[1 + 6 * k + 5] + rt;
      bk = k;
    }
  const float ru = lr_opaque(ruw);  // recompute (row, column): not kept live from the first loop
#pragma unroll
  for (int n = 0; n < kLrPer; ++n) {
    const int q = threadIdx.x + kLrThreads * n;
    if (q >= npx) continue;
    const int i = lr_div(q, ru), j = q - i * uw, x = XS(n) & 255;
    int v = x;
#pragma unroll
    for (int k = 0; k < kNumLrSets; ++k)
      if (k == bk)
        v = sgr_project_xqd(x, (int16_t)(fv[k][n] & 0xFFFF), (int16_t)(fv[k][n] >> 16), sgr_param(lr_set(k), 0),
                            sgr_param(lr_set(k), 2), xq[k][0], xq[k][1]);
    out[po + (long)(y0 + i) * w + x0 + j] = (uint8_t)v;
  }
  if (threadIdx.x == 0) {
    int* P = prm + ((long)b * nu + u) * 3;
    P[0] = bk < 0 ? -1 : lr_set(bk);
    P[1] = bk < 0 ? 0 : xq[bk][0];
    P[2] = bk < 0 ? 0 : xq[bk][1];
  }
}
#undef XS

// ----------------------------------------------------------------- deblocking filter ----
// k_deblock: one workgroup per 64x64 output tile.  The tile plus an 8-pixel ring is staged
// in LDS once (dword loads); the vertical edges x0..x0+64 are filtered on all 80 rows (the
// ring rows feed the horizontal taps), then the horizontal edges y0..y0+64 on the tile's
// 64 columns, and the 64x64 interior is written back — both passes of AV1 7.14 in one
// launch with one HBM read and one write per pixel.  Edges of a pass never share taps
// (av1_defs.h lf_edge), so every (line, edge) item of a pass is independent.
constexpr int kLfT = 64, kLfR = 8, kLfP = kLfT + 2 * kLfR;  // tile, ring, LDS pitch (80)

__global__ void __launch_bounds__(256) k_deblock(const uint8_t* __restrict__ in, uint8_t* __restrict__ out, int w,
                                                 int h, int chroma, const uint32_t* __restrict__ info, int sharp,
                                                 int estep) {
  __shared__ __attribute__((aligned(16))) uint8_t T[kLfP * kLfP];
  const int x0 = blockIdx.x * kLfT, y0 = blockIdx.y * kLfT, b = blockIdx.z, w4 = w >> 2;
  const uint8_t* P = in + (long)b * w * h;
  const uint32_t* I = info + (long)b * w4 * (h >> 2);
  for (int i = threadIdx.x; i < kLfP * (kLfP / 4); i += blockDim.x) {
    const int r = i / (kLfP / 4), c4 = i - r * (kLfP / 4), y = y0 - kLfR + r, x = x0 - kLfR + c4 * 4;
    uint32_t v = 0;
    if (y >= 0 && y < h && x >= 0 && x < w) v = *(const uint32_t*)(P + (long)y * w + x);
    *(uint32_t*)(T + r * kLfP + c4 * 4) = v;
  }
  __syncthreads();
  // pass 0: vertical edges x0, x0 + estep, .., x0 + 64 (17 at estep 4) x 80 rows; item =
  // edge * 80 + row.  estep > 4 when every transform / block edge of the plane lies on that
  // grid (the AV1 encoder: 16 luma, 8 chroma): the skipped positions hold no edge.
  const int ne = kLfT / estep + 1;
  for (int i = threadIdx.x; i < ne * kLfP; i += blockDim.x) {
    const int e = i / kLfP, r = i - e * kLfP, y = y0 - kLfR + r, x = x0 + e * estep;
    if (y < 0 || y >= h || x >= w) continue;
    const uint32_t* row = I + (long)(y >> 2) * w4;
    int lvl = 0;
    const int size = lf_edge(x > 0 ? row[(x >> 2) - 1] : 0u, row[x >> 2], x, w, 0, chroma, &lvl);
    if (size) lf_filter(T + r * kLfP + kLfR + e * estep, 1, size, lvl, sharp);
  }
  __syncthreads();
  // pass 1: horizontal edges y0 .. y0+64 (step estep) x 64 columns; item = edge * 64 + column
  for (int i = threadIdx.x; i < ne * kLfT; i += blockDim.x) {
    const int e = i / kLfT, c = i - e * kLfT, y = y0 + e * estep, x = x0 + c;
    if (y >= h || x >= w) continue;
    int lvl = 0;
    const int size = lf_edge(y > 0 ? I[(long)((y >> 2) - 1) * w4 + (x >> 2)] : 0u, I[(long)(y >> 2) * w4 + (x >> 2)],
                             y, h, 1, chroma, &lvl);
    if (size) lf_filter(T + (kLfR + e * estep) * kLfP + kLfR + c, kLfP, size, lvl, sharp);
  }
  __syncthreads();
  uint8_t* O = out + (long)b * w * h;
  for (int i = threadIdx.x; i < kLfT * (kLfT / 4); i += blockDim.x) {
    const int r = i / (kLfT / 4), c4 = i - r * (kLfT / 4), y = y0 + r, x = x0 + c4 * 4;
    if (y < h && x < w) *(uint32_t*)(O + (long)y * w + x) = *(const uint32_t*)(T + (kLfR + r) * kLfP + kLfR + c4 * 4);
  }
}

thread_local std::string g_av1_gpu_err;
int av1_status(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e == hipSuccess) return 0;
  g_av1_gpu_err = std::string(what) + ": " + hipGetErrorString(e);
  return -1;
}
bool bad_geo(int w, int h, int B, int mult, const char* what) {
  if (w < mult || h < mult || (w % mult) || (h % mult) || B < 1 || B > 65535) {
    g_av1_gpu_err = std::string(what) + ": bad geometry";
    return true;
  }
  return false;
}
inline unsigned nunits(int w, int h) { return (unsigned)(((w + kRu - 1) / kRu) * ((h + kRu - 1) / kRu)); }

}  // namespace
}  // namespace gpu
}  // namespace tv

using namespace tv::gpu;

extern "C" {
const char* tv_av1_gpu_last_error() { return g_av1_gpu_err.c_str(); }

// B luma planes (w, h multiples of 8) -> dir/var [B][w/8 * h/8]
int tv_gpu_cdef_dirs(const uint8_t* Y, int w, int h, int B, uint8_t* dir, int* var, void* stream) {
  if (bad_geo(w, h, B, 8, "cdef_dirs")) return -1;
  const int n8 = (w / 8) * (h / 8);
  k_cdef_dir<<<dim3((n8 + 3) / 4, B), 256, 0, (hipStream_t)stream>>>(Y, w, h, dir, var);
  return av1_status("cdef_dirs");
}
// sse: [B][nfb][64] (uint64)
int tv_gpu_cdef_search(const uint8_t* src, const uint8_t* rec, int w, int h, int B, int chroma, const uint8_t* dir,
                       const int* var, int luma_w8, int luma_n8, int damping, unsigned long long* sse, void* stream,
                       unsigned long long pmask, int checker) {
  if (bad_geo(w, h, B, chroma ? 4 : 8, "cdef_search") || damping < 3 || damping > 6 || !pmask) return -1;
  const int fbs = chroma ? 32 : 64, nfb = ((w + fbs - 1) / fbs) * ((h + fbs - 1) / fbs);
  k_cdef_search<<<dim3(nfb, B), 256, 0, (hipStream_t)stream>>>(src, rec, w, h, chroma, dir, var, luma_w8, luma_n8,
                                                               damping, sse, pmask, checker);
  return av1_status("cdef_search");
}
int tv_gpu_cdef_apply(const uint8_t* rec, int w, int h, int B, int chroma, const uint8_t* dir, const int* var,
                      int luma_w8, int luma_n8, int damping, const int8_t* fb_preset, uint8_t* out, void* stream) {
  if (bad_geo(w, h, B, chroma ? 4 : 8, "cdef_apply") || damping < 3 || damping > 6) return -1;
  const int fbs = chroma ? 32 : 64, nfb = ((w + fbs - 1) / fbs) * ((h + fbs - 1) / fbs);
  k_cdef_apply<<<dim3(nfb, B), 256, 0, (hipStream_t)stream>>>(rec, w, h, chroma, dir, var, luma_w8, luma_n8, damping,
                                                              fb_preset, out);
  return av1_status("cdef_apply");
}
// encoder restoration search of set `set`: prm [B][nu][3], unit SSE [B][nu], restored planes
int tv_gpu_sgr_search(const uint8_t* src, const uint8_t* rec, int w, int h, int B, int set, int* prm, long long* sse,
                      uint8_t* out, void* stream) {
  if (bad_geo(w, h, B, 2, "sgr_search") || set < 0 || set > 15) return -1;
  k_sgr_search<<<dim3(nunits(w, h), B), 256, 0, (hipStream_t)stream>>>(src, rec, w, h, set, prm, sse, out);
  return av1_status("sgr_search");
}
// encoder restoration choice over every lr_set() candidate: rate [B] (int64), prm
// [B][nu][3], restored planes (unrestored units copied).  lr_count_units rounding keeps every
// unit within 95 columns x 103 rows, the kernel's register / LDS footprint
int tv_gpu_sgr_select(const uint8_t* src, const uint8_t* cdef, const uint8_t* dbk, int w, int h, int ss, int B,
                      const long long* rate, int* prm, uint8_t* out, void* stream) {
  if (bad_geo(w, h, B, 2, "sgr_select") || ss < 0 || ss > 1) return -1;
  const int nu = lr_count_units(w) * lr_count_units(h);
  k_sgr_select<<<dim3(nu, B), kLrThreads, 0, (hipStream_t)stream>>>(src, cdef, dbk, w, h, ss, rate, prm, out);
  return av1_status("sgr_select");
}
int tv_gpu_wiener_apply(const uint8_t* rec, int w, int h, int B, const int* coef, uint8_t* out, void* stream) {
  if (bad_geo(w, h, B, 2, "wiener_apply")) return -1;
  k_wiener_apply<<<dim3(nunits(w, h), B), 256, 0, (hipStream_t)stream>>>(rec, w, h, coef, out);
  return av1_status("wiener_apply");
}
int tv_gpu_wiener_stats(const uint8_t* src, const uint8_t* rec, int w, int h, int B, int dir, const int* other,
                        long long* stats, void* stream) {
  if (bad_geo(w, h, B, 2, "wiener_stats")) return -1;
  k_wiener_stats<<<dim3(nunits(w, h), B), 256, 0, (hipStream_t)stream>>>(src, rec, w, h, dir, other, stats);
  return av1_status("wiener_stats");
}
int tv_gpu_sgr_stats(const uint8_t* src, const uint8_t* rec, int w, int h, int B, int set, long long* stats,
                     void* stream) {
  if (bad_geo(w, h, B, 2, "sgr_stats") || set < 0 || set > 15) return -1;
  k_sgr<true><<<dim3(nunits(w, h), B), 256, 0, (hipStream_t)stream>>>(src, rec, w, h, set, nullptr, stats, nullptr);
  return av1_status("sgr_stats");
}
// B planes (w, h multiples of 4), info [B][h/4][w/4] (av1_defs.h layout), sharp 0..7
// estep: edge grid in samples (4 = every 4x4 boundary; 8 / 16 only when all transform and
// block edges of the plane lie on that grid)
int tv_gpu_av1_deblock_step(const uint8_t* in, uint8_t* out, int w, int h, int B, int chroma, const uint32_t* info,
                            int sharp, int estep, void* stream) {
  if (bad_geo(w, h, B, 4, "av1_deblock") || sharp < 0 || sharp > 7 || (estep != 4 && estep != 8 && estep != 16))
    return -1;
  k_deblock<<<dim3((w + kLfT - 1) / kLfT, (h + kLfT - 1) / kLfT, B), 256, 0, (hipStream_t)stream>>>(in, out, w, h,
                                                                                                  chroma, info, sharp,
                                                                                                  estep);
  return av1_status("av1_deblock");
}
int tv_gpu_av1_deblock(const uint8_t* in, uint8_t* out, int w, int h, int B, int chroma, const uint32_t* info,
                       int sharp, void* stream) {
  return tv_gpu_av1_deblock_step(in, out, w, h, B, chroma, info, sharp, 4, stream);
}
int tv_gpu_sgr_apply(const uint8_t* rec, int w, int h, int B, const int* params, uint8_t* out, void* stream) {
  if (bad_geo(w, h, B, 2, "sgr_apply")) return -1;
  k_sgr<false><<<dim3(nunits(w, h), B), 256, 0, (hipStream_t)stream>>>(nullptr, rec, w, h, 0, params, nullptr, out);
  return av1_status("sgr_apply");
}
}
