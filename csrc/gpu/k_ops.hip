// k_ops.hip — pre-processing kernels of the transcode pipeline:
//
//  k_resize_h / k_resize_v   separable windowed-sinc (Lanczos-a) resampling of one plane.
//                            Filter tables (start index + Q14 taps per output coordinate,
//                            widened by the scale ratio when down-scaling, i.e. ffmpeg
//                            `scale=-2:H:flags=lanczos` semantics) are built on the host.
//                            H pass: a 256-wide row tile of the source is staged in LDS and
//                            every lane reads its taps from LDS; V pass reads the int16
//                            intermediate column-coalesced.
//  k_rgb_to_i420             packed RGB24 -> I420, BT.601/BT.709, limited range; one thread
//                            per 2x2 block (chroma = mean of the 4 converted pixels).
//  k_p010_to_i420            10-bit P010 (semi-planar, MSB aligned) -> 8-bit I420 (rounding).
//  k_tonemap_pq              HDR10 (P010, BT.2020 PQ) -> SDR I420 BT.709: PQ EOTF, BT.2390
//                            EETF roll-off (knee on max-RGB), BT.2020->709 gamut matrix,
//                            BT.709 OETF; one thread per 2x2 block.
//  k_overlay_mask            burn a host-rasterised label mask (0 keep / 1 border / 2 glyph)
//                            into a batch of frames (reference `drawtext text=%{n}`,
//                            worker/tasks.py:2377-2395).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>
#include <string>

namespace tv {
namespace ops {

__device__ __forceinline__ int clampi(int v, int lo, int hi) { return v < lo ? lo : (v > hi ? hi : v); }
__device__ __forceinline__ uint8_t sat8(int v) { return (uint8_t)clampi(v, 0, 255); }

constexpr int kTile = 256;

// ---------------------------------------------------------------- resize (H pass)
// tmp[y][x] = sum_k w[x][k] * src[y][ix[x]+k]  (Q14 weights, result kept at Q6 in int16)
// blockIdx.z = frame of a batch (source frame stride sfs, tmp frame stride tfs).
__global__ void __launch_bounds__(kTile) k_resize_h(const uint8_t* __restrict__ src, int sw, int sstride, long sfs,
                                                    int16_t* __restrict__ tmp, long tfs, int dw,
                                                    const int* __restrict__ ix, const int16_t* __restrict__ wx,
                                                    int taps) {
  __shared__ uint8_t row[kTile * 8 + 64];
  const int y = blockIdx.y, x0 = blockIdx.x * kTile, x = x0 + threadIdx.x;
  const uint8_t* s = src + blockIdx.z * sfs + (long)y * sstride;
  tmp += blockIdx.z * tfs;
  // source span touched by this tile of outputs
  const int lo = ix[x0];
  const int hi = ix[min(x0 + kTile, dw) - 1] + taps;  // exclusive
  const int span = hi - lo;
  const bool staged = span <= (int)sizeof(row);
  if (staged)
    for (int i = threadIdx.x; i < span; i += kTile) row[i] = s[clampi(lo + i, 0, sw - 1)];
  __syncthreads();
  if (x >= dw) return;
  const int b = ix[x];
  const int16_t* w = wx + (long)x * taps;
  int acc = 0;
  if (staged) {
    for (int k = 0; k < taps; ++k) acc += w[k] * row[b + k - lo];
  } else {
    for (int k = 0; k < taps; ++k) acc += w[k] * s[clampi(b + k, 0, sw - 1)];
  }
  tmp[(long)y * dw + x] = (int16_t)clampi((acc + (1 << 7)) >> 8, -32768, 32767);  // Q14 -> Q6
}

// ---------------------------------------------------------------- resize (V pass)
// Writes a pw x ph (>= dw x dh) output: columns/rows past the picture replicate its last
// column/row, i.e. the edge padding an encoder wants up to its coded size comes for free.
__global__ void __launch_bounds__(kTile) k_resize_v(const int16_t* __restrict__ tmp, long tfs, int sh, int dw,
                                                    uint8_t* __restrict__ dst, long dfs, int dstride, int dh, int pw,
                                                    int ph, const int* __restrict__ iy,
                                                    const int16_t* __restrict__ wy, int taps) {
  const int x = blockIdx.x * kTile + threadIdx.x, y = blockIdx.y;
  if (x >= pw || y >= ph) return;
  const int xs = min(x, dw - 1), ys = min(y, dh - 1);
  tmp += blockIdx.z * tfs;
  const int b = iy[ys];
  const int16_t* w = wy + (long)ys * taps;
  int acc = 0;
  for (int k = 0; k < taps; ++k) acc += w[k] * tmp[(long)clampi(b + k, 0, sh - 1) * dw + xs];
  dst[blockIdx.z * dfs + (long)y * dstride + x] = sat8((acc + (1 << 19)) >> 20);  // Q14 * Q6 -> Q0
}

// ------------------------------------------------------- fused 2-D resize (batched)
// One workgroup = a 64 x TH output tile of one frame (blockIdx.z): the clamped source window
// it needs is staged in LDS once, the H pass writes its rows x 64 int16 intermediate to LDS,
// the V pass reads it from there — no global int16 round trip (the two-pass kernels above
// write + re-read sh x dw x 2 bytes per plane).  Same arithmetic and clamping as
// k_resize_h/k_resize_v, so the result is bit-identical; output columns/rows past dw/dh
// replicate the last ones (edge padding to pw x ph).  LDS: R x Wp source bytes + R x 64 x 2
// intermediate, R/Wp chosen by the host from the tables (resize2d_plan in models/abr.py).
constexpr int kR2W = 64;
template <int MAXT>
__global__ void __launch_bounds__(256) k_resize2d(const uint8_t* __restrict__ src, int sw, int sh, int sstride,
                                                  long sfs, uint8_t* __restrict__ dst, int dw, int dh, int dstride,
                                                  long dfs, int pw, int ph, int th, int wp,
                                                  const int* __restrict__ ix, const int16_t* __restrict__ wx, int tx,
                                                  const int* __restrict__ iy, const int16_t* __restrict__ wy,
                                                  int ty) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int x0 = blockIdx.x * kR2W, y0 = blockIdx.y * th;
  src += blockIdx.z * sfs;
  dst += blockIdx.z * dfs;
  const int xa = min(x0, dw - 1), xb = min(x0 + kR2W - 1, dw - 1);
  const int ya = min(y0, dh - 1), yb = min(y0 + th - 1, dh - 1);
  const int clo = ix[xa], W = ix[xb] + tx - clo;
  const int rlo = iy[ya], R = iy[yb] + ty - rlo;
  uint8_t* ssrc = smem;                                                   // R x wp
  int16_t* stmp = reinterpret_cast<int16_t*>(smem + ((R * wp + 15) & ~15));  // R x 64
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int r = wv; r < R; r += 4) {
    const uint8_t* s = src + (long)clampi(rlo + r, 0, sh - 1) * sstride;
    for (int c = lane; c < W; c += 64) ssrc[r * wp + c] = s[clampi(clo + c, 0, sw - 1)];
  }
  __syncthreads();
  {
    // a lane's output column is fixed for every row: its taps live in registers
    const int x = min(x0 + lane, dw - 1);
    const int b = ix[x] - clo;
    int wr[MAXT];
#pragma unroll
    for (int k = 0; k < MAXT; ++k) wr[k] = k < tx ? wx[(long)x * tx + k] : 0;
    for (int r = wv; r < R; r += 4) {
      const uint8_t* s = ssrc + r * wp + b;
      int acc = 0;
#pragma unroll
      for (int k = 0; k < MAXT; ++k)
        if (k < tx) acc += wr[k] * s[k];
      stmp[r * kR2W + lane] = (int16_t)clampi((acc + (1 << 7)) >> 8, -32768, 32767);  // Q14 -> Q6
    }
  }
  __syncthreads();
  const int x = x0 + lane;
  if (x >= pw) return;
  // one output row per wave per iteration: row index, filter start and taps are wave-uniform
  // (scalar loads)
  for (int yl = __builtin_amdgcn_readfirstlane(wv); yl < th; yl += 4) {
    const int y = y0 + yl;
    if (y >= ph) break;
    const int ys = min(y, dh - 1);
    const int b = iy[ys] - rlo;
    const int16_t* w = wy + (long)ys * ty;
    int acc = 0;
    for (int k = 0; k < ty; ++k) acc += w[k] * stmp[(b + k) * kR2W + lane];
    dst[(long)y * dstride + x] = sat8((acc + (1 << 19)) >> 20);  // Q14 * Q6 -> Q0
  }
}

// ------------------------------------------------------------------- RGB -> I420
struct YuvMat {
  float ry, gy, by, ru, gu, bu, rv, gv, bv;
};
__device__ __forceinline__ YuvMat yuv_mat(int bt709) {
  // limited range: Y = 16 + 219*Y', C = 128 + 224*C'
  if (bt709) return {0.2126f, 0.7152f, 0.0722f, -0.1146f, -0.3854f, 0.5f, 0.5f, -0.4542f, -0.0458f};
  return {0.299f, 0.587f, 0.114f, -0.168736f, -0.331264f, 0.5f, 0.5f, -0.418688f, -0.081312f};
}

__global__ void k_rgb_to_i420(const uint8_t* __restrict__ rgb, int w, int h, int stride, uint8_t* __restrict__ Y,
                              uint8_t* __restrict__ U, uint8_t* __restrict__ V, int bt709) {
  const int cx = blockIdx.x * blockDim.x + threadIdx.x, cy = blockIdx.y;
  if (cx >= w / 2 || cy >= h / 2) return;
  const YuvMat m = yuv_mat(bt709);
  float su = 0.f, sv = 0.f;
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int x = 2 * cx + i, y = 2 * cy + j;
      const uint8_t* p = rgb + (long)y * stride + 3 * x;
      const float r = p[0] / 255.f, g = p[1] / 255.f, b = p[2] / 255.f;
      Y[(long)y * w + x] = sat8(__float2int_rn(16.f + 219.f * (m.ry * r + m.gy * g + m.by * b)));
      su += m.ru * r + m.gu * g + m.bu * b;
      sv += m.rv * r + m.gv * g + m.bv * b;
    }
  U[(long)cy * (w / 2) + cx] = sat8(__float2int_rn(128.f + 224.f * su * 0.25f));
  V[(long)cy * (w / 2) + cx] = sat8(__float2int_rn(128.f + 224.f * sv * 0.25f));
}

// ------------------------------------------------------------------ P010 -> I420
__global__ void k_p010_to_i420(const uint16_t* __restrict__ y16, const uint16_t* __restrict__ uv16, int w, int h,
                               uint8_t* __restrict__ Y, uint8_t* __restrict__ U, uint8_t* __restrict__ V) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= w || y >= h) return;
  Y[(long)y * w + x] = (uint8_t)min(255, ((y16[(long)y * w + x] >> 6) + 2) >> 2);
  if (!(x & 1) && !(y & 1)) {
    const long c = (long)(y >> 1) * w + x;  // interleaved UV row of w samples
    const long o = (long)(y >> 1) * (w >> 1) + (x >> 1);
    U[o] = (uint8_t)min(255, ((uv16[c] >> 6) + 2) >> 2);
    V[o] = (uint8_t)min(255, ((uv16[c + 1] >> 6) + 2) >> 2);
  }
}

// --------------------------------------------------------------- HDR10 tone-map
// x^y for x >= 0, y > 0 on the transcendental unit: v_log_f32 + v_exp_f32 (~1 ulp each)
// instead of the ~40-instruction libm powf; the tone-map does 12 per pixel and was the
// ladder's top pre-processing kernel (27 ms / 16 8K frames with powf).
__device__ __forceinline__ float fpow(float x, float y) {
  return __builtin_amdgcn_exp2f(y * __builtin_amdgcn_logf(x));
}
__device__ __forceinline__ float pq_eotf(float e) {  // -> linear, 1.0 = 10000 nits
  const float m1 = 0.1593017578125f, m2 = 78.84375f, c1 = 0.8359375f, c2 = 18.8515625f, c3 = 18.6875f;
  const float p = fpow(fminf(fmaxf(e, 0.f), 1.f), 1.f / m2);  // PQ signal is in [0, 1]
  return fpow(fmaxf(p - c1, 0.f) * __builtin_amdgcn_rcpf(c2 - c3 * p), 1.f / m1);
}
__device__ __forceinline__ float pq_oetf(float l) {
  const float m1 = 0.1593017578125f, m2 = 78.84375f, c1 = 0.8359375f, c2 = 18.8515625f, c3 = 18.6875f;
  const float p = powf(fmaxf(l, 0.f), m1);
  return powf((c1 + c2 * p) / (1.f + c3 * p), m2);
}
__device__ __forceinline__ float bt709_oetf(float l) {
  l = fminf(fmaxf(l, 0.f), 1.f);
  return l < 0.018f ? 4.5f * l : 1.099f * fpow(l, 0.45f) - 0.099f;
}
// BT.2390 EETF on PQ-encoded luminance: source peak src_pq, target peak dst_pq
__device__ __forceinline__ float eetf(float e, float src_pq, float dst_pq) {
  const float inv = __builtin_amdgcn_rcpf(src_pq);
  const float en = e * inv, maxl = dst_pq * inv;
  const float ks = 1.5f * maxl - 0.5f;
  float o = en;
  if (en > ks) {
    const float t = (en - ks) * __builtin_amdgcn_rcpf(1.f - ks), t2 = t * t, t3 = t2 * t;
    o = (2 * t3 - 3 * t2 + 1) * ks + (t3 - 2 * t2 + t) * (1.f - ks) + (-2 * t3 + 3 * t2) * maxl;
  }
  return o * src_pq;
}

// blockIdx.z = frame of a batch: P010 frames back to back (luma w*h, chroma w*h/2 samples),
// output planes advance by ofs bytes per frame.
__global__ void k_tonemap_pq(const uint16_t* __restrict__ y16, const uint16_t* __restrict__ uv16, int w, int h,
                             uint8_t* __restrict__ Y, uint8_t* __restrict__ U, uint8_t* __restrict__ V, long ofs,
                             float src_peak_nits, float dst_peak_nits) {
  const int cx = blockIdx.x * blockDim.x + threadIdx.x, cy = blockIdx.y;
  if (cx >= w / 2 || cy >= h / 2) return;
  const long z = blockIdx.z;
  y16 += z * w * h;
  uv16 += z * w * h / 2;
  Y += z * ofs;
  U += z * ofs;
  V += z * ofs;
  const long c = (long)cy * w + 2 * cx;
  // limited-range 10-bit chroma
  const float cb = ((uv16[c] >> 6) - 512.f) * (1.f / 896.f), cr = ((uv16[c + 1] >> 6) - 512.f) * (1.f / 896.f);
  const float src_pq = pq_oetf(src_peak_nits / 10000.f), dst_pq = pq_oetf(dst_peak_nits / 10000.f);
  const float lm_floor = pq_eotf(1e-6f);
  const YuvMat m = yuv_mat(1);
  float su = 0.f, sv = 0.f;
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int x = 2 * cx + i, y = 2 * cy + j;
      const float yp = ((y16[(long)y * w + x] >> 6) - 64.f) * (1.f / 876.f);
      // BT.2020 NCL Y'CbCr -> R'G'B' (PQ)
      float r = yp + 1.4746f * cr, g = yp - 0.16455f * cb - 0.57135f * cr, b = yp + 1.8814f * cb;
      // tone-map on max(R,G,B) in the PQ domain, scale linear RGB by the luminance ratio
      const float mx = fmaxf(fmaxf(r, g), fmaxf(b, 1e-6f));
      const float lt = pq_eotf(eetf(mx, src_pq, dst_pq));
      const float r0 = pq_eotf(r), g0 = pq_eotf(g), b0 = pq_eotf(b);
      const float lm = fmaxf(fmaxf(r0, g0), fmaxf(b0, lm_floor));  // == pq_eotf(mx): monotonic
      const float sc = lm > 1e-6f ? lt * __builtin_amdgcn_rcpf(lm) : 0.f;  // near-black: no ratio blow-up
      const float norm = 10000.f / dst_peak_nits;  // target peak -> 1.0
      const float R = r0 * sc * norm, G = g0 * sc * norm, B = b0 * sc * norm;
      // BT.2020 -> BT.709 primaries (linear)
      const float r7 = 1.6605f * R - 0.5876f * G - 0.0728f * B;
      const float g7 = -0.1246f * R + 1.1329f * G - 0.0083f * B;
      const float b7 = -0.0182f * R - 0.1006f * G + 1.1187f * B;
      const float rr = bt709_oetf(r7), gg = bt709_oetf(g7), bb = bt709_oetf(b7);
      Y[(long)y * w + x] = sat8(__float2int_rn(16.f + 219.f * (m.ry * rr + m.gy * gg + m.by * bb)));
      su += m.ru * rr + m.gu * gg + m.bu * bb;
      sv += m.rv * rr + m.gv * gg + m.bv * bb;
    }
  U[(long)cy * (w / 2) + cx] = sat8(__float2int_rn(128.f + 224.f * su * 0.25f));
  V[(long)cy * (w / 2) + cx] = sat8(__float2int_rn(128.f + 224.f * sv * 0.25f));
}

// ------------------------------------------------------- synthetic HDR10 source
// Seeded procedural P010 (BT.2020 PQ, limited range) frames for the ABR-ladder benchmark:
// smooth gradients, coarse + fine texture and sparse ~1000-nit highlights, translated by
// (3, 1) pixels per frame so motion search has real work.  One thread per 2x2 block,
// blockIdx.z = frame (t = t0 + z).
__device__ __forceinline__ uint32_t hash3(uint32_t x, uint32_t y, uint32_t s) {
  uint32_t h = x * 0x8da6b343u ^ y * 0xd8163841u ^ s * 0xcb1ab31fu;
  h ^= h >> 15;
  h *= 0x2c1b3c6du;
  h ^= h >> 12;
  h *= 0x297a2d39u;
  return h ^ (h >> 15);
}

__global__ void k_synth_p010(uint16_t* __restrict__ y16, uint16_t* __restrict__ uv16, int w, int h, int t0,
                             uint32_t seed) {
  const int cx = blockIdx.x * blockDim.x + threadIdx.x, cy = blockIdx.y;
  if (cx >= w / 2 || cy >= h / 2) return;
  const long z = blockIdx.z;
  const int t = t0 + (int)z;
  y16 += z * w * h;
  uv16 += z * w * h / 2;
  const int px = 2 * cx + 3 * t, py = 2 * cy + t;  // pattern coordinates (global motion)
  const float base = 0.36f + 0.2f * __sinf(px * 0.0041f + py * 0.0023f) + 0.1f * __sinf(py * 0.0107f - px * 0.0031f);
  const uint32_t cell = hash3((uint32_t)px >> 6, (uint32_t)py >> 6, seed);
  const float hi = (cell & 15u) == 0u ? 0.34f : 0.f;  // sparse highlight tiles (~1000 nits)
  const float coarse = ((hash3((uint32_t)px >> 3, (uint32_t)py >> 3, seed + 1u) & 255u) / 255.f - 0.5f) * 0.07f;
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float fine = ((hash3((uint32_t)(px + i), (uint32_t)(py + j), seed + 2u) & 15u) / 15.f - 0.5f) * 0.012f;
      const float yv = fminf(fmaxf(base + hi + coarse + fine, 0.f), 1.f);
      y16[(long)(2 * cy + j) * w + 2 * cx + i] = (uint16_t)((64 + __float2int_rn(yv * 876.f)) << 6);
    }
  const float cb = 0.09f * __sinf(px * 0.0019f + t * 0.01f) + ((cell >> 4) & 7u) * 0.004f;
  const float cr = 0.07f * __cosf(py * 0.0027f) - ((cell >> 8) & 7u) * 0.003f;
  const long c = (long)cy * w + 2 * cx;
  uv16[c] = (uint16_t)((512 + __float2int_rn(cb * 896.f)) << 6);
  uv16[c + 1] = (uint16_t)((512 + __float2int_rn(cr * 896.f)) << 6);
}

// ---------------------------------------------------------------- label overlay
// frames: n x (Y | U | V) I420 at w x h; masks: n x (mh x mw), placed at (x0, y0) (even).
__global__ void k_overlay_mask(uint8_t* __restrict__ frames, int w, int h, const uint8_t* __restrict__ masks,
                               int mw, int mh, int x0, int y0) {
  const int mx = blockIdx.x * blockDim.x + threadIdx.x, my = blockIdx.y, f = blockIdx.z;
  if (mx >= mw || my >= mh) return;
  const int x = x0 + mx, y = y0 + my;
  if (x < 0 || y < 0 || x >= w || y >= h) return;
  const uint8_t m = masks[((long)f * mh + my) * mw + mx];
  if (!m) return;
  uint8_t* Y = frames + (long)f * (w * h * 3 / 2);
  Y[(long)y * w + x] = m == 2 ? 235 : 16;
  if (!(x & 1) && !(y & 1)) {
    uint8_t* U = Y + (long)w * h;
    uint8_t* V = U + (long)(w / 2) * (h / 2);
    U[(long)(y / 2) * (w / 2) + x / 2] = 128;
    V[(long)(y / 2) * (w / 2) + x / 2] = 128;
  }
}


// ---------------------------------------------------------------- bwdif deinterlace
// Bob-Weaver deinterlacing of one plane, one output frame per input frame (reference
// `bwdif=mode=send_frame`, worker/tasks.py:62-63): lines of the kept field are copied, each
// missing line is predicted temporally from the same-parity lines of the two frames around
// it (prev2/next2), refined by an edge-aware spatial interpolator (4-tap, or a 5-line
// low/high-frequency blend when the vertical edge is strong) and clamped to the temporal
// uncertainty `diff` widened by the spatial check.
__device__ __forceinline__ void bwdif_px(const uint8_t* __restrict__ prev, const uint8_t* __restrict__ cur,
                                         const uint8_t* __restrict__ next, uint8_t* __restrict__ out, int w, int h,
                                         int keep, int x, int y) {
  const long o = (long)y * w + x;
  if ((y & 1) == keep || y < 2 || y >= h - 2) {  // kept field (and border lines: bob)
    if ((y & 1) == keep) {
      out[o] = cur[o];
    } else {
      const int up = y > 0 ? cur[o - w] : cur[o + w], dn = y < h - 1 ? cur[o + w] : cur[o - w];
      out[o] = (uint8_t)((up + dn + 1) >> 1);
    }
    return;
  }
  // same-parity temporal neighbours: the missing line lies between prev's and cur's field
  const uint8_t* p2 = prev;
  const uint8_t* n2 = cur;
  auto at = [&](const uint8_t* f, int dy) { return (int)f[(long)clampi(y + dy, 0, h - 1) * w + x]; };
  const int c = at(cur, -1), e = at(cur, 1);
  const int d = (at(p2, 0) + at(n2, 0)) >> 1;
  const int td0 = abs(at(p2, 0) - at(n2, 0));
  const int td1 = (abs(at(prev, -1) - c) + abs(at(prev, 1) - e)) >> 1;
  const int td2 = (abs(at(next, -1) - c) + abs(at(next, 1) - e)) >> 1;
  int diff = max(td0 >> 1, max(td1, td2));
  int v;
  if (!diff) {
    v = d;
  } else {
    const int b = ((at(p2, -2) + at(n2, -2)) >> 1) - c;
    const int f = ((at(p2, 2) + at(n2, 2)) >> 1) - e;
    const int dc = d - c, de = d - e;
    const int mx = max(max(de, dc), min(b, f));
    const int mn = min(min(de, dc), max(b, f));
    diff = max(max(diff, mn), -mx);
    int interp;
    if (abs(c - e) > td0) {
      interp = ((5570 * (at(p2, 0) + at(n2, 0)) - 3801 * (at(p2, -2) + at(n2, -2) + at(p2, 2) + at(n2, 2)) +
                 1016 * (at(p2, -4) + at(n2, -4) + at(p2, 4) + at(n2, 4))) >> 2) +
               4309 * (c + e) - 213 * (at(cur, -3) + at(cur, 3));
    } else {
      interp = 5077 * (c + e) - 981 * (at(cur, -3) + at(cur, 3));
    }
    interp >>= 13;
    v = clampi(interp, d - diff, d + diff);
  }
  out[o] = sat8(v);
}
__global__ void k_bwdif(const uint8_t* __restrict__ prev, const uint8_t* __restrict__ cur,
                        const uint8_t* __restrict__ next, uint8_t* __restrict__ out, int w, int h, int keep) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= w || y >= h) return;
  bwdif_px(prev, cur, next, out, w, h, keep, x, y);
}
// A whole segment in one launch: z = frame * nplanes + plane; frame i from (i-1, i, i+1) with
// the segment's edges repeated (send_frame per part).  Planes are packed (pitch = width).
struct BwdifPlanes {
  long off[3];
  int w[3], h[3];
  int n;
};
__global__ void k_bwdif_seg(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, long fs, int nframes,
                            BwdifPlanes pl, int keep) {
  const int i = blockIdx.z / pl.n, p = blockIdx.z - i * pl.n;
  const int w = pl.w[p], h = pl.h[p];
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= w || y >= h) return;
  const long o = pl.off[p];
  const uint8_t* cur = src + (long)i * fs + o;
  const uint8_t* prev = src + (long)(i > 0 ? i - 1 : 0) * fs + o;
  const uint8_t* next = src + (long)(i + 1 < nframes ? i + 1 : nframes - 1) * fs + o;
  bwdif_px(prev, cur, next, dst + (long)i * fs + o, w, h, keep, x, y);
}

// ------------------------------------------------------------------------ SSIM
// Mean SSIM over 8x8 windows on a 4-sample grid (x264/libvpx convention): one thread per
// window computes the five moments, a wave reduction + one atomic per wave accumulates
// (sum of SSIM, window count) in double.
__global__ void __launch_bounds__(256) k_ssim(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b, int w,
                                              int h, int stride_a, int stride_b, double* __restrict__ acc) {
  const int nx = (w - 8) / 4 + 1, ny = (h - 8) / 4 + 1;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  double v = 0.0;
  if (i < nx * ny) {
    const int x0 = (i % nx) * 4, y0 = (i / nx) * 4;
    int sa = 0, sb = 0, saa = 0, sbb = 0, sab = 0;
    for (int y = 0; y < 8; ++y)
      for (int x = 0; x < 8; ++x) {
        const int p = a[(long)(y0 + y) * stride_a + x0 + x], q = b[(long)(y0 + y) * stride_b + x0 + x];
        sa += p;
        sb += q;
        saa += p * p;
        sbb += q * q;
        sab += p * q;
      }
    const double n = 64.0, c1 = 6.5025, c2 = 58.5225;  // (0.01*255)^2, (0.03*255)^2
    const double ma = sa / n, mb = sb / n;
    const double va = saa / n - ma * ma, vb = sbb / n - mb * mb, cov = sab / n - ma * mb;
    v = ((2 * ma * mb + c1) * (2 * cov + c2)) / ((ma * ma + mb * mb + c1) * (va + vb + c2));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(acc, v);
}

}  // namespace ops
}  // namespace tv

// ------------------------------------------------------------------- C API
// Every entry point takes device pointers and the caller's stream; returns 0 / -1.
namespace {
thread_local std::string g_ops_err;
int ops_status() {
  const hipError_t e = hipGetLastError();
  if (e == hipSuccess) return 0;
  g_ops_err = hipGetErrorString(e);
  return -1;
}
inline unsigned cdiv(long a, long b) { return (unsigned)((a + b - 1) / b); }
}  // namespace

extern "C" {
const char* tv_ops_last_error() { return g_ops_err.c_str(); }

int tv_resize_plane(const uint8_t* src, int sw, int sh, int sstride, uint8_t* dst, int dw, int dh, int dstride,
                    const int* ix, const int16_t* wx, int tx, const int* iy, const int16_t* wy, int ty,
                    int16_t* tmp, void* stream) {
  if (sw <= 0 || sh <= 0 || dw <= 0 || dh <= 0 || tx <= 0 || ty <= 0 || tx > 64 || ty > 64) {
    g_ops_err = "tv_resize_plane: bad geometry";
    return -1;
  }
  auto s = static_cast<hipStream_t>(stream);
  tv::ops::k_resize_h<<<dim3(cdiv(dw, tv::ops::kTile), sh), tv::ops::kTile, 0, s>>>(src, sw, sstride, 0, tmp, 0, dw,
                                                                                     ix, wx, tx);
  tv::ops::k_resize_v<<<dim3(cdiv(dw, tv::ops::kTile), dh), tv::ops::kTile, 0, s>>>(tmp, 0, sh, dw, dst, 0, dstride,
                                                                                     dh, dw, dh, iy, wy, ty);
  return ops_status();
}

int tv_rgb_to_i420(const uint8_t* rgb, int w, int h, int stride, uint8_t* y, uint8_t* u, uint8_t* v, int bt709,
                   void* stream) {
  if ((w | h) & 1) {
    g_ops_err = "tv_rgb_to_i420: odd size";
    return -1;
  }
  tv::ops::k_rgb_to_i420<<<dim3(cdiv(w / 2, 128), h / 2), 128, 0, static_cast<hipStream_t>(stream)>>>(
      rgb, w, h, stride, y, u, v, bt709);
  return ops_status();
}

int tv_p010_to_i420(const uint16_t* y16, const uint16_t* uv16, int w, int h, uint8_t* y, uint8_t* u, uint8_t* v,
                    void* stream) {
  if ((w | h) & 1) {
    g_ops_err = "tv_p010_to_i420: odd size";
    return -1;
  }
  tv::ops::k_p010_to_i420<<<dim3(cdiv(w, 256), h), 256, 0, static_cast<hipStream_t>(stream)>>>(y16, uv16, w, h, y,
                                                                                                u, v);
  return ops_status();
}

int tv_tonemap_pq(const uint16_t* y16, const uint16_t* uv16, int w, int h, uint8_t* y, uint8_t* u, uint8_t* v,
                  float src_peak, float dst_peak, void* stream) {
  if ((w | h) & 1 || src_peak <= dst_peak) {
    g_ops_err = "tv_tonemap_pq: odd size or src_peak <= dst_peak";
    return -1;
  }
  tv::ops::k_tonemap_pq<<<dim3(cdiv(w / 2, 128), h / 2), 128, 0, static_cast<hipStream_t>(stream)>>>(
      y16, uv16, w, h, y, u, v, 0, src_peak, dst_peak);
  return ops_status();
}

// n frames: P010 in (y16: n x w*h, uv16: n x w*h/2), I420 out n x (Y | U | V) back to back.
int tv_tonemap_pq_batch(const uint16_t* y16, const uint16_t* uv16, int w, int h, int n, uint8_t* out,
                        float src_peak, float dst_peak, void* stream) {
  if ((w | h) & 1 || w <= 0 || h <= 0 || n <= 0 || n > 65535 || src_peak <= dst_peak) {
    g_ops_err = "tv_tonemap_pq_batch: bad geometry or src_peak <= dst_peak";
    return -1;
  }
  const long ysz = (long)w * h, csz = ysz / 4;
  tv::ops::k_tonemap_pq<<<dim3(cdiv(w / 2, 128), h / 2, n), 128, 0, static_cast<hipStream_t>(stream)>>>(
      y16, uv16, w, h, out, out + ysz, out + ysz + csz, ysz + 2 * csz, src_peak, dst_peak);
  return ops_status();
}

int tv_synth_p010(uint16_t* y16, uint16_t* uv16, int w, int h, int n, int t0, uint32_t seed, void* stream) {
  if ((w | h) & 1 || w <= 0 || h <= 0 || n <= 0 || n > 65535) {
    g_ops_err = "tv_synth_p010: bad geometry";
    return -1;
  }
  tv::ops::k_synth_p010<<<dim3(cdiv(w / 2, 128), h / 2, n), 128, 0, static_cast<hipStream_t>(stream)>>>(
      y16, uv16, w, h, t0, seed);
  return ops_status();
}

// Batched Lanczos resample of one plane of n frames (frame strides sfs / dfs bytes) into a
// pw x ph edge-padded destination.  th > 0: fused 2-D kernel with th-row output tiles,
// source rows staged at wp bytes pitch, smem bytes of LDS (host-planned); th == 0: the
// two-pass kernels through tmp (n x sh x dw int16).
int tv_resize_batch(const uint8_t* src, int sw, int sh, int sstride, long sfs, uint8_t* dst, int dw, int dh,
                    int dstride, long dfs, int pw, int ph, int n, const int* ix, const int16_t* wx, int tx,
                    const int* iy, const int16_t* wy, int ty, int16_t* tmp, int th, int wp, int smem,
                    void* stream) {
  if (sw <= 0 || sh <= 0 || dw <= 0 || dh <= 0 || pw < dw || ph < dh || dstride < pw || n <= 0 || n > 65535 ||
      tx <= 0 || ty <= 0 || tx > 64 || ty > 64 || sh > 65535 || ph > 65535 || th < 0 || smem < 0 ||
      smem > 64 * 1024 || (th > 0 && wp < tx)) {
    g_ops_err = "tv_resize_batch: bad geometry";
    return -1;
  }
  auto s = static_cast<hipStream_t>(stream);
  if (th > 0) {
    const dim3 grid(cdiv(pw, tv::ops::kR2W), cdiv(ph, th), n);
    if (tx <= 16)
      tv::ops::k_resize2d<16><<<grid, 256, smem, s>>>(src, sw, sh, sstride, sfs, dst, dw, dh, dstride, dfs, pw, ph,
                                                       th, wp, ix, wx, tx, iy, wy, ty);
    else if (tx <= 32)
      tv::ops::k_resize2d<32><<<grid, 256, smem, s>>>(src, sw, sh, sstride, sfs, dst, dw, dh, dstride, dfs, pw, ph,
                                                       th, wp, ix, wx, tx, iy, wy, ty);
    else
      tv::ops::k_resize2d<64><<<grid, 256, smem, s>>>(src, sw, sh, sstride, sfs, dst, dw, dh, dstride, dfs, pw, ph,
                                                       th, wp, ix, wx, tx, iy, wy, ty);
    return ops_status();
  }
  const long tfs = (long)sh * dw;
  tv::ops::k_resize_h<<<dim3(cdiv(dw, tv::ops::kTile), sh, n), tv::ops::kTile, 0, s>>>(src, sw, sstride, sfs, tmp,
                                                                                        tfs, dw, ix, wx, tx);
  tv::ops::k_resize_v<<<dim3(cdiv(pw, tv::ops::kTile), ph, n), tv::ops::kTile, 0, s>>>(
      tmp, tfs, sh, dw, dst, dfs, dstride, dh, pw, ph, iy, wy, ty);
  return ops_status();
}

int tv_overlay_mask(uint8_t* frames, int n, int w, int h, const uint8_t* masks, int mw, int mh, int x0, int y0,
                    void* stream) {
  if (n <= 0 || mw <= 0 || mh <= 0 || (x0 & 1) || (y0 & 1)) {
    g_ops_err = "tv_overlay_mask: bad arguments";
    return -1;
  }
  tv::ops::k_overlay_mask<<<dim3(cdiv(mw, 128), mh, n), 128, 0, static_cast<hipStream_t>(stream)>>>(
      frames, w, h, masks, mw, mh, x0, y0);
  return ops_status();
}
// bwdif over a segment of n packed frames (frame stride fs bytes; np planes at byte offsets
// off[] of sizes w[] x h[]), one launch for every frame and plane
int tv_bwdif_segment(const uint8_t* src, uint8_t* dst, long fs, int n, int np, const long* off, const int* w,
                     const int* h, int tff, void* stream) {
  if (n <= 0 || np < 1 || np > 3 || n * np > 65535) {
    g_ops_err = "tv_bwdif_segment: bad arguments";
    return -1;
  }
  tv::ops::BwdifPlanes pl{};
  int mw = 0, mh = 0;
  for (int p = 0; p < np; ++p) {
    if (w[p] <= 0 || h[p] < 4 || off[p] < 0 || off[p] + (long)w[p] * h[p] > fs) {
      g_ops_err = "tv_bwdif_segment: bad plane geometry";
      return -1;
    }
    pl.off[p] = off[p];
    pl.w[p] = w[p];
    pl.h[p] = h[p];
    mw = w[p] > mw ? w[p] : mw;
    mh = h[p] > mh ? h[p] : mh;
  }
  pl.n = np;
  tv::ops::k_bwdif_seg<<<dim3(cdiv(mw, 256), mh, n * np), 256, 0, static_cast<hipStream_t>(stream)>>>(
      src, dst, fs, n, pl, tff ? 0 : 1);
  return ops_status();
}
int tv_bwdif_plane(const uint8_t* prev, const uint8_t* cur, const uint8_t* next, uint8_t* out, int w, int h,
                   int tff, void* stream) {
  if (w <= 0 || h < 4) {
    g_ops_err = "tv_bwdif_plane: bad geometry";
    return -1;
  }
  tv::ops::k_bwdif<<<dim3(cdiv(w, 256), h), 256, 0, static_cast<hipStream_t>(stream)>>>(prev, cur, next, out, w, h,
                                                                                          tff ? 0 : 1);
  return ops_status();
}
}

extern "C" int tv_ssim_plane(const uint8_t* a, const uint8_t* b, int w, int h, int stride_a, int stride_b, double* acc,
                             void* stream) {
  if (w < 8 || h < 8) {
    g_ops_err = "tv_ssim_plane: plane smaller than 8x8";
    return -1;
  }
  const long n = (long)((w - 8) / 4 + 1) * ((h - 8) / 4 + 1);
  tv::ops::k_ssim<<<cdiv(n, 256), 256, 0, static_cast<hipStream_t>(stream)>>>(a, b, w, h, stride_a, stride_b, acc);
  return ops_status();
}
