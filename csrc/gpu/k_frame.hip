// k_frame.hip — frame-level kernels: synthetic source, PSNR SSE, quarter-pel phase planes,
// in-loop deblocking.  Batched: blockIdx.z (or .y) selects the segment.
#include <cstdlib>
#include <cstring>

#include "gpu_common.h"
#include "k_encode.h"
#include "tv/synth.h"

namespace tv {
namespace gpu {

// ---------------------------------- synthetic source ------------------------------------
// One workgroup row-tile; the per-frame object trajectories are evaluated once per
// workgroup into LDS (they were 18 hashes per pixel before).  Each thread produces 4
// horizontally adjacent samples (one dword store): the value-noise octaves keep their
// lattice-corner hashes across the 4 samples (a cell is >= 4 px wide, so the cell changes at
// most once: 2 new hashes instead of 4 per octave per sample), and the row terms (cell row,
// vertical smoothstep) are computed once.  Bit-identical to synth_sample_ctx (tv/synth.h),
// which the CPU golden encoder uses.
struct VNoiseRow {
  int sh, sy;
  int32_t cy, cx;
  uint32_t seed;
  int a, b, c, d;
  __device__ void init(int32_t py16, int lp, uint32_t sd) {
    sh = lp + 4;
    seed = sd;
    cy = py16 >> sh;
    const int fy = (int)((py16 - (cy << sh)) << 8 >> sh);
    sy = (fy * fy * (768 - 2 * fy)) >> 16;
    cx = INT32_MIN;
  }
  __device__ int eval(int32_t px16) {
    const int32_t nx = px16 >> sh;
    if (nx != cx) {
      if (nx == cx + 1) {
        a = b;
        c = d;
      } else {
        a = synth_hash(nx, cy, seed) & 255;
        c = synth_hash(nx, cy + 1, seed) & 255;
      }
      b = synth_hash(nx + 1, cy, seed) & 255;
      d = synth_hash(nx + 1, cy + 1, seed) & 255;
      cx = nx;
    }
    const int fx = (int)((px16 - (cx << sh)) << 8 >> sh);
    const int sx = (fx * fx * (768 - 2 * fx)) >> 16;
    const int top = a * 256 + (b - a) * sx;
    const int bot = c * 256 + (d - c) * sx;
    return (top * 256 + (bot - top) * sy) >> 16;
  }
};

__device__ __forceinline__ int synth_objects(const SynthFrameCtx& f, int c, int xl, int yl, int v, unsigned rows) {
  for (; rows; rows &= rows - 1) {  // later objects on top: ascending k over the row's objects
    const int k = __builtin_ctz(rows);
    const SynthObject& o = f.obj[k];
    const int32_t rx16 = xl * 16 - f.ox[k], ry16 = yl * 16 - f.oy[k];
    if (rx16 < 0 || rx16 >= o.w * 16) continue;
    if (o.shape == 1) {
      const int64_t dx = 2 * (int64_t)rx16 - o.w * 16, dy = 2 * (int64_t)ry16 - o.h * 16;
      const int64_t ww = (int64_t)o.w * 16, hh = (int64_t)o.h * 16;
      if (dx * dx * hh * hh + dy * dy * ww * ww > ww * ww * hh * hh) continue;
    }
    if (c == 0) {
      v = 40 + ((synth_vnoise(rx16, ry16, 4, o.seed) * 3 + synth_vnoise(rx16, ry16, 2, o.seed + 5)) >> 2) * 3 / 4;
    } else {
      v = 64 + (int)(synth_hash(k, c, f.seed) & 127) + (synth_vnoise(rx16, ry16, 5, o.seed + c) >> 3);
    }
  }
  return v;
}

// kTex: the textured variant (seed bit 31) is a separate instantiation so the smooth source
// keeps its register budget (a runtime branch doubled its time).  The objects are filtered
// once per item by their vertical extent before the per-sample horizontal / shape tests.
// (16 samples per item shared more cell hashes but cut occupancy 22 -> 13 waves/CU and was
// 16 % slower: profiles/README.md.)
template <bool kTex>
__global__ void __launch_bounds__(256) k_synth(FrameSet src, Geo g, uint32_t seed, FrameIdx fi) {
  const int c = blockIdx.y, b = blockIdx.z;
  const int pw = c ? g.W / 2 : g.W, ph = c ? g.H / 2 : g.H;
  const int dw = c ? g.dw / 2 : g.dw, dh = c ? g.dh / 2 : g.dh;
  __shared__ SynthFrameCtx ctx;
  if (threadIdx.x == 0) synth_frame_ctx(seed, fi.t[b], g.dw, g.dh, ctx);
  __syncthreads();
  uint8_t* P = src.plane(c, b, g);
  const int s = c ? 1 : 0, pq = pw >> 2;  // pw is a multiple of 16
  constexpr bool tex = kTex;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < pq * ph; i += gridDim.x * blockDim.x) {
    const int y = i / pq, x0 = (i - y * pq) * 4;
    const int yc = tv_min(y, dh - 1), yl = yc << s;
    const int32_t by16 = yl * 16 + ctx.t * (tex ? 36 : 12);
    unsigned rows = 0;
#pragma unroll
    for (int k = 0; k < kSynthObjects; ++k) {
      const int32_t ry16 = yl * 16 - ctx.oy[k];
      rows |= (ry16 >= 0 && ry16 < ctx.obj[k].h * 16) ? 1u << k : 0u;
    }
    VNoiseRow n0, n1, n2, n3;
    if (c == 0) {
      n0.init(by16, 7, ctx.seed);
      n1.init(by16, 5, ctx.seed + 1);
      n2.init(by16, 3, ctx.seed + 2);
      if (tex) n3.init(by16, 1, ctx.seed + 3);
    } else {
      n0.init(by16, 8, ctx.seed + 10 * c);
    }
    uint32_t word = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int xc = tv_min(x0 + j, dw - 1), xl = xc << s;
      const int32_t bx16 = xl * 16 + ctx.t * (tex ? 88 : 36);
      int v;
      if (c == 0 && tex)
        v = (n0.eval(bx16) * 3 + n1.eval(bx16) * 2 + n2.eval(bx16) * 2 + n3.eval(bx16)) >> 3;
      else if (c == 0)
        v = (n0.eval(bx16) * 5 + n1.eval(bx16) * 2 + n2.eval(bx16)) >> 3;
      else
        v = 96 + (n0.eval(bx16) >> 1);
      if (rows) v = synth_objects(ctx, c, xl, yl, v, rows);
      if (tex) {  // per-frame grain, as synth_sample_ctx
        const uint32_t gr = synth_hash(xc + ctx.t * 7919, yc + c * 104729, ctx.seed ^ 0x5bd1e995u);
        v += c ? (int)(gr & 3) - 2 : (int)(gr & 7) - 4;
      }
      word |= (uint32_t)clip_pixel(v) << (8 * j);
    }
    *reinterpret_cast<uint32_t*>(P + (long)y * pw + x0) = word;
  }
}

// ------------------------------------------ SSE -----------------------------------------
// One workgroup per (row block, plane, segment); 4-byte vector loads along rows.
__global__ void __launch_bounds__(256) k_sse(FrameSet a, FrameSet r, Geo g, unsigned long long* sse) {
  const int c = blockIdx.y, b = blockIdx.z;
  const int pw = c ? g.W / 2 : g.W;
  const int dw = c ? g.dw / 2 : g.dw, dh = c ? g.dh / 2 : g.dh;
  const uint8_t* A = a.plane(c, b, g);
  const uint8_t* R = r.plane(c, b, g);
  const int wq = (dw + 3) >> 2;  // 4-pixel groups per row (pw is a multiple of 16)
  unsigned s = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < wq * dh; i += gridDim.x * blockDim.x) {
    const int y = i / wq, x = (i - y * wq) * 4;
    const uint32_t va = *reinterpret_cast<const uint32_t*>(A + (long)y * pw + x);
    const uint32_t vr = *reinterpret_cast<const uint32_t*>(R + (long)y * pw + x);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int d = (int)((va >> (8 * k)) & 255) - (int)((vr >> (8 * k)) & 255);
      s += (x + k < dw) ? (unsigned)(d * d) : 0u;
    }
  }
  unsigned long long t = s;
  for (int o = 32; o > 0; o >>= 1) t += __shfl_xor(t, o, 64);
  __shared__ unsigned long long part[4];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = t;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(sse + b * 3 + c, part[0] + part[1] + part[2] + part[3]);
}

// --------------------------------- quarter-pel phase planes -----------------------------
// Plane p = fx + 4*fy holds the exact HEVC 8-tap interpolated luma sample at every integer
// position of the padded domain [-8, W+8) x [-8, H+8) (beyond 4 samples outside the
// picture the clamped interpolation is constant, so clamping the query to the pad is
// exact).  Motion search and luma motion compensation then become plain byte loads.
//
// One 32x32 output tile per workgroup, all 16 planes.  The 8-tap filters run on the packed
// integer dot-product units instead of scalar multiply-adds:
//  * horizontal (int8 samples): a sample window of 8 bytes is two dwords (v_alignbyte from
//    the tile row held as dwords in LDS); samples are biased to signed bytes (x ^ 0x80) so
//    each half is one v_dot4_i32_i8 against the packed taps, the bias is 128 * sum(taps) =
//    8192 added back — 2 dot4 per output instead of 8 MACs;
//  * vertical over integer rows: the 4x4 byte blocks of 8 rows are transposed with 16
//    v_perm_b32, then 2 dot4 per output;
//  * vertical over the 16-bit horizontal intermediates: row pairs are packed with v_perm and
//    reduced with v_dot2_i32_i16 (4 per output).
// Every product and sum is exact (|intermediate| < 2^15, |2-D sum| < 2^21): bit-identical
// to tv::mc_luma_sample.
typedef short tv_short2 __attribute__((ext_vector_type(2)));

__device__ constexpr uint32_t pack_taps4(int f, int k0) {
  return (uint32_t)(uint8_t)kLumaFilter[f][k0] | (uint32_t)(uint8_t)kLumaFilter[f][k0 + 1] << 8 |
         (uint32_t)(uint8_t)kLumaFilter[f][k0 + 2] << 16 | (uint32_t)(uint8_t)kLumaFilter[f][k0 + 3] << 24;
}
__device__ constexpr uint32_t pack_taps2(int f, int k0) {
  return (uint32_t)(uint16_t)kLumaFilter[f][k0] | (uint32_t)(uint16_t)kLumaFilter[f][k0 + 1] << 16;
}
__device__ __forceinline__ int dot4(uint32_t a, uint32_t b, int c) {
  return __builtin_amdgcn_sdot4((int)a, (int)b, c, false);
}
__device__ __forceinline__ int dot2(uint32_t a, uint32_t b, int c) {
  return __builtin_amdgcn_sdot2(__builtin_bit_cast(tv_short2, a), __builtin_bit_cast(tv_short2, b), c, false);
}
__device__ __forceinline__ uint32_t pack4_pixels(int v0, int v1, int v2, int v3) {
  return (uint32_t)clip_pixel(v0) | (uint32_t)clip_pixel(v1) << 8 | (uint32_t)clip_pixel(v2) << 16 |
         (uint32_t)clip_pixel(v3) << 24;
}

constexpr int kPhW = 10;  // dwords per staged source row: 40 bytes = tile 32 + 8 tap reach
__global__ void __launch_bounds__(256) k_phase_planes(FrameSet ref, uint8_t* phase, Geo g) {
  const int tid = threadIdx.x;
  const int L = xcd_remap(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z),
                          gridDim.x * gridDim.y * gridDim.z);
  const int tpf = gridDim.x * gridDim.y, b = L / tpf, tyi = (L - b * tpf) / gridDim.x;
  const int tx0 = (L - b * tpf - tyi * gridDim.x) * 32 - 8, ty0 = tyi * 32 - 8;
  const uint8_t* R = ref.plane(0, b, g);
  // raw[rr] dword w = samples (tx0 - 4 + 4w .. +3, ty0 - 3 + rr), clamped, biased to int8
  __shared__ uint32_t raw[39][kPhW];
  // hf[fx-1][rr][c]: horizontal filter fx at (tx0 + c, ty0 - 3 + rr)
  __shared__ __align__(16) int16_t hf[3][39][32];
  for (int i = tid; i < 39 * kPhW; i += 256) {
    const int rr = i / kPhW, w = i - rr * kPhW;
    const uint8_t* row = R + (long)clip3(0, g.H - 1, ty0 - 3 + rr) * g.W;
    const int x = tx0 - 4 + 4 * w;
    uint32_t v;
    if (x >= 0 && x + 3 < g.W) {
      v = *reinterpret_cast<const uint32_t*>(row + x);  // x is 4-aligned (tx0 = 32k - 8)
    } else {
      v = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) v |= (uint32_t)row[clip3(0, g.W - 1, x + k)] << (8 * k);
    }
    raw[rr][w] = v ^ 0x80808080u;
  }
  __syncthreads();
  // horizontal pass: item = (row, 4 output columns), the 3 fractional filters at once
  for (int i = tid; i < 39 * 8; i += 256) {
    const int rr = i >> 3, c4 = i & 7;
    // column c = 4*c4 + j takes bytes c+1 .. c+8 of the row (taps at x-3 .. x+4)
    const uint32_t w0 = raw[rr][c4], w1 = raw[rr][c4 + 1], w2 = raw[rr][c4 + 2];
    int out[3][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t lo = j == 3 ? w1 : __builtin_amdgcn_alignbyte(w1, w0, j + 1);
      const uint32_t hi = j == 3 ? w2 : __builtin_amdgcn_alignbyte(w2, w1, j + 1);
#pragma unroll
      for (int f = 1; f < 4; ++f) out[f - 1][j] = dot4(lo, pack_taps4(f, 0), dot4(hi, pack_taps4(f, 4), 8192));
    }
#pragma unroll
    for (int f = 0; f < 3; ++f) {
      uint2 v;
      v.x = (uint32_t)(uint16_t)out[f][0] | (uint32_t)out[f][1] << 16;
      v.y = (uint32_t)(uint16_t)out[f][2] | (uint32_t)out[f][3] << 16;
      *reinterpret_cast<uint2*>(&hf[f][rr][4 * c4]) = v;
    }
  }
  __syncthreads();
  const int r = tid >> 3, c0 = (tid & 7) * 4;
  const int X = tx0 + c0, Y = ty0 + r;
  if (X + 8 >= g.pw16 || Y >= g.H + 8) return;
  uint8_t* base = phase + (long)b * 16 * g.psz + (long)(Y + 8) * g.pw16 + (X + 8);
  auto store = [&](int plane, uint32_t w) { *reinterpret_cast<uint32_t*>(base + (long)plane * g.psz) = w; };
  // ---- fx = 0: integer column, rows Y-3 .. Y+4 = raw rows r .. r+7, word c0/4 + 1
  {
    uint32_t R8[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) R8[k] = raw[r + k][(c0 >> 2) + 1];
    store(0, R8[3] ^ 0x80808080u);
    uint32_t C[2][4];  // C[h][j]: column j, rows 4h .. 4h+3 (one byte each)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t* q = R8 + 4 * h;
      const uint32_t t01l = __builtin_amdgcn_perm(q[1], q[0], 0x05010400u);
      const uint32_t t01h = __builtin_amdgcn_perm(q[1], q[0], 0x07030602u);
      const uint32_t t23l = __builtin_amdgcn_perm(q[3], q[2], 0x05010400u);
      const uint32_t t23h = __builtin_amdgcn_perm(q[3], q[2], 0x07030602u);
      C[h][0] = __builtin_amdgcn_perm(t23l, t01l, 0x05040100u);
      C[h][1] = __builtin_amdgcn_perm(t23l, t01l, 0x07060302u);
      C[h][2] = __builtin_amdgcn_perm(t23h, t01h, 0x05040100u);
      C[h][3] = __builtin_amdgcn_perm(t23h, t01h, 0x07060302u);
    }
#pragma unroll
    for (int fy = 1; fy < 4; ++fy) {
      int v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        v[j] = dot4(C[0][j], pack_taps4(fy, 0), dot4(C[1][j], pack_taps4(fy, 4), 8192 + 32)) >> 6;  // rounding folded in
      store(4 * fy, pack4_pixels(v[0], v[1], v[2], v[3]));
    }
  }
  // ---- fx = 1..3: vertical over the int16 intermediates, row pairs packed for v_dot2
#pragma unroll
  for (int fx = 1; fx < 4; ++fx) {
    uint2 H8[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) H8[k] = *reinterpret_cast<const uint2*>(&hf[fx - 1][r + k][c0]);
    {
      const int h0 = (int16_t)(H8[3].x & 0xffff), h1 = (int16_t)(H8[3].x >> 16);
      const int h2 = (int16_t)(H8[3].y & 0xffff), h3 = (int16_t)(H8[3].y >> 16);
      store(fx, pack4_pixels((h0 + 32) >> 6, (h1 + 32) >> 6, (h2 + 32) >> 6, (h3 + 32) >> 6));
    }
    uint32_t P[4][4];  // P[m][j]: column j, rows 2m (low half) and 2m + 1 (high half)
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      P[m][0] = __builtin_amdgcn_perm(H8[2 * m + 1].x, H8[2 * m].x, 0x05040100u);
      P[m][1] = __builtin_amdgcn_perm(H8[2 * m + 1].x, H8[2 * m].x, 0x07060302u);
      P[m][2] = __builtin_amdgcn_perm(H8[2 * m + 1].y, H8[2 * m].y, 0x05040100u);
      P[m][3] = __builtin_amdgcn_perm(H8[2 * m + 1].y, H8[2 * m].y, 0x07060302u);
    }
#pragma unroll
    for (int fy = 1; fy < 4; ++fy) {
      int v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        int a = dot2(P[0][j], pack_taps2(fy, 0), 0);
        a = dot2(P[1][j], pack_taps2(fy, 2), a);
        a = dot2(P[2][j], pack_taps2(fy, 4), a);
        a = dot2(P[3][j], pack_taps2(fy, 6), a);
        v[j] = ((a >> 6) + 32) >> 6;
      }
      store(fx + 4 * fy, pack4_pixels(v[0], v[1], v[2], v[3]));
    }
  }
}

// ------------------------------------ deblocking ----------------------------------------
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) k_deblock(FrameSet rec, DecisionSet dec, Geo g, int horizontal) {
  const int b = blockIdx.y;
  const int qp = dec.qp[b];
  const long ub = b * g.usz;
  const uint8_t* cl = dec.cu_log2 + ub;
  const uint8_t* in = dec.intra + ub;
  const uint8_t* cb = dec.cbf + ub;
  const int16_t* mv = dec.mv + 2 * ub;
  const uint8_t* dir = dec.dir ? dec.dir + ub : nullptr;  // B pictures
  const int16_t* mv1 = dec.mv1 ? dec.mv1 + 2 * ub : nullptr;
  const uint8_t* tu = dec.tu ? dec.tu + ub : nullptr;  // RQT-split 32x32 CUs (P pictures)
  uint8_t* Y = rec.plane(0, b, g);
  uint8_t* U = rec.plane(1, b, g);
  uint8_t* V = rec.plane(2, b, g);
  const int W = g.W, H = g.H, Wc = W / 2;
  const int qpc = chroma_qp(qp, 0);
  const int nl = horizontal ? (H / 8 - 1) * (W / 4) : (W / 8 - 1) * (H / 4);
  const int nc = horizontal ? (H / 16 - 1) * (Wc / 4) : (W / 16 - 1) * (H / 8);
  // Each item's samples are moved as aligned dwords into registers (a vertical edge: the
  // 8 bytes x-4..x+3 of each of its 4 lines; a horizontal edge: 8 rows x the segment's 4
  // columns), filtered there by the shared tv::deblock_* functions and written back the same
  // way: 8 dword loads per luma segment instead of 32 byte loads.  Items of a pass never
  // share a dword (edges are 8 samples apart), so the write-back of unchanged bytes is safe.
  auto ld = [](const uint8_t* p) { return *reinterpret_cast<const uint32_t*>(p); };
  auto st = [](uint8_t* p, uint32_t v) { *reinterpret_cast<uint32_t*>(p) = v; };
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nl + nc; i += gridDim.x * blockDim.x) {
    if (i < nl) {
      if (!horizontal) {
        const int x = 8 * (1 + i % (W / 8 - 1)), y = 4 * (i / (W / 8 - 1));
        const int bs = deblock_edge_bs(cl, in, cb, mv, g.w8, x - 1, y, x, y, dir, mv1, tu);
        if (bs) {
          uint32_t v[4][2];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            v[k][0] = ld(Y + (long)(y + k) * W + x - 4);
            v[k][1] = ld(Y + (long)(y + k) * W + x);
          }
          deblock_luma_edge4(reinterpret_cast<uint8_t*>(&v[0][1]), 1, 8, bs, qp);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            st(Y + (long)(y + k) * W + x - 4, v[k][0]);
            st(Y + (long)(y + k) * W + x, v[k][1]);
          }
        }
      } else {
        const int y = 8 * (1 + i % (H / 8 - 1)), x = 4 * (i / (H / 8 - 1));
        const int bs = deblock_edge_bs(cl, in, cb, mv, g.w8, x, y - 1, x, y, dir, mv1, tu);
        if (bs) {
          uint32_t v[8];  // rows y-4 .. y+3, columns x .. x+3
#pragma unroll
          for (int r = 0; r < 8; ++r) v[r] = ld(Y + (long)(y - 4 + r) * W + x);
          deblock_luma_edge4(reinterpret_cast<uint8_t*>(&v[4]), 4, 1, bs, qp);
#pragma unroll
          for (int r = 1; r < 7; ++r) st(Y + (long)(y - 4 + r) * W + x, v[r]);  // rows p2..q2
        }
      }
    } else {
      const int j = i - nl;
      if (!horizontal) {
        const int xc = 8 * (1 + j % (W / 16 - 1)), yc = 4 * (j / (W / 16 - 1));
        const int bs = deblock_edge_bs(cl, in, cb, mv, g.w8, 2 * xc - 1, 2 * yc, 2 * xc, 2 * yc, dir, mv1, tu);
        if (bs == 2) {
#pragma unroll
          for (int pl = 0; pl < 2; ++pl) {
            uint8_t* P = pl ? V : U;
            uint32_t v[4][2];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              v[k][0] = ld(P + (long)(yc + k) * Wc + xc - 4);
              v[k][1] = ld(P + (long)(yc + k) * Wc + xc);
            }
            deblock_chroma_edge(reinterpret_cast<uint8_t*>(&v[0][1]), 1, 8, 4, qpc);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              st(P + (long)(yc + k) * Wc + xc - 4, v[k][0]);
              st(P + (long)(yc + k) * Wc + xc, v[k][1]);
            }
          }
        }
      } else {
        const int yc = 8 * (1 + j % (H / 16 - 1)), xc = 4 * (j / (H / 16 - 1));
        const int bs = deblock_edge_bs(cl, in, cb, mv, g.w8, 2 * xc, 2 * yc - 1, 2 * xc, 2 * yc, dir, mv1, tu);
        if (bs == 2) {
#pragma unroll
          for (int pl = 0; pl < 2; ++pl) {
            uint8_t* P = pl ? V : U;
            uint32_t v[4];  // rows yc-2 .. yc+1
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = ld(P + (long)(yc - 2 + r) * Wc + xc);
            deblock_chroma_edge(reinterpret_cast<uint8_t*>(&v[2]), 4, 1, 4, qpc);
            st(P + (long)(yc - 1) * Wc + xc, v[1]);
            st(P + (long)yc * Wc + xc, v[2]);
          }
        }
      }
    }
  }
}

// ------------------------------------ launchers -----------------------------------------
void launch_synth(FrameSet src, const Geo& g, uint32_t seed, const FrameIdx& fi, int B, hipStream_t s) {
  dim3 grid((unsigned)tv_min(512, (int)((g.ysz + 1023) / 1024)), 3, B);
  if (synth_textured(seed))
    k_synth<true><<<grid, 256, 0, s>>>(src, g, seed, fi);
  else
    k_synth<false><<<grid, 256, 0, s>>>(src, g, seed, fi);
}
// One picture of B device-resident segments ([segment][frame][Y | U | V] at the coded size,
// segment stride seg_stride bytes) into the B source planes: one launch instead of 3 B
// copyBuffer blits in front of every picture's analysis (the node job's file sources).
__global__ void __launch_bounds__(256) k_gather_frames(const uint8_t* frames, long seg_stride, FrameSet src, Geo g,
                                                       int B) {
  const long f16 = (g.ysz + 2 * g.csz) / 16, y16 = g.ysz / 16, c16 = g.csz / 16;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < B * f16; i += (long)gridDim.x * 256) {
    const int b = (int)(i / f16);
    const long r = i - b * f16;
    const uint4 v = reinterpret_cast<const uint4*>(frames + b * seg_stride)[r];
    uint4* d = r < y16 ? reinterpret_cast<uint4*>(src.y + b * g.ysz) + r
               : r < y16 + c16 ? reinterpret_cast<uint4*>(src.u + b * g.csz) + (r - y16)
                               : reinterpret_cast<uint4*>(src.v + b * g.csz) + (r - y16 - c16);
    *d = v;
  }
}
void launch_gather_frames(const uint8_t* frames, long seg_stride, FrameSet src, const Geo& g, int B, hipStream_t s) {
  const long n = B * (g.ysz + 2 * g.csz) / 16;
  k_gather_frames<<<(unsigned)tv_min(4096L, (n + 255) / 256), 256, 0, s>>>(frames, seg_stride, src, g, B);
}
// Per-frame slice QPs into the device slot: the values travel as kernel arguments (64 per
// launch) instead of a pinned-host -> device hipMemcpyAsync, which this runtime runs as a
// blit kernel that reads host memory over PCIe (~77 us per picture in the kernel trace).
struct QpArgs {
  int8_t q[64];
};
__global__ void __launch_bounds__(64) k_set_qp(int8_t* dst, QpArgs a, int n) {
  if ((int)threadIdx.x < n) dst[threadIdx.x] = a.q[threadIdx.x];
}
void launch_set_qp(int8_t* dst, const int8_t* host, int n, hipStream_t s) {
  for (int o = 0; o < n; o += 64) {
    QpArgs a;
    const int m = n - o < 64 ? n - o : 64;
    std::memcpy(a.q, host + o, (size_t)m);
    k_set_qp<<<1, 64, 0, s>>>(dst + o, a, m);
  }
}

void launch_sse(FrameSet a, FrameSet r, const Geo& g, unsigned long long* sse, int B, hipStream_t s) {
  dim3 grid((unsigned)tv_min(256, (int)((g.ysz / 4 + 4095) / 4096)), 3, B);
  k_sse<<<grid, 256, 0, s>>>(a, r, g, sse);
}
void launch_phase_planes(FrameSet ref, uint8_t* phase, const Geo& g, int B, hipStream_t s) {
  dim3 grid((g.W + 16 + 31) / 32, (g.H + 16 + 31) / 32, B);
  k_phase_planes<<<grid, 256, 0, s>>>(ref, phase, g);
}
// ---------------------------------------- SAO ------------------------------------------
// One block per CTB: statistics -> integer RD decision -> the SAO'd CTB, in one launch.  The
// deblocked CTB of every component plus a one-sample border is staged in LDS (-1 marks
// samples outside the picture; every global load of the stage is issued before the first
// store), so the EO neighbour reads of both the statistics and the filter never touch global
// memory, and the filtered CTB is written straight from the tile (no separate apply pass
// re-reading the deblocked frame).  Statistics without LDS-atomic storms:
//   * EO: each thread accumulates its samples' 4 classes x 4 categories (count, sum) in
//     registers; one DPP wave reduction per counter, one LDS add per wave;
//   * band: per wave, loop over the distinct bands present (ballot + readlane): one wave
//     reduction and one LDS add per distinct band.
// Then the shared integer RD decision (tv::sao_item / sao_window / sao_finish_pos: identical
// to the CPU golden model), the band-position argmin of the 3 components on 3 waves.
constexpr int kSaoT = 34;   // luma tile side with border
constexpr int kSaoTc = 18;  // chroma
// Tile rows are stored with pitch T + 2 and one column of offset, so a sample pair (even x,
// x + 1) of the CTB is one aligned dword: the packed statistics read pairs as ds_read_b32.
constexpr int kSaoP = kSaoT + 2, kSaoPc = kSaoTc + 2;
constexpr int kSaoTile = kSaoT * kSaoP + 2 * kSaoTc * kSaoPc;
constexpr int kSaoStage = (kSaoTile + 255) / 256;
// tile index of (row, col) of component c (row / col 0 = the one-sample border)
__device__ __forceinline__ int sao_tix(int c, int row, int col) {
  return c == 0 ? row * kSaoP + col + 1 : kSaoT * kSaoP + (c - 1) * kSaoTc * kSaoPc + row * kSaoPc + col + 1;
}
typedef short sao_s2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ sao_s2 sao_pair(uint32_t w) { return __builtin_bit_cast(sao_s2, w); }
typedef unsigned short sao_u2 __attribute__((ext_vector_type(2)));
// per half: -1, 0, 1 for |d| < 2^15 -- shifts and an OR (v_pk_ashrrev / v_pk_lshrrev), no
// compares: (d >> 15) is -1 for d < 0, ((-d) >>> 15) is 1 for d > 0
__device__ __forceinline__ sao_s2 sao_sign2(sao_s2 d) {
  const sao_s2 z = {0, 0};
  const sao_u2 f = {15, 15};
  return (d >> 15) | __builtin_bit_cast(sao_s2, __builtin_bit_cast(sao_u2, z - d) >> f);
}
__device__ __forceinline__ sao_s2 sao_relu2(sao_s2 e) { return e & ~(e >> 15); }  // max(e, 0)
// v_pk_max_i16 / v_pk_min_i16 (clang lowers a packed clamp to -1..1 as a sign idiom of
// per-half compares and selects, so these are spelled out)
__device__ __forceinline__ sao_s2 sao_pkmax(sao_s2 a, sao_s2 b) {
  uint32_t r;
  asm("v_pk_max_i16 %0, %1, %2" : "=v"(r) : "v"(__builtin_bit_cast(uint32_t, a)), "v"(__builtin_bit_cast(uint32_t, b)));
  return sao_pair(r);
}
__device__ __forceinline__ sao_s2 sao_pkmin(sao_s2 a, sao_s2 b) {
  uint32_t r;
  asm("v_pk_min_i16 %0, %1, %2" : "=v"(r) : "v"(__builtin_bit_cast(uint32_t, a)), "v"(__builtin_bit_cast(uint32_t, b)));
  return sao_pair(r);
}

__device__ __forceinline__ void sao_tile_pos(int i, int& c, int& j) {
  c = i < kSaoT * kSaoT ? 0 : (i < kSaoT * kSaoT + kSaoTc * kSaoTc ? 1 : 2);
  j = c == 0 ? i : i - kSaoT * kSaoT - (c - 1) * kSaoTc * kSaoTc;
}

__global__ void __launch_bounds__(256) k_sao_decide(FrameSet src, FrameSet deb, FrameSet out, uint32_t* sao, Geo g,
                                                    const int8_t* qp, const RcTables* rc, int diag,
                                                    unsigned long long* sse) {
  const int tid = threadIdx.x, lane = tid & 63;
  int ctu, b;
  xcd_ctb(ctu, b);
  const long long lam16 = rc->sao_lam16[qp[b]];
  const int cx = ctu % g.wc, cy = ctu / g.wc;
  __shared__ SaoStats st[3];
  __shared__ __align__(16) int16_t tile[kSaoTile];  // luma 34 x 34, then Cb, Cr 18 x 18 (sao_tix)
  __shared__ int bpos[3];
  // band statistics: a packed (sum * 2048 + count) histogram per component with 16 copies
  // (lane & 15), so same-band lanes of a wave rarely hit one LDS address
  __shared__ int bh[3][32][16];
  for (int i = tid; i < 3 * (int)(sizeof(SaoStats) / 4); i += 256) reinterpret_cast<int*>(st)[i] = 0;
  if (kSaoBandOffsets)
    for (int i = tid; i < 3 * 32 * 16; i += 256) (&bh[0][0][0])[i] = 0;
  {  // deblocked CTB + 1-sample ring as aligned dwords (a CTB edge is a multiple of 4, so a
     // dword is wholly inside or wholly outside the plane): luma 34 rows x 10 dwords (items
     // tid, tid + 256), chroma 2 x 18 rows x 6 dwords (item tid); each slot has one component,
     // so the row / dword split is a division by a constant.  Every load is issued before the
     // first LDS store.  The 4 bytes land as two int16 pairs (v_perm), each one aligned
     // dword store: dword d of a row covers tile columns 4d - 3 .. 4d, so pair 0 is stored
     // for d >= 1 and pair 1 for d < last (column -1 / T are the pitch padding, never read).
    uint32_t* tile32 = reinterpret_cast<uint32_t*>(tile);
    uint32_t v[3];
    int at[3], dw[3], nd[3];
    bool act[3], in[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      int c, row, d;
      if (k < 2) {
        const int i = tid + 256 * k;
        c = 0;
        row = i / 10;
        d = i - 10 * row;
        act[k] = i < 34 * 10;
      } else {
        const int pl = tid >= 108 ? 1 : 0, j = tid - 108 * pl;
        c = 1 + pl;
        row = j / 6;
        d = j - 6 * row;
        act[k] = tid < 2 * 108;
      }
      const int n = c ? 16 : 32, w = c ? g.W / 2 : g.W, h = c ? g.H / 2 : g.H;
      const int x = cx * n - 4 + 4 * d, y = cy * n - 1 + row;
      in[k] = act[k] && x >= 0 && x < w && y >= 0 && y < h;
      v[k] = in[k] ? *reinterpret_cast<const uint32_t*>(deb.plane(c, b, g) + (long)y * w + x) : 0u;
      at[k] = (sao_tix(c, row, -1) >> 1) + 2 * d - 1;  // dword of tile columns 4d - 3, 4d - 2
      dw[k] = d;
      nd[k] = c ? 6 : 10;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      if (!act[k]) continue;
      const uint32_t lo = in[k] ? __builtin_amdgcn_perm(0u, v[k], 0x0c010c00u) : 0xFFFFFFFFu;  // outside: -1 pairs
      const uint32_t hi = in[k] ? __builtin_amdgcn_perm(0u, v[k], 0x0c030c02u) : 0xFFFFFFFFu;
      if (dw[k] >= 1) tile32[at[k]] = lo;
      if (dw[k] < nd[k] - 1) tile32[at[k] + 1] = hi;
    }
  }
  // one region per wave: waves 0/1 = luma rows 0-15 / 16-31, wave 2 = Cb, wave 3 = Cr.
  // Counts and sums travel packed as sum * 2048 + count (count <= 1024, |sum| <= 255 * 1024):
  // one wave reduction per EO counter, not two.
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: scalar component logic
  const int c = wave < 2 ? 0 : wave - 1;
  const int n = c ? 16 : 32, w = c ? g.W / 2 : g.W;
  const int nsh = c ? 4 : 5;  // log2 n: the sample index splits with shifts, not a runtime division
  const int iters = c ? 4 : 8;
  const uint8_t* S = src.plane(c, b, g) + (long)(cy * n) * w + cx * n;
  // A CTB away from the picture edge has no outside (-1) neighbours: its statistics run on
  // sample PAIRS in packed 16-bit arithmetic (v_pk_*: two samples per instruction, the 9
  // neighbour dwords of a pair read once for all 4 classes).  Edge CTBs take the per-sample
  // path with the validity checks.  Both give the same counters.
  static_assert(!kSaoBandOffsets, "the packed statistics carry no band histogram");
  const bool packed = !(diag & 16);  // 16: TV_SAO_PACKED=0 (A/B: per-sample statistics and filter)
  const bool interior = cx > 0 && cy > 0 && cx < g.wc - 1 && cy < g.hc - 1 && packed;
  diag &= 15;
  const int piters = c ? 2 : 4;  // pairs per lane: luma 16 rows x 16 pairs, chroma 16 x 8
  int sv[8] = {};
  uint32_t sp[4] = {};
  if (interior) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // source pairs of this lane, loads in flight together
      const int pidx = lane + 64 * k;
      const int ly = (c == 0 ? wave * 16 : 0) + (pidx >> (nsh - 1)), lx = 2 * (pidx & ((n >> 1) - 1));
      sp[k] = k < piters ? *reinterpret_cast<const uint16_t*>(S + ly * w + lx) : 0u;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) {  // source samples of this lane, loads in flight together
      const int i = (c == 0 ? wave * 512 : 0) + lane + 64 * k;
      sv[k] = k < iters ? S[(i >> nsh) * w + (i & (n - 1))] : 0;
    }
  }
  __syncthreads();
  // timing diagnostics only (TV_DIAG_SAO_STOP=1/2/3: stop after staging / statistics /
  // decision; the output is then incomplete) -- never set in production
  if (diag == 1) {
    if (tid == 0) sao[3 * ((long)b * g.wc * g.hc + ctu)] = (uint32_t)(sv[0] + sp[0] + tile[tid]);
    return;
  }
  int eo[4][4];
  if (interior) {
    const uint32_t* tile32 = reinterpret_cast<const uint32_t*>(tile);
    // per half and (class, category): sum(orig - deb) * 16 + count, one v_pk_mad per bin
    // (count <= 4 samples per half, |sum| <= 4 * 255: |acc| < 2^14)
    sao_s2 acc[4][4];
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[d][q] = sao_s2{0, 0};
    const sao_s2 zero = {0, 0}, one = {1, 1}, mone = {-1, -1}, sixteen = {16, 16};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k >= piters) break;
      const int pidx = lane + 64 * k;
      const int ly = (c == 0 ? wave * 16 : 0) + (pidx >> (nsh - 1)), lx = 2 * (pidx & ((n >> 1) - 1));
      uint32_t Pv[3], Cv[3], Nv[3];  // rows ly - 1, ly, ly + 1: dwords at lx - 2, lx, lx + 2
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int i0 = sao_tix(c, ly + r, lx + 1) >> 1;  // tile column lx + 1 = sample lx (even index)
        Pv[r] = tile32[i0 - 1];
        Cv[r] = tile32[i0];
        Nv[r] = tile32[i0 + 1];
      }
      sao_s2 L[3], R[3], Cc[3];
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        L[r] = sao_pair(__builtin_amdgcn_alignbyte(Cv[r], Pv[r], 2));  // samples (lx - 1, lx)
        R[r] = sao_pair(__builtin_amdgcn_alignbyte(Nv[r], Cv[r], 2));  // samples (lx + 1, lx + 2)
        Cc[r] = sao_pair(Cv[r]);
      }
      const sao_s2 v = Cc[1];
      const uint32_t o = sp[k];
      const sao_s2 orig = {(short)(o & 255), (short)(o >> 8)};
      const sao_s2 w = (orig - v) * sixteen + one;
      // classes (sao_eo_dir): 0 horizontal, 1 vertical, 2 135 degrees, 3 45 degrees
      const sao_s2 A[4] = {L[1], Cc[0], L[0], R[0]}, Bn[4] = {R[1], Cc[2], R[2], L[2]};
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const sao_s2 e = sao_pkmin(sao_pkmax(v - A[d], mone), one) + sao_pkmin(sao_pkmax(v - Bn[d], mone), one);
        const sao_s2 pos = sao_pkmax(e, zero), neg = sao_pkmax(zero - e, zero);
        const sao_s2 is[4] = {neg >> one, neg & one, pos & one, pos >> one};  // categories 1..4
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[d][q] += w * is[q];
      }
    }
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
      for (int q = 0; q < 4; ++q) {  // both halves: F = 16 * sum + count (count <= 8)
        const int F = __builtin_amdgcn_sdot2(acc[d][q], one, 0, false), C = F & 15;
        eo[d][q] = (F - C) * 128 + C;  // sum * 2048 + count
      }
  } else {
    // EO statistics per lane in one 64-bit register per class: four signed 16-bit fields
    // (category 1..4) of sum(orig - deb) * 16 + count over the lane's <= 8 samples (|field| <=
    // 255 * 8 * 16 + 8 < 2^15), added as one shifted 64-bit value per (sample, class) instead
    // of four compare/select/adds; unpacked into the wave-sum format afterwards.
    unsigned long long eo64[4] = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k >= iters) break;
      const int i = (c == 0 ? wave * 512 : 0) + lane + 64 * k;
      const int lx = i & (n - 1), ly = i >> nsh;
      const int v = tile[sao_tix(c, ly + 1, lx + 1)];
      const int d16 = (sv[k] - v) * 16 + 1;
      const unsigned long long p64 = (unsigned long long)(long long)d16;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        int dx, dy;
        sao_eo_dir(d, dx, dy);
        const int a = tile[sao_tix(c, ly + 1 + dy, lx + 1 + dx)], bb = tile[sao_tix(c, ly + 1 - dy, lx + 1 - dx)];
        const int e = tv_min(tv_max(v - a, -1), 1) + tv_min(tv_max(v - bb, -1), 1);  // -2..2, 0 = none
        const int f = e + 2 - (e > 0);  // category 1..4 -> field 0..3 (e = 0 is masked below)
        eo64[d] += (a >= 0 && bb >= 0 && e != 0) ? p64 << (16 * f) : 0ull;
      }
      if (kSaoBandOffsets) atomicAdd(&bh[c][v >> 3][lane & 15], (sv[k] - v) * 2048 + 1);  // band statistics
    }
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      unsigned long long acc = eo64[d];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int fv = (int)(int16_t)(acc & 0xffffu);  // 16 * sum + count
        acc = (acc - (unsigned long long)(long long)fv) >> 16;
        const int cnt = fv & 15;
        eo[d][q] = ((fv - cnt) >> 4) * 2048 + cnt;  // sum * 2048 + count, as before
      }
    }
  }
  {  // the 16 counters of the wave in one transpose-reduce: each exchange step (lanes 32,
     // 16, 8, 4 apart) halves the values a lane holds -- it keeps one half and adds the
     // partner's copy of it -- so lane L ends with counter (L >> 2) summed over 16 lanes; two
     // quad DPP adds finish the sum (~40 VALU instead of 16 full wave reductions).  Lanes 32
     // / 16 apart swap with v_permlane32_swap / v_permlane16_swap (gfx950), lanes 8 apart
     // with a DPP row rotate; the halves are chosen with xor masks, not selects (a select
     // of two array elements became a dynamically indexed array)
    int t[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) t[k] = eo[k >> 2][k & 3];
#pragma unroll
    for (int j = 0; j < 8; ++j) {  // lanes 0-31 keep t[j], lanes 32-63 t[j + 8]
      const auto r = __builtin_amdgcn_permlane32_swap((unsigned)t[j], (unsigned)t[j + 8], false, false);
      t[j] = (int)(r[0] + r[1]);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // even 16-lane rows keep t[j], odd rows t[j + 4]
      const auto r = __builtin_amdgcn_permlane16_swap((unsigned)t[j], (unsigned)t[j + 4], false, false);
      t[j] = (int)(r[0] + r[1]);
    }
    const int m8 = -((lane >> 3) & 1), m4 = -((lane >> 2) & 1);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int x = (t[j] ^ t[j + 2]) & m8;
      t[j] = (t[j] ^ x) + dpp::mov<dpp::kRowRor8>(t[j + 2] ^ x);
    }
    {
      const int x = (t[0] ^ t[1]) & m4;
      t[0] = (t[0] ^ x) + __shfl_xor(t[1] ^ x, 4, 64);
    }
    int tot = t[0];
    tot += dpp::mov<dpp::kQuadXor1>(tot);
    tot += dpp::mov<dpp::kQuadXor2>(tot);
    const int k = lane >> 2;  // class k >> 2, category (k & 3) + 1
    if ((lane & 3) == 0 && (tot & 2047)) {
      atomicAdd(&st[c].eo_n[k >> 2][(k & 3) + 1], tot & 2047);
      atomicAdd(&st[c].eo_s[k >> 2][(k & 3) + 1], (tot - (tot & 2047)) / 2048);
    }
  }
  __shared__ SaoTables tab;
  __shared__ uint32_t prm[3];
  __syncthreads();
  if (kSaoBandOffsets && tid < 96) {  // fold the histogram copies into the band counters
    const int cc = tid >> 5, band = tid & 31;
    int tot = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) tot += bh[cc][band][k];
    st[cc].bo_n[band] = tot & 2047;
    st[cc].bo_s[band] = (tot - (tot & 2047)) / 2048;
  }
  __syncthreads();
  if (diag == 2) {
    if (tid == 0) sao[3 * ((long)b * g.wc * g.hc + ctu)] = (uint32_t)st[0].eo_n[0][1];
    return;
  }
  // 144 offset/cost items in parallel (the 96 band items only with band offsets on)
  if (tid < kSaoItems && (kSaoBandOffsets || tid % 48 < 16)) sao_item(st, lam16, tid, tab);
  __syncthreads();
  if (kSaoBandOffsets && tid < 96) sao_window(tid, tab);  // 3 x 32 band windows
  __syncthreads();
  if (!kSaoBandOffsets) {
    if (tid < 3) bpos[tid] = 0;
  } else if (wave < 3) {  // best band position of component `wave`: first minimum over 32 windows
    long long j = lane < 32 ? tab.win_j[wave][lane] : LLONG_MAX;
    int p = lane < 32 ? lane : 64;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const long long j2 = __shfl_xor(j, o);
      const int p2 = __shfl_xor(p, o);
      if (j2 < j || (j2 == j && p2 < p)) {
        j = j2;
        p = p2;
      }
    }
    if (lane == 0) bpos[wave] = p;
  }
  __syncthreads();
  if (tid == 0) {
    sao_finish_pos(tab, lam16, bpos, prm);
    uint32_t* o = sao + 3 * ((long)b * g.wc * g.hc + ctu);
    o[0] = prm[0];
    o[1] = prm[1];
    o[2] = prm[2];
  }
  if (diag == 3) return;
  __syncthreads();
  // the SAO'd CTB from the tile, 4 samples per dword store: luma 32 rows x 8, chroma 16 x 4;
  // the squared error against the source (display area) is summed on the way (no k_sse).
  // Packed: the dword's samples are two int16 pairs of the tile (aligned dwords; the EO
  // neighbours of a +-1 column shift are v_alignbyte of two), the category index e + 2 of
  // both halves selects the biased offsets with one v_perm, and the squared error is a
  // v_dot2 of the differences.  Neighbours outside the picture (-1) leave the sample as is.
  static_assert(!kSaoBandOffsets, "the SAO filter has no band-offset path");
  unsigned e2[3] = {0, 0, 0};
  const uint32_t* tile32 = reinterpret_cast<const uint32_t*>(tile);
  for (int i = tid; i < 256 + 128; i += 256) {
    const int cc = i < 256 ? 0 : (i < 320 ? 1 : 2);
    const int j = cc == 0 ? i : i - 256 - (cc - 1) * 64;
    const int nd = cc ? 4 : 8, nn = cc ? 16 : 32, ww = cc ? g.W / 2 : g.W;
    const int ly = j >> (cc ? 2 : 3), lx0 = 4 * (j & (nd - 1));  // nd = 4 / 8 dwords per row
    const uint32_t p = prm[cc];
    const long at = (long)(cy * nn + ly) * ww + cx * nn + lx0;
    const int dwc = cc ? g.dw / 2 : g.dw, dhc = cc ? g.dh / 2 : g.dh;
    const bool want_sse = sse && cy * nn + ly < dhc;
    const uint32_t sw = want_sse ? *reinterpret_cast<const uint32_t*>(src.plane(cc, b, g) + at) : 0u;
    uint32_t word = 0;
    if (packed) {
      const int i0 = sao_tix(cc, ly + 1, lx0 + 1) >> 1;  // pairs (lx0, lx0 + 1), (lx0 + 2, lx0 + 3)
      const uint32_t C0 = tile32[i0], C1 = tile32[i0 + 1];
      if (sao_type(p) == 2) {
        int dx, dy;
        sao_eo_dir(sao_class(p), dx, dy);
        const int pd = (cc ? kSaoPc : kSaoP) >> 1;  // dwords per tile row
        const int ra = i0 + dy * pd, rb = i0 - dy * pd;
        const uint32_t Wa[4] = {tile32[ra - 1], tile32[ra], tile32[ra + 1], tile32[ra + 2]};
        const uint32_t Wb[4] = {tile32[rb - 1], tile32[rb], tile32[rb + 1], tile32[rb + 2]};
        // pair k of a row shifted by s columns (s = -1, 0, 1): dwords W[k .. k + 2] = columns
        // lx0 + 2k - 2 .. lx0 + 2k + 3
        auto shifted = [](const uint32_t* W, int k, int s) -> uint32_t {
          return s == 0 ? W[k + 1] : s < 0 ? __builtin_amdgcn_alignbyte(W[k + 1], W[k], 2)
                                           : __builtin_amdgcn_alignbyte(W[k + 2], W[k + 1], 2);
        };
        // biased offsets (o + 8) by category index e + 2: bytes {o0, o1, 8 (none), o2 | o3}
        const uint32_t t0 = ((p >> 7) & 15) | ((p >> 11) & 15) << 8 | 8u << 16 | ((p >> 15) & 15) << 24;
        const uint32_t t1 = (p >> 19) & 15;
        const sao_s2 two = {2, 2}, eight = {8, 8};
        const sao_u2 u8s = {8, 8};
        uint32_t r2[2];
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const sao_s2 v = sao_pair(k ? C1 : C0);
          const sao_s2 A = sao_pair(shifted(Wa, k, dx)), B = sao_pair(shifted(Wb, k, -dx));
          const sao_s2 inv = (A | B) >> 15;  // -1 where a neighbour is outside the picture
          const sao_s2 e = (sao_sign2(v - A) + sao_sign2(v - B)) & ~inv;
          const uint32_t sel = __builtin_bit_cast(uint32_t, e + two) | 0x0c000c00u;
          const sao_s2 off = sao_pair(__builtin_amdgcn_perm(t1, t0, sel));
          const sao_s2 r = sao_relu2(v + off - eight);  // -7 .. 262 -> 0 .. 262
          // >= 256 -> low byte 0xFF (only the low byte of each half is kept)
          r2[k] = __builtin_bit_cast(uint32_t, r | (sao_s2{0, 0} - __builtin_bit_cast(sao_s2, __builtin_bit_cast(sao_u2, r) >> u8s)));
        }
        word = __builtin_amdgcn_perm(r2[1], r2[0], 0x06040200u);
      } else {
        word = __builtin_amdgcn_perm(C1, C0, 0x06040200u);
      }
    } else {
      int dx = 0, dy = 0;
      if (sao_type(p) == 2) sao_eo_dir(sao_class(p), dx, dy);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int lx = lx0 + q;
        const int v = tile[sao_tix(cc, ly + 1, lx + 1)];
        const int r = sao_type(p) ? sao_sample_nb(v, tile[sao_tix(cc, ly + 1 + dy, lx + 1 + dx)],
                                                  tile[sao_tix(cc, ly + 1 - dy, lx + 1 - dx)], p)
                                  : v;
        word |= (uint32_t)r << (8 * q);
      }
    }
    *reinterpret_cast<uint32_t*>(out.plane(cc, b, g) + at) = word;
    if (want_sse) {
      if (cx * nn + lx0 + 4 <= dwc) {  // the whole dword is in the display area
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const uint32_t sel = h ? 0x0c030c02u : 0x0c010c00u;
          const sao_s2 d = sao_pair(__builtin_amdgcn_perm(0u, sw, sel)) - sao_pair(__builtin_amdgcn_perm(0u, word, sel));
          const sao_u2 dd = __builtin_bit_cast(sao_u2, d * d);  // <= 65025 per half
          e2[cc] = __builtin_amdgcn_udot2(dd, sao_u2{1, 1}, e2[cc], false);
        }
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int d = (int)((sw >> (8 * q)) & 255) - (int)((word >> (8 * q)) & 255);
          e2[cc] += cx * nn + lx0 + q < dwc ? (unsigned)(d * d) : 0u;
        }
      }
    }
  }
  if (sse) {
    __shared__ unsigned long long esum[3];
    if (tid < 3) esum[tid] = 0;
    __syncthreads();
#pragma unroll
    for (int c2 = 0; c2 < 3; ++c2) {
      const int t = wave_sum((int)e2[c2]);  // <= 2 dwords x 4 x 65025 per lane: fits
      if (lane == 0 && t) atomicAdd(&esum[c2], (unsigned long long)(unsigned)t);
    }
    __syncthreads();
    if (tid < 3 && esum[tid]) atomicAdd(sse + b * 3 + tid, esum[tid]);
  }
}

void launch_sao(FrameSet src, FrameSet deb, FrameSet out, uint32_t* sao, const int8_t* qp, const RcTables* rc,
                const Geo& g, int B, hipStream_t s, unsigned long long* sse) {
  static const int diag = [] {
    const char* e = std::getenv("TV_DIAG_SAO_STOP");
    const char* pk = std::getenv("TV_SAO_PACKED");
    return (e ? std::atoi(e) : 0) | (pk && std::atoi(pk) == 0 ? 16 : 0);
  }();
  k_sao_decide<<<dim3(g.wc * g.hc, B), 256, 0, s>>>(src, deb, out, sao, g, qp, rc, diag, sse);
}

void launch_deblock(FrameSet rec, DecisionSet dec, const Geo& g, int B, hipStream_t s) {
  dim3 grid((unsigned)tv_min(1024, (int)(g.ysz / 32 / 256 + 1)), B);
  k_deblock<<<grid, 256, 0, s>>>(rec, dec, g, 0);
  k_deblock<<<grid, 256, 0, s>>>(rec, dec, g, 1);
}

}  // namespace gpu
}  // namespace tv
