// k_compact.hip — coefficient compaction before the device->host transfer.
//
// A 1080p frame's dense level planes are 6.3 MB (int16) but at QP 27 only a few percent of
// the 4x4 coefficient groups are non-zero.  Per CTB: a 64-bit luma + 2x16-bit chroma mask
// of non-zero 4x4 groups and their count; per segment an exclusive scan over CTBs; then the
// non-zero groups are packed (16 x int16 each, CTB order: Y raster, Cb raster, Cr raster).
// The CABAC writer reads levels straight from this form (tv::FrameData compact mode).
#include "gpu_common.h"
#include "k_encode.h"

namespace tv {
namespace gpu {

// one wave per CTB: lanes 0..63 = luma groups, then 32 chroma groups
__global__ void __launch_bounds__(256) k_sb_count(DecisionSet dec, Geo g, CompactSet cs) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ctu = blockIdx.x * 4 + wave, b = blockIdx.y;
  const int nctu = g.wc * g.hc;
  if (ctu >= nctu) return;
  const int cx = (ctu % g.wc) * 32, cy = (ctu / g.wc) * 32;
  const int16_t* Y = dec.coef_y + b * g.ysz;
  // the 8x8 unit's cbf bits (luma 1, Cb 2, Cr 4) say which groups can hold levels at all: a
  // TB with cbf 0 is not coded, so its (zero) level rows are not read -- at QP 27 most of the
  // 6.3 MB of dense level planes per 1080p frame
  const uint8_t* cbf = dec.cbf + b * g.usz + (long)(cy >> 3) * g.w8 + (cx >> 3);
  bool nzy = false;
  {
    const int sx = lane & 7, sy = lane >> 3;
    if (cbf[(sy >> 1) * g.w8 + (sx >> 1)] & 1) {
      const int16_t* p = Y + (long)(cy + 4 * sy) * g.W + cx + 4 * sx;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint2 v = *reinterpret_cast<const uint2*>(p + (long)r * g.W);
        nzy |= (v.x | v.y) != 0;
      }
    }
  }
  bool nzc = false;
  if (lane < 32) {
    const int16_t* C = (lane < 16 ? dec.coef_u : dec.coef_v) + b * g.csz;
    const int l = lane & 15, sx = l & 3, sy = l >> 2, Wc = g.W / 2;
    if (cbf[sy * g.w8 + sx] & (lane < 16 ? 2 : 4)) {  // chroma 4x4 group (sx, sy) = luma unit (sx, sy)
      const int16_t* p = C + (long)(cy / 2 + 4 * sy) * Wc + cx / 2 + 4 * sx;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint2 v = *reinterpret_cast<const uint2*>(p + (long)r * Wc);
        nzc |= (v.x | v.y) != 0;
      }
    }
  }
  const unsigned long long my = __ballot(nzy);
  const unsigned long long mc = __ballot(nzc);
  if (lane == 0) {
    const long i = (long)b * nctu + ctu;
    cs.mask_y[i] = my;
    cs.mask_c[i] = (unsigned)mc;
    cs.count[i] = __popcll(my) + __popcll(mc);
  }
}

// exclusive scan of per-CTB counts, one workgroup per segment
__global__ void __launch_bounds__(1024) k_sb_scan(Geo g, CompactSet cs) {
  const int b = blockIdx.x, tid = threadIdx.x, nctu = g.wc * g.hc;
  __shared__ int part[1024];
  const int per = (nctu + 1023) / 1024;
  const int lo = tid * per, hi = tv_min(nctu, lo + per);
  const int* cnt = cs.count + (long)b * nctu;
  int s = 0;
  for (int i = lo; i < hi; ++i) s += cnt[i];
  part[tid] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {  // Hillis-Steele inclusive scan
    const int v = tid >= o ? part[tid - o] : 0;
    __syncthreads();
    part[tid] += v;
    __syncthreads();
  }
  int run = tid ? part[tid - 1] : 0;
  int* off = cs.offset + (long)b * nctu;
  for (int i = lo; i < hi; ++i) {
    off[i] = run;
    run += cnt[i];
  }
  if (tid == 1023) cs.total[b] = part[1023];
}

// pack the non-zero groups: one wave per CTB, lane = group bit (luma 0..63, then chroma
// 0..31): a set bit's output slot is the popcount of the bits below it, and its lane copies
// the group's 4 rows (no per-lane walk over the mask)
__global__ void __launch_bounds__(256) k_sb_pack(DecisionSet dec, Geo g, CompactSet cs) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ctu = blockIdx.x * 4 + wave, b = blockIdx.y;
  const int nctu = g.wc * g.hc;
  if (ctu >= nctu) return;
  const int cx = (ctu % g.wc) * 32, cy = (ctu / g.wc) * 32;
  const long i = (long)b * nctu + ctu;
  const unsigned long long my = cs.mask_y[i];
  const unsigned mc = cs.mask_c[i];
  const int ny = __popcll(my);
  // segments are packed back to back (one device->host copy per frame for all of them): the
  // groups of the segments before b, summed across the wave
  int pre = 0;
  for (int k = lane; k < b; k += 64) pre += cs.total[k];
  const long base = wave_sum(pre);
  int16_t* out = cs.packed + (base + cs.offset[i]) * 16;
  if ((my >> lane) & 1) {
    const int gi = __popcll(my & ((1ull << lane) - 1)), sx = lane & 7, sy = lane >> 3;
    const int16_t* src = dec.coef_y + b * g.ysz + (long)(cy + 4 * sy) * g.W + cx + 4 * sx;
#pragma unroll
    for (int row = 0; row < 4; ++row)
      *reinterpret_cast<uint2*>(out + gi * 16 + row * 4) = *reinterpret_cast<const uint2*>(src + (long)row * g.W);
  }
  if (lane < 32 && ((mc >> lane) & 1)) {
    const int gi = ny + __popc(mc & ((1u << lane) - 1)), l = lane & 15, sx = l & 3, sy = l >> 2;
    const long stride = g.W / 2;
    const int16_t* src = (lane < 16 ? dec.coef_u : dec.coef_v) + b * g.csz + (long)(cy / 2 + 4 * sy) * stride + cx / 2 + 4 * sx;
#pragma unroll
    for (int row = 0; row < 4; ++row)
      *reinterpret_cast<uint2*>(out + gi * 16 + row * 4) = *reinterpret_cast<const uint2*>(src + row * stride);
  }
}

__global__ void __launch_bounds__(256) k_pack_flags(DecisionSet dec, uint8_t* flags, long n) {
  for (long u = blockIdx.x * 256L + threadIdx.x; u < n; u += (long)gridDim.x * 256) {
    const int d = dec.dir ? dec.dir[u] : 1;
    // size code 3: an RQT-split inter CU, its size in the intra bit (0: 32x32, 1: 16x16)
    const bool sp = dec.tu && dec.tu[u];
    const int l = sp ? 3 : dec.cu_log2[u] - 3, in = sp ? (dec.cu_log2[u] == 4) : dec.intra[u];
    flags[u] = (uint8_t)(l | (in << 2) | ((dec.cbf[u] & 7) << 3) | (d << 6));
  }
}

void launch_pack_flags(DecisionSet dec, uint8_t* flags, const Geo& g, int B, hipStream_t s) {
  const long n = (long)B * g.usz;
  k_pack_flags<<<(unsigned)tv_min(1024L, (n + 255) / 256), 256, 0, s>>>(dec, flags, n);
}

void launch_compact(DecisionSet dec, const Geo& g, CompactSet cs, int B, hipStream_t s) {
  const int nctu = g.wc * g.hc;
  k_sb_count<<<dim3((nctu + 3) / 4, B), 256, 0, s>>>(dec, g, cs);
  k_sb_scan<<<B, 1024, 0, s>>>(g, cs);
  k_sb_pack<<<dim3((nctu + 3) / 4, B), 256, 0, s>>>(dec, g, cs);
}

}  // namespace gpu
}  // namespace tv
