// k_stage.hip — device-side staging of job sources into the encode engine (no host bounce).
//
// The job path (worker / node executor) feeds engines from device buffers: a source
// segment is uploaded once (or received over RCCL, or generated on the GPU), optionally
// tone-mapped / Lanczos-resized, and written straight into the engine's coded-size staging
// layout [segment][frame][Y | U | V] — the edge padding to the coded size is done here, on
// the GPU, instead of numpy on the host (reference analogue: ffmpeg's `scale` +
// `format=nv12,hwupload` chain, worker/tasks.py:436-449).
//
//  k_pad_plane   display-size plane -> coded-size plane with edge replication, batched
//  tv_synth_batch  the seeded synthetic source (tv/synth.h) generated for n frames on the
//                  GPU at coded size in planar-batched layout (Y of every frame, then U, V)
#include <hip/hip_runtime.h>

#include <string>

#include "gpu_common.h"
#include "k_encode.h"

namespace tv {
namespace gpu {

// dst[f][y][x] = src[f][min(y, sh-1)][min(x, sw-1)] for x < pw, y < ph; 4 bytes per thread
__global__ void __launch_bounds__(256) k_pad_plane(const uint8_t* __restrict__ src, int sw, int sh, int sstride, long sfs,
                                                   uint8_t* __restrict__ dst, int pw, int ph, int dstride, long dfs) {
  const int f = blockIdx.z, y = blockIdx.y;
  const int x0 = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (x0 >= pw) return;
  const uint8_t* S = src + f * sfs + (long)tv_min(y, sh - 1) * sstride;
  uint8_t* D = dst + f * dfs + (long)y * dstride;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (x0 + k < pw) D[x0 + k] = S[tv_min(x0 + k, sw - 1)];
}

// 8x8 block means of n luma planes (scene-cut thumbnails, models/scenecut.py): one thread per
// block, straight from the 8- or 16-bit samples (the sum of 64 samples and the / 64 are exact
// in float, so any summation order gives the same value; 10-bit samples are scaled by 1/4).
template <typename T>
__global__ void __launch_bounds__(256) k_thumbs8(const T* __restrict__ y, int tw, int stride, long fs, float* out,
                                                 float scale) {
  const int x = blockIdx.x * 256 + threadIdx.x, r = blockIdx.y, f = blockIdx.z;
  if (x >= tw) return;
  const T* p = y + (long)f * fs + (long)(8 * r) * stride + 8 * x;
  unsigned s = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) s += p[(long)j * stride + i];
  out[((long)f * gridDim.y + r) * tw + x] = (float)s * scale / 64.0f;
}
}  // namespace gpu
}  // namespace tv

namespace {
thread_local std::string g_stage_err;
int stage_status() {
  const hipError_t e = hipGetLastError();
  if (e == hipSuccess) return 0;
  g_stage_err = hipGetErrorString(e);
  return -1;
}
}  // namespace

extern "C" {
const char* tv_stage_last_error() { return g_stage_err.c_str(); }

// 8x8 block means of n luma planes (element offsets / strides; bits 8 or 10) -> out
// [n][h / 8][w / 8] float
int tv_thumbs8_batch(const void* y, int bits, int w, int h, int stride, long fs, int n, float* out, void* stream) {
  const int tw = w / 8, th = h / 8;
  if (tw <= 0 || th <= 0 || th > 65535 || n <= 0 || n > 65535 || stride < w) {
    g_stage_err = "tv_thumbs8_batch: bad geometry";
    return -1;
  }
  const dim3 grid((unsigned)((tw + 255) / 256), (unsigned)th, (unsigned)n);
  hipStream_t st = static_cast<hipStream_t>(stream);
  if (bits > 8)
    tv::gpu::k_thumbs8<uint16_t><<<grid, 256, 0, st>>>(static_cast<const uint16_t*>(y), tw, stride, fs, out, 0.25f);
  else
    tv::gpu::k_thumbs8<uint8_t><<<grid, 256, 0, st>>>(static_cast<const uint8_t*>(y), tw, stride, fs, out, 1.0f);
  return stage_status();
}

// n frames of one plane: display (sw x sh, row stride sstride, frame stride sfs) -> coded
// (pw x ph, row stride dstride, frame stride dfs) with edge replication
int tv_pad_batch(const uint8_t* src, int sw, int sh, int sstride, long sfs, uint8_t* dst, int pw, int ph, int dstride,
                 long dfs, int n, void* stream) {
  if (sw <= 0 || sh <= 0 || pw < sw || ph < sh || dstride < pw || sstride < sw || n <= 0 || n > 65535 ||
      ph > 65535) {
    g_stage_err = "tv_pad_batch: bad geometry";
    return -1;
  }
  const dim3 grid((unsigned)((pw / 4 + 255) / 256 + 1), (unsigned)ph, (unsigned)n);
  tv::gpu::k_pad_plane<<<grid, 256, 0, static_cast<hipStream_t>(stream)>>>(src, sw, sh, sstride, sfs, dst, pw, ph,
                                                                          dstride, dfs);
  return stage_status();
}

// Synthetic frames t[0..n) of a w x h (display) source at coded size, planar-batched:
// Y planes of all n frames, then U planes, then V planes (coded pitch, edge replicated).
int tv_synth_batch(uint8_t* dst, int w, int h, int n, const int* t, uint32_t seed, void* stream) {
  if (w < 2 || h < 2 || (w & 1) || (h & 1) || n <= 0) {
    g_stage_err = "tv_synth_batch: bad geometry";
    return -1;
  }
  const tv::gpu::Geo g = tv::gpu::make_geo(w, h);
  for (int b0 = 0; b0 < n; b0 += tv::gpu::kMaxBatch) {
    const int B = tv::tv_min(tv::gpu::kMaxBatch, n - b0);
    tv::gpu::FrameSet fs{dst + b0 * g.ysz, dst + n * g.ysz + b0 * g.csz, dst + n * g.ysz + n * g.csz + b0 * g.csz};
    tv::gpu::FrameIdx fi{};
    for (int b = 0; b < B; ++b) fi.t[b] = t[b0 + b];
    tv::gpu::launch_synth(fs, g, seed, fi, B, static_cast<hipStream_t>(stream));
  }
  return stage_status();
}
}
