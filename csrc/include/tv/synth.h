// synth.h — deterministic synthetic video source (seed, frame) -> 8-bit 4:2:0 samples.
//
// The benchmark configs use "synthetic YUV frames / random-seed inputs" (BASELINE.json).
// Pure integer arithmetic so the CPU generator and the HIP generator kernel produce
// byte-identical frames.  Content: a value-noise textured background panning at a
// sub-pixel velocity, plus several textured objects with their own motion (occlusions,
// edges), so motion estimation / skip / intra paths are all exercised like real video.
//
// Seeds with bit 31 set select the *textured* variant (camera-like, hard to compress): a
// 2-pixel lattice detail octave on the background, per-pixel temporal grain (+-4 luma,
// +-2 chroma, a new pattern every frame), a 2.4x faster pan and objects twice as fast.
#pragma once
#include <cstdint>

#include "hevc_defs.h"

namespace tv {

TV_HD uint32_t synth_hash(int32_t x, int32_t y, uint32_t seed) {
  uint32_t h = (uint32_t)x * 374761393u + (uint32_t)y * 668265263u + seed * 2246822519u;
  h = (h ^ (h >> 13)) * 1274126177u;
  return h ^ (h >> 16);
}

// value noise at position (px16, py16) in 1/16-pel units, lattice period 2^lp pixels.
// returns 0..255
TV_HD int synth_vnoise(int32_t px16, int32_t py16, int lp, uint32_t seed) {
  const int sh = lp + 4;
  const int32_t cx = px16 >> sh, cy = py16 >> sh;
  const int fx = (int)((px16 - (cx << sh)) << 8 >> sh);  // 0..255
  const int fy = (int)((py16 - (cy << sh)) << 8 >> sh);
  const int sx = (fx * fx * (768 - 2 * fx)) >> 16;  // smoothstep, 0..256
  const int sy = (fy * fy * (768 - 2 * fy)) >> 16;
  const int a = synth_hash(cx, cy, seed) & 255, b = synth_hash(cx + 1, cy, seed) & 255;
  const int c = synth_hash(cx, cy + 1, seed) & 255, d = synth_hash(cx + 1, cy + 1, seed) & 255;
  const int top = a * 256 + (b - a) * sx;
  const int bot = c * 256 + (d - c) * sx;
  return (top * 256 + (bot - top) * sy) >> 16;
}

struct SynthObject {
  int32_t x16, y16;    // top-left at frame 0 (1/16 pel)
  int32_t vx16, vy16;  // velocity per frame (1/16 pel)
  int32_t w, h;        // size in pixels
  uint32_t seed;
  int shape;  // 0 rect, 1 ellipse
};

TV_HD SynthObject synth_object(uint32_t seed, int k, int W, int H) {
  SynthObject o;
  const uint32_t h0 = synth_hash(k, 17, seed), h1 = synth_hash(k, 29, seed), h2 = synth_hash(k, 43, seed);
  o.w = W / 10 + (int)(h0 % (uint32_t)(W / 6 + 1));
  o.h = H / 10 + (int)(h1 % (uint32_t)(H / 6 + 1));
  o.x16 = (int32_t)((h2 % (uint32_t)W) * 16);
  o.y16 = (int32_t)(((h2 >> 12) % (uint32_t)H) * 16);
  o.vx16 = (int32_t)((h0 >> 16) % 161) - 80;  // up to +-5 px / frame
  o.vy16 = (int32_t)((h1 >> 16) % 97) - 48;   // up to +-3 px / frame
  o.seed = seed * 7919u + (uint32_t)k * 104729u + 1u;
  o.shape = (int)((h2 >> 28) & 1);
  return o;
}

constexpr int kSynthObjects = 6;

// Per-frame state: object positions after bouncing (computed once per frame).
struct SynthFrameCtx {
  uint32_t seed;
  int t, W, H;
  SynthObject obj[kSynthObjects];
  int32_t ox[kSynthObjects], oy[kSynthObjects];
};

constexpr uint32_t kSynthTextured = 0x80000000u;
TV_HD bool synth_textured(uint32_t seed) { return (seed & kSynthTextured) != 0; }

TV_HD void synth_frame_ctx(uint32_t seed, int t, int W, int H, SynthFrameCtx& f) {
  const int speed = synth_textured(seed) ? 2 : 1;
  f.seed = seed;
  f.t = t;
  f.W = W;
  f.H = H;
  for (int k = 0; k < kSynthObjects; ++k) {
    const SynthObject o = synth_object(seed, k, W, H);
    f.obj[k] = o;
    // bounce inside the frame: triangle wave of the trajectory
    const int32_t spanx = (W - o.w) * 16, spany = (H - o.h) * 16;
    int32_t ox = o.x16 + o.vx16 * speed * t, oy = o.y16 + o.vy16 * speed * t;
    if (spanx > 0) {
      int32_t m = ox % (2 * spanx);
      if (m < 0) m += 2 * spanx;
      ox = m < spanx ? m : 2 * spanx - m;
    }
    if (spany > 0) {
      int32_t m = oy % (2 * spany);
      if (m < 0) m += 2 * spany;
      oy = m < spany ? m : 2 * spany - m;
    }
    f.ox[k] = ox;
    f.oy[k] = oy;
  }
}

// Sample of plane c (0=Y,1=U,2=V) at component coordinates (x, y).
TV_HD int synth_sample_ctx(const SynthFrameCtx& f, int c, int x, int y) {
  const int s = c ? 1 : 0;
  const int xl = x << s, yl = y << s;  // luma-grid position
  // background pan: (2.25, 0.75) px/frame, textured (5.5, 2.25)
  const uint32_t seed = f.seed;
  const bool tex = synth_textured(seed);
  const int32_t bx16 = xl * 16 + f.t * (tex ? 88 : 36), by16 = yl * 16 + f.t * (tex ? 36 : 12);
  int v;
  if (c == 0) {
    if (tex)
      v = (synth_vnoise(bx16, by16, 7, seed) * 3 + synth_vnoise(bx16, by16, 5, seed + 1) * 2 +
           synth_vnoise(bx16, by16, 3, seed + 2) * 2 + synth_vnoise(bx16, by16, 1, seed + 3)) >> 3;
    else
      v = (synth_vnoise(bx16, by16, 7, seed) * 5 + synth_vnoise(bx16, by16, 5, seed + 1) * 2 +
           synth_vnoise(bx16, by16, 3, seed + 2)) >> 3;
  } else {
    v = 96 + (synth_vnoise(bx16, by16, 8, seed + 10 * c) >> 1);
  }
  for (int k = 0; k < kSynthObjects; ++k) {  // later objects on top
    const SynthObject& o = f.obj[k];
    const int32_t rx16 = xl * 16 - f.ox[k], ry16 = yl * 16 - f.oy[k];
    if (rx16 < 0 || ry16 < 0 || rx16 >= o.w * 16 || ry16 >= o.h * 16) continue;
    if (o.shape == 1) {
      const int64_t dx = 2 * (int64_t)rx16 - o.w * 16, dy = 2 * (int64_t)ry16 - o.h * 16;
      const int64_t ww = (int64_t)o.w * 16, hh = (int64_t)o.h * 16;
      if (dx * dx * hh * hh + dy * dy * ww * ww > ww * ww * hh * hh) continue;
    }
    if (c == 0) {
      v = 40 + ((synth_vnoise(rx16, ry16, 4, o.seed) * 3 + synth_vnoise(rx16, ry16, 2, o.seed + 5)) >> 2) * 3 / 4;
    } else {
      v = 64 + (int)(synth_hash(k, c, seed) & 127) + (synth_vnoise(rx16, ry16, 5, o.seed + c) >> 3);
    }
  }
  if (tex) {  // sensor-like grain, independent every frame
    const uint32_t g = synth_hash(x + f.t * 7919, y + c * 104729, seed ^ 0x5bd1e995u);
    v += c ? (int)(g & 3) - 2 : (int)(g & 7) - 4;
  }
  return clip_pixel(v);
}

TV_HD int synth_sample(uint32_t seed, int t, int c, int x, int y, int W, int H) {
  SynthFrameCtx f;
  synth_frame_ctx(seed, t, W, H, f);
  return synth_sample_ctx(f, c, x, y);
}

}  // namespace tv
