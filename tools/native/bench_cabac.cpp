// Micro-benchmark of the CABAC slice writer on CPU-encoder decisions (1080p synthetic).
//   g++ -O2 -std=c++17 -Icsrc/include tools/native/bench_cabac.cpp -Lthinvids_amd/_lib -ltvcore -o /tmp/bench_cabac
//   /tmp/bench_cabac [qp] [reps] [compact: 1 = the GPU engine's compact level layout] [textured: 1]
#include <chrono>
#include <cstdio>
#include <vector>

#include "tv/cpu_encoder.h"
#include "tv/hevc_codec.h"
#include "tv/synth.h"

using namespace tv;

int main(int argc, char** argv) {
  const int W = 1920, H = 1080, qp = argc > 1 ? atoi(argv[1]) : 27;
  SeqConfig cfg;
  cfg.width = W;
  cfg.height = H;
  cfg.qp = qp;
  cfg.finalize();
  CpuEncoder enc(cfg, 16);
  std::vector<uint8_t> planes[3] = {std::vector<uint8_t>(W * H), std::vector<uint8_t>(W * H / 4),
                                    std::vector<uint8_t>(W * H / 4)};
  std::vector<FrameDecisions> decs;
  std::vector<uint8_t> out;
  for (int t = 0; t < 3; ++t) {
    SynthFrameCtx ctx;
    synth_frame_ctx(argc > 4 && atoi(argv[4]) ? 1u | kSynthTextured : 1u, t, W, H, ctx);
    for (int c = 0; c < 3; ++c) {
      const int w = c ? W / 2 : W, h = c ? H / 2 : H;
      for (int j = 0; j < h; ++j)
        for (int i = 0; i < w; ++i) planes[c][(size_t)j * w + i] = (uint8_t)synth_sample_ctx(ctx, c, i, j);
    }
    const uint8_t* p[3] = {planes[0].data(), planes[1].data(), planes[2].data()};
    const int s[3] = {W, W / 2, W / 2};
    out.clear();
    enc.encode_frame(p, s, t == 0, t, out);
    decs.push_back(enc.dec);
  }
  for (int t = 0; t < 3; ++t) {
    const FrameDecisions& d = decs[t];
    FrameData f;
    f.w8 = d.w8;
    f.h8 = d.h8;
    f.cu_log2 = d.cu_log2.data();
    f.intra = d.intra.data();
    f.ipm = d.ipm.data();
    f.mv = d.mv.data();
    f.cbf = d.cbf.data();
    f.coef[0] = d.coef_y.data();
    f.coef[1] = d.coef_u.data();
    f.coef[2] = d.coef_v.data();
    // the GPU engine's compact level layout (k_compact.hip): per CTB the non-zero 4x4 groups
    // (luma bit sy*8+sx, Cb bits 0..15, Cr 16..31), group offsets, 16 levels per group
    const int wc = cfg.coded_w / 32, hc = cfg.coded_h / 32, Wc = cfg.coded_w / 2;
    std::vector<uint64_t> my(wc * hc, 0);
    std::vector<uint32_t> mc(wc * hc, 0);
    std::vector<int32_t> off(wc * hc, 0);
    std::vector<int16_t> packed;
    for (int ctb = 0; ctb < wc * hc; ++ctb) {
      const int cx = ctb % wc, cy = ctb / wc;
      off[ctb] = (int32_t)(packed.size() / 16);
      auto group = [&](const int16_t* plane, int stride, int x, int y, bool& any) {
        int16_t g16[16];
        any = false;
        for (int j = 0; j < 4; ++j)
          for (int i = 0; i < 4; ++i) {
            g16[j * 4 + i] = plane[(size_t)(y + j) * stride + x + i];
            any = any || g16[j * 4 + i];
          }
        if (any) packed.insert(packed.end(), g16, g16 + 16);
      };
      for (int bit = 0; bit < 64; ++bit) {
        bool any;
        group(d.coef_y.data(), cfg.coded_w, cx * 32 + (bit & 7) * 4, cy * 32 + (bit >> 3) * 4, any);
        if (any) my[ctb] |= 1ull << bit;
      }
      for (int c = 0; c < 2; ++c)
        for (int bit = 0; bit < 16; ++bit) {
          bool any;
          group((c ? d.coef_v : d.coef_u).data(), Wc, cx * 16 + (bit & 3) * 4, cy * 16 + (bit >> 2) * 4, any);
          if (any) mc[ctb] |= 1u << (bit + 16 * c);
        }
    }
    if (argc > 3 && atoi(argv[3])) {
      f.sb_mask_y = my.data();
      f.sb_mask_c = mc.data();
      f.sb_offset = off.data();
      f.sb_packed = packed.data();
      f.wc = wc;
    }
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    size_t bytes = 0;
    double ms = 1e30, sum = 0;  // best and mean of the repetitions (the host is shared: min is stable)
    for (int r = 0; r < reps; ++r) {
      out.clear();
      auto t0 = std::chrono::steady_clock::now();
      bytes = write_slice(cfg, f, t, t == 0, out);
      const double d = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      ms = d < ms ? d : ms;
      sum += d;
    }
    printf("frame %d (%s): %zu bytes, %.3f ms / slice (min), %.3f mean, %.1f MB/s\n", t, t ? "P" : "I", bytes, ms,
           sum / reps, bytes / ms / 1e3);
  }
  return 0;
}
