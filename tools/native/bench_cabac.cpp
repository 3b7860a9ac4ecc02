// Micro-benchmark of the CABAC slice writer on CPU-encoder decisions (1080p synthetic).
//   g++ -O2 -std=c++17 -Icsrc/include tools/native/bench_cabac.cpp -Lthinvids_amd/_lib -ltvcore -o /tmp/bench_cabac
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
    synth_frame_ctx(1, t, W, H, ctx);
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
    const int reps = argc > 2 ? atoi(argv[2]) : 20;
    size_t bytes = 0;
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < reps; ++r) {
      out.clear();
      bytes = write_slice(cfg, f, t, t == 0, out);
    }
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / reps;
    printf("frame %d (%s): %zu bytes, %.3f ms / slice, %.1f MB/s\n", t, t ? "P" : "I", bytes, ms, bytes / ms / 1e3);
  }
  return 0;
}
