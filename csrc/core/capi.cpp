// capi.cpp — extern "C" surface of libtvcore.so (loaded from Python with ctypes).
#include <cstring>
#include <exception>
#include <memory>
#include <string>
#include <vector>

#include "tv/container.h"
#include "tv/cpu_encoder.h"
#include "tv/hevc_codec.h"
#include "tv/synth.h"

using namespace tv;

namespace {
thread_local std::string g_err;
template <class F> int guard(F&& f) {
  try {
    f();
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}
struct Bytes {
  std::vector<uint8_t> v;
};
}  // namespace

extern "C" {

const char* tv_last_error() { return g_err.c_str(); }
int tv_core_version() { return 1; }

// ------------------------------------ byte buffers --------------------------------------
void* tv_bytes_new() { return new Bytes(); }
void tv_bytes_free(void* b) { delete static_cast<Bytes*>(b); }
size_t tv_bytes_size(void* b) { return static_cast<Bytes*>(b)->v.size(); }
const uint8_t* tv_bytes_data(void* b) { return static_cast<Bytes*>(b)->v.data(); }
void tv_bytes_clear(void* b) { static_cast<Bytes*>(b)->v.clear(); }

// ------------------------------------ synthetic source ----------------------------------
void tv_synth_frame(uint32_t seed, int t, int W, int H, uint8_t* y, uint8_t* u, uint8_t* v) {
  SynthFrameCtx ctx;
  synth_frame_ctx(seed, t, W, H, ctx);
  for (int c = 0; c < 3; ++c) {
    uint8_t* P = c == 0 ? y : (c == 1 ? u : v);
    const int w = c ? W / 2 : W, h = c ? H / 2 : H;
    for (int j = 0; j < h; ++j)
      for (int i = 0; i < w; ++i) P[(size_t)j * w + i] = (uint8_t)synth_sample_ctx(ctx, c, i, j);
  }
}

// ------------------------------------ CPU encoder ---------------------------------------
void* tv_cpu_encoder_new(int width, int height, int qp, int deblock, int range, int max_merge) {
  SeqConfig cfg;
  cfg.width = width;
  cfg.height = height;
  cfg.qp = qp;
  cfg.set_flags(deblock);  // 1 deblocking, 2 SAO, 4 WPP, 8 no RQT, 16 no intra-in-P
  cfg.max_merge_cand = max_merge;
  cfg.finalize();
  CpuEncoder* e = nullptr;  // a bad config becomes tv_last_error, not an abort across the FFI
  guard([&] { e = new CpuEncoder(cfg, range); });
  return e;
}
// hierarchical-B golden encoder (mgop > 1): frames go in the plan's coding order
void* tv_cpu_encoder_new_b(int width, int height, int qp, int deblock, int range, int max_merge, int mgop) {
  SeqConfig cfg;
  cfg.width = width;
  cfg.height = height;
  cfg.qp = qp;
  cfg.set_flags(deblock);
  cfg.max_merge_cand = max_merge;
  cfg.mgop = mgop;
  cfg.finalize();
  CpuEncoder* e = nullptr;
  guard([&] { e = new CpuEncoder(cfg, range); });
  return e;
}
// plan the next segment; disp (capacity nframes) receives the coding order's display indices
int tv_cpu_encoder_begin_gop(void* e, int nframes, int* disp) {
  return guard([&] {
    auto* enc = static_cast<CpuEncoder*>(e);
    enc->begin_gop(nframes);
    for (size_t k = 0; k < enc->plan().pics.size(); ++k) disp[k] = enc->plan().pics[k].disp;
  });
}
// GOP plan of nframes with mini-GOP mgop: per coded picture (coding order) display index,
// slice type, list-0 / list-1 reference, temporal layer; info = {dpb_size, num_reorder}
int tv_gop_plan(int nframes, int mgop, int* disp, int* type, int* ref0, int* ref1, int* layer, int* info) {
  const GopPlan g = plan_gop(nframes, mgop);
  for (size_t k = 0; k < g.pics.size(); ++k) {
    disp[k] = g.pics[k].disp;
    type[k] = g.pics[k].type;
    ref0[k] = g.pics[k].ref[0];
    ref1[k] = g.pics[k].ref[1];
    layer[k] = g.pics[k].layer;
  }
  info[0] = g.dpb_size;
  info[1] = g.num_reorder;
  return (int)g.pics.size();
}
void* tv_cpu_encoder_new_crf(int width, int height, int qp, int deblock, int range, int max_merge, int crf) {
  SeqConfig cfg;
  cfg.width = width;
  cfg.height = height;
  cfg.qp = qp;
  cfg.set_flags(deblock);
  cfg.max_merge_cand = max_merge;
  cfg.crf = crf;
  cfg.finalize();
  CpuEncoder* e = nullptr;  // a bad config becomes tv_last_error, not an abort across the FFI
  guard([&] { e = new CpuEncoder(cfg, range); });
  return e;
}
void tv_cpu_encoder_free(void* e) { delete static_cast<CpuEncoder*>(e); }
int tv_cpu_encoder_encode(void* e, const uint8_t* y, const uint8_t* u, const uint8_t* v, int sy,
                          int sc, int idr, int poc, void* out) {
  return guard([&] {
    const uint8_t* planes[3] = {y, u, v};
    const int strides[3] = {sy, sc, sc};
    static_cast<CpuEncoder*>(e)->encode_frame(planes, strides, idr != 0, poc, static_cast<Bytes*>(out)->v);
  });
}
// same with an explicit slice QP for this frame (rate control)
int tv_cpu_encoder_encode_qp(void* e, const uint8_t* y, const uint8_t* u, const uint8_t* v, int sy, int sc, int idr,
                             int poc, int qp, void* out) {
  return guard([&] {
    const uint8_t* planes[3] = {y, u, v};
    const int strides[3] = {sy, sc, sc};
    static_cast<CpuEncoder*>(e)->encode_frame(planes, strides, idr != 0, poc, static_cast<Bytes*>(out)->v, qp);
  });
}
// copy the coded-size reconstruction
void tv_cpu_encoder_recon(void* e, uint8_t* y, uint8_t* u, uint8_t* v) {
  const Picture& p = static_cast<CpuEncoder*>(e)->recon();
  std::memcpy(y, p.y.data(), p.y.size());
  std::memcpy(u, p.u.data(), p.u.size());
  std::memcpy(v, p.v.data(), p.v.size());
}
void tv_cpu_encoder_decisions(void* e, uint8_t* cu_log2, uint8_t* intra, uint8_t* ipm, int16_t* mv,
                              uint8_t* cbf) {
  const FrameDecisions& d = static_cast<CpuEncoder*>(e)->dec;
  std::memcpy(cu_log2, d.cu_log2.data(), d.cu_log2.size());
  std::memcpy(intra, d.intra.data(), d.intra.size());
  std::memcpy(ipm, d.ipm.data(), d.ipm.size());
  std::memcpy(mv, d.mv.data(), d.mv.size() * 2);
  std::memcpy(cbf, d.cbf.data(), d.cbf.size());
}

// ---------------------------- decisions -> reconstruction / bitstream ---------------------
// Reconstruct a frame from externally supplied decisions (golden model for the GPU).
// src/ref/rec planes are coded size. coef planes are outputs.  ref may be null for intra.
int tv_reconstruct_frame(int width, int height, int qp, int deblock, const uint8_t* src_y,
                         const uint8_t* src_u, const uint8_t* src_v, const uint8_t* ref_y,
                         const uint8_t* ref_u, const uint8_t* ref_v, const uint8_t* cu_log2,
                         const uint8_t* intra, const uint8_t* ipm, const int16_t* mv,
                         uint8_t* cbf_out, int16_t* cy, int16_t* cu, int16_t* cv, uint8_t* rec_y,
                         uint8_t* rec_u, uint8_t* rec_v) {
  return guard([&] {
    SeqConfig cfg;
    cfg.width = width;
    cfg.height = height;
    cfg.qp = qp;
    cfg.deblock = deblock != 0;
    cfg.rqt = false;  // no transform splits (tv_write_frame codes every split flag as 0)
    cfg.finalize();
    const int W = cfg.coded_w, H = cfg.coded_h;
    Picture src, ref, rec;
    src.alloc(W, H);
    rec.alloc(W, H);
    std::memcpy(src.y.data(), src_y, src.y.size());
    std::memcpy(src.u.data(), src_u, src.u.size());
    std::memcpy(src.v.data(), src_v, src.v.size());
    if (ref_y) {
      ref.alloc(W, H);
      std::memcpy(ref.y.data(), ref_y, ref.y.size());
      std::memcpy(ref.u.data(), ref_u, ref.u.size());
      std::memcpy(ref.v.data(), ref_v, ref.v.size());
    }
    FrameDecisions fd;
    fd.alloc(W, H);
    std::memcpy(fd.cu_log2.data(), cu_log2, fd.cu_log2.size());
    std::memcpy(fd.intra.data(), intra, fd.intra.size());
    std::memcpy(fd.ipm.data(), ipm, fd.ipm.size());
    std::memcpy(fd.mv.data(), mv, fd.mv.size() * 2);
    reconstruct_frame(cfg, src, ref_y ? &ref : nullptr, fd, rec);
    std::memcpy(cbf_out, fd.cbf.data(), fd.cbf.size());
    std::memcpy(cy, fd.coef_y.data(), fd.coef_y.size() * 2);
    std::memcpy(cu, fd.coef_u.data(), fd.coef_u.size() * 2);
    std::memcpy(cv, fd.coef_v.data(), fd.coef_v.size() * 2);
    std::memcpy(rec_y, rec.y.data(), rec.y.size());
    std::memcpy(rec_u, rec.u.data(), rec.u.size());
    std::memcpy(rec_v, rec.v.data(), rec.v.size());
  });
}

// Write parameter sets (if idr) + a slice NAL from decision arrays.
int tv_write_frame(int width, int height, int qp, int deblock, int max_merge, int idr, int poc,
                   const uint8_t* cu_log2, const uint8_t* intra, const uint8_t* ipm,
                   const int16_t* mv, const uint8_t* cbf, const int16_t* cy, const int16_t* cu,
                   const int16_t* cv, void* out) {
  return guard([&] {
    SeqConfig cfg;
    cfg.width = width;
    cfg.height = height;
    cfg.qp = qp;
    cfg.deblock = deblock != 0;
    cfg.max_merge_cand = max_merge;
    cfg.finalize();  // no tu plane: inter CUs code split_transform_flag 0
    FrameData f;
    f.w8 = cfg.w8();
    f.h8 = cfg.h8();
    f.cu_log2 = cu_log2;
    f.intra = intra;
    f.ipm = ipm;
    f.mv = mv;
    f.cbf = cbf;
    f.coef[0] = cy;
    f.coef[1] = cu;
    f.coef[2] = cv;
    auto& o = static_cast<Bytes*>(out)->v;
    if (idr) write_parameter_sets(cfg, o);
    write_slice(cfg, f, poc, idr != 0, o);
  });
}

// ------------------------------------ decoder -------------------------------------------
void* tv_decoder_new() { return new HevcDecoder(); }
void tv_decoder_free(void* d) { delete static_cast<HevcDecoder*>(d); }
int tv_decoder_decode(void* d, const uint8_t* data, size_t n) {
  return guard([&] { static_cast<HevcDecoder*>(d)->decode(data, n); });
}
int tv_decoder_decode_range(void* d, const uint8_t* data, size_t n, int first, int count) {
  return guard([&] { static_cast<HevcDecoder*>(d)->decode_range(data, n, first, count); });
}
// header-only probe: geometry + picture count, no slice decoding
// spatial MV scaling of the B-slice AMVP (8.5.3.2.7), exported for the formula test
void tv_hevc_scale_mv(int mvx, int mvy, int td, int tb, int* out) {
  const Mv m = scale_mv(Mv{mvx, mvy}, td, tb);
  out[0] = m.x;
  out[1] = m.y;
}
// display index - decoding index of every picture (hierarchical-B reordering); returns the
// picture count (out receives at most cap values)
int tv_hevc_display_offsets(const uint8_t* data, size_t n, int* out, int cap) {
  int r = -1;
  guard([&] {
    const std::vector<int> off = display_offsets(data, n);
    for (int i = 0; i < (int)off.size() && i < cap; ++i) out[i] = off[i];
    r = (int)off.size();
  });
  return r;
}
int tv_hevc_probe(const uint8_t* data, size_t n, int* w, int* h, int* pictures, int* idrs) {
  return guard([&] {
    const StreamInfo s = probe_annexb(data, n);
    *w = s.width;
    *h = s.height;
    *pictures = s.pictures;
    *idrs = s.idrs;
  });
}
void tv_decoder_info(void* d, int* w, int* h, int* cw, int* ch, int* nframes) {
  auto* D = static_cast<HevcDecoder*>(d);
  *w = D->width;
  *h = D->height;
  *cw = D->coded_w;
  *ch = D->coded_h;
  *nframes = (int)D->pictures.size();
}
// copy frame idx; cropped=1 -> display size, else coded size
int tv_decoder_frame(void* d, int idx, int cropped, uint8_t* y, uint8_t* u, uint8_t* v) {
  return guard([&] {
    auto* D = static_cast<HevcDecoder*>(d);
    const Picture& p = D->pictures.at(idx).pic;
    const int w = cropped ? D->width : p.w, h = cropped ? D->height : p.h;
    for (int c = 0; c < 3; ++c) {
      uint8_t* dst = c == 0 ? y : (c == 1 ? u : v);
      const int cw = c ? w / 2 : w, chh = c ? h / 2 : h, sw = p.pw(c);
      for (int j = 0; j < chh; ++j) std::memcpy(dst + (size_t)j * cw, p.plane(c) + (size_t)j * sw, cw);
    }
  });
}

// ------------------------------------ containers ----------------------------------------
int tv_mux_mp4(const uint8_t* annexb, size_t n, int w, int h, int fps_num, int fps_den, void* out) {
  return guard([&] { static_cast<Bytes*>(out)->v = mux_mp4(annexb, n, w, h, fps_num, fps_den); });
}
int tv_mux_mp4_file(const uint8_t* const* segs, const size_t* sizes, int nseg, int w, int h, int fps_num, int fps_den,
                    const char* path, unsigned long long* out_size) {
  return guard([&] { *out_size = mux_mp4_file(segs, sizes, nseg, w, h, fps_num, fps_den, path); });
}
int tv_mux_file(const uint8_t* const* segs, const size_t* sizes, int nseg, int w, int h, int fps_num, int fps_den,
                const SideTrack* tracks, int ntracks, int container, const char* path, unsigned long long* out_size) {
  return guard([&] {
    *out_size = mux_file(segs, sizes, nseg, w, h, fps_num, fps_den, tracks, ntracks, container, path);
  });
}
size_t tv_side_track_size() { return sizeof(SideTrack); }
int tv_demux_mp4(const uint8_t* mp4, size_t n, int* w, int* h, int* nframes, int* timescale,
                 int* delta, void* out) {
  return guard([&] { static_cast<Bytes*>(out)->v = demux_mp4(mp4, n, w, h, nframes, timescale, delta); });
}

}  // extern "C"
