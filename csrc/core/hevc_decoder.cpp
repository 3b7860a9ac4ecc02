// hevc_decoder.cpp — decoder oracle for the HEVC syntax subset this engine emits
// (Main profile, CTB 32, min CB 8, TB = CB, 2Nx2N, I/P slices, 1 reference, deblocking).
//
// There is no ffmpeg/HM/libde265 in the image, so conformance of the
// encoder is checked by decoding every produced stream with this independent parser and
// requiring decoded == encoder reconstruction, bit for bit.  It is also the probe used by
// the stitch stage for the `dest_*` job fields (reference worker/tasks.py:2225-2274).
#include <climits>
#include <algorithm>
#include <cstring>
#include <stdexcept>

#include "tv/bitstream.h"
#include "tv/cabac.h"
#include "tv/hevc_codec.h"

namespace tv {

namespace {

constexpr uint8_t kCtxIdxMap4x4[16] = {0, 1, 4, 5, 2, 3, 4, 5, 6, 6, 8, 8, 7, 7, 8, 8};
constexpr uint8_t kMinInGroup[10] = {0, 1, 2, 3, 4, 6, 8, 12, 16, 24};

struct Sps {
  int width = 0, height = 0, coded_w = 0, coded_h = 0;
  int conf[4] = {0, 0, 0, 0};
  int log2_poc_lsb = 8;
  int depth_inter = 0;  // max_transform_hierarchy_depth_inter (0 or 1)
  bool sao = false;
  bool valid = false;
};
struct Pps {
  int init_qp = 26;
  bool deblock = true;
  bool sign_hiding = false;
  bool wpp = false;
  bool valid = false;
};

void fail(const char* m) { throw std::runtime_error(std::string("hevc decoder: ") + m); }

void skip_ptl(BitReader& br) {
  br.u(2);
  br.u(1);
  br.u(5);
  br.u(32);
  br.u(4);
  br.u(32);
  br.u(11);
  br.u(1);
  br.u(8);
}

Sps parse_sps(BitReader& br) {
  Sps s;
  br.u(4);
  if (br.u(3) != 0) fail("sub-layers unsupported");
  br.u(1);
  skip_ptl(br);
  br.ue();
  if (br.ue() != 1) fail("chroma_format_idc != 1");
  s.coded_w = (int)br.ue();
  s.coded_h = (int)br.ue();
  if (br.u(1)) {
    for (int i = 0; i < 4; ++i) s.conf[i] = (int)br.ue();
  }
  s.width = s.coded_w - 2 * (s.conf[0] + s.conf[1]);
  s.height = s.coded_h - 2 * (s.conf[2] + s.conf[3]);
  if (br.ue() != 0 || br.ue() != 0) fail("bit depth != 8");
  s.log2_poc_lsb = (int)br.ue() + 4;
  const int ordering = (int)br.u(1);
  (void)ordering;
  br.ue();
  br.ue();
  br.ue();
  const int min_cb = (int)br.ue() + 3;
  const int ctb = min_cb + (int)br.ue();
  const int min_tb = (int)br.ue() + 2;
  const int max_tb = min_tb + (int)br.ue();
  const int dinter = (int)br.ue(), dintra = (int)br.ue();
  if (min_cb != kMinCbLog2 || ctb != kCtbLog2 || min_tb != kMinTbLog2 || max_tb != kMaxTbLog2 ||
      dinter > 1 || dintra != 0)
    fail("unsupported block-size configuration");
  s.depth_inter = dinter;
  if (br.u(1)) fail("scaling lists unsupported");
  if (br.u(1)) fail("AMP unsupported");
  s.sao = br.u(1) != 0;
  if (br.u(1)) fail("PCM unsupported");
  const int nrps = (int)br.ue();
  if (nrps != 1) fail("expected one st_ref_pic_set");
  if (br.ue() != 1 || br.ue() != 0 || br.ue() != 0 || br.u(1) != 1) fail("unsupported RPS");
  if (br.u(1)) fail("long-term refs unsupported");
  if (br.u(1)) fail("TMVP unsupported");
  if (br.u(1)) fail("strong intra smoothing unsupported");
  br.u(1);  // vui (we never write one)
  s.valid = true;
  return s;
}

Pps parse_pps(BitReader& br) {
  Pps p;
  br.ue();
  br.ue();
  if (br.u(1)) fail("dependent slices unsupported");
  if (br.u(1)) fail("output_flag_present unsupported");
  if (br.u(3)) fail("extra slice header bits unsupported");
  p.sign_hiding = br.u(1) != 0;
  if (p.sign_hiding) fail("sign data hiding unsupported");
  if (br.u(1)) fail("cabac_init_present unsupported");
  br.ue();
  br.ue();
  p.init_qp = 26 + br.se();
  if (br.u(1)) fail("constrained intra unsupported");
  if (br.u(1)) fail("transform skip unsupported");
  if (br.u(1)) fail("cu_qp_delta unsupported");
  if (br.se() != 0 || br.se() != 0) fail("chroma qp offsets unsupported");
  br.u(1);
  if (br.u(1) || br.u(1)) fail("weighted prediction unsupported");
  if (br.u(1)) fail("transquant bypass unsupported");
  if (br.u(1)) fail("tiles unsupported");
  p.wpp = br.u(1) != 0;
  br.u(1);
  if (br.u(1)) {
    if (br.u(1)) fail("deblocking override unsupported");
    p.deblock = br.u(1) == 0;
    if (p.deblock) {
      if (br.se() != 0 || br.se() != 0) fail("deblocking offsets unsupported");
    }
  }
  p.valid = true;
  return p;
}

class SliceDecoder {
 public:
  // ref[0] / ref[1]: RefPicList0[0] / RefPicList1[0] (B slices), ref_poc their POCs
  SliceDecoder(const Sps& sps, const Pps& pps, int stype, int qp, int max_merge, BitReader* br,
               Picture* cur, const Picture* const* ref, const int* ref_poc, int poc, FrameDecisions* fd, bool sao,
               std::vector<size_t> row_start = {})
      : sps_(sps), islice_(stype == 2), bslice_(stype == 0), qp_(qp), max_merge_(max_merge), dec_(br), br_(br),
        cur_(cur), ref_(ref[0]), ref1_(ref[1]), poc_(poc), fd_(fd), sao_(sao), row_start_(std::move(row_start)) {
    (void)pps;
    ref_poc_[0] = ref_poc[0];
    ref_poc_[1] = ref_poc[1];
    ctx_.init(islice_ ? 0 : (bslice_ ? 2 : 1), qp);
    skip_.assign((size_t)fd->w8 * fd->h8, 0);
    decoded_.assign((size_t)fd->w8 * fd->h8, 0);
    dec_.start();
  }

  // WPP (row_start_ = byte position of every CTB row's substream in the RBSP): each row
  // restarts the arithmetic decoder at its entry point with the contexts stored after the
  // second CTB of the row above (9.3.1 / 9.3.2.4)
  void run() {
    const int wc = sps_.coded_w >> kCtbLog2, hc = sps_.coded_h >> kCtbLog2;
    const bool wpp = !row_start_.empty();
    if (wpp && (int)row_start_.size() != hc) fail("entry points do not match the CTB rows");
    ContextSet synced{};
    for (int cy = 0; cy < hc; ++cy) {
      if (wpp && cy > 0) {
        br_->seek(row_start_[cy] * 8);
        dec_.start();
        ctx_ = synced;
      }
      for (int cx = 0; cx < wc; ++cx) {
        if (sao_) parse_sao(cx, cy);
        quadtree(cx << kCtbLog2, cy << kCtbLog2, kCtbLog2, 0);
        if (wpp && cx == 1) synced = ctx_;
        const int end = dec_.decode_terminate();
        const bool last = (cy == hc - 1) && (cx == wc - 1);
        if (end != (last ? 1 : 0)) fail("end_of_slice_segment_flag mismatch");
        if (wpp && !last && cx == wc - 1 && dec_.decode_terminate() != 1) fail("end_of_subset_one_bit missing");
      }
    }
  }

 private:
  int unit(int x, int y) const { return (y >> 3) * fd_->w8 + (x >> 3); }
  bool avail(int xc, int yc, int xn, int yn) const {
    return zscan_available(xc, yc, xn, yn, sps_.coded_w, sps_.coded_h);
  }
  int bin(int ctx) { return dec_.decode_bin(ctx_.c[ctx]); }

  void parse_sao(int cx, int cy) {
    const int wc = sps_.coded_w >> kCtbLog2;
    uint32_t* p = fd_->sao.data() + 3 * (size_t)(cy * wc + cx);
    if (cx > 0 && bin(CTX_SAO_MERGE)) {
      for (int c = 0; c < 3; ++c) p[c] = p[c - 3];
      return;
    }
    if (cy > 0 && bin(CTX_SAO_MERGE)) {
      for (int c = 0; c < 3; ++c) p[c] = p[c - 3 * wc];
      return;
    }
    int type = 0, eo = 0;
    for (int c = 0; c < 3; ++c) {
      if (c < 2) {
        type = bin(CTX_SAO_TYPE) ? (dec_.decode_bypass() ? 2 : 1) : 0;
      }
      int off[4] = {0, 0, 0, 0}, cls = 0;
      if (type) {
        for (int i = 0; i < 4; ++i) {
          int a = 0;
          while (a < kSaoMaxOff && dec_.decode_bypass()) ++a;
          off[i] = a;
        }
        if (type == 1) {
          for (int i = 0; i < 4; ++i)
            if (off[i] && dec_.decode_bypass()) off[i] = -off[i];
          cls = (int)dec_.decode_bypass_bins(5);
        } else {
          if (c < 2) eo = (int)dec_.decode_bypass_bins(2);
          cls = eo;
          off[2] = -off[2];
          off[3] = -off[3];
        }
      }
      p[c] = sao_pack(type, cls, off);
    }
  }

  void quadtree(int x0, int y0, int log2, int depth) {
    bool split = false;
    if (log2 > kMinCbLog2) {
      int inc = 0;
      if (avail(x0, y0, x0 - 1, y0) && (kCtbLog2 - fd_->cu_log2[unit(x0 - 1, y0)]) > depth) ++inc;
      if (avail(x0, y0, x0, y0 - 1) && (kCtbLog2 - fd_->cu_log2[unit(x0, y0 - 1)]) > depth) ++inc;
      split = bin(CTX_SPLIT_CU + inc);
    }
    if (split) {
      const int h = 1 << (log2 - 1);
      quadtree(x0, y0, log2 - 1, depth + 1);
      quadtree(x0 + h, y0, log2 - 1, depth + 1);
      quadtree(x0, y0 + h, log2 - 1, depth + 1);
      quadtree(x0 + h, y0 + h, log2 - 1, depth + 1);
    } else {
      coding_unit(x0, y0, log2);
    }
  }

  void fill(int x0, int y0, int log2, int intra, int ipm, Mv mv, int cbf, int skip) {
    const int n = 1 << (log2 - 3);
    for (int j = 0; j < n; ++j)
      for (int i = 0; i < n; ++i) {
        const int u = unit(x0 + 8 * i, y0 + 8 * j);
        fd_->cu_log2[u] = (uint8_t)log2;
        fd_->intra[u] = (uint8_t)intra;
        fd_->ipm[u] = (uint8_t)ipm;
        fd_->mv[2 * u] = (int16_t)mv.x;
        fd_->mv[2 * u + 1] = (int16_t)mv.y;
        fd_->cbf[u] = (uint8_t)cbf;
        fd_->tu[u] = 0;
        skip_[u] = (uint8_t)skip;
        decoded_[u] = 1;
      }
  }

  bool inter_at(int xc, int yc, int xn, int yn, Mv& mv) const {
    if (!avail(xc, yc, xn, yn)) return false;
    const int u = unit(xn, yn);
    if (!decoded_[u] || fd_->intra[u]) return false;
    mv.x = fd_->mv[2 * u];
    mv.y = fd_->mv[2 * u + 1];
    return true;
  }
  bool motion_at(int xc, int yc, int xn, int yn, Motion& m) const {
    if (!avail(xc, yc, xn, yn)) return false;
    const int u = unit(xn, yn);
    if (!decoded_[u] || fd_->intra[u]) return false;
    m.dir = fd_->dir[u];
    m.mv[0] = Mv{fd_->mv[2 * u], fd_->mv[2 * u + 1]};
    m.mv[1] = Mv{fd_->mv1[2 * u], fd_->mv1[2 * u + 1]};
    return true;
  }
  void fill_motion(int x0, int y0, int log2, const Motion& m) {
    const int n = 1 << (log2 - 3);
    for (int j = 0; j < n; ++j)
      for (int i = 0; i < n; ++i) {
        const int u = unit(x0 + 8 * i, y0 + 8 * j);
        fd_->dir[u] = (uint8_t)m.dir;
        fd_->mv1[2 * u] = (int16_t)m.mv[1].x;
        fd_->mv1[2 * u + 1] = (int16_t)m.mv[1].y;
      }
  }

  // B-slice inter CU: skip / merge / AMVP per list (7.3.8.5-7.3.8.6)
  void coding_unit_b(int x0, int y0, int log2, bool skip) {
    const int N = 1 << log2;
    auto at = [&](int xn, int yn, Motion& o) { return motion_at(x0, y0, xn, yn, o); };
    Motion m;
    bool has_res = !skip;
    bool merge = skip;
    if (!skip) {
      if (bin(CTX_PRED_MODE)) fail("intra CU in a B slice unsupported");
      if (!bin(CTX_PART_MODE)) fail("only 2Nx2N inter partitions supported");
      merge = bin(CTX_MERGE_FLAG) != 0;
    }
    if (merge) {
      const int mi = parse_merge_idx();
      Motion cand[5];
      merge_candidates_b(x0, y0, N, N, max_merge_, ref_poc_[0] == ref_poc_[1], at, cand);
      m = cand[mi];
    } else {
      m.dir = bin(CTX_INTER_PRED_IDC + (kCtbLog2 - log2)) ? 3 : (bin(CTX_INTER_PRED_IDC + 4) ? 2 : 1);
      for (int X = 0; X < 2; ++X) {
        if (!((m.dir >> X) & 1)) continue;
        const Mv d = parse_mvd();
        const int sel = bin(CTX_MVP_FLAG);
        Mv mvp[2];
        amvp_candidates_b(x0, y0, N, N, X, ref_poc_, poc_, at, mvp);
        m.mv[X].x = (int16_t)(mvp[sel].x + d.x);
        m.mv[X].y = (int16_t)(mvp[sel].y + d.y);
      }
      has_res = bin(CTX_RQT_ROOT_CBF) != 0;
    }
    if (!(m.dir & 1)) m.mv[0] = Mv{};
    if (!(m.dir & 2)) m.mv[1] = Mv{};
    fill(x0, y0, log2, 0, 1, m.mv[0], 0, skip ? 1 : 0);
    fill_motion(x0, y0, log2, m);
    int cbf = 0;
    if (has_res) cbf = transform_tree(x0, y0, log2, false, 0);
    fill(x0, y0, log2, 0, 1, m.mv[0], cbf & 7, skip ? 1 : 0);
    set_split_cbf(x0, y0, log2, cbf);
    if (cbf >> 12) {
      const int h = 1 << (log2 - 1);
      for (int q = 0; q < 4; ++q) recon_motion(x0 + (q & 1) * h, y0 + (q >> 1) * h, log2 - 1, m, (cbf >> (3 * q)) & 7);
    } else {
      recon_motion(x0, y0, log2, m, cbf);
    }
  }
  // an RQT-split CU (transform_tree result bit 12): per-unit cbf of its 16x16 TB, tu = 1
  void set_split_cbf(int x0, int y0, int log2, int res) {
    if (!(res >> 12)) return;
    const int n = 1 << (log2 - 3), hb = n >> 1;  // units per side, per quadrant side
    for (int j = 0; j < n; ++j)
      for (int i = 0; i < n; ++i) {
        const int u = unit(x0 + 8 * i, y0 + 8 * j), q = (j / hb) * 2 + i / hb;
        fd_->cbf[u] = (uint8_t)((res >> (3 * q)) & 7);
        fd_->tu[u] = 1;
      }
  }
  void recon_motion(int x0, int y0, int log2, const Motion& m, int cbf) {
    if (m.dir == 1) return recon_inter(x0, y0, log2, m.mv[0], cbf, ref_);
    if (m.dir == 2) return recon_inter(x0, y0, log2, m.mv[1], cbf, ref1_);
    if (!ref_ || !ref1_) fail("bi-prediction without two references");
    const int N = 1 << log2, W = sps_.coded_w, Wc = W >> 1;
    int pred[32 * 32];
    const int16_t v0[2] = {(int16_t)m.mv[0].x, (int16_t)m.mv[0].y}, v1[2] = {(int16_t)m.mv[1].x, (int16_t)m.mv[1].y};
    predict_bi_block(*ref_, *ref1_, 0, x0, y0, N, N, v0, v1, pred);
    recon_tb(fd_->coef_y.data() + (size_t)y0 * W + x0, W, cbf & 1, log2, qp_, pred, cur_->y.data() + (size_t)y0 * W + x0, W);
    const int qpc = chroma_qp(qp_, 0);
    for (int c = 1; c <= 2; ++c) {
      predict_bi_block(*ref_, *ref1_, c, x0 >> 1, y0 >> 1, N >> 1, N >> 1, v0, v1, pred);
      const int16_t* L = (c == 1 ? fd_->coef_u : fd_->coef_v).data() + (size_t)(y0 >> 1) * Wc + (x0 >> 1);
      recon_tb(L, Wc, (cbf >> c) & 1, log2 - 1, qpc, pred, cur_->plane(c) + (size_t)(y0 >> 1) * Wc + (x0 >> 1), Wc);
    }
  }

  int parse_merge_idx() {
    if (max_merge_ <= 1) return 0;
    int idx = 0;
    if (bin(CTX_MERGE_IDX)) {
      idx = 1;
      while (idx < max_merge_ - 1 && dec_.decode_bypass()) ++idx;
    }
    return idx;
  }

  int parse_eg1() {
    int k = 1;
    uint32_t v = 0;
    while (dec_.decode_bypass()) {
      v += 1u << k;
      ++k;
      if (k > 30) fail("bad EG1");
    }
    v += dec_.decode_bypass_bins(k);
    return (int)v;
  }

  Mv parse_mvd() {
    const int gx = bin(CTX_MVD_G0), gy = bin(CTX_MVD_G0);
    int g1x = 0, g1y = 0;
    if (gx) g1x = bin(CTX_MVD_G1);
    if (gy) g1y = bin(CTX_MVD_G1);
    Mv d;
    if (gx) {
      int a = 1;
      if (g1x) a = parse_eg1() + 2;
      d.x = dec_.decode_bypass() ? -a : a;
    }
    if (gy) {
      int a = 1;
      if (g1y) a = parse_eg1() + 2;
      d.y = dec_.decode_bypass() ? -a : a;
    }
    return d;
  }

  void coding_unit(int x0, int y0, int log2) {
    const int N = 1 << log2;
    if (!islice_) {
      int inc = 0;
      if (avail(x0, y0, x0 - 1, y0) && skip_[unit(x0 - 1, y0)]) ++inc;
      if (avail(x0, y0, x0, y0 - 1) && skip_[unit(x0, y0 - 1)]) ++inc;
      const int skip = bin(CTX_CU_SKIP + inc);
      if (bslice_) {
        coding_unit_b(x0, y0, log2, skip != 0);
        return;
      }
      auto f = [&](int xn, int yn, Mv& m) { return inter_at(x0, y0, xn, yn, m); };
      if (skip) {
        const int mi = parse_merge_idx();
        Mv cand[5];
        merge_candidates(x0, y0, N, N, max_merge_, f, cand);
        fill(x0, y0, log2, 0, 1, cand[mi], 0, 1);
        recon_inter(x0, y0, log2, cand[mi], 0, ref_);
        return;
      }
      const int intra = bin(CTX_PRED_MODE);
      if (!intra) {
        if (!bin(CTX_PART_MODE)) fail("only 2Nx2N inter partitions supported");
        Mv mv;
        bool has_res;
        if (bin(CTX_MERGE_FLAG)) {
          const int mi = parse_merge_idx();
          Mv cand[5];
          merge_candidates(x0, y0, N, N, max_merge_, f, cand);
          mv = cand[mi];
          has_res = true;  // rqt_root_cbf inferred 1
        } else {
          const Mv d = parse_mvd();
          const int sel = bin(CTX_MVP_FLAG);
          Mv mvp[2];
          amvp_candidates(x0, y0, N, N, f, mvp);
          mv.x = (int16_t)(mvp[sel].x + d.x);
          mv.y = (int16_t)(mvp[sel].y + d.y);
          has_res = bin(CTX_RQT_ROOT_CBF);
        }
        int cbf = 0;
        fill(x0, y0, log2, 0, 1, mv, 0, 0);
        if (has_res) cbf = transform_tree(x0, y0, log2, false, 0);
        fill(x0, y0, log2, 0, 1, mv, cbf & 7, 0);
        set_split_cbf(x0, y0, log2, cbf);
        if (cbf >> 12) {  // inter prediction is per sample: the quadrants predict like the CU
          const int h = 1 << (log2 - 1);
          for (int q = 0; q < 4; ++q)
            recon_inter(x0 + (q & 1) * h, y0 + (q >> 1) * h, log2 - 1, mv, (cbf >> (3 * q)) & 7, ref_);
        } else {
          recon_inter(x0, y0, log2, mv, cbf, ref_);
        }
        return;
      }
    }
    // intra
    if (log2 == kMinCbLog2 && !bin(CTX_PART_MODE)) fail("NxN intra partitions unsupported");
    const int pflag = bin(CTX_PREV_INTRA);
    int candA = 1, candB = 1;
    if (avail(x0, y0, x0 - 1, y0) && fd_->intra[unit(x0 - 1, y0)]) candA = fd_->ipm[unit(x0 - 1, y0)];
    if (avail(x0, y0, x0, y0 - 1) && fd_->intra[unit(x0, y0 - 1)] &&
        (y0 - 1) >= ((y0 >> kCtbLog2) << kCtbLog2))
      candB = fd_->ipm[unit(x0, y0 - 1)];
    int mpm[3];
    intra_mpm_list(candA, candB, mpm);
    int mode;
    if (pflag) {
      int idx = dec_.decode_bypass();
      if (idx) idx += dec_.decode_bypass();
      mode = mpm[idx];
    } else {
      mode = (int)dec_.decode_bypass_bins(5);
      int s[3] = {mpm[0], mpm[1], mpm[2]};
      std::sort(s, s + 3);
      for (int i = 0; i < 3; ++i)
        if (mode >= s[i]) ++mode;
    }
    int cidx = 4;
    if (bin(CTX_CHROMA_PRED)) cidx = (int)dec_.decode_bypass_bins(2);
    const int cmode = chroma_intra_mode(cidx, mode);
    fill(x0, y0, log2, 1, mode, Mv{}, 0, 0);
    const int cbf = transform_tree(x0, y0, log2, true, mode, cmode);
    fill(x0, y0, log2, 1, mode, Mv{}, cbf, 0);
    recon_intra(x0, y0, log2, mode, cmode, cbf);
  }

  // returns cbf bits; parses coefficients into fd_ planes.  An inter CU's transform tree may
  // split once (RQT, max_transform_hierarchy_depth_inter 1): then bit 12 is set and bits
  // 3q..3q+2 hold quadrant q's cbfs.
  int transform_tree(int x0, int y0, int log2, bool intra, int mode, int cmode = 0) {
    if (!intra && sps_.depth_inter > 0 && bin(CTX_SPLIT_TF + 5 - log2)) {
      if (log2 < 4) fail("transform split below 16x16 unsupported");
      const int h = 1 << (log2 - 1), l = log2 - 1;
      const int W = sps_.coded_w, Wc = W >> 1;
      clear_tb(fd_->coef_y.data() + (size_t)y0 * W + x0, W, log2);
      clear_tb(fd_->coef_u.data() + (size_t)(y0 >> 1) * Wc + (x0 >> 1), Wc, log2 - 1);
      clear_tb(fd_->coef_v.data() + (size_t)(y0 >> 1) * Wc + (x0 >> 1), Wc, log2 - 1);
      const int cb0 = bin(CTX_CBF_CHROMA + 0), cr0 = bin(CTX_CBF_CHROMA + 0);
      int res = 1 << 12;
      for (int q = 0; q < 4; ++q) {
        const int x = x0 + (q & 1) * h, y = y0 + (q >> 1) * h;
        const int cb = cb0 ? bin(CTX_CBF_CHROMA + 1) : 0, cr = cr0 ? bin(CTX_CBF_CHROMA + 1) : 0;
        const int cl = bin(CTX_CBF_LUMA + 0);
        if (cl) residual(fd_->coef_y.data() + (size_t)y * W + x, W, l, 0, 0);
        if (cb) residual(fd_->coef_u.data() + (size_t)(y >> 1) * Wc + (x >> 1), Wc, l - 1, 1, 0);
        if (cr) residual(fd_->coef_v.data() + (size_t)(y >> 1) * Wc + (x >> 1), Wc, l - 1, 2, 0);
        res |= (cl | (cb << 1) | (cr << 2)) << (3 * q);
      }
      return res;
    }
    const int cb = bin(CTX_CBF_CHROMA + 0);
    const int cr = bin(CTX_CBF_CHROMA + 0);
    int cl = 1;
    if (intra || cb || cr) cl = bin(CTX_CBF_LUMA + 1);
    const int W = sps_.coded_w, Wc = W >> 1;
    clear_tb(fd_->coef_y.data() + (size_t)y0 * W + x0, W, log2);
    clear_tb(fd_->coef_u.data() + (size_t)(y0 >> 1) * Wc + (x0 >> 1), Wc, log2 - 1);
    clear_tb(fd_->coef_v.data() + (size_t)(y0 >> 1) * Wc + (x0 >> 1), Wc, log2 - 1);
    if (cl)
      residual(fd_->coef_y.data() + (size_t)y0 * W + x0, W, log2, 0, scan_idx_for(intra, log2, 0, mode));
    if (cb)
      residual(fd_->coef_u.data() + (size_t)(y0 >> 1) * Wc + (x0 >> 1), Wc, log2 - 1, 1,
               scan_idx_for(intra, log2 - 1, 1, cmode));
    if (cr)
      residual(fd_->coef_v.data() + (size_t)(y0 >> 1) * Wc + (x0 >> 1), Wc, log2 - 1, 2,
               scan_idx_for(intra, log2 - 1, 2, cmode));
    return cl | (cb << 1) | (cr << 2);
  }
  static void clear_tb(int16_t* p, int s, int log2) {
    const int N = 1 << log2;
    for (int j = 0; j < N; ++j) std::memset(p + (size_t)j * s, 0, N * sizeof(int16_t));
  }

  int parse_last_prefix(int log2N, int cIdx, int base) {
    int off, shift;
    if (cIdx == 0) {
      off = 3 * (log2N - 2) + ((log2N - 1) >> 2);
      shift = (log2N + 1) >> 2;
    } else {
      off = 15;
      shift = log2N - 2;
    }
    const int cmax = (log2N << 1) - 1;
    int p = 0;
    while (p < cmax && bin(base + off + (p >> shift))) ++p;
    return p;
  }
  int last_from(int prefix) {
    if (prefix <= 3) return prefix;
    const int nb = (prefix >> 1) - 1;
    return kMinInGroup[prefix] + (int)dec_.decode_bypass_bins(nb);
  }
  int parse_remaining(int rice) {
    int p = 0;
    while (dec_.decode_bypass()) {
      if (++p > 32) fail("bad coeff_abs_level_remaining");
    }
    if (p < 4) return (p << rice) + (rice ? (int)dec_.decode_bypass_bins(rice) : 0);
    const int nb = p - 3 + rice;
    return (((1 << (p - 3)) + 2) << rice) + (int)dec_.decode_bypass_bins(nb);
  }

  void residual(int16_t* blk, int stride, int log2N, int cIdx, int scanIdx) {
    const int nsb = 1 << (log2N - 2);
    int px = parse_last_prefix(log2N, cIdx, CTX_LAST_X);
    int py = parse_last_prefix(log2N, cIdx, CTX_LAST_Y);
    int lx = last_from(px), ly = last_from(py);
    if (scanIdx == 2) std::swap(lx, ly);
    // locate last sub-block / position in scan order
    int lastSb = -1, lastN = -1;
    for (int i = 0; i < nsb * nsb && lastSb < 0; ++i) {
      int xs, ys;
      subblock_pos(log2N, scanIdx, i, xs, ys);
      if (xs != (lx >> 2) || ys != (ly >> 2)) continue;
      for (int n = 0; n < 16; ++n) {
        int xc, yc;
        coef_pos_in_sb(scanIdx, n, xc, yc);
        if (xc == (lx & 3) && yc == (ly & 3)) {
          lastSb = i;
          lastN = n;
        }
      }
    }
    if (lastSb < 0) fail("bad last position");
    uint8_t csbf[8][8];
    std::memset(csbf, 0, sizeof(csbf));
    int c1 = 1;
    for (int i = lastSb; i >= 0; --i) {
      int xs, ys;
      subblock_pos(log2N, scanIdx, i, xs, ys);
      bool inferDc = false;
      if (i < lastSb && i > 0) {
        int ctx = 0;
        if (xs < nsb - 1) ctx += csbf[xs + 1][ys];
        if (ys < nsb - 1) ctx += csbf[xs][ys + 1];
        ctx = ctx > 1 ? 1 : ctx;
        csbf[xs][ys] = (uint8_t)bin(CTX_CSBF + ctx + (cIdx ? 2 : 0));
        inferDc = true;
      } else {
        csbf[xs][ys] = 1;
      }
      if (!csbf[xs][ys]) continue;
      int prevCsbf = 0;
      if (xs < nsb - 1) prevCsbf += csbf[xs + 1][ys];
      if (ys < nsb - 1) prevCsbf += csbf[xs][ys + 1] << 1;
      int sig[16];
      std::memset(sig, 0, sizeof(sig));
      if (i == lastSb) sig[lastN] = 1;
      const int nStart = (i == lastSb) ? lastN - 1 : 15;
      for (int n = nStart; n >= 0; --n) {
        if (n == 0 && inferDc) {
          sig[0] = 1;
          break;
        }
        int xc, yc;
        coef_pos_in_sb(scanIdx, n, xc, yc);
        sig[n] = bin(CTX_SIG + sig_ctx(log2N, cIdx, scanIdx, xs, ys, xc, yc, prevCsbf));
        if (sig[n]) inferDc = false;
      }
      int pos[16], absv[16], cnt = 0;
      for (int n = 15; n >= 0; --n)
        if (sig[n]) {
          pos[cnt] = n;
          absv[cnt] = 1;
          ++cnt;
        }
      int ctxSet = (i > 0 && cIdx == 0) ? 2 : 0;
      if (c1 == 0) ++ctxSet;
      c1 = 1;
      const int g1base = CTX_G1 + 4 * ctxSet + (cIdx ? 16 : 0);
      const int nG1 = cnt < 8 ? cnt : 8;
      int firstG2 = -1;
      for (int k = 0; k < nG1; ++k) {
        const int g1 = bin(g1base + c1);
        if (g1) {
          absv[k] = 2;
          c1 = 0;
          if (firstG2 < 0) firstG2 = k;
        } else if (c1 > 0 && c1 < 3) {
          ++c1;
        }
      }
      if (firstG2 >= 0 && bin(CTX_G2 + ctxSet + (cIdx ? 4 : 0))) absv[firstG2] = 3;
      int signs[16];
      for (int k = 0; k < cnt; ++k) signs[k] = dec_.decode_bypass();
      int rice = 0;
      bool firstC2 = true;
      for (int k = 0; k < cnt; ++k) {
        const int base = (k < 8) ? (firstC2 ? 3 : 2) : 1;
        if (absv[k] >= base) {
          absv[k] = base + parse_remaining(rice);
          if (absv[k] > 3 * (1 << rice)) rice = tv_min(rice + 1, 4);
        }
        if (absv[k] >= 2) firstC2 = false;
      }
      for (int k = 0; k < cnt; ++k) {
        int xc, yc;
        coef_pos_in_sb(scanIdx, pos[k], xc, yc);
        const int v = signs[k] ? -absv[k] : absv[k];
        blk[(size_t)((ys << 2) + yc) * stride + (xs << 2) + xc] = (int16_t)v;
      }
    }
  }

  static int sig_ctx(int log2N, int cIdx, int scanIdx, int xs, int ys, int xp, int yp, int prevCsbf) {
    int sigCtx;
    if (log2N == 2) {
      sigCtx = kCtxIdxMap4x4[(yp << 2) + xp];
    } else if (xs == 0 && ys == 0 && xp == 0 && yp == 0) {
      sigCtx = 0;
    } else {
      if (prevCsbf == 0) sigCtx = (xp + yp == 0) ? 2 : (xp + yp < 3) ? 1 : 0;
      else if (prevCsbf == 1) sigCtx = (yp == 0) ? 2 : (yp == 1) ? 1 : 0;
      else if (prevCsbf == 2) sigCtx = (xp == 0) ? 2 : (xp == 1) ? 1 : 0;
      else sigCtx = 2;
      if (cIdx == 0 && (xs > 0 || ys > 0)) sigCtx += 3;
      if (log2N == 3) sigCtx += (scanIdx == 0) ? 9 : 15;
      else sigCtx += (cIdx == 0) ? 21 : 12;
    }
    return cIdx == 0 ? sigCtx : 27 + sigCtx;
  }

  void recon_inter(int x0, int y0, int log2, Mv mv, int cbf, const Picture* ref) {
    if (!ref) fail("inter prediction without a reference");
    const int N = 1 << log2, W = sps_.coded_w, Wc = W >> 1;
    int pred[32 * 32];
    predict_inter_block(*ref, 0, x0, y0, N, N, mv.x, mv.y, pred);
    recon_tb(fd_->coef_y.data() + (size_t)y0 * W + x0, W, cbf & 1, log2, qp_, pred,
             cur_->y.data() + (size_t)y0 * W + x0, W);
    const int qpc = chroma_qp(qp_, 0);
    for (int c = 1; c <= 2; ++c) {
      predict_inter_block(*ref, c, x0 >> 1, y0 >> 1, N >> 1, N >> 1, mv.x, mv.y, pred);
      const int16_t* L = (c == 1 ? fd_->coef_u : fd_->coef_v).data() + (size_t)(y0 >> 1) * Wc + (x0 >> 1);
      recon_tb(L, Wc, (cbf >> c) & 1, log2 - 1, qpc, pred, cur_->plane(c) + (size_t)(y0 >> 1) * Wc + (x0 >> 1), Wc);
    }
  }

  void recon_intra(int x0, int y0, int log2, int mode, int cmode, int cbf) {
    const int W = sps_.coded_w, Wc = W >> 1;
    int pred[32 * 32];
    predict_intra_tb(*cur_, 0, x0, y0, log2, mode, pred);
    recon_tb(fd_->coef_y.data() + (size_t)y0 * W + x0, W, cbf & 1, log2, qp_, pred,
             cur_->y.data() + (size_t)y0 * W + x0, W);
    const int qpc = chroma_qp(qp_, 0);
    for (int c = 1; c <= 2; ++c) {
      predict_intra_tb(*cur_, c, x0 >> 1, y0 >> 1, log2 - 1, cmode, pred);
      const int16_t* L = (c == 1 ? fd_->coef_u : fd_->coef_v).data() + (size_t)(y0 >> 1) * Wc + (x0 >> 1);
      recon_tb(L, Wc, (cbf >> c) & 1, log2 - 1, qpc, pred, cur_->plane(c) + (size_t)(y0 >> 1) * Wc + (x0 >> 1), Wc);
    }
  }

  const Sps& sps_;
  bool islice_, bslice_;
  int qp_, max_merge_;
  CabacDecoder dec_;
  BitReader* br_;
  ContextSet ctx_;
  Picture* cur_;
  const Picture *ref_, *ref1_;
  int poc_, ref_poc_[2];
  FrameDecisions* fd_;
  bool sao_;
  std::vector<size_t> row_start_;
  std::vector<uint8_t> skip_, decoded_;
};

}  // namespace

StreamInfo probe_annexb(const uint8_t* data, size_t n) {
  StreamInfo info;
  for (const auto& nal : split_annexb(data, n)) {
    if (nal.size < 3) continue;
    const int type = nal.type();
    if (type == NAL_SPS) {
      std::vector<uint8_t> rbsp = unescape_rbsp(nal.data + 2, nal.size - 2);
      BitReader br(rbsp.data(), rbsp.size());
      const Sps sps = parse_sps(br);
      info.width = sps.width;
      info.height = sps.height;
      info.coded_w = sps.coded_w;
      info.coded_h = sps.coded_h;
    } else if (type <= 21 && (nal.data[2] & 0x80)) {  // first_slice_segment_in_pic_flag
      ++info.pictures;
      if (type == NAL_IDR_W_RADL || type == NAL_IDR_N_LP) ++info.idrs;
    }
  }
  return info;
}

std::vector<int> display_offsets(const uint8_t* data, size_t n) {
  // slice headers only: POC per picture (IDR resets it), then each coded video sequence's
  // pictures ranked by POC
  std::vector<int> poc, cvs_of;
  int log2_lsb = 8, prev = 0, cvs = -1;
  for (const auto& nal : split_annexb(data, n)) {
    if (nal.size < 3) continue;
    const int t = nal.type();
    if (t == NAL_SPS) {
      std::vector<uint8_t> rbsp = unescape_rbsp(nal.data + 2, nal.size - 2);
      BitReader br(rbsp.data(), rbsp.size());
      log2_lsb = parse_sps(br).log2_poc_lsb;
      continue;
    }
    if (t > 21 || !(nal.data[2] & 0x80)) continue;
    const bool idr = t == NAL_IDR_W_RADL || t == NAL_IDR_N_LP;
    int p = 0;
    if (idr) {
      ++cvs;
    } else {
      std::vector<uint8_t> rbsp = unescape_rbsp(nal.data + 2, std::min<size_t>(nal.size - 2, 32));
      BitReader br(rbsp.data(), rbsp.size());
      br.u(1);                   // first_slice_segment_in_pic_flag
      if (t >= 16) br.u(1);      // no_output_of_prior_pics_flag (IRAP)
      br.ue();                   // slice_pic_parameter_set_id
      br.ue();                   // slice_type (no extra header bits / output flag in our PPS)
      const int lsb = (int)br.u(log2_lsb), max_lsb = 1 << log2_lsb;
      const int prev_lsb = prev & (max_lsb - 1);
      int msb = prev - prev_lsb;
      if (lsb < prev_lsb && prev_lsb - lsb >= max_lsb / 2) msb += max_lsb;
      else if (lsb > prev_lsb && lsb - prev_lsb > max_lsb / 2) msb -= max_lsb;
      p = msb + lsb;
      if (cvs < 0) cvs = 0;
    }
    prev = p;
    poc.push_back(p);
    cvs_of.push_back(cvs);
  }
  std::vector<int> off(poc.size(), 0);
  for (size_t a = 0; a < poc.size();) {
    size_t b = a;
    while (b < poc.size() && cvs_of[b] == cvs_of[a]) ++b;
    for (size_t i = a; i < b; ++i) {
      int rank = 0;
      for (size_t j = a; j < b; ++j) rank += poc[j] < poc[i] || (poc[j] == poc[i] && j < i);
      off[i] = (int)(a + rank) - (int)i;
    }
    a = b;
  }
  return off;
}

void HevcDecoder::decode(const uint8_t* data, size_t n) { decode_range(data, n, 0, -1); }

void HevcDecoder::decode_range(const uint8_t* data, size_t n, int first, int count) {
  Sps sps;
  Pps pps;
  const auto nals = split_annexb(data, n);
  // picture index of every slice NAL and the last IDR at or before `first`.  Pictures of one
  // coded video sequence (IDR to IDR) occupy the same index range in decoding and output
  // order (closed GOPs), so whole sequences are decoded and reordered by POC.
  int start_pic = 0;
  {
    int k = 0;
    for (const auto& nal : nals) {
      if (nal.size < 3) continue;
      const int t = nal.type();
      if (t > 21 || !(nal.data[2] & 0x80)) continue;
      if ((t == NAL_IDR_W_RADL || t == NAL_IDR_N_LP) && k <= first) start_pic = k;
      ++k;
    }
  }
  const int end_pic = count < 0 ? INT_MAX : first + count;
  struct DpbPic {
    int poc;
    Picture pic;
  };
  std::vector<DpbPic> dpb;          // reference pictures of the current sequence
  std::vector<DecodedPicture> cvs;  // decoded pictures of the current sequence (decoding order)
  int cvs_start = 0;                // output index of the sequence's first picture
  int prev_poc = 0;
  auto flush = [&] {
    std::stable_sort(cvs.begin(), cvs.end(), [](const DecodedPicture& a, const DecodedPicture& b) { return a.poc < b.poc; });
    for (size_t i = 0; i < cvs.size(); ++i) {
      const int o = cvs_start + (int)i;
      if (o >= first && o < end_pic) pictures.push_back(std::move(cvs[i]));
    }
    cvs_start += (int)cvs.size();
    cvs.clear();
  };
  int pic = -1;
  for (const auto& nal : nals) {
    if (nal.size < 2) continue;
    const int type = nal.type();
    if (type <= 21 && nal.size >= 3 && (nal.data[2] & 0x80)) {
      ++pic;
      const bool is_idr = type == NAL_IDR_W_RADL || type == NAL_IDR_N_LP;
      if (pic < start_pic) continue;
      if (is_idr && pic > start_pic && pic >= end_pic) break;
    } else if (type <= 21 && pic < start_pic) {
      continue;
    }
    std::vector<size_t> removed;  // escaped indices of the emulation-prevention bytes
    std::vector<uint8_t> rbsp = unescape_rbsp_map(nal.data + 2, nal.size - 2, &removed);
    BitReader br(rbsp.data(), rbsp.size());
    if (type == NAL_VPS || type == NAL_AUD || type >= 36) continue;
    if (type == NAL_SPS) {
      sps = parse_sps(br);
      width = sps.width;
      height = sps.height;
      coded_w = sps.coded_w;
      coded_h = sps.coded_h;
      continue;
    }
    if (type == NAL_PPS) {
      pps = parse_pps(br);
      continue;
    }
    if (type > 21) continue;
    if (!sps.valid || !pps.valid) fail("slice before parameter sets");
    const bool idr = (type == NAL_IDR_W_RADL || type == NAL_IDR_N_LP);
    if (!br.u(1)) fail("multiple slices per picture unsupported");
    if (type >= 16 && type <= 23) br.u(1);  // no_output_of_prior_pics_flag
    br.ue();
    const int stype = (int)br.ue();
    if (stype > 2) fail("bad slice_type");
    const bool islice = stype == 2;
    int poc = 0;
    std::vector<int> rps_poc, rps_used;  // the picture's reference picture set
    if (idr) {
      flush();
      cvs_start = pic;
      dpb.clear();
      prev_poc = 0;
    } else {
      const int lsb = (int)br.u(sps.log2_poc_lsb), max_lsb = 1 << sps.log2_poc_lsb;
      const int prev_lsb = prev_poc & (max_lsb - 1), prev_msb = prev_poc - prev_lsb;
      int msb = prev_msb;  // 8.3.1
      if (lsb < prev_lsb && prev_lsb - lsb >= max_lsb / 2) msb += max_lsb;
      else if (lsb > prev_lsb && lsb - prev_lsb > max_lsb / 2) msb -= max_lsb;
      poc = msb + lsb;
      if (br.u(1)) {  // short_term_ref_pic_set_sps_flag: the SPS set {-1, used}
        rps_poc.push_back(poc - 1);
        rps_used.push_back(1);
      } else {  // st_ref_pic_set(num_short_term_ref_pic_sets)
        if (br.u(1)) fail("inter RPS prediction unsupported");
        const int nn = (int)br.ue(), np = (int)br.ue();
        if (nn + np > kMaxRps) fail("RPS too large");
        for (int i = 0, p = poc; i < nn; ++i) {
          p -= (int)br.ue() + 1;
          rps_poc.push_back(p);
          rps_used.push_back((int)br.u(1));
        }
        for (int i = 0, p = poc; i < np; ++i) {
          p += (int)br.ue() + 1;
          rps_poc.push_back(p);
          rps_used.push_back((int)br.u(1));
        }
      }
    }
    bool sao = false;
    if (sps.sao) {
      const bool l = br.u(1), c = br.u(1);
      sao = l || c;
      if (l != c) fail("partial SAO unsupported");
    }
    int max_merge = 5;
    if (!islice) {
      if (br.u(1)) fail("num_ref_idx override unsupported");
      if (stype == 0 && br.u(1)) fail("mvd_l1_zero_flag unsupported");
      max_merge = 5 - (int)br.ue();
    }
    const int qp = pps.init_qp + br.se();
    std::vector<size_t> entry;  // substream sizes (escaped bytes)
    if (pps.wpp) {
      const uint32_t n = br.ue();
      if (n) {
        const int len = (int)br.ue() + 1;
        if (len > 32) fail("bad offset_len");
        for (uint32_t i = 0; i < n; ++i) entry.push_back((size_t)br.u(len) + 1);
      }
    }
    // byte_alignment()
    if (br.bit() != 1) fail("missing alignment bit");
    while (br.pos() & 7)
      if (br.bit() != 0) fail("bad alignment bits");
    std::vector<size_t> row_start;
    if (pps.wpp) {  // entry points count emulation-prevention bytes: map them to RBSP bytes
      const size_t d0 = br.byte_pos();
      size_t esc = d0;
      for (size_t e : removed)
        if (e <= esc) ++esc;  // escaped index of RBSP byte d0
      auto rbsp_of = [&](size_t e) {
        size_t k = 0;
        while (k < removed.size() && removed[k] < e) ++k;
        return e - k;
      };
      row_start.push_back(d0);
      for (size_t s : entry) {
        esc += s;
        row_start.push_back(rbsp_of(esc));
      }
    }
    // reference marking (8.3.2): pictures outside the RPS leave the DPB; lists with one
    // active entry each (8.3.4): L0 = the closest used past picture (else future), L1 = the
    // closest used future picture (else past)
    const Picture* ref[2] = {nullptr, nullptr};
    int ref_poc[2] = {-1, -1};
    if (!idr) {
      std::vector<DpbPic> kept;
      for (auto& d : dpb)
        for (int p : rps_poc)
          if (d.poc == p) {
            kept.push_back(std::move(d));
            break;
          }
      dpb = std::move(kept);
      int before = INT_MIN, after = INT_MAX;
      for (size_t i = 0; i < rps_poc.size(); ++i) {
        if (!rps_used[i]) continue;
        const int p = rps_poc[i];
        bool present = false;
        for (const auto& d : dpb) present = present || d.poc == p;
        if (!present) fail("reference picture missing from the DPB");
        if (p < poc) before = std::max(before, p);
        else after = std::min(after, p);
      }
      const int l0 = before != INT_MIN ? before : after, l1 = after != INT_MAX ? after : before;
      if (l0 == INT_MAX) fail("inter slice without a reference");
      ref_poc[0] = l0;
      ref_poc[1] = stype == 0 ? l1 : -1;
      for (const auto& d : dpb) {
        if (d.poc == ref_poc[0]) ref[0] = &d.pic;
        if (d.poc == ref_poc[1]) ref[1] = &d.pic;
      }
    }
    DecodedPicture dp;
    dp.poc = poc;
    dp.idr = idr;
    dp.pic.alloc(sps.coded_w, sps.coded_h);
    last_decisions.alloc(sps.coded_w, sps.coded_h);
    if (stype == 0) {
      last_decisions.has_refs = true;
      last_decisions.refs.type = 0;
      last_decisions.refs.poc = poc;
      last_decisions.refs.ref_poc[0] = ref_poc[0];
      last_decisions.refs.ref_poc[1] = ref_poc[1];
    }
    SliceDecoder sd(sps, pps, stype, qp, max_merge, &br, &dp.pic, ref, ref_poc, poc, &last_decisions, sao, row_start);
    sd.run();
    if (pps.deblock) deblock_picture(dp.pic, last_decisions.view(), qp);
    if (sao) sao_picture(dp.pic, last_decisions.sao.data());
    dpb.push_back(DpbPic{poc, dp.pic});
    prev_poc = poc;
    cvs.push_back(std::move(dp));
  }
  flush();
}

}  // namespace tv
