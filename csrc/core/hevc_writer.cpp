// hevc_writer.cpp — HEVC parameter sets and CABAC slice-data writer.
//
// Consumes the per-frame decision arrays (FrameData) produced by the analysis stage and
// emits a Main-profile Annex-B bitstream.  Skip / merge / AMVP syntax is chosen here from
// the final motion field (the GPU only decides motion vectors and residuals), which keeps
// the GPU analysis fully parallel while the serial CABAC runs on CPU threads — the
// MI355X-native split of the reference's single ffmpeg call (reference
// worker/tasks.py:1532-1586).
#include <emmintrin.h>
#include <algorithm>
#include <cstring>
#include <stdexcept>

#include "tv/bitstream.h"
#include "tv/cabac.h"
#include "tv/hevc_codec.h"

namespace tv {

const uint8_t kRangeTabLps[64][4] = {
    {128, 176, 208, 240}, {128, 167, 197, 227}, {128, 158, 187, 216}, {123, 150, 178, 205},
    {116, 142, 169, 195}, {111, 135, 160, 185}, {105, 128, 152, 175}, {100, 122, 144, 166},
    {95, 116, 137, 158},  {90, 110, 130, 150},  {85, 104, 123, 142},  {81, 99, 117, 135},
    {77, 94, 111, 128},   {73, 89, 105, 122},   {69, 85, 100, 116},   {66, 80, 95, 110},
    {62, 76, 90, 104},    {59, 72, 86, 99},     {56, 69, 81, 94},     {53, 65, 77, 89},
    {51, 62, 73, 85},     {48, 59, 69, 80},     {46, 56, 66, 76},     {43, 53, 63, 72},
    {41, 50, 59, 69},     {39, 48, 56, 65},     {37, 45, 54, 62},     {35, 43, 51, 59},
    {33, 41, 48, 56},     {32, 39, 46, 53},     {30, 37, 43, 50},     {29, 35, 41, 48},
    {27, 33, 39, 45},     {26, 31, 37, 43},     {24, 30, 35, 41},     {23, 28, 33, 39},
    {22, 27, 32, 37},     {21, 26, 30, 35},     {20, 24, 29, 33},     {19, 23, 27, 31},
    {18, 22, 26, 30},     {17, 21, 25, 28},     {16, 20, 23, 27},     {15, 19, 22, 25},
    {14, 18, 21, 24},     {14, 17, 20, 23},     {13, 16, 19, 22},     {12, 15, 18, 21},
    {12, 14, 17, 20},     {11, 14, 16, 19},     {11, 13, 15, 18},     {10, 12, 15, 17},
    {10, 12, 14, 16},     {9, 11, 13, 15},      {9, 11, 12, 14},      {8, 10, 12, 14},
    {8, 9, 11, 13},       {7, 9, 11, 12},       {7, 9, 10, 12},       {7, 8, 10, 11},
    {6, 8, 9, 11},        {6, 7, 9, 10},        {6, 7, 8, 9},         {2, 2, 2, 2}};
const uint8_t kTransIdxLps[64] = {0,  0,  1,  2,  2,  4,  4,  5,  6,  7,  8,  9,  9,  11, 11, 12,
                                  13, 13, 15, 15, 16, 16, 18, 18, 19, 19, 21, 21, 22, 22, 23, 24,
                                  24, 25, 26, 26, 27, 27, 28, 29, 29, 30, 30, 30, 31, 32, 32, 33,
                                  33, 33, 34, 34, 35, 35, 35, 36, 36, 36, 37, 37, 37, 38, 38, 63};

int SeqConfig::level_idc() const {
  const long long ps = (long long)coded_w * coded_h;
  if (ps <= 2228224) return 123;  // 4.1
  if (ps <= 8912896) return 153;  // 5.1
  return 186;                     // 6.2
}

static void write_ptl(BitWriter& bw, int level) {
  bw.put(0, 2);  // general_profile_space
  bw.put(0, 1);  // general_tier_flag
  bw.put(1, 5);  // general_profile_idc = Main
  bw.put((1u << 30) | (1u << 29), 32);  // compatibility flags [1] and [2]
  bw.put(1, 1);  // progressive_source
  bw.put(0, 1);  // interlaced_source
  bw.put(0, 1);  // non_packed_constraint
  bw.put(1, 1);  // frame_only_constraint
  bw.put(0, 32);
  bw.put(0, 11);  // 43 reserved zero bits
  bw.put(0, 1);   // general_inbld_flag (reserved)
  bw.put((uint32_t)level, 8);
}

void write_parameter_sets(const SeqConfig& cfg, std::vector<uint8_t>& out) {
  if ((cfg.width & 1) || (cfg.height & 1)) throw std::runtime_error("odd picture size");
  {  // VPS
    BitWriter bw;
    bw.put(0, 4);       // vps_video_parameter_set_id
    bw.put(1, 1);       // vps_base_layer_internal_flag
    bw.put(1, 1);       // vps_base_layer_available_flag
    bw.put(0, 6);       // vps_max_layers_minus1
    bw.put(0, 3);       // vps_max_sub_layers_minus1
    bw.put(1, 1);       // vps_temporal_id_nesting_flag
    bw.put(0xffff, 16); // reserved
    write_ptl(bw, cfg.level_idc());
    bw.put(1, 1);  // vps_sub_layer_ordering_info_present_flag
    bw.ue((uint32_t)std::max(1, cfg.dpb_size - 1));  // vps_max_dec_pic_buffering_minus1
    bw.ue((uint32_t)cfg.num_reorder);                 // vps_max_num_reorder_pics
    bw.ue(0);      // vps_max_latency_increase_plus1
    bw.put(0, 6);  // vps_max_layer_id
    bw.ue(0);      // vps_num_layer_sets_minus1
    bw.put(0, 1);  // vps_timing_info_present_flag
    bw.put(0, 1);  // vps_extension_flag
    bw.trailing_bits();
    append_nal(out, NAL_VPS, bw.bytes());
  }
  {  // SPS
    BitWriter bw;
    bw.put(0, 4);  // sps_video_parameter_set_id
    bw.put(0, 3);  // sps_max_sub_layers_minus1
    bw.put(1, 1);  // sps_temporal_id_nesting_flag
    write_ptl(bw, cfg.level_idc());
    bw.ue(0);  // sps_seq_parameter_set_id
    bw.ue(1);  // chroma_format_idc 4:2:0
    bw.ue((uint32_t)cfg.coded_w);
    bw.ue((uint32_t)cfg.coded_h);
    const bool crop = cfg.coded_w != cfg.width || cfg.coded_h != cfg.height;
    bw.put(crop ? 1 : 0, 1);
    if (crop) {
      bw.ue(0);
      bw.ue((uint32_t)(cfg.coded_w - cfg.width) / 2);
      bw.ue(0);
      bw.ue((uint32_t)(cfg.coded_h - cfg.height) / 2);
    }
    bw.ue(0);  // bit_depth_luma_minus8
    bw.ue(0);  // bit_depth_chroma_minus8
    bw.ue(4);  // log2_max_pic_order_cnt_lsb_minus4 -> 8 bits
    bw.put(1, 1);  // sps_sub_layer_ordering_info_present_flag
    bw.ue((uint32_t)std::max(1, cfg.dpb_size - 1));  // sps_max_dec_pic_buffering_minus1
    bw.ue((uint32_t)cfg.num_reorder);                 // sps_max_num_reorder_pics
    bw.ue(0);      // sps_max_latency_increase_plus1
    bw.ue(kMinCbLog2 - 3);           // log2_min_luma_coding_block_size_minus3
    bw.ue(kCtbLog2 - kMinCbLog2);    // log2_diff_max_min_luma_coding_block_size
    bw.ue(kMinTbLog2 - 2);           // log2_min_luma_transform_block_size_minus2
    bw.ue(kMaxTbLog2 - kMinTbLog2);  // log2_diff_max_min_luma_transform_block_size
    bw.ue(cfg.rqt ? 1 : 0);  // max_transform_hierarchy_depth_inter (RQT: 32x32 -> 4 x 16x16)
    bw.ue(0);      // max_transform_hierarchy_depth_intra
    bw.put(0, 1);  // scaling_list_enabled_flag
    bw.put(0, 1);  // amp_enabled_flag
    bw.put(cfg.sao ? 1 : 0, 1);  // sample_adaptive_offset_enabled_flag
    bw.put(0, 1);  // pcm_enabled_flag
    bw.ue(1);      // num_short_term_ref_pic_sets
    // st_ref_pic_set(0): one negative picture at delta -1, used by current
    bw.ue(1);      // num_negative_pics
    bw.ue(0);      // num_positive_pics
    bw.ue(0);      // delta_poc_s0_minus1
    bw.put(1, 1);  // used_by_curr_pic_s0_flag
    bw.put(0, 1);  // long_term_ref_pics_present_flag
    bw.put(0, 1);  // sps_temporal_mvp_enabled_flag
    bw.put(0, 1);  // strong_intra_smoothing_enabled_flag
    bw.put(0, 1);  // vui_parameters_present_flag
    bw.put(0, 1);  // sps_extension_present_flag
    bw.trailing_bits();
    append_nal(out, NAL_SPS, bw.bytes());
  }
  {  // PPS
    BitWriter bw;
    bw.ue(0);      // pps_pic_parameter_set_id
    bw.ue(0);      // pps_seq_parameter_set_id
    bw.put(0, 1);  // dependent_slice_segments_enabled_flag
    bw.put(0, 1);  // output_flag_present_flag
    bw.put(0, 3);  // num_extra_slice_header_bits
    bw.put(0, 1);  // sign_data_hiding_enabled_flag
    bw.put(0, 1);  // cabac_init_present_flag
    bw.ue(0);      // num_ref_idx_l0_default_active_minus1
    bw.ue(0);      // num_ref_idx_l1_default_active_minus1
    bw.se(cfg.qp - 26);  // init_qp_minus26
    bw.put(0, 1);  // constrained_intra_pred_flag
    bw.put(0, 1);  // transform_skip_enabled_flag
    bw.put(0, 1);  // cu_qp_delta_enabled_flag
    bw.se(0);      // pps_cb_qp_offset
    bw.se(0);      // pps_cr_qp_offset
    bw.put(0, 1);  // pps_slice_chroma_qp_offsets_present_flag
    bw.put(0, 1);  // weighted_pred_flag
    bw.put(0, 1);  // weighted_bipred_flag
    bw.put(0, 1);  // transquant_bypass_enabled_flag
    bw.put(0, 1);  // tiles_enabled_flag
    bw.put(cfg.wpp ? 1 : 0, 1);  // entropy_coding_sync_enabled_flag
    bw.put(0, 1);  // pps_loop_filter_across_slices_enabled_flag
    bw.put(1, 1);  // deblocking_filter_control_present_flag
    bw.put(0, 1);  //   deblocking_filter_override_enabled_flag
    bw.put(cfg.deblock ? 0 : 1, 1);  // pps_deblocking_filter_disabled_flag
    if (cfg.deblock) {
      bw.se(0);  // pps_beta_offset_div2
      bw.se(0);  // pps_tc_offset_div2
    }
    bw.put(0, 1);  // pps_scaling_list_data_present_flag
    bw.put(0, 1);  // lists_modification_present_flag
    bw.ue(0);      // log2_parallel_merge_level_minus2
    bw.put(0, 1);  // slice_segment_header_extension_present_flag
    bw.put(0, 1);  // pps_extension_present_flag
    bw.trailing_bits();
    append_nal(out, NAL_PPS, bw.bytes());
  }
}

// ------------------------------------ slice data ----------------------------------------
namespace {

constexpr uint8_t kCtxIdxMap4x4[16] = {0, 1, 4, 5, 2, 3, 4, 5, 6, 6, 8, 8, 7, 7, 8, 8};
constexpr uint8_t kGroupIdx[32] = {0, 1, 2, 3, 4, 4, 5, 5, 6, 6, 6, 6, 7, 7, 7, 7,
                                   8, 8, 8, 8, 8, 8, 8, 8, 9, 9, 9, 9, 9, 9, 9, 9};
constexpr uint8_t kMinInGroup[10] = {0, 1, 2, 3, 4, 6, 8, 12, 16, 24};

class SliceWriter {
 public:
  SliceWriter(const SeqConfig& cfg, const FrameData& fd, bool islice, BitWriter* bw)
      : cfg_(cfg), fd_(fd), islice_(islice), bslice_(fd.refs && fd.refs->type == 0), enc_(bw) {
    skip_.assign((size_t)fd.w8 * fd.h8, 0);
    // initType 0 / 1 / 2 for I / P / B (no cabac_init_flag); contexts start from SliceQpY
    ctx_.init(islice ? 0 : (bslice_ ? 2 : 1), fd.qp >= 0 ? fd.qp : cfg.qp);
    enc_.start();
  }

  // rows (WPP): one BitWriter per CTB row; row 0 may be the slice's own writer
  void write_all(std::vector<BitWriter>* rows = nullptr) {
    const int wc = cfg_.coded_w >> kCtbLog2, hc = cfg_.coded_h >> kCtbLog2;
    ContextSet synced{};  // WPP: the contexts after the second CTB of the row above
    for (int cy = 0; cy < hc; ++cy) {
      if (rows && cy > 0) {  // a new substream: fresh arithmetic coder, synced contexts
        enc_.rebind(&(*rows)[cy]);
        enc_.start();
        ctx_ = synced;
      }
      for (int cx = 0; cx < wc; ++cx) {
        if (cfg_.sao) write_sao(cx, cy, wc);
        quadtree(cx << kCtbLog2, cy << kCtbLog2, kCtbLog2, 0);
        const bool last = (cy == hc - 1) && (cx == wc - 1);
        if (rows && cx == 1) synced = ctx_;  // storage process (9.3.2.4) after CtbAddrX == 1
        enc_.encode_terminate(last ? 1 : 0);  // end_of_slice_segment_flag
        if (rows && !last && cx == wc - 1) {   // end_of_subset_one_bit + byte_alignment()
          enc_.encode_terminate(1);
          enc_.finish();
          (*rows)[cy].put_bit(1);
          (*rows)[cy].align_zero();
        }
      }
    }
    enc_.finish();
  }

 private:
  int unit(int x, int y) const { return (y >> 3) * fd_.w8 + (x >> 3); }
  bool avail(int xc, int yc, int xn, int yn) const {
    return zscan_available(xc, yc, xn, yn, cfg_.coded_w, cfg_.coded_h);
  }
  // the left / upper neighbour of a CU always precedes it in z-scan order (one slice, no
  // tiles): only the picture edge makes them unavailable
  static bool has_left(int x0) { return x0 > 0; }
  static bool has_up(int y0) { return y0 > 0; }
  void bin(int b, int ctx) { enc_.encode_bin(b, ctx_.c[ctx]); }

  // sao() (7.3.8.3).  Merges are chosen by exact parameter equality with the left / upper
  // CTB, so they never change the reconstruction.
  void write_sao(int cx, int cy, int wc) {
    const uint32_t none[3] = {sao_off_param(), sao_off_param(), sao_off_param()};
    const uint32_t* p = fd_.sao ? fd_.sao + 3 * (size_t)(cy * wc + cx) : none;
    auto same = [&](const uint32_t* q) { return q[0] == p[0] && q[1] == p[1] && q[2] == p[2]; };
    if (cx > 0) {
      const bool m = fd_.sao && same(p - 3);
      bin(m, CTX_SAO_MERGE);
      if (m) return;
    }
    if (cy > 0) {
      const bool m = fd_.sao && same(p - 3 * (size_t)wc);
      bin(m, CTX_SAO_MERGE);
      if (m) return;
    }
    for (int c = 0; c < 3; ++c) {
      const int t = sao_type(p[c]);
      if (c < 2) {  // sao_type_idx_luma / _chroma: TR cMax 2, first bin context coded
        bin(t != 0, CTX_SAO_TYPE);
        if (t) enc_.encode_bypass(t == 2);
      }
      if (!t) continue;
      for (int i = 0; i < 4; ++i) {  // sao_offset_abs: TR bypass, cMax 7
        const int a = tv_abs(sao_offset(p[c], i));
        for (int k = 0; k < a; ++k) enc_.encode_bypass(1);
        if (a < kSaoMaxOff) enc_.encode_bypass(0);
      }
      if (t == 1) {
        for (int i = 0; i < 4; ++i)
          if (sao_offset(p[c], i)) enc_.encode_bypass(sao_offset(p[c], i) < 0);
        enc_.encode_bypass_bins((uint32_t)sao_class(p[c]), 5);  // sao_band_position
      } else if (c < 2) {
        enc_.encode_bypass_bins((uint32_t)sao_class(p[c]), 2);  // sao_eo_class_luma / _chroma
      }
    }
  }

  void quadtree(int x0, int y0, int log2, int depth) {
    const int u = unit(x0, y0);
    const bool split = fd_.cu_log2[u] < log2;
    if (log2 > kMinCbLog2) {
      int inc = 0;
      if (has_left(x0) && (kCtbLog2 - fd_.cu_log2[unit(x0 - 1, y0)]) > depth) ++inc;
      if (has_up(y0) && (kCtbLog2 - fd_.cu_log2[unit(x0, y0 - 1)]) > depth) ++inc;
      bin(split ? 1 : 0, CTX_SPLIT_CU + inc);
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

  void set_skip(int x0, int y0, int log2, uint8_t v) {
    const int n = 1 << (log2 - 3);
    for (int j = 0; j < n; ++j)
      for (int i = 0; i < n; ++i) skip_[unit(x0 + 8 * i, y0 + 8 * j)] = v;
  }

  bool inter_at(int xc, int yc, int xn, int yn, Mv& mv) const {
    if (!avail(xc, yc, xn, yn)) return false;
    const int u = unit(xn, yn);
    if (fd_.intra[u]) return false;
    mv.x = fd_.mv[2 * u];
    mv.y = fd_.mv[2 * u + 1];
    return true;
  }

  // Index of `mv` in the P-slice merge list of the 2Nx2N PU at (x0, y0) (the list of
  // merge_candidates(), hevc_codec.h, 8.5.3.2.2-3), or -1: the list is built in order and the
  // search stops at the first match.  A1, B1 and B2 precede the PU in z-scan whenever they
  // are inside the picture, so only B0 and A0 need the z-scan availability test.
  int merge_index_p(int x0, int y0, int N, Mv mv) const {
    const int maxc = cfg_.max_merge_cand;
    auto get = [&](int xn, int yn, Mv& m) {
      const int u = unit(xn, yn);
      if (fd_.intra[u]) return false;
      m.x = fd_.mv[2 * u];
      m.y = fd_.mv[2 * u + 1];
      return true;
    };
    Mv a1, b1, b0, a0, b2;
    int n = 0;
    const bool avA1 = x0 > 0 && get(x0 - 1, y0 + N - 1, a1);
    if (avA1) {
      if (a1 == mv) return 0;
      if (++n == maxc) return -1;
    }
    const bool avB1 = y0 > 0 && get(x0 + N - 1, y0 - 1, b1);
    const bool fB1 = avB1 && !(avA1 && a1 == b1);
    if (fB1) {
      if (b1 == mv) return n;
      if (++n == maxc) return -1;
    }
    const bool avB0 = avail(x0, y0, x0 + N, y0 - 1) && get(x0 + N, y0 - 1, b0);
    const bool fB0 = avB0 && !(avB1 && b1 == b0);
    if (fB0) {
      if (b0 == mv) return n;
      if (++n == maxc) return -1;
    }
    const bool avA0 = avail(x0, y0, x0 - 1, y0 + N) && get(x0 - 1, y0 + N, a0);
    const bool fA0 = avA0 && !(avA1 && a1 == a0);
    if (fA0) {
      if (a0 == mv) return n;
      if (++n == maxc) return -1;
    }
    const bool avB2 = x0 > 0 && y0 > 0 && get(x0 - 1, y0 - 1, b2);
    if (avB2 && !(avA1 && a1 == b2) && !(avB1 && b1 == b2) && (int)avA1 + (int)fB1 + (int)fB0 + (int)fA0 < 4) {
      if (b2 == mv) return n;
      if (++n == maxc) return -1;
    }
    return (mv.x == 0 && mv.y == 0) ? n : -1;  // zero candidates fill the list
  }

  Motion motion_of(int u) const {
    Motion m;
    m.dir = fd_.dir ? fd_.dir[u] : 1;
    m.mv[0] = Mv{fd_.mv[2 * u], fd_.mv[2 * u + 1]};
    if (fd_.mv1) m.mv[1] = Mv{fd_.mv1[2 * u], fd_.mv1[2 * u + 1]};
    return m;
  }
  bool motion_at(int xc, int yc, int xn, int yn, Motion& m) const {
    if (!avail(xc, yc, xn, yn)) return false;
    const int u = unit(xn, yn);
    if (fd_.intra[u]) return false;
    m = motion_of(u);
    return true;
  }

  // B-slice inter CU (7.3.8.5 / 7.3.8.6): skip / merge when the PU's motion equals a merge
  // candidate, else inter_pred_idc + per-list mvd / mvp flag against the AMVP lists
  void coding_unit_b(int x0, int y0, int log2, int cbf) {
    const int u = unit(x0, y0), N = 1 << log2;
    const Motion m = motion_of(u);
    const SliceRefs& r = *fd_.refs;
    auto at = [&](int xn, int yn, Motion& o) { return motion_at(x0, y0, xn, yn, o); };
    Motion cand[5];
    const int nc = merge_candidates_b(x0, y0, N, N, cfg_.max_merge_cand, r.ref_poc[0] == r.ref_poc[1], at, cand);
    int merge_idx = -1;
    for (int i = 0; i < nc; ++i)
      if (cand[i] == m) {
        merge_idx = i;
        break;
      }
    const bool skip = merge_idx >= 0 && cbf == 0;
    int inc = 0;
    if (has_left(x0) && skip_[unit(x0 - 1, y0)]) ++inc;
    if (has_up(y0) && skip_[unit(x0, y0 - 1)]) ++inc;
    bin(skip ? 1 : 0, CTX_CU_SKIP + inc);
    set_skip(x0, y0, log2, skip ? 1 : 0);
    if (skip) {
      write_merge_idx(merge_idx);
      return;
    }
    bin(0, CTX_PRED_MODE);  // MODE_INTER
    bin(1, CTX_PART_MODE);  // 2Nx2N
    bin(merge_idx >= 0 ? 1 : 0, CTX_MERGE_FLAG);
    if (merge_idx >= 0) {
      write_merge_idx(merge_idx);
    } else {
      // inter_pred_idc (9.3.4.2.2): bin 0 (PRED_BI?) at ctx CtDepth, bin 1 (L1?) at ctx 4
      bin(m.dir == 3 ? 1 : 0, CTX_INTER_PRED_IDC + (kCtbLog2 - log2));
      if (m.dir != 3) bin(m.dir == 2 ? 1 : 0, CTX_INTER_PRED_IDC + 4);
      for (int X = 0; X < 2; ++X) {
        if (!((m.dir >> X) & 1)) continue;
        Mv mvp[2];
        amvp_candidates_b(x0, y0, N, N, X, r.ref_poc, r.poc, at, mvp);
        const Mv v = m.mv[X];
        const int c0 = mvd_cost(v.x - mvp[0].x) + mvd_cost(v.y - mvp[0].y);
        const int c1 = mvd_cost(v.x - mvp[1].x) + mvd_cost(v.y - mvp[1].y);
        const int sel = c1 < c0 ? 1 : 0;
        write_mvd(v.x - mvp[sel].x, v.y - mvp[sel].y);
        bin(sel, CTX_MVP_FLAG);
      }
      bin(cbf ? 1 : 0, CTX_RQT_ROOT_CBF);
      if (!cbf) return;
    }
    transform_tree(x0, y0, log2, false, 0);
  }

  void coding_unit(int x0, int y0, int log2) {
    const int u = unit(x0, y0);
    const int N = 1 << log2;
    const bool intra = fd_.intra[u] != 0;
    const int cbf = cu_cbf(x0, y0, log2);
    if (bslice_ && !intra) {
      coding_unit_b(x0, y0, log2, cbf);
      return;
    }
    if (bslice_) {  // intra CU in a B slice
      int inc = 0;
      if (has_left(x0) && skip_[unit(x0 - 1, y0)]) ++inc;
      if (has_up(y0) && skip_[unit(x0, y0 - 1)]) ++inc;
      bin(0, CTX_CU_SKIP + inc);
      set_skip(x0, y0, log2, 0);
      bin(1, CTX_PRED_MODE);
    } else if (!islice_) {
      // decide skip / merge / amvp from the motion field
      Mv mv{fd_.mv[2 * u], fd_.mv[2 * u + 1]};
      const int merge_idx = intra ? -1 : merge_index_p(x0, y0, N, mv);
      const bool skip = !intra && merge_idx >= 0 && cbf == 0;
      int inc = 0;
      if (has_left(x0) && skip_[unit(x0 - 1, y0)]) ++inc;
      if (has_up(y0) && skip_[unit(x0, y0 - 1)]) ++inc;
      bin(skip ? 1 : 0, CTX_CU_SKIP + inc);
      set_skip(x0, y0, log2, skip ? 1 : 0);
      if (skip) {
        write_merge_idx(merge_idx);
        return;
      }
      bin(intra ? 1 : 0, CTX_PRED_MODE);  // pred_mode_flag
      if (!intra) {
        bin(1, CTX_PART_MODE);  // part_mode 2Nx2N
        const bool merge = merge_idx >= 0;
        bin(merge ? 1 : 0, CTX_MERGE_FLAG);
        if (merge) {
          write_merge_idx(merge_idx);
        } else {
          Mv mvp[2];
          auto f = [&](int xn, int yn, Mv& m) { return inter_at(x0, y0, xn, yn, m); };
          amvp_candidates(x0, y0, N, N, f, mvp);
          const int c0 = mvd_cost(mv.x - mvp[0].x) + mvd_cost(mv.y - mvp[0].y);
          const int c1 = mvd_cost(mv.x - mvp[1].x) + mvd_cost(mv.y - mvp[1].y);
          const int sel = c1 < c0 ? 1 : 0;
          write_mvd(mv.x - mvp[sel].x, mv.y - mvp[sel].y);
          bin(sel, CTX_MVP_FLAG);
          bin(cbf ? 1 : 0, CTX_RQT_ROOT_CBF);
          if (!cbf) return;
        }
        transform_tree(x0, y0, log2, false, 0);
        return;
      }
    }
    // intra CU
    if (log2 == kMinCbLog2) bin(1, CTX_PART_MODE);  // 2Nx2N
    const int mode = fd_.ipm[u];
    int candA = 1, candB = 1;
    if (has_left(x0) && fd_.intra[unit(x0 - 1, y0)]) candA = fd_.ipm[unit(x0 - 1, y0)];
    if (has_up(y0) && fd_.intra[unit(x0, y0 - 1)] && (y0 - 1) >= ((y0 >> kCtbLog2) << kCtbLog2))
      candB = fd_.ipm[unit(x0, y0 - 1)];
    int mpm[3];
    intra_mpm_list(candA, candB, mpm);
    int idx = -1;
    for (int i = 0; i < 3; ++i)
      if (mpm[i] == mode) idx = i;
    bin(idx >= 0 ? 1 : 0, CTX_PREV_INTRA);
    if (idx >= 0) {
      enc_.encode_bypass(idx > 0);
      if (idx > 0) enc_.encode_bypass(idx > 1);
    } else {
      // rem_intra_luma_pred_mode: the mode minus the MPMs below it (order-free count)
      const int rem = mode - (mode > mpm[0]) - (mode > mpm[1]) - (mode > mpm[2]);
      enc_.encode_bypass_bins((uint32_t)rem, 5);
    }
    bin(0, CTX_CHROMA_PRED);  // intra_chroma_pred_mode = 4 (DM)
    transform_tree(x0, y0, log2, true, mode);
  }

  static int mvd_cost(int d) {  // bins of one mvd component (approx)
    int a = d < 0 ? -d : d;
    if (a == 0) return 1;
    if (a == 1) return 3;
    int v = a - 2, k = 1, n = 0;
    while (v >= (1 << k)) {
      v -= 1 << k;
      ++k;
      ++n;
    }
    return 3 + n + 1 + k;
  }

  void write_merge_idx(int idx) {
    if (cfg_.max_merge_cand <= 1) return;
    bin(idx > 0 ? 1 : 0, CTX_MERGE_IDX);
    for (int i = 1; i < cfg_.max_merge_cand - 1 && idx >= i; ++i) enc_.encode_bypass(idx > i);
  }

  void write_eg1(uint32_t v) {  // k-th order Exp-Golomb, k = 1, bypass
    int k = 1;
    while (v >= (1u << k)) {
      enc_.encode_bypass(1);
      v -= 1u << k;
      ++k;
    }
    enc_.encode_bypass(0);
    enc_.encode_bypass_bins(v, k);
  }

  void write_mvd(int dx, int dy) {
    const int ax = dx < 0 ? -dx : dx, ay = dy < 0 ? -dy : dy;
    bin(ax > 0, CTX_MVD_G0);
    bin(ay > 0, CTX_MVD_G0);
    if (ax > 0) bin(ax > 1, CTX_MVD_G1);
    if (ay > 0) bin(ay > 1, CTX_MVD_G1);
    if (ax > 0) {
      if (ax > 1) write_eg1((uint32_t)(ax - 2));
      enc_.encode_bypass(dx < 0);
    }
    if (ay > 0) {
      if (ay > 1) write_eg1((uint32_t)(ay - 2));
      enc_.encode_bypass(dy < 0);
    }
  }

  bool tu_split(int x0, int y0) const { return fd_.tu && fd_.tu[unit(x0, y0)]; }
  // cbf bits of the CU at (x0, y0): an RQT-split CU's are the OR of its four TBs'
  int cu_cbf(int x0, int y0, int log2) const {
    if (!tu_split(x0, y0)) return fd_.cbf[unit(x0, y0)];
    const int h = 1 << (log2 - 1);
    int c = 0;
    for (int q = 0; q < 4; ++q) c |= fd_.cbf[unit(x0 + (q & 1) * h, y0 + (q >> 1) * h)];
    return c;
  }
  // An inter CU (32x32 or 16x16) split once (7.3.8.8 at trafoDepth 0 -> 1): the chroma cbfs
  // at depth 0 are the OR of the quadrants', then per quadrant in z-order its chroma cbfs
  // (under a set parent), cbf_luma (always coded at depth 1) and the residuals.
  void transform_split(int x0, int y0, int log2) {
    const int h = 1 << (log2 - 1), l = log2 - 1;
    int c[4], cb0 = 0, cr0 = 0;
    for (int q = 0; q < 4; ++q) {
      c[q] = fd_.cbf[unit(x0 + (q & 1) * h, y0 + (q >> 1) * h)];
      cb0 |= (c[q] >> 1) & 1;
      cr0 |= (c[q] >> 2) & 1;
    }
    bin(cb0, CTX_CBF_CHROMA + 0);
    bin(cr0, CTX_CBF_CHROMA + 0);
    for (int q = 0; q < 4; ++q) {
      const int x = x0 + (q & 1) * h, y = y0 + (q >> 1) * h;
      const int cl = c[q] & 1, cb = (c[q] >> 1) & 1, cr = (c[q] >> 2) & 1;
      if (cb0) bin(cb, CTX_CBF_CHROMA + 1);
      if (cr0) bin(cr, CTX_CBF_CHROMA + 1);
      bin(cl, CTX_CBF_LUMA + 0);
      TbView v;
      if (cl) {
        tb_view(0, x, y, l, v);
        residual(v, l, 0, 0);
      }
      if (cb) {
        tb_view(1, x >> 1, y >> 1, l - 1, v);
        residual(v, l - 1, 1, 0);
      }
      if (cr) {
        tb_view(2, x >> 1, y >> 1, l - 1, v);
        residual(v, l - 1, 2, 0);
      }
    }
  }

  void transform_tree(int x0, int y0, int log2, bool intra, int mode) {
    if (!intra && cfg_.rqt) {  // split_transform_flag of an inter CU (depth 0, ctx 5 - log2)
      const bool split = tu_split(x0, y0);
      bin(split ? 1 : 0, CTX_SPLIT_TF + 5 - log2);
      if (split) return transform_split(x0, y0, log2);
    }
    const int cbf = fd_.cbf[unit(x0, y0)];
    const int cl = cbf & 1, cb = (cbf >> 1) & 1, cr = (cbf >> 2) & 1;
    // log2 >= 3 here, so chroma cbfs are coded at depth 0
    bin(cb, CTX_CBF_CHROMA + 0);
    bin(cr, CTX_CBF_CHROMA + 0);
    if (intra || cb || cr) bin(cl, CTX_CBF_LUMA + 1);
    else if (!cl) throw std::runtime_error("inter CU with rqt_root_cbf=1 but no residual");
    const int cmode = intra ? chroma_intra_mode(4, mode) : 0;
    TbView v;
    if (cl) {
      tb_view(0, x0, y0, log2, v);
      residual(v, log2, 0, scan_idx_for(intra, log2, 0, mode));
    }
    if (cb) {
      tb_view(1, x0 >> 1, y0 >> 1, log2 - 1, v);
      residual(v, log2 - 1, 1, scan_idx_for(intra, log2 - 1, 1, cmode));
    }
    if (cr) {
      tb_view(2, x0 >> 1, y0 >> 1, log2 - 1, v);
      residual(v, log2 - 1, 2, scan_idx_for(intra, log2 - 1, 2, cmode));
    }
  }

  // Levels of the TB of component c at component position (x, y), as its 4x4 sub-blocks:
  // sb[ys * nsb + xs] points at the sub-block's top-left level (row stride `stride`) and bit
  // ys * nsb + xs of `nz` is set iff it holds a non-zero level.  Dense planes (CPU path) are
  // scanned once; the compact GPU form reads the CTB group masks and points straight into the
  // packed groups (stride 4) — no gather, and zero sub-blocks are never touched.
  struct TbView {
    const int16_t* sb[64];
    int stride;
    uint64_t nz;
  };
  void tb_view(int c, int x, int y, int log2N, TbView& v) const {
    const int nsb = 1 << (log2N - 2);
    v.nz = 0;
    if (!fd_.sb_packed) {
      v.stride = c ? cfg_.coded_w >> 1 : cfg_.coded_w;
      const int16_t* base = fd_.coef[c] + (size_t)y * v.stride + x;
      for (int ys = 0; ys < nsb; ++ys)
        for (int xs = 0; xs < nsb; ++xs) {
          const int16_t* p = base + (size_t)(4 * ys) * v.stride + 4 * xs;
          v.sb[ys * nsb + xs] = p;
          uint64_t any = 0;
          for (int r = 0; r < 4; ++r) {
            uint64_t w;
            std::memcpy(&w, p + (size_t)r * v.stride, 8);
            any |= w;
          }
          if (any) v.nz |= 1ull << (ys * nsb + xs);
        }
      return;
    }
    // a TB (= CU) never straddles a CTB: its groups are a rectangle of the CTB's group mask
    // (luma 8 groups per row; Cb / Cr 4 per row at bit 0 / 16), pointers only for set bits
    v.stride = 4;
    const int sh = c ? 4 : 5, gw = c ? 4 : 8;
    const int ctb = (y >> sh) * fd_.wc + (x >> sh);
    const uint64_t my = fd_.sb_mask_y[ctb];
    const uint64_t m = c ? (uint64_t)fd_.sb_mask_c[ctb] : my;
    const int base = (c == 2 ? 16 : 0) + ((y & ((1 << sh) - 1)) >> 2) * gw + ((x & ((1 << sh) - 1)) >> 2);
    const uint64_t row = (1ull << nsb) - 1;
    for (int ys = 0; ys < nsb; ++ys) v.nz |= ((m >> (base + ys * gw)) & row) << (ys * nsb);
    const int16_t* groups = fd_.sb_packed + (size_t)fd_.sb_offset[ctb] * 16;
    const int skip = c ? __builtin_popcountll(my) : 0;
    for (uint64_t b = v.nz; b; b &= b - 1) {
      const int r = __builtin_ctzll(b), bit = base + (r >> (log2N - 2)) * gw + (r & (nsb - 1));
      v.sb[r] = groups + (size_t)(skip + __builtin_popcountll(m & ((1ull << bit) - 1))) * 16;
    }
  }

  void write_last_prefix(int pos, int log2N, int cIdx, int base) {
    const int prefix = kGroupIdx[pos];
    int off, shift;
    if (cIdx == 0) {
      off = 3 * (log2N - 2) + ((log2N - 1) >> 2);
      shift = (log2N + 1) >> 2;
    } else {
      off = 15;
      shift = log2N - 2;
    }
    const int cmax = (log2N << 1) - 1;
    for (int i = 0; i < prefix; ++i) bin(1, base + off + (i >> shift));
    if (prefix < cmax) bin(0, base + off + (prefix >> shift));
  }
  void write_last_suffix(int pos) {
    const int prefix = kGroupIdx[pos];
    if (prefix > 3) {
      const int nb = (prefix >> 1) - 1;
      enc_.encode_bypass_bins((uint32_t)(pos - kMinInGroup[prefix]), nb);
    }
  }

  // coeff_abs_level_remaining: TR prefix (p ones, a zero) + rice bits, or the escape
  // (4 ones, exp-Golomb order rice+1); prefixes go out as one bypass run.
  void write_remaining(int v, int rice) {
    if (v < (4 << rice)) {
      const int p = v >> rice;  // <= 3
      enc_.encode_bypass_bins(((1u << (p + 1)) - 2) << rice | (uint32_t)(v & ((1 << rice) - 1)), p + 1 + rice);
    } else {
      int k = rice + 1, ones = 0;
      uint32_t s = (uint32_t)(v - (4 << rice));
      while (s >= (1u << k)) {
        s -= 1u << k;
        ++k;
        ++ones;
      }
      // 4 + ones prefix ones, a zero, then k suffix bits (k <= 15 + ..: split the long runs)
      const int np = 4 + ones + 1;
      if (np <= 24) enc_.encode_bypass_bins((1u << np) - 2, np);
      else {
        for (int i = 0; i < 4 + ones; ++i) enc_.encode_bypass(1);
        enc_.encode_bypass(0);
      }
      enc_.encode_bypass_bins(s, k);
    }
  }

  // In-sub-block scan positions (packed x | y << 2) of scanIdx 0/1/2.
  static const uint8_t* in_sb_scan(int scanIdx) {
    return scanIdx == 0 ? kScanDiag4x4 : (scanIdx == 1 ? kScanHor4x4 : kScanVer4x4);
  }
  // sigCtx pattern (0..2) of the 16 scan positions for each prevCsbf (H.265 9.3.4.2.5),
  // precomputed per scanIdx so the per-coefficient context is one table lookup.
  struct SigPattern {
    uint8_t p[3][4][16], p4[3][16];  // p4: 4x4 TBs (ctxIdxMap of the position)
    uint16_t lo[3][256], hi[3][256];  // raster non-zero mask (bit y * 4 + x) -> scan-order mask
    SigPattern() {
      for (int sc = 0; sc < 3; ++sc) {
        int inv[16];
        for (int n = 0; n < 16; ++n) {
          p4[sc][n] = kCtxIdxMap4x4[in_sb_scan(sc)[n]];
          inv[in_sb_scan(sc)[n]] = n;
        }
        for (int v = 0; v < 256; ++v) {
          lo[sc][v] = hi[sc][v] = 0;
          for (int j = 0; j < 8; ++j)
            if ((v >> j) & 1) {
              lo[sc][v] |= (uint16_t)(1u << inv[j]);
              hi[sc][v] |= (uint16_t)(1u << inv[j + 8]);
            }
        }
      }
      for (int sc = 0; sc < 3; ++sc)
        for (int pc = 0; pc < 4; ++pc)
          for (int n = 0; n < 16; ++n) {
            const int xp = in_sb_scan(sc)[n] & 3, yp = in_sb_scan(sc)[n] >> 2;
            int v;
            if (pc == 0) v = (xp + yp == 0) ? 2 : (xp + yp < 3) ? 1 : 0;
            else if (pc == 1) v = (yp == 0) ? 2 : (yp == 1) ? 1 : 0;
            else if (pc == 2) v = (xp == 0) ? 2 : (xp == 1) ? 1 : 0;
            else v = 2;
            p[sc][pc][n] = (uint8_t)v;
          }
    }
  };

  // Sub-block scan of each TB size / scanIdx: raster index (ys * nsb + xs) of scan position
  // i, and the scan position of each raster index.
  struct SbScan {
    uint8_t pos[4][3][64], inv[4][3][64];
    SbScan() {
      for (int l = 0; l < 4; ++l)
        for (int sc = 0; sc < 3; ++sc)
          for (int i = 0; i < (1 << (2 * l)); ++i) {
            int xs, ys;
            subblock_pos(l + 2, sc, i, xs, ys);
            pos[l][sc][i] = (uint8_t)((ys << l) + xs);
            inv[l][sc][(ys << l) + xs] = (uint8_t)i;
          }
    }
  };

  void residual(const TbView& v, int log2N, int cIdx, int scanIdx) {
    static const SigPattern kPat;
    static const SbScan kSb;
    const int nsb = 1 << (log2N - 2);  // sub-blocks per side
    const uint8_t* ps = in_sb_scan(scanIdx);
    const uint8_t* sbpos = kSb.pos[log2N - 2][scanIdx];
    const uint8_t* sbinv = kSb.inv[log2N - 2][scanIdx];
    // last significant coefficient in scan order: the non-zero sub-block latest in scan
    // order, then its last non-zero scan position
    if (!v.nz) throw std::runtime_error("residual_coding of an all-zero block");
    int lastSb = 0;
    for (uint64_t b = v.nz; b; b &= b - 1) lastSb = tv_max(lastSb, (int)sbinv[__builtin_ctzll(b)]);
    auto sig_mask = [&](const int16_t* b) {  // bit n: scan position n is non-zero
      // four rows of four levels -> 16 bytes (saturating: non-zero stays non-zero) -> raster
      // mask -> scan order through two byte tables
      const size_t st = (size_t)v.stride;
      const __m128i r01 = _mm_unpacklo_epi64(_mm_loadl_epi64((const __m128i*)b),
                                             _mm_loadl_epi64((const __m128i*)(b + st)));
      const __m128i r23 = _mm_unpacklo_epi64(_mm_loadl_epi64((const __m128i*)(b + 2 * st)),
                                             _mm_loadl_epi64((const __m128i*)(b + 3 * st)));
      const __m128i z = _mm_cmpeq_epi8(_mm_packs_epi16(r01, r23), _mm_setzero_si128());
      const unsigned raster = ~(unsigned)_mm_movemask_epi8(z) & 0xffffu;
      return (unsigned)(kPat.lo[scanIdx][raster & 255] | kPat.hi[scanIdx][raster >> 8]);
    };
    const unsigned lastMask = sig_mask(v.sb[sbpos[lastSb]]);
    const int lastN = 31 - __builtin_clz(lastMask);
    {
      const int xs = sbpos[lastSb] & (nsb - 1), ys = sbpos[lastSb] >> (log2N - 2);
      int xc, yc;
      coef_pos_in_sb(scanIdx, lastN, xc, yc);
      int lx = (xs << 2) + xc, ly = (ys << 2) + yc;
      if (scanIdx == 2) std::swap(lx, ly);
      write_last_prefix(lx, log2N, cIdx, CTX_LAST_X);
      write_last_prefix(ly, log2N, cIdx, CTX_LAST_Y);
      write_last_suffix(lx);
      write_last_suffix(ly);
    }
    // context offset added to the 0..2 pattern (H.265 9.3.4.2.5), per sub-block class
    const int sizeOff = log2N == 3 ? (scanIdx == 0 ? 9 : 15) : (cIdx == 0 ? 21 : 12);
    const int compOff = CTX_SIG + (cIdx ? 27 : 0);
    uint64_t coded = 0;  // coded_sub_block_flag per raster sub-block (1 = coded / inferred)
    int c1 = 1;
    for (int i = lastSb; i >= 0; --i) {
      const int r = sbpos[i], xs = r & (nsb - 1), ys = r >> (log2N - 2);
      const bool any = (v.nz >> r) & 1;
      // csbf of the right / lower neighbours (both later in scan order, already decided)
      const int right = xs < nsb - 1 ? (int)((coded >> (r + 1)) & 1) : 0;
      const int below = ys < nsb - 1 ? (int)((coded >> (r + nsb)) & 1) : 0;
      bool inferDc = false;
      if (i < lastSb && i > 0) {
        bin(any ? 1 : 0, CTX_CSBF + (right | below) + (cIdx ? 2 : 0));
        if (!any) continue;
        inferDc = true;
      }
      coded |= 1ull << r;
      // DC sub-block: coded (inferred) even when empty
      const int16_t* b = any ? v.sb[r] : nullptr;
      const unsigned m = i == lastSb ? lastMask : (any ? sig_mask(b) : 0u);
      // significance
      const int prevCsbf = right + (below << 1);
      const uint8_t* pat = log2N == 2 ? kPat.p4[scanIdx] : kPat.p[scanIdx][prevCsbf];
      const int add = log2N == 2 ? compOff : compOff + sizeOff + ((cIdx == 0 && i > 0) ? 3 : 0);
      const int nStart = (i == lastSb) ? lastN - 1 : 15;
      const bool dcInferred = inferDc && (m & ((2u << nStart) - 2)) == 0;
      if (nStart >= 1)
        enc_.encode_run(nStart, [&](int k, int& bn, CtxState*& cs) {
          bn = (m >> (nStart - k)) & 1;
          cs = &ctx_.c[add + pat[nStart - k]];
        });
      if (nStart >= 0 && !dcInferred)  // the TB's DC has its own context
        bin(m & 1, (log2N > 2 && i == 0) ? compOff : add + pat[0]);
      // levels, in reverse scan order
      int absv[16], signs[16], cnt = 0;
      for (unsigned s = m; s; ++cnt) {
        const int n = 31 - __builtin_clz(s);
        s &= ~(1u << n);
        const int x = b[(ps[n] >> 2) * v.stride + (ps[n] & 3)];
        absv[cnt] = x < 0 ? -x : x;
        signs[cnt] = x < 0;
      }
      int ctxSet = (i > 0 && cIdx == 0) ? 2 : 0;
      if (c1 == 0) ++ctxSet;
      c1 = 1;
      const int g1base = CTX_G1 + 4 * ctxSet + (cIdx ? 16 : 0);
      const int nG1 = cnt < 8 ? cnt : 8;
      int firstG2 = -1;
      enc_.encode_run(nG1, [&](int k, int& bn, CtxState*& cs) {
        bn = absv[k] > 1;
        cs = &ctx_.c[g1base + c1];
        if (bn) {
          c1 = 0;
          if (firstG2 < 0) firstG2 = k;
        } else if (c1 > 0 && c1 < 3) {
          ++c1;
        }
      });
      if (firstG2 >= 0) bin(absv[firstG2] > 2, CTX_G2 + ctxSet + (cIdx ? 4 : 0));
      uint32_t sbits = 0;
      for (int k = 0; k < cnt; ++k) sbits = (sbits << 1) | (uint32_t)signs[k];
      enc_.encode_bypass_bins(sbits, cnt);
      int rice = 0;
      bool firstC2 = true;
      for (int k = 0; k < cnt; ++k) {
        const int base = (k < 8) ? (firstC2 ? 3 : 2) : 1;
        if (absv[k] >= base) {
          write_remaining(absv[k] - base, rice);
          if (absv[k] > 3 * (1 << rice)) rice = tv_min(rice + 1, 4);
        }
        if (absv[k] >= 2) firstC2 = false;
      }
    }
  }

  const SeqConfig& cfg_;
  const FrameData& fd_;
  bool islice_, bslice_;
  CabacEncoder enc_;
  ContextSet ctx_;
  std::vector<uint8_t> skip_;
};

}  // namespace

size_t finish_wpp_slice(BitWriter& hdr, const std::vector<BitWriter>& rows, int nal, std::vector<uint8_t>& out) {
  std::vector<const uint8_t*> p(rows.size());
  std::vector<size_t> n(rows.size());
  for (size_t r = 0; r < rows.size(); ++r) {
    p[r] = rows[r].bytes().data();
    n[r] = rows[r].bytes().size();
  }
  return finish_wpp_slice(hdr, p.data(), n.data(), (int)rows.size(), nal, out);
}

size_t finish_wpp_slice(BitWriter& hdr, const uint8_t* const* rows, const size_t* sizes, int nrows, int nal,
                        std::vector<uint8_t>& out) {
  std::vector<size_t> esc(nrows > 1 ? nrows - 1 : 0);
  size_t mx = 1;
  for (int r = 0; r + 1 < nrows; ++r) {
    esc[r] = escaped_size(rows[r], sizes[r]);
    mx = std::max(mx, esc[r]);
  }
  hdr.ue((uint32_t)esc.size());  // num_entry_point_offsets
  if (!esc.empty()) {
    int len = 1;
    while (len < 32 && ((mx - 1) >> len)) ++len;
    hdr.ue((uint32_t)(len - 1));  // offset_len_minus1
    for (size_t e : esc) hdr.put((uint32_t)(e - 1), len);
  }
  hdr.put_bit(1);  // byte_alignment()
  hdr.align_zero();
  for (int r = 0; r < nrows; ++r) hdr.put_bytes(rows[r], sizes[r]);
  const size_t before = out.size();
  append_nal(out, nal, hdr.bytes());
  return out.size() - before;
}

SliceRefs slice_refs(const CodedPic& p) {
  SliceRefs r;
  r.type = p.type;
  r.poc = p.disp;
  r.ref_poc[0] = p.ref[0];
  r.ref_poc[1] = p.ref[1];
  if ((int)p.rps.size() > kMaxRps) throw std::runtime_error("reference picture set too large");
  r.nrps = (int)p.rps.size();
  for (int i = 0; i < r.nrps; ++i) {
    r.rps_poc[i] = p.rps[i];
    r.rps_used[i] = (uint8_t)p.rps_used[i];
  }
  return r;
}

int write_slice_header(const SeqConfig& cfg, int slice_qp, const SliceRefs* r, int poc, bool idr, BitWriter& bw) {
  if (r) {
    idr = r->type == 2;
    poc = r->poc;
  }
  const int stype = r ? r->type : (idr ? 2 : 1);
  const int nal = idr ? NAL_IDR_N_LP : NAL_TRAIL_R;
  bw.put(1, 1);  // first_slice_segment_in_pic_flag
  if (idr) bw.put(0, 1);  // no_output_of_prior_pics_flag
  bw.ue(0);               // slice_pic_parameter_set_id
  bw.ue((uint32_t)stype);  // slice_type: B = 0, P = 1, I = 2
  if (!idr) {
    bw.put((uint32_t)(poc & 0xff), 8);  // slice_pic_order_cnt_lsb
    if (!r) {
      bw.put(1, 1);  // short_term_ref_pic_set_sps_flag (idx 0 implied)
    } else {  // explicit st_ref_pic_set(num_short_term_ref_pic_sets = 1)
      bw.put(0, 1);  // short_term_ref_pic_set_sps_flag
      bw.put(0, 1);  // inter_ref_pic_set_prediction_flag (stRpsIdx != 0: present)
      int neg[kMaxRps], pos[kMaxRps], un[kMaxRps], up[kMaxRps], nn = 0, np = 0;
      for (int i = 0; i < r->nrps; ++i) {
        if (r->rps_poc[i] < poc) {
          neg[nn] = r->rps_poc[i];
          un[nn++] = r->rps_used[i];
        } else {
          pos[np] = r->rps_poc[i];
          up[np++] = r->rps_used[i];
        }
      }
      // S0: decreasing POC (closest first); S1: increasing POC
      for (int i = 0; i < nn; ++i)
        for (int j = i + 1; j < nn; ++j)
          if (neg[j] > neg[i]) {
            std::swap(neg[i], neg[j]);
            std::swap(un[i], un[j]);
          }
      for (int i = 0; i < np; ++i)
        for (int j = i + 1; j < np; ++j)
          if (pos[j] < pos[i]) {
            std::swap(pos[i], pos[j]);
            std::swap(up[i], up[j]);
          }
      bw.ue((uint32_t)nn);  // num_negative_pics
      bw.ue((uint32_t)np);  // num_positive_pics
      for (int i = 0, prev = poc; i < nn; prev = neg[i++]) {
        bw.ue((uint32_t)(prev - neg[i] - 1));  // delta_poc_s0_minus1
        bw.put(un[i], 1);                      // used_by_curr_pic_s0_flag
      }
      for (int i = 0, prev = poc; i < np; prev = pos[i++]) {
        bw.ue((uint32_t)(pos[i] - prev - 1));  // delta_poc_s1_minus1
        bw.put(up[i], 1);                      // used_by_curr_pic_s1_flag
      }
    }
  }
  if (cfg.sao) {
    bw.put(1, 1);  // slice_sao_luma_flag
    bw.put(1, 1);  // slice_sao_chroma_flag
  }
  if (!idr) {
    bw.put(0, 1);  // num_ref_idx_active_override_flag (one picture per list)
    if (stype == 0) bw.put(0, 1);  // mvd_l1_zero_flag
    bw.ue((uint32_t)(5 - cfg.max_merge_cand));  // five_minus_max_num_merge_cand
  }
  bw.se(slice_qp >= 0 ? slice_qp - cfg.qp : 0);  // slice_qp_delta (per-frame rate control)
  return nal;
}

size_t write_slice(const SeqConfig& cfg, const FrameData& fd, int poc, bool idr,
                   std::vector<uint8_t>& out) {
  BitWriter bw;
  const int nal = write_slice_header(cfg, fd.qp, fd.refs, poc, idr, bw);
  if (fd.refs) idr = fd.refs->type == 2;
  if (!cfg.wpp) {
    // byte_alignment()
    bw.put_bit(1);
    bw.align_zero();
    SliceWriter sw(cfg, fd, idr, &bw);
    sw.write_all();
    bw.trailing_bits();
    const size_t before = out.size();
    append_nal(out, nal, bw.bytes());
    return out.size() - before;
  }
  // WPP: the CTB rows are coded first (one substream each), then the header can carry their
  // entry points (sizes after emulation prevention, which each substream's own bytes fix)
  const int hc = cfg.coded_h >> kCtbLog2;
  std::vector<BitWriter> rows(hc);
  {
    SliceWriter sw(cfg, fd, idr, &rows[0]);
    sw.write_all(&rows);
  }
  rows[hc - 1].trailing_bits();  // rbsp_slice_segment_trailing_bits
  return finish_wpp_slice(bw, rows, nal, out);
}

}  // namespace tv

// ------------------------------------------------------------------ table export --------
// Every H.265 table the encoder (and its decoder oracle) codes with, exported by name for
// tests/test_hevc_spec_tables.py, which diffs them against an independently transcribed copy
// that shares no header with csrc/.  Returns the number of values (written to out when cap
// allows), -1 for an unknown name.  "ctx:<element>" = the element's init values, initType 0
// (I), 1 (P), 2 (B) concatenated, as the spec's ctxIdx tables list them.
namespace {
struct CtxRange {
  const char* name;
  int off, n;
};
constexpr CtxRange kCtxRanges[] = {
    {"sao_merge_flag", tv::CTX_SAO_MERGE, 1},        {"sao_type_idx", tv::CTX_SAO_TYPE, 1},
    {"split_cu_flag", tv::CTX_SPLIT_CU, 3},          {"cu_transquant_bypass_flag", tv::CTX_TQ_BYPASS, 1},
    {"cu_skip_flag", tv::CTX_CU_SKIP, 3},            {"pred_mode_flag", tv::CTX_PRED_MODE, 1},
    {"part_mode", tv::CTX_PART_MODE, 1},             {"prev_intra_luma_pred_flag", tv::CTX_PREV_INTRA, 1},
    {"intra_chroma_pred_mode", tv::CTX_CHROMA_PRED, 1}, {"rqt_root_cbf", tv::CTX_RQT_ROOT_CBF, 1},
    {"merge_flag", tv::CTX_MERGE_FLAG, 1},           {"merge_idx", tv::CTX_MERGE_IDX, 1},
    {"inter_pred_idc", tv::CTX_INTER_PRED_IDC, 5},   {"ref_idx", tv::CTX_REF_IDX, 2},
    {"mvp_flag", tv::CTX_MVP_FLAG, 1},               {"split_transform_flag", tv::CTX_SPLIT_TF, 3},
    {"cbf_luma", tv::CTX_CBF_LUMA, 2},               {"cbf_chroma", tv::CTX_CBF_CHROMA, 4},
    {"abs_mvd_greater0_flag", tv::CTX_MVD_G0, 1},    {"abs_mvd_greater1_flag", tv::CTX_MVD_G1, 1},
    {"cu_qp_delta_abs", tv::CTX_CU_QP_DELTA, 2},     {"transform_skip_flag", tv::CTX_TRANSFORM_SKIP, 2},
    {"last_sig_coeff_x_prefix", tv::CTX_LAST_X, 18}, {"last_sig_coeff_y_prefix", tv::CTX_LAST_Y, 18},
    {"coded_sub_block_flag", tv::CTX_CSBF, 4},       {"sig_coeff_flag", tv::CTX_SIG, 44},
    {"coeff_abs_level_greater1_flag", tv::CTX_G1, 24}, {"coeff_abs_level_greater2_flag", tv::CTX_G2, 6},
};
}  // namespace

extern "C" int tv_hevc_spec_table(const char* name, int* out, int cap) {
  using namespace tv;
  std::vector<int> v;
  const std::string s(name ? name : "");
  auto put = [&](const auto* a, int n) {
    for (int i = 0; i < n; ++i) v.push_back((int)a[i]);
  };
  if (s.rfind("ctx:", 0) == 0) {
    bool found = false;
    for (const auto& r : kCtxRanges)
      if (s.compare(4, std::string::npos, r.name) == 0) {
        for (int t = 0; t < 3; ++t)
          for (int i = 0; i < r.n; ++i) v.push_back(ctx_init_table().v[t][r.off + i]);
        found = true;
      }
    if (!found) return -1;
  } else if (s == "range_tab_lps") {
    put(&kRangeTabLps[0][0], 256);
  } else if (s == "trans_idx_lps") {
    put(kTransIdxLps, 64);
  } else if (s == "trans_idx_mps") {
    put(kTransIdxMps, 64);
  } else if (s == "ctx_idx_map") {
    put(kCtxIdxMap4x4, 16);
  } else if (s == "group_idx") {
    put(kGroupIdx, 32);
  } else if (s == "min_in_group") {
    put(kMinInGroup, 10);
  } else if (s == "dct32") {
    put(&kDct32.m[0][0], 1024);
  } else if (s == "level_scale") {
    for (int q = 0; q < 6; ++q) v.push_back(level_scale(q));
  } else if (s == "beta") {
    put(kBetaTable, 52);
  } else if (s == "tc") {
    put(kTcTable, 54);
  } else if (s == "chroma_qp") {  // QpC of qPi = 0..57 (4:2:0)
    for (int q = 0; q <= 57; ++q) v.push_back(chroma_qp(q, 0));
  } else if (s == "intra_pred_angle") {
    put(kIntraPredAngle, 35);
  } else if (s == "inv_angle") {
    put(kInvAngle, 15);
  } else if (s == "intra_filter") {  // filterFlag of (log2 size 2..5, mode 0..34)
    for (int l = 2; l <= 5; ++l)
      for (int m = 0; m < 35; ++m) v.push_back(intra_filter_refs(l, m) ? 1 : 0);
  } else if (s == "luma_filter") {
    put(&kLumaFilter[0][0], 32);
  } else if (s == "chroma_filter") {
    put(&kChromaFilter[0][0], 32);
  } else if (s == "scan_diag4x4") {
    put(kScanDiag4x4, 16);
  } else if (s == "scan_hor4x4") {
    put(kScanHor4x4, 16);
  } else if (s == "scan_ver4x4") {
    put(kScanVer4x4, 16);
  } else if (s == "scan_diag8x8") {
    put(kScanDiag8x8.s, 64);
  } else if (s == "scan_idx") {  // scanIdx of (log2 size 2..3, mode 0..34), intra luma
    for (int l = 2; l <= 3; ++l)
      for (int m = 0; m < 35; ++m) v.push_back(scan_idx_for(true, l, 0, m));
  } else {
    return -1;
  }
  for (int i = 0; i < (int)v.size() && i < cap; ++i) out[i] = v[i];
  return (int)v.size();
}
