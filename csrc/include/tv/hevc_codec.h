// hevc_codec.h — host-side HEVC codec API: sequence configuration, the per-frame
// "decision" layout produced by the analysis stage (GPU kernels or the CPU reference
// encoder), the CABAC syntax writer, the decoder oracle and picture reconstruction helpers.
//
// Decision layout (all arrays indexed by 8x8 unit u = y8 * w8 + x8 of the coded picture;
// every unit of a CU carries the CU's values, so neighbour lookups are O(1)):
//   cu_log2[u]  log2 size of the covering CU (3..5)
//   intra[u]    1 = MODE_INTRA, 0 = MODE_INTER
//   ipm[u]      luma intra prediction mode (intra CUs)
//   mv[2u+0/1]  quarter-pel motion vector (inter CUs; list-0 reference)
//   dir[u]      B slices only: 1 = list 0, 2 = list 1, 3 = bi-prediction (P slices: 1)
//   mv1[2u+..]  B slices only: the list-1 motion vector
//   cbf[u]      bit0 = cbf_luma, bit1 = cbf_cb, bit2 = cbf_cr
//   coef[c]     quantised levels, each TB stored at its picture position (int16 planes,
//               luma stride = coded_w, chroma stride = coded_w/2)
#pragma once
#include <cstdint>
#include <cstdlib>
#include <string>
#include <vector>

#include "gop.h"
#include "hevc_defs.h"
#include "hevc_mvpred.h"

namespace tv {

struct SeqConfig {
  int width = 0, height = 0;      // display size (conformance window)
  int coded_w = 0, coded_h = 0;   // multiples of the CTB size
  int qp = 27;
  int max_merge_cand = 5;
  int crf = 0;  // > 0: per-frame QP from the lookahead complexity (tv/rc_model.h)
  bool deblock = true;
  bool sao = false;
  // wavefront parallel processing (entropy_coding_sync_enabled_flag): one CABAC substream per
  // CTB row, contexts synced from the row above after its second CTB, entry points in the
  // slice header -- the rows can be entropy-coded in parallel (the GPU CABAC path)
  bool wpp = false;
  // hierarchical-B coding structure (tv/gop.h): mini-GOP size (1 = I P P P ...), and the
  // DPB size / reorder depth the parameter sets announce for it
  int mgop = 1;
  int dpb_size = 2, num_reorder = 0;
  // intra 16x16 CUs in P pictures (tv/me_model.h, pintra_*)
  bool pintra = true;
  // residual quadtree: inter 32x32 CUs of P pictures may code four 16x16 TBs
  // (max_transform_hierarchy_depth_inter 1; hevc_defs.h rqt_split)
  bool rqt = true;
  // constant-QP I P P P: the low-delay QP cascade of tv/gop.h ippp_qp_offset
  bool cascade = false;
  // RDOQ-lite: inter TBs drop trailing lone-+-1 coefficient groups (hevc_defs.h kRdoqMode)
  bool rdoq = true;
  // All of these change the bitstream: they are explicit configuration (the C API's flag bits 3 / 4,
  // EncodeSpec.rqt / .pintra, part of the engine key and the checkpoint fingerprint), never
  // read from the environment here.
  // Flag bits of the C API's `deblock` argument: 1 deblocking, 2 SAO, 4 WPP, 8 no RQT,
  // 16 no intra-in-P (32: GPU engine only, CABAC on the host), 64 I P P P QP cascade,
  // 128 no RDOQ-lite
  void set_flags(int f) {
    deblock = (f & 1) != 0;
    sao = (f & 2) != 0;
    wpp = (f & 4) != 0;
    rqt = !(f & 8);
    pintra = !(f & 16);
    cascade = (f & 64) != 0;
    rdoq = !(f & 128);
  }
  int fps_num = 30, fps_den = 1;
  void finalize() {
    coded_w = (width + kCtb - 1) / kCtb * kCtb;
    coded_h = (height + kCtb - 1) / kCtb * kCtb;
  }
  int w8() const { return coded_w >> 3; }
  int h8() const { return coded_h >> 3; }
  int level_idc() const;
};

// Coding-structure part of a slice header (hierarchical-B streams, tv/gop.h): slice type,
// POC, the list-0 / list-1 reference POCs and the explicit reference picture set.
constexpr int kMaxRps = 16;
struct SliceRefs {
  int type = 2;                  // 2 = I, 1 = P, 0 = B
  int poc = 0;
  int ref_poc[2] = {-1, -1};
  int nrps = 0;
  int rps_poc[kMaxRps] = {};
  uint8_t rps_used[kMaxRps] = {};
};
SliceRefs slice_refs(const CodedPic& p);

struct FrameData {
  int w8 = 0, h8 = 0;
  const uint8_t* cu_log2 = nullptr;
  const uint8_t* intra = nullptr;
  const uint8_t* ipm = nullptr;
  const int16_t* mv = nullptr;
  const uint8_t* cbf = nullptr;
  const int16_t* coef[3] = {nullptr, nullptr, nullptr};
  // compact levels (GPU path; used when sb_packed != nullptr): per-CTB masks of non-zero
  // 4x4 groups (luma bit = sy*8+sx; chroma Cb bits 0..15 / Cr 16..31), exclusive group
  // offsets, and 16 levels per group packed in CTB order (Y, Cb, Cr raster).
  const uint64_t* sb_mask_y = nullptr;
  const uint32_t* sb_mask_c = nullptr;
  const int32_t* sb_offset = nullptr;
  const int16_t* sb_packed = nullptr;
  int wc = 0;  // CTBs per row
  // SAO parameters, 3 packed words (Y, Cb, Cr) per CTB in raster order (nullptr: SAO off)
  const uint32_t* sao = nullptr;
  int qp = -1;  // slice QP (rate control); -1: the sequence QP (PPS init_qp)
  // hierarchical-B streams: the slice's coding structure (nullptr: IPPP, SPS RPS 0) and, for
  // B slices, per-unit prediction direction and list-1 vectors
  const SliceRefs* refs = nullptr;
  const uint8_t* dir = nullptr;
  const int16_t* mv1 = nullptr;
  // 1: the unit's inter 32x32 CU codes four 16x16 TBs (RQT split); cbf[u] is then the cbf of
  // the unit's 16x16 TB (nullptr: no splits)
  const uint8_t* tu = nullptr;
};

// Owning storage for one frame's decisions (CPU side).
struct FrameDecisions {
  int w8 = 0, h8 = 0, cw = 0, ch = 0;
  std::vector<uint8_t> cu_log2, intra, ipm, cbf, tu;
  std::vector<int16_t> mv, coef_y, coef_u, coef_v;
  std::vector<uint32_t> sao;  // 3 per CTB
  int qp = -1;                // slice QP of this frame (-1: sequence QP)
  std::vector<uint8_t> dir;   // B slices (see FrameData)
  std::vector<int16_t> mv1;
  SliceRefs refs;
  bool has_refs = false;      // refs describe this slice (hierarchical-B stream)
  void alloc(int coded_w, int coded_h) {
    has_refs = false;
    sao.assign(3 * (size_t)(coded_w >> kCtbLog2) * (coded_h >> kCtbLog2), sao_off_param());
    qp = -1;
    cw = coded_w;
    ch = coded_h;
    w8 = coded_w >> 3;
    h8 = coded_h >> 3;
    const size_t n = (size_t)w8 * h8;
    cu_log2.assign(n, 3);
    intra.assign(n, 0);
    ipm.assign(n, 1);
    cbf.assign(n, 0);
    tu.assign(n, 0);
    mv.assign(2 * n, 0);
    dir.assign(n, 1);
    mv1.assign(2 * n, 0);
    coef_y.assign((size_t)coded_w * coded_h, 0);
    coef_u.assign((size_t)coded_w * coded_h / 4, 0);
    coef_v.assign((size_t)coded_w * coded_h / 4, 0);
  }
  FrameData view() const {
    FrameData f;
    f.w8 = w8;
    f.h8 = h8;
    f.cu_log2 = cu_log2.data();
    f.intra = intra.data();
    f.ipm = ipm.data();
    f.mv = mv.data();
    f.cbf = cbf.data();
    f.tu = tu.data();
    f.coef[0] = coef_y.data();
    f.coef[1] = coef_u.data();
    f.coef[2] = coef_v.data();
    f.sao = sao.data();
    f.wc = cw >> kCtbLog2;
    f.qp = qp;
    if (has_refs) {
      f.refs = &refs;
      if (refs.type == 0) {
        f.dir = dir.data();
        f.mv1 = mv1.data();
      }
    }
    return f;
  }
};

// A planar 8-bit 4:2:0 picture buffer
struct Picture {
  int w = 0, h = 0;  // luma size
  std::vector<uint8_t> y, u, v;
  void alloc(int W, int H) {
    w = W;
    h = H;
    y.assign((size_t)W * H, 0);
    u.assign((size_t)W * H / 4, 128);
    v.assign((size_t)W * H / 4, 128);
  }
  uint8_t* plane(int c) { return c == 0 ? y.data() : (c == 1 ? u.data() : v.data()); }
  const uint8_t* plane(int c) const { return c == 0 ? y.data() : (c == 1 ? u.data() : v.data()); }
  int pw(int c) const { return c ? w / 2 : w; }
  int ph(int c) const { return c ? h / 2 : h; }
};

// ----------------------------- bitstream generation -------------------------------------
void write_parameter_sets(const SeqConfig& cfg, std::vector<uint8_t>& out);
class BitWriter;
// WPP slice assembly: `hdr` holds the slice header up to slice_qp_delta; appends the entry
// points of the row substreams, byte_alignment(), the substreams (the last one already ends
// in rbsp_slice_segment_trailing_bits) and emits the NAL.  Returns bytes appended.
size_t finish_wpp_slice(BitWriter& hdr, const uint8_t* const* rows, const size_t* sizes, int nrows, int nal,
                        std::vector<uint8_t>& out);
// Slice segment header up to slice_qp_delta (`r`: the hierarchical-B coding structure, or
// nullptr for I P P P); returns the NAL unit type.  slice_qp < 0: the sequence QP.
int write_slice_header(const SeqConfig& cfg, int slice_qp, const SliceRefs* r, int poc, bool idr, BitWriter& bw);
// Encode one picture as a single slice NAL; returns bytes appended.
size_t write_slice(const SeqConfig& cfg, const FrameData& fd, int poc, bool idr,
                   std::vector<uint8_t>& out);

// ------------------------------ reconstruction helpers ----------------------------------
// Intra prediction of a TB in component cIdx at component position (x,y).
void predict_intra_tb(const Picture& rec, int cIdx, int x, int y, int log2N, int mode, int* pred);
// Inter prediction (uni, L0) of a w x h block of component cIdx at component position (x,y).
void predict_inter_block(const Picture& ref, int cIdx, int x, int y, int w, int h, int mvx,
                         int mvy, int* pred);
// Bi-prediction (8.5.3.3.4.2): both lists' 14-bit intermediate samples, (p0 + p1 + 64) >> 7.
void predict_bi_block(const Picture& ref0, const Picture& ref1, int cIdx, int x, int y, int w, int h,
                      const int16_t* mv0, const int16_t* mv1, int* pred);
// Dequantise + inverse transform the levels of a TB (plane stride `ls`) and add to `pred`,
// writing the clipped reconstruction into `dst` (stride ds).  cbf=false -> copy pred.
void recon_tb(const int16_t* levels, int ls, bool cbf, int log2N, int qp, const int* pred,
              uint8_t* dst, int ds);
// In-loop deblocking of a reconstructed picture given the frame decisions (B slices: the
// boundary strength compares prediction directions and both lists' vectors).
void deblock_picture(Picture& pic, const FrameData& fd, int qp);
// SAO statistics of CTB (cx, cy), component c: source vs deblocked picture.
void sao_ctb_stats(const Picture& src, const Picture& deb, int c, int cx, int cy, SaoStats& st);
// Encoder: decide per-CTB SAO parameters (3 per CTB) for a deblocked picture.
void sao_decide_picture(const Picture& src, const Picture& deb, int qp, uint32_t* params);
// Apply SAO in place (uses an internal copy of the deblocked samples).
void sao_picture(Picture& pic, const uint32_t* params);

// derived chroma intra mode for intra_chroma_pred_mode idx (4 = DM)
inline int chroma_intra_mode(int chroma_idx, int luma_mode) {
  if (chroma_idx == 4) return luma_mode;
  static const int m[4] = {0, 26, 10, 1};
  return m[chroma_idx] == luma_mode ? 34 : m[chroma_idx];
}

// ------------------------------------- decoder ------------------------------------------
struct DecodedPicture {
  int poc = 0;
  bool idr = false;
  Picture pic;  // coded size (includes padding rows/cols)
};

class HevcDecoder {
 public:
  // Decode a complete Annex-B elementary stream.  Throws std::runtime_error on syntax
  // violations of the supported subset.
  void decode(const uint8_t* data, size_t n);
  // Decode only pictures [first, first + count) (decode order == output order here): parsing
  // starts at the last IDR at or before `first`, earlier pictures are skipped without
  // decoding and only the requested ones are kept (random access into a long stream).
  void decode_range(const uint8_t* data, size_t n, int first, int count);
  std::vector<DecodedPicture> pictures;
  int width = 0, height = 0;          // conformance-cropped size
  int coded_w = 0, coded_h = 0;
  // decisions parsed from the last decoded picture (for tests)
  FrameDecisions last_decisions;

 private:
  struct Impl;
};

// Header-only probe of an Annex-B stream: SPS geometry and the picture count (one slice
// per picture), no slice data decoded.
struct StreamInfo {
  int width = 0, height = 0, coded_w = 0, coded_h = 0, pictures = 0, idrs = 0;
};
StreamInfo probe_annexb(const uint8_t* data, size_t n);
// Composition offset of every picture (decoding order): display index - decoding index,
// from the slice headers' POCs ranked within each coded video sequence (0 everywhere for
// I P P P streams; hierarchical-B streams reorder).  Used by the MP4 / Matroska muxers.
std::vector<int> display_offsets(const uint8_t* data, size_t n);

// ------------------------------------- containers ---------------------------------------
// Build an ISO-BMFF (.mp4, 'hvc1') file from an Annex-B HEVC stream.  Returns bytes.
std::vector<uint8_t> mux_mp4(const uint8_t* annexb, size_t n, int width, int height,
                             int fps_num, int fps_den);
// Stream the concatenation of Annex-B segments straight into a faststart MP4 file (the
// sample tables come from a scan of the segments; payload is written once, never copied
// into one big buffer).  Returns the file size.
uint64_t mux_mp4_file(const uint8_t* const* segs, const size_t* sizes, int nseg, int width, int height, int fps_num,
                      int fps_den, const char* path);
// Parse an mp4 produced by mux_mp4 back to Annex-B (probe / round trip).
std::vector<uint8_t> demux_mp4(const uint8_t* mp4, size_t n, int* width, int* height,
                               int* nframes, int* timescale, int* sample_delta);

}  // namespace tv
