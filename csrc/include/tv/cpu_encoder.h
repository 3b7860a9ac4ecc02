// cpu_encoder.h — scalar reference encoder API (software path / golden model).
#pragma once
#include <vector>

#include "hevc_codec.h"

namespace tv {

double lambda_sad(int qp);
// Copy a display-size 4:2:0 frame into a coded-size picture with edge replication.
void pad_source(const uint8_t* const planes[3], const int strides[3], int width, int height,
                Picture& dst);
void analyze_intra(const SeqConfig& cfg, const Picture& src, FrameDecisions& fd);
// Hierarchical motion search (tv/me_model.h): quarter-res luma of a source picture, the
// per-CTB coarse field of qcur vs qprev, and the full-res refinement + CU split decision.
void quarter_luma(const Picture& src, std::vector<uint8_t>& q);
void coarse_search(const uint8_t* qcur, const uint8_t* qprev, int W, int H, int range, const int* penmv,
                   int16_t* cmv, int* ccost);
void analyze_inter(const SeqConfig& cfg, const Picture& src, const Picture& ref, const int16_t* cmv,
                   const int16_t* prev_mv, int range, FrameDecisions& fd);
// intra quadrants of a P picture: cand = [hc][wc][4] candidate bytes (tv/me_model.h pintra_*)
void apply_pintra(const uint8_t* cand, int wc, int hc, FrameDecisions& fd);
// B pictures (tv/gop.h): both lists' searches, then per block the best of list 0, list 1
// and their 8-bit average (bi-prediction), then the same CU split.
void analyze_inter_b(const SeqConfig& cfg, const Picture& src, const Picture& ref0, const Picture& ref1,
                     const int16_t* cmv0, const int16_t* cmv1, const int16_t* prev_mv, const int* range,
                     FrameDecisions& fd);
// Pass B: prediction + transform/quant + reconstruction (+ deblocking) from decisions
// (ref1 != nullptr: a B picture, fd.dir / fd.mv1 select the lists).
void reconstruct_frame(const SeqConfig& cfg, const Picture& src, const Picture* ref,
                       FrameDecisions& fd, Picture& rec, const Picture* ref1 = nullptr);

class CpuEncoder {
 public:
  explicit CpuEncoder(const SeqConfig& cfg, int search_range = 64);
  // Appends VPS/SPS/PPS (for IDR) and one slice NAL to `out`.  qp >= 0: this frame's slice
  // QP (rate control), else the sequence QP.
  void encode_frame(const uint8_t* const planes[3], const int strides[3], bool idr, int poc,
                    std::vector<uint8_t>& out, int qp = -1);
  // Hierarchical-B streams (cfg.mgop > 1): plan the next segment of `nframes` frames; the
  // frames are then passed in the plan's coding order (display index = plan().pics[k].disp),
  // each call coding the next picture of the plan (`idr` / `poc` are taken from the plan).
  void begin_gop(int nframes);
  const GopPlan& plan() const { return plan_; }
  const Picture& recon() const { return rec_; }
  const SeqConfig& config() const { return cfg_; }
  FrameDecisions dec;

 private:
  SeqConfig cfg_;
  int range_;
  Picture src_, rec_, ref_;
  std::vector<uint8_t> qcur_, qprev_;  // quarter-res source luma (current / previous frame)
  std::vector<int16_t> prev_mv_;       // previous frame's MV field (temporal candidate)
  // hierarchical-B state: the segment plan, the next coded picture, and the DPB (display
  // index -> reconstruction + quarter-res source luma of the reference pictures)
  GopPlan plan_;
  int next_ = 0;
  struct DpbEntry {
    int disp;
    Picture rec;
    std::vector<uint8_t> q;
  };
  std::vector<DpbEntry> dpb_;
  void encode_b_structured(std::vector<uint8_t>& out, int qp);
};

}  // namespace tv
