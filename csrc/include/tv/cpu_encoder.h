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
void analyze_inter(const SeqConfig& cfg, const Picture& src, const Picture& ref, int range,
                   FrameDecisions& fd);
// Pass B: prediction + transform/quant + reconstruction (+ deblocking) from decisions.
void reconstruct_frame(const SeqConfig& cfg, const Picture& src, const Picture* ref,
                       FrameDecisions& fd, Picture& rec);

class CpuEncoder {
 public:
  explicit CpuEncoder(const SeqConfig& cfg, int search_range = 8);
  // Appends VPS/SPS/PPS (for IDR) and one slice NAL to `out`.
  void encode_frame(const uint8_t* const planes[3], const int strides[3], bool idr, int poc,
                    std::vector<uint8_t>& out);
  const Picture& recon() const { return rec_; }
  const SeqConfig& config() const { return cfg_; }
  FrameDecisions dec;

 private:
  SeqConfig cfg_;
  int range_;
  Picture src_, rec_, ref_;
};

}  // namespace tv
