// mpeg2.h — MPEG-2 video (ISO/IEC 13818-2, Main Profile @ Main Level, 4:2:0): the decoder
// that makes DVD titles (MakeMKV remuxes with `-c copy`, /root/reference/rips/dvd_rip_queue.py:
// 1649-1668) transcodable, and an independent stream writer that produces the test fixtures.
//
// Decoder: frame and field pictures; I / P / B; frame, field and 16x8 motion compensation,
// frame / field DCT, skipped macroblocks, both coefficient tables, alternate scan, linear and
// non-linear quantiser scale, loaded quantiser matrices, open / closed GOPs with random access
// at I pictures.  Dual-prime prediction is refused (DVD encoders do not emit it).
// The inverse DCT is the separable double-precision definition of 13818-2 Annex A rounded to
// nearest (IEEE 1180 conformant); other conformant decoders may differ by +-1 on some samples.
//
// Writer: a deliberately simple encoder (small motion search, seeded mode choices that visit
// every macroblock type / motion type / DCT type / skip rule the decoder handles).  Its
// reconstruction is the decoder's specification in the tests.
#pragma once
#include <cstddef>
#include <cstdint>
#include <functional>
#include <memory>
#include <vector>

namespace tv::mpeg2 {

struct SeqHeader {
  int width = 0, height = 0;  // horizontal / vertical_size
  int aspect = 0, frame_rate_code = 0, bit_rate = 0, vbv = 0;
  int progressive_seq = 1, chroma_format = 1, profile_level = 0, low_delay = 0;
  int fr_ext_n = 0, fr_ext_d = 0;
  bool mpeg2 = false;                 // a sequence_extension followed
  uint8_t intra_q[64], inter_q[64];   // raster order
  uint8_t cintra_q[64], cinter_q[64]; // chroma (4:2:0: equal to the luma ones unless loaded)
  SeqHeader();
  int mb_width() const { return (width + 15) / 16; }
  int mb_height() const { return progressive_seq ? (height + 15) / 16 : 2 * ((height + 31) / 32); }
  void fps(int& num, int& den) const;
};

// a frame buffer at the coded size (multiples of 16 / 32), planes back to back
struct Image {
  int w = 0, h = 0;  // coded luma size
  std::vector<uint8_t> y, u, v;
  void alloc(int cw, int ch);
};

// random-access points: I pictures (with the headers before them)
struct Rap {
  size_t offset = 0;      // first byte to decode from (sequence / GOP header or the picture)
  size_t seq_offset = 0;  // the sequence header in force
  int frames_before = 0;  // frames before this picture in decoding order
  bool closed = true;     // no leading B pictures reference the previous GOP
};

struct StreamIndex {
  SeqHeader seq;
  int frames = 0;           // frame pictures + field-picture pairs
  bool interlaced = false;  // some frame is coded interlaced (progressive_frame == 0)
  int top_field_first = 1;  // of the first interlaced frame
  bool field_pictures = false;
  std::vector<Rap> raps;
};

StreamIndex index_stream(const uint8_t* d, size_t n);

constexpr int kNumStats = 18;
extern const char* const kStatNames[kNumStats];

class Decoder {
 public:
  // frames in display order, numbered from `base`; returning false stops the decode
  using Sink = std::function<bool(int display_index, const Image& frame)>;
  Decoder();
  ~Decoder();
  // decode d[start, n) after parsing the sequence header at seq_off (which may be == start)
  void decode(const uint8_t* d, size_t n, size_t seq_off, size_t start, int base, const Sink& sink);
  // syntax-element counters of every decode so far (kStatNames)
  const int64_t* stats() const;

 private:
  struct Impl;
  std::unique_ptr<Impl> p_;
};

struct EncConfig {
  int width = 0, height = 0;  // multiples of 16 (32 when interlaced)
  int frame_rate_code = 4;    // 30000/1001
  int gop = 12;               // I-picture distance
  int bframes = 2;            // B pictures between references
  int qscale_code = 6;
  bool interlaced = false;     // progressive_sequence 0: field / frame motion + DCT type per MB
  bool field_pictures = false; // code each frame as two field pictures (I frames: I + P field)
  bool top_field_first = true;
  bool alternate_scan = false, intra_vlc = false, q_scale_type = false;
  int intra_dc_precision = 0;  // 0..2 (8..10 bits)
  bool custom_matrices = false;
  bool closed_gop = true;
  bool vary_quant = false;     // macroblock_quant changes
  int slices_per_row = 1;
  int f_code = 2;
  int search = 6;              // full-pel search radius
  uint32_t seed = 1;           // exercise choices
};

// display-order I420 frames at width x height -> elementary stream; units[k] = the bytes of the
// k-th frame in decoding order (headers before it included), unit_display[k] its display index;
// recon = the reconstruction in display order (the decoder's expected output)
std::vector<uint8_t> encode(const EncConfig& cfg, const std::vector<const uint8_t*>& frames,
                            std::vector<size_t>* units, std::vector<int>* unit_display, std::vector<Image>* recon);

}  // namespace tv::mpeg2
