// mux_internal.h — pieces shared by the MP4 (mp4.cpp) and Matroska (mkv.cpp) writers.
#pragma once

#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "tv/bitstream.h"
#include "tv/container.h"
#include "tv/hevc_codec.h"

namespace tv {
namespace muxi {

// One video sample = references to its NAL units (in-band parameter sets first when they
// change between segments) — the payload is never copied until it is written.
struct Sample {
  std::vector<NalView> nals;
  uint32_t size = 0;  // length-prefixed bytes (HEVC) / raw OBU bytes (AV1)
  bool sync = false;
  bool raw = false;   // AV1: the single view is the temporal unit's OBUs, written as is
  int cto = 0;        // composition offset in frames: display index - decoding index (B frames)
};

enum MuxCodec : int { MUX_HEVC = 0, MUX_AV1 = 1 };

struct MuxPlan {
  int codec = MUX_HEVC;
  std::vector<uint8_t> vps, sps, pps;
  std::vector<uint8_t> av1c;  // AV1CodecConfigurationRecord (AV1 only)
  bool ps_consistent = true;
  std::vector<Sample> samples;
  uint64_t mdat_payload = 0;
  bool reordered = false;  // some sample has cto != 0 (ctts + edit list / Matroska PTS)
};

// Scan the segments (in order) into samples; no payload bytes are copied.  Annex-B HEVC,
// or AV1 low-overhead OBU streams (detected by a leading temporal delimiter OBU): one
// sample per temporal unit without its temporal delimiter (AV1-ISOBMFF 2.4), the first
// sequence header OBU copied into the av1C record.
MuxPlan plan_mux(const uint8_t* const* segs, const size_t* sizes, int nseg);
bool is_av1_stream(const uint8_t* p, size_t n);

// HEVCDecoderConfigurationRecord (ISO/IEC 14496-15 8.3.3.1) from the parameter sets; the
// payload of MP4's 'hvcC' box and Matroska's V_MPEGH/ISO/HEVC CodecPrivate.
std::vector<uint8_t> hvcc_record(const MuxPlan& P);

inline void put_be32(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24);
  p[1] = (uint8_t)(v >> 16);
  p[2] = (uint8_t)(v >> 8);
  p[3] = (uint8_t)v;
}

// Append video sample `s` (4-byte length-prefixed NAL units) to `out`.
inline void append_sample(const Sample& s, std::vector<uint8_t>& out) {
  if (s.raw) {
    for (const auto& v : s.nals) out.insert(out.end(), v.data, v.data + v.size);
    return;
  }
  for (const auto& nal : s.nals) {
    uint8_t len[4];
    put_be32(len, (uint32_t)nal.size);
    out.insert(out.end(), len, len + 4);
    out.insert(out.end(), nal.data, nal.data + nal.size);
  }
}

// Reads side-stream sample payloads from the source file (by offset) or from memory.
class SideReader {
 public:
  explicit SideReader(const SideTrack& t) : t_(t) {
    if (t.path && t.path[0]) {
      f_ = std::fopen(t.path, "rb");
      if (!f_) throw std::runtime_error(std::string("mux: cannot open side-stream source ") + t.path);
    } else if (t.nsamples > 0 && !t.data) {
      throw std::runtime_error("mux: side stream without payload");
    }
  }
  ~SideReader() {
    if (f_) std::fclose(f_);
  }
  SideReader(const SideReader&) = delete;
  SideReader& operator=(const SideReader&) = delete;
  void append(int64_t i, std::vector<uint8_t>& out) {
    const size_t n = t_.sizes[i], o = out.size();
    out.resize(o + n);
    if (f_) {
      if (fseeko(f_, (off_t)t_.offsets[i], SEEK_SET) != 0 || std::fread(out.data() + o, 1, n, f_) != n)
        throw std::runtime_error("mux: short read of a side-stream sample");
    } else {
      std::memcpy(out.data() + o, t_.data + t_.offsets[i], n);
    }
  }

 private:
  const SideTrack& t_;
  FILE* f_ = nullptr;
};

// Validates a side track's tables before any of it is dereferenced.
inline void check_side(const SideTrack& t, bool mkv) {
  if (t.kind != SIDE_AUDIO && t.kind != SIDE_SUBTITLE) throw std::runtime_error("mux: bad side-stream kind");
  if (t.timescale <= 0) throw std::runtime_error("mux: side stream without a timescale");
  if (t.nsamples < 0 || (t.nsamples > 0 && (!t.offsets || !t.sizes || !t.pts || !t.durs)))
    throw std::runtime_error("mux: side stream without sample tables");
  if (t.codec == SIDE_OPAQUE && !mkv) throw std::runtime_error("mux: opaque side streams need Matroska");
  if (t.codec == SIDE_OPAQUE && !(t.mkv_codec_id && t.mkv_codec_id[0]))
    throw std::runtime_error("mux: opaque side stream without a codec id");
  if (t.codec == SIDE_MP4_ENTRY && (mkv || t.priv_size < 8))
    throw std::runtime_error("mux: MP4 sample-entry passthrough needs MP4 and an entry");
  if (t.codec == SIDE_PCM_S16LE && t.channels <= 0) throw std::runtime_error("mux: PCM without channels");
  if (t.codec < SIDE_AAC || t.codec > SIDE_MP4_ENTRY) throw std::runtime_error("mux: unknown side-stream codec");
  if (t.kind == SIDE_SUBTITLE && t.codec != SIDE_SUBRIP && t.codec != SIDE_OPAQUE)
    throw std::runtime_error("mux: subtitle streams are SubRip text or Matroska passthrough");
}

uint64_t write_mkv(const MuxPlan& P, int width, int height, int fps_num, int fps_den, const SideTrack* tracks,
                   int ntracks, const char* path);

}  // namespace muxi
}  // namespace tv
