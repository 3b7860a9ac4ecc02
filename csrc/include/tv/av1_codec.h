// av1_codec.h — host side of the AV1 encode path (BASELINE config #4):
// OBU / uncompressed-header / tile syntax writer, the decoder oracle that parses the same
// streams back and reconstructs them, and the C++ golden encoder whose decisions and
// reconstruction the gfx950 engine (csrc/gpu/k_av1_enc.hip) reproduces bit for bit.
// Coding-tool subset and substituted tables: tv/av1_enc.h.
#pragma once
#include <cstdint>
#include <vector>

#include "tv/av1_enc.h"

namespace tv {
namespace av1 {

struct SeqGeo {
  int dw, dh;  // display (render) size
  int W, H;    // coded size (multiples of 16)
  int bw, bh;  // 16x16 blocks
  int sbw, sbh;
  int nblk() const { return bw * bh; }
  int nsb() const { return sbw * sbh; }
  // 64x64 restoration units of plane p (7.17 count_units_in_frame; plane 0 has the most)
  int lr_ux(int p) const { int n = ((p ? W / 2 : W) + 32) / 64; return n > 1 ? n : 1; }
  int lr_uy(int p) const { int n = ((p ? H / 2 : H) + 32) / 64; return n > 1 ? n : 1; }
  int lr_nu() const { return lr_ux(0) * lr_uy(0); }
};
SeqGeo make_seq_geo(int dw, int dh);

// Frame-level parameters (uncompressed header fields chosen by the encoder).
struct FrameParams {
  int key = 1;
  int qindex = 100;
  int lf[4] = {0, 0, 0, 0};  // loop_filter_level[0..3]
  int sharp = 0;
  int cdef_damping = 3;      // 3..6
  int cdef_bits = 3;
  uint8_t cdef_y[8] = {0};   // preset index pri * 4 + sec_idx (sec_idx 3 -> strength 4)
  uint8_t cdef_uv[8] = {0};
};

// Decisions of one frame.  Levels are raster order inside each transform block.  A null
// level pointer means "all TBs of that plane are packed": blocks whose nonzero mask
// (mode word bits 10-12) has the plane's bit set appear consecutively in raster block
// order in ly / lu / lv.  `packed` selects that layout (`scan_packed`: eob-truncated).
struct FrameDecisions {
  FrameParams fp;
  const uint32_t* mode = nullptr;   // [nblk]
  const uint32_t* mv = nullptr;     // [nblk]
  const int16_t* ly = nullptr;      // [nblk or packed][256]
  const int16_t* lu = nullptr;      // [..][64]
  const int16_t* lv = nullptr;      // [..][64]
  const int8_t* cdef_idx = nullptr; // [nsb]  (-1: every block of the SB is skip)
  const int32_t* lr = nullptr;      // [3][nu_luma][3] per plane, per 64x64 unit: (sgr set | -1, xqd0, xqd1)
  bool packed = false;
  // with packed: each nonzero TB is [eob, eob levels in zigzag_scan order] (int16), TBs
  // back to back (the GPU engine's eob-truncated device->host layout)
  bool scan_packed = false;
};

// Owned variant (decoder output / golden encoder).
struct FrameData {
  FrameParams fp;
  std::vector<uint32_t> mode, mv;
  std::vector<int16_t> ly, lu, lv;  // full (unpacked) [nblk][256|64]
  std::vector<int8_t> cdef_idx;
  std::vector<int32_t> lr;          // [3][nu_luma][3]
  FrameDecisions view() const;
};

// Entropy state carried between the frames of one stream: the CDFs saved at the end of the
// previous frame (disable_frame_end_update_cdf = 0), loaded by an inter frame through
// primary_ref_frame = 0.  Opaque bytes of the internal CDF set.
struct EntropyState {
  std::vector<uint8_t> saved;
};

// Temporal unit of one frame: temporal delimiter [+ sequence header] + OBU_FRAME.  `st`
// carries the CDFs from frame to frame (required for inter frames, updated by every frame).
std::vector<uint8_t> write_temporal_unit(const SeqGeo& g, const FrameDecisions& d, bool seq_header, EntropyState* st);

struct Planes {
  std::vector<uint8_t> y, u, v;  // coded size
};

// Reconstruction of one frame from its decisions (prediction + residual, deblocking,
// CDEF); `ref` = previous reconstructed frame (inter frames).  Used by the decoder oracle.
void reconstruct(const SeqGeo& g, const FrameDecisions& d, const Planes* ref, Planes& out);

// Decoder oracle: parse a stream of temporal units (IVF payloads or concatenated OBUs),
// returning every shown frame (coded size) and the parsed decisions.
struct Decoded {
  SeqGeo geo{};
  std::vector<Planes> frames;
  std::vector<FrameData> data;
};
Decoded decode_stream(const uint8_t* p, size_t n);

// Golden encoder (the GPU engine's specification): encode `nframes` I420 frames of coded
// size (edge-padded) as one closed GOP; key frame first.  Returns the per-frame decisions
// and final (post-filter) reconstructions.
struct GoldenOut {
  std::vector<FrameData> frames;
  std::vector<Planes> recon;
};
GoldenOut golden_encode(const SeqGeo& g, const std::vector<Planes>& src, int qindex);

// CDEF preset choice shared with the GPU kernel: greedy luma presets on the SSE of active
// 64x64 blocks, per-index chroma preset, joint reassignment.  sse_* [nfb][64].
void cdef_choose(const uint64_t* sse_y, const uint64_t* sse_uv, const uint8_t* active, int nfb, uint8_t* ytab,
                 uint8_t* uvtab, int8_t* fb_idx);

}  // namespace av1
}  // namespace tv
