// gop.h — coding structure of one closed GOP (segment): hierarchical-B mini-GOPs.
//
// With a mini-GOP of M frames (M = 1: I P P P ..., the low-delay structure) the anchors are
// display frames 0, M, 2M, ... and the last frame of the segment; anchor 0 is the IDR, every
// other anchor is a P picture predicted from the previous anchor.  The frames between two
// anchors lo < hi are B pictures coded by bisection: mid = (lo + hi) / 2 is predicted from
// lo (list 0, past) and hi (list 1, future), then the two halves recurse — so every B
// picture has exactly one reference per list, and the deeper a picture sits in the tree the
// higher its temporal layer (and its QP offset).  The plan also carries each picture's
// reference picture set (the pictures the decoder must keep), from which the parameter
// sets' DPB size and reorder depth follow.  Shared by the CPU golden encoder, the GPU engine
// and the bitstream writer, so all three agree on order, references and QPs.
#pragma once
#include <algorithm>
#include <cstdlib>
#include <vector>

namespace tv {

struct CodedPic {
  int disp = 0;                  // display index in the segment == POC
  int type = 2;                  // 2 = I, 1 = P, 0 = B (slice_type values)
  int ref[2] = {-1, -1};         // display index of the list-0 / list-1 reference (-1: none)
  int layer = 0;                 // 0 = I / P anchors, 1.. = B bisection depth
  std::vector<int> rps;          // pictures kept in the DPB while this one decodes (display idx)
  std::vector<int> rps_used;     // 1 = referenced by this picture
  bool referenced = false;       // some later picture predicts from this one
};

struct GopPlan {
  std::vector<CodedPic> pics;    // coding order
  int dpb_size = 1;              // max pictures held (references + the current one)
  int num_reorder = 0;           // sps_max_num_reorder_pics
  int max_layer = 0;
};

inline void gop_bisect(int lo, int hi, int layer, std::vector<CodedPic>& out) {
  if (hi - lo <= 1) return;
  const int mid = (lo + hi) >> 1;
  CodedPic p;
  p.disp = mid;
  p.type = 0;
  p.ref[0] = lo;
  p.ref[1] = hi;
  p.layer = layer;
  out.push_back(p);
  gop_bisect(lo, mid, layer + 1, out);
  gop_bisect(mid, hi, layer + 1, out);
}

// Plan a segment of `nframes` frames (first one IDR) with mini-GOP `mgop` (1 = no B frames).
inline GopPlan plan_gop(int nframes, int mgop) {
  GopPlan g;
  if (nframes < 1) return g;
  if (mgop < 1) mgop = 1;
  CodedPic i0;
  i0.disp = 0;
  g.pics.push_back(i0);
  for (int lo = 0; lo < nframes - 1;) {
    const int hi = std::min(lo + mgop, nframes - 1);
    CodedPic p;
    p.disp = hi;
    p.type = 1;
    p.ref[0] = lo;
    g.pics.push_back(p);
    gop_bisect(lo, hi, 1, g.pics);
    lo = hi;
  }
  const int n = (int)g.pics.size();
  // reference picture sets: a picture stays while any later picture (coding order) uses it
  std::vector<int> last_use(nframes, -1);
  for (int k = 0; k < n; ++k)
    for (int l = 0; l < 2; ++l)
      if (g.pics[k].ref[l] >= 0) last_use[g.pics[k].ref[l]] = k;
  for (int k = 0; k < n; ++k) {
    CodedPic& p = g.pics[k];
    p.referenced = last_use[p.disp] > k;
    if (p.type == 2) continue;  // IDR: empty RPS
    for (int j = 0; j < k; ++j) {
      const int d = g.pics[j].disp;
      if (last_use[d] >= k) {
        p.rps.push_back(d);
        p.rps_used.push_back(d == p.ref[0] || d == p.ref[1] ? 1 : 0);
      }
    }
    g.dpb_size = std::max(g.dpb_size, (int)p.rps.size() + 1);
    g.max_layer = std::max(g.max_layer, p.layer);
  }
  // reorder depth: pictures that precede one in coding order but follow it in display order
  for (int k = 0; k < n; ++k) {
    int c = 0;
    for (int j = 0; j < k; ++j) c += g.pics[j].disp > g.pics[k].disp;
    g.num_reorder = std::max(g.num_reorder, c);
  }
  return g;
}

// Motion search range of a reference `dist` pictures away in a hierarchical-B GOP: the
// anchors' range covers M frames of motion, nearer references need proportionally less
// (range * dist / 4, in steps of 16, at least 16) -- the coarse quarter-res search shrinks
// quadratically with it.  I P P P streams keep the configured range.
inline int gop_search_range(int range, int dist, int mgop) {
  if (mgop <= 1) return range;
  const int r = (range * dist + 63) / 64 * 16;
  return std::min(range, std::max(16, r));
}

// QP offset of a temporal layer (hierarchical-B QP cascade).  IPPP streams: none.  With B
// frames the anchor P pictures take +1 and B layer L takes +3 + L: the B pictures are never
// (layer max) or briefly referenced, so their bits buy little quality for the rest of the
// GOP.  Chosen from the golden encoder's rate-distortion curves on the bench content
// (tools/rd_curve.py, profiles/README.md): +1/+2/+3/+4 -13.6 %, +1/+3/+4/+5 -16.7 %,
// +1/+4/+5/+6 -19.6 % BD-rate against the IPPP stream at M = 8.
inline int gop_layer_qp_offset(int type, int layer, int mgop) {
  if (mgop <= 1 || type == 2) return 0;
  return layer == 0 ? 1 : 3 + layer;
}

// Constant-QP I P P P streams (SeqConfig::cascade): the IDR at QP - 5 and the P pictures in
// an 8-picture low-delay hierarchy +1 0 +1 -1 +1 0 +1 -3 (mean 0, so the nominal QP keeps its
// rate point): every 8th P picture is a high-quality anchor the following ones predict from.
// Golden encoder, 64 frames of the bench content at 640x360, QP 22-37 (tools/rd_curve.py,
// profiles/README.md round 5): -4.5 % BD-rate smooth, -2.8 % textured against flat QP; at
// QP 27 +0.37 dB for +3 % rate.  Explicit per-frame QPs (2-pass plans) and CRF are not
// cascaded.
inline int ippp_qp_offset(int poc) {
  constexpr int kP[8] = {1, 0, 1, -1, 1, 0, 1, -3};
  return poc == 0 ? -5 : kP[(poc - 1) & 7];
}

}  // namespace tv
