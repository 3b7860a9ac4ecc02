// cpu_encoder.cpp — scalar C++ reference HEVC encoder.
//
// Plays the role of the reference's `software_encode` path (libx264 veryfast,
// reference worker/tasks.py:1558-1571; ffmpeg/libx264 are absent from this image,
// SURVEY.md §2.3 K6) and is the golden model for the GPU reconstruction stage: given the
// same decisions (CU sizes, modes, MVs) `reconstruct_frame` produces the levels and the
// reconstruction the HIP kernels must reproduce bit-exactly.
//
// Algorithm (same two-pass structure as the GPU pipeline):
//   pass A  analysis: intra mode / CU split from SATD against source neighbours (I),
//           motion search SAD + sub-pel refine + CU split (P)
//   pass B  reconstruction: prediction, forward transform, deadzone quantisation,
//           dequantisation, exact inverse transform, clipping; then deblocking.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>
#include <stdexcept>

#include "tv/cpu_encoder.h"
#include "tv/me_model.h"
#include "tv/rc_model.h"

namespace tv {

namespace {

int satd8x8(const int* d, int stride) {
  int m[64];
  for (int j = 0; j < 8; ++j)
    for (int i = 0; i < 8; ++i) m[j * 8 + i] = d[j * stride + i];
  for (int j = 0; j < 8; ++j) {  // horizontal butterflies
    int* r = m + j * 8;
    for (int s = 1; s < 8; s <<= 1)
      for (int i = 0; i < 8; ++i)
        if (!(i & s)) {
          const int a = r[i], b = r[i + s];
          r[i] = a + b;
          r[i + s] = a - b;
        }
  }
  for (int i = 0; i < 8; ++i)  // vertical
    for (int s = 1; s < 8; s <<= 1)
      for (int j = 0; j < 8; ++j)
        if (!(j & s)) {
          const int a = m[j * 8 + i], b = m[(j + s) * 8 + i];
          m[j * 8 + i] = a + b;
          m[(j + s) * 8 + i] = a - b;
        }
  int sum = 0;
  for (int k = 0; k < 64; ++k) sum += tv_abs(m[k]);
  return (sum + 2) >> 2;
}

int block_satd(const uint8_t* src, int ss, const int* pred, int N) {
  int diff[32 * 32];
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < N; ++i) diff[j * N + i] = src[j * ss + i] - pred[j * N + i];
  int s = 0;
  for (int by = 0; by < N; by += 8)
    for (int bx = 0; bx < N; bx += 8) s += satd8x8(diff + by * N + bx, N);
  return s;
}

}  // namespace

double lambda_sad(int qp) { return std::sqrt(0.57 * std::pow(2.0, (qp - 12) / 3.0)); }

void pad_source(const uint8_t* const planes[3], const int strides[3], int width, int height,
                Picture& dst) {
  for (int c = 0; c < 3; ++c) {
    const int w = c ? width / 2 : width, h = c ? height / 2 : height;
    const int pw = dst.pw(c), ph = dst.ph(c);
    uint8_t* D = dst.plane(c);
    for (int y = 0; y < ph; ++y) {
      const uint8_t* S = planes[c] + (size_t)tv_min(y, h - 1) * strides[c];
      for (int x = 0; x < pw; ++x) D[(size_t)y * pw + x] = S[tv_min(x, w - 1)];
    }
  }
}

// ------------------------------------ analysis ------------------------------------------
namespace {
struct IntraBest {
  int cost, mode;
};
// two-stage mode search (tv/me_model.h kIntraCoarseModes): planar, DC and every 4th angular
// mode, then the +-1/+-2 neighbours of the best coarse angular mode; SATD against the SOURCE
// neighbours' prediction + the mode penalty (k_intra_analysis / k_pintra_analysis)
IntraBest intra_best_mode(const Picture& src, int W, double lam, int x, int y, int log2, int* pred) {
  unsigned best = 0xffffffffu, best_ang = 0xffffffffu;
  auto eval = [&](int m) {
    predict_intra_tb(src, 0, x, y, log2, m, pred);
    int c = block_satd(src.y.data() + (size_t)y * W + x, W, pred, 1 << log2);
    c += (int)(lam * (m <= 1 ? 2 : 5));
    const unsigned v = ((unsigned)c << 6) | (unsigned)m;
    best = v < best ? v : best;
    if (m >= 2) best_ang = v < best_ang ? v : best_ang;
  };
  for (int i = 0; i < kIntraCoarseModes; ++i) eval(intra_coarse_mode(i));
  const int ma = (int)(best_ang & 63);
  for (int i = 0; i < 4; ++i) {
    const int m = intra_refine_mode(ma, i);
    if (m >= 2) eval(m);
  }
  return IntraBest{(int)(best >> 6), (int)(best & 63)};
}
}  // namespace

void analyze_intra(const SeqConfig& cfg, const Picture& src, FrameDecisions& fd) {
  const double lam = lambda_sad(cfg.qp);
  const int W = cfg.coded_w, H = cfg.coded_h;
  int pred[32 * 32];
  using Best = IntraBest;
  auto best_mode = [&](int x, int y, int log2) -> Best { return intra_best_mode(src, W, lam, x, y, log2, pred); };
  for (int cy = 0; cy < H; cy += 32)
    for (int cx = 0; cx < W; cx += 32) {
      // bottom-up quadtree on source-based costs
      const Best b32 = best_mode(cx, cy, 5);
      int sum16 = 0;
      int split16[4];
      Best b16s[4];
      for (int q = 0; q < 4; ++q) {
        const int x = cx + (q & 1) * 16, y = cy + (q >> 1) * 16;
        const Best b16 = best_mode(x, y, 4);
        int sum8 = 0;
        Best b8s[4];
        for (int r = 0; r < 4; ++r) {
          b8s[r] = best_mode(x + (r & 1) * 8, y + (r >> 1) * 8, 3);
          sum8 += b8s[r].cost + (int)(lam * 3);
        }
        split16[q] = sum8 < b16.cost + (int)(lam * 3);
        b16s[q] = b16;
        const int c16 = split16[q] ? sum8 : b16.cost + (int)(lam * 3);
        sum16 += c16;
        for (int r = 0; r < 4; ++r) {
          const int u = ((y >> 3) + (r >> 1)) * fd.w8 + (x >> 3) + (r & 1);
          fd.cu_log2[u] = split16[q] ? 3 : 4;
          fd.ipm[u] = (uint8_t)(split16[q] ? b8s[r].mode : b16.mode);
        }
      }
      if (b32.cost + (int)(lam * 3) <= sum16) {
        for (int j = 0; j < 4; ++j)
          for (int i = 0; i < 4; ++i) {
            const int u = ((cy >> 3) + j) * fd.w8 + (cx >> 3) + i;
            fd.cu_log2[u] = 5;
            fd.ipm[u] = (uint8_t)b32.mode;
          }
      }
      for (int j = 0; j < 4; ++j)
        for (int i = 0; i < 4; ++i) fd.intra[((cy >> 3) + j) * fd.w8 + (cx >> 3) + i] = 1;
    }
}

void quarter_luma(const Picture& src, std::vector<uint8_t>& q) {
  const int W = src.w, H = src.h, qw = W / 4, qh = H / 4;
  q.assign((size_t)qw * qh, 0);
  for (int y = 0; y < qh; ++y)
    for (int x = 0; x < qw; ++x) {
      int s = 0;
      for (int j = 0; j < 4; ++j)
        for (int i = 0; i < 4; ++i) s += src.y[(size_t)(4 * y + j) * W + 4 * x + i];
      q[(size_t)y * qw + x] = (uint8_t)((s + 8) >> 4);
    }
}

void coarse_search(const uint8_t* qcur, const uint8_t* qprev, int W, int H, int range, const int* penmv,
                   int16_t* cmv, int* ccost) {
  const int qw = W / 4, qh = H / 4, wc = W / kCtb, hc = H / kCtb, rq = range / 4;
  for (int cyi = 0; cyi < hc; ++cyi)
    for (int cxi = 0; cxi < wc; ++cxi) {
      const int x0 = 8 * cxi, y0 = 8 * cyi;
      unsigned best = 0xffffffffu;
      for (int dy = -rq; dy <= rq; ++dy)
        for (int dx = -rq; dx <= rq; ++dx) {
          int sad = 0;
          for (int j = 0; j < 8; ++j) {
            const int ry = clip3(0, qh - 1, y0 + j + dy);
            for (int i = 0; i < 8; ++i)
              sad += tv_abs(qcur[(size_t)(y0 + j) * qw + x0 + i] - qprev[(size_t)ry * qw + clip3(0, qw - 1, x0 + i + dx)]);
          }
          const unsigned idx = (unsigned)((dy + rq) * (2 * rq + 1) + dx + rq);
          const unsigned v = ((unsigned)(sad + me_coarse_pen(penmv, dx, dy)) << 13) | idx;
          best = v < best ? v : best;
        }
      const int idx = (int)(best & 8191), side = 2 * rq + 1;
      const int o = cyi * wc + cxi;
      cmv[2 * o] = (int16_t)(4 * (idx % side - rq));
      cmv[2 * o + 1] = (int16_t)(4 * (idx / side - rq));
      ccost[o] = (int)(best >> 13);
    }
}

namespace {
// block geometry of the 21 ME blocks: 16 x 8x8 (raster), 4 x 16x16, 1 x 32x32
void me_blk(int bi, int& bx, int& by, int& n) {
  if (bi < 16) {
    bx = (bi & 3) * 8, by = (bi >> 2) * 8, n = 8;
  } else if (bi < 20) {
    bx = ((bi - 16) & 1) * 16, by = ((bi - 16) >> 1) * 16, n = 16;
  } else {
    bx = by = 0, n = 32;
  }
}
int me_blk8_of(int q, int r) { return (((q >> 1) * 2 + (r >> 1)) << 2) + (q & 1) * 2 + (r & 1); }

// Motion search of one CTB against one reference: the 21 blocks' best cost (SAD + MV rate),
// vector and rate part (the GPU's k_inter_me computes exactly this).
struct CtbMe {
  int cost[21], mv[21][2], pen[21];
};
void me_ctb(const SeqConfig& cfg, const Picture& src, const Picture& ref, const int16_t* cmv, const int16_t* prev_mv,
            int range, int cxi, int cyi, int w8, CtbMe& out) {
  const double lam = lambda_sad(cfg.qp);
  const int W = cfg.coded_w, H = cfg.coded_h, wc = W / kCtb, hc = H / kCtb;
  int penmv[64];
  for (int i = 0; i < 64; ++i) penmv[i] = (int)(lam * i);
  const uint8_t* S = src.y.data();
  const uint8_t* R = ref.y.data();
  auto sad8 = [&](int x, int y, int dx, int dy) {  // one 8x8 block, integer displacement
    int s = 0;
    for (int j = 0; j < 8; ++j) {
      const int ry = clip3(0, H - 1, y + j + dy);
      for (int i = 0; i < 8; ++i)
        s += tv_abs(S[(size_t)(y + j) * W + x + i] - R[(size_t)ry * W + clip3(0, W - 1, x + i + dx)]);
    }
    return s;
  };
  auto sad_qpel = [&](int x, int y, int N, int mvx, int mvy) {
    int s = 0;
    const int fx = mvx & 3, fy = mvy & 3, bx = x + (mvx >> 2), by = y + (mvy >> 2);
    for (int j = 0; j < N; ++j)
      for (int i = 0; i < N; ++i)
        s += tv_abs(S[(size_t)(y + j) * W + x + i] - mc_luma_sample(R, W, W, H, bx + i, by + j, fx, fy));
    return s;
  };
  const int lim = range - 4;
  const int cx = cxi * kCtb, cy = cyi * kCtb;
  const int u0 = (cy >> 3) * w8 + (cx >> 3);
  int cand[kMeMaxCand][2], pmv[2];
  const int nc = me_candidates(cmv, wc, hc, cxi, cyi, prev_mv[2 * u0], prev_mv[2 * u0 + 1], lim, cand, pmv);
  // integer refinement: the 21 block costs at every window position (8x8 SADs reused)
  unsigned best[21];
  for (int k = 0; k < 21; ++k) best[k] = 0xffffffffu;
  for (int pos = 0; pos < nc * kMePosPerCand; ++pos) {
    int mx, my;
    me_pos_to_mv(pos, cand, mx, my);
    const unsigned pen = (unsigned)penmv[me_pen_index(4 * mx - pmv[0], 4 * my - pmv[1])];
    int s8[16], s16[4] = {0, 0, 0, 0}, s32 = 0;
    for (int k = 0; k < 16; ++k) {
      s8[k] = sad8(cx + (k & 3) * 8, cy + (k >> 2) * 8, mx, my);
      s16[((k >> 3) << 1) | ((k >> 1) & 1)] += s8[k];
      s32 += s8[k];
    }
    auto upd = [&](int bi, int sad) {
      const unsigned v = ((unsigned)sad + pen) << 11 | (unsigned)pos;
      best[bi] = v < best[bi] ? v : best[bi];
    };
    for (int k = 0; k < 16; ++k) upd(k, s8[k]);
    for (int q = 0; q < 4; ++q) upd(16 + q, s16[q]);
    upd(20, s32);
  }
  for (int bi = 0; bi < 21; ++bi) {
    int mx, my;
    me_pos_to_mv((int)(best[bi] & 2047), cand, mx, my);
    int* bmv = out.mv[bi];
    bmv[0] = 4 * mx;
    bmv[1] = 4 * my;
    out.cost[bi] = (int)(best[bi] >> 11);
    int bx, by, n;
    me_blk(bi, bx, by, n);
    // half then quarter pel refinement (centre wins ties, then the lowest neighbour)
    for (int step = 2; step >= 1; step >>= 1) {
      const int c0x = bmv[0], c0y = bmv[1];
      for (int k = 0; k < 8; ++k) {
        int ox, oy;
        me_cand_offset(k, ox, oy);
        const int qx = c0x + ox * step, qy = c0y + oy * step;
        const int c = sad_qpel(cx + bx, cy + by, n, qx, qy) + penmv[me_pen_index(qx - pmv[0], qy - pmv[1])];
        if (c < out.cost[bi]) {
          out.cost[bi] = c;
          bmv[0] = qx;
          bmv[1] = qy;
        }
      }
    }
    out.pen[bi] = penmv[me_pen_index(bmv[0] - pmv[0], bmv[1] - pmv[1])];
  }
}

// Bottom-up CU split of one CTB from per-block costs; writes cu_log2 and the block's index
// into `sel` per 8x8 unit (the caller copies that block's motion).
void split_ctb(const int* bcost, int pen_split, int sel[16], uint8_t l2[16]) {
  int sum16 = 0;
  for (int q = 0; q < 4; ++q) {
    int sum8 = 0;
    for (int r = 0; r < 4; ++r) sum8 += bcost[me_blk8_of(q, r)] + pen_split;
    const bool split = sum8 < bcost[16 + q] + pen_split;
    sum16 += split ? sum8 : bcost[16 + q] + pen_split;
    for (int r = 0; r < 4; ++r) {
      const int ux = (q & 1) * 2 + (r & 1), uy = (q >> 1) * 2 + (r >> 1);
      sel[uy * 4 + ux] = split ? me_blk8_of(q, r) : 16 + q;
      l2[uy * 4 + ux] = split ? 3 : 4;
    }
  }
  if (bcost[20] + pen_split <= sum16)
    for (int k = 0; k < 16; ++k) {
      sel[k] = 20;
      l2[k] = 5;
    }
}
}  // namespace

// Intra candidate of the P-picture quadrant at (x, y) (tv/me_model.h pintra_*): 0x80 | mode
// when the best intra mode's SAD + penalty beats the quadrant's 16x16 inter cost, else 0.
static uint8_t pintra_candidate(const Picture& src, int W, double lam, int x, int y, int inter_cost) {
  if (inter_cost <= kPIntraGate * 256) return 0;
  int pred[16 * 16];
  auto sad_of = [&]() {
    int s = 0;
    for (int j = 0; j < 16; ++j)
      for (int i = 0; i < 16; ++i) s += tv_abs((int)src.y[(size_t)(y + j) * W + x + i] - pred[j * 16 + i]);
    return s;
  };
  predict_intra_tb(src, 0, x, y, 4, 1, pred);  // DC first: hopeless quadrants skip the search
  if (!pintra_worth_search(sad_of(), (int)(lam * kPIntraPenBits), inter_cost)) return 0;
  const IntraBest ib = intra_best_mode(src, W, lam, x, y, 4, pred);
  predict_intra_tb(src, 0, x, y, 4, ib.mode, pred);
  return pintra_cost(sad_of(), (int)(lam * kPIntraPenBits)) < inter_cost ? (uint8_t)(0x80 | ib.mode) : (uint8_t)0;
}

void analyze_inter(const SeqConfig& cfg, const Picture& src, const Picture& ref, const int16_t* cmv,
                   const int16_t* prev_mv, int range, FrameDecisions& fd) {
  const double lam = lambda_sad(cfg.qp);
  const int pen_split = (int)(lam * 4);
  const int wc = cfg.coded_w / kCtb, hc = cfg.coded_h / kCtb;
  std::vector<uint8_t> cand(cfg.pintra ? (size_t)wc * hc * 4 : 0, 0);
  for (int cyi = 0; cyi < hc; ++cyi)
    for (int cxi = 0; cxi < wc; ++cxi) {
      CtbMe me;
      me_ctb(cfg, src, ref, cmv, prev_mv, range, cxi, cyi, fd.w8, me);
      int sel[16];
      uint8_t l2[16];
      split_ctb(me.cost, pen_split, sel, l2);
      const int u0 = (cyi * kCtb >> 3) * fd.w8 + (cxi * kCtb >> 3);
      for (int k = 0; k < 16; ++k) {
        const int u = u0 + (k >> 2) * fd.w8 + (k & 3);
        fd.cu_log2[u] = l2[k];
        fd.mv[2 * u] = (int16_t)me.mv[sel[k]][0];
        fd.mv[2 * u + 1] = (int16_t)me.mv[sel[k]][1];
        fd.intra[u] = 0;
        fd.ipm[u] = 1;
      }
      if (cfg.pintra)
        for (int q = 0; q < 4; ++q)
          cand[((size_t)cyi * wc + cxi) * 4 + q] = pintra_candidate(
              src, cfg.coded_w, lam, cxi * kCtb + (q & 1) * 16, cyi * kCtb + (q >> 1) * 16, me.cost[16 + q]);
    }
  if (cfg.pintra) apply_pintra(cand.data(), wc, hc, fd);
}

// Accepted intra quadrants (tv/me_model.h pintra_accepted) into the decisions: the CTB becomes
// four 16x16 CUs (a 32x32 inter CU's vector kept by the other quadrants), the quadrant a
// 16x16 intra CU with vector 0 (k_pintra_select).
void apply_pintra(const uint8_t* cand, int wc, int hc, FrameDecisions& fd) {
  for (int cyi = 0; cyi < hc; ++cyi)
    for (int cxi = 0; cxi < wc; ++cxi) {
      bool acc[4], any = false;
      for (int q = 0; q < 4; ++q) any |= acc[q] = pintra_accepted(cand, wc, hc, cxi, cyi, q);
      if (!any) continue;
      const int u0 = (cyi * kCtb >> 3) * fd.w8 + (cxi * kCtb >> 3);
      const bool whole = fd.cu_log2[u0] == 5;
      for (int k = 0; k < 16; ++k) {
        const int u = u0 + (k >> 2) * fd.w8 + (k & 3), q = ((k >> 3) << 1) | ((k >> 1) & 1);
        if (whole) fd.cu_log2[u] = 4;
        if (!acc[q]) continue;
        fd.cu_log2[u] = 4;
        fd.intra[u] = 1;
        fd.ipm[u] = (uint8_t)(cand[((size_t)cyi * wc + cxi) * 4 + q] & 63);
        fd.mv[2 * u] = fd.mv[2 * u + 1] = 0;
      }
    }
}

int bipred_sad(const Picture& src, const Picture& ref0, const Picture& ref1, int x, int y, int n, const int* mv0,
               const int* mv1) {
  const int W = src.w, H = src.h;
  int s = 0;
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) {
      const int p0 = mc_luma_sample(ref0.y.data(), W, W, H, x + i + (mv0[0] >> 2), y + j + (mv0[1] >> 2), mv0[0] & 3, mv0[1] & 3);
      const int p1 = mc_luma_sample(ref1.y.data(), W, W, H, x + i + (mv1[0] >> 2), y + j + (mv1[1] >> 2), mv1[0] & 3, mv1[1] & 3);
      s += tv_abs((int)src.y[(size_t)(y + j) * W + x + i] - ((p0 + p1 + 1) >> 1));
    }
  return s;
}

void analyze_inter_b(const SeqConfig& cfg, const Picture& src, const Picture& ref0, const Picture& ref1,
                     const int16_t* cmv0, const int16_t* cmv1, const int16_t* prev_mv, const int* range,
                     FrameDecisions& fd) {
  const int pen_split = (int)(lambda_sad(cfg.qp) * 4);
  const int wc = cfg.coded_w / kCtb, hc = cfg.coded_h / kCtb;
  for (int cyi = 0; cyi < hc; ++cyi)
    for (int cxi = 0; cxi < wc; ++cxi) {
      const int cx = cxi * kCtb, cy = cyi * kCtb;
      CtbMe m0, m1;
      me_ctb(cfg, src, ref0, cmv0, prev_mv, range[0], cxi, cyi, fd.w8, m0);
      me_ctb(cfg, src, ref1, cmv1, prev_mv, range[1], cxi, cyi, fd.w8, m1);
      int cost[21], dir[21];
      for (int bi = 0; bi < 21; ++bi) {
        int bx, by, n;
        me_blk(bi, bx, by, n);
        const int cb = bipred_sad(src, ref0, ref1, cx + bx, cy + by, n, m0.mv[bi], m1.mv[bi]) + m0.pen[bi] + m1.pen[bi];
        cost[bi] = m0.cost[bi];
        dir[bi] = 1;
        if (m1.cost[bi] < cost[bi]) {
          cost[bi] = m1.cost[bi];
          dir[bi] = 2;
        }
        if (cb < cost[bi]) {
          cost[bi] = cb;
          dir[bi] = 3;
        }
      }
      int sel[16];
      uint8_t l2[16];
      split_ctb(cost, pen_split, sel, l2);
      const int u0 = (cy >> 3) * fd.w8 + (cx >> 3);
      for (int k = 0; k < 16; ++k) {
        const int u = u0 + (k >> 2) * fd.w8 + (k & 3), b = sel[k];
        fd.cu_log2[u] = l2[k];
        fd.dir[u] = (uint8_t)dir[b];
        fd.mv[2 * u] = (int16_t)(dir[b] & 1 ? m0.mv[b][0] : 0);
        fd.mv[2 * u + 1] = (int16_t)(dir[b] & 1 ? m0.mv[b][1] : 0);
        fd.mv1[2 * u] = (int16_t)(dir[b] & 2 ? m1.mv[b][0] : 0);
        fd.mv1[2 * u + 1] = (int16_t)(dir[b] & 2 ? m1.mv[b][1] : 0);
        fd.intra[u] = 0;
        fd.ipm[u] = 1;
      }
    }
}

// -------------------------------- reconstruction ----------------------------------------
// Transform + quantise one TB of residual; writes levels into the plane; returns cbf.
static int code_tb(const int* resid, int log2N, int qp, bool intra, int16_t* lev, int ls, int rdoq) {
  const int N = 1 << log2N;
  int coef[32 * 32];
  forward_transform(resid, log2N, coef);
  int nz = 0, sumabs = 0;
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < N; ++i) {
      const int l = quant_level(coef[j * N + i], qp, log2N, intra);
      lev[j * ls + i] = (int16_t)l;
      nz += l != 0;
      sumabs += tv_abs(l);
    }
  // RDOQ-lite (inter TBs of 8x8 and up): walking the 4x4 coefficient groups in reverse
  // up-right diagonal scan, each trailing group whose only level is a lone +-1 is dropped
  // (its coded_sub_block_flag, significance, greater1 and sign bins and the longer last-
  // position code cost more than the level saves), up to the first group holding anything
  // else; the DC group stays, and with the default mode so do the groups before the TB's
  // anti-diagonal (kRdoqMode, rdoq_dmin).  Mode 1 at 640x360: textured -1.27 % BD-rate,
  // smooth -0.11 % (trimming groups of two +-1s as well: +0.46 / -0.51 %; every lone group,
  // not only trailing ones: -0.14 / -0.17 %).  k_inter_recon mirrors this (golden tests).
  if (!intra && rdoq && log2N >= 3) {
    const int s = N >> 2;
    for (int d = 2 * s - 2; d >= rdoq_dmin(rdoq, s); --d) {
      bool stop = false;
      for (int gy = tv_max(0, d - s + 1); gy <= tv_min(d, s - 1) && !stop; ++gy) {
        const int gx = d - gy;
        int t = 0;
        for (int j = 0; j < 4; ++j)
          for (int i = 0; i < 4; ++i) t += tv_abs(lev[(gy * 4 + j) * ls + gx * 4 + i]);
        if (t == 0) continue;
        if (t != 1) { stop = true; break; }
        for (int j = 0; j < 4; ++j)
          for (int i = 0; i < 4; ++i) lev[(gy * 4 + j) * ls + gx * 4 + i] = 0;
        nz -= 1;
        sumabs -= 1;
      }
      if (stop) break;
    }
  }
  // cheap RD heuristic: a lone +-1 outside DC in an inter block costs more than it saves
  if (!intra && nz == 1 && sumabs == 1 && lev[0] == 0) {
    for (int j = 0; j < N; ++j)
      for (int i = 0; i < N; ++i) lev[j * ls + i] = 0;
    nz = 0;
  }
  return nz ? 1 : 0;
}

void reconstruct_frame(const SeqConfig& cfg, const Picture& src, const Picture* ref,
                       FrameDecisions& fd, Picture& rec, const Picture* ref1) {
  const int W = cfg.coded_w, Wc = W >> 1, qp = cfg.qp, qpc = chroma_qp(qp, 0);
  int pred[32 * 32], resid[32 * 32];
  // walk CUs in z-order per CTU (needed for intra; harmless for inter).  code_tbs codes the
  // CU's TBs at (x0, y0) of size 2^log2 (a whole CU, or one 16x16 quadrant of an RQT-split CU:
  // inter prediction is per sample, so a quadrant predicts exactly like its CU).
  auto code_tbs = [&](int x0, int y0, int log2) {
    const int u = (y0 >> 3) * fd.w8 + (x0 >> 3);
    const bool intra = fd.intra[u] != 0;
    const int N = 1 << log2;
    int cbf = 0;
    for (int c = 0; c < 3; ++c) {
      const int l2 = c ? log2 - 1 : log2, n = 1 << l2;
      const int x = c ? x0 >> 1 : x0, y = c ? y0 >> 1 : y0;
      const int stride = c ? Wc : W;
      const int dir = ref1 ? fd.dir[u] : 1;
      if (intra) predict_intra_tb(rec, c, x, y, l2, fd.ipm[u], pred);
      else if (dir == 1) predict_inter_block(*ref, c, x, y, n, n, fd.mv[2 * u], fd.mv[2 * u + 1], pred);
      else if (dir == 2) predict_inter_block(*ref1, c, x, y, n, n, fd.mv1[2 * u], fd.mv1[2 * u + 1], pred);
      else predict_bi_block(*ref, *ref1, c, x, y, n, n, &fd.mv[2 * u], &fd.mv1[2 * u], pred);
      const uint8_t* S = src.plane(c) + (size_t)y * stride + x;
      for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) resid[j * n + i] = S[j * stride + i] - pred[j * n + i];
      int16_t* L = (c == 0 ? fd.coef_y : (c == 1 ? fd.coef_u : fd.coef_v)).data() + (size_t)y * stride + x;
      const int qq = c ? qpc : qp;
      const int cb = code_tb(resid, l2, qq, intra, L, stride, cfg.rdoq ? kRdoqMode : 0);
      cbf |= cb << c;
      recon_tb(L, stride, cb, l2, qq, pred, rec.plane(c) + (size_t)y * stride + x, stride);
    }
    for (int j = 0; j < (N >> 3); ++j)
      for (int i = 0; i < (N >> 3); ++i) fd.cbf[u + j * fd.w8 + i] = (uint8_t)cbf;
  };
  auto do_cu = [&](int x0, int y0, int log2) {
    const int u = (y0 >> 3) * fd.w8 + (x0 >> 3);
    if (cfg.rqt && ref && log2 >= kRqtMinLog2 && !fd.intra[u]) {  // RQT decision (hevc_defs.h rqt_split)
      const int N = 1 << log2, h = N >> 1, dir = ref1 ? fd.dir[u] : 1;
      if (dir == 1) predict_inter_block(*ref, 0, x0, y0, N, N, fd.mv[2 * u], fd.mv[2 * u + 1], pred);
      else if (dir == 2) predict_inter_block(*ref1, 0, x0, y0, N, N, fd.mv1[2 * u], fd.mv1[2 * u + 1], pred);
      else predict_bi_block(*ref, *ref1, 0, x0, y0, N, N, &fd.mv[2 * u], &fd.mv1[2 * u], pred);
      int sad4[4] = {0, 0, 0, 0};
      for (int j = 0; j < N; ++j)
        for (int i = 0; i < N; ++i)
          sad4[(j / h) * 2 + i / h] += tv_abs((int)src.y[(size_t)(y0 + j) * W + x0 + i] - pred[j * N + i]);
      if (rqt_split(sad4, h * h)) {
        for (int q = 0; q < 4; ++q) code_tbs(x0 + (q & 1) * h, y0 + (q >> 1) * h, log2 - 1);
        for (int j = 0; j < (N >> 3); ++j)
          for (int i = 0; i < (N >> 3); ++i) fd.tu[u + j * fd.w8 + i] = 1;
        return;
      }
    }
    code_tbs(x0, y0, log2);
  };
  for (int cy = 0; cy < cfg.coded_h; cy += 32)
    for (int cx = 0; cx < W; cx += 32) {
      // z-order traversal
      for (int q = 0; q < 4; ++q) {
        const int x16 = cx + (q & 1) * 16, y16 = cy + (q >> 1) * 16;
        const int l = fd.cu_log2[(cy >> 3) * fd.w8 + (cx >> 3)];
        if (l == 5) {
          if (q == 0) do_cu(cx, cy, 5);
          continue;
        }
        const int l16 = fd.cu_log2[(y16 >> 3) * fd.w8 + (x16 >> 3)];
        if (l16 == 4) {
          do_cu(x16, y16, 4);
        } else {
          for (int r = 0; r < 4; ++r) do_cu(x16 + (r & 1) * 8, y16 + (r >> 1) * 8, 3);
        }
      }
    }
  if (cfg.deblock) deblock_picture(rec, fd.view(), qp);
  if (cfg.sao) {  // SAO decisions on the deblocked picture, then the in-loop filter itself
    sao_decide_picture(src, rec, qp, fd.sao.data());
    sao_picture(rec, fd.sao.data());
  }
}

// ------------------------------------ driver --------------------------------------------
CpuEncoder::CpuEncoder(const SeqConfig& cfg, int search_range) : cfg_(cfg), range_(search_range) {
  if (search_range < 16 || search_range > 128 || (search_range & 15))
    throw std::runtime_error("search range must be a multiple of 16 in 16..128");
  cfg_.finalize();
  if (cfg_.mgop > 1) {  // parameter sets announce the steady-state DPB / reorder needs
    const GopPlan g = plan_gop(2 * cfg_.mgop + 1, cfg_.mgop);
    cfg_.dpb_size = g.dpb_size;
    cfg_.num_reorder = g.num_reorder;
  }
  src_.alloc(cfg_.coded_w, cfg_.coded_h);
  rec_.alloc(cfg_.coded_w, cfg_.coded_h);
  ref_.alloc(cfg_.coded_w, cfg_.coded_h);
  dec.alloc(cfg_.coded_w, cfg_.coded_h);
}

void CpuEncoder::begin_gop(int nframes) {
  if (cfg_.mgop <= 1) throw std::runtime_error("begin_gop: B frames are off (mgop <= 1)");
  plan_ = plan_gop(nframes, cfg_.mgop);
  next_ = 0;
  dpb_.clear();
}

void CpuEncoder::encode_b_structured(std::vector<uint8_t>& out, int qp) {
  if (next_ >= (int)plan_.pics.size()) throw std::runtime_error("encode: GOP plan exhausted (call begin_gop)");
  const CodedPic& p = plan_.pics[next_++];
  dec.alloc(cfg_.coded_w, cfg_.coded_h);
  const int wc = cfg_.coded_w / kCtb, hc = cfg_.coded_h / kCtb;
  std::vector<uint8_t> q;
  quarter_luma(src_, q);
  auto find = [&](int d) -> DpbEntry& {
    for (auto& e : dpb_)
      if (e.disp == d) return e;
    throw std::runtime_error("reference picture not in the encoder DPB");
  };
  SeqConfig fc = cfg_;
  const int base = qp >= 0 ? qp : cfg_.qp;
  fc.qp = clip3(0, 51, base + gop_layer_qp_offset(p.type, p.layer, cfg_.mgop));
  std::vector<int16_t> cmv[2];
  int rng[2] = {range_, range_};
  int penmv[64];
  for (int i = 0; i < 64; ++i) penmv[i] = (int)(lambda_sad(cfg_.qp) * i);
  for (int l = 0; l < 2; ++l) {
    if (p.ref[l] < 0) continue;
    cmv[l].assign(2 * (size_t)wc * hc, 0);
    std::vector<int> ccost((size_t)wc * hc);
    rng[l] = gop_search_range(range_, std::abs(p.disp - p.ref[l]), cfg_.mgop);
    coarse_search(q.data(), find(p.ref[l]).q.data(), cfg_.coded_w, cfg_.coded_h, rng[l], penmv, cmv[l].data(),
                  ccost.data());
  }
  if (prev_mv_.empty()) prev_mv_.assign(2 * (size_t)dec.w8 * dec.h8, 0);
  dec.refs = slice_refs(p);  // before reconstruction: B deblocking reads the directions
  dec.has_refs = true;
  if (p.type == 2) {
    write_parameter_sets(cfg_, out);
    analyze_intra(fc, src_, dec);
    reconstruct_frame(fc, src_, nullptr, dec, rec_);
  } else if (p.type == 1) {
    const Picture& r0 = find(p.ref[0]).rec;
    analyze_inter(fc, src_, r0, cmv[0].data(), prev_mv_.data(), rng[0], dec);
    reconstruct_frame(fc, src_, &r0, dec, rec_);
  } else {
    const Picture& r0 = find(p.ref[0]).rec;
    const Picture& r1 = find(p.ref[1]).rec;
    analyze_inter_b(fc, src_, r0, r1, cmv[0].data(), cmv[1].data(), prev_mv_.data(), rng, dec);
    reconstruct_frame(fc, src_, &r0, dec, rec_, &r1);
  }
  prev_mv_ = dec.mv;
  dec.qp = fc.qp;
  write_slice(cfg_, dec.view(), p.disp, p.type == 2, out);
  // DPB: keep what later pictures reference (this picture's RPS, plus itself if referenced)
  std::vector<DpbEntry> kept;
  for (auto& e : dpb_)
    if (std::find(p.rps.begin(), p.rps.end(), e.disp) != p.rps.end()) kept.push_back(std::move(e));
  dpb_ = std::move(kept);
  if (p.referenced) dpb_.push_back(DpbEntry{p.disp, rec_, std::move(q)});
}

void CpuEncoder::encode_frame(const uint8_t* const planes[3], const int strides[3], bool idr,
                              int poc, std::vector<uint8_t>& out, int qp) {
  pad_source(planes, strides, cfg_.width, cfg_.height, src_);
  if (cfg_.mgop > 1) {
    encode_b_structured(out, qp);
    return;
  }
  dec.alloc(cfg_.coded_w, cfg_.coded_h);
  const int wc = cfg_.coded_w / kCtb, hc = cfg_.coded_h / kCtb, qw = cfg_.coded_w / 4;
  quarter_luma(src_, qcur_);
  // coarse lookahead: penalties at the sequence QP (the frame QP may depend on its result)
  std::vector<int16_t> cmv(2 * (size_t)wc * hc);
  std::vector<int> ccost((size_t)wc * hc);
  if (!idr) {
    int penmv[64];
    for (int i = 0; i < 64; ++i) penmv[i] = (int)(lambda_sad(cfg_.qp) * i);
    coarse_search(qcur_.data(), qprev_.data(), cfg_.coded_w, cfg_.coded_h, range_, penmv, cmv.data(), ccost.data());
  }
  SeqConfig fc = cfg_;  // this frame's QP drives lambda, quantisation, deblocking and SAO
  if (qp >= 0) {
    fc.qp = qp;
  } else if (cfg_.crf > 0) {  // CRF: QP from the lookahead complexity of this frame
    uint64_t sum = 0;
    for (int cy = 0; cy < hc; ++cy)
      for (int cx = 0; cx < wc; ++cx)
        sum += idr ? rc_block_activity(qcur_.data() + (size_t)(8 * cy) * qw + 8 * cx, qw)
                   : (uint64_t)ccost[(size_t)cy * wc + cx];
    fc.qp = rc_crf_qp(cfg_.crf, idr, sum, wc * hc);
  } else if (cfg_.cascade) {
    fc.qp = clip3(0, 51, cfg_.qp + ippp_qp_offset(idr ? 0 : poc));
  }
  if (idr) {
    write_parameter_sets(cfg_, out);
    analyze_intra(fc, src_, dec);
    reconstruct_frame(fc, src_, nullptr, dec, rec_);
  } else {
    std::swap(ref_, rec_);
    analyze_inter(fc, src_, ref_, cmv.data(), prev_mv_.data(), range_, dec);
    reconstruct_frame(fc, src_, &ref_, dec, rec_);
  }
  std::swap(qcur_, qprev_);
  prev_mv_ = dec.mv;
  dec.qp = fc.qp;
  write_slice(cfg_, dec.view(), poc, idr, out);
}

}  // namespace tv
