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

#include "tv/cpu_encoder.h"

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

int mv_bits(int dx, int dy) { return mv_bits_est(dx, dy); }

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
void analyze_intra(const SeqConfig& cfg, const Picture& src, FrameDecisions& fd) {
  const double lam = lambda_sad(cfg.qp);
  const int W = cfg.coded_w, H = cfg.coded_h;
  int pred[32 * 32];
  struct Best {
    int cost, mode;
  };
  auto best_mode = [&](int x, int y, int log2) -> Best {
    Best b{INT_MAX, 1};
    for (int m = 0; m < 35; ++m) {
      predict_intra_tb(src, 0, x, y, log2, m, pred);
      int c = block_satd(src.y.data() + (size_t)y * W + x, W, pred, 1 << log2);
      c += (int)(lam * (m <= 1 ? 2 : 5));
      if (c < b.cost) b = Best{c, m};
    }
    return b;
  };
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

void analyze_inter(const SeqConfig& cfg, const Picture& src, const Picture& ref, int range,
                   FrameDecisions& fd) {
  const double lam = lambda_sad(cfg.qp);
  const int W = cfg.coded_w, H = cfg.coded_h;
  const uint8_t* S = src.y.data();
  const uint8_t* R = ref.y.data();
  auto sad_int = [&](int x, int y, int N, int dx, int dy) {
    int s = 0;
    for (int j = 0; j < N; ++j) {
      const int ry = clip3(0, H - 1, y + j + dy);
      for (int i = 0; i < N; ++i) {
        const int rx = clip3(0, W - 1, x + i + dx);
        s += tv_abs(S[(size_t)(y + j) * W + x + i] - R[(size_t)ry * W + rx]);
      }
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
  struct Res {
    int cost;
    int mvx, mvy;
  };
  auto search = [&](int x, int y, int N) -> Res {
    Res best{INT_MAX, 0, 0};
    for (int dy = -range; dy <= range; ++dy)
      for (int dx = -range; dx <= range; ++dx) {
        const int c = sad_int(x, y, N, dx, dy) + (int)(lam * mv_bits(4 * dx, 4 * dy));
        if (c < best.cost) best = Res{c, 4 * dx, 4 * dy};
      }
    // half then quarter pel refinement
    for (int step = 2; step >= 1; step >>= 1) {
      Res cen = best;
      for (int k = 0; k < 8; ++k) {
        static const int ox[8] = {-1, 0, 1, -1, 1, -1, 0, 1}, oy[8] = {-1, -1, -1, 0, 0, 1, 1, 1};
        const int mx = cen.mvx + ox[k] * step, my = cen.mvy + oy[k] * step;
        const int c = sad_qpel(x, y, N, mx, my) + (int)(lam * mv_bits(mx, my));
        if (c < best.cost) best = Res{c, mx, my};
      }
    }
    return best;
  };
  for (int cy = 0; cy < H; cy += 32)
    for (int cx = 0; cx < W; cx += 32) {
      const Res r32 = search(cx, cy, 32);
      int sum16 = 0;
      for (int q = 0; q < 4; ++q) {
        const int x = cx + (q & 1) * 16, y = cy + (q >> 1) * 16;
        const Res r16 = search(x, y, 16);
        Res r8[4];
        int sum8 = 0;
        for (int k = 0; k < 4; ++k) {
          r8[k] = search(x + (k & 1) * 8, y + (k >> 1) * 8, 8);
          sum8 += r8[k].cost + (int)(lam * 4);
        }
        const bool split = sum8 < r16.cost + (int)(lam * 4);
        sum16 += split ? sum8 : r16.cost + (int)(lam * 4);
        for (int k = 0; k < 4; ++k) {
          const int u = ((y >> 3) + (k >> 1)) * fd.w8 + (x >> 3) + (k & 1);
          fd.cu_log2[u] = split ? 3 : 4;
          fd.mv[2 * u] = (int16_t)(split ? r8[k].mvx : r16.mvx);
          fd.mv[2 * u + 1] = (int16_t)(split ? r8[k].mvy : r16.mvy);
        }
      }
      if (r32.cost + (int)(lam * 4) <= sum16) {
        for (int j = 0; j < 4; ++j)
          for (int i = 0; i < 4; ++i) {
            const int u = ((cy >> 3) + j) * fd.w8 + (cx >> 3) + i;
            fd.cu_log2[u] = 5;
            fd.mv[2 * u] = (int16_t)r32.mvx;
            fd.mv[2 * u + 1] = (int16_t)r32.mvy;
          }
      }
      for (int j = 0; j < 4; ++j)
        for (int i = 0; i < 4; ++i) fd.intra[((cy >> 3) + j) * fd.w8 + (cx >> 3) + i] = 0;
    }
}

// -------------------------------- reconstruction ----------------------------------------
// Transform + quantise one TB of residual; writes levels into the plane; returns cbf.
static int code_tb(const int* resid, int log2N, int qp, bool intra, int16_t* lev, int ls) {
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
  // cheap RD heuristic: a lone +-1 outside DC in an inter block costs more than it saves
  if (!intra && nz == 1 && sumabs == 1 && lev[0] == 0) {
    for (int j = 0; j < N; ++j)
      for (int i = 0; i < N; ++i) lev[j * ls + i] = 0;
    nz = 0;
  }
  return nz ? 1 : 0;
}

void reconstruct_frame(const SeqConfig& cfg, const Picture& src, const Picture* ref,
                       FrameDecisions& fd, Picture& rec) {
  const int W = cfg.coded_w, Wc = W >> 1, qp = cfg.qp, qpc = chroma_qp(qp, 0);
  int pred[32 * 32], resid[32 * 32];
  // walk CUs in z-order per CTU (needed for intra; harmless for inter)
  auto do_cu = [&](int x0, int y0, int log2) {
    const int u = (y0 >> 3) * fd.w8 + (x0 >> 3);
    const bool intra = fd.intra[u] != 0;
    const int N = 1 << log2;
    int cbf = 0;
    for (int c = 0; c < 3; ++c) {
      const int l2 = c ? log2 - 1 : log2, n = 1 << l2;
      const int x = c ? x0 >> 1 : x0, y = c ? y0 >> 1 : y0;
      const int stride = c ? Wc : W;
      if (intra) predict_intra_tb(rec, c, x, y, l2, fd.ipm[u], pred);
      else predict_inter_block(*ref, c, x, y, n, n, fd.mv[2 * u], fd.mv[2 * u + 1], pred);
      const uint8_t* S = src.plane(c) + (size_t)y * stride + x;
      for (int j = 0; j < n; ++j)
        for (int i = 0; i < n; ++i) resid[j * n + i] = S[j * stride + i] - pred[j * n + i];
      int16_t* L = (c == 0 ? fd.coef_y : (c == 1 ? fd.coef_u : fd.coef_v)).data() + (size_t)y * stride + x;
      const int qq = c ? qpc : qp;
      const int cb = code_tb(resid, l2, qq, intra, L, stride);
      cbf |= cb << c;
      recon_tb(L, stride, cb, l2, qq, pred, rec.plane(c) + (size_t)y * stride + x, stride);
    }
    for (int j = 0; j < (N >> 3); ++j)
      for (int i = 0; i < (N >> 3); ++i) fd.cbf[u + j * fd.w8 + i] = (uint8_t)cbf;
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
  cfg_.finalize();
  src_.alloc(cfg_.coded_w, cfg_.coded_h);
  rec_.alloc(cfg_.coded_w, cfg_.coded_h);
  ref_.alloc(cfg_.coded_w, cfg_.coded_h);
  dec.alloc(cfg_.coded_w, cfg_.coded_h);
}

void CpuEncoder::encode_frame(const uint8_t* const planes[3], const int strides[3], bool idr,
                              int poc, std::vector<uint8_t>& out) {
  pad_source(planes, strides, cfg_.width, cfg_.height, src_);
  dec.alloc(cfg_.coded_w, cfg_.coded_h);
  if (idr) {
    write_parameter_sets(cfg_, out);
    analyze_intra(cfg_, src_, dec);
    reconstruct_frame(cfg_, src_, nullptr, dec, rec_);
  } else {
    std::swap(ref_, rec_);
    analyze_inter(cfg_, src_, ref_, range_, dec);
    reconstruct_frame(cfg_, src_, &ref_, dec, rec_);
  }
  write_slice(cfg_, dec.view(), poc, idr, out);
}

}  // namespace tv
