// hevc_recon.cpp — picture reconstruction primitives shared by the CPU reference encoder
// and the decoder oracle: intra/inter prediction of a block, residual reconstruction of a
// TB and the in-loop deblocking filter.  Bit-exact with the HIP kernels (tests compare).
#include <cstring>

#include "tv/hevc_codec.h"

namespace tv {

void predict_intra_tb(const Picture& rec, int cIdx, int x, int y, int log2N, int mode, int* pred) {
  const int N = 1 << log2N;
  const int s = cIdx ? 1 : 0;
  const int pw = rec.pw(cIdx);
  const uint8_t* P = rec.plane(cIdx);
  const int W = rec.w, H = rec.h;
  const int xL = x << s, yL = y << s;
  int left[65], top[65];
  bool la[65], ta[65];
  // corner
  {
    const bool a = zscan_available(xL, yL, (x - 1) << s, (y - 1) << s, W, H);
    la[0] = ta[0] = a;
    left[0] = top[0] = a ? P[(y - 1) * pw + (x - 1)] : 0;
  }
  for (int i = 0; i < 2 * N; ++i) {
    const bool al = zscan_available(xL, yL, (x - 1) << s, (y + i) << s, W, H);
    la[i + 1] = al;
    left[i + 1] = al ? P[(y + i) * pw + (x - 1)] : 0;
    const bool at = zscan_available(xL, yL, (x + i) << s, (y - 1) << s, W, H);
    ta[i + 1] = at;
    top[i + 1] = at ? P[(y - 1) * pw + (x + i)] : 0;
  }
  intra_substitute(left, top, la, ta, N);
  if (cIdx == 0 && intra_filter_refs(log2N, mode)) intra_smooth_refs(left, top, N);
  intra_pred_from_refs(left, top, log2N, mode, cIdx == 0 && N < 32, pred);
}

void predict_inter_block(const Picture& ref, int cIdx, int x, int y, int w, int h, int mvx, int mvy,
                         int* pred) {
  const uint8_t* P = ref.plane(cIdx);
  const int pw = ref.pw(cIdx), ph = ref.ph(cIdx);
  if (cIdx == 0) {
    const int fx = mvx & 3, fy = mvy & 3;
    const int bx = x + (mvx >> 2), by = y + (mvy >> 2);
    for (int j = 0; j < h; ++j)
      for (int i = 0; i < w; ++i) pred[j * w + i] = mc_luma_sample(P, pw, pw, ph, bx + i, by + j, fx, fy);
  } else {
    const int fx = mvx & 7, fy = mvy & 7;
    const int bx = x + (mvx >> 3), by = y + (mvy >> 3);
    for (int j = 0; j < h; ++j)
      for (int i = 0; i < w; ++i)
        pred[j * w + i] = mc_chroma_sample(P, pw, pw, ph, bx + i, by + j, fx, fy);
  }
}

void recon_tb(const int16_t* levels, int ls, bool cbf, int log2N, int qp, const int* pred,
              uint8_t* dst, int ds) {
  const int N = 1 << log2N;
  if (!cbf) {
    for (int j = 0; j < N; ++j)
      for (int i = 0; i < N; ++i) dst[j * ds + i] = (uint8_t)clip_pixel(pred[j * N + i]);
    return;
  }
  int coef[32 * 32], res[32 * 32];
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < N; ++i) coef[j * N + i] = dequant_level(levels[j * ls + i], qp, log2N);
  inverse_transform(coef, log2N, res);
  for (int j = 0; j < N; ++j)
    for (int i = 0; i < N; ++i) dst[j * ds + i] = (uint8_t)clip_pixel(pred[j * N + i] + res[j * N + i]);
}

namespace {
inline int edge_bs(const FrameData& fd, int xp, int yp, int xq, int yq) {
  return deblock_edge_bs(fd.cu_log2, fd.intra, fd.cbf, fd.mv, fd.w8, xp, yp, xq, yq);
}
}  // namespace

void deblock_picture(Picture& pic, const FrameData& fd, int qp) {
  const int W = pic.w, H = pic.h, Wc = W / 2, Hc = H / 2;
  uint8_t* Y = pic.y.data();
  uint8_t* U = pic.u.data();
  uint8_t* V = pic.v.data();
  const int qpc = chroma_qp(qp, 0);
  // vertical edges (horizontal filtering)
  for (int y = 0; y < H; y += 4)
    for (int x = 8; x < W; x += 8) {
      const int bs = edge_bs(fd, x - 1, y, x, y);
      if (bs) deblock_luma_edge4(Y + (size_t)y * W + x, 1, W, bs, qp);
    }
  for (int yc = 0; yc < Hc; yc += 4)
    for (int xc = 8; xc < Wc; xc += 8) {
      const int bs = edge_bs(fd, 2 * xc - 1, 2 * yc, 2 * xc, 2 * yc);
      if (bs == 2) {
        deblock_chroma_edge(U + (size_t)yc * Wc + xc, 1, Wc, 4, qpc);
        deblock_chroma_edge(V + (size_t)yc * Wc + xc, 1, Wc, 4, qpc);
      }
    }
  // horizontal edges (vertical filtering)
  for (int y = 8; y < H; y += 8)
    for (int x = 0; x < W; x += 4) {
      const int bs = edge_bs(fd, x, y - 1, x, y);
      if (bs) deblock_luma_edge4(Y + (size_t)y * W + x, W, 1, bs, qp);
    }
  for (int yc = 8; yc < Hc; yc += 8)
    for (int xc = 0; xc < Wc; xc += 4) {
      const int bs = edge_bs(fd, 2 * xc, 2 * yc - 1, 2 * xc, 2 * yc);
      if (bs == 2) {
        deblock_chroma_edge(U + (size_t)yc * Wc + xc, Wc, 1, 4, qpc);
        deblock_chroma_edge(V + (size_t)yc * Wc + xc, Wc, 1, 4, qpc);
      }
    }
}

}  // namespace tv
