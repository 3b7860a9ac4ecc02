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
    const bool a = zscan_available(xL, yL, (x - 1) * (1 << s), (y - 1) * (1 << s), W, H);
    la[0] = ta[0] = a;
    left[0] = top[0] = a ? P[(y - 1) * pw + (x - 1)] : 0;
  }
  for (int i = 0; i < 2 * N; ++i) {
    const bool al = zscan_available(xL, yL, (x - 1) * (1 << s), (y + i) * (1 << s), W, H);
    la[i + 1] = al;
    left[i + 1] = al ? P[(y + i) * pw + (x - 1)] : 0;
    const bool at = zscan_available(xL, yL, (x + i) * (1 << s), (y - 1) * (1 << s), W, H);
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

void predict_bi_block(const Picture& ref0, const Picture& ref1, int cIdx, int x, int y, int w, int h,
                      const int16_t* mv0, const int16_t* mv1, int* pred) {
  const Picture* R[2] = {&ref0, &ref1};
  const int16_t* M[2] = {mv0, mv1};
  const int pw = ref0.pw(cIdx), ph = ref0.ph(cIdx);
  for (int j = 0; j < h; ++j)
    for (int i = 0; i < w; ++i) {
      int p[2];
      for (int l = 0; l < 2; ++l) {
        const uint8_t* P = R[l]->plane(cIdx);
        const int mvx = M[l][0], mvy = M[l][1];
        p[l] = cIdx == 0 ? mc_luma_inter(P, pw, pw, ph, x + (mvx >> 2) + i, y + (mvy >> 2) + j, mvx & 3, mvy & 3)
                         : mc_chroma_inter(P, pw, pw, ph, x + (mvx >> 3) + i, y + (mvy >> 3) + j, mvx & 7, mvy & 7);
      }
      pred[j * w + i] = bipred_sample(p[0], p[1]);
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
  return deblock_edge_bs(fd.cu_log2, fd.intra, fd.cbf, fd.mv, fd.w8, xp, yp, xq, yq, fd.dir, fd.mv1, fd.tu);
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

// ------------------------------------------------------------------------------ SAO
void sao_ctb_stats(const Picture& src, const Picture& deb, int c, int cx, int cy, SaoStats& st) {
  std::memset(&st, 0, sizeof(st));
  const int w = deb.pw(c), h = deb.ph(c), n = c ? kCtb / 2 : kCtb;
  const uint8_t* S = src.plane(c);
  const uint8_t* D = deb.plane(c);
  for (int y = cy * n; y < (cy + 1) * n && y < h; ++y)
    for (int x = cx * n; x < (cx + 1) * n && x < w; ++x) {
      const int v = D[y * w + x], diff = (int)S[y * w + x] - v;
      st.bo_n[v >> 3] += 1;
      st.bo_s[v >> 3] += diff;
      for (int k = 0; k < 4; ++k) {
        int dx, dy;
        sao_eo_dir(k, dx, dy);
        const int ax = x + dx, ay = y + dy, bx = x - dx, by = y - dy;
        if (ax < 0 || ay < 0 || bx < 0 || by < 0 || ax >= w || ay >= h || bx >= w || by >= h) continue;
        const int cat = sao_eo_category(v, D[ay * w + ax], D[by * w + bx]);
        st.eo_n[k][cat] += 1;
        st.eo_s[k][cat] += diff;
      }
    }
}

void sao_decide_picture(const Picture& src, const Picture& deb, int qp, uint32_t* params) {
  const int wc = deb.w >> kCtbLog2, hc = deb.h >> kCtbLog2;
  const long long lam16 = sao_lambda16(qp);
  for (int cy = 0; cy < hc; ++cy)
    for (int cx = 0; cx < wc; ++cx) {
      SaoStats st[3];
      for (int c = 0; c < 3; ++c) sao_ctb_stats(src, deb, c, cx, cy, st[c]);
      sao_decide(st, lam16, params + 3 * (size_t)(cy * wc + cx));
    }
}

void sao_picture(Picture& pic, const uint32_t* params) {
  const int wc = pic.w >> kCtbLog2;
  for (int c = 0; c < 3; ++c) {
    const int w = pic.pw(c), h = pic.ph(c), n = c ? kCtb / 2 : kCtb;
    std::vector<uint8_t> deb(pic.plane(c), pic.plane(c) + (size_t)w * h);
    uint8_t* out = pic.plane(c);
    for (int y = 0; y < h; ++y)
      for (int x = 0; x < w; ++x) {
        const uint32_t p = params[3 * (size_t)((y / n) * wc + x / n) + c];
        if (sao_type(p)) out[y * w + x] = (uint8_t)sao_sample(deb.data(), w, h, x, y, p);
      }
  }
}

}  // namespace tv
