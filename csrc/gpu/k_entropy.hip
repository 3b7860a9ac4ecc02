// k_entropy.hip — HEVC CABAC on the GPU (entropy_coding_sync / WPP substreams).
//
// The host CABAC writer (csrc/core/hevc_writer.cpp) costs 8 busy cores per GPU on the bench
// content and 15 on grain; on an 8-GPU node a rank owns 1/8 of the host.  Every syntax
// decision is already fixed when a picture's kernels finish, so entropy coding splits into
//   1. binarisation — data-parallel: one thread per CTB turns the CTB's decisions and compact
//      levels into a token list (context-coded bins with their context index, bypass runs,
//      terminate bins, WPP control marks), run twice: count, exclusive scan, write;
//   2. arithmetic coding — serial per WPP substream: one workgroup per slice, one lane per CTB
//      row; lane r starts once lane r-1 stored its contexts after CTB 1 (9.3.2.4), the
//      context states live in LDS ([ctx][row] bytes), the coder state in registers;
//   3. packing — the rows' bytes are compacted per slice for one device->host copy.
// The host only writes the slice header, the entry points and emulation prevention.
//
// Byte-for-byte the output of tv::write_slice with SeqConfig::wpp (the CPU writer stays the
// oracle: tests/test_gpu_entropy.py).  The per-CU skip / merge choice is made in a pre-pass
// (k_ent_cu) so a CTB's cu_skip_flag context can read its left / upper neighbours'.
// Reference: the reference entropy-codes in VA-API fixed function (worker/tasks.py:1573-1586).
#include <cstdlib>
#include <stdexcept>
#include <string>

#include "gpu_common.h"
#include "k_encode.h"
#include "tv/cabac.h"
#include "tv/hevc_mvpred.h"

namespace tv {
namespace gpu {

namespace {

// ---- token format (32 bits, type in bits 30..31) ----------------------------------------
//   CTX : bits 27..28 = number of bins n (1..3); bin i at bits 9i..9i+8 = ctx | bin << 8
//   BYP : bits 16..20 = count (1..16), bits 0..15 = the bins, MSB first
//   TERM: bit 0 = the terminating bin
//   CTRL: 0 = SYNC (store the row's contexts for the row below), 1 = FLUSH (end of substream:
//         flush the coder, '1' bit, byte alignment)
constexpr uint32_t kTkCtx = 0u << 30, kTkByp = 1u << 30, kTkTerm = 2u << 30, kTkCtrl = 3u << 30;
constexpr uint32_t kCtrlSync = 0, kCtrlFlush = 1;
static_assert(CTX_COUNT <= kEntCtx && kEntCtx <= 256, "context index must fit 8 bits");

struct TokSink {
  uint32_t* out;  // nullptr: count only
  int cap;        // tokens past `cap` are counted, not written
  int n = 0;
  uint32_t pc = 0, pb = 0;  // pending context bins / bypass bins
  int npc = 0, npb = 0;
  __device__ __forceinline__ void put(uint32_t t) {
    if (out && n < cap) out[n] = t;
    ++n;
  }
  __device__ __forceinline__ void flush_c() {
    if (npc) put(kTkCtx | ((uint32_t)npc << 27) | pc);
    npc = 0;
    pc = 0;
  }
  __device__ __forceinline__ void flush_b() {
    if (npb) put(kTkByp | ((uint32_t)npb << 16) | pb);
    npb = 0;
    pb = 0;
  }
  __device__ __forceinline__ void bin(int b, int ctx) {
    flush_b();
    pc |= (uint32_t)(ctx | (b << 8)) << (9 * npc);
    if (++npc == 3) flush_c();
  }
  // consecutive bypass bins are one run: equiprobable bins, so splitting or merging a run
  // never changes the arithmetic code
  __device__ __forceinline__ void bypass(uint32_t v, int nb) {
    flush_c();
    while (nb > 0) {
      const int take = tv_min(nb, 16 - npb);
      nb -= take;
      pb = (pb << take) | ((v >> nb) & ((1u << take) - 1));
      npb += take;
      if (npb == 16) flush_b();
    }
  }
  __device__ __forceinline__ void term(int b) {
    flush_c();
    flush_b();
    put(kTkTerm | (uint32_t)b);
  }
  __device__ __forceinline__ void ctrl(uint32_t c) {
    flush_c();
    flush_b();
    put(kTkCtrl | c);
  }
};

// Residual-coding tables (H.265 9.3.4.2.x), built at compile time, copied to LDS by every
// binariser workgroup: per-bin table reads from global / constant memory were the kernel's
// critical path (a dependent ~1 us round trip per bin).
struct BinTables {
  uint8_t scan4[3][16];      // in-sub-block scan position -> raster (x | y << 2), scanIdx 0/1/2
  uint8_t map4[3][16];       // 4x4 TBs: ctxIdxMap of the position
  uint8_t sigpat[3][4][16];  // larger TBs: sigCtx pattern (0..2) per scanIdx, prevCsbf, position
  uint8_t group_idx[32];
  uint8_t min_in_group[16];
  uint8_t sbpos[4][3][64];   // sub-block scans of every TB size (log2 - 2): raster index of scan pos
  uint8_t sbinv[4][3][64];   // and its inverse (hevc_defs.h subblock_pos)
};
constexpr BinTables make_tables() {
  BinTables t{};
  constexpr uint8_t map[16] = {0, 1, 4, 5, 2, 3, 4, 5, 6, 6, 8, 8, 7, 7, 8, 8};
  constexpr uint8_t gi[32] = {0, 1, 2, 3, 4, 4, 5, 5, 6, 6, 6, 6, 7, 7, 7, 7,
                              8, 8, 8, 8, 8, 8, 8, 8, 9, 9, 9, 9, 9, 9, 9, 9};
  constexpr uint8_t mg[10] = {0, 1, 2, 3, 4, 6, 8, 12, 16, 24};
  for (int i = 0; i < 32; ++i) t.group_idx[i] = gi[i];
  for (int i = 0; i < 10; ++i) t.min_in_group[i] = mg[i];
  for (int sc = 0; sc < 3; ++sc)
    for (int n = 0; n < 16; ++n) {
      const uint8_t pos = sc == 0 ? kScanDiag4x4[n] : (sc == 1 ? kScanHor4x4[n] : kScanVer4x4[n]);
      t.scan4[sc][n] = pos;
      t.map4[sc][n] = map[pos];
      const int xp = pos & 3, yp = pos >> 2;
      for (int pc = 0; pc < 4; ++pc) {
        int v = 2;
        if (pc == 0) v = (xp + yp == 0) ? 2 : (xp + yp < 3) ? 1 : 0;
        else if (pc == 1) v = (yp == 0) ? 2 : (yp == 1) ? 1 : 0;
        else if (pc == 2) v = (xp == 0) ? 2 : (xp == 1) ? 1 : 0;
        t.sigpat[sc][pc][n] = (uint8_t)v;
      }
    }
  for (int l = 0; l < 4; ++l)
    for (int sc = 0; sc < 3; ++sc)
      for (int i = 0; i < (1 << (2 * l)); ++i) {
        int xs = 0, ys = 0;
        if (l == 1) {
          const uint8_t q = sc == 0 ? kScanDiag2x2[i] : (sc == 1 ? kScanHor2x2[i] : kScanVer2x2[i]);
          xs = q & 3;
          ys = q >> 2;
        } else if (l == 2) {
          xs = kScanDiag4x4[i] & 3;
          ys = kScanDiag4x4[i] >> 2;
        } else if (l == 3) {
          xs = kScanDiag8x8.s[i] & 7;
          ys = kScanDiag8x8.s[i] >> 3;
        }
        t.sbpos[l][sc][i] = (uint8_t)((ys << l) + xs);
        t.sbinv[l][sc][(ys << l) + xs] = (uint8_t)i;
      }
  return t;
}
__constant__ BinTables c_tab = make_tables();
static_assert(sizeof(BinTables) % 4 == 0, "copied as words");

// level at raster position p (0..15) of a 4x4 group held as 8 packed int16 pairs
__device__ __forceinline__ int level_at(const uint4& lo, const uint4& hi, int p) {
  const int q = p >> 1;
  const uint32_t a = (q & 1) ? lo.y : lo.x, b = (q & 1) ? lo.w : lo.z;
  const uint32_t c = (q & 1) ? hi.y : hi.x, d = (q & 1) ? hi.w : hi.z;
  const uint32_t e = (q & 2) ? b : a, f = (q & 2) ? d : c;
  const uint32_t w = (q & 4) ? f : e;
  return (int)(int16_t)(w >> ((p & 1) * 16));
}

// One segment's picture, as the binariser sees it (device pointers at segment b).
struct SegView {
  const uint8_t *cu_log2, *intra, *ipm, *cbf, *tu, *dir;
  const int16_t *mv, *mv1;
  const uint8_t* skip;
  const int8_t* midx;
  const unsigned long long* mask_y;
  const unsigned* mask_c;
  const int* sb_off;
  const int16_t* packed;
  const uint32_t* sao;
  int w8, wc, hc, W, H;
  long ubase = 0;  // first unit of the planes' window (k_ent_bin stages a window in LDS)
};

__device__ __forceinline__ SegView seg_view(const EntropyArgs& a, int b) {
  const long U = a.g.usz, nctu = (long)a.g.wc * a.g.hc;
  SegView v;
  v.cu_log2 = a.dec.cu_log2 + b * U;
  v.intra = a.dec.intra + b * U;
  v.ipm = a.dec.ipm + b * U;
  v.cbf = a.dec.cbf + b * U;
  v.tu = a.dec.tu ? a.dec.tu + b * U : nullptr;
  v.dir = a.dec.dir ? a.dec.dir + b * U : nullptr;
  v.mv = a.dec.mv + b * U * 2;
  v.mv1 = a.dec.mv1 ? a.dec.mv1 + b * U * 2 : nullptr;
  v.skip = a.skip + b * U;
  v.midx = a.midx + b * U;
  v.mask_y = a.cs.mask_y + b * nctu;
  v.mask_c = a.cs.mask_c + b * nctu;
  v.sb_off = a.cs.offset + b * nctu;
  long base = 0;  // segments' packed levels are back to back (k_sb_pack)
  for (int k = 0; k < b; ++k) base += a.cs.total[k];
  v.packed = a.cs.packed + base * 16;
  v.sao = a.sao ? a.sao + b * nctu * 3 : nullptr;
  v.w8 = a.g.w8;
  v.wc = a.g.wc;
  v.hc = a.g.hc;
  v.W = a.g.W;
  v.H = a.g.H;
  return v;
}

__device__ __forceinline__ int unit_of(const SegView& v, int x, int y) { return (int)((y >> 3) * v.w8 + (x >> 3) - v.ubase); }
__device__ __forceinline__ Motion motion_of(const SegView& v, int u) {
  Motion m;
  m.dir = v.dir ? v.dir[u] : 1;
  m.mv[0] = Mv{v.mv[2 * u], v.mv[2 * u + 1]};
  if (v.mv1) m.mv[1] = Mv{v.mv1[2 * u], v.mv1[2 * u + 1]};
  return m;
}
__device__ __forceinline__ int cu_cbf(const SegView& v, int x0, int y0, int log2) {
  const int u = unit_of(v, x0, y0);
  if (!(v.tu && v.tu[u])) return v.cbf[u];
  const int h = 1 << (log2 - 1);
  int c = 0;
  for (int q = 0; q < 4; ++q) c |= v.cbf[unit_of(v, x0 + (q & 1) * h, y0 + (q >> 1) * h)];
  return c;
}

// Index of the PU's vector in its P-slice merge list, or -1 (hevc_writer.cpp merge_index_p).
__device__ __forceinline__ int merge_index_p(const SegView& v, int x0, int y0, int N, Mv mv, int maxc) {
  auto get = [&](int xn, int yn, Mv& m) {
    const int u = unit_of(v, xn, yn);
    if (v.intra[u]) return false;
    m.x = v.mv[2 * u];
    m.y = v.mv[2 * u + 1];
    return true;
  };
  Mv a1, b1, b0, a0, b2;
  int n = 0;
  const bool avA1 = x0 > 0 && get(x0 - 1, y0 + N - 1, a1);
  if (avA1) {
    if (a1 == mv) return 0;
    if (++n == maxc) return -1;
  }
  const bool avB1 = y0 > 0 && get(x0 + N - 1, y0 - 1, b1);
  const bool fB1 = avB1 && !(avA1 && a1 == b1);
  if (fB1) {
    if (b1 == mv) return n;
    if (++n == maxc) return -1;
  }
  const bool avB0 = zscan_available(x0, y0, x0 + N, y0 - 1, v.W, v.H) && get(x0 + N, y0 - 1, b0);
  const bool fB0 = avB0 && !(avB1 && b1 == b0);
  if (fB0) {
    if (b0 == mv) return n;
    if (++n == maxc) return -1;
  }
  const bool avA0 = zscan_available(x0, y0, x0 - 1, y0 + N, v.W, v.H) && get(x0 - 1, y0 + N, a0);
  const bool fA0 = avA0 && !(avA1 && a1 == a0);
  if (fA0) {
    if (a0 == mv) return n;
    if (++n == maxc) return -1;
  }
  const bool avB2 = x0 > 0 && y0 > 0 && get(x0 - 1, y0 - 1, b2);
  if (avB2 && !(avA1 && a1 == b2) && !(avB1 && b1 == b2) && (int)avA1 + (int)fB1 + (int)fB0 + (int)fA0 < 4) {
    if (b2 == mv) return n;
    if (++n == maxc) return -1;
  }
  return (mv.x == 0 && mv.y == 0) ? n : -1;
}

__device__ __forceinline__ int mvd_cost(int d) {
  int a = d < 0 ? -d : d;
  if (a == 0) return 1;
  if (a == 1) return 3;
  int vv = a - 2, k = 1, n = 0;
  while (vv >= (1 << k)) {
    vv -= 1 << k;
    ++k;
    ++n;
  }
  return 3 + n + 1 + k;
}

// ------------------------------------------------------------------ binariser (one CTB)
struct CtbBinariser {
  const SegView v;  // by value: a reference put the view in scratch and its plane pointers
                    // (LDS in k_ent_bin) became flat accesses
  const EntropyPic& p;
  TokSink& s;
  const BinTables& T;  // LDS
  bool err = false;

  __device__ __forceinline__ int unit(int x, int y) const { return unit_of(v, x, y); }
  __device__ __forceinline__ void bin(int b, int ctx) { s.bin(b, ctx); }
  __device__ __forceinline__ int skip_inc(int x0, int y0) const {
    int inc = 0;
    if (x0 > 0 && v.skip[unit(x0 - 1, y0)]) ++inc;
    if (y0 > 0 && v.skip[unit(x0, y0 - 1)]) ++inc;
    return inc;
  }

  __device__ __forceinline__ void sao(int cx, int cy) {
    const uint32_t off = sao_off_param();
    const uint32_t* q = v.sao ? v.sao + 3 * (cy * v.wc + cx) : nullptr;
    const uint32_t pr[3] = {q ? q[0] : off, q ? q[1] : off, q ? q[2] : off};
    auto same = [&](const uint32_t* o) { return o[0] == pr[0] && o[1] == pr[1] && o[2] == pr[2]; };
    if (cx > 0) {
      const bool m = q && same(q - 3);
      bin(m, CTX_SAO_MERGE);
      if (m) return;
    }
    if (cy > 0) {
      const bool m = q && same(q - 3 * v.wc);
      bin(m, CTX_SAO_MERGE);
      if (m) return;
    }
    for (int c = 0; c < 3; ++c) {
      const int t = sao_type(pr[c]);
      if (c < 2) {
        bin(t != 0, CTX_SAO_TYPE);
        if (t) s.bypass(t == 2, 1);
      }
      if (!t) continue;
      for (int i = 0; i < 4; ++i) {  // sao_offset_abs: TR, cMax 7
        const int a = tv_abs(sao_offset(pr[c], i));
        if (a < kSaoMaxOff) s.bypass(((1u << a) - 1) << 1, a + 1);
        else s.bypass((1u << a) - 1, a);
      }
      if (t == 1) {
        for (int i = 0; i < 4; ++i)
          if (sao_offset(pr[c], i)) s.bypass(sao_offset(pr[c], i) < 0, 1);
        s.bypass((uint32_t)sao_class(pr[c]), 5);
      } else if (c < 2) {
        s.bypass((uint32_t)sao_class(pr[c]), 2);
      }
    }
  }

  __device__ __forceinline__ void merge_idx_syntax(int idx) {
    if (p.max_merge <= 1) return;
    bin(idx > 0, CTX_MERGE_IDX);
    for (int i = 1; i < p.max_merge - 1 && idx >= i; ++i) s.bypass(idx > i, 1);
  }
  __device__ __forceinline__ void eg1(uint32_t val) {
    int k = 1;
    while (val >= (1u << k)) {
      s.bypass(1, 1);
      val -= 1u << k;
      ++k;
    }
    s.bypass(0, 1);
    s.bypass(val, k);
  }
  __device__ __forceinline__ void mvd(int dx, int dy) {
    const int ax = dx < 0 ? -dx : dx, ay = dy < 0 ? -dy : dy;
    bin(ax > 0, CTX_MVD_G0);
    bin(ay > 0, CTX_MVD_G0);
    if (ax > 0) bin(ax > 1, CTX_MVD_G1);
    if (ay > 0) bin(ay > 1, CTX_MVD_G1);
    if (ax > 0) {
      if (ax > 1) eg1((uint32_t)(ax - 2));
      s.bypass(dx < 0, 1);
    }
    if (ay > 0) {
      if (ay > 1) eg1((uint32_t)(ay - 2));
      s.bypass(dy < 0, 1);
    }
  }

  // ---- residual_coding (7.3.8.11) from the compact levels ----
  struct Tb {
    uint64_t nz, m;
    int base, gw, skipc;
    const int16_t* groups;
  };
  __device__ __forceinline__ void tb_view(int c, int x, int y, int log2N, Tb& t) const {
    const int nsb = 1 << (log2N - 2), sh = c ? 4 : 5;
    t.gw = c ? 4 : 8;
    const int ctb = (y >> sh) * v.wc + (x >> sh);
    const uint64_t my = v.mask_y[ctb];
    t.m = c ? (uint64_t)v.mask_c[ctb] : my;
    t.base = (c == 2 ? 16 : 0) + ((y & ((1 << sh) - 1)) >> 2) * t.gw + ((x & ((1 << sh) - 1)) >> 2);
    const uint64_t row = (1ull << nsb) - 1;
    t.nz = 0;
    for (int ys = 0; ys < nsb; ++ys) t.nz |= ((t.m >> (t.base + ys * t.gw)) & row) << (ys * nsb);
    t.groups = v.packed + (long)v.sb_off[ctb] * 16;
    t.skipc = c ? __popcll(my) : 0;
  }
  __device__ __forceinline__ const int16_t* group_of(const Tb& t, int log2N, int r) const {
    const int bit = t.base + (r >> (log2N - 2)) * t.gw + (r & ((1 << (log2N - 2)) - 1));
    return t.groups + (long)(t.skipc + __popcll(t.m & ((1ull << bit) - 1))) * 16;
  }
  // bit n: scan position n of the group (levels in lo / hi) is non-zero
  __device__ __forceinline__ unsigned sig_mask(const uint4& lo, const uint4& hi, int scanIdx) const {
    const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    unsigned raster = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      raster |= (((w[j] & 0xffffu) != 0) ? 1u : 0u) << (2 * j) | (((w[j] >> 16) != 0) ? 1u : 0u) << (2 * j + 1);
    unsigned m = 0;
    const uint8_t* sc = T.scan4[scanIdx];
#pragma unroll
    for (int n = 0; n < 16; ++n) m |= ((raster >> sc[n]) & 1u) << n;
    return m;
  }
  __device__ __forceinline__ static void load_group(const int16_t* g, uint4& lo, uint4& hi) {
    lo = *reinterpret_cast<const uint4*>(g);
    hi = *reinterpret_cast<const uint4*>(g + 8);
  }
  __device__ __forceinline__ void last_prefix(int pos, int log2N, int cIdx, int base) {
    const int prefix = T.group_idx[pos];
    int off, shift;
    if (cIdx == 0) {
      off = 3 * (log2N - 2) + ((log2N - 1) >> 2);
      shift = (log2N + 1) >> 2;
    } else {
      off = 15;
      shift = log2N - 2;
    }
    const int cmax = (log2N << 1) - 1;
    for (int i = 0; i < prefix; ++i) bin(1, base + off + (i >> shift));
    if (prefix < cmax) bin(0, base + off + (prefix >> shift));
  }
  __device__ __forceinline__ void last_suffix(int pos) {
    const int prefix = T.group_idx[pos];
    if (prefix > 3) s.bypass((uint32_t)(pos - T.min_in_group[prefix]), (prefix >> 1) - 1);
  }
  __device__ __forceinline__ void remaining(int val, int rice) {
    if (val < (4 << rice)) {
      const int pfx = val >> rice;
      s.bypass(((1u << (pfx + 1)) - 2) << rice | (uint32_t)(val & ((1 << rice) - 1)), pfx + 1 + rice);
    } else {
      int k = rice + 1, ones = 0;
      uint32_t r = (uint32_t)(val - (4 << rice));
      while (r >= (1u << k)) {
        r -= 1u << k;
        ++k;
        ++ones;
      }
      const int np = 4 + ones + 1;
      for (int done = 0; done < np - 1;) {  // np - 1 ones, then a zero
        const int take = tv_min(np - 1 - done, 16);
        s.bypass((1u << take) - 1, take);
        done += take;
      }
      s.bypass(0, 1);
      s.bypass(r, k);
    }
  }
  __device__ __forceinline__ void residual(const Tb& t, int log2N, int cIdx, int scanIdx) {
    const int nsb = 1 << (log2N - 2), lsb = log2N - 2;
    if (!t.nz) {
      err = true;
      return;
    }
    // last significant sub-block in scan order, then its last non-zero position
    const uint8_t* sbpos = T.sbpos[lsb][scanIdx];
    const uint8_t* sbinv = T.sbinv[lsb][scanIdx];
    int lastSb = 0;
    for (uint64_t bb = t.nz; bb; bb &= bb - 1) lastSb = tv_max(lastSb, (int)sbinv[__ffsll((long long)bb) - 1]);
    const int lxs = sbpos[lastSb] & (nsb - 1), lys = sbpos[lastSb] >> lsb;
    uint4 llo, lhi;
    load_group(group_of(t, log2N, lys * nsb + lxs), llo, lhi);
    const unsigned lastMask = sig_mask(llo, lhi, scanIdx);
    const int lastN = 31 - __clz(lastMask);
    {
      const int pc = T.scan4[scanIdx][lastN];
      int lx = (lxs << 2) + (pc & 3), ly = (lys << 2) + (pc >> 2);
      if (scanIdx == 2) {
        const int tmp = lx;
        lx = ly;
        ly = tmp;
      }
      last_prefix(lx, log2N, cIdx, CTX_LAST_X);
      last_prefix(ly, log2N, cIdx, CTX_LAST_Y);
      last_suffix(lx);
      last_suffix(ly);
    }
    const int sizeOff = log2N == 3 ? (scanIdx == 0 ? 9 : 15) : (cIdx == 0 ? 21 : 12);
    const int compOff = CTX_SIG + (cIdx ? 27 : 0);
    uint64_t coded = 0;
    int c1 = 1;
    for (int i = lastSb; i >= 0; --i) {
      const int r = sbpos[i], xs = r & (nsb - 1), ys = r >> lsb;
      const bool any = (t.nz >> r) & 1;
      const int right = xs < nsb - 1 ? (int)((coded >> (r + 1)) & 1) : 0;
      const int below = ys < nsb - 1 ? (int)((coded >> (r + nsb)) & 1) : 0;
      bool inferDc = false;
      if (i < lastSb && i > 0) {
        bin(any ? 1 : 0, CTX_CSBF + (right | below) + (cIdx ? 2 : 0));
        if (!any) continue;
        inferDc = true;
      }
      coded |= 1ull << r;
      uint4 lo = llo, hi = lhi;
      if (i != lastSb && any) load_group(group_of(t, log2N, r), lo, hi);
      const unsigned m = i == lastSb ? lastMask : (any ? sig_mask(lo, hi, scanIdx) : 0u);
      const int prevCsbf = right + (below << 1);
      const int add = log2N == 2 ? compOff : compOff + sizeOff + ((cIdx == 0 && i > 0) ? 3 : 0);
      const int nStart = (i == lastSb) ? lastN - 1 : 15;
      const bool dcInferred = inferDc && (m & ((2u << nStart) - 2)) == 0;
      const uint8_t* pat = log2N == 2 ? T.map4[scanIdx] : T.sigpat[scanIdx][prevCsbf];
      for (int n = nStart; n >= 1; --n) bin((m >> n) & 1, add + pat[n]);
      if (nStart >= 0 && !dcInferred) bin(m & 1, (log2N > 2 && i == 0) ? compOff : add + pat[0]);
      // levels in reverse scan order, read from the group's registers (two passes: greater-1
      // / greater-2 flags and signs, then the remaining absolute levels)
      const uint8_t* sc = T.scan4[scanIdx];
      int ctxSet = (i > 0 && cIdx == 0) ? 2 : 0;
      if (c1 == 0) ++ctxSet;
      c1 = 1;
      const int g1base = CTX_G1 + 4 * ctxSet + (cIdx ? 16 : 0);
      uint32_t sbits = 0;
      int cnt = 0, g2 = -1;
      for (unsigned sm = m; sm; ++cnt) {
        const int n = 31 - __clz(sm);
        sm &= ~(1u << n);
        const int x = level_at(lo, hi, sc[n]), a = x < 0 ? -x : x;
        sbits = (sbits << 1) | (x < 0 ? 1u : 0u);
        if (cnt < 8) {
          const int bn = a > 1;
          bin(bn, g1base + c1);
          if (bn) {
            c1 = 0;
            if (g2 < 0) g2 = a > 2;
          } else if (c1 > 0 && c1 < 3) {
            ++c1;
          }
        }
      }
      if (g2 >= 0) bin(g2, CTX_G2 + ctxSet + (cIdx ? 4 : 0));
      if (cnt) s.bypass(sbits, cnt);
      int rice = 0, k = 0;
      bool firstC2 = true;
      for (unsigned sm = m; sm; ++k) {
        const int n = 31 - __clz(sm);
        sm &= ~(1u << n);
        const int x = level_at(lo, hi, sc[n]), a = x < 0 ? -x : x;
        const int base = (k < 8) ? (firstC2 ? 3 : 2) : 1;
        if (a >= base) {
          remaining(a - base, rice);
          if (a > 3 * (1 << rice)) rice = tv_min(rice + 1, 4);
        }
        if (a >= 2) firstC2 = false;
      }
    }
  }

  __device__ __forceinline__ bool tu_split(int x0, int y0) const { return v.tu && v.tu[unit(x0, y0)]; }

  // transform_tree (7.3.8.8) of a CU: depth 0, or (inter CUs with RQT) four depth-1 TUs.  One
  // residual call site and one TU loop, so the whole binariser inlines into registers.
  __device__ __forceinline__ void transform_tree(int x0, int y0, int log2, bool intra, int mode) {
    bool split = false;
    if (!intra && p.rqt) {  // split_transform_flag of an inter CU (depth 0, ctx 5 - log2)
      split = tu_split(x0, y0);
      bin(split ? 1 : 0, CTX_SPLIT_TF + 5 - log2);
    }
    const int h = 1 << (log2 - 1), l = split ? log2 - 1 : log2;
    int cb0 = 0, cr0 = 0;
    if (split) {  // chroma cbfs at depth 0: the OR of the quadrants'
      for (int q = 0; q < 4; ++q) {
        const int c = v.cbf[unit(x0 + (q & 1) * h, y0 + (q >> 1) * h)];
        cb0 |= (c >> 1) & 1;
        cr0 |= (c >> 2) & 1;
      }
      bin(cb0, CTX_CBF_CHROMA + 0);
      bin(cr0, CTX_CBF_CHROMA + 0);
    }
    const int cmode = intra ? mode : 0;  // chroma: DM (intra_chroma_pred_mode 4)
    for (int q = 0; q < (split ? 4 : 1); ++q) {
      const int x = x0 + (q & 1) * h, y = y0 + (q >> 1) * h;
      const int cbf = v.cbf[unit(x, y)];
      const int cl = cbf & 1, cb = (cbf >> 1) & 1, cr = (cbf >> 2) & 1;
      if (split) {
        if (cb0) bin(cb, CTX_CBF_CHROMA + 1);
        if (cr0) bin(cr, CTX_CBF_CHROMA + 1);
        bin(cl, CTX_CBF_LUMA + 0);
      } else {
        bin(cb, CTX_CBF_CHROMA + 0);  // log2 >= 3: chroma cbfs coded at depth 0
        bin(cr, CTX_CBF_CHROMA + 0);
        if (intra || cb || cr) bin(cl, CTX_CBF_LUMA + 1);
        else if (!cl) err = true;  // inter CU with rqt_root_cbf = 1 but no residual
      }
      for (int c = 0; c < 3; ++c) {
        if (!((cbf >> c) & 1)) continue;
        const int lc = c ? l - 1 : l;
        Tb t;
        tb_view(c, c ? x >> 1 : x, c ? y >> 1 : y, lc, t);
        residual(t, lc, c, split ? 0 : scan_idx_for(intra, lc, c, c ? cmode : mode));
      }
    }
  }

  __device__ __forceinline__ void amvp_mvd(int x0, int y0, int N, int X, const Motion& m) {
    auto at = [&](int xn, int yn, Motion& o) {
      if (!zscan_available(x0, y0, xn, yn, v.W, v.H)) return false;
      const int un = unit(xn, yn);
      if (v.intra[un]) return false;
      o = motion_of(v, un);
      return true;
    };
    Mv mvp[2];
    if (p.type == 0) {
      amvp_candidates_b(x0, y0, N, N, X, p.ref_poc, p.poc, at, mvp);
    } else {
      auto f = [&](int xn, int yn, Mv& o) {
        Motion mm;
        if (!at(xn, yn, mm)) return false;
        o = mm.mv[0];
        return true;
      };
      amvp_candidates(x0, y0, N, N, f, mvp);
    }
    const Mv vv = m.mv[X];
    const int c0 = mvd_cost(vv.x - mvp[0].x) + mvd_cost(vv.y - mvp[0].y);
    const int c1 = mvd_cost(vv.x - mvp[1].x) + mvd_cost(vv.y - mvp[1].y);
    const int sel = c1 < c0 ? 1 : 0;
    mvd(vv.x - mvp[sel].x, vv.y - mvp[sel].y);
    bin(sel, CTX_MVP_FLAG);
  }

  // coding_unit (7.3.8.5): skip / merge / AMVP from the motion field (P and B), intra modes
  __device__ __forceinline__ void coding_unit(int x0, int y0, int log2) {
    const int u = unit(x0, y0), N = 1 << log2;
    const bool intra = v.intra[u] != 0;
    const int cbf = cu_cbf(v, x0, y0, log2);
    const bool islice = p.type == 2, bslice = p.type == 0;
    if (!islice) {
      const int merge_idx = intra ? -1 : v.midx[u];
      const bool skip = !intra && merge_idx >= 0 && cbf == 0;
      bin(skip ? 1 : 0, CTX_CU_SKIP + skip_inc(x0, y0));
      if (skip) {
        merge_idx_syntax(merge_idx);
        return;
      }
      bin(intra ? 1 : 0, CTX_PRED_MODE);  // pred_mode_flag
      if (!intra) {
        bin(1, CTX_PART_MODE);  // part_mode 2Nx2N
        bin(merge_idx >= 0 ? 1 : 0, CTX_MERGE_FLAG);
        if (merge_idx >= 0) {
          merge_idx_syntax(merge_idx);
        } else {
          const Motion m = motion_of(v, u);
          if (bslice) {  // inter_pred_idc: bin 0 (PRED_BI?) at ctx CtDepth, bin 1 (L1?) at ctx 4
            bin(m.dir == 3 ? 1 : 0, CTX_INTER_PRED_IDC + (kCtbLog2 - log2));
            if (m.dir != 3) bin(m.dir == 2 ? 1 : 0, CTX_INTER_PRED_IDC + 4);
          }
          for (int X = 0; X < 2; ++X)
            if ((m.dir >> X) & 1) amvp_mvd(x0, y0, N, X, m);
          bin(cbf ? 1 : 0, CTX_RQT_ROOT_CBF);
          if (!cbf) return;
        }
        transform_tree(x0, y0, log2, false, 0);
        return;
      }
    }
    if (log2 == kMinCbLog2) bin(1, CTX_PART_MODE);  // 2Nx2N
    const int mode = v.ipm[u];
    int candA = 1, candB = 1;
    if (x0 > 0 && v.intra[unit(x0 - 1, y0)]) candA = v.ipm[unit(x0 - 1, y0)];
    if (y0 > 0 && v.intra[unit(x0, y0 - 1)] && (y0 - 1) >= ((y0 >> kCtbLog2) << kCtbLog2))
      candB = v.ipm[unit(x0, y0 - 1)];
    int mpm[3];
    intra_mpm_list(candA, candB, mpm);
    const int idx = mpm[0] == mode ? 0 : (mpm[1] == mode ? 1 : (mpm[2] == mode ? 2 : -1));
    bin(idx >= 0 ? 1 : 0, CTX_PREV_INTRA);
    if (idx >= 0) {
      if (idx == 0) s.bypass(0, 1);
      else s.bypass(idx == 1 ? 2 : 3, 2);
    } else {  // rem_intra_luma_pred_mode: the mode minus the MPMs below it
      const int rem = mode - (mode > mpm[0]) - (mode > mpm[1]) - (mode > mpm[2]);
      s.bypass((uint32_t)rem, 5);
    }
    bin(0, CTX_CHROMA_PRED);  // intra_chroma_pred_mode = 4 (DM)
    transform_tree(x0, y0, log2, true, mode);
  }

  // coding_quadtree of the 32x32 CTB as a z-order walk (one split-flag and one coding_unit
  // call site), then the end-of-CTB syntax and the WPP marks
  __device__ __forceinline__ void ctb(int cx, int cy, bool sao_on) {
    if (sao_on) sao(cx, cy);
    const int X = cx << kCtbLog2, Y = cy << kCtbLog2;
    for (int z = 0; z < 16;) {
      const int x = X + 8 * ((z & 1) | ((z >> 1) & 2)), y = Y + 8 * (((z >> 1) & 1) | ((z >> 2) & 2));
      int l = z == 0 ? 5 : ((z & 3) == 0 ? 4 : 3);
      for (; l > kMinCbLog2; --l) {  // split_cu_flag of every node that starts here, top down
        const bool split = v.cu_log2[unit(x, y)] < l;
        const int depth = kCtbLog2 - l;
        int inc = 0;
        if (x > 0 && (kCtbLog2 - v.cu_log2[unit(x - 1, y)]) > depth) ++inc;
        if (y > 0 && (kCtbLog2 - v.cu_log2[unit(x, y - 1)]) > depth) ++inc;
        bin(split ? 1 : 0, CTX_SPLIT_CU + inc);
        if (!split) break;
      }
      coding_unit(x, y, l);
      z += 1 << (2 * (l - kMinCbLog2));
    }
    const bool last = cy == v.hc - 1 && cx == v.wc - 1;
    if (cx == 1) s.ctrl(kCtrlSync);  // 9.3.2.4 storage after the row's second CTB
    s.term(last ? 1 : 0);           // end_of_slice_segment_flag
    if (!last && cx == v.wc - 1) s.term(1);  // end_of_subset_one_bit
    if (cx == v.wc - 1) s.ctrl(kCtrlFlush);  // + byte_alignment() / slice trailing bits
  }
};

// ------------------------------------------------------------------ kernels
// Per CU: the merge candidate its motion matches (-1: none) and, for every unit it covers,
// the skip flag (the cu_skip_flag context of the CUs to its right / below).
__global__ void __launch_bounds__(256) k_ent_cu(EntropyArgs a) {
  const int b = blockIdx.y;
  const long u = (long)blockIdx.x * 256 + threadIdx.x;
  if (u >= a.g.usz) return;
  const SegView v = seg_view(a, b);
  const int x8 = (int)(u % v.w8), y8 = (int)(u / v.w8);
  const int l = v.cu_log2[u], s = 1 << (l - 3);
  if ((x8 & (s - 1)) || (y8 & (s - 1))) return;  // not the CU's top-left unit
  const int x0 = x8 * 8, y0 = y8 * 8, N = 8 * s;
  int midx = -1;
  if (!v.intra[u]) {
    if (a.pic.type == 1) {
      midx = merge_index_p(v, x0, y0, N, Mv{v.mv[2 * u], v.mv[2 * u + 1]}, a.pic.max_merge);
    } else {
      auto at = [&](int xn, int yn, Motion& o) {
        if (!zscan_available(x0, y0, xn, yn, v.W, v.H)) return false;
        const int un = unit_of(v, xn, yn);
        if (v.intra[un]) return false;
        o = motion_of(v, un);
        return true;
      };
      Motion cand[5];
      const int nc = merge_candidates_b(x0, y0, N, N, a.pic.max_merge, a.pic.ref_poc[0] == a.pic.ref_poc[1], at, cand);
      const Motion m = motion_of(v, (int)u);
      for (int i = 0; i < nc; ++i)
        if (cand[i] == m) {
          midx = i;
          break;
        }
    }
  }
  const uint8_t sk = (uint8_t)(!v.intra[u] && midx >= 0 && cu_cbf(v, x0, y0, l) == 0);
  uint8_t* skip = a.skip + (long)b * a.g.usz;
  for (int j = 0; j < s; ++j)
    for (int i = 0; i < s; ++i) skip[u + (long)j * v.w8 + i] = sk;
  a.midx[(long)b * a.g.usz + u] = (int8_t)midx;
}

// One thread per CTB: count (WRITE = false) or write its tokens.
// One thread per CTB.  REGION (the single full pass): the CTB's tokens into its fixed region
// (kEntRegionTokens) and its exact count.  !REGION (after the scan): only CTBs whose tokens
// did not fit binarise again, straight into the picture's token list; the others were moved by
// k_ent_place.  (A count pass + write pass binarised every CTB twice.)
// One workgroup per CTB row (one thread per CTB, 64 * ceil(wc / 64) threads).  The row's
// decision planes -- the 4 unit rows of the CTB row and the one above (left / upper / upper-
// right neighbours), all columns, a contiguous range of every plane -- are staged in LDS by
// the whole workgroup first, so the per-CTB syntax walk reads LDS instead of issuing chains
// of dependent global loads (one thread per CTB left every neighbour check a ~1 us round
// trip).  REGION (the single full pass): the CTB's tokens into its fixed region
// (kEntRegionTokens) and its exact count.  !REGION (after the scan): only rows with a CTB whose
// tokens did not fit binarise again, straight into the picture's token list; the others were
// moved by k_ent_place.  (A count pass + write pass binarised every CTB twice.)
struct BinStage {  // byte offsets of the staged planes in dynamic LDS (nu units each)
  int nu, cu, in, ipm, cbf, tu, sk, mi, dir, mv, mv1, bytes;
};
__host__ __device__ inline BinStage bin_stage(int w8, bool tu, bool bpic) {
  BinStage t;
  t.nu = 5 * w8;
  int o = 0;
  t.cu = o; o += t.nu;
  t.in = o; o += t.nu;
  t.ipm = o; o += t.nu;
  t.cbf = o; o += t.nu;
  t.sk = o; o += t.nu;
  t.mi = o; o += t.nu;
  t.tu = tu ? o : -1; o += tu ? t.nu : 0;
  t.dir = bpic ? o : -1; o += bpic ? t.nu : 0;
  o = (o + 15) & ~15;
  t.mv = o; o += 4 * t.nu;
  t.mv1 = bpic ? o : -1; o += bpic ? 4 * t.nu : 0;
  t.bytes = o;
  return t;
}
template <bool REGION>
__global__ void __launch_bounds__(256) k_ent_bin(EntropyArgs a) {
  __shared__ BinTables T;
  extern __shared__ __align__(16) uint8_t dyn[];
  const int b = blockIdx.y, nctu = a.g.wc * a.g.hc, wc = a.g.wc, w8 = a.g.w8;
  const int cy = blockIdx.x, cx = threadIdx.x;
  const int ctu = cy * wc + cx;
  const long i = (long)b * nctu + ctu;
  bool work = cx < wc;
  if (!REGION) {  // the whole workgroup leaves unless one of its CTBs overflowed
    work = work && !*a.status && a.ctb_cnt[i] > kEntRegionTokens;
    if (__syncthreads_or(work) == 0) return;
  }
  const int nt = blockDim.x;
  {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(&c_tab);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&T);
    for (int k = threadIdx.x; k < (int)(sizeof(BinTables) / 4); k += nt) dst[k] = src[k];
  }
  SegView v = seg_view(a, b);
  const bool bpic = v.dir != nullptr;
  const BinStage L = bin_stage(w8, v.tu != nullptr, bpic);
  const int uy0 = cy > 0 ? 4 * cy - 1 : 0, nrows = 4 * cy + 4 - uy0;
  const long u0 = (long)uy0 * w8;  // first staged unit
  const int nw = nrows * w8 / 4;   // dwords of a byte plane's window (w8 is a multiple of 4)
  // the staging helpers return the window pointer (no reference into v: taking a field's
  // address put the whole view in scratch and every plane access became a flat one)
  auto stage8 = [&](int off, const uint8_t* p) -> const uint8_t* {
    if (off < 0) return p;  // only tu / dir are optional (bin_stage): the rest are always staged
    const uint32_t* g32 = reinterpret_cast<const uint32_t*>(p + u0);
    uint32_t* l32 = reinterpret_cast<uint32_t*>(dyn + off);
    for (int k = threadIdx.x; k < nw; k += nt) l32[k] = g32[k];
    return dyn + off;  // unit_of subtracts v.ubase: unit(x, y) indexes the window (no pointer below dyn)
  };
  auto stage16 = [&](int off, const int16_t* p) -> const int16_t* {
    if (off < 0) return p;
    const uint32_t* g32 = reinterpret_cast<const uint32_t*>(p + 2 * u0);
    uint32_t* l32 = reinterpret_cast<uint32_t*>(dyn + off);
    for (int k = threadIdx.x; k < nrows * w8; k += nt) l32[k] = g32[k];
    return reinterpret_cast<const int16_t*>(dyn + off);
  };
  // planes that are always staged take the offset unconditionally (max(off, 0) is off), so
  // the compiler sees LDS pointers (ds_* instead of flat_* accesses in the binariser)
  v.cu_log2 = stage8(tv_max(L.cu, 0), v.cu_log2);
  v.intra = stage8(tv_max(L.in, 0), v.intra);
  v.ipm = stage8(tv_max(L.ipm, 0), v.ipm);
  v.cbf = stage8(tv_max(L.cbf, 0), v.cbf);
  v.skip = stage8(tv_max(L.sk, 0), v.skip);
  v.midx = reinterpret_cast<const int8_t*>(stage8(tv_max(L.mi, 0), reinterpret_cast<const uint8_t*>(v.midx)));
  v.tu = stage8(L.tu, v.tu);
  v.dir = stage8(L.dir, v.dir);
  v.mv = stage16(tv_max(L.mv, 0), v.mv);
  v.mv1 = stage16(L.mv1, v.mv1);
  v.ubase = u0;
  __syncthreads();
  if (!work) return;
  uint32_t* out;
  int cap;
  if (REGION) {
    out = a.regions + i * kEntRegionTokens;
    cap = kEntRegionTokens;
  } else {
    long base = 0;
    for (int k = 0; k < b; ++k) base += a.seg_tok[k];
    out = a.tokens + base + a.ctb_off[i];
    cap = 1 << 30;
  }
  TokSink s{out, cap};
  CtbBinariser z{v, a.pic, s, T};
  z.ctb(cx, cy, a.pic.sao != 0);
  s.flush_c();
  s.flush_b();
  if (z.err) atomicOr(a.status, 2);
  if (REGION) a.ctb_cnt[i] = s.n;
}

// the CTBs whose tokens fit their region: region -> the picture's token list (one wave per CTB)
__global__ void __launch_bounds__(256) k_ent_place(EntropyArgs a) {
  const int b = blockIdx.y, nctu = a.g.wc * a.g.hc;
  const int ctu = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (ctu >= nctu || *a.status) return;
  const long i = (long)b * nctu + ctu;
  const int n = a.ctb_cnt[i];
  if (n > kEntRegionTokens) return;  // binarised again by k_ent_bin<false>
  long base = 0;
  for (int k = 0; k < b; ++k) base += a.seg_tok[k];
  uint32_t* dst = a.tokens + base + a.ctb_off[i];
  const uint32_t* src = a.regions + i * kEntRegionTokens;
  for (int k = lane; k < n; k += 64) dst[k] = src[k];
}

// exclusive scan of the CTB token counts, one workgroup per segment; capacity check
__global__ void __launch_bounds__(1024) k_ent_scan(EntropyArgs a) {
  const int b = blockIdx.x, tid = threadIdx.x, nctu = a.g.wc * a.g.hc;
  __shared__ int part[1024];
  const int per = (nctu + 1023) / 1024;
  const int lo = tid * per, hi = tv_min(nctu, lo + per);
  const int* cnt = a.ctb_cnt + (long)b * nctu;
  int s = 0;
  for (int k = lo; k < hi; ++k) s += cnt[k];
  part[tid] = s;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    const int vv = tid >= o ? part[tid - o] : 0;
    __syncthreads();
    part[tid] += vv;
    __syncthreads();
  }
  int run = tid ? part[tid - 1] : 0;
  int* off = a.ctb_off + (long)b * nctu;
  for (int k = lo; k < hi; ++k) {
    off[k] = run;
    run += cnt[k];
  }
  if (tid == 1023) a.seg_tok[b] = part[1023];
}

// capacity check over all segments (one thread): the token and staging buffers
__global__ void k_ent_check(EntropyArgs a, int B) {
  long t = 0;
  for (int k = 0; k < B; ++k) t += a.seg_tok[k];
  if (t > a.tok_cap) atomicOr(a.status, 1);
}

// ---- arithmetic coder -------------------------------------------------------------------

// Staging of a row's output: 4-aligned, 3 bytes per token + 20 of slack per row (a context-coded
// token is at most 3 bins x 6 renormalisation bits, a bypass token 16 bits; the flush adds <= 4
// bytes), so rows never overlap.
__device__ __forceinline__ long stage_off(long tpos, long row_idx) { return (3 * tpos + 20 * row_idx + 3) & ~3L; }

constexpr int kCtxN = CTX_COUNT;
constexpr int kTokT = 64;   // token ring entries
constexpr int kTokK = 32;   // tokens per refill


// One WAVE per CTB row (substream), one active lane: every value of the coder is wave-uniform
// (the compiler runs it on the scalar unit; context states and tables in LDS).  A lane-per-row
// layout executed the union of every row's path each iteration with two thirds of the rows
// still waiting on WPP (~1500 clocks per bin); this runs ~700 (TV_ENT_DEBUG).  (Context states
// in VGPRs via wave-uniform indexed moves measured slower: ~970.)  The WPP storage (9.3.2.4) goes to the row below through
// global memory: agent-scope relaxed stores (sc1), vmcnt(0), flag; the reader polls the flag and
// reads the contexts with agent-scope loads -- no fences (an agent fence is a whole-L2 write-back
// or invalidate on this XCD).  Workgroups are dispatched in
// row order, so a row only ever waits on a row that is already running.  Tokens come through a
// 64-entry LDS ring refilled 32 at a time (a token load kept in registers across the loop's
// branches forces a vmcnt(0) wait at its use); output bytes leave as dword stores.
__global__ void __launch_bounds__(64) k_ent_ac(EntropyArgs a) {
  __shared__ uint8_t lps[256], tlps[64], ctx[kEntCtx];
  for (int k = threadIdx.x; k < 256; k += 64) lps[k] = a.tab->lps[k];
  tlps[threadIdx.x] = a.tab->tlps[threadIdx.x];
  __syncthreads();
  if (threadIdx.x != 0) return;
  __builtin_amdgcn_s_setprio(3);  // a latency-bound chain beside the analysis waves
  const int b = blockIdx.y;
  const int wc = a.g.wc, hc = a.g.hc, nctu = wc * hc;
  __shared__ uint4 tring[kTokT / 4];
  const uint32_t* tring32 = reinterpret_cast<const uint32_t*>(tring);
  int* wflag = a.wflag + (long)b * hc;
  uint32_t* wctx = reinterpret_cast<uint32_t*>(a.wctx + (long)b * hc * kEntCtx);
  // rows blockIdx.x, + gridDim.x, ...: fewer waves per picture than rows, so fewer of them sit
  // resident waiting for the WPP diagonal.  With more than one row per wave, wave 0's second
  // row waits on the last wave (dispatched after it): a picture's <= 256 waves are co-resident
  // on 256 CUs as long as the analysis waves drain, and the wait times out into the host path.
  auto code_row = [&](const int row) {
  if (*a.status) {  // the binariser gave up on this picture: the host codes it
    __hip_atomic_store(&wflag[row], 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  long tbase = 0;
  for (int k = 0; k < b; ++k) tbase += a.seg_tok[k];
  const int* off = a.ctb_off + (long)b * nctu;
  const long tpos = tbase + off[row * wc];
  long ntok = (row + 1 < hc ? tbase + off[(row + 1) * wc] : tbase + a.seg_tok[b]) - tpos;
  uint32_t* out = reinterpret_cast<uint32_t*>(a.stage + stage_off(tpos, (long)b * hc + row));
  long head = tpos, tail = tpos & ~3L;  // next token to code / to load (whole uint4s)
  const uint4* gtok = reinterpret_cast<const uint4*>(a.tokens);
  auto refill = [&]() {
    uint4 v[kTokK / 4];
#pragma unroll
    for (int k = 0; k < kTokK / 4; ++k) v[k] = gtok[(tail >> 2) + k];
#pragma unroll
    for (int k = 0; k < kTokK / 4; ++k) tring[((tail >> 2) + k) & (kTokT / 4 - 1)] = v[k];
    tail += kTokK;
  };
  refill();
  refill();
  auto abort_row = [&](int code) {
    atomicOr(a.status, code);
    __hip_atomic_store(&wflag[row], 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  const unsigned long long w0 = wall_clock64();
  // contexts: row 0 from the init table, else the row above's after its CTB 1
  const uint32_t* src;
  if (row == 0) {
    src = reinterpret_cast<const uint32_t*>(a.tab->init[a.pic.init_type][clip3(0, 51, (int)a.dec.qp[b])]);
  } else {
    int f = 0;
    // agent-scope polls go past the XCD's L2 to the fabric, all rows of a picture on one line:
    // a few quick polls, then ~3 us apart (a row waits ~2 CTBs of every row above it)
    for (int spin = 0; (f = __hip_atomic_load(&wflag[row - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) == 0;
         ++spin) {
      if (spin > (1 << 23)) {  // ~25 s: the row above never came (never expected)
        abort_row(32);
        return;
      }
      if (spin < 8)
        __builtin_amdgcn_s_sleep(4);
      else
        __builtin_amdgcn_s_sleep(127);
    }
    if (f != 1) {  // the row above aborted: so does this one
      __hip_atomic_store(&wflag[row], 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    src = wctx + (long)(row - 1) * (kEntCtx / 4);
  }
  uint32_t* ctx32 = reinterpret_cast<uint32_t*>(ctx);
  if (row == 0) {
#pragma unroll
    for (int i = 0; i < kEntCtx / 4; ++i) ctx32[i] = src[i];
  } else {  // agent-scope loads (sc1): the row above may run on another XCD
    uint32_t t[kEntCtx / 4];
#pragma unroll
    for (int i = 0; i < kEntCtx / 4; ++i) t[i] = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int i = 0; i < kEntCtx / 4; ++i) ctx32[i] = t[i];
  }
  // coder state (CabacEncoder): low, range, bits left, outstanding bytes, buffered byte
  uint32_t low = 0, range = 510, buffered = 0xff;
  int bl = 23, nbuf = 0, pos = 0;
  uint32_t ow = 0;  // output bytes not yet stored (little-endian = memory order)
  const unsigned long long w1 = wall_clock64(), c1 = clock64();
  long nctxbins = 0, ntoks = 0;
  auto put = [&](uint32_t byte) {
    ow |= (byte & 255) << (8 * (pos & 3));
    if ((++pos & 3) == 0) {
      out[(pos >> 2) - 1] = ow;
      ow = 0;
    }
  };
  auto write_out = [&]() {  // CabacEncoder::write_out
    const uint32_t lead = low >> (24 - bl);
    bl += 8;
    low &= 0xffffffffu >> bl;
    if (lead == 0xff) {
      nbuf++;
    } else if (nbuf > 0) {
      const uint32_t carry = lead >> 8;
      put(buffered + carry);
      buffered = lead & 0xff;
      const uint32_t byte = (0xff + carry) & 0xff;
      for (; nbuf > 1; --nbuf) put(byte);
    } else {
      nbuf = 1;
      buffered = lead;
    }
  };
  // a row longer than its token count is a corrupt token stream -- abort, never hang
  bool synced = false;
  while (true) {
    if (ntok-- <= 0) {  // no FLUSH before the row's tokens ran out
      abort_row(4);
      return;
    }
    if (tail - head < kTokK) refill();
    const uint32_t tok = __builtin_amdgcn_readfirstlane(tring32[head & (kTokT - 1)]);
    ++head;
    ++ntoks;
    const uint32_t ty = tok >> 30;
    if (ty == 0) {  // 1..3 context-coded bins (CabacEncoder::bin_step)
      const int nbins = (tok >> 27) & 3;
      nctxbins += nbins;
      for (int k = 0; k < nbins; ++k) {
        const uint32_t f = (tok >> (9 * k)) & 511;
        const int c = (int)(f & 255);
        const int sv = ctx[c];
        const int st = sv & 63, mps = sv >> 6;
        const uint32_t lp = lps[st * 4 + ((range >> 6) & 3)];
        int nsv;
        const uint32_t rmps = range - lp;
        if ((int)(f >> 8) != mps) {  // LPS
          const int nb = __clz(lp) - 23;
          low = (low + rmps) << nb;
          range = lp << nb;
          bl -= nb;
          nsv = tlps[st] | ((mps ^ (st == 0 ? 1 : 0)) << 6);
        } else {
          const int nb = __clz(rmps) - 23;  // 0 or 1
          low <<= nb;
          range = rmps << nb;
          bl -= nb;
          nsv = (st < 62 ? st + 1 : st) | (mps << 6);
        }
        ctx[c] = (uint8_t)nsv;
        if (bl < 12) write_out();
      }
    } else if (ty == 1) {  // bypass bins, MSB first, <= 8 per step (encode_bypass_bins)
      int n = (tok >> 16) & 31;
      while (n > 0) {
        const int m = n > 8 ? 8 : n;
        n -= m;
        low = (low << m) + range * ((tok >> n) & ((1u << m) - 1));
        bl -= m;
        if (bl < 12) write_out();
      }
    } else if (ty == 2) {  // terminating bin (encode_terminate)
      range -= 2;
      if (tok & 1) {
        low += range;
        low <<= 7;
        range = 2 << 7;
        bl -= 7;
        if (bl < 12) write_out();
      } else if (range < 256) {
        low <<= 1;
        range <<= 1;
        bl--;
        if (bl < 12) write_out();
      }
    } else if ((tok & 0xff) == kCtrlSync) {  // 9.3.2.4 storage for the row below
      uint32_t* dst = wctx + (long)row * (kEntCtx / 4);
      // agent-scope stores (sc1, written through to the fabric), completed before the flag:
      // an agent release fence here wrote back the whole L2 of the XCD for every row, which
      // cost the concurrently running analysis kernels ~9 % of the step
      uint32_t t[kEntCtx / 4];
#pragma unroll
      for (int i = 0; i < kEntCtx / 4; ++i) t[i] = ctx32[i];
#pragma unroll
      for (int i = 0; i < kEntCtx / 4; ++i) __hip_atomic_store(dst + i, t[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(&wflag[row], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      synced = true;
    } else {  // finish() + '1' + byte alignment (end_of_subset_one_bit / slice trailing bits)
      if ((low >> (32 - bl)) != 0) {
        put(buffered + 1);
        for (; nbuf > 1; --nbuf) put(0x00);
        low -= 1u << (32 - bl);
      } else {
        if (nbuf > 0) put(buffered);
        for (; nbuf > 1; --nbuf) put(0xff);
      }
      const int nb = 24 - bl;  // 1..12 bits of low >> 8, then the '1', then zeros
      uint32_t v = (((low >> 8) & ((1u << nb) - 1)) << 1) | 1u;
      int t = nb + 1;
      const int pad = (8 - (t & 7)) & 7;
      v <<= pad;
      t += pad;
      while (t > 0) {
        t -= 8;
        put((v >> t) & 0xff);
      }
      uint8_t* o8 = reinterpret_cast<uint8_t*>(out);
      for (int k = pos & ~3; k < pos; ++k) o8[k] = (uint8_t)(ow >> (8 * (k & 3)));
      a.row_bytes[(long)b * hc + row] = pos;
      if (!synced) abort_row(4);  // a substream that never stored its contexts (corrupt stream)
      if (a.dbg) {  // TV_ENT_DEBUG: rows, context bins, tokens, coding clocks, wait ticks, max row span
        atomicAdd(&a.dbg[0], 1ull);
        atomicAdd(&a.dbg[1], (unsigned long long)nctxbins);
        atomicAdd(&a.dbg[2], (unsigned long long)ntoks);
        atomicAdd(&a.dbg[3], clock64() - c1);
        atomicAdd(&a.dbg[4], w1 - w0);
        atomicMax(&a.dbg[5], wall_clock64() - w0);
      }
      break;
    }
  }
  };
  for (int row = blockIdx.x; row < hc; row += gridDim.x) code_row(row);
}

// ---- lane-per-substream coder --------------------------------------------------------------
// One WAVE per CTB row index r, one LANE per segment: lane b codes substream (b, r).  Rows of
// different segments are independent, so every lane of the wave is busy (the single-lane
// coder above keeps 816 mostly idle waves resident at the 1080p bench shape; this one 34).
// The WPP storage after CTB 1 (9.3.2.4) goes from lane b of wave r - 1 to lane b of wave r
// through global memory (agent-scope stores / loads + flag, as above).
//
// Every lane executes one coder OPERATION per iteration -- a context-coded bin, a bypass run
// of up to 16 bins, or a terminating bin -- in one branch-free form:
//   low = ((low << pre) + add) << post,  range = nr << post,  bits_left -= pre + post,
//   post = clz(nr) - 23
// (bypass: pre = n, add = range * bins, nr = range; context bin: pre = 0, add = LPS ? range -
// rLPS : 0, nr = LPS ? rLPS : range - rLPS; terminate: pre = 0, add = bin ? range - 2 : 0, nr =
// bin ? 2 : range - 2).  `low` is 64-bit so a whole 16-bin bypass run fits before the byte
// output (CabacEncoder::write_out, at most twice per operation).  Bytes depend only on the
// sequence of interval updates, not on when they are written out, so the output is the host
// writer's byte for byte.
//
// LDS, per wave: the context states as [ctx][lane] dwords (a lane's reads hit bank lane % 32
// whatever the context: conflict-free), a per-lane token ring [slot][lane] refilled 16 tokens
// at a time one block of iterations ahead (the dwordx4 loads of block k are stored into the
// ring at block k + 1, so their latency hides behind 8 iterations), and the rLPS / transIdxLps
// tables (rLPS of the four range quarters packed in one dword per state).
constexpr int kLnRing = 64;  // token slots per lane
constexpr int kLnRefill = 16;
constexpr int kLnBlock = 8;  // iterations between refills (<= kLnRefill / tokens per iteration)

__global__ void __launch_bounds__(64) k_ent_ac_lanes(EntropyArgs a, int B) {
  __shared__ uint32_t ctxL[kEntCtx * 64];
  __shared__ uint32_t ring[kLnRing * 64];
  __shared__ uint32_t lps4[64], tl[64];
  const int lane = threadIdx.x, row = blockIdx.x;
  const int b = blockIdx.y * 64 + lane;
  {
    uint32_t v = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) v |= (uint32_t)a.tab->lps[lane * 4 + q] << (8 * q);
    lps4[lane] = v;
    tl[lane] = a.tab->tlps[lane];
  }
  const int wc = a.g.wc, hc = a.g.hc, nctu = wc * hc;
  bool active = b < B;
  int* flag = a.wflag + (long)b * hc + row;
  auto abort_lane = [&](int code) {
    atomicOr(a.status, code);
    __hip_atomic_store(flag, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    active = false;
  };
  if (*a.status) {  // the binariser gave up on this picture: the host codes it
    if (active) __hip_atomic_store(flag, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  // the lane's token range: segments back to back (exclusive prefix of seg_tok over the wave)
  const int stok = active ? a.seg_tok[b] : 0;
  int pre_tok = stok;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(pre_tok, o, 64);
    if (lane >= o) pre_tok += t;
  }
  long tbase = pre_tok - stok;
  for (int k = 0; k < blockIdx.y * 64; ++k) tbase += a.seg_tok[k];  // lane groups before this one
  const int* off = a.ctb_off + (long)(active ? b : 0) * nctu;
  const long tpos = tbase + off[row * wc];
  const long tend = row + 1 < hc ? tbase + off[(row + 1) * wc] : tbase + stok;
  uint32_t* out = reinterpret_cast<uint32_t*>(a.stage + stage_off(tpos, (long)(active ? b : 0) * hc + row));
  const unsigned long long w0 = wall_clock64();
  // WPP: wait for the row above of every lane's segment (rows of a picture progress together)
  if (row > 0) {
    const int* up = flag - 1;
    for (int spin = 0;; ++spin) {
      const int f = active ? __hip_atomic_load(up, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 1;
      if (f == 2 && active) {  // the row above aborted: so does this one
        __hip_atomic_store(flag, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        active = false;
      }
      if (__all(f != 0)) break;
      if (spin > (1 << 23)) {  // ~25 s: the row above never came (never expected)
        if (active && f == 0) abort_lane(32);
        break;
      }
      if (spin < 8)
        __builtin_amdgcn_s_sleep(4);
      else
        __builtin_amdgcn_s_sleep(127);
    }
  }
  // contexts: row 0 from the init table, else the row above's after its CTB 1
  if (active) {
    if (row == 0) {
      const uint8_t* src = a.tab->init[a.pic.init_type][clip3(0, 51, (int)a.dec.qp[b])];
      for (int c = 0; c < kEntCtx; c += 4) {
        const uint32_t w = *reinterpret_cast<const uint32_t*>(src + c);
#pragma unroll
        for (int q = 0; q < 4; ++q) ctxL[(c + q) * 64 + lane] = (w >> (8 * q)) & 255;
      }
    } else {
      const uint32_t* src = reinterpret_cast<const uint32_t*>(a.wctx + ((long)b * hc + row - 1) * kEntCtx);
      uint32_t t[kEntCtx / 4];
#pragma unroll
      for (int i = 0; i < kEntCtx / 4; ++i) t[i] = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int i = 0; i < kEntCtx / 4; ++i)
#pragma unroll
        for (int q = 0; q < 4; ++q) ctxL[(4 * i + q) * 64 + lane] = (t[i] >> (8 * q)) & 255;
    }
  }
  // token ring: 32 tokens now, then 16 per block one block ahead
  const uint4* gtok = reinterpret_cast<const uint4*>(a.tokens);
  long head = tpos, tail = tpos & ~3L;
  if (active) {
    uint4 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = gtok[(tail >> 2) + k];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int s0 = (int)((tail + 4 * k) & (kLnRing - 1));
      ring[(s0 + 0) * 64 + lane] = v[k].x;
      ring[(s0 + 1) * 64 + lane] = v[k].y;
      ring[(s0 + 2) * 64 + lane] = v[k].z;
      ring[(s0 + 3) * 64 + lane] = v[k].w;
    }
    tail += 32;
  }
  __syncthreads();  // tables (every lane wrote one entry)
  // coder state (CabacEncoder), low widened to 64 bits
  unsigned long long low = 0;
  uint32_t range = 510, buffered = 0xff, ow = 0;
  int bl = 23, nbuf = 0, pos = 0;
  int sub = 0;  // next bin of a context token
  long left = tend - tpos;  // tokens this substream may still consume
  bool synced = false;
  uint32_t tok = active ? ring[(head & (kLnRing - 1)) * 64 + lane] : 0;
  long nctxbins = 0, ntoks = 0;
  const unsigned long long w1 = wall_clock64(), c1 = clock64();
  auto put = [&](uint32_t byte) {
    ow |= (byte & 255) << (8 * (pos & 3));
    if ((++pos & 3) == 0) {
      out[(pos >> 2) - 1] = ow;
      ow = 0;
    }
  };
  uint4 pend[kLnRefill / 4];
  bool pending = false;
  while (__any(active)) {
    if (active && pending) {  // the block-ahead refill lands in the ring
#pragma unroll
      for (int k = 0; k < kLnRefill / 4; ++k) {
        const int s0 = (int)((tail + 4 * k) & (kLnRing - 1));
        ring[(s0 + 0) * 64 + lane] = pend[k].x;
        ring[(s0 + 1) * 64 + lane] = pend[k].y;
        ring[(s0 + 2) * 64 + lane] = pend[k].z;
        ring[(s0 + 3) * 64 + lane] = pend[k].w;
      }
      tail += kLnRefill;
    }
    pending = active && tail - head <= kLnRing - 2 * kLnRefill && tail < tend;
    if (pending) {
#pragma unroll
      for (int k = 0; k < kLnRefill / 4; ++k) pend[k] = gtok[(tail >> 2) + k];
    }
    for (int it = 0; it < kLnBlock; ++it) {
      if (!active) break;
      const uint32_t ty = tok >> 30;
      const bool isC = ty == 0, isB = ty == 1, isT = ty == 2;
      const int nbins = (tok >> 27) & 3;
      const bool more = isC && sub + 1 < nbins;  // the token has another bin after this one
      // the next token, read while this operation runs
      const uint32_t ntok = ring[((head + 1) & (kLnRing - 1)) * 64 + lane];
      const uint32_t f = (tok >> (9 * sub)) & 511;
      const int c = isC ? (int)(f & 255) : 0;
      const uint32_t sv = ctxL[c * 64 + lane];
      const uint32_t st = sv & 63, mps = (sv >> 6) & 1;
      const uint32_t lp = (lps4[st] >> (8 * ((range >> 6) & 3))) & 255;
      const uint32_t tlp = tl[st];
      const uint32_t rmps = range - lp;
      const bool lpsb = isC && (f >> 8) != mps;
      const uint32_t tb = tok & 1;
      const int bn = (tok >> 16) & 31;
      const uint32_t nr = isC ? (lpsb ? lp : rmps) : isT ? (tb ? 2u : range - 2) : range;
      const unsigned long long add = isC ? (lpsb ? rmps : 0u) : isT ? (tb ? range - 2 : 0u)
                                   : isB ? (unsigned long long)range * (tok & 0xffffu) : 0ull;
      const int prs = isB ? bn : 0;
      const int post = __clz(nr) - 23;
      low = ((low << prs) + add) << post;
      range = nr << post;
      bl -= prs + post;
      if (isC) {
        const uint32_t nsv = lpsb ? (tlp | ((mps ^ (st == 0 ? 1u : 0u)) << 6)) : ((st < 62 ? st + 1 : st) | (mps << 6));
        ctxL[c * 64 + lane] = nsv;
        ++nctxbins;
      }
      while (bl < 12) {  // CabacEncoder::write_out (bl >= -4 here: <= 16 bits per operation)
        const uint32_t lead = (uint32_t)(low >> (24 - bl));
        bl += 8;
        low &= (1ull << (32 - bl)) - 1;
        if (lead == 0xff) {
          nbuf++;
        } else if (nbuf > 0) {
          const uint32_t carry = lead >> 8;
          put(buffered + carry);
          buffered = lead & 0xff;
          const uint32_t byte = (0xff + carry) & 0xff;
          for (; nbuf > 1; --nbuf) put(byte);
        } else {
          nbuf = 1;
          buffered = lead;
        }
      }
      if (ty == 3) {
        if ((tok & 0xff) == kCtrlSync) {  // 9.3.2.4 storage for the row below
          uint32_t* dst = reinterpret_cast<uint32_t*>(a.wctx + ((long)b * hc + row) * kEntCtx);
          uint32_t t[kEntCtx / 4];
#pragma unroll
          for (int i = 0; i < kEntCtx / 4; ++i)
            t[i] = ctxL[(4 * i) * 64 + lane] | ctxL[(4 * i + 1) * 64 + lane] << 8 | ctxL[(4 * i + 2) * 64 + lane] << 16 |
                   ctxL[(4 * i + 3) * 64 + lane] << 24;
#pragma unroll
          for (int i = 0; i < kEntCtx / 4; ++i) __hip_atomic_store(dst + i, t[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          __hip_atomic_store(flag, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          synced = true;
        } else {  // finish() + '1' + byte alignment (end_of_subset_one_bit / slice trailing bits)
          const unsigned long long top = 1ull << (32 - bl);
          if (low >= top) {
            put(buffered + 1);
            for (; nbuf > 1; --nbuf) put(0x00);
            low -= top;
          } else {
            if (nbuf > 0) put(buffered);
            for (; nbuf > 1; --nbuf) put(0xff);
          }
          const int nb = 24 - bl;  // 1..12 bits of low >> 8, then the '1', then zeros
          uint32_t v = ((((uint32_t)low >> 8) & ((1u << nb) - 1)) << 1) | 1u;
          int t = nb + 1;
          const int pad = (8 - (t & 7)) & 7;
          v <<= pad;
          t += pad;
          while (t > 0) {
            t -= 8;
            put((v >> t) & 0xff);
          }
          uint8_t* o8 = reinterpret_cast<uint8_t*>(out);
          for (int k = pos & ~3; k < pos; ++k) o8[k] = (uint8_t)(ow >> (8 * (k & 3)));
          a.row_bytes[(long)b * hc + row] = pos;
          if (!synced) {
            abort_lane(4);  // a substream that never stored its contexts (corrupt stream)
          } else {
            active = false;
          }
          if (a.dbg) {  // TV_ENT_DEBUG: rows, context bins, tokens, coding clocks, wait ticks, max row span
            atomicAdd(&a.dbg[0], 1ull);
            atomicAdd(&a.dbg[1], (unsigned long long)nctxbins);
            atomicAdd(&a.dbg[2], (unsigned long long)ntoks);
            atomicAdd(&a.dbg[3], clock64() - c1);
            atomicAdd(&a.dbg[4], w1 - w0);
            atomicMax(&a.dbg[5], wall_clock64() - w0);
          }
          break;
        }
      }
      if (more) {
        ++sub;
      } else {
        sub = 0;
        ++head;
        ++ntoks;
        tok = ntok;
        if (--left <= 0) {  // no FLUSH before the row's tokens ran out
          abort_lane(4);
          break;
        }
      }
    }
  }
}
// Slice b's rows back to back after slices 0..b-1, written straight into the pinned host slot
// (device-visible): the head (sizes), the slice QP and the payload -- the host needs no copy.
__global__ void __launch_bounds__(256) k_ent_pack(EntropyArgs a, int B) {
  const int b = blockIdx.x, hc = a.g.hc, wc = a.g.wc, nctu = wc * hc;
  int* hseg = a.hhead + (a.seg_bytes - a.status);
  int* hrow = a.hhead + (a.row_bytes - a.status);
  __shared__ long s_base;
  __shared__ int s_pre[256];
  __shared__ int s_bad;
  if (threadIdx.x == 0) {
    long base = 0;
    for (long k = 0; k < (long)b * hc; ++k) base += a.row_bytes[k];
    s_base = base;
    int run = 0;
    for (int r = 0; r < hc; ++r) {
      s_pre[r] = run;
      run += a.row_bytes[(long)b * hc + r];
    }
    hseg[b] = run;
    a.hqp[b] = a.dec.qp[b];
    s_bad = *a.status;
    if (base + run > a.hout_cap) {
      atomicOr(a.status, 8);
      s_bad = 8;
    }
  }
  __syncthreads();
  if (!s_bad) {
    for (int r = threadIdx.x; r < hc; r += 256) hrow[(long)b * hc + r] = a.row_bytes[(long)b * hc + r];
    long tbase = 0;
    for (int k = 0; k < b; ++k) tbase += a.seg_tok[k];
    const int* off = a.ctb_off + (long)b * nctu;
    for (int r = 0; r < hc; ++r) {
      const uint8_t* src = a.stage + stage_off(tbase + off[r * wc], (long)b * hc + r);
      uint8_t* dst = a.hout + s_base + s_pre[r];
      const int n = a.row_bytes[(long)b * hc + r];
      for (int k = threadIdx.x; k < n; k += 256) dst[k] = src[k];
    }
  }
  // no system fence: the host reads the slot after the stream's completion event
}

// the picture's final status into the host slot (after every pack workgroup)
__global__ void k_ent_status(EntropyArgs a) {
  a.hhead[0] = *a.status;
}

}  // namespace

void launch_entropy_bin(const EntropyArgs& a, int B, hipStream_t s) {
  const int nctu = a.g.wc * a.g.hc;
  if (a.g.wc < 2) throw std::runtime_error("GPU entropy coding needs at least 2 CTB columns");
  if (a.g.hc > 256) throw std::runtime_error("GPU entropy coding supports at most 256 CTB rows");
  (void)hipMemsetAsync(a.status, 0, sizeof(int), s);
  if (a.pic.type != 2) k_ent_cu<<<dim3((unsigned)((a.g.usz + 255) / 256), B), 256, 0, s>>>(a);
  if (a.g.wc > 256) throw std::runtime_error("GPU entropy coding supports at most 256 CTB columns");
  const BinStage L = bin_stage(a.g.w8, a.dec.tu != nullptr, a.dec.dir != nullptr);
  const dim3 rows(a.g.hc, B);
  const int nthr = 64 * ((a.g.wc + 63) / 64);
  k_ent_bin<true><<<rows, nthr, L.bytes, s>>>(a);
  k_ent_scan<<<B, 1024, 0, s>>>(a);
  k_ent_check<<<1, 1, 0, s>>>(a, B);
  k_ent_place<<<dim3((nctu + 3) / 4, B), 256, 0, s>>>(a);
  k_ent_bin<false><<<rows, nthr, L.bytes, s>>>(a);
}

void launch_entropy_ac(const EntropyArgs& a, int B, hipStream_t s) {
  // TV_ENT_ROWS_PER_WAVE (1..8, default 1): substream rows coded by one wave, strided
  static const int rpw = [] {
    const char* e = std::getenv("TV_ENT_ROWS_PER_WAVE");
    const int v = e ? std::atoi(e) : 1;
    return v < 1 ? 1 : v > 8 ? 8 : v;
  }();
  // TV_ENT_CODER=lanes: the lane-per-substream coder (one wave per CTB row index, one lane per
  // segment) -- byte-exact, 24x fewer waves, but ~1300 clocks per operation against ~610 per
  // bin here, so a picture's substreams take ~2x longer and the slot pipeline stalls
  // (profiles/README.md, round 6).  The single-lane wave coder stays the default.
  const char* ce = std::getenv("TV_ENT_CODER");  // per launch (tests switch it)
  const bool lane_coder = ce && std::string(ce) == "lanes";
  (void)hipMemsetAsync(a.wflag, 0, (size_t)B * a.g.hc * sizeof(int), s);
  if (!lane_coder)
    k_ent_ac<<<dim3((a.g.hc + rpw - 1) / rpw, B), 64, 0, s>>>(a);
  else
    k_ent_ac_lanes<<<dim3(a.g.hc, (B + 63) / 64), 64, 0, s>>>(a, B);
  k_ent_pack<<<B, 256, 0, s>>>(a, B);
  k_ent_status<<<1, 1, 0, s>>>(a);
}

void entropy_tables(EntropyTables& t) {
  for (int ty = 0; ty < 3; ++ty)
    for (int q = 0; q < 52; ++q) {
      ContextSet cs;
      cs.init(ty, q);
      for (int c = 0; c < CTX_COUNT; ++c) t.init[ty][q][c] = (uint8_t)(cs.c[c].state | (cs.c[c].mps << 6));
    }
  for (int s = 0; s < 64; ++s) {
    for (int q = 0; q < 4; ++q) t.lps[s * 4 + q] = kRangeTabLps[s][q];
    t.tlps[s] = kTransIdxLps[s];
  }
}

}  // namespace gpu
}  // namespace tv
