// cabac.h — HEVC CABAC arithmetic coder (encoder + decoder) and context-model tables.
// Host-only.  Context init values transcribed from ITU-T H.265 §9.3.2.2 (Tables 9-5..9-37)
// for initType 0 (I), 1 (P), 2 (B).
#pragma once
#include <cstdint>
#include <vector>

#include "bitstream.h"

namespace tv {

// Flat context index layout
enum CtxOffset : int {
  CTX_SAO_MERGE = 0,
  CTX_SAO_TYPE = CTX_SAO_MERGE + 1,
  CTX_SPLIT_CU = CTX_SAO_TYPE + 1,          // 3
  CTX_TQ_BYPASS = CTX_SPLIT_CU + 3,         // 1
  CTX_CU_SKIP = CTX_TQ_BYPASS + 1,          // 3
  CTX_PALETTE_UNUSED = CTX_CU_SKIP + 3,     // (none)
  CTX_PRED_MODE = CTX_PALETTE_UNUSED,       // 1
  CTX_PART_MODE = CTX_PRED_MODE + 1,        // 4
  CTX_PREV_INTRA = CTX_PART_MODE + 4,       // 1
  CTX_CHROMA_PRED = CTX_PREV_INTRA + 1,     // 1
  CTX_RQT_ROOT_CBF = CTX_CHROMA_PRED + 1,   // 1
  CTX_MERGE_FLAG = CTX_RQT_ROOT_CBF + 1,    // 1
  CTX_MERGE_IDX = CTX_MERGE_FLAG + 1,       // 1
  CTX_INTER_PRED_IDC = CTX_MERGE_IDX + 1,   // 5
  CTX_REF_IDX = CTX_INTER_PRED_IDC + 5,     // 2
  CTX_MVP_FLAG = CTX_REF_IDX + 2,           // 1
  CTX_SPLIT_TF = CTX_MVP_FLAG + 1,          // 3
  CTX_CBF_LUMA = CTX_SPLIT_TF + 3,          // 2
  CTX_CBF_CHROMA = CTX_CBF_LUMA + 2,        // 4
  CTX_MVD_G0 = CTX_CBF_CHROMA + 4,          // 1
  CTX_MVD_G1 = CTX_MVD_G0 + 1,              // 1
  CTX_CU_QP_DELTA = CTX_MVD_G1 + 1,         // 2
  CTX_TRANSFORM_SKIP = CTX_CU_QP_DELTA + 2, // 2
  CTX_LAST_X = CTX_TRANSFORM_SKIP + 2,      // 18
  CTX_LAST_Y = CTX_LAST_X + 18,             // 18
  CTX_CSBF = CTX_LAST_Y + 18,               // 4
  CTX_SIG = CTX_CSBF + 4,                   // 42 (44 incl. RExt transform-skip ctx)
  CTX_G1 = CTX_SIG + 44,                    // 24
  CTX_G2 = CTX_G1 + 24,                     // 6
  CTX_COUNT = CTX_G2 + 6
};

// init values [initType][ctx]
struct CtxInitTable {
  uint8_t v[3][CTX_COUNT];
};

inline const CtxInitTable& ctx_init_table() {
  static const CtxInitTable t = [] {
    CtxInitTable r{};
    auto set = [&](int off, int n, std::initializer_list<int> i0, std::initializer_list<int> i1,
                   std::initializer_list<int> i2) {
      const std::initializer_list<int>* L[3] = {&i0, &i1, &i2};
      for (int t = 0; t < 3; ++t) {
        int k = 0;
        for (int x : *L[t]) {
          if (k < n) r.v[t][off + k] = (uint8_t)x;
          ++k;
        }
        for (; k < n; ++k) r.v[t][off + k] = 154;  // unused contexts: CNU
      }
    };
    set(CTX_SAO_MERGE, 1, {153}, {153}, {153});
    set(CTX_SAO_TYPE, 1, {200}, {185}, {160});
    set(CTX_SPLIT_CU, 3, {139, 141, 157}, {107, 139, 126}, {107, 139, 126});
    set(CTX_TQ_BYPASS, 1, {154}, {154}, {154});
    set(CTX_CU_SKIP, 3, {154, 154, 154}, {197, 185, 201}, {197, 185, 201});
    set(CTX_PRED_MODE, 1, {154}, {149}, {134});
    set(CTX_PART_MODE, 4, {184, 154, 154, 154}, {154, 139, 154, 154}, {154, 139, 154, 154});
    set(CTX_PREV_INTRA, 1, {184}, {154}, {183});
    set(CTX_CHROMA_PRED, 1, {63}, {152}, {152});
    set(CTX_RQT_ROOT_CBF, 1, {154}, {79}, {79});
    set(CTX_MERGE_FLAG, 1, {154}, {110}, {154});
    set(CTX_MERGE_IDX, 1, {154}, {122}, {137});
    set(CTX_INTER_PRED_IDC, 5, {154, 154, 154, 154, 154}, {95, 79, 63, 31, 31}, {95, 79, 63, 31, 31});
    set(CTX_REF_IDX, 2, {154, 154}, {153, 153}, {153, 153});
    set(CTX_MVP_FLAG, 1, {154}, {168}, {168});
    set(CTX_SPLIT_TF, 3, {153, 138, 138}, {124, 138, 94}, {224, 167, 122});
    set(CTX_CBF_LUMA, 2, {111, 141}, {153, 111}, {153, 111});
    set(CTX_CBF_CHROMA, 4, {94, 138, 182, 154}, {149, 107, 167, 154}, {149, 92, 167, 154});
    set(CTX_MVD_G0, 1, {154}, {140}, {169});
    set(CTX_MVD_G1, 1, {154}, {198}, {198});
    set(CTX_CU_QP_DELTA, 2, {154, 154}, {154, 154}, {154, 154});
    set(CTX_TRANSFORM_SKIP, 2, {139, 139}, {139, 139}, {139, 139});
    const std::initializer_list<int> last0 = {110, 110, 124, 125, 140, 153, 125, 127, 140,
                                              109, 111, 143, 127, 111, 79,  108, 123, 63};
    const std::initializer_list<int> last1 = {125, 110, 94,  110, 95,  79,  125, 111, 110,
                                              78,  110, 111, 111, 95,  94,  108, 123, 108};
    const std::initializer_list<int> last2 = {125, 110, 124, 110, 95,  94,  125, 111, 111,
                                              79,  125, 126, 111, 111, 79,  108, 123, 93};
    set(CTX_LAST_X, 18, last0, last1, last2);
    set(CTX_LAST_Y, 18, last0, last1, last2);
    set(CTX_CSBF, 4, {91, 171, 134, 141}, {121, 140, 61, 154}, {121, 140, 61, 154});
    set(CTX_SIG, 44,
        {111, 111, 125, 110, 110, 94,  124, 108, 124, 107, 125, 141, 179, 153, 125,
         107, 125, 141, 179, 153, 125, 107, 125, 141, 179, 153, 125, 140, 139, 182,
         182, 152, 136, 152, 136, 153, 136, 139, 111, 136, 139, 111, 141, 111},
        {155, 154, 139, 153, 139, 123, 123, 63,  153, 166, 183, 140, 136, 153, 154,
         166, 183, 140, 136, 153, 154, 166, 183, 140, 136, 153, 154, 170, 153, 123,
         123, 107, 121, 107, 121, 167, 151, 183, 140, 151, 183, 140, 140, 140},
        {170, 154, 139, 153, 139, 123, 123, 63,  124, 166, 183, 140, 136, 153, 154,
         166, 183, 140, 136, 153, 154, 166, 183, 140, 136, 153, 154, 170, 153, 138,
         138, 122, 121, 122, 121, 167, 151, 183, 140, 151, 183, 140, 140, 140});
    set(CTX_G1, 24,
        {140, 92, 137, 138, 140, 152, 138, 139, 153, 74, 149, 92,
         139, 107, 122, 152, 140, 179, 166, 182, 140, 227, 122, 197},
        {154, 196, 196, 167, 154, 152, 167, 182, 182, 134, 149, 136,
         153, 121, 136, 122, 169, 208, 166, 167, 154, 152, 167, 182},
        {154, 196, 167, 167, 154, 152, 167, 182, 182, 134, 149, 136,
         153, 121, 136, 137, 169, 194, 166, 167, 154, 167, 137, 182});
    set(CTX_G2, 6, {138, 153, 136, 167, 152, 152}, {107, 167, 91, 122, 107, 167},
        {107, 167, 91, 107, 107, 167});
    return r;
  }();
  return t;
}

extern const uint8_t kRangeTabLps[64][4];
extern const uint8_t kTransIdxLps[64];
// MPS transition: state + 1, saturating at 62 (state 63 is the terminate state)
struct TransMps {
  uint8_t t[64];
  constexpr TransMps() : t() {
    for (int i = 0; i < 64; ++i) t[i] = (uint8_t)(i < 62 ? i + 1 : i);
  }
};
constexpr TransMps kTransMpsTab{};
constexpr const uint8_t* kTransIdxMps = kTransMpsTab.t;

struct CtxState {
  uint8_t state;  // pStateIdx
  uint8_t mps;    // valMps
};

struct ContextSet {
  CtxState c[CTX_COUNT];
  void init(int init_type, int qp) {
    const auto& t = ctx_init_table();
    for (int i = 0; i < CTX_COUNT; ++i) {
      const int iv = t.v[init_type][i];
      const int slope = iv >> 4, off = iv & 15;
      const int m = slope * 5 - 45, n = (off << 3) - 16;
      int q = qp < 0 ? 0 : (qp > 51 ? 51 : qp);
      int pre = ((m * q) >> 4) + n;
      pre = pre < 1 ? 1 : (pre > 126 ? 126 : pre);
      if (pre <= 63) {
        c[i].state = (uint8_t)(63 - pre);
        c[i].mps = 0;
      } else {
        c[i].state = (uint8_t)(pre - 64);
        c[i].mps = 1;
      }
    }
  }
};

// ----------------------------------- encoder --------------------------------------------
class CabacEncoder {
 public:
  explicit CabacEncoder(BitWriter* bw) : bw_(bw) {}
  void rebind(BitWriter* bw) { bw_ = bw; }
  void start() {
    low_ = 0;
    range_ = 510;
    bits_left_ = 23;
    num_buffered_ = 0;
    buffered_ = 0xff;
  }
  // Both outcomes are formed and selected, renormalisation is one clz.
  static inline void bin_step(uint32_t& low, uint32_t& range, int& bits_left, int bin, CtxState& ctx) {
    const uint32_t lps = kRangeTabLps[ctx.state][(range >> 6) & 3];
    const uint32_t rmps = range - lps;
    const bool is_lps = bin != ctx.mps;
    const uint32_t r = is_lps ? lps : rmps;
    const uint32_t l = is_lps ? low + rmps : low;
    const int nb = __builtin_clz(r) - 23;  // shifts bringing r (>= 6) to >= 256; 0 if already
    low = l << nb;
    range = r << nb;
    bits_left -= nb;
    ctx.mps = (uint8_t)(ctx.mps ^ (is_lps & (ctx.state == 0)));
    ctx.state = is_lps ? kTransIdxLps[ctx.state] : kTransIdxMps[ctx.state];
  }
  void encode_bin(int bin, CtxState& ctx) {
    bin_step(low_, range_, bits_left_, bin, ctx);
    test_write_out();
  }
  // A run of `count` context-coded bins with the coder state in registers (the members are
  // only touched around the byte output): next(k, bin, ctx) names the k-th bin and context.
  template <class F>
  void encode_run(int count, F&& next) {
    uint32_t low = low_, range = range_;
    int bl = bits_left_;
    for (int k = 0; k < count; ++k) {
      int bin;
      CtxState* c;
      next(k, bin, c);
      bin_step(low, range, bl, bin, *c);
      if (bl < 12) {
        low_ = low;
        bits_left_ = bl;
        write_out();
        low = low_;
        bl = bits_left_;
      }
    }
    low_ = low;
    range_ = range;
    bits_left_ = bl;
  }
  void encode_bypass(int bin) {
    low_ <<= 1;
    if (bin) low_ += range_;
    bits_left_--;
    test_write_out();
  }
  void encode_bypass_bins(uint32_t value, int n) {
    while (n > 8) {
      n -= 8;
      uint32_t pattern = value >> n;
      low_ <<= 8;
      low_ += range_ * pattern;
      value -= pattern << n;
      bits_left_ -= 8;
      test_write_out();
    }
    low_ <<= n;
    low_ += range_ * value;
    bits_left_ -= n;
    test_write_out();
  }
  void encode_terminate(int bin) {
    range_ -= 2;
    if (bin) {
      low_ += range_;
      low_ <<= 7;
      range_ = 2 << 7;
      bits_left_ -= 7;
    } else if (range_ >= 256) {
      return;
    } else {
      low_ <<= 1;
      range_ <<= 1;
      bits_left_--;
    }
    test_write_out();
  }
  // flush after the terminating bin (end_of_slice_segment_flag == 1)
  void finish() {
    if ((low_ >> (32 - bits_left_)) != 0) {
      bw_->put(buffered_ + 1, 8);
      while (num_buffered_ > 1) {
        bw_->put(0x00, 8);
        num_buffered_--;
      }
      low_ -= 1u << (32 - bits_left_);
    } else {
      if (num_buffered_ > 0) bw_->put(buffered_, 8);
      while (num_buffered_ > 1) {
        bw_->put(0xff, 8);
        num_buffered_--;
      }
    }
    bw_->put(low_ >> 8, 24 - bits_left_);
  }
  // fractional-bit estimate is not needed by the engine; count of bins for stats
 private:
  static int renorm_bits(uint32_t lps) {  // shifts bringing lps (6..255) to >= 256
    return __builtin_clz(lps) - 23;
  }
  void test_write_out() {
    if (bits_left_ < 12) write_out();
  }
  void write_out() {
    uint32_t lead = low_ >> (24 - bits_left_);
    bits_left_ += 8;
    low_ &= 0xffffffffu >> bits_left_;
    if (lead == 0xff) {
      num_buffered_++;
    } else if (num_buffered_ > 0) {
      uint32_t carry = lead >> 8;
      uint32_t byte = buffered_ + carry;
      buffered_ = lead & 0xff;
      bw_->put(byte, 8);
      byte = (0xff + carry) & 0xff;
      while (num_buffered_ > 1) {
        bw_->put(byte, 8);
        num_buffered_--;
      }
    } else {
      num_buffered_ = 1;
      buffered_ = lead;
    }
  }
  BitWriter* bw_;
  uint32_t low_ = 0, range_ = 510;
  int bits_left_ = 23;
  int num_buffered_ = 0;
  uint32_t buffered_ = 0xff;
};

// ----------------------------------- decoder --------------------------------------------
class CabacDecoder {
 public:
  explicit CabacDecoder(BitReader* br) : br_(br) {}
  void start() {
    range_ = 510;
    offset_ = 0;
    for (int i = 0; i < 9; ++i) offset_ = (offset_ << 1) | (uint32_t)br_->bit_or_zero();
  }
  int decode_bin(CtxState& ctx) {
    uint32_t lps = kRangeTabLps[ctx.state][(range_ >> 6) & 3];
    range_ -= lps;
    int bin;
    if (offset_ >= range_) {
      bin = 1 - ctx.mps;
      offset_ -= range_;
      range_ = lps;
      if (ctx.state == 0) ctx.mps = (uint8_t)(1 - ctx.mps);
      ctx.state = kTransIdxLps[ctx.state];
    } else {
      bin = ctx.mps;
      if (ctx.state < 62) ++ctx.state;
    }
    while (range_ < 256) {
      range_ <<= 1;
      offset_ = (offset_ << 1) | (uint32_t)br_->bit_or_zero();
    }
    return bin;
  }
  int decode_bypass() {
    offset_ = (offset_ << 1) | (uint32_t)br_->bit_or_zero();
    if (offset_ >= range_) {
      offset_ -= range_;
      return 1;
    }
    return 0;
  }
  uint32_t decode_bypass_bins(int n) {
    uint32_t v = 0;
    for (int i = 0; i < n; ++i) v = (v << 1) | (uint32_t)decode_bypass();
    return v;
  }
  int decode_terminate() {
    range_ -= 2;
    if (offset_ >= range_) return 1;
    while (range_ < 256) {
      range_ <<= 1;
      offset_ = (offset_ << 1) | (uint32_t)br_->bit_or_zero();
    }
    return 0;
  }

 private:
  BitReader* br_;
  uint32_t range_ = 510, offset_ = 0;
};

}  // namespace tv
