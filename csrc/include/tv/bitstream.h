// bitstream.h — RBSP bit writer/reader, Exp-Golomb, NAL (Annex-B) encapsulation with
// emulation prevention.  Host-only.
#pragma once
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <vector>

namespace tv {

class BitWriter {
 public:
  void put(uint32_t v, int n) {  // n <= 32, MSB first
    if (nbits_ == 0 && n == 8) {  // byte-aligned byte: the CABAC output path
      buf_.push_back((uint8_t)v);
      return;
    }
    for (int i = n - 1; i >= 0; --i) put_bit((v >> i) & 1);
  }
  void put_bit(int b) {
    cur_ = (uint8_t)((cur_ << 1) | (b & 1));
    if (++nbits_ == 8) {
      buf_.push_back(cur_);
      cur_ = 0;
      nbits_ = 0;
    }
  }
  void ue(uint32_t v) {
    const uint64_t x = (uint64_t)v + 1;
    int len = 0;
    while ((x >> (len + 1)) != 0) ++len;
    put(0, len);
    for (int i = len; i >= 0; --i) put_bit((int)((x >> i) & 1));
  }
  void se(int32_t v) { ue(v > 0 ? (uint32_t)(2 * v - 1) : (uint32_t)(-2 * (int64_t)v)); }
  void trailing_bits() {  // rbsp_trailing_bits
    put_bit(1);
    while (nbits_) put_bit(0);
  }
  void align_zero() {
    while (nbits_) put_bit(0);
  }
  bool aligned() const { return nbits_ == 0; }
  void put_bytes(const uint8_t* p, size_t n) {
    if (!aligned()) throw std::runtime_error("put_bytes on unaligned writer");
    buf_.insert(buf_.end(), p, p + n);
  }
  const std::vector<uint8_t>& bytes() const { return buf_; }
  std::vector<uint8_t>& bytes() { return buf_; }
  size_t bit_count() const { return buf_.size() * 8 + nbits_; }

 private:
  std::vector<uint8_t> buf_;
  uint8_t cur_ = 0;
  int nbits_ = 0;
};

class BitReader {
 public:
  BitReader(const uint8_t* p, size_t n) : p_(p), n_(n) {}
  int bit() {
    if (pos_ >= n_ * 8) throw std::runtime_error("bitreader overrun");
    int b = (p_[pos_ >> 3] >> (7 - (pos_ & 7))) & 1;
    ++pos_;
    return b;
  }
  // past the end of the slice the CABAC engine may read a few padding bits: return 0
  int bit_or_zero() { return pos_ < n_ * 8 ? bit() : (++pos_, 0); }
  uint32_t u(int n) {
    uint32_t v = 0;
    for (int i = 0; i < n; ++i) v = (v << 1) | (uint32_t)bit();
    return v;
  }
  uint32_t ue() {
    int lz = 0;
    while (bit() == 0) {
      if (++lz > 31) throw std::runtime_error("bad exp-golomb");
    }
    return (uint32_t)(((1ULL << lz) - 1) + u(lz));
  }
  int32_t se() {
    uint32_t k = ue();
    return (k & 1) ? (int32_t)((k + 1) / 2) : -(int32_t)(k / 2);
  }
  void byte_align() { pos_ = (pos_ + 7) & ~(size_t)7; }
  void seek(size_t bit_pos) { pos_ = bit_pos; }
  size_t pos() const { return pos_; }
  size_t byte_pos() const { return pos_ >> 3; }
  size_t size() const { return n_; }

 private:
  const uint8_t* p_;
  size_t n_;
  size_t pos_ = 0;
};

// NAL unit types used by the engine
enum NalType : int {
  NAL_TRAIL_N = 0,
  NAL_TRAIL_R = 1,
  NAL_IDR_W_RADL = 19,
  NAL_IDR_N_LP = 20,
  NAL_VPS = 32,
  NAL_SPS = 33,
  NAL_PPS = 34,
  NAL_AUD = 35,
};

// Append an Annex-B NAL (start code + header + EPB-escaped RBSP) to `out`.
inline void append_nal(std::vector<uint8_t>& out, int nal_type, const std::vector<uint8_t>& rbsp,
                       bool long_start_code = true) {
  if (long_start_code) out.push_back(0);
  out.push_back(0);
  out.push_back(0);
  out.push_back(1);
  out.push_back((uint8_t)((nal_type & 0x3f) << 1));  // forbidden 0, type, layer id msb 0
  out.push_back(1);                                  // layer id lsbs 0, temporal_id_plus1 = 1
  int zeros = 0;
  for (uint8_t b : rbsp) {
    if (zeros >= 2 && b <= 3) {
      out.push_back(3);
      zeros = 0;
    }
    out.push_back(b);
    zeros = (b == 0) ? zeros + 1 : 0;
  }
}

// Remove emulation-prevention bytes from an escaped NAL payload.
inline std::vector<uint8_t> unescape_rbsp(const uint8_t* p, size_t n) {
  std::vector<uint8_t> r;
  r.reserve(n);
  int zeros = 0;
  for (size_t i = 0; i < n; ++i) {
    if (zeros >= 2 && p[i] == 3) {
      zeros = 0;
      continue;
    }
    r.push_back(p[i]);
    zeros = p[i] == 0 ? zeros + 1 : 0;
  }
  return r;
}

// Size of `n` RBSP bytes after emulation prevention, when the byte before them is nonzero
// (a WPP substream: the previous one ends in its alignment '1' bit, the slice header in its
// byte_alignment()), so its escaping depends on its own bytes only.
inline size_t escaped_size(const uint8_t* p, size_t n) {
  size_t out = n;
  int zeros = 0;
  for (size_t i = 0; i < n; ++i) {
    if (zeros >= 2 && p[i] <= 3) {
      ++out;
      zeros = 0;
    }
    zeros = p[i] == 0 ? zeros + 1 : 0;
  }
  return out;
}
// unescape_rbsp that also records the escaped index of every removed byte (entry point
// offsets count emulation-prevention bytes)
inline std::vector<uint8_t> unescape_rbsp_map(const uint8_t* p, size_t n, std::vector<size_t>* removed) {
  std::vector<uint8_t> r;
  r.reserve(n);
  int zeros = 0;
  for (size_t i = 0; i < n; ++i) {
    if (zeros >= 2 && p[i] == 3) {
      zeros = 0;
      removed->push_back(i);
      continue;
    }
    r.push_back(p[i]);
    zeros = p[i] == 0 ? zeros + 1 : 0;
  }
  return r;
}

struct NalView {
  const uint8_t* data;  // first header byte
  size_t size;          // header + escaped payload
  int type() const { return (data[0] >> 1) & 0x3f; }
};

// Split an Annex-B byte stream into NAL units.
inline std::vector<NalView> split_annexb(const uint8_t* p, size_t n) {
  std::vector<NalView> nals;
  size_t i = 0, start = SIZE_MAX;
  while (i + 2 < n) {
    if (p[i] == 0 && p[i + 1] == 0 && p[i + 2] == 1) {
      if (start != SIZE_MAX) {
        size_t end = i;
        while (end > start && p[end - 1] == 0) --end;  // trailing_zero_8bits / 4-byte code
        nals.push_back({p + start, end - start});
      }
      i += 3;
      start = i;
    } else {
      ++i;
    }
  }
  if (start != SIZE_MAX && start < n) nals.push_back({p + start, n - start});
  return nals;
}

}  // namespace tv
