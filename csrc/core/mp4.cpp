// mp4.cpp — minimal ISO-BMFF writer/reader for one HEVC video track.
//
// Replaces the reference's `ffmpeg -f concat -c copy -movflags +faststart` stitch step
// (reference worker/tasks.py:2047-2069): the concatenated Annex-B segments become 'hvc1'
// samples (length-prefixed NAL units, parameter sets hoisted into hvcC), moov placed
// before mdat (faststart layout).
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>

#include "tv/bitstream.h"
#include "tv/hevc_codec.h"

namespace tv {

namespace {

struct Box {
  std::vector<uint8_t> b;
  void u8(uint32_t v) { b.push_back((uint8_t)v); }
  void u16(uint32_t v) {
    u8(v >> 8);
    u8(v);
  }
  void u32(uint32_t v) {
    u16(v >> 16);
    u16(v);
  }
  void u64(uint64_t v) {
    u32((uint32_t)(v >> 32));
    u32((uint32_t)v);
  }
  void str(const char* s, size_t n) { b.insert(b.end(), s, s + n); }
  void bytes(const std::vector<uint8_t>& v) { b.insert(b.end(), v.begin(), v.end()); }
  void bytes(const uint8_t* p, size_t n) { b.insert(b.end(), p, p + n); }
  void zeros(size_t n) { b.insert(b.end(), n, 0); }
};

std::vector<uint8_t> box(const char* type, const std::vector<uint8_t>& payload) {
  Box o;
  o.u32((uint32_t)(payload.size() + 8));
  o.str(type, 4);
  o.bytes(payload);
  return o.b;
}
std::vector<uint8_t> fullbox(const char* type, int version, uint32_t flags,
                             const std::vector<uint8_t>& payload) {
  Box o;
  o.u8((uint32_t)version);
  o.u8(flags >> 16);
  o.u16(flags & 0xffff);
  o.bytes(payload);
  return box(type, o.b);
}
std::vector<uint8_t> cat(std::initializer_list<std::vector<uint8_t>> parts) {
  std::vector<uint8_t> r;
  for (const auto& p : parts) r.insert(r.end(), p.begin(), p.end());
  return r;
}
void matrix(Box& o) {
  const uint32_t m[9] = {0x00010000, 0, 0, 0, 0x00010000, 0, 0, 0, 0x40000000};
  for (uint32_t v : m) o.u32(v);
}

// One sample = references to its NAL units (in-band parameter sets first when they change
// between segments) — the payload is never copied until it is written.
struct Sample {
  std::vector<NalView> nals;
  uint32_t size = 0;  // length-prefixed bytes
  bool sync = false;
};

struct MuxPlan {
  std::vector<uint8_t> vps, sps, pps;
  bool ps_consistent = true;
  std::vector<Sample> samples;
  uint64_t mdat_payload = 0;
};

// Scan the Annex-B segments (in order) into samples; no payload bytes are copied.
MuxPlan plan_mux(const uint8_t* const* segs, const size_t* sizes, int nseg) {
  MuxPlan P;
  std::vector<NalView> pending_ps;
  for (int k = 0; k < nseg; ++k) {
    for (const auto& nal : split_annexb(segs[k], sizes[k])) {
      const int t = nal.type();
      if (t == NAL_VPS || t == NAL_SPS || t == NAL_PPS) {
        auto& slot = t == NAL_VPS ? P.vps : (t == NAL_SPS ? P.sps : P.pps);
        const std::vector<uint8_t> bytes(nal.data, nal.data + nal.size);
        if (slot.empty()) slot = bytes;
        else if (slot != bytes) P.ps_consistent = false;
        pending_ps.push_back(nal);
        continue;
      }
      if (t > 31) continue;  // AUD / SEI etc. dropped
      Sample s;
      s.sync = (t >= 16 && t <= 23);
      s.nals = pending_ps;  // kept only if the parameter sets turn out inconsistent
      s.nals.push_back(nal);
      pending_ps.clear();
      P.samples.push_back(std::move(s));
    }
  }
  if (P.sps.empty() || P.pps.empty() || P.vps.empty()) throw std::runtime_error("mux_mp4: missing parameter sets");
  for (auto& s : P.samples) {
    if (P.ps_consistent) s.nals.erase(s.nals.begin(), s.nals.end() - 1);  // parameter sets live in hvcC
    s.size = 0;
    for (const auto& n : s.nals) s.size += 4 + (uint32_t)n.size;
    P.mdat_payload += s.size;
  }
  return P;
}

// ftyp + moov (faststart) + the mdat header, for a plan whose payload follows directly
std::vector<uint8_t> mp4_header(const MuxPlan& P, int width, int height, int fps_num, int fps_den) {
  const auto& samples = P.samples;
  const uint32_t timescale = (uint32_t)fps_num * 1000u;
  const uint32_t delta = (uint32_t)fps_den * 1000u;
  const uint64_t dur_media = (uint64_t)samples.size() * delta;
  const uint64_t dur_ms = dur_media * 1000 / timescale;

  // hvcC from the SPS profile_tier_level
  std::vector<uint8_t> sps_rbsp = unescape_rbsp(P.sps.data() + 2, P.sps.size() - 2);
  if (sps_rbsp.size() < 13) throw std::runtime_error("mux_mp4: short SPS");
  Box hv;
  hv.u8(1);
  hv.bytes(sps_rbsp.data() + 1, 1 + 4 + 6 + 1);  // profile byte, compat(4), constraints(6), level
  hv.u16(0xF000);
  hv.u8(0xFC);
  hv.u8(0xFC | 1);
  hv.u8(0xF8);
  hv.u8(0xF8);
  hv.u16(0);
  hv.u8((0u << 6) | (1u << 3) | (1u << 2) | 3u);
  hv.u8(3);
  for (const auto* ps : {&P.vps, &P.sps, &P.pps}) {
    hv.u8(0x80 | (((*ps)[0] >> 1) & 0x3f));
    hv.u16(1);
    hv.u16((uint32_t)ps->size());
    hv.bytes(*ps);
  }
  Box se;  // VisualSampleEntry
  se.zeros(6);
  se.u16(1);
  se.zeros(16);
  se.u16((uint32_t)width);
  se.u16((uint32_t)height);
  se.u32(0x00480000);
  se.u32(0x00480000);
  se.u32(0);
  se.u16(1);
  {
    char name[32] = {0};
    const char* nm = "thinvids-amd HEVC";
    name[0] = (char)std::strlen(nm);
    std::memcpy(name + 1, nm, std::strlen(nm));
    se.str(name, 32);
  }
  se.u16(0x0018);
  se.u16(0xffff);
  se.bytes(box("hvcC", hv.b));
  const auto entry = box(P.ps_consistent ? "hvc1" : "hev1", se.b);
  Box stsd;
  stsd.u32(1);
  stsd.bytes(entry);
  Box stts;
  stts.u32(1);
  stts.u32((uint32_t)samples.size());
  stts.u32(delta);
  Box stss;
  {
    std::vector<uint32_t> sync;
    for (size_t i = 0; i < samples.size(); ++i)
      if (samples[i].sync) sync.push_back((uint32_t)i + 1);
    stss.u32((uint32_t)sync.size());
    for (auto s : sync) stss.u32(s);
  }
  Box stsc;
  stsc.u32(1);
  stsc.u32(1);
  stsc.u32((uint32_t)samples.size());
  stsc.u32(1);
  Box stsz;
  stsz.u32(0);
  stsz.u32((uint32_t)samples.size());
  for (const auto& s : samples) stsz.u32(s.size);
  const uint64_t mdat_payload = P.mdat_payload;
  const bool large = mdat_payload + (1 << 20) > 0xffffffffull;
  auto build_moov = [&](uint64_t chunk_off) {
    Box co;
    co.u32(1);
    if (large) co.u64(chunk_off);
    else co.u32((uint32_t)chunk_off);
    const auto stbl = box("stbl", cat({fullbox("stsd", 0, 0, stsd.b), fullbox("stts", 0, 0, stts.b),
                                       fullbox("stss", 0, 0, stss.b), fullbox("stsc", 0, 0, stsc.b),
                                       fullbox("stsz", 0, 0, stsz.b),
                                       fullbox(large ? "co64" : "stco", 0, 0, co.b)}));
    Box vmhd;
    vmhd.zeros(8);
    Box dref;
    dref.u32(1);
    dref.bytes(fullbox("url ", 0, 1, {}));
    const auto dinf = box("dinf", fullbox("dref", 0, 0, dref.b));
    const auto minf = box("minf", cat({fullbox("vmhd", 0, 1, vmhd.b), dinf, stbl}));
    Box mdhd;
    mdhd.u32(0);
    mdhd.u32(0);
    mdhd.u32(timescale);
    mdhd.u32((uint32_t)dur_media);
    mdhd.u16(0x55C4);  // 'und'
    mdhd.u16(0);
    Box hdlr;
    hdlr.u32(0);
    hdlr.str("vide", 4);
    hdlr.zeros(12);
    hdlr.str("VideoHandler", 13);
    const auto mdia = box("mdia", cat({fullbox("mdhd", 0, 0, mdhd.b), fullbox("hdlr", 0, 0, hdlr.b), minf}));
    Box tkhd;
    tkhd.u32(0);
    tkhd.u32(0);
    tkhd.u32(1);
    tkhd.u32(0);
    tkhd.u32((uint32_t)dur_ms);
    tkhd.zeros(8);
    tkhd.u16(0);
    tkhd.u16(0);
    tkhd.u16(0);
    tkhd.u16(0);
    matrix(tkhd);
    tkhd.u32((uint32_t)width << 16);
    tkhd.u32((uint32_t)height << 16);
    const auto trak = box("trak", cat({fullbox("tkhd", 0, 3, tkhd.b), mdia}));
    Box mvhd;
    mvhd.u32(0);
    mvhd.u32(0);
    mvhd.u32(1000);
    mvhd.u32((uint32_t)dur_ms);
    mvhd.u32(0x00010000);
    mvhd.u16(0x0100);
    mvhd.zeros(10);
    matrix(mvhd);
    mvhd.zeros(24);
    mvhd.u32(2);
    return box("moov", cat({fullbox("mvhd", 0, 0, mvhd.b), trak}));
  };
  Box ftyp;
  ftyp.str("isom", 4);
  ftyp.u32(512);
  ftyp.str("isomiso2hvc1mp41", 16);
  const auto ftyp_box = box("ftyp", ftyp.b);
  const size_t moov_size = build_moov(0).size();
  const uint64_t mdat_hdr = large ? 16 : 8;
  const uint64_t chunk_off = ftyp_box.size() + moov_size + mdat_hdr;
  std::vector<uint8_t> out = ftyp_box;
  const auto moov = build_moov(chunk_off);
  out.insert(out.end(), moov.begin(), moov.end());
  Box mh;
  if (large) {
    mh.u32(1);
    mh.str("mdat", 4);
    mh.u64(mdat_payload + 16);
  } else {
    mh.u32((uint32_t)(mdat_payload + 8));
    mh.str("mdat", 4);
  }
  out.insert(out.end(), mh.b.begin(), mh.b.end());
  return out;
}

void put_len(uint8_t* p, uint32_t v) {
  p[0] = (uint8_t)(v >> 24);
  p[1] = (uint8_t)(v >> 16);
  p[2] = (uint8_t)(v >> 8);
  p[3] = (uint8_t)v;
}

}  // namespace

std::vector<uint8_t> mux_mp4(const uint8_t* annexb, size_t n, int width, int height, int fps_num,
                             int fps_den) {
  const MuxPlan P = plan_mux(&annexb, &n, 1);
  std::vector<uint8_t> out = mp4_header(P, width, height, fps_num, fps_den);
  size_t o = out.size();
  out.resize(o + P.mdat_payload);
  for (const auto& s : P.samples)
    for (const auto& nal : s.nals) {
      put_len(out.data() + o, (uint32_t)nal.size);
      std::memcpy(out.data() + o + 4, nal.data, nal.size);
      o += 4 + nal.size;
    }
  return out;
}

uint64_t mux_mp4_file(const uint8_t* const* segs, const size_t* sizes, int nseg, int width, int height, int fps_num,
                      int fps_den, const char* path) {
  const MuxPlan P = plan_mux(segs, sizes, nseg);
  const std::vector<uint8_t> head = mp4_header(P, width, height, fps_num, fps_den);
  FILE* f = std::fopen(path, "wb");
  if (!f) throw std::runtime_error(std::string("mux_mp4_file: cannot open ") + path);
  std::vector<uint8_t> buf;
  buf.reserve(8 << 20);
  bool ok = std::fwrite(head.data(), 1, head.size(), f) == head.size();
  auto flush = [&] {
    ok = ok && std::fwrite(buf.data(), 1, buf.size(), f) == buf.size();
    buf.clear();
  };
  for (const auto& s : P.samples) {
    for (const auto& nal : s.nals) {
      uint8_t len[4];
      put_len(len, (uint32_t)nal.size);
      buf.insert(buf.end(), len, len + 4);
      buf.insert(buf.end(), nal.data, nal.data + nal.size);
    }
    if (buf.size() >= (8u << 20)) flush();
  }
  flush();
  ok = (std::fclose(f) == 0) && ok;
  if (!ok) throw std::runtime_error(std::string("mux_mp4_file: write failed: ") + path);
  return head.size() + P.mdat_payload;
}

// ------------------------------------- demux --------------------------------------------
namespace {
struct Reader {
  const uint8_t* p;
  size_t n;
  uint32_t u32(size_t o) const {
    if (o + 4 > n) throw std::runtime_error("demux: truncated");
    return (uint32_t)p[o] << 24 | (uint32_t)p[o + 1] << 16 | (uint32_t)p[o + 2] << 8 | p[o + 3];
  }
  uint64_t u64(size_t o) const { return (uint64_t)u32(o) << 32 | u32(o + 4); }
  uint16_t u16(size_t o) const {
    if (o + 2 > n) throw std::runtime_error("demux: truncated");
    return (uint16_t)(p[o] << 8 | p[o + 1]);
  }
};
// find child box of `type` within [start, end); returns payload offset and size
bool find_box(const Reader& r, size_t start, size_t end, const char* type, size_t* off, size_t* sz) {
  size_t o = start;
  while (o + 8 <= end) {
    uint64_t s = r.u32(o);
    size_t hdr = 8;
    if (s == 1) {
      s = r.u64(o + 8);
      hdr = 16;
    } else if (s == 0) {
      s = end - o;
    }
    if (s < hdr || o + s > end) throw std::runtime_error("demux: bad box size");
    if (std::memcmp(r.p + o + 4, type, 4) == 0) {
      *off = o + hdr;
      *sz = (size_t)s - hdr;
      return true;
    }
    o += (size_t)s;
  }
  return false;
}
void need(bool ok, const char* what) {
  if (!ok) throw std::runtime_error(std::string("demux: missing ") + what);
}
}  // namespace

std::vector<uint8_t> demux_mp4(const uint8_t* mp4, size_t n, int* width, int* height, int* nframes,
                               int* timescale, int* sample_delta) {
  Reader r{mp4, n};
  size_t o, s, o2, s2;
  need(find_box(r, 0, n, "moov", &o, &s), "moov");
  need(find_box(r, o, o + s, "trak", &o, &s), "trak");
  size_t tk, tks;
  need(find_box(r, o, o + s, "tkhd", &tk, &tks), "tkhd");
  *width = (int)(r.u32(tk + 4 + 72) >> 16);
  *height = (int)(r.u32(tk + 4 + 76) >> 16);
  need(find_box(r, o, o + s, "mdia", &o, &s), "mdia");
  need(find_box(r, o, o + s, "mdhd", &o2, &s2), "mdhd");
  *timescale = (int)r.u32(o2 + 12);
  need(find_box(r, o, o + s, "minf", &o, &s), "minf");
  need(find_box(r, o, o + s, "stbl", &o, &s), "stbl");
  size_t sd, sds, tt, tts, sz, szs, co, cos;
  need(find_box(r, o, o + s, "stsd", &sd, &sds), "stsd");
  need(find_box(r, o, o + s, "stts", &tt, &tts), "stts");
  need(find_box(r, o, o + s, "stsz", &sz, &szs), "stsz");
  bool co64 = false;
  if (!find_box(r, o, o + s, "stco", &co, &cos)) {
    need(find_box(r, o, o + s, "co64", &co, &cos), "stco");
    co64 = true;
  }
  *sample_delta = (int)r.u32(tt + 12);
  std::vector<uint8_t> out;
  // sample entry: stsd payload = ver/flags(4) count(4) entry
  const size_t entry = sd + 8;
  const size_t entry_size = r.u32(entry);
  const size_t hvcc_search = entry + 8 + 78;
  size_t hc, hcs;
  need(find_box(r, hvcc_search, entry + entry_size, "hvcC", &hc, &hcs), "hvcC");
  size_t p = hc + 22;
  const int narr = mp4[p++];
  for (int a = 0; a < narr; ++a) {
    ++p;
    const int cnt = r.u16(p);
    p += 2;
    for (int k = 0; k < cnt; ++k) {
      const int len = r.u16(p);
      p += 2;
      const uint8_t sc[4] = {0, 0, 0, 1};
      out.insert(out.end(), sc, sc + 4);
      out.insert(out.end(), mp4 + p, mp4 + p + len);
      p += len;
    }
  }
  const uint32_t count = r.u32(sz + 8);
  *nframes = (int)count;
  uint64_t off = co64 ? r.u64(co + 8) : r.u32(co + 8);
  for (uint32_t i = 0; i < count; ++i) {
    const uint32_t ssz = r.u32(sz + 12 + 4 * i);
    uint64_t q = off, end = off + ssz;
    if (end > n) throw std::runtime_error("demux: sample beyond file");
    while (q + 4 <= end) {
      const uint32_t len = r.u32((size_t)q);
      q += 4;
      if (q + len > end) throw std::runtime_error("demux: bad NAL length");
      const uint8_t sc[4] = {0, 0, 0, 1};
      out.insert(out.end(), sc, sc + 4);
      out.insert(out.end(), mp4 + q, mp4 + q + len);
      q += len;
    }
    off = end;
  }
  return out;
}

}  // namespace tv
