// mp4.cpp — ISO-BMFF writer/reader: the HEVC video track plus the source's side streams.
//
// Replaces the reference's `ffmpeg -f concat -c copy -movflags +faststart` stitch step
// (reference worker/tasks.py:2047-2069) and its audio carriage (`-c:a`, :68): the
// concatenated Annex-B segments become 'hvc1' samples (length-prefixed NAL units,
// parameter sets hoisted into hvcC), audio (AAC 'mp4a' / PCM 'sowt') and subtitles
// (3GPP timed text 'tx3g') become further tracks, chunks are interleaved by time (one
// second per chunk) and moov is placed before mdat (faststart layout).
#include <algorithm>
#include <memory>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>

#include "mux_internal.h"
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
  void u24(uint32_t v) {
    u8(v >> 16);
    u16(v);
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

// ISO 639-2/T packed into mdhd's 15 bits ('und' when absent or malformed)
uint16_t pack_lang(const char* l) {
  char c[3] = {'u', 'n', 'd'};
  if (l && l[0] >= 'a' && l[0] <= 'z' && l[1] >= 'a' && l[1] <= 'z' && l[2] >= 'a' && l[2] <= 'z')
    c[0] = l[0], c[1] = l[1], c[2] = l[2];
  return (uint16_t)(((c[0] - 0x60) << 10) | ((c[1] - 0x60) << 5) | (c[2] - 0x60));
}

// MPEG-4 descriptor (tag, expandable size, payload)
void descriptor(Box& o, int tag, const std::vector<uint8_t>& payload) {
  o.u8((uint32_t)tag);
  size_t n = payload.size();
  uint8_t sz[4];
  int k = 0;
  do {
    sz[k++] = (uint8_t)(n & 0x7f);
    n >>= 7;
  } while (n && k < 4);
  for (int i = k - 1; i >= 0; --i) o.u8(sz[i] | (i ? 0x80u : 0u));
  o.bytes(payload);
}

std::vector<uint8_t> audio_entry(const SideTrack& t) {
  if (t.codec == SIDE_MP4_ENTRY) return std::vector<uint8_t>(t.priv, t.priv + t.priv_size);
  Box a;
  a.zeros(6);
  a.u16(1);
  a.zeros(8);
  a.u16((uint32_t)std::max(1, t.channels));
  a.u16(16);
  a.u32(0);
  a.u32((uint32_t)std::min(t.sample_rate, 65535) << 16);
  if (t.codec == SIDE_PCM_S16LE) return box("sowt", a.b);
  // esds: ES_Descriptor{DecoderConfigDescriptor{DecoderSpecificInfo = ASC}, SLConfig}
  Box dsi, dcd, es, sl;
  dsi.bytes(t.priv, (size_t)t.priv_size);
  dcd.u8(0x40);  // MPEG-4 audio
  dcd.u8((0x05 << 2) | 1);
  dcd.u24(0);
  dcd.u32(0);
  dcd.u32(0);
  descriptor(dcd, 0x05, dsi.b);
  es.u16(0);
  es.u8(0);
  descriptor(es, 0x04, dcd.b);
  sl.u8(2);
  descriptor(es, 0x06, sl.b);
  Box esd;
  descriptor(esd, 0x03, es.b);
  a.bytes(fullbox("esds", 0, 0, esd.b));
  return box("mp4a", a.b);
}

std::vector<uint8_t> text_entry() {  // 3GPP TS 26.245 TextSampleEntry, bottom-centred white
  Box t;
  t.zeros(6);
  t.u16(1);
  t.u32(0);       // displayFlags
  t.u8(1);        // horizontal: centre
  t.u8(0xff);     // vertical: bottom
  t.u32(0);       // background rgba
  t.zeros(8);     // BoxRecord
  t.u16(0);       // StyleRecord: startChar
  t.u16(0);       //   endChar
  t.u16(1);       //   font-ID
  t.u8(0);        //   face-style-flags
  t.u8(18);       //   font-size
  t.u32(0xffffffff);
  Box ft;
  ft.u16(1);
  ft.u16(1);
  ft.u8(5);
  ft.str("Serif", 5);
  t.bytes(box("ftab", ft.b));
  return box("tx3g", t.b);
}

// Sample/chunk tables of one trak
struct TrakTables {
  uint64_t nsamples = 0;
  uint32_t const_size = 0;             // stsz sample_size (PCM frames) or 0 = per-sample table
  std::vector<uint32_t> sizes;
  std::vector<std::pair<uint32_t, uint32_t>> stts;  // (count, delta)
  std::vector<uint32_t> chunk_n;       // samples per chunk
  std::vector<uint64_t> chunk_off;     // filled once the mdat layout is known
  std::vector<uint32_t> sync;          // 1-based; empty = every sample is a sync sample
  bool has_stss = false;
  uint64_t media_dur = 0;
  // B frames: composition offsets (count, offset) and the edit list's media_time that maps
  // the first displayed frame to time 0 (offsets are shifted to be non-negative)
  std::vector<std::pair<uint32_t, uint32_t>> ctts;
  int64_t edit_media_time = -1;
  void ctts_from(const std::vector<int>& cto, uint32_t delta) {
    int mn = 0;
    for (int c : cto) mn = std::min(mn, c);
    for (int c : cto) {
      const uint32_t o = (uint32_t)(c - mn) * delta;
      if (!ctts.empty() && ctts.back().second == o) ++ctts.back().first;
      else ctts.push_back({1, o});
    }
    edit_media_time = (int64_t)(-mn) * delta;
  }
  void delta(uint32_t d) {
    if (!stts.empty() && stts.back().second == d) ++stts.back().first;
    else stts.push_back({1, d});
    media_dur += d;
  }
};

// One mdat chunk: `count` consecutive samples of a track, written at time `t` (seconds).
// For subtitles `first` indexes the expanded (gap-filled) sample list.
struct Chunk {
  int track;  // 0 = video, k = side track k-1
  int64_t first, count;
  double t;
  uint64_t bytes;
};

// Subtitle cues on a continuous timeline: 3GPP text tracks have no gaps, so the time
// between cues becomes empty samples (index -1).
struct TextSample {
  int64_t src;
  uint32_t dur;
};
std::vector<TextSample> text_timeline(const SideTrack& t) {
  std::vector<TextSample> out;
  int64_t cur = 0;
  for (int64_t i = 0; i < t.nsamples; ++i) {
    const int64_t p = std::max<int64_t>(t.pts[i], cur);
    if (p > cur) out.push_back({-1, (uint32_t)(p - cur)});
    int64_t end = std::max<int64_t>(t.pts[i] + (int64_t)t.durs[i], p + 1);
    if (i + 1 < t.nsamples && t.pts[i + 1] > p) end = std::min<int64_t>(end, t.pts[i + 1]);  // overlap: cut
    out.push_back({i, (uint32_t)(end - p)});
    cur = end;
  }
  return out;
}

std::vector<uint8_t> stbl_box(const std::vector<uint8_t>& entry, const TrakTables& T, bool large) {
  Box stsd;
  stsd.u32(1);
  stsd.bytes(entry);
  Box stts;
  stts.u32((uint32_t)T.stts.size());
  for (auto [c, d] : T.stts) {
    stts.u32(c);
    stts.u32(d);
  }
  Box stsc;  // runs of equal samples-per-chunk
  {
    std::vector<std::pair<uint32_t, uint32_t>> runs;
    for (size_t c = 0; c < T.chunk_n.size(); ++c)
      if (runs.empty() || runs.back().second != T.chunk_n[c]) runs.push_back({(uint32_t)c + 1, T.chunk_n[c]});
    stsc.u32((uint32_t)runs.size());
    for (auto [first, n] : runs) {
      stsc.u32(first);
      stsc.u32(n);
      stsc.u32(1);
    }
  }
  Box stsz;
  stsz.u32(T.const_size);
  stsz.u32((uint32_t)T.nsamples);
  if (!T.const_size)
    for (auto s : T.sizes) stsz.u32(s);
  Box co;
  co.u32((uint32_t)T.chunk_off.size());
  for (auto o : T.chunk_off) {
    if (large) co.u64(o);
    else co.u32((uint32_t)o);
  }
  std::vector<uint8_t> parts = cat({fullbox("stsd", 0, 0, stsd.b), fullbox("stts", 0, 0, stts.b)});
  if (!T.ctts.empty()) {
    Box ctts;
    ctts.u32((uint32_t)T.ctts.size());
    for (auto [c, o] : T.ctts) {
      ctts.u32(c);
      ctts.u32(o);
    }
    parts = cat({parts, fullbox("ctts", 0, 0, ctts.b)});
  }
  if (T.has_stss) {
    Box stss;
    stss.u32((uint32_t)T.sync.size());
    for (auto s : T.sync) stss.u32(s);
    parts = cat({parts, fullbox("stss", 0, 0, stss.b)});
  }
  return box("stbl", cat({parts, fullbox("stsc", 0, 0, stsc.b), fullbox("stsz", 0, 0, stsz.b),
                          fullbox(large ? "co64" : "stco", 0, 0, co.b)}));
}

struct TrakInfo {
  uint32_t id;
  const char* handler;  // 'vide' / 'soun' / 'sbtl'
  const char* hname;
  uint32_t timescale;
  uint16_t lang;
  bool enabled;
  uint16_t alt_group, volume;
  int width, height;  // tkhd presentation size (video / text)
  std::vector<uint8_t> entry;
};

std::vector<uint8_t> trak_box(const TrakInfo& I, const TrakTables& T, bool large) {
  const uint64_t dur_ms = T.media_dur * 1000 / I.timescale;
  Box vmhd;
  vmhd.zeros(8);
  Box smhd;
  smhd.zeros(4);
  std::vector<uint8_t> mhd;
  if (!std::strcmp(I.handler, "vide")) mhd = fullbox("vmhd", 0, 1, vmhd.b);
  else if (!std::strcmp(I.handler, "soun")) mhd = fullbox("smhd", 0, 0, smhd.b);
  else mhd = fullbox("nmhd", 0, 0, {});
  Box dref;
  dref.u32(1);
  dref.bytes(fullbox("url ", 0, 1, {}));
  const auto dinf = box("dinf", fullbox("dref", 0, 0, dref.b));
  const auto minf = box("minf", cat({mhd, dinf, stbl_box(I.entry, T, large)}));
  Box mdhd;
  mdhd.u32(0);
  mdhd.u32(0);
  mdhd.u32(I.timescale);
  mdhd.u32((uint32_t)T.media_dur);
  mdhd.u16(I.lang);
  mdhd.u16(0);
  Box hdlr;
  hdlr.u32(0);
  hdlr.str(I.handler, 4);
  hdlr.zeros(12);
  hdlr.str(I.hname, std::strlen(I.hname) + 1);
  const auto mdia = box("mdia", cat({fullbox("mdhd", 0, 0, mdhd.b), fullbox("hdlr", 0, 0, hdlr.b), minf}));
  Box tkhd;
  tkhd.u32(0);
  tkhd.u32(0);
  tkhd.u32(I.id);
  tkhd.u32(0);
  tkhd.u32((uint32_t)dur_ms);
  tkhd.zeros(8);
  tkhd.u16(0);            // layer
  tkhd.u16(I.alt_group);
  tkhd.u16(I.volume);
  tkhd.u16(0);
  matrix(tkhd);
  tkhd.u32((uint32_t)I.width << 16);
  tkhd.u32((uint32_t)I.height << 16);
  if (T.edit_media_time >= 0) {  // edts/elst: the presentation starts at the first display frame
    Box elst;
    elst.u32(1);
    elst.u32((uint32_t)dur_ms);  // segment_duration (movie timescale, ms)
    elst.u32((uint32_t)T.edit_media_time);
    elst.u32(0x00010000);        // media_rate 1.0
    const auto edts = box("edts", fullbox("elst", 0, 0, elst.b));
    return box("trak", cat({fullbox("tkhd", 0, I.enabled ? 3 : 2, tkhd.b), edts, mdia}));
  }
  return box("trak", cat({fullbox("tkhd", 0, I.enabled ? 3 : 2, tkhd.b), mdia}));
}

}  // namespace

namespace muxi {

bool is_av1_stream(const uint8_t* p, size_t n) { return n >= 2 && p[0] == 0x12 && p[1] == 0x00; }

namespace {
size_t leb128(const uint8_t* p, size_t n, size_t& pos) {
  size_t v = 0;
  for (int i = 0; i < 8; ++i) {
    if (pos >= n) throw std::runtime_error("mux: truncated AV1 OBU size");
    const uint8_t b = p[pos++];
    v |= (size_t)(b & 0x7f) << (7 * i);
    if (!(b & 0x80)) return v;
  }
  throw std::runtime_error("mux: bad AV1 OBU size");
}
MuxPlan plan_mux_av1(const uint8_t* const* segs, const size_t* sizes, int nseg) {
  MuxPlan P;
  P.codec = MUX_AV1;
  std::vector<uint8_t> seqhdr;
  for (int k = 0; k < nseg; ++k) {
    const uint8_t* p = segs[k];
    const size_t n = sizes[k];
    size_t pos = 0;
    Sample* cur = nullptr;
    bool seen_frame = false;
    while (pos < n) {
      const size_t start = pos;
      const uint8_t h = p[pos++];
      const int type = (h >> 3) & 15;
      if (h & 4) ++pos;  // extension header
      if (!(h & 2)) throw std::runtime_error("mux: AV1 OBU without a size field");
      const size_t sz = leb128(p, n, pos);
      if (pos + sz > n) throw std::runtime_error("mux: truncated AV1 OBU");
      const size_t end = pos + sz;
      if (type == 2) {  // temporal delimiter: a new sample starts after it
        P.samples.emplace_back();
        cur = &P.samples.back();
        cur->raw = true;
        seen_frame = false;
        pos = end;
        continue;
      }
      if (!cur) throw std::runtime_error("mux: AV1 stream does not start with a temporal delimiter");
      if (type == 1 && seqhdr.empty()) seqhdr.assign(p + start, p + end);
      if ((type == 6 || type == 3) && sz > 0 && !seen_frame) {  // first frame header of the TU
        seen_frame = true;
        cur->sync = !(p[pos] >> 7) && ((p[pos] >> 5) & 3) == 0;  // not show_existing, KEY_FRAME
      }
      if (!cur->nals.empty() && cur->nals.back().data + cur->nals.back().size == p + start)
        cur->nals.back().size += end - start;  // contiguous OBUs stay one view
      else
        cur->nals.push_back(NalView{p + start, end - start});
      pos = end;
    }
  }
  if (seqhdr.empty()) throw std::runtime_error("mux: AV1 stream without a sequence header");
  // AV1CodecConfigurationRecord: marker/version, profile/level, tier + colour flags (8-bit
  // 4:2:0, chroma_sample_position 0: the encoder's sequence header), no presentation delay
  P.av1c = {0x81, (uint8_t)((0 << 5) | 31), 0x0C, 0x00};
  P.av1c.insert(P.av1c.end(), seqhdr.begin(), seqhdr.end());
  for (auto& s : P.samples) {
    s.size = 0;
    for (const auto& v : s.nals) s.size += (uint32_t)v.size;
    P.mdat_payload += s.size;
  }
  return P;
}
}  // namespace

MuxPlan plan_mux(const uint8_t* const* segs, const size_t* sizes, int nseg) {
  if (nseg > 0 && is_av1_stream(segs[0], sizes[0])) return plan_mux_av1(segs, sizes, nseg);
  MuxPlan P;
  std::vector<NalView> pending_ps;
  for (int k = 0; k < nseg; ++k) {
    const size_t first = P.samples.size();
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
    // composition offsets from the slice POCs (hierarchical-B segments are reordered)
    const std::vector<int> off = display_offsets(segs[k], sizes[k]);
    if (off.size() != P.samples.size() - first) throw std::runtime_error("mux: picture count mismatch");
    for (size_t i = 0; i < off.size(); ++i) {
      P.samples[first + i].cto = off[i];
      P.reordered = P.reordered || off[i] != 0;
    }
  }
  if (P.sps.empty() || P.pps.empty() || P.vps.empty()) throw std::runtime_error("mux: missing parameter sets");
  for (auto& s : P.samples) {
    if (P.ps_consistent) s.nals.erase(s.nals.begin(), s.nals.end() - 1);  // parameter sets live in hvcC
    s.size = 0;
    for (const auto& n : s.nals) s.size += 4 + (uint32_t)n.size;
    P.mdat_payload += s.size;
  }
  return P;
}

std::vector<uint8_t> hvcc_record(const MuxPlan& P) {
  std::vector<uint8_t> sps_rbsp = unescape_rbsp(P.sps.data() + 2, P.sps.size() - 2);
  if (sps_rbsp.size() < 13) throw std::runtime_error("mux: short SPS");
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
  return hv.b;
}

}  // namespace muxi

namespace {

using muxi::MuxPlan;

// VisualSampleEntry of the video track: 'hvc1' / 'hev1' + hvcC, or 'av01' + av1C
std::vector<uint8_t> visual_entry(const muxi::MuxPlan& P, int width, int height) {
  Box se;
  se.zeros(6);
  se.u16(1);
  se.zeros(16);
  se.u16((uint32_t)width);
  se.u16((uint32_t)height);
  se.u32(0x00480000);
  se.u32(0x00480000);
  se.u32(0);
  se.u16(1);
  char name[32] = {0};
  const char* nm = P.codec == muxi::MUX_AV1 ? "thinvids-amd AV1" : "thinvids-amd HEVC";
  name[0] = (char)std::strlen(nm);
  std::memcpy(name + 1, nm, std::strlen(nm));
  se.str(name, 32);
  se.u16(0x0018);
  se.u16(0xffff);
  if (P.codec == muxi::MUX_AV1) {
    se.bytes(box("av1C", P.av1c));
    return box("av01", se.b);
  }
  se.bytes(box("hvcC", muxi::hvcc_record(P)));
  return box(P.ps_consistent ? "hvc1" : "hev1", se.b);
}

// moov of the given tracks (chunk offsets already filled in)
std::vector<uint8_t> moov_box(const std::vector<TrakInfo>& I, const std::vector<TrakTables>& T, bool large) {
  uint64_t movie_ms = 0;
  for (size_t k = 0; k < T.size(); ++k) movie_ms = std::max(movie_ms, T[k].media_dur * 1000 / I[k].timescale);
  Box mvhd;
  mvhd.u32(0);
  mvhd.u32(0);
  mvhd.u32(1000);
  mvhd.u32((uint32_t)movie_ms);
  mvhd.u32(0x00010000);
  mvhd.u16(0x0100);
  mvhd.zeros(10);
  matrix(mvhd);
  mvhd.zeros(24);
  mvhd.u32((uint32_t)T.size() + 1);
  std::vector<uint8_t> body = fullbox("mvhd", 0, 0, mvhd.b);
  for (size_t k = 0; k < T.size(); ++k) {
    const auto tb = trak_box(I[k], T[k], large);
    body.insert(body.end(), tb.begin(), tb.end());
  }
  return box("moov", body);
}

std::vector<uint8_t> ftyp_box(int codec) {
  Box ftyp;
  ftyp.str("isom", 4);
  ftyp.u32(512);
  ftyp.str(codec == muxi::MUX_AV1 ? "isomiso2av01mp41" : "isomiso2hvc1mp41", 16);
  return box("ftyp", ftyp.b);
}

// Faststart MP4 of the plan + side tracks.  Returns the file size.
// Output goes to `mem` when it is non-null, else to the file `path`.
uint64_t write_mp4(const MuxPlan& P, int width, int height, int fps_num, int fps_den, const SideTrack* tracks,
                   int ntracks, const char* path, std::vector<uint8_t>* mem = nullptr) {
  const int ntrak = 1 + ntracks;
  std::vector<TrakTables> T(ntrak);
  std::vector<TrakInfo> I(ntrak);
  std::vector<std::vector<TextSample>> text(ntrak);
  std::vector<Chunk> chunks;
  // ---- video: one chunk per second when interleaving, one chunk otherwise
  const uint32_t vts = (uint32_t)fps_num * 1000u, vdelta = (uint32_t)fps_den * 1000u;
  {
    auto& V = T[0];
    V.nsamples = P.samples.size();
    V.has_stss = true;
    for (size_t i = 0; i < P.samples.size(); ++i) {
      V.sizes.push_back(P.samples[i].size);
      V.delta(vdelta);
      if (P.samples[i].sync) V.sync.push_back((uint32_t)i + 1);
    }
    if (P.reordered) {
      std::vector<int> cto;
      for (const auto& smp : P.samples) cto.push_back(smp.cto);
      V.ctts_from(cto, vdelta);
    }
    const int64_t per = ntracks ? std::max<int64_t>(1, (fps_num + fps_den - 1) / fps_den) : (int64_t)V.nsamples;
    for (int64_t f = 0; f < (int64_t)V.nsamples; f += per) {
      const int64_t n = std::min<int64_t>(per, (int64_t)V.nsamples - f);
      uint64_t b = 0;
      for (int64_t i = f; i < f + n; ++i) b += P.samples[i].size;
      chunks.push_back({0, f, n, (double)f * fps_den / fps_num, b});
      V.chunk_n.push_back((uint32_t)n);
    }
    I[0] = {1, "vide", "VideoHandler", vts, pack_lang(nullptr), true, 0, 0, width, height, visual_entry(P, width, height)};
  }
  // ---- side tracks
  bool first_audio = true;
  for (int k = 0; k < ntracks; ++k) {
    const SideTrack& t = tracks[k];
    muxi::check_side(t, false);
    auto& S = T[k + 1];
    const int tk = k + 1;
    const double ts = t.timescale;
    if (t.kind == SIDE_AUDIO) {
      const bool pcm = t.codec == SIDE_PCM_S16LE;
      I[tk] = {(uint32_t)tk + 1, "soun", "SoundHandler", (uint32_t)t.timescale, pack_lang(t.lang), first_audio,
               1, 0x0100, 0, 0, audio_entry(t)};
      first_audio = false;
      if (pcm) {  // one MP4 sample per PCM frame, one chunk per source block
        const uint32_t fb = (uint32_t)t.channels * 2;
        S.const_size = fb;
        for (int64_t i = 0; i < t.nsamples; ++i) {
          const uint32_t n = t.sizes[i] / fb;
          if (!n) continue;
          S.nsamples += n;
          if (!S.stts.empty()) S.stts.back().first += n;
          else S.stts.push_back({n, 1});
          S.media_dur += n;
          S.chunk_n.push_back(n);
          chunks.push_back({tk, i, 1, t.pts[i] / ts, (uint64_t)n * fb});
        }
      } else {  // AAC access units, ~1 s per chunk
        int64_t f = 0;
        while (f < t.nsamples) {
          int64_t e = f;
          uint64_t b = 0, d = 0;
          while (e < t.nsamples && (e == f || d < (uint64_t)t.timescale)) {
            b += t.sizes[e];
            d += t.durs[e];
            S.sizes.push_back(t.sizes[e]);
            S.delta(t.durs[e]);
            ++e;
          }
          chunks.push_back({tk, f, e - f, t.pts[f] / ts, b});
          S.chunk_n.push_back((uint32_t)(e - f));
          f = e;
        }
        S.nsamples = (uint64_t)t.nsamples;
      }
    } else {  // subtitles: tx3g samples (u16 length + UTF-8), gaps as empty samples
      if (t.codec != SIDE_SUBRIP) throw std::runtime_error("mux: MP4 carries text subtitles only");
      I[tk] = {(uint32_t)tk + 1, "sbtl", "SubtitleHandler", (uint32_t)t.timescale, pack_lang(t.lang),
               t.is_default != 0, 2, 0, width, height, text_entry()};
      text[tk] = text_timeline(t);
      int64_t at = 0;
      for (size_t j = 0; j < text[tk].size(); ++j) {
        const auto& x = text[tk][j];
        const uint32_t sz = 2 + (x.src >= 0 ? t.sizes[x.src] : 0);
        S.sizes.push_back(sz);
        S.delta(x.dur);
        S.chunk_n.push_back(1);
        chunks.push_back({tk, (int64_t)j, 1, at / ts, sz});
        at += x.dur;
      }
      S.nsamples = text[tk].size();
    }
  }
  // ---- layout: chunks in time order (video first on ties), offsets after the header
  std::stable_sort(chunks.begin(), chunks.end(), [](const Chunk& a, const Chunk& b) {
    return a.t < b.t || (a.t == b.t && a.track < b.track);
  });
  uint64_t payload = 0;
  for (const auto& c : chunks) payload += c.bytes;
  const bool large = payload + (1 << 20) > 0xffffffffull;
  auto build_moov = [&](uint64_t base) {
    for (auto& x : T) x.chunk_off.clear();
    uint64_t o = base;
    for (const auto& c : chunks) {
      T[c.track].chunk_off.push_back(o);
      o += c.bytes;
    }
    return moov_box(I, T, large);
  };
  const auto ftyp_b = ftyp_box(P.codec);
  const uint64_t mdat_hdr = large ? 16 : 8;
  const size_t moov_size = build_moov(0).size();  // offsets do not change the size
  std::vector<uint8_t> head = ftyp_b;
  const auto moov = build_moov(ftyp_b.size() + moov_size + mdat_hdr);
  head.insert(head.end(), moov.begin(), moov.end());
  Box mh;
  if (large) {
    mh.u32(1);
    mh.str("mdat", 4);
    mh.u64(payload + 16);
  } else {
    mh.u32((uint32_t)(payload + 8));
    mh.str("mdat", 4);
  }
  head.insert(head.end(), mh.b.begin(), mh.b.end());
  // ---- payload, streamed
  std::vector<std::unique_ptr<muxi::SideReader>> rd;
  for (int k = 0; k < ntracks; ++k) rd.emplace_back(new muxi::SideReader(tracks[k]));
  FILE* f = nullptr;
  if (!mem) {
    f = std::fopen(path, "wb");
    if (!f) throw std::runtime_error(std::string("mux: cannot open ") + path);
  }
  std::vector<uint8_t> local;
  std::vector<uint8_t>& buf = mem ? *mem : local;
  buf.clear();
  buf.reserve(mem ? head.size() + payload : (8u << 20));
  bool ok = true;
  auto flush = [&] {
    if (f) {
      ok = ok && std::fwrite(buf.data(), 1, buf.size(), f) == buf.size();
      buf.clear();
    }
  };
  buf.insert(buf.end(), head.begin(), head.end());
  try {
    for (const auto& c : chunks) {
      if (c.track == 0) {
        for (int64_t i = c.first; i < c.first + c.count; ++i) muxi::append_sample(P.samples[i], buf);
      } else {
        const SideTrack& t = tracks[c.track - 1];
        if (t.kind == SIDE_SUBTITLE) {
          const auto& x = text[c.track][c.first];
          const uint32_t n = x.src >= 0 ? t.sizes[x.src] : 0;
          buf.push_back((uint8_t)(n >> 8));
          buf.push_back((uint8_t)n);
          if (x.src >= 0) rd[c.track - 1]->append(x.src, buf);
        } else if (t.codec == SIDE_PCM_S16LE) {
          const size_t o = buf.size();
          rd[c.track - 1]->append(c.first, buf);
          buf.resize(o + c.bytes);  // whole frames only
        } else {
          for (int64_t i = c.first; i < c.first + c.count; ++i) rd[c.track - 1]->append(i, buf);
        }
      }
      if (buf.size() >= (8u << 20)) flush();
    }
    flush();
  } catch (...) {
    if (f) std::fclose(f);
    throw;
  }
  if (f) ok = (std::fclose(f) == 0) && ok;
  if (!ok) throw std::runtime_error(std::string("mux: write failed: ") + path);
  return head.size() + payload;
}

// Streaming faststart writer of one video track (no side tracks): segments are appended as
// they arrive and their samples go straight to disk; the head (ftyp + moov + 'free' padding)
// is reserved up front from the sample-count bound and written in place at close(), so the
// finished file is faststart without a second copy of the payload.  The moov size is bounded
// by a fixed part plus 12 bytes per sample (stsz 4 + stss 4 when every sample were a sync
// sample, + slack); co64 chunk offsets make the bound independent of the file size.
class Mp4Stream {
 public:
  Mp4Stream(const char* path, int width, int height, int fps_num, int fps_den, uint64_t max_samples)
      : path_(path), w_(width), h_(height), fn_(fps_num), fd_(fps_den), max_(max_samples) {
    if (fps_num <= 0 || fps_den <= 0) throw std::runtime_error("mux stream: bad frame rate");
    if (!max_samples) throw std::runtime_error("mux stream: no samples expected");
    reserve_ = 8192 + 20 * max_samples;  // stsz + stss + ctts entries
    f_ = std::fopen(path, "wb");
    if (!f_) throw std::runtime_error(std::string("mux stream: cannot open ") + path);
    std::vector<uint8_t> z(reserve_, 0);
    if (std::fwrite(z.data(), 1, z.size(), f_) != z.size()) fail("write failed");
  }
  ~Mp4Stream() {
    if (f_) std::fclose(f_);
  }
  void append(const uint8_t* seg, size_t n) {
    if (!f_) throw std::runtime_error("mux stream: closed");
    const MuxPlan P = muxi::plan_mux(&seg, &n, 1);
    if (!have_) {
      head_.codec = P.codec;
      head_.vps = P.vps;
      head_.sps = P.sps;
      head_.pps = P.pps;
      head_.av1c = P.av1c;
      have_ = true;
    } else if (P.codec != head_.codec || P.vps != head_.vps || P.sps != head_.sps || P.pps != head_.pps ||
               P.av1c != head_.av1c || !P.ps_consistent) {
      fail("segments with different parameter sets (use the whole-job muxer)");
    }
    if (!P.ps_consistent) fail("segment with inconsistent parameter sets");
    if (sizes_.size() + P.samples.size() > max_) fail("more samples than reserved");
    buf_.clear();
    for (const auto& smp : P.samples) {
      muxi::append_sample(smp, buf_);
      sizes_.push_back(smp.size);
      cto_.push_back(smp.cto);
      reordered_ = reordered_ || smp.cto != 0;
      if (smp.sync) sync_.push_back((uint32_t)sizes_.size());
    }
    if (std::fwrite(buf_.data(), 1, buf_.size(), f_) != buf_.size()) fail("write failed");
    payload_ += buf_.size();
  }
  uint64_t close() {
    if (!f_) throw std::runtime_error("mux stream: closed");
    if (!have_ || sizes_.empty()) fail("no samples");
    std::vector<TrakTables> T(1);
    std::vector<TrakInfo> I(1);
    auto& V = T[0];
    V.nsamples = sizes_.size();
    V.has_stss = true;
    V.sizes = sizes_;
    V.sync = sync_;
    for (size_t i = 0; i < sizes_.size(); ++i) V.delta((uint32_t)fd_ * 1000u);
    if (reordered_) V.ctts_from(cto_, (uint32_t)fd_ * 1000u);
    V.chunk_n = {(uint32_t)sizes_.size()};
    V.chunk_off = {reserve_};
    I[0] = {1, "vide", "VideoHandler", (uint32_t)fn_ * 1000u, pack_lang(nullptr), true, 0, 0, w_, h_,
            visual_entry(head_, w_, h_)};
    const auto ftyp = ftyp_box(head_.codec);
    const auto moov = moov_box(I, T, true);
    const uint64_t used = ftyp.size() + moov.size() + 16;  // + the 64-bit mdat header
    if (used + 8 > reserve_) fail("moov exceeds the reserved head");
    Box head;
    head.bytes(ftyp);
    head.bytes(moov);
    head.u32((uint32_t)(reserve_ - used));  // 'free' padding up to the mdat header
    head.str("free", 4);
    head.zeros(reserve_ - used - 8);
    head.u32(1);
    head.str("mdat", 4);
    head.u64(payload_ + 16);
    if (head.b.size() != reserve_) fail("head layout");
    if (std::fseek(f_, 0, SEEK_SET) != 0 || std::fwrite(head.b.data(), 1, head.b.size(), f_) != head.b.size())
      fail("head write failed");
    const bool ok = std::fclose(f_) == 0;
    f_ = nullptr;
    if (!ok) throw std::runtime_error("mux stream: close failed: " + path_);
    return reserve_ + payload_;
  }
  uint64_t samples() const { return sizes_.size(); }

 private:
  [[noreturn]] void fail(const char* what) {
    throw std::runtime_error(std::string("mux stream: ") + what + ": " + path_);
  }
  std::string path_;
  int w_, h_, fn_, fd_;
  uint64_t max_, reserve_ = 0, payload_ = 0;
  FILE* f_ = nullptr;
  MuxPlan head_;
  bool have_ = false;
  std::vector<uint32_t> sizes_, sync_;
  std::vector<int> cto_;
  bool reordered_ = false;
  std::vector<uint8_t> buf_;
};

}  // namespace

uint64_t mux_file(const uint8_t* const* segs, const size_t* sizes, int nseg, int width, int height, int fps_num,
                  int fps_den, const SideTrack* tracks, int ntracks, int container, const char* path) {
  if (fps_num <= 0 || fps_den <= 0) throw std::runtime_error("mux: bad frame rate");
  const MuxPlan P = muxi::plan_mux(segs, sizes, nseg);
  if (container == CONTAINER_MKV) return muxi::write_mkv(P, width, height, fps_num, fps_den, tracks, ntracks, path);
  return write_mp4(P, width, height, fps_num, fps_den, tracks, ntracks, path);
}

uint64_t mux_mp4_file(const uint8_t* const* segs, const size_t* sizes, int nseg, int width, int height, int fps_num,
                      int fps_den, const char* path) {
  return mux_file(segs, sizes, nseg, width, height, fps_num, fps_den, nullptr, 0, CONTAINER_MP4, path);
}

std::vector<uint8_t> mux_mp4(const uint8_t* annexb, size_t n, int width, int height, int fps_num,
                             int fps_den) {
  if (fps_num <= 0 || fps_den <= 0) throw std::runtime_error("mux: bad frame rate");
  std::vector<uint8_t> out;
  write_mp4(muxi::plan_mux(&annexb, &n, 1), width, height, fps_num, fps_den, nullptr, 0, nullptr, &out);
  return out;
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
  size_t mo, ms;
  need(find_box(r, 0, n, "moov", &mo, &ms), "moov");
  // the video trak: the first whose handler is 'vide' (side-stream traks are skipped)
  size_t o = 0, s = 0, to = mo, tkh = 0;
  bool found = false;
  while (!found) {
    size_t t, ts;
    need(find_box(r, to, mo + ms, "trak", &t, &ts), "video trak");
    to = t + ts;
    size_t md, mds, hd, hds;
    if (find_box(r, t, t + ts, "mdia", &md, &mds) && find_box(r, md, md + mds, "hdlr", &hd, &hds) &&
        hd + 12 <= n && std::memcmp(mp4 + hd + 8, "vide", 4) == 0) {
      size_t tks;
      need(find_box(r, t, t + ts, "tkhd", &tkh, &tks), "tkhd");
      o = md;
      s = mds;
      found = true;
    }
  }
  size_t o2, s2;
  *width = (int)(r.u32(tkh + 4 + 72) >> 16);
  *height = (int)(r.u32(tkh + 4 + 76) >> 16);
  need(find_box(r, o, o + s, "mdhd", &o2, &s2), "mdhd");
  *timescale = (int)r.u32(o2 + 12);
  need(find_box(r, o, o + s, "minf", &o, &s), "minf");
  need(find_box(r, o, o + s, "stbl", &o, &s), "stbl");
  size_t sd, sds, tt, tts, sz, szs, sc, scs, co, cos;
  need(find_box(r, o, o + s, "stsd", &sd, &sds), "stsd");
  need(find_box(r, o, o + s, "stts", &tt, &tts), "stts");
  need(find_box(r, o, o + s, "stsz", &sz, &szs), "stsz");
  need(find_box(r, o, o + s, "stsc", &sc, &scs), "stsc");
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
      if (p + len > n) throw std::runtime_error("demux: truncated hvcC");
      const uint8_t scode[4] = {0, 0, 0, 1};
      out.insert(out.end(), scode, scode + 4);
      out.insert(out.end(), mp4 + p, mp4 + p + len);
      p += len;
    }
  }
  const uint32_t const_size = r.u32(sz + 4);
  const uint32_t count = r.u32(sz + 8);
  *nframes = (int)count;
  const uint32_t nchunks = r.u32(co + 4), nsc = r.u32(sc + 4);
  // walk chunks (stsc runs) and their samples
  uint32_t i = 0;
  for (uint32_t e = 0; e < nsc && i < count; ++e) {
    const uint32_t first = r.u32(sc + 8 + 12 * e), per = r.u32(sc + 8 + 12 * e + 4);
    const uint32_t last = e + 1 < nsc ? r.u32(sc + 8 + 12 * (e + 1)) - 1 : nchunks;
    if (first < 1 || last > nchunks) throw std::runtime_error("demux: bad stsc");
    for (uint32_t c = first; c <= last && i < count; ++c) {
      uint64_t off = co64 ? r.u64(co + 8 + 8 * (size_t)(c - 1)) : r.u32(co + 8 + 4 * (size_t)(c - 1));
      for (uint32_t k = 0; k < per && i < count; ++k, ++i) {
        const uint32_t ssz = const_size ? const_size : r.u32(sz + 12 + 4 * (size_t)i);
        uint64_t q = off, end = off + ssz;
        if (end > n) throw std::runtime_error("demux: sample beyond file");
        while (q + 4 <= end) {
          const uint32_t len = r.u32((size_t)q);
          q += 4;
          if (q + len > end) throw std::runtime_error("demux: bad NAL length");
          const uint8_t scode[4] = {0, 0, 0, 1};
          out.insert(out.end(), scode, scode + 4);
          out.insert(out.end(), mp4 + q, mp4 + q + len);
          q += len;
        }
        off = end;
      }
    }
  }
  if (i != count) throw std::runtime_error("demux: sample table shorter than stsz");
  return out;
}

}  // namespace tv

// ------------------------------------- streaming writer C API ---------------------------
namespace {
thread_local std::string g_mp4s_err;
}
extern "C" {
void* tv_mp4s_open(const char* path, int width, int height, int fps_num, int fps_den, unsigned long long max_samples) {
  try {
    return new tv::Mp4Stream(path, width, height, fps_num, fps_den, max_samples);
  } catch (const std::exception& e) {
    g_mp4s_err = e.what();
    return nullptr;
  }
}
int tv_mp4s_append(void* h, const uint8_t* data, size_t n) {
  try {
    static_cast<tv::Mp4Stream*>(h)->append(data, n);
    return 0;
  } catch (const std::exception& e) {
    g_mp4s_err = e.what();
    return -1;
  }
}
// finishes the file (returns 0 and its size in *bytes) and frees the handle either way
int tv_mp4s_close(void* h, unsigned long long* bytes) {
  auto* s = static_cast<tv::Mp4Stream*>(h);
  int rc = 0;
  try {
    *bytes = s->close();
  } catch (const std::exception& e) {
    g_mp4s_err = e.what();
    rc = -1;
  }
  delete s;
  return rc;
}
void tv_mp4s_abort(void* h) { delete static_cast<tv::Mp4Stream*>(h); }
const char* tv_mp4s_last_error() { return g_mp4s_err.c_str(); }
}
