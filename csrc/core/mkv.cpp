// mkv.cpp — Matroska writer: HEVC video + the source's audio and subtitle streams.
//
// The reference switches the final container to .mkv whenever the source carries
// copy-safe English subtitles and remuxes them with ffmpeg (reference
// worker/tasks.py:2126-2223, codec list :536-546).  This writer produces that file
// directly from the gathered segment buffers: EBML header, Segment{SeekHead, Info,
// Tracks, Clusters, Cues}.  Timestamps are in milliseconds (TimestampScale 1e6 ns); a
// cluster starts at every video keyframe (and at least every 5 s), and each keyframe
// cluster gets a CuePoint, so players seek to GOP starts.  Side streams are copied
// sample for sample (SimpleBlock; subtitles as BlockGroup + BlockDuration).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>

#include "mux_internal.h"

namespace tv {
namespace muxi {

namespace {

// EBML element IDs (Matroska specification, RFC 9559)
enum : uint32_t {
  kEBML = 0x1A45DFA3, kEBMLVersion = 0x4286, kEBMLReadVersion = 0x42F7, kEBMLMaxIDLength = 0x42F2,
  kEBMLMaxSizeLength = 0x42F3, kDocType = 0x4282, kDocTypeVersion = 0x4287, kDocTypeReadVersion = 0x4285,
  kSegment = 0x18538067, kSeekHead = 0x114D9B74, kSeek = 0x4DBB, kSeekID = 0x53AB, kSeekPosition = 0x53AC,
  kInfo = 0x1549A966, kTimestampScale = 0x2AD7B1, kDuration = 0x4489, kMuxingApp = 0x4D80, kWritingApp = 0x5741,
  kTracks = 0x1654AE6B, kTrackEntry = 0xAE, kTrackNumber = 0xD7, kTrackUID = 0x73C5, kTrackType = 0x83,
  kFlagDefault = 0x88, kFlagLacing = 0x9C, kDefaultDuration = 0x23E383, kLanguage = 0x22B59C, kCodecID = 0x86,
  kCodecPrivate = 0x63A2, kVideo = 0xE0, kPixelWidth = 0xB0, kPixelHeight = 0xBA, kAudio = 0xE1,
  kSamplingFrequency = 0xB5, kChannels = 0x9F, kBitDepth = 0x6264, kCluster = 0x1F43B675, kTimestamp = 0xE7,
  kSimpleBlock = 0xA3, kBlockGroup = 0xA0, kBlock = 0xA1, kBlockDuration = 0x9B, kCues = 0x1C53BB6B,
  kCuePoint = 0xBB, kCueTime = 0xB3, kCueTrackPositions = 0xB7, kCueTrack = 0xF7, kCueClusterPosition = 0xF1,
};

struct Ebml {
  std::vector<uint8_t> b;
  void id(uint32_t v) {
    const int n = v > 0xFFFFFF ? 4 : v > 0xFFFF ? 3 : v > 0xFF ? 2 : 1;
    for (int i = n - 1; i >= 0; --i) b.push_back((uint8_t)(v >> (8 * i)));
  }
  void size(uint64_t n) {  // shortest vint (all-ones is reserved for "unknown")
    int len = 1;
    while (len < 8 && n >= (1ull << (7 * len)) - 1) ++len;
    const uint64_t v = n | (1ull << (7 * len));
    for (int i = len - 1; i >= 0; --i) b.push_back((uint8_t)(v >> (8 * i)));
  }
  void size8(uint64_t n) {
    b.push_back(0x01);
    for (int i = 6; i >= 0; --i) b.push_back((uint8_t)(n >> (8 * i)));
  }
  void uint(uint32_t eid, uint64_t v, int fixed = 0) {
    int n = 1;
    while (n < 8 && (v >> (8 * n))) ++n;
    if (fixed) n = fixed;
    id(eid);
    size((uint64_t)n);
    for (int i = n - 1; i >= 0; --i) b.push_back((uint8_t)(v >> (8 * i)));
  }
  void flt(uint32_t eid, double v) {
    uint64_t u;
    std::memcpy(&u, &v, 8);
    id(eid);
    size(8);
    for (int i = 7; i >= 0; --i) b.push_back((uint8_t)(u >> (8 * i)));
  }
  void str(uint32_t eid, const std::string& s) { bin(eid, (const uint8_t*)s.data(), s.size()); }
  void bin(uint32_t eid, const uint8_t* p, size_t n) {
    id(eid);
    size(n);
    b.insert(b.end(), p, p + n);
  }
  void master(uint32_t eid, const Ebml& c) {
    id(eid);
    size(c.b.size());
    b.insert(b.end(), c.b.begin(), c.b.end());
  }
};

std::string lang_of(const SideTrack& t) {
  std::string l(t.lang, strnlen(t.lang, 4));
  return l.size() == 3 ? l : "und";
}

const char* codec_id(const SideTrack& t) {
  switch (t.codec) {
    case SIDE_AAC: return "A_AAC";
    case SIDE_PCM_S16LE: return "A_PCM/INT/LIT";
    case SIDE_SUBRIP: return "S_TEXT/UTF8";
    default: return t.mkv_codec_id;
  }
}

// one block to place: track 0 = video sample `idx`, k = side track k-1 sample `idx`
struct Ev {
  int64_t ms;  // ordering time (video: decode time)
  int track;
  int64_t idx;
  int64_t pts = 0;  // video: presentation time (ms)
};

// SeekHead with fixed-width positions, so it can be rewritten in place once Cues is placed
Ebml seek_head(uint64_t info, uint64_t tracks, uint64_t cues) {
  Ebml sh;
  const uint32_t ids[3] = {kInfo, kTracks, kCues};
  const uint64_t pos[3] = {info, tracks, cues};
  for (int k = 0; k < 3; ++k) {
    Ebml s, idb;
    idb.id(ids[k]);
    s.bin(kSeekID, idb.b.data(), idb.b.size());
    s.uint(kSeekPosition, pos[k], 8);
    sh.master(kSeek, s);
  }
  return sh;
}

}  // namespace

uint64_t write_mkv(const MuxPlan& P, int width, int height, int fps_num, int fps_den, const SideTrack* tracks,
                   int ntracks, const char* path) {
  for (int k = 0; k < ntracks; ++k) check_side(tracks[k], true);
  auto video_ms = [&](int64_t i) { return (int64_t)std::llround((double)i * 1000.0 * fps_den / fps_num); };
  // ---- Info / Tracks
  double dur_ms = (double)P.samples.size() * 1000.0 * fps_den / fps_num;
  for (int k = 0; k < ntracks; ++k) {
    const SideTrack& t = tracks[k];
    if (t.nsamples)
      dur_ms = std::max(dur_ms, (double)(t.pts[t.nsamples - 1] + t.durs[t.nsamples - 1]) * 1000.0 / t.timescale);
  }
  Ebml info;
  info.uint(kTimestampScale, 1000000);
  info.flt(kDuration, dur_ms);
  info.str(kMuxingApp, "thinvids-amd");
  info.str(kWritingApp, "thinvids-amd");
  Ebml trk;
  {
    Ebml e, v;
    e.uint(kTrackNumber, 1);
    e.uint(kTrackUID, 1);
    e.uint(kTrackType, 1);
    e.uint(kFlagLacing, 0);
    e.uint(kDefaultDuration, (uint64_t)std::llround(1e9 * fps_den / fps_num));
    e.str(kLanguage, "und");
    e.str(kCodecID, P.codec == MUX_AV1 ? "V_AV1" : "V_MPEGH/ISO/HEVC");
    const auto hv = P.codec == MUX_AV1 ? P.av1c : hvcc_record(P);
    e.bin(kCodecPrivate, hv.data(), hv.size());
    v.uint(kPixelWidth, (uint64_t)width);
    v.uint(kPixelHeight, (uint64_t)height);
    e.master(kVideo, v);
    trk.master(kTrackEntry, e);
  }
  for (int k = 0; k < ntracks; ++k) {
    const SideTrack& t = tracks[k];
    Ebml e;
    e.uint(kTrackNumber, (uint64_t)k + 2);
    e.uint(kTrackUID, (uint64_t)k + 2);
    e.uint(kTrackType, t.kind == SIDE_AUDIO ? 2 : 0x11);
    e.uint(kFlagDefault, t.is_default ? 1 : 0);
    e.uint(kFlagLacing, 0);
    e.str(kLanguage, lang_of(t));
    e.str(kCodecID, codec_id(t));
    if (t.priv_size) e.bin(kCodecPrivate, t.priv, (size_t)t.priv_size);
    if (t.kind == SIDE_AUDIO) {
      Ebml a;
      a.flt(kSamplingFrequency, (double)(t.sample_rate > 0 ? t.sample_rate : t.timescale));
      a.uint(kChannels, (uint64_t)std::max(1, t.channels));
      if (t.bits > 0) a.uint(kBitDepth, (uint64_t)t.bits);
      e.master(kAudio, a);
    }
    trk.master(kTrackEntry, e);
  }
  // ---- events in presentation order (video first on ties)
  std::vector<Ev> ev;
  ev.reserve(P.samples.size());
  // video blocks stay in decoding order (sorted by decode time) but carry presentation
  // timestamps (B frames: the sample's composition offset)
  for (size_t i = 0; i < P.samples.size(); ++i)
    ev.push_back({video_ms((int64_t)i), 0, (int64_t)i, video_ms((int64_t)i + P.samples[i].cto)});
  for (int k = 0; k < ntracks; ++k)
    for (int64_t i = 0; i < tracks[k].nsamples; ++i)
      ev.push_back({(int64_t)((__int128)tracks[k].pts[i] * 1000 / tracks[k].timescale), k + 1, i, 0});
  std::stable_sort(ev.begin(), ev.end(), [](const Ev& a, const Ev& b) {
    return a.ms < b.ms || (a.ms == b.ms && a.track < b.track);
  });
  // ---- write: header, segment with placeholder size, SeekHead placeholder, Info, Tracks
  FILE* f = std::fopen(path, "wb");
  if (!f) throw std::runtime_error(std::string("mux: cannot open ") + path);
  std::vector<std::unique_ptr<SideReader>> rd;
  bool ok = true;
  uint64_t pos = 0;
  auto put = [&](const std::vector<uint8_t>& b) {
    ok = ok && std::fwrite(b.data(), 1, b.size(), f) == b.size();
    pos += b.size();
  };
  try {
    for (int k = 0; k < ntracks; ++k) rd.emplace_back(new SideReader(tracks[k]));
    Ebml hdr, eh;
    eh.uint(kEBMLVersion, 1);
    eh.uint(kEBMLReadVersion, 1);
    eh.uint(kEBMLMaxIDLength, 4);
    eh.uint(kEBMLMaxSizeLength, 8);
    eh.str(kDocType, "matroska");
    eh.uint(kDocTypeVersion, 4);
    eh.uint(kDocTypeReadVersion, 2);
    hdr.master(kEBML, eh);
    hdr.id(kSegment);
    hdr.size8(0);
    put(hdr.b);
    const uint64_t seg_size_at = pos - 8, seg0 = pos;
    Ebml sh0;
    sh0.master(kSeekHead, seek_head(0, 0, 0));
    const uint64_t sh_at = pos;
    put(sh0.b);
    const uint64_t info_at = pos - seg0;
    Ebml ib;
    ib.master(kInfo, info);
    put(ib.b);
    const uint64_t tracks_at = pos - seg0;
    Ebml tb;
    tb.master(kTracks, trk);
    put(tb.b);
    // ---- clusters
    Ebml cues;
    Ebml cl;  // current cluster's children
    int64_t cl_ms = -1;
    bool cl_key = false;
    auto close_cluster = [&] {
      if (cl_ms < 0) return;
      if (cl_key) {
        Ebml cp, tp;
        cp.uint(kCueTime, (uint64_t)cl_ms);
        tp.uint(kCueTrack, 1);
        tp.uint(kCueClusterPosition, pos - seg0);
        cp.master(kCueTrackPositions, tp);
        cues.master(kCuePoint, cp);
      }
      Ebml c;
      c.master(kCluster, cl);
      put(c.b);
      cl.b.clear();
      cl_ms = -1;
    };
    std::vector<uint8_t> payload;
    for (const auto& e : ev) {
      const bool key = e.track == 0 && P.samples[e.idx].sync;
      if (cl_ms < 0 || key || e.ms - cl_ms > 5000) {
        close_cluster();
        cl_ms = e.ms;
        cl_key = key;
        cl.uint(kTimestamp, (uint64_t)cl_ms);
      }
      payload.clear();
      payload.push_back((uint8_t)(0x80 | (e.track + 1)));  // track number vint (< 127 tracks)
      const int64_t rel = (e.track == 0 ? e.pts : e.ms) - cl_ms;
      payload.push_back((uint8_t)(rel >> 8));
      payload.push_back((uint8_t)rel);
      const SideTrack* t = e.track ? &tracks[e.track - 1] : nullptr;
      const bool sub = t && t->kind == SIDE_SUBTITLE;
      payload.push_back(sub ? 0x00 : (!t ? (key ? 0x80 : 0x00) : 0x80));
      if (!t) append_sample(P.samples[e.idx], payload);
      else rd[e.track - 1]->append(e.idx, payload);
      if (sub) {
        Ebml g;
        g.bin(kBlock, payload.data(), payload.size());
        g.uint(kBlockDuration, (uint64_t)((__int128)t->durs[e.idx] * 1000 / t->timescale));
        cl.master(kBlockGroup, g);
      } else {
        cl.bin(kSimpleBlock, payload.data(), payload.size());
      }
    }
    close_cluster();
    const uint64_t cues_at = pos - seg0;
    Ebml cb;
    cb.master(kCues, cues);
    put(cb.b);
    // ---- patch SeekHead and the Segment size
    const uint64_t end = pos;
    Ebml sh;
    sh.master(kSeekHead, seek_head(info_at, tracks_at, cues_at));
    Ebml ss;
    ss.size8(end - seg0);
    ok = ok && sh.b.size() == sh0.b.size();
    ok = ok && fseeko(f, (off_t)sh_at, SEEK_SET) == 0 && std::fwrite(sh.b.data(), 1, sh.b.size(), f) == sh.b.size();
    ok = ok && fseeko(f, (off_t)seg_size_at, SEEK_SET) == 0 &&
         std::fwrite(ss.b.data() + 0, 1, 8, f) == 8;
    pos = end;
  } catch (...) {
    std::fclose(f);
    throw;
  }
  ok = (std::fclose(f) == 0) && ok;
  if (!ok) throw std::runtime_error(std::string("mux: write failed: ") + path);
  return pos;
}

}  // namespace muxi
}  // namespace tv
