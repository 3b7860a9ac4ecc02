// sanitize_core.cpp — host sanitizer driver for the C++ codec core (SURVEY.md §5.2 "build
// the C++ engine with -fsanitize=address,undefined for the CPU golden model").
//
// Built together with csrc/core/*.cpp under -fsanitize=address,undefined by
// tools/sanitize_core.sh (tests/test_sanitize.py runs it on the CPU): a golden-encoder
// round trip (IDR + P frames with deblocking and SAO) through the oracle decoder, MP4
// mux/demux, MP4 and Matroska muxing with audio + subtitle side streams, the AV1 multi-symbol range coder and the CDEF direction search.  Any
// out-of-bounds access, use-after-free, leak or undefined behaviour aborts with a report;
// a functional mismatch exits 1.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unistd.h>
#include <vector>

#include "tv/container.h"
#include "tv/mpeg2.h"

extern "C" {
const char* tv_last_error();
void* tv_bytes_new();
void tv_bytes_free(void*);
size_t tv_bytes_size(void*);
const uint8_t* tv_bytes_data(void*);
void tv_bytes_clear(void*);
void tv_synth_frame(uint32_t seed, int t, int W, int H, uint8_t* y, uint8_t* u, uint8_t* v);
void* tv_cpu_encoder_new(int width, int height, int qp, int deblock, int range, int max_merge);
void tv_cpu_encoder_free(void*);
int tv_cpu_encoder_encode(void*, const uint8_t*, const uint8_t*, const uint8_t*, int sy, int sc, int idr, int poc,
                          void* out);
void tv_cpu_encoder_recon(void*, uint8_t*, uint8_t*, uint8_t*);
void* tv_decoder_new();
void tv_decoder_free(void*);
int tv_decoder_decode(void*, const uint8_t*, size_t);
void tv_decoder_info(void*, int*, int*, int*, int*, int*);
int tv_decoder_frame(void*, int idx, int cropped, uint8_t*, uint8_t*, uint8_t*);
int tv_mux_mp4(const uint8_t*, size_t, int w, int h, int fps_num, int fps_den, void* out);
int tv_demux_mp4(const uint8_t*, size_t, int* w, int* h, int* nframes, int* timescale, int* delta, void* out);
int tv_mux_file(const uint8_t* const* segs, const size_t* sizes, int nseg, int w, int h, int fps_num, int fps_den,
                const tv::SideTrack* tracks, int ntracks, int container, const char* path, unsigned long long* out);
int tv_av1_rc_roundtrip(const int* sym, const int* alpha, const int* ctx, int n, int nctx, int adapt, void* out,
                        int* dec);
void tv_av1_cdef_find_dirs(const uint8_t* Y, int w, int h, uint8_t* dir, int* var);
}

static int fail(const char* what) {
  std::fprintf(stderr, "FAIL: %s (%s)\n", what, tv_last_error());
  return 1;
}

static uint32_t rng_state = 12345u;
static uint32_t rnd() {
  rng_state = rng_state * 1664525u + 1013904223u;
  return rng_state >> 8;
}

int main() {
  // 1) HEVC golden encoder -> oracle decoder, odd display size (coded-size padding paths)
  for (int sao = 0; sao < 2; ++sao) {
    const int W = 136, H = 72, N = 4;
    const int CW = (W + 31) / 32 * 32, CH = (H + 31) / 32 * 32;
    void* enc = tv_cpu_encoder_new(W, H, 27, 1 | (sao << 1), 16, 5);
    if (!enc) return fail("encoder_new");
    void* frame = tv_bytes_new();
    std::vector<uint8_t> stream, y(W * H), u(W * H / 4), v(W * H / 4);
    for (int t = 0; t < N; ++t) {
      tv_synth_frame(7u, t, W, H, y.data(), u.data(), v.data());
      tv_bytes_clear(frame);
      if (tv_cpu_encoder_encode(enc, y.data(), u.data(), v.data(), W, W / 2, t == 0, t, frame)) return fail("encode");
      stream.insert(stream.end(), tv_bytes_data(frame), tv_bytes_data(frame) + tv_bytes_size(frame));
    }
    std::vector<uint8_t> ry(CW * CH), ru(CW * CH / 4), rv(CW * CH / 4);
    tv_cpu_encoder_recon(enc, ry.data(), ru.data(), rv.data());
    void* dec = tv_decoder_new();
    if (tv_decoder_decode(dec, stream.data(), stream.size())) return fail("decode");
    int w, h, cw, ch, n;
    tv_decoder_info(dec, &w, &h, &cw, &ch, &n);
    if (w != W || h != H || n != N || cw != CW || ch != CH) return fail("decoder geometry");
    std::vector<uint8_t> dy(CW * CH), du(CW * CH / 4), dv(CW * CH / 4);
    if (tv_decoder_frame(dec, N - 1, 0, dy.data(), du.data(), dv.data())) return fail("decoder frame");
    if (dy != ry || du != ru || dv != rv) return fail("decoded != encoder reconstruction");
    // 2) MP4 mux / demux round trip of the elementary stream
    void* mp4 = tv_bytes_new();
    void* es = tv_bytes_new();
    if (tv_mux_mp4(stream.data(), stream.size(), W, H, 30, 1, mp4)) return fail("mux");
    int mw, mh, mn, ts, dl;
    if (tv_demux_mp4(tv_bytes_data(mp4), tv_bytes_size(mp4), &mw, &mh, &mn, &ts, &dl, es)) return fail("demux");
    if (mw != W || mh != H || mn != N) return fail("demux geometry");
    // 2b) the same stream with an in-memory audio track and a subtitle track with a gap and
    //     an overlap, as interleaved MP4 and as Matroska, then the MP4 video back out
    {
      std::vector<uint8_t> pay(4000);
      for (auto& b : pay) b = (uint8_t)rnd();
      const int na = 20;
      std::vector<uint64_t> ao(na);
      std::vector<uint32_t> as(na), ad(na, 1024);
      std::vector<int64_t> ap(na);
      for (int i = 0; i < na; ++i) ao[i] = (uint64_t)i * 150, as[i] = 100 + (uint32_t)(rnd() % 50), ap[i] = 1024 * i;
      const uint8_t asc[2] = {0x11, 0x90};
      const char text[] = "firstsecond";
      const uint64_t so[2] = {0, 5};
      const uint32_t ss[2] = {5, 6}, sd[2] = {900, 300};
      const int64_t sp[2] = {40, 500};
      tv::SideTrack tr[2] = {};
      tr[0] = {tv::SIDE_AUDIO, tv::SIDE_AAC, 48000, 2, 48000, 16, 1, 0, {'e', 'n', 'g', 0}, nullptr, asc, 2,
               nullptr, pay.data(), na, ao.data(), as.data(), ap.data(), ad.data()};
      tr[1] = {tv::SIDE_SUBTITLE, tv::SIDE_SUBRIP, 1000, 0, 0, 0, 0, 0, {'e', 'n', 'g', 0}, nullptr, nullptr, 0,
               nullptr, (const uint8_t*)text, 2, so, ss, sp, sd};
      const uint8_t* segs[1] = {stream.data()};
      const size_t sizes[1] = {stream.size()};
      unsigned long long bytes = 0;
      char mp4p[] = "/tmp/tv_sanitize_XXXXXX";
      const int fd = mkstemp(mp4p);
      if (fd < 0) return fail("mkstemp");
      close(fd);
      if (tv_mux_file(segs, sizes, 1, W, H, 25, 1, tr, 2, tv::CONTAINER_MKV, mp4p, &bytes) || bytes < stream.size())
        return fail("mkv mux");
      if (tv_mux_file(segs, sizes, 1, W, H, 25, 1, tr, 2, tv::CONTAINER_MP4, mp4p, &bytes)) return fail("mp4 mux");
      std::vector<uint8_t> file(bytes);
      FILE* f = std::fopen(mp4p, "rb");
      const bool rd = f && std::fread(file.data(), 1, file.size(), f) == file.size();
      if (f) std::fclose(f);
      std::remove(mp4p);
      if (!rd) return fail("mp4 read back");
      void* es2 = tv_bytes_new();
      if (tv_demux_mp4(file.data(), file.size(), &mw, &mh, &mn, &ts, &dl, es2) || mn != N) return fail("side demux");
      tv_bytes_free(es2);
    }
    tv_bytes_free(mp4);
    tv_bytes_free(es);
    tv_decoder_free(dec);
    tv_bytes_free(frame);
    tv_cpu_encoder_free(enc);
  }
  // 3) AV1 range coder: random symbols over 6 contexts of alphabets 2..16, adaptive CDFs
  {
    const int n = 4000, nctx = 6;
    int alpha[nctx];
    for (int c = 0; c < nctx; ++c) alpha[c] = 2 + (int)(rnd() % 15);
    std::vector<int> sym(n), ctx(n), dec(n);
    for (int i = 0; i < n; ++i) {
      ctx[i] = (int)(rnd() % nctx);
      const int a = alpha[ctx[i]];
      sym[i] = (rnd() % 4) ? (int)(rnd() % 2) % a : (int)(rnd() % a);  // skewed
    }
    std::vector<int> alphas(n);
    for (int i = 0; i < n; ++i) alphas[i] = alpha[ctx[i]];
    void* out = tv_bytes_new();
    if (tv_av1_rc_roundtrip(sym.data(), alphas.data(), ctx.data(), n, nctx, 1, out, dec.data()))
      return fail("range coder");
    if (dec != sym) return fail("range coder round trip");
    tv_bytes_free(out);
  }
  // 4) CDEF direction search on a textured plane with a non-multiple-of-64 size
  {
    const int w = 120, h = 72;
    std::vector<uint8_t> Y(w * h);
    for (int i = 0; i < w * h; ++i) Y[i] = (uint8_t)((i % w) * 3 + (i / w) * 5 + (rnd() & 15));
    std::vector<uint8_t> dir((w / 8) * (h / 8));
    std::vector<int> var((w / 8) * (h / 8));
    tv_av1_cdef_find_dirs(Y.data(), w, h, dir.data(), var.data());
    for (uint8_t d : dir)
      if (d > 7) return fail("cdef direction out of range");
  }
  // 5) MPEG-2: writer -> decoder round trip (frame and field pictures, open GOP), then
  //    randomly damaged copies of the streams (bit flips, truncation) must decode or fail
  //    cleanly -- a DVD source is untrusted input
  {
    const int W = 96, H = 64, N = 8;
    std::vector<std::vector<uint8_t>> frames(N, std::vector<uint8_t>(W * H * 3 / 2));
    for (int t = 0; t < N; ++t) {
      uint8_t* f = frames[t].data();
      tv_synth_frame(11, t, W, H, f, f + W * H, f + W * H * 5 / 4);
    }
    std::vector<const uint8_t*> ptrs;
    for (auto& f : frames) ptrs.push_back(f.data());
    for (int cfgi = 0; cfgi < 3; ++cfgi) {
      tv::mpeg2::EncConfig c;
      c.width = W;
      c.height = H;
      c.gop = 5;
      c.interlaced = cfgi > 0;
      c.field_pictures = cfgi == 2;
      c.closed_gop = cfgi != 1;
      c.vary_quant = true;
      std::vector<tv::mpeg2::Image> rec;
      const std::vector<uint8_t> es = tv::mpeg2::encode(c, ptrs, nullptr, nullptr, &rec);
      int got = 0;
      tv::mpeg2::Decoder dec;
      dec.decode(es.data(), es.size(), 0, 0, 0, [&](int k, const tv::mpeg2::Image& im) {
        if (std::memcmp(im.y.data(), rec[k].y.data(), (size_t)W * H) != 0) got = -1000;
        ++got;
        return true;
      });
      if (got != N) return fail("mpeg2 round trip");
      for (int it = 0; it < 150; ++it) {
        std::vector<uint8_t> d = es;
        const int nflip = 1 + (int)(rnd() % 16);
        for (int k = 0; k < nflip; ++k) d[rnd() % d.size()] ^= (uint8_t)(1 + rnd() % 255);
        if (rnd() % 4 == 0) d.resize(rnd() % d.size());
        try {
          tv::mpeg2::index_stream(d.data(), d.size());
          tv::mpeg2::Decoder dd;
          dd.decode(d.data(), d.size(), 0, 0, 0, [](int, const tv::mpeg2::Image&) { return true; });
        } catch (const std::exception&) {
        }
      }
    }
  }
  std::puts("sanitize_core: ok");
  return 0;
}
