// container.h — output containers carrying the encoded HEVC video plus the source's
// side streams (audio, subtitles).
//
// The reference gets these from ffmpeg: the encode step transcodes audio (`-c:a aac`,
// reference worker/tasks.py:68) and the stitch step remuxes English subtitles into a
// Matroska file when the source has copy-safe ones, MP4 otherwise (:2126-2223).  Here the
// stitcher writes the final file in one pass: video samples straight from the gathered
// Annex-B segment buffers, side-stream samples read from the source file by offset (or
// from memory for converted text), interleaved by time.  Audio is carried as-is (no
// re-encode: there is no AAC encoder in this image, and a copy is lossless).
#pragma once

#include <cstddef>
#include <cstdint>

namespace tv {

enum SideKind : int32_t { SIDE_AUDIO = 1, SIDE_SUBTITLE = 2 };
// SIDE_OPAQUE = a Matroska track copied verbatim (codec id + private data + blocks), only
// into Matroska; SIDE_MP4_ENTRY = an MP4 track copied verbatim (`priv` holds its whole
// sample-entry box), only into MP4.
enum SideCodec : int32_t { SIDE_AAC = 1, SIDE_PCM_S16LE = 2, SIDE_SUBRIP = 3, SIDE_OPAQUE = 4, SIDE_MP4_ENTRY = 5 };
enum ContainerKind : int32_t { CONTAINER_MP4 = 0, CONTAINER_MKV = 1 };

// One side stream, laid out for ctypes.  Sample i is `sizes[i]` bytes at `offsets[i]` of
// the file `path` (or of `data` when path is null), presented at `pts[i]` for `durs[i]`
// ticks of `timescale`.  SUBRIP samples are bare UTF-8 cue text; PCM samples are blocks of
// interleaved little-endian frames.
struct SideTrack {
  int32_t kind, codec, timescale, channels, sample_rate, bits, is_default, reserved;
  char lang[4];  // ISO 639-2 code, NUL-padded ("" = und)
  const char* mkv_codec_id;
  const uint8_t* priv;  // AAC AudioSpecificConfig / Matroska CodecPrivate
  uint64_t priv_size;
  const char* path;
  const uint8_t* data;
  int64_t nsamples;
  const uint64_t* offsets;
  const uint32_t* sizes;
  const int64_t* pts;
  const uint32_t* durs;
};

// Write the concatenated Annex-B segments (video track 1) plus `ntracks` side streams as a
// faststart MP4 or a Matroska file at `path`; returns the file size.
uint64_t mux_file(const uint8_t* const* segs, const size_t* sizes, int nseg, int width, int height, int fps_num,
                  int fps_den, const SideTrack* tracks, int ntracks, int container, const char* path);

}  // namespace tv
