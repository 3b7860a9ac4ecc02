// io.cpp — source ingest for the node job: parallel positional reads of a raw-video byte
// range straight into a caller-owned (pinned) buffer, and read-ahead hints.
//
// The reference moves source bytes as ffmpeg stream-copy chunks over HTTP
// (worker/tasks.py:1146-1162 segment, :1497-1525 GET part).  Here a rank reads its own
// segment of a raw y4m / yuv file at page-cache / NVMe speed: the range is
// cut into `threads` contiguous stripes, each read with pread() by its own thread directly
// into its slice of the destination (no intermediate bytes objects, no GIL), then the
// caller issues ONE host->device copy of the pinned buffer.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {
thread_local std::string g_io_err;

// Reads [off, off + n) of fd into dst; returns bytes read (short only at EOF) or -errno.
int64_t read_range(int fd, int64_t off, int64_t n, uint8_t* dst) {
  int64_t done = 0;
  while (done < n) {
    const size_t want = (size_t)std::min<int64_t>(n - done, int64_t(1) << 30);
    const ssize_t r = ::pread(fd, dst + done, want, (off_t)(off + done));
    if (r < 0) {
      if (errno == EINTR) continue;
      return -errno;
    }
    if (r == 0) break;
    done += r;
  }
  return done;
}
}  // namespace

extern "C" {

const char* tv_io_last_error() { return g_io_err.c_str(); }

// Parallel read of `nbytes` at `offset` into dst with up to `threads` threads.  Returns the
// number of bytes read (== nbytes unless the file ends first) or -1 (tv_io_last_error).
long long tv_pread_parallel(const char* path, long long offset, long long nbytes, void* dst, int threads) {
  const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) {
    g_io_err = std::string("open ") + path + ": " + std::strerror(errno);
    return -1;
  }
  ::posix_fadvise(fd, (off_t)offset, (off_t)nbytes, POSIX_FADV_SEQUENTIAL);
  // stripes of >= 8 MiB, so small reads stay single-threaded
  const int64_t min_stripe = int64_t(8) << 20;
  int nt = (int)std::max<int64_t>(1, std::min<int64_t>(std::max(1, threads), (nbytes + min_stripe - 1) / min_stripe));
  const int64_t stripe = (nbytes + nt - 1) / nt;
  std::vector<int64_t> got(nt, 0);
  auto work = [&](int t) {
    const int64_t o = (int64_t)t * stripe;
    const int64_t n = std::max<int64_t>(0, std::min<int64_t>(stripe, nbytes - o));
    got[t] = n ? read_range(fd, offset + o, n, static_cast<uint8_t*>(dst) + o) : 0;
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
  ::close(fd);
  int64_t total = 0;
  for (int t = 0; t < nt; ++t) {
    if (got[t] < 0) {
      g_io_err = std::string("pread ") + path + ": " + std::strerror((int)-got[t]);
      return -1;
    }
    const int64_t want = std::max<int64_t>(0, std::min<int64_t>(stripe, nbytes - (int64_t)t * stripe));
    total += got[t];
    if (got[t] < want) break;  // EOF inside this stripe: later stripes are past the end
  }
  return total;
}

// Read-ahead hint for a range a rank will read soon (the next claim's segment).
int tv_readahead(const char* path, long long offset, long long nbytes) {
  const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return -1;
  const int rc = ::posix_fadvise(fd, (off_t)offset, (off_t)nbytes, POSIX_FADV_WILLNEED);
  ::close(fd);
  return rc;
}

}  // extern "C"
