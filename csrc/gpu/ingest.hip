// ingest.hip — file -> HBM ingest of a raw-video byte range with the disk/page-cache reads
// and the host->device DMA overlapped (the node job's y4m path, ops/stage.read_y4m_device).
//
// Reference: a worker fetches its source part over HTTP from the master and ffmpeg decodes
// it (worker/tasks.py:1497-1525, :1146-1162).  Here a rank reads its own range of a raw
// y4m / yuv file and the frames must reach HBM at the encoder's rate
// (1080p at ~7.5k frames/s is ~23 GB/s per GPU).  A read-then-copy does the two at the sum
// of their times; this pipeline does them at the max:
//
//   T reader threads; chunk k (CHUNK bytes of the range) belongs to thread k % T, which
//   waits until ring slot k % S is free (the event of the DMA that last used it), pread()s
//   the chunk into that pinned slot, then enqueues its hipMemcpyAsync to the destination
//   and records the slot's event on the caller's stream.  With S = 2T slots every thread
//   always has a free slot while its previous DMA is in flight, so the SDMA engine streams
//   chunks back to back while the threads keep reading.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {
thread_local std::string g_ingest_err;

int64_t pread_all(int fd, uint8_t* dst, int64_t n, int64_t off) {
  int64_t done = 0;
  while (done < n) {
    const ssize_t r = ::pread(fd, dst + done, (size_t)(n - done), (off_t)(off + done));
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

const char* tv_ingest_last_error() { return g_ingest_err.c_str(); }

// Reads [offset, offset + nbytes) of `path` into device memory `dst` through the pinned
// ring `ring` (ring_bytes, split into 2 * threads slots), DMA on `stream`.  Returns 0 when
// every byte was read and its copy enqueued and completed, -1 otherwise
// (tv_ingest_last_error).  times[0] = summed read seconds over threads, times[1] = wall.
int tv_ingest_h2d(const char* path, long long offset, long long nbytes, void* dst, void* ring, long long ring_bytes,
                  int threads, void* stream, double* times) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  const int fd = ::open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) {
    g_ingest_err = std::string("open ") + path + ": " + std::strerror(errno);
    return -1;
  }
  ::posix_fadvise(fd, (off_t)offset, (off_t)nbytes, POSIX_FADV_SEQUENTIAL);
  const int T = std::max(1, threads);
  const int S = 2 * T;
  int64_t chunk = (ring_bytes / S) & ~int64_t(4095);
  if (chunk < (1 << 20)) {
    ::close(fd);
    g_ingest_err = "ingest ring too small";
    return -1;
  }
  const int64_t nchunks = (nbytes + chunk - 1) / chunk;
  hipStream_t st = static_cast<hipStream_t>(stream);
  std::vector<hipEvent_t> ev(S);
  std::vector<char> used(S, 0);
  for (auto& e : ev) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
  std::atomic<bool> failed{false};
  std::mutex err_mu;
  std::string err;  // set by the first failing thread; g_ingest_err is the caller's thread-local
  std::vector<double> read_s(T, 0.0);
  auto fail = [&](const std::string& m) {
    std::lock_guard<std::mutex> g(err_mu);
    if (!failed.exchange(true)) err = m;
  };
  auto work = [&](int t) {
    for (int64_t k = t; k < nchunks && !failed.load(); k += T) {
      const int s = (int)(k % S);  // slots k % S with k = t (mod T) are touched by thread t only
      if (used[s] && hipEventSynchronize(ev[s]) != hipSuccess) return fail("hipEventSynchronize failed");
      const int64_t off = k * chunk, n = std::min<int64_t>(chunk, nbytes - off);
      uint8_t* slot = static_cast<uint8_t*>(ring) + (int64_t)s * chunk;
      const auto r0 = clk::now();
      const int64_t got = pread_all(fd, slot, n, offset + off);
      read_s[t] += std::chrono::duration<double>(clk::now() - r0).count();
      if (got != n)
        return fail(std::string("pread ") + path + (got < 0 ? std::string(": ") + std::strerror((int)-got)
                                                             : std::string(": short read (file ends)")));
      if (hipMemcpyAsync(static_cast<uint8_t*>(dst) + off, slot, (size_t)n, hipMemcpyHostToDevice, st) != hipSuccess ||
          hipEventRecord(ev[s], st) != hipSuccess)
        return fail("hipMemcpyAsync / hipEventRecord failed");
      used[s] = 1;
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < T; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
  const hipError_t se = hipStreamSynchronize(st);  // the ring is reused by the next call
  for (auto& e : ev) (void)hipEventDestroy(e);
  ::close(fd);
  if (se != hipSuccess && !failed.load()) fail(std::string("hipStreamSynchronize: ") + hipGetErrorString(se));
  if (failed.load()) g_ingest_err = err;
  if (times) {
    double rs = 0;
    for (double x : read_s) rs += x;
    times[0] = rs;
    times[1] = std::chrono::duration<double>(clk::now() - t0).count();
  }
  return failed.load() ? -1 : 0;
}

}  // extern "C"
