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
//   Copies go to D = TV_INGEST_STREAMS (default 4) copy streams of their own, thread t on
//   stream t % D, ordered after the caller's stream: one DMA queue moved ~23-25 GB/s, four
//   ~28-31 GB/s (round 5, 1080p y4m job 4942 -> 5192-5282 frames/s).  D = 1 copies on the
//   caller's stream.
//   Round 6: hipMemcpyAsync moves a pinned-host -> device chunk with a blit kernel on this
//   runtime (`__amd_rocclr_copyBuffer`), CU time taken from the encoder running beside the
//   next claim's ingest; the chunks now go to the SDMA engines (hsa_amd_memory_async_copy,
//   one completion signal per ring slot).  TV_INGEST_DMA=hip keeps the HIP copies.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace {
thread_local std::string g_ingest_err;

// per-device copy streams for TV_INGEST_STREAMS > 1 (created once, kept for the process)
std::vector<hipStream_t>& copy_streams(int want) {
  static std::mutex mu;
  static std::vector<std::vector<hipStream_t>> per_dev;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> g(mu);
  if ((int)per_dev.size() <= dev) per_dev.resize(dev + 1);
  auto& v = per_dev[dev];
  while ((int)v.size() < want) {
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) break;
    v.push_back(s);
  }
  return v;
}

int ingest_streams() {
  static const int n = [] {
    const char* e = std::getenv("TV_INGEST_STREAMS");
    const int v = e ? std::atoi(e) : 4;
    return std::max(1, std::min(8, v));
  }();
  return n;
}

// the CPU agent (source of host -> device SDMA copies), found once; handle 0: none
hsa_agent_t cpu_agent() {
  static const hsa_agent_t a = [] {
    hsa_agent_t r{0};
    hsa_iterate_agents(
        [](hsa_agent_t x, void* data) {
          hsa_device_type_t t;
          if (hsa_agent_get_info(x, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
            *static_cast<hsa_agent_t*>(data) = x;
            return HSA_STATUS_INFO_BREAK;
          }
          return HSA_STATUS_SUCCESS;
        },
        &r);
    return r;
  }();
  return a;
}

bool use_sdma() {
  static const bool on = [] {
    const char* e = std::getenv("TV_INGEST_DMA");
    return !(e && std::string(e) == "hip");
  }();
  return on;
}

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
  std::vector<hipStream_t> cs(1, st);
  if (ingest_streams() > 1) {  // copy streams start after the caller's stream (dst allocation)
    const auto& v = copy_streams(ingest_streams());
    if (!v.empty()) {
      cs.assign(v.begin(), v.end());
      hipEvent_t start;
      (void)hipEventCreateWithFlags(&start, hipEventDisableTiming);
      (void)hipEventRecord(start, st);
      for (hipStream_t c : cs) (void)hipStreamWaitEvent(c, start, 0);
      (void)hipEventDestroy(start);
    }
  }
  std::vector<hipEvent_t> ev(S);
  std::vector<char> used(S, 0);
  for (auto& e : ev) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
  // SDMA mode: the destination was allocated on the caller's stream, so that stream drains
  // first (the prefetch stream is idle; the first claim's load runs before its encode)
  hsa_agent_t cpu = cpu_agent(), gpu{0};
  bool sdma = use_sdma() && cpu.handle != 0;
  if (sdma) {
    hsa_amd_pointer_info_t info{};
    info.size = sizeof(info);
    sdma = hsa_amd_pointer_info(dst, &info, nullptr, nullptr, nullptr) == HSA_STATUS_SUCCESS &&
           info.type == HSA_EXT_POINTER_TYPE_HSA;
    gpu = info.agentOwner;
  }
  std::vector<hsa_signal_t> sig(sdma ? S : 0);
  for (auto& g : sig)
    if (hsa_signal_create(0, 0, nullptr, &g) != HSA_STATUS_SUCCESS) sdma = false;
  if (sdma && hipStreamSynchronize(st) != hipSuccess) sdma = false;
  auto wait_sig = [&](hsa_signal_t g) {
    while (hsa_signal_wait_scacquire(g, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED) >= 1) {
    }
  };
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
      if (used[s]) {
        if (sdma) wait_sig(sig[s]);
        else if (hipEventSynchronize(ev[s]) != hipSuccess) return fail("hipEventSynchronize failed");
      }
      const int64_t off = k * chunk, n = std::min<int64_t>(chunk, nbytes - off);
      uint8_t* slot = static_cast<uint8_t*>(ring) + (int64_t)s * chunk;
      const auto r0 = clk::now();
      const int64_t got = pread_all(fd, slot, n, offset + off);
      read_s[t] += std::chrono::duration<double>(clk::now() - r0).count();
      if (got != n)
        return fail(std::string("pread ") + path + (got < 0 ? std::string(": ") + std::strerror((int)-got)
                                                             : std::string(": short read (file ends)")));
      if (sdma) {
        hsa_signal_store_relaxed(sig[s], 1);
        if (hsa_amd_memory_async_copy(static_cast<uint8_t*>(dst) + off, gpu, slot, cpu, (size_t)n, 0, nullptr, sig[s]) !=
            HSA_STATUS_SUCCESS) {
          hsa_signal_store_relaxed(sig[s], 0);
          return fail("hsa_amd_memory_async_copy failed");
        }
      } else {
        hipStream_t q = cs[t % cs.size()];
        if (hipMemcpyAsync(static_cast<uint8_t*>(dst) + off, slot, (size_t)n, hipMemcpyHostToDevice, q) != hipSuccess ||
            hipEventRecord(ev[s], q) != hipSuccess)
          return fail("hipMemcpyAsync / hipEventRecord failed");
      }
      used[s] = 1;
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < T; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
  hipError_t se = hipSuccess;  // the ring is reused by the next call
  for (hipStream_t c : cs) {
    const hipError_t e = hipStreamSynchronize(c);
    if (se == hipSuccess) se = e;
  }
  for (auto& g : sig) {
    wait_sig(g);
    hsa_signal_destroy(g);
  }
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
