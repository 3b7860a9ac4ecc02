// engine.hip — native GPU encode engine for one MI355X (one process per GPU).
//
// Encodes a BATCH of B independent GOP-aligned segments in lock-step: frame f of every
// segment is processed by the same kernel launches (B x CTUs workgroups per launch).
// Per frame: synth/upload -> analysis -> reconstruction -> deblock -> SSE on one HIP
// stream; the decision/level planes are copied into a ring of pinned host slots and a
// CPU thread pool entropy-codes (CABAC) every (segment, frame) slice while the GPU moves
// on — the serial entropy stage overlaps the parallel GPU stages.
//
// Replaces the per-part `encode` task's ffmpeg invocation (reference
// worker/tasks.py:1532-1651); the control plane (worker/encode.py) drives this engine.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "k_encode.h"
#include "tv/me_model.h"
#include "tv/cpu_encoder.h"
#include "tv/bitstream.h"
#include "tv/hevc_codec.h"

#define HIP_OK(x)                                                                        \
  do {                                                                                   \
    hipError_t e_ = (x);                                                                 \
    if (e_ != hipSuccess)                                                                \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(e_) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__));               \
  } while (0)

namespace tv {
namespace gpu {

// Device -> host copies of the fetch threads on the SDMA engines (hsa_amd_memory_async_copy)
// instead of hipMemcpyAsync, which on this runtime moves a device -> pinned-host copy with a
// blit kernel (`__amd_rocclr_copyBuffer`: 6.7 % of the 1080p bench's kernel time, CUs taken
// from the analysis kernels).  The fetch thread has already waited for the slot's event, so
// the copies need no stream ordering; it blocks on one completion signal per batch.
// TV_D2H=hip keeps the HIP path (also the fallback when no CPU agent is found).
class SdmaD2H {
 public:
  static SdmaD2H& get() {
    static SdmaD2H s;
    return s;
  }
  bool on() const { return on_; }
  struct Batch {
    std::vector<std::pair<void*, std::pair<const void*, size_t>>> items;
    void add(void* dst, const void* src, size_t n) {
      if (n) items.push_back({dst, {src, n}});
    }
  };
  // every copy of the batch, then wait for all of them
  void run(const Batch& b) {
    if (b.items.empty()) return;
    hsa_signal_t sig;
    if (hsa_signal_create((hsa_signal_value_t)b.items.size(), 0, nullptr, &sig) != HSA_STATUS_SUCCESS)
      throw std::runtime_error("hsa_signal_create failed");
    for (const auto& it : b.items) {
      hsa_amd_pointer_info_t info{};
      info.size = sizeof(info);
      if (hsa_amd_pointer_info(it.second.first, &info, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS ||
          info.type != HSA_EXT_POINTER_TYPE_HSA) {
        hsa_signal_destroy(sig);
        throw std::runtime_error("SDMA D2H: source is not HSA device memory");
      }
      if (hsa_amd_memory_async_copy(it.first, cpu_, it.second.first, info.agentOwner, it.second.second, 0, nullptr,
                                    sig) != HSA_STATUS_SUCCESS) {
        hsa_signal_destroy(sig);
        throw std::runtime_error("hsa_amd_memory_async_copy failed");
      }
    }
    while (hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED) >= 1) {
    }
    hsa_signal_destroy(sig);
  }

 private:
  SdmaD2H() {
    const char* e = getenv("TV_D2H");
    if (e && std::string(e) == "hip") return;
    hsa_iterate_agents(
        [](hsa_agent_t a, void* data) {
          hsa_device_type_t t;
          if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
            *static_cast<hsa_agent_t*>(data) = a;
            return HSA_STATUS_INFO_BREAK;
          }
          return HSA_STATUS_SUCCESS;
        },
        &cpu_);
    on_ = cpu_.handle != 0;
  }
  hsa_agent_t cpu_{0};
  bool on_ = false;
};


// ROCTx ranges (TV_ROCTX=1): host-side frame / D2H / entropy stages appear next to the
// kernels in `rocprofv3 --marker-trace --kernel-trace` timelines.
inline bool roctx_on() {
  static const bool on = [] {
    const char* e = getenv("TV_ROCTX");
    return e && *e == '1';
  }();
  return on;
}
struct Range {
  explicit Range(const char* name) : on(roctx_on()) {
    if (on) roctxRangePushA(name);
  }
  ~Range() {
    if (on) roctxRangePop();
  }
  bool on;
};

class ThreadPool {
 public:
  ThreadPool(int n, int device) {
    for (int i = 0; i < n; ++i)
      workers_.emplace_back([this, device] {
        (void)hipSetDevice(device);
        for (;;) {
          std::function<void()> job;
          {
            std::unique_lock<std::mutex> lk(mu_);
            cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
            if (stop_ && q_.empty()) return;
            job = std::move(q_.front());
            q_.pop_front();
          }
          job();
        }
      });
  }
  ~ThreadPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }
  void submit(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      q_.push_back(std::move(f));
    }
    cv_.notify_one();
  }
  int size() const { return (int)workers_.size(); }

 private:
  std::vector<std::thread> workers_;
  std::deque<std::function<void()>> q_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false;
};

struct EngineCfg {
  int width, height, qp, batch, gop, range, deblock, threads, device, max_merge;
  uint32_t seed;
  int groups;
  int crf;  // > 0: in-engine CRF (per-frame QP from the lookahead, tv/rc_model.h)
  int mgop = 1;  // hierarchical-B mini-GOP (tv/gop.h); 1 = I P P P
};

// One group of segments on its own HIP stream (buffers, pinned slot ring, events).
class Core {
  size_t dev_bytes_ = 0, host_bytes_ = 0;
  template <class T> void dev_alloc(T** p, size_t n) {
    HIP_OK(hipMalloc(p, n));
    dev_bytes_ += n;
  }
  template <class T> void host_alloc(T** p, size_t n) {
    HIP_OK(hipHostMalloc(p, n, hipHostMallocDefault));
    host_bytes_ += n;
  }

 public:
  Core(const EngineCfg& c, ThreadPool* pool) : cfg_(c), g_(make_geo(c.width, c.height)), pool_(pool) {
    if (c.batch < 1 || c.batch > kMaxBatch) throw std::runtime_error("batch must be 1..64");
    if (c.range < 16 || c.range > 128 || (c.range & 15))
      throw std::runtime_error("search range must be a multiple of 16 in 16..128");
    if ((c.width & 1) || (c.height & 1)) throw std::runtime_error("odd frame size");
    if (c.width < 64 || c.height < 64) throw std::runtime_error("frame must be at least 64x64");
    HIP_OK(hipSetDevice(c.device));
    fetch_ = std::make_unique<ThreadPool>(1, c.device);
    HIP_OK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    {  // I-frame wavefront stream: highest priority, so its 100+ short dependent launches are
       // dispatched ahead of the other stream group's queued P-frame workgroups
      int lo = 0, hi = 0;
      HIP_OK(hipDeviceGetStreamPriorityRange(&lo, &hi));
      HIP_OK(hipStreamCreateWithPriority(&istream_, hipStreamNonBlocking, hi));
      HIP_OK(hipEventCreateWithFlags(&iev_[0], hipEventDisableTiming));
      HIP_OK(hipEventCreateWithFlags(&iev_[1], hipEventDisableTiming));
    }
    const long B = c.batch;
    nctu_ = g_.wc * g_.hc;
    // bit 2: WPP substreams, bit 3: no RQT, bit 4: no intra-in-P, bit 5: CABAC on the host
    // (WPP streams are entropy-coded on the GPU unless bit 5 asks for the host writer)
    gpu_ent_ = gpu_entropy(c);
    if (gpu_ent_) HIP_OK(hipEventCreateWithFlags(&eev_, hipEventDisableTiming));  // estream_: init_entropy_stream()
    auto alloc_set = [&](FrameSet& f) {
      dev_alloc(&f.y, B * g_.ysz);
      dev_alloc(&f.u, B * g_.csz);
      dev_alloc(&f.v, B * g_.csz);
    };
    alloc_set(src_);
    // Decoded picture buffer (tv/gop.h): every picture is reconstructed into a free DPB entry
    // that keeps its final (deblocked + SAO) samples, the 16 quarter-pel phase planes of its
    // luma (only when a later picture references it) and its quarter-res source luma (the
    // coarse search's reference); an entry is free again once no later picture needs it.
    // I P P P needs 2 entries, hierarchical-B mini-GOPs of M frames log2(M) + 2.  With SAO
    // one scratch set holds the deblocked picture the filter reads.
    if (c.mgop < 1 || c.mgop > 32 || (c.mgop & (c.mgop - 1))) throw std::runtime_error("bframes must be a power of 2 <= 32");
    if (c.mgop > 1 && c.crf > 0) throw std::runtime_error("in-engine CRF is not supported with B frames");
    ndpb_ = c.mgop > 1 ? plan_gop(2 * c.mgop + 1, c.mgop).dpb_size : 2;
    if (ndpb_ > kMaxDpb) throw std::runtime_error("DPB too large");
    qsz_ = (long)(g_.W / 4) * (g_.H / 4);
    for (int k = 0; k < ndpb_; ++k) {
      alloc_set(dpb_[k].rec);
      dev_alloc(&dpb_[k].phase, B * 16 * g_.psz);
      dev_alloc(&dpb_[k].q, B * qsz_);
    }
    if (c.deblock & 2) alloc_set(deb_);
    dev_alloc(&coef_y_, B * g_.ysz * sizeof(int16_t));
    dev_alloc(&coef_u_, B * g_.csz * sizeof(int16_t));
    dev_alloc(&coef_v_, B * g_.csz * sizeof(int16_t));
    dev_alloc(&d_sse_, B * 3 * sizeof(unsigned long long));
    dev_alloc(&count_scratch_, B * nctu_ * sizeof(int));
    // hierarchical motion search: coarse field (+ cost) per list; B pictures: per-list fine
    // search results for the bi decision
    dev_alloc(&cmv_, 2 * B * nctu_ * 2 * sizeof(int16_t));
    dev_alloc(&ccost_, 2 * B * nctu_ * sizeof(int));
    if (c.mgop > 1) dev_alloc(&meout_, 2 * B * nctu_ * sizeof(CtbMeOut));
    if (!(c.deblock & 16)) {  // intra-in-P scores and lists (tv/me_model.h pintra_*)
      uint8_t* m = nullptr;
      dev_alloc(&m, pintra_bytes(B, nctu_));
      const long n = B * nctu_;
      pi_.qcost = reinterpret_cast<int*>(m);
      pi_.gate = reinterpret_cast<int*>(m + align(n * 16));
      pi_.pass = reinterpret_cast<int*>(m + 2 * align(n * 16));
      pi_.clist = reinterpret_cast<int*>(m + 3 * align(n * 16));
      pi_.count = reinterpret_cast<int*>(m + 4 * align(n * 16));
      pi_.cand = m + 4 * align(n * 16) + 256;
    }
    cap_ = g_.ysz + 2 * g_.csz;
    // per-slot device + pinned host buffers: decisions | masks | offsets | totals | packed |
    // entropy head | entropy payload (device only: it lands in the host slot's packed region)
    slot_bytes(B, g_, gpu_ent_, slot_bytes_, slot_host_bytes_);
    if (gpu_ent_) {  // per-lane entropy scratch (each lane's stream codes one picture at a time)
      tok_cap_ = tok_capacity(B, g_);
      EntropyTables* t = nullptr;
      dev_alloc(&t, sizeof(EntropyTables));
      std::unique_ptr<EntropyTables> ht(new EntropyTables());
      entropy_tables(*ht);
      HIP_OK(hipMemcpy(t, ht.get(), sizeof(EntropyTables), hipMemcpyHostToDevice));
      for (int l = 0; l < ent_lanes(); ++l) {  // one allocation carved like ent_core_bytes()
        EntScratch& e = ent_[l];
        uint8_t* q = nullptr;
        dev_alloc(&q, ent_core_bytes(B, g_));
        e.base = q;
        e.regions = reinterpret_cast<uint32_t*>(q);
        q += align(B * nctu_ * kEntRegion * 4);
        e.tokens = reinterpret_cast<uint32_t*>(q);
        q += align((tok_cap_ + kTokPad) * 4);
        e.stage = q;
        q += align(3 * tok_cap_ + 20 * B * g_.hc + 16);
        e.ctb_cnt = reinterpret_cast<int*>(q);
        q += align(B * nctu_ * 4);
        e.ctb_off = reinterpret_cast<int*>(q);
        q += align(B * nctu_ * 4);
        e.seg_tok = reinterpret_cast<int*>(q);
        q += align(B * 4);
        e.wflag = reinterpret_cast<int*>(q);
        q += align(B * g_.hc * 4);
        e.wctx = q;
        dev_alloc(&e.skip, B * g_.usz);
        dev_alloc(&e.midx, B * g_.usz);
        e.tab = t;
      }
      const char* dbg = getenv("TV_ENT_DEBUG");
      if (dbg && *dbg == '1') {
        dev_alloc(&ent_dbg_, 8 * sizeof(unsigned long long));
        HIP_OK(hipMemset(ent_dbg_, 0, 8 * sizeof(unsigned long long)));
      }
    }
    host_alloc(&qhost_, (size_t)c.gop * B);
    host_alloc(&quni_, (size_t)B);
    std::memset(quni_, c.qp, (size_t)B);
    nslots_ = slot_count();
    slots_.reset(new Slot[nslots_]);
    for (int k = 0; k < nslots_; ++k) {
      Slot& s = slots_[k];
      dev_alloc(&s.dev, slot_bytes_);
      host_alloc(&s.host, slot_host_bytes_);
      // waited on by the fetch thread: see sync_mode()
      HIP_OK(hipEventCreateWithFlags(&s.ev, hipEventDisableTiming | (sync_mode() == 2 ? hipEventBlockingSync : 0)));

      s.pending = 0;
    }
    HIP_OK(hipEventCreate(&t0_));
    HIP_OK(hipEventCreate(&t1_));
    // decision constants of every QP (rate control picks the QP per segment and frame on the
    // device): identical integer rounding to the CPU reference encoder
    {
      RcTables t{};
      for (int q = 0; q < 52; ++q) {
        const double lam = lambda_sad(q);
        Penalties& p = t.pen[q];
        p.mode_dcpl = (int)(lam * 2);
        p.mode_ang = (int)(lam * 5);
        p.split_intra = (int)(lam * 3);
        p.split_inter = (int)(lam * 4);
        p.pintra = (int)(lam * kPIntraPenBits);
        for (int i = 0; i < 64; ++i) p.mv[i] = (int)(lam * i);
        t.sao_lam16[q] = sao_lambda16(q);
      }
      dev_alloc(&rc_, sizeof(RcTables));
      HIP_OK(hipMemcpy(rc_, &t, sizeof(RcTables), hipMemcpyHostToDevice));
    }
    seq_.width = c.width;
    seq_.height = c.height;
    seq_.qp = c.qp;
    seq_.deblock = (c.deblock & 1) != 0;  // bit 0: deblocking, bit 1: SAO
    seq_.sao = (c.deblock & 2) != 0;
    seq_.max_merge_cand = c.max_merge;
    seq_.wpp = (c.deblock & 4) != 0;
    seq_.rqt = !(c.deblock & 8);
    seq_.pintra = !(c.deblock & 16);
    seq_.cascade = (c.deblock & 64) != 0;
    seq_.rdoq = !(c.deblock & 128);
    g_.rdoq = seq_.rdoq ? kRdoqMode : 0;
    seq_.mgop = c.mgop;
    if (c.mgop > 1) {
      const GopPlan gp = plan_gop(2 * c.mgop + 1, c.mgop);
      seq_.dpb_size = gp.dpb_size;
      seq_.num_reorder = gp.num_reorder;
    }
    seq_.finalize();
  }

  // The core's entropy stream, created by the Engine after every core's main stream: HIP
  // assigns streams to its (GPU_MAX_HW_QUEUES, 4 by default) hardware queues in creation order,
  // and a hardware queue runs its packets in order -- a main stream sharing a queue with an
  // entropy stream waits behind the latency-bound coder (measured: main-stream queues 36 %
  // busy).  Main streams first, then the entropy streams, gives each its own queue at 2 cores.
  // lane l's stream (the engine creates lane 0 of every core, then lane 1 of every core:
  // with GPU_MAX_HW_QUEUES = 4 the main streams and the lane-0 coders get a hardware queue
  // each; creating core 0's two lanes before core 1's put core 1's lane 0 on its main
  // stream's queue and cost 30 % at 1080p)
  void init_entropy_stream(int l) {
    if (l < ent_lanes()) init_entropy_lane(estream_[l]);
  }
  void init_entropy_lane(hipStream_t& estream_) {
    if (gpu_ent_ && !estream_) HIP_OK(hipStreamCreateWithFlags(&estream_, hipStreamNonBlocking));
  }

  // device / pinned-host bytes this group allocated (the engine's HBM footprint)
  size_t dev_bytes() const { return dev_bytes_; }
  size_t host_bytes() const { return host_bytes_; }

  // The same byte counts computed without allocating anything (EngineCache budgets and
  // auto-batch sizing decide before building an engine).  Mirrors the constructor above,
  // term by term; tests/test_hbm_budget.py checks estimate == footprint on the GPU.
  static void estimate(const EngineCfg& c, size_t& dev, size_t& host) {
    const Geo g = make_geo(c.width, c.height);
    const size_t B = (size_t)c.batch, nctu = (size_t)g.wc * g.hc, set = B * (g.ysz + 2 * g.csz);
    const int ndpb = c.mgop > 1 ? plan_gop(2 * c.mgop + 1, c.mgop).dpb_size : 2;
    const size_t qsz = (size_t)(g.W / 4) * (g.H / 4);
    const bool ge = gpu_entropy(c);
    long slot = 0, slot_host = 0;
    slot_bytes((long)B, g, ge, slot, slot_host);
    const size_t ent = ge ? env_lanes() * (2 * B * g.usz + ent_core_bytes((long)B, g)) + sizeof(EntropyTables) : 0;
    dev = set + ndpb * (set + B * 16 * g.psz + B * qsz) + ((c.deblock & 2) ? set : 0) + 2 * set +
          B * 3 * sizeof(unsigned long long) + B * nctu * sizeof(int) + 2 * B * nctu * 2 * sizeof(int16_t) +
          2 * B * nctu * sizeof(int) + (c.mgop > 1 ? 2 * B * nctu * sizeof(CtbMeOut) : 0) +
          (!(c.deblock & 16) ? pintra_bytes((long)B, (long)nctu) : 0) + (size_t)slot_count() * slot +
          sizeof(RcTables) + ent;
    host = (size_t)c.gop * B + B + (size_t)slot_count() * slot_host;
  }

  ~Core() {
    fetch_.reset();  // the fetch thread drains (every issued slot was waited for by finish())
    if (ent_dbg_) {
      unsigned long long h[8] = {};
      (void)hipDeviceSynchronize();
      (void)hipMemcpy(h, ent_dbg_, sizeof(h), hipMemcpyDeviceToHost);
      const double n = h[0] ? (double)h[0] : 1.0;
      fprintf(stderr, "[tv entropy] rows %llu: ctx bins/row %.0f, tokens/row %.0f, clocks/ctx bin %.1f, "
              "wait us/row %.1f, coding us/row %.1f, max row span us %.1f\n", h[0], h[1] / n, h[2] / n,
              h[1] ? (double)h[3] / h[1] : 0.0, h[4] / n / 100.0, h[3] / n / 2400.0, h[5] / 100.0);
      (void)hipFree(ent_dbg_);
    }
    (void)hipStreamSynchronize(stream_);
    for (auto* p : {src_.y, src_.u, src_.v, deb_.y, deb_.u, deb_.v}) (void)hipFree(p);
    for (int k = 0; k < ndpb_; ++k)
      for (auto* p : {dpb_[k].rec.y, dpb_[k].rec.u, dpb_[k].rec.v, dpb_[k].phase, dpb_[k].q}) (void)hipFree(p);
    (void)hipFree(meout_);
    (void)hipFree(pi_.qcost);
    (void)hipFree(coef_y_);
    (void)hipFree(coef_u_);
    (void)hipFree(coef_v_);
    (void)hipFree(d_sse_);
    (void)hipFree(count_scratch_);
    (void)hipFree(cmv_);
    (void)hipFree(ccost_);
    (void)hipFree(rc_);
    if (ent_[0].tab) (void)hipFree(ent_[0].tab);
    for (const EntScratch& e : ent_)
      for (void* p : {(void*)e.skip, (void*)e.midx, (void*)e.base}) (void)hipFree(p);
    (void)hipHostFree(qhost_);
    (void)hipHostFree(quni_);
    for (int k = 0; k < nslots_; ++k) {
      Slot& s = slots_[k];
      (void)hipFree(s.dev);
      (void)hipHostFree(s.host);
      (void)hipEventDestroy(s.ev);

    }
    (void)hipEventDestroy(t0_);
    (void)hipEventDestroy(t1_);
    (void)hipStreamDestroy(stream_);
    (void)hipEventDestroy(iev_[0]);
    (void)hipEventDestroy(iev_[1]);
    (void)hipStreamDestroy(istream_);
    for (hipStream_t es : estream_)
      if (es) (void)hipStreamDestroy(es);

    if (dstream_) (void)hipStreamDestroy(dstream_);
    if (eev_) (void)hipEventDestroy(eev_);
  }

  const std::vector<uint8_t>& segment(int b) const { return out_.at(b); }
  double sse(int b, int c) const { return sse_host_[b * 3 + c]; }
  long coef_bytes() const { return coef_bytes_; }
  long ent_fallbacks() const { return ent_fallbacks_; }
  long ent_host_pictures() const { return ent_host_pics_; }
  long ent_lane_pictures(int l) const { return (l >= 0 && l < kMaxEntLanes) ? ent_lane_pics_[l] : 0; }
  int host_share() const { return host_share_; }
  static std::atomic<int>& host_inflight() {  // pictures in the (process-wide) host writer pool
    static std::atomic<int> n{0};
    return n;
  }
  int ent_status() const { return ent_status_; }
  bool gpu_entropy_on() const { return gpu_ent_; }
  double entropy_ms() const { return entropy_ns_ / 1e6; }
  const Geo& geo() const { return g_; }
  // reconstruction of the segment's last display frame (after finish())
  FrameSet last_recon() const { return dpb_[last_entry_].rec; }
  hipStream_t stream() const { return stream_; }

 private:
  // frames in flight per core (host issue runs this far ahead of CABAC): TV_SLOTS, default 4
  static int slot_count() {
    static const int n = [] {
      const char* e = getenv("TV_SLOTS");
      const int v = e ? atoi(e) : 4;
      return v < 2 ? 2 : (v > 16 ? 16 : v);
    }();
    return n;
  }
  static long align(long n) { return (n + 255) & ~255L; }
  // WPP streams are entropy-coded on the GPU (k_entropy.hip) unless bit 5 asks for the host
  // WPP on, not forced to the host, and a geometry the coder handles (>= 2 CTB columns for the
  // 9.3.2.4 storage after CTB 1, <= 256 rows and columns): anything else uses the host writer from the start
  static bool gpu_entropy(const EngineCfg& c) {
    if (!((c.deblock & 4) && !(c.deblock & 32))) return false;
    const Geo g = make_geo(c.width, c.height);
    return g.wc >= 2 && g.wc <= 256 && g.hc <= 256;
  }
  // token capacity of the per-core entropy scratch: one token per luma sample of every
  // segment (the bench's textured I pictures use about a third of that); a picture that
  // needs more is coded by the host writer instead (status != 0)
  static long tok_capacity(long B, const Geo& g) {
    const char* e = getenv("TV_ENT_TOKENS_PER_PX");  // read per engine (tests shrink it)
    const double per = e ? atof(e) : 1.0;  // textured I pictures at QP 22 use more than 0.5
    return (long)(per * B * g.ysz) + 1024;
  }
  static constexpr long kTokPad = 64;
  static constexpr long kEntRegion = kEntRegionTokens;
  // head of the entropy outputs: status, seg_bytes[B], row_bytes[B][hc]
  static long ent_head_bytes(long B, const Geo& g) { return 16 + 4 * B + 4 * B * g.hc; }
  static void slot_bytes(long B, const Geo& g, bool ge, long& dev, long& host) {
    const long nctu = (long)g.wc * g.hc, cap = g.ysz + 2 * g.csz;
    host = align(B * g.usz) + align(B * g.usz * 4) + align(B * nctu * 8) + align(B * nctu * 4) + align(B * nctu * 4) +
           align(B * 4) + align(B * nctu * 12) + align(B) + align(B * g.usz) + align(B * g.usz * 4) +
           align(B * g.usz * 5) + align(B * cap * 2) + (ge ? align(ent_head_bytes(B, g)) : 0);
    // (the GPU entropy payload goes straight into the host slot's `packed` region)
    dev = host;
  }
  // per-core entropy scratch (the entropy stream codes one picture at a time): CTB token
  // regions of the single binarisation pass, the picture's contiguous token lists, CTB offsets,
  // segment totals, coder output staging and the rows' WPP hand-off
  static long ent_core_bytes(long B, const Geo& g) {
    const long cap = tok_capacity(B, g), nctu = (long)g.wc * g.hc;
    return align(B * nctu * kEntRegion * 4) + align((cap + kTokPad) * 4) + align(3 * cap + 20 * B * g.hc + 16) +
           2 * align(B * nctu * 4) + align(B * 4) + align(B * g.hc * 4) + align(B * g.hc * kEntCtx);
  }
  // qcost, gate list, pass lists, candidate list (16 bytes per CTB each), counters, candidate bytes
  static size_t pintra_bytes(long B, long nctu) { return 4 * align(B * nctu * 16) + 256 + align(B * nctu * 4); }
  struct Slot {
    uint8_t* dev = nullptr;
    uint8_t* host = nullptr;
    hipEvent_t ev{};
    std::atomic<int> pending{0};
    std::atomic<int> host_coded{0};  // hybrid entropy: slices of a host-routed picture still open
    bool qp_dirty = true;  // the slot's device QP array may not hold the sequence QP
  };
  // carve one slot buffer (device or host) into its arrays
  struct Parts {
    uint8_t *flags, *cu_log2, *intra, *ipm, *cbf, *dir, *tu;
    int16_t *mv, *mv1;
    unsigned long long* mask_y;
    unsigned* mask_c;
    int *count, *offset, *total;
    int16_t* packed;
    uint32_t* sao;
    int8_t* qp;
    int* ent_head;     // GPU entropy: status, seg_bytes[B], row_bytes[B][hc]
  };
  Parts carve(uint8_t* base) const {
    const long B = cfg_.batch, U = g_.usz;
    Parts p;
    // D2H order: flags (one byte per unit: the CU's cu_log2 / intra / cbf / dir, packed by
    // k_pack_flags) .. qp is the head every picture copies; ipm (I pictures) and mv1 (B
    // pictures) follow; the separate decision planes the kernels write stay on the device
    // and are re-expanded from the flags into the host slot by each segment's CABAC task.
    uint8_t* q = base;
    p.flags = q;
    q += align(B * U);
    p.mv = reinterpret_cast<int16_t*>(q);
    q += align(B * U * 4);
    p.mask_y = reinterpret_cast<unsigned long long*>(q);
    q += align(B * nctu_ * 8);
    p.mask_c = reinterpret_cast<unsigned*>(q);
    q += align(B * nctu_ * 4);
    p.offset = reinterpret_cast<int*>(q);
    q += align(B * nctu_ * 4);
    p.total = reinterpret_cast<int*>(q);
    q += align(B * 4);
    p.sao = reinterpret_cast<uint32_t*>(q);
    q += align(B * nctu_ * 12);
    p.qp = reinterpret_cast<int8_t*>(q);
    q += align(B);
    p.ipm = q;
    q += align(B * U);
    p.mv1 = reinterpret_cast<int16_t*>(q);
    q += align(B * U * 4);
    p.cu_log2 = q;
    p.intra = q + B * U;
    p.cbf = q + 2 * B * U;
    p.dir = q + 3 * B * U;
    p.tu = q + 4 * B * U;
    q += align(B * U * 5);
    p.packed = reinterpret_cast<int16_t*>(q);
    q += align(B * cap_ * 2);
    p.ent_head = reinterpret_cast<int*>(q);
    q += gpu_ent_ ? align(ent_head_bytes(B, g_)) : 0;
    p.count = nullptr;  // device count array lives in the scratch below
    return p;
  }
  DecisionSet slot_dec(const Slot& s) const {
    const Parts p = carve(s.dev);
    DecisionSet d;
    d.qp = p.qp;
    d.cu_log2 = p.cu_log2;
    d.intra = p.intra;
    d.ipm = p.ipm;
    d.cbf = p.cbf;
    d.mv = p.mv;
    d.coef_y = coef_y_;
    d.coef_u = coef_u_;
    d.coef_v = coef_v_;
    return d;
  }
  // the slot's decisions of a B picture (direction and list-1 planes attached)
  DecisionSet slot_dec_b(const Slot& s) const {
    DecisionSet d = slot_dec(s);
    const Parts p = carve(s.dev);
    d.dir = p.dir;
    d.mv1 = p.mv1;
    return d;
  }
  CompactSet slot_compact(const Slot& s) const {
    const Parts p = carve(s.dev);
    CompactSet c;
    c.mask_y = p.mask_y;
    c.mask_c = p.mask_c;
    c.count = reinterpret_cast<int*>(coef_count_scratch());
    c.offset = p.offset;
    c.total = p.total;
    c.packed = p.packed;
    c.cap = cap_;
    return c;
  }
  // per-CTB counts are consumed by the scan within the same frame: one scratch suffices
  void* coef_count_scratch() const { return count_scratch_; }

  // segment b's decision planes in the host slot from the transferred flag bytes
  void expand_flags(const Slot& s, int b) const {
    const Parts p = carve(s.host);
    const long U = g_.usz, o = b * U;
    for (long u = 0; u < U; ++u) {
      const uint8_t f = p.flags[o + u];
      const bool sp = (f & 3) == 3;  // an RQT-split inter CU: its size (32 / 16) in bit 2
      p.cu_log2[o + u] = (uint8_t)(sp ? ((f >> 2) & 1 ? 4 : 5) : 3 + (f & 3));
      p.tu[o + u] = (uint8_t)sp;
      p.intra[o + u] = (uint8_t)(sp ? 0 : (f >> 2) & 1);
      p.cbf[o + u] = (uint8_t)((f >> 3) & 7);
      p.dir[o + u] = (uint8_t)(f >> 6);
    }
  }
  // host view of segment b in a slot (compact levels)
  FrameData host_view(const Slot& s, int b, const SliceRefs* refs) const {
    const Parts p = carve(s.host);
    const long U = g_.usz;
    FrameData f;
    f.w8 = g_.w8;
    f.h8 = g_.h8;
    f.cu_log2 = p.cu_log2 + b * U;
    f.intra = p.intra + b * U;
    f.ipm = p.ipm + b * U;
    f.cbf = p.cbf + b * U;
    f.tu = p.tu + b * U;
    f.mv = p.mv + b * U * 2;
    f.sb_mask_y = reinterpret_cast<const uint64_t*>(p.mask_y + (long)b * nctu_);
    f.sb_mask_c = p.mask_c + (long)b * nctu_;
    f.sb_offset = p.offset + (long)b * nctu_;
    long base = 0;  // segments' packed levels are back to back
    for (int k = 0; k < b; ++k) base += p.total[k];
    f.sb_packed = p.packed + base * 16;
    f.wc = g_.wc;
    f.sao = seq_.sao ? p.sao + (long)b * nctu_ * 3 : nullptr;
    f.qp = p.qp[b];
    f.refs = refs;  // hierarchical-B streams: slice type, POCs, RPS
    if (refs && refs->type == 0) {
      f.dir = p.dir + b * U;
      f.mv1 = p.mv1 + b * U * 2;
    }
    return f;
  }

  // worker: fetch exactly the used bytes of slot s from the device on a private stream
  // wait for everything queued on `st` without spinning a CPU core
  // Host waits for GPU work: TV_SYNC_MODE=poll (default: hipEventQuery + 40 us sleeps), spin
  // (hipStreamSynchronize / hipEventSynchronize spin) or block (blocking-sync events).
  // Round 2, when a pool thread per in-flight slot waited, spin won (7510-7632 vs poll
  // 6399-6663 frames/s); since each stream group's slots complete in order on one fetch
  // thread with 3 more slots queued behind it, the wake-up latency is hidden: same-box A/B
  // (profiles/r3s2_sync_ab.txt) spin 7127 / 7091 frames/s at 10.5 / 10.3 busy cores, poll
  // 7124 / 7104 at 8.2 / 8.1, block 7121 / 7121 at 10.0 / 10.1.
  static int sync_mode() {
    static const int m = [] {
      const char* e = getenv("TV_SYNC_MODE");
      if (e && std::string(e) == "spin") return 1;
      if (e && std::string(e) == "block") return 2;
      return 0;
    }();
    return m;
  }
  static void wait_event(hipEvent_t ev) {
    if (sync_mode() == 0) {
      hipError_t e;
      while ((e = hipEventQuery(ev)) == hipErrorNotReady) std::this_thread::sleep_for(std::chrono::microseconds(40));
      HIP_OK(e);
    } else {
      HIP_OK(hipEventSynchronize(ev));
    }
  }
  static void sleep_sync(hipStream_t st) {
    if (sync_mode() == 1) {
      HIP_OK(hipStreamSynchronize(st));
      return;
    }
    thread_local hipEvent_t ev = nullptr;
    if (!ev) HIP_OK(hipEventCreateWithFlags(&ev, hipEventDisableTiming | (sync_mode() == 2 ? hipEventBlockingSync : 0)));
    HIP_OK(hipEventRecord(ev, st));
    wait_event(ev);
  }
  // GPU entropy: the pack kernel stored status, sizes, slice QPs and payload straight into the
  // pinned host slot (no copy engine, no blit kernel); false: the device could not code this
  // picture (capacity), the caller falls back to the host writer
  bool fetch_entropy(Slot& s, int B) {
    wait_event(s.ev);  // the pack kernel wrote head, slice QPs and payload into the host slot
    const Parts h = carve(s.host);
    if (h.ent_head[0] != 0) {
      ent_fallbacks_++;
      ent_status_ |= h.ent_head[0];
      return false;
    }
    long total = 0;
    for (int b = 0; b < B; ++b) total += h.ent_head[4 + b];
    coef_bytes_ += total;
    if ((total / B) * 100 > (long)g_.ysz)
      ent_dense_run_.fetch_add(1, std::memory_order_relaxed);
    else
      ent_dense_run_.store(0, std::memory_order_relaxed);
    return true;
  }
  // slice b of picture f from the GPU's substreams: header, entry points, emulation prevention
  void assemble_slice(const Slot& s, int b, int f) {
    const Parts h = carve(s.host);
    const int* seg = h.ent_head + 4;
    const int* rows = h.ent_head + 4 + cfg_.batch + (long)b * g_.hc;
    long off = 0;
    for (int k = 0; k < b; ++k) off += seg[k];
    const uint8_t* p = reinterpret_cast<const uint8_t*>(h.packed) + off;
    std::vector<const uint8_t*> ptrs(g_.hc);
    std::vector<size_t> sizes(g_.hc);
    for (int r = 0; r < g_.hc; ++r) {
      ptrs[r] = p;
      sizes[r] = (size_t)rows[r];
      p += rows[r];
    }
    const CodedPic& pic = plan_.pics[f];
    BitWriter hdr;
    const int nal = write_slice_header(seq_, h.qp[b], seq_.mgop > 1 ? &refs_[f] : nullptr, pic.disp, pic.type == 2, hdr);
    finish_wpp_slice(hdr, ptrs.data(), sizes.data(), g_.hc, nal, slices_[b][f]);
  }
  EntropyArgs entropy_args(const Slot& s, const DecisionSet& dec, const CodedPic& pic, int lane) const {
    const EntScratch& ent = ent_[lane];
    EntropyArgs a{};
    a.g = g_;
    a.pic.type = pic.type;
    a.pic.init_type = pic.type == 2 ? 0 : (pic.type == 1 ? 1 : 2);
    a.pic.poc = pic.disp;
    a.pic.ref_poc[0] = pic.ref[0];
    a.pic.ref_poc[1] = pic.ref[1];
    a.pic.sao = seq_.sao;
    a.pic.rqt = seq_.rqt;
    a.pic.max_merge = seq_.max_merge_cand;
    a.dec = dec;
    a.cs = slot_compact(s);
    const Parts d = carve(s.dev);
    a.sao = seq_.sao ? d.sao : nullptr;
    a.skip = ent.skip;
    a.midx = ent.midx;
    a.ctb_cnt = ent.ctb_cnt;
    a.regions = ent.regions;
    a.ctb_off = ent.ctb_off;
    a.seg_tok = ent.seg_tok;
    a.tokens = ent.tokens;
    a.tok_cap = tok_cap_;
    a.stage = ent.stage;
    a.wflag = ent.wflag;
    a.wctx = ent.wctx;
    a.tab = ent.tab;
    a.status = d.ent_head;
    a.seg_bytes = d.ent_head + 4;
    a.row_bytes = d.ent_head + 4 + cfg_.batch;
    const Parts h = carve(s.host);  // the pack kernel's destination (pinned, device-visible)
    HIP_OK(hipHostGetDevicePointer(reinterpret_cast<void**>(&a.hhead), h.ent_head, 0));
    HIP_OK(hipHostGetDevicePointer(reinterpret_cast<void**>(&a.hqp), h.qp, 0));
    HIP_OK(hipHostGetDevicePointer(reinterpret_cast<void**>(&a.hout), h.packed, 0));
    a.hout_cap = (long)cfg_.batch * cap_ * 2;
    a.dbg = ent_dbg_;
    return a;
  }

  void fetch_slot(Slot& s, int B, int ptype) {
    // the core's D2H stream: used by its one fetch thread only, destroyed with the core (a
    // thread_local stream outlived the engine and kept a hardware queue referenced)
    if (!dstream_) HIP_OK(hipStreamCreateWithFlags(&dstream_, hipStreamNonBlocking));
    hipStream_t ws = dstream_;
    wait_event(s.ev);
    const Parts d = carve(s.dev), h = carve(s.host);
    const long U = g_.usz;
    // Every D2H copy is a blit-kernel launch (~10 us of CU time each): the full-batch case
    // moves the whole contiguous header (decision planes .. SAO params) in one copy and all
    // segments' packed levels (back to back) in a second one.
    // a P picture with intra quadrants needs the mode plane too (right after the head)
    const bool pipm = ptype == 1 && pi_.qcost;
    SdmaD2H& dma = SdmaD2H::get();
    SdmaD2H::Batch batch;
    auto d2h = [&](void* dst, const void* src, size_t n) {
      if (dma.on()) batch.add(dst, src, n);
      else HIP_OK(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, ws));
    };
    auto drain = [&] {
      if (dma.on()) {
        dma.run(batch);
        batch.items.clear();
      } else {
        sleep_sync(ws);
      }
    };
    if (B == cfg_.batch) {
      const long head = (pipm ? d.ipm + B * U : reinterpret_cast<uint8_t*>(d.qp) + B) - d.flags;
      d2h(h.flags, d.flags, head);
    } else {
      if (pipm) d2h(h.ipm, d.ipm, B * U);  // partial batch: each plane is laid out for cfg_.batch segments
      d2h(h.total, d.total, B * 4);
      d2h(h.qp, d.qp, B);
      d2h(h.flags, d.flags, B * U);
      if (ptype != 2) d2h(h.mv, d.mv, B * U * 4);
      if (seq_.sao) d2h(h.sao, d.sao, B * nctu_ * 12);
      d2h(h.mask_y, d.mask_y, B * nctu_ * 8);
      d2h(h.mask_c, d.mask_c, B * nctu_ * 4);
      d2h(h.offset, d.offset, B * nctu_ * 4);
    }
    if (ptype == 2) d2h(h.ipm, d.ipm, B * U);
    if (ptype == 0) d2h(h.mv1, d.mv1, B * U * 4);
    drain();
    long groups = 0;
    for (int b = 0; b < B; ++b) groups += h.total[b];
    const long bytes = groups * 16 * 2;
    if (groups > (long)B * cap_ / 16) throw std::runtime_error("compact level overflow");
    if (bytes) d2h(h.packed, d.packed, bytes);
    drain();
    coef_bytes_ += bytes;
  }


 public:
  // ---- one encode call, split so the Engine can interleave several cores' frames ----
  // qmap: this core's [nseg][nframes] slice QPs (nullptr: the sequence QP everywhere)
  void begin(int nseg, int nframes, const int8_t* qmap) {
    if (nseg < 1 || nseg > cfg_.batch) throw std::runtime_error("nseg out of range");
    if (nframes < 1 || nframes > cfg_.gop) throw std::runtime_error("nframes out of range");
    B_ = nseg;
    F_ = nframes;
    plan_ = plan_gop(nframes, cfg_.mgop);
    refs_.assign(plan_.pics.size(), SliceRefs{});
    for (size_t k = 0; k < plan_.pics.size(); ++k) refs_[k] = slice_refs(plan_.pics[k]);
    for (auto& e : dpb_) e.disp = -1;
    // per-picture QPs in coding order: the caller's base (display order) + the layer offset
    // constant QP, I P P P, cascade on: per-picture QPs like an explicit map (CRF keeps its own)
    const bool cascade = !qmap && seq_.cascade && cfg_.mgop <= 1 && cfg_.crf <= 0;
    qmap_given_ = qmap != nullptr || cfg_.mgop > 1 || cascade;
    for (int k = 0; k < nframes; ++k)
      for (int b = 0; b < nseg; ++b) {
        const CodedPic& p = plan_.pics[k];
        // only the caller's QP is range-checked; the cascade / layer offsets clip (as the golden
        // encoder does, cpu_encoder.cpp), so QP 0..4 and 51 keep working with the cascade on
        const int q0 = qmap ? qmap[b * nframes + p.disp] : cfg_.qp;
        if (q0 < 0 || q0 > 51) throw std::runtime_error("slice QP out of range");
        const int base = q0 + (cascade ? ippp_qp_offset(p.disp) : 0);
        qhost_[k * nseg + b] = (int8_t)clip3(0, 51, base + gop_layer_qp_offset(p.type, p.layer, cfg_.mgop));
      }
    last_frames_ = nframes;
    out_.assign(B_, {});
    coef_bytes_ = 0;
    entropy_ns_ = 0;
    slices_.assign(B_, std::vector<std::vector<uint8_t>>(F_));
    failed_ = 0;
    err_.clear();
    HIP_OK(hipMemsetAsync(d_sse_, 0, B_ * 3 * sizeof(unsigned long long), stream_));
    HIP_OK(hipEventRecord(t0_, stream_));
  }

  // Enqueue frame f of every segment (upload(f, B) fills src_ on stream()), then hand its
  // decisions to the CABAC pool.  Blocks only when the slot ring is full.
  template <class Upload> void issue(int f, Upload&& upload) {
    const int B = B_, F = F_;
    Range frame_range(plan_.pics[f].type == 2 ? "engine.frame.intra" : "engine.frame.inter");
    Slot& s = slots_[f % nslots_];
    wait_slot(s);
    const DecisionSet dec0 = slot_dec(s);
    // this frame's QPs: copied only when they differ from what the slot already holds (a
    // constant-QP stream pays nothing per frame; a QP map or CRF rewrites them every frame)
    if (qmap_given_) {
      launch_set_qp(dec0.qp, qhost_ + f * B, B, stream_);
      s.qp_dirty = true;
    } else if (s.qp_dirty) {  // back to the sequence QP for every segment slot
      launch_set_qp(dec0.qp, quni_, cfg_.batch, stream_);
      s.qp_dirty = false;
    }
    if (cfg_.crf > 0 && !qmap_given_) s.qp_dirty = true;  // k_rc_crf overwrites them
    const CodedPic& pic = plan_.pics[f];
    const bool intra = pic.type == 2, bpic = pic.type == 0;
    upload(pic.disp, B);
    // a free DPB entry: none of the pictures this or a later picture still references
    int e = -1;
    for (int k = 0; k < ndpb_ && e < 0; ++k) {
      const int d = dpb_[k].disp;
      if (d < 0 || std::find(pic.rps.begin(), pic.rps.end(), d) == pic.rps.end()) e = k;
    }
    if (e < 0) throw std::runtime_error("no free DPB entry");
    auto entry_of = [&](int disp) -> DpbEntry& {
      for (int k = 0; k < ndpb_; ++k)
        if (dpb_[k].disp == disp) return dpb_[k];
      throw std::runtime_error("reference picture not in the DPB");
    };
    DpbEntry& cur_e = dpb_[e];
    const FrameSet fin_set = cur_e.rec;
    const FrameSet cur = seq_.sao ? deb_ : fin_set;  // SAO filters deb_ into the entry
    DecisionSet dec = bpic ? slot_dec_b(s) : dec0;
    if (!intra && seq_.rqt) dec.tu = carve(s.dev).tu;  // RQT: P and B pictures
    // TV_SYNC_DEBUG=1: synchronise and check after every stage (fault isolation)
    auto stage = [&](const char* name) {
      if (!sync_debug_) return;
      const hipError_t e1 = hipGetLastError(), e2 = hipStreamSynchronize(stream_);
      if (e1 != hipSuccess || e2 != hipSuccess)
        throw std::runtime_error(std::string("stage ") + name + " failed: " +
                                 hipGetErrorString(e1 != hipSuccess ? e1 : e2));
    };
    stage("upload");
    launch_quarter(src_, cur_e.q, g_, B, stream_);  // lookahead plane (coarse reference of later pictures)
    // the previous coded picture's decisions still sit in its slot (reused only nslots_ frames later)
    const int16_t* prev_mv = f ? slot_dec(slots_[(f - 1) % nslots_]).mv : nullptr;
    const long cstride = (long)B * nctu_;
    MeBuffers me[2];
    int rng[2] = {cfg_.range, cfg_.range};
    for (int l = 0; l < 2; ++l) {
      if (pic.ref[l] < 0) continue;
      me[l] = MeBuffers{cur_e.q, entry_of(pic.ref[l]).q, prev_mv, cmv_ + l * cstride * 2, ccost_ + l * cstride};
      rng[l] = gop_search_range(cfg_.range, std::abs(pic.disp - pic.ref[l]), cfg_.mgop);
      launch_coarse_me(me[l], g_, rc_, cfg_.qp, rng[l], B, stream_);
    }
    if (cfg_.crf > 0 && !qmap_given_) launch_rc_crf(cur_e.q, ccost_, dec.qp, g_, cfg_.crf, intra, B, stream_);
    if (intra) {  // fork onto the priority stream and join back
      HIP_OK(hipEventRecord(iev_[0], stream_));
      HIP_OK(hipStreamWaitEvent(istream_, iev_[0], 0));
      launch_intra_frame(src_, cur, dec, g_, rc_, B, istream_);
      HIP_OK(hipEventRecord(iev_[1], istream_));
      HIP_OK(hipStreamWaitEvent(stream_, iev_[1], 0));
    } else if (!bpic) {
      const DpbEntry& r0 = entry_of(pic.ref[0]);
      launch_inter_frame(src_, r0.rec, r0.phase, cur, dec, g_, rc_, rng[0], me[0], B, stream_,
                         pi_.qcost ? &pi_ : nullptr);
    } else {
      const DpbEntry& r0 = entry_of(pic.ref[0]);
      const DpbEntry& r1 = entry_of(pic.ref[1]);
      launch_inter_frame_b(src_, r0.rec, r0.phase, r1.rec, r1.phase, cur, dec, g_, rc_, rng, me[0], me[1], meout_,
                           B, stream_);
    }
    stage(intra ? "intra" : "inter");
    launch_compact(dec, g_, slot_compact(s), B, stream_);
    launch_pack_flags(dec, carve(s.dev).flags, g_, B, stream_);
    stage("compact");
    if (seq_.deblock) launch_deblock(cur, dec, g_, B, stream_);
    stage("deblock");
    if (seq_.sao) launch_sao(src_, cur, fin_set, carve(s.dev).sao, dec.qp, rc_, g_, B, stream_, d_sse_);
    stage("sao");
    cur_e.disp = pic.disp;
    if (pic.disp == F - 1) last_entry_ = e;
    if (pic.referenced) launch_phase_planes(fin_set, cur_e.phase, g_, B, stream_);  // a later picture's reference
    stage("phase_planes");
    if (!seq_.sao) launch_sse(src_, fin_set, g_, d_sse_, B, stream_);  // with SAO: summed by k_sao_decide
    stage("sse");
    HIP_OK(hipGetLastError());
    // hybrid entropy (TV_ENT_HOST = n > 0): while fewer than n pictures sit in the host writer
    // pool, the next one is coded there (its decisions are fetched as in host mode) and its
    // entropy kernels never compete with the analysis kernels; otherwise the GPU codes it
    const bool on_host = gpu_ent_ && host_share() > 0 && host_inflight().load(std::memory_order_relaxed) < host_share();
    if (on_host) {
      host_inflight().fetch_add(1, std::memory_order_relaxed);
      ent_host_pics_++;
    }
    const bool use_gpu = gpu_ent_ && !on_host;
    if (use_gpu) {  // entropy coding on its own stream: the next picture's kernels run meanwhile
      // one lane, or pictures alternating between two when the content is dense: measured at
      // 1080p, textured content (~3x the bins) codes 4365 vs 3765 frames/s with two lanes, but
      // smooth content 6636 vs 7100 (a second coder in flight slows the analysis kernels more
      // than it helps); the switch: the last three coded pictures' payloads above 0.01 bytes
      // per luma sample (smooth P pictures ~0.005, textured ~0.015; an I picture alone does
      // not switch).  An event query per picture to find a busy
      // lane serialised the issue thread (-14 %).
      const bool dense = ent_dense_run_.load(std::memory_order_relaxed) >= dense_after();  // not just an I picture
      const int lane = (ent_lanes() > 1 && dense) ? f % ent_lanes() : 0;
      HIP_OK(hipEventRecord(eev_, stream_));
      HIP_OK(hipStreamWaitEvent(estream_[lane], eev_, 0));
      // binarisation on the core's entropy stream (one picture at a time: its scratch is per
      // core), the serial arithmetic coder on the slot's own stream, so the coders of the
      // pictures in flight overlap (each is a handful of latency-bound waves)
      const EntropyArgs ea = entropy_args(s, dec, pic, lane);
      static const bool serial = [] {  // TV_ENT_SERIAL=1: entropy on the main stream (diagnostics)
        const char* e = getenv("TV_ENT_SERIAL");
        return e && *e == '1';
      }();
      hipStream_t es = serial ? stream_ : estream_[lane];
      launch_entropy_bin(ea, B, es);
      launch_entropy_ac(ea, B, es);
      stage("entropy");
      HIP_OK(hipGetLastError());
      HIP_OK(hipEventRecord(s.ev, es));
      ent_lane_pics_[lane]++;
    } else {
      HIP_OK(hipEventRecord(s.ev, stream_));
    }
    s.pending.store(B + 1, std::memory_order_release);
    // The slot's GPU wait + D2H runs on this core's one fetch thread (slots complete in
    // stream order, so a FIFO of waits loses nothing): one thread per core spins on the
    // completion events instead of one pool thread per in-flight slot, and the pool's
    // threads only ever run CABAC.
    if (on_host) s.host_coded.store(B, std::memory_order_relaxed);
    fetch_->submit([this, &s, B, f, use_gpu] {
      bool gpu = false;  // the GPU coded the picture: only the slice NALs are assembled here
      try {
        Range r("engine.d2h");
        gpu = use_gpu && fetch_entropy(s, B);

        if (!gpu) fetch_slot(s, B, plan_.pics[f].type);
      } catch (const std::exception& e) {
        fail(e);
        if (s.host_coded.exchange(0, std::memory_order_relaxed))  // hand back its host-writer share
          host_inflight().fetch_sub(1, std::memory_order_relaxed);
        release(s, B + 1);
        return;
      }
      release(s, 1);
      for (int b = 0; b < B; ++b)
        pool_->submit([this, &s, b, f, gpu] {
          try {
            Range r(gpu ? "engine.slice_nal" : "engine.cabac_slice");
            const auto c0 = std::chrono::steady_clock::now();
            const CodedPic& p = plan_.pics[f];
            if (gpu) {
              assemble_slice(s, b, f);
            } else {
              expand_flags(s, b);
              write_slice(seq_, host_view(s, b, seq_.mgop > 1 ? &refs_[f] : nullptr), p.disp, p.type == 2,
                          slices_[b][f]);
            }
            entropy_ns_ += std::chrono::duration_cast<std::chrono::nanoseconds>(
                               std::chrono::steady_clock::now() - c0).count();
          } catch (const std::exception& e) {
            fail(e);
          }
          if (s.host_coded.load(std::memory_order_relaxed) && s.host_coded.fetch_sub(1) == 1)
            host_inflight().fetch_sub(1, std::memory_order_relaxed);  // the picture's last slice
          release(s, 1);
        });
    });
  }

  void end_record() { HIP_OK(hipEventRecord(t1_, stream_)); }

  void finish() {
    for (int k = 0; k < nslots_; ++k) wait_slot(slots_[k]);
    sleep_sync(stream_);
    if (failed_) throw std::runtime_error("encode failed: " + err_);
    std::vector<unsigned long long> sse(B_ * 3);
    HIP_OK(hipMemcpy(sse.data(), d_sse_, B_ * 3 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    sse_host_.assign(sse.begin(), sse.end());
    for (int b = 0; b < B_; ++b) {
      write_parameter_sets(seq_, out_[b]);
      for (int f = 0; f < F_; ++f) out_[b].insert(out_[b].end(), slices_[b][f].begin(), slices_[b][f].end());
    }
  }

  // Single-core encode (groups == 1)
  template <class Upload> void run(int nseg, int nframes, Upload&& upload) {
    begin(nseg, nframes, nullptr);
    for (int f = 0; f < nframes; ++f) issue(f, upload);
    end_record();
    finish();
  }

  FrameSet src() const { return src_; }
  hipEvent_t t0() const { return t0_; }
  hipEvent_t t1() const { return t1_; }
  long entropy_ns() const { return entropy_ns_; }

 private:
  // Slot hand-back: the host thread sleeps on a condition variable instead of spinning, so
  // eight ranks on one node do not burn cores the CABAC pools need.
  void release(Slot& s, int n) {
    if (s.pending.fetch_sub(n, std::memory_order_acq_rel) == n) {
      std::lock_guard<std::mutex> lk(slot_mu_);
      slot_cv_.notify_all();
    }
  }
  void wait_slot(Slot& s) {
    std::unique_lock<std::mutex> lk(slot_mu_);
    slot_cv_.wait(lk, [&] { return s.pending.load(std::memory_order_acquire) == 0; });
  }
  void fail(const std::exception& e) {
    std::lock_guard<std::mutex> lk(err_mu_);
    err_ = e.what();
    failed_ = 1;
  }

  EngineCfg cfg_;
  Geo g_;
  SeqConfig seq_;
  RcTables* rc_ = nullptr;
  // GPU entropy coding (k_entropy.hip): its own stream per core, per-core scratch
  bool gpu_ent_ = false;
  // entropy lanes: pictures alternate between lanes (own scratch + stream), so the coders of
  // two pictures overlap (TV_ENT_LANES, default 2; textured content needed more than one)
  static constexpr int kMaxEntLanes = 4;
  static int env_lanes() {
    const char* e = getenv("TV_ENT_LANES");
    const int v = e ? atoi(e) : 2;
    return v < 1 ? 1 : (v > kMaxEntLanes ? kMaxEntLanes : v);
  }
  int ent_lanes_ = env_lanes();
  // TV_ENT_DENSE_AFTER (default 3): consecutive dense pictures before the second lane is used
  // (0: alternate lanes from the first picture -- the tests' way into the two-lane path)
  int dense_after_ = [] {  // read per engine (tests set it)
    const char* e = getenv("TV_ENT_DENSE_AFTER");
    return e ? std::max(0, atoi(e)) : 3;
  }();
  int dense_after() const { return dense_after_; }
  int ent_lanes() const { return ent_lanes_; }
  hipStream_t estream_[kMaxEntLanes] = {};
  std::atomic<int> ent_dense_run_{0};  // consecutive GPU-coded pictures above 0.01 bytes per sample
  long ent_lane_pics_[kMaxEntLanes] = {};
  hipStream_t dstream_ = nullptr;  // D2H copies of host-coded slots (the fetch thread's)
  hipEvent_t eev_ = nullptr;
  struct EntScratch {
    uint8_t* skip = nullptr;
    int8_t* midx = nullptr;
    uint8_t* base = nullptr;  // the ent_core_bytes() allocation
    uint32_t *regions = nullptr, *tokens = nullptr;
    uint8_t* stage = nullptr;
    int *ctb_cnt = nullptr, *ctb_off = nullptr, *seg_tok = nullptr, *wflag = nullptr;
    uint8_t* wctx = nullptr;
    EntropyTables* tab = nullptr;
  } ent_[kMaxEntLanes];
  long tok_cap_ = 0, slot_host_bytes_ = 0;
  unsigned long long* ent_dbg_ = nullptr;  // TV_ENT_DEBUG=1: coder counters (EntropyArgs::dbg)
  std::atomic<long> ent_fallbacks_{0};
  std::atomic<long> ent_host_pics_{0};
  // hybrid entropy: pictures allowed in the host writer at once (TV_ENT_HOST, read when the
  // core is built; 0 = every picture on the GPU)
  int host_share_ = [] {
    const char* e = getenv("TV_ENT_HOST");
    return e ? atoi(e) : 0;
  }();
  std::atomic<int> ent_status_{0};
  bool qmap_given_ = false;  // an explicit QP map (2-pass plan) overrides in-engine CRF
  int8_t* qhost_ = nullptr;  // pinned [frame][segment] slice QPs of the current call
  int8_t* quni_ = nullptr;   // pinned: the sequence QP for every segment slot
  hipStream_t stream_{}, istream_{};
  hipEvent_t iev_[2]{};
  static constexpr int kMaxDpb = 8;
  struct DpbEntry {
    FrameSet rec{};
    uint8_t* phase = nullptr;
    uint8_t* q = nullptr;
    int disp = -1;  // display index of the picture held (-1: free)
  };
  FrameSet src_{}, deb_{};
  DpbEntry dpb_[kMaxDpb];
  int ndpb_ = 2, last_entry_ = 0;
  GopPlan plan_;
  std::vector<SliceRefs> refs_;
  CtbMeOut* meout_ = nullptr;
  PIntraBuffers pi_{};  // qcost == nullptr: intra-in-P off (TV_PINTRA=0)
  int16_t *coef_y_ = nullptr, *coef_u_ = nullptr, *coef_v_ = nullptr;
  unsigned long long* d_sse_ = nullptr;
  void* count_scratch_ = nullptr;
  int16_t* cmv_ = nullptr;
  int* ccost_ = nullptr;
  long qsz_ = 0;
  int nctu_ = 0;
  int last_frames_ = 1;
  const bool sync_debug_ = [] {
    const char* e = getenv("TV_SYNC_DEBUG");
    return e && *e == '1';
  }();
  long cap_ = 0;
  std::unique_ptr<Slot[]> slots_;
  int nslots_ = 0;
  long slot_bytes_ = 0;
  hipEvent_t t0_{}, t1_{};
  ThreadPool* pool_;
  int B_ = 0, F_ = 0;
  std::vector<std::vector<std::vector<uint8_t>>> slices_;
  std::mutex slot_mu_;
  std::condition_variable slot_cv_;
  std::atomic<int> failed_{0};
  std::string err_;
  std::mutex err_mu_;
  std::vector<std::vector<uint8_t>> out_;
  std::vector<double> sse_host_;
  std::atomic<long> coef_bytes_{0};
  std::atomic<long> entropy_ns_{0};
  std::unique_ptr<ThreadPool> fetch_;  // declared last: its thread stops before anything above is freed
};

// The engine: `groups` cores, each owning batch/groups segments on its own stream.  Frame f
// of core g is issued in host step f + g, so the cores run one frame apart: while one
// core's I-frame CTB wavefront (latency-bound, ~1 wave per CU) runs, the other cores'
// motion search / reconstruction kernels fill the rest of the GPU.
class Engine {
 public:
  explicit Engine(const EngineCfg& c) : cfg_(c) {
    if (c.batch < 1 || c.batch > kMaxBatch) throw std::runtime_error("batch must be 1..64");
    HIP_OK(hipSetDevice(c.device));
    int G = c.groups < 1 ? 1 : c.groups;
    if (G > c.batch) G = c.batch;
    per_ = (c.batch + G - 1) / G;
    G = (c.batch + per_ - 1) / per_;
    pool_ = std::make_unique<ThreadPool>(c.threads, c.device);
    for (int g = 0; g < G; ++g) {
      EngineCfg cc = c;
      cc.batch = std::min(per_, c.batch - g * per_);
      cores_.push_back(std::make_unique<Core>(cc, pool_.get()));
    }
    for (int l = 0; l < 4; ++l)  // Core::kMaxEntLanes
      for (auto& core : cores_) core->init_entropy_stream(l);
  }
  ~Engine() {
    intra_timing_report();
    cores_.clear();
    pool_.reset();
  }

  // Encode nseg segments of the synthetic source: segment b = frames [starts[b], +gop).
  void encode_synth(const int* starts, int nseg, int nframes, const int8_t* qmap) {
    run(nseg, nframes, qmap, [&](Core& core, int b0, int f, int B) {
      FrameIdx fi{};
      for (int b = 0; b < B; ++b) fi.t[b] = starts[b0 + b] + f;
      launch_synth(core.src(), core.geo(), cfg_.seed, fi, B, core.stream());
    });
  }

  // Encode nseg segments of nframes (1..gop) host frames each, coded-size planar I420 laid
  // out [segment][frame][Y | U | V] (planes padded to the coded size by the caller).
  void encode_host(const uint8_t* frames, int nseg, int nframes, const int8_t* qmap) {
    encode_mem(frames, nseg, nframes, qmap);
  }

  // Same layout, but the frames already live in device memory on this GPU (produced by
  // the caller's pre-processing kernels, e.g. the ABR ladder's tone-map + Lanczos rungs):
  // device-to-device copies into each group's source planes, no PCIe crossing.  The
  // caller must have finished writing them (its stream synchronised) before the call.
  void encode_device(const uint8_t* frames, int nseg, int nframes, const int8_t* qmap) {
    if (reinterpret_cast<uintptr_t>(frames) % 16) {  // the gather kernel reads uint4s
      encode_mem(frames, nseg, nframes, qmap);
      return;
    }
    run(nseg, nframes, qmap, [&](Core& core, int b0, int f, int B) {
      const Geo& g = core.geo();
      const long fsz = g.ysz + 2 * g.csz;
      launch_gather_frames(frames + ((long)b0 * nframes + f) * fsz, (long)nframes * fsz, core.src(), g, B,
                           core.stream());
    });
  }

 private:
  // hipMemcpyDefault: the runtime resolves host (pageable / pinned) vs device pointers.
  void encode_mem(const uint8_t* frames, int nseg, int nframes, const int8_t* qmap) {
    run(nseg, nframes, qmap, [&](Core& core, int b0, int f, int B) {
      const Geo& g = core.geo();
      const long fsz = g.ysz + 2 * g.csz;
      const FrameSet src = core.src();
      for (int b = 0; b < B; ++b) {
        const uint8_t* p = frames + ((long)(b0 + b) * nframes + f) * fsz;
        HIP_OK(hipMemcpyAsync(src.y + b * g.ysz, p, g.ysz, hipMemcpyDefault, core.stream()));
        HIP_OK(hipMemcpyAsync(src.u + b * g.csz, p + g.ysz, g.csz, hipMemcpyDefault, core.stream()));
        HIP_OK(hipMemcpyAsync(src.v + b * g.csz, p + g.ysz + g.csz, g.csz, hipMemcpyDefault, core.stream()));
      }
    });
  }

 public:

  const std::vector<uint8_t>& segment(int b) const { return core_of(b).segment(b % per_); }
  double sse(int b, int c) const { return core_of(b).sse(b % per_, c); }
  double gpu_ms() const { return gpu_ms_; }
  double wall_ms() const { return wall_ms_; }
  long coef_bytes() const {
    long n = 0;
    for (int g = 0; g < used_; ++g) n += cores_[g]->coef_bytes();
    return n;
  }
  double entropy_ms() const {
    double n = 0;
    for (int g = 0; g < used_; ++g) n += cores_[g]->entropy_ms();
    return n;
  }
  // GPU entropy coding: on?, pictures the host writer had to code instead (since construction)
  // and the OR of their device status words (1 token capacity, 2/4 syntax, 8 payload capacity)
  void entropy_stats(int& on, long& fallbacks, int& status) const {
    on = cores_[0]->gpu_entropy_on() ? 1 : 0;
    fallbacks = 0;
    status = 0;
    for (const auto& c : cores_) {
      fallbacks += c->ent_fallbacks();
      status |= c->ent_status();
    }
  }
  long entropy_host_pictures() const {
    long n = 0;
    for (const auto& c : cores_) n += c->ent_host_pictures();
    return n;
  }
  long entropy_lane_pictures(int l) const {
    long n = 0;
    for (const auto& c : cores_) n += c->ent_lane_pictures(l);
    return n;
  }
  const Geo& geo() const { return cores_[0]->geo(); }
  size_t dev_bytes() const {
    size_t n = 0;
    for (const auto& c : cores_) n += c->dev_bytes();
    return n;
  }
  size_t host_bytes() const {
    size_t n = 0;
    for (const auto& c : cores_) n += c->host_bytes();
    return n;
  }
  // footprint of an engine of config c (the group split of the constructor), no allocation
  static void estimate(const EngineCfg& c, size_t& dev, size_t& host) {
    int G = c.groups < 1 ? 1 : c.groups;
    if (G > c.batch) G = c.batch;
    const int per = (c.batch + G - 1) / G;
    G = (c.batch + per - 1) / per;
    dev = host = 0;
    for (int g = 0; g < G; ++g) {
      EngineCfg cc = c;
      cc.batch = std::min(per, c.batch - g * per);
      size_t d = 0, h = 0;
      Core::estimate(cc, d, h);
      dev += d;
      host += h;
    }
  }
  FrameSet last_recon(int b, int& local) const {
    local = b % per_;
    return core_of(b).last_recon();
  }

 private:
  const Core& core_of(int b) const {
    if (b < 0 || b / per_ >= used_) throw std::runtime_error("segment index out of range");
    return *cores_[b / per_];
  }
  // qmap: [nseg][nframes] slice QPs (nullptr: the sequence QP)
  template <class Upload> void run(int nseg, int nframes, const int8_t* qmap, Upload&& upload) {
    if (nseg < 1 || nseg > cfg_.batch) throw std::runtime_error("nseg out of range");
    HIP_OK(hipSetDevice(cfg_.device));  // the calling host thread may be new (ABR rung threads)
    const auto w0 = std::chrono::steady_clock::now();
    used_ = (nseg + per_ - 1) / per_;
    for (int g = 0; g < used_; ++g)
      cores_[g]->begin(std::min(per_, nseg - g * per_), nframes, qmap ? qmap + (long)g * per_ * nframes : nullptr);
    for (int t = 0; t < nframes + used_ - 1; ++t)
      for (int g = 0; g < used_; ++g) {
        const int f = t - g;
        if (f < 0 || f >= nframes) continue;
        Core& core = *cores_[g];
        core.issue(f, [&](int ff, int B) { upload(core, g * per_, ff, B); });
        if (f == nframes - 1) core.end_record();
      }
    std::string err;
    for (int g = 0; g < used_; ++g) {
      try {
        cores_[g]->finish();
      } catch (const std::exception& e) {
        if (err.empty()) err = e.what();
      }
    }
    if (!err.empty()) throw std::runtime_error(err);
    float ms = 0;
    HIP_OK(hipEventElapsedTime(&ms, cores_[0]->t0(), cores_[used_ - 1]->t1()));
    gpu_ms_ = ms;
    wall_ms_ = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - w0).count();
  }

  EngineCfg cfg_;
  int per_ = 1, used_ = 0;
  std::unique_ptr<ThreadPool> pool_;
  std::vector<std::unique_ptr<Core>> cores_;
  double gpu_ms_ = 0, wall_ms_ = 0;
};

}  // namespace gpu
}  // namespace tv

// ------------------------------------- C API --------------------------------------------
namespace {
thread_local std::string g_gpu_err;
template <class F> int gguard(F&& f) {
  try {
    f();
    return 0;
  } catch (const std::exception& e) {
    g_gpu_err = e.what();
    return -1;
  }
}
}  // namespace

extern "C" {
const char* tv_gpu_last_error() { return g_gpu_err.c_str(); }

int tv_gpu_device_count() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

void* tv_engine_new(int width, int height, int qp, int batch, int gop, int range, int deblock,
                    uint32_t seed, int threads, int device, int max_merge, int crf) {
  void* r = nullptr;
  gguard([&] {
    // TV_ENGINE_GROUPS: segment groups on separate streams, one frame apart (default 2)
    const char* ge = getenv("TV_ENGINE_GROUPS");
    const int groups = ge ? std::max(1, atoi(ge)) : (batch >= 2 ? 2 : 1);
    if (crf < 0 || crf > 51) throw std::runtime_error("crf must be 0 (off) or 1..51");
    tv::gpu::EngineCfg c{width, height, qp, batch, gop, range, deblock, threads, device, max_merge, seed, groups, crf};
    r = new tv::gpu::Engine(c);
  });
  return r;
}
// hierarchical-B engine (tv/gop.h): mgop = mini-GOP size (power of 2; 1 = I P P P)
void* tv_engine_new_b(int width, int height, int qp, int batch, int gop, int range, int deblock, uint32_t seed,
                      int threads, int device, int max_merge, int crf, int mgop) {
  void* r = nullptr;
  gguard([&] {
    const char* ge = getenv("TV_ENGINE_GROUPS");
    const int groups = ge ? std::max(1, atoi(ge)) : (batch >= 2 ? 2 : 1);
    if (crf < 0 || crf > 51) throw std::runtime_error("crf must be 0 (off) or 1..51");
    tv::gpu::EngineCfg c{width, height, qp, batch, gop, range, deblock, threads, device, max_merge, seed, groups, crf};
    c.mgop = mgop;
    r = new tv::gpu::Engine(c);
  });
  return r;
}
void tv_engine_free(void* e) { delete static_cast<tv::gpu::Engine*>(e); }
// qmap (nullable): [nseg][nframes] slice QPs chosen by the caller's rate control
int tv_engine_encode_synth(void* e, const int* starts, int nseg, int nframes, const int8_t* qmap) {
  return gguard([&] { static_cast<tv::gpu::Engine*>(e)->encode_synth(starts, nseg, nframes, qmap); });
}
int tv_engine_encode_host(void* e, const uint8_t* frames, int nseg, int nframes, const int8_t* qmap) {
  return gguard([&] { static_cast<tv::gpu::Engine*>(e)->encode_host(frames, nseg, nframes, qmap); });
}
size_t tv_engine_segment_size(void* e, int b) { return static_cast<tv::gpu::Engine*>(e)->segment(b).size(); }
void tv_engine_segment_copy(void* e, int b, uint8_t* dst) {
  const auto& v = static_cast<tv::gpu::Engine*>(e)->segment(b);
  std::memcpy(dst, v.data(), v.size());
}
void tv_engine_sse(void* e, int b, double* out3) {
  for (int c = 0; c < 3; ++c) out3[c] = static_cast<tv::gpu::Engine*>(e)->sse(b, c);
}
void tv_engine_timing(void* e, double* gpu_ms, double* wall_ms, double* entropy_ms, double* coef_mb) {
  auto* E = static_cast<tv::gpu::Engine*>(e);
  *gpu_ms = E->gpu_ms();
  *wall_ms = E->wall_ms();
  *entropy_ms = E->entropy_ms();
  *coef_mb = E->coef_bytes() / 1e6;
}
void tv_engine_entropy_stats(void* e, int* on, long long* fallbacks, int* status) {
  long f = 0;
  static_cast<tv::gpu::Engine*>(e)->entropy_stats(*on, f, *status);
  *fallbacks = f;
}
// pictures the hybrid policy (TV_ENT_HOST) sent to the host writer since construction
long long tv_engine_entropy_host_pictures(void* e) {
  return static_cast<tv::gpu::Engine*>(e)->entropy_host_pictures();
}
// pictures GPU coder lane l coded since construction (lane 1 only on dense content)
long long tv_engine_entropy_lane_pictures(void* e, int lane) {
  return static_cast<tv::gpu::Engine*>(e)->entropy_lane_pictures(lane);
}
// The same for an engine not built yet (same arguments as tv_engine_new_b's geometry part)
int tv_engine_estimate(int width, int height, int batch, int gop, int deblock, int mgop, unsigned long long* dev,
                       unsigned long long* host) {
  return gguard([&] {
    const char* ge = getenv("TV_ENGINE_GROUPS");
    const int groups = ge ? std::max(1, atoi(ge)) : (batch >= 2 ? 2 : 1);
    tv::gpu::EngineCfg c{width, height, 27, batch, gop, 64, deblock, 1, 0, 5, 1u, groups, 0};
    c.mgop = mgop;
    size_t d = 0, h = 0;
    tv::gpu::Engine::estimate(c, d, h);
    *dev = d;
    *host = h;
  });
}
// HBM / pinned-host bytes the engine allocated at construction (EngineCache byte budget)
void tv_engine_footprint(void* e, unsigned long long* dev, unsigned long long* host) {
  auto* E = static_cast<tv::gpu::Engine*>(e);
  *dev = E->dev_bytes();
  *host = E->host_bytes();
}
// copy the last frame's coded-size reconstruction of segment b (tests)
int tv_engine_encode_device(void* e, const uint8_t* dframes, int nseg, int nframes, const int8_t* qmap) {
  return gguard([&] { static_cast<tv::gpu::Engine*>(e)->encode_device(dframes, nseg, nframes, qmap); });
}
int tv_engine_last_recon(void* e, int b, uint8_t* y, uint8_t* u, uint8_t* v) {
  return gguard([&] {
    auto* E = static_cast<tv::gpu::Engine*>(e);
    const auto& g = E->geo();
    int lb = 0;
    auto r = E->last_recon(b, lb);
    HIP_OK(hipMemcpy(y, r.y + lb * g.ysz, g.ysz, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(u, r.u + lb * g.csz, g.csz, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(v, r.v + lb * g.csz, g.csz, hipMemcpyDeviceToHost));
  });
}
}
