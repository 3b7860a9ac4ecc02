// bench_av1w.cpp — single-thread timing (and gprof target) of the AV1 OBU writer on dumped
// engine decisions: tools/av1_writer_bench.py --dump FILE writes them.
//   g++ -O2 -pg -std=c++17 -Icsrc/include tools/native/bench_av1w.cpp csrc/core/*.cpp -o /tmp/bench_av1w
//   /tmp/bench_av1w FILE [reps]; gprof /tmp/bench_av1w gmon.out
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

extern "C" {
void* tv_av1c_state_new();
void tv_av1c_state_free(void* s);
int tv_av1c_write_tu(void* state, int dw, int dh, const int* fparams, const uint32_t* mode, const uint32_t* mv,
                     const int16_t* ly, const int16_t* lu, const int16_t* lv, const int8_t* cdef_idx, const int32_t* lr,
                     int packed, int seq_header, void* out);
}

template <class T> std::vector<T> rd(FILE* f) {
  int64_t n = 0;
  if (fread(&n, 8, 1, f) != 1) exit(2);
  std::vector<T> v((size_t)n);
  if (n && fread(v.data(), sizeof(T), (size_t)n, f) != (size_t)n) exit(2);
  return v;
}

int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "rb");
  const int reps = argc > 2 ? atoi(argv[2]) : 10;
  int hdr[3];
  if (fread(hdr, 4, 3, f) != 3) return 2;
  struct Fr {
    std::vector<int32_t> fp, lr;
    std::vector<uint32_t> mode, mv;
    std::vector<int16_t> l[3];
    std::vector<int8_t> cdef;
  };
  std::vector<Fr> fr(hdr[2]);
  for (auto& x : fr) {
    x.fp = rd<int32_t>(f);
    x.mode = rd<uint32_t>(f);
    x.mv = rd<uint32_t>(f);
    for (auto& l : x.l) l = rd<int16_t>(f);
    x.cdef = rd<int8_t>(f);
    x.lr = rd<int32_t>(f);
  }
  std::vector<double> best(fr.size(), 1e9);
  std::vector<uint8_t> out;
  for (int r = 0; r < reps; ++r) {
    void* st = tv_av1c_state_new();
    for (size_t i = 0; i < fr.size(); ++i) {
      out.clear();
      const auto t0 = std::chrono::steady_clock::now();
      if (tv_av1c_write_tu(st, hdr[0], hdr[1], fr[i].fp.data(), fr[i].mode.data(), fr[i].mv.data(), fr[i].l[0].data(),
                           fr[i].l[1].data(), fr[i].l[2].data(), fr[i].cdef.data(), fr[i].lr.data(), 2, i == 0,
                           &out) != 0)
        return 3;
      best[i] = std::min(best[i], std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
    }
    tv_av1c_state_free(st);
  }
  for (size_t i = 0; i < fr.size(); ++i) printf("frame %zu: %.2f ms\n", i, best[i]);
  return 0;
}
