// k_encode.h — host-visible declarations of the encode-pipeline kernels.
#pragma once
#include <hip/hip_runtime.h>

#include "gpu_common.h"

namespace tv {
namespace gpu {

constexpr int kMaxBatch = 64;

struct FrameIdx {
  int t[kMaxBatch];  // source frame index per segment
};

// Integer rate penalties (lambda * bits) precomputed on the host exactly like the CPU
// reference encoder computes them, so GPU and CPU decisions agree.
struct Penalties {
  int mode_dcpl, mode_ang, split_intra, split_inter, pintra;
  int mv[64];
};
// Every QP's decision constants (device-resident, indexed by the per-segment slice QP of
// the frame being coded: rate control changes QP per segment and frame).
struct RcTables {
  Penalties pen[52];
  long long sao_lam16[52];
};

void launch_synth(FrameSet src, const Geo& g, uint32_t seed, const FrameIdx& fi, int B, hipStream_t s);
void launch_gather_frames(const uint8_t* frames, long seg_stride, FrameSet src, const Geo& g, int B, hipStream_t s);
// n slice QPs from host memory into device memory as kernel arguments (no blit copy)
void launch_set_qp(int8_t* dst, const int8_t* host, int n, hipStream_t s);
void launch_sse(FrameSet a, FrameSet r, const Geo& g, unsigned long long* sse, int B, hipStream_t s);
bool intra_timing();
void intra_timing_report();
void launch_intra_frame(FrameSet src, FrameSet rec, DecisionSet dec, const Geo& g, const RcTables* rc, int B,
                        hipStream_t s);
// Hierarchical motion-search state of one P frame (tv/me_model.h): quarter-res source luma
// of this and the previous frame, the previous frame's MV field (temporal candidate) and the
// per-CTB coarse field (B x nctu x 2 int16 / B x nctu int).
struct MeBuffers {
  const uint8_t* qcur;
  const uint8_t* qprev;
  const int16_t* prev_mv;
  int16_t* cmv;
  int* ccost;
};
void launch_quarter(FrameSet src, uint8_t* q, const Geo& g, int B, hipStream_t s);
// quarter-res coarse search of this frame vs the previous (penalties at the sequence QP)
void launch_coarse_me(const MeBuffers& me, const Geo& g, const RcTables* rc, int seq_qp, int range, int B,
                      hipStream_t s);
// CRF: per-segment frame QP from the lookahead complexity into qp[B]
void launch_rc_crf(const uint8_t* q, const int* ccost, int8_t* qp, const Geo& g, int crf, bool intra, int B,
                   hipStream_t s);
// Intra 16x16 CUs in P pictures (tv/me_model.h pintra_*): k_inter_me lists the quadrants
// whose inter cost passes the gate, k_pintra_analysis scores them, k_pintra_select accepts
// and lists them per reconstruction pass, k_pintra_recon codes pass q after k_inter_recon.
struct PIntraBuffers {
  int* qcost;     // [B][nctu][4] best 16x16 inter cost per quadrant
  uint8_t* cand;  // [B][nctu][4] 0x80 | mode for a candidate, else 0
  int* count;     // [6] gated, accepted of pass 0..3, candidates (zeroed per frame)
  int* gate;      // [B * nctu * 4] gated quadrant indices ((b * nctu + ctu) * 4 + q)
  int* clist;     // [B * nctu * 4] candidate quadrant indices
  int* pass;      // [4][B * nctu] accepted CTBs (b * nctu + ctu) of each pass
};
void launch_pintra_decide(FrameSet src, DecisionSet dec, const Geo& g, const RcTables* rc, const PIntraBuffers& pi,
                          int B, hipStream_t s);
void launch_pintra_recon(FrameSet src, FrameSet rec, DecisionSet dec, const Geo& g, const PIntraBuffers& pi, int B,
                         hipStream_t s);
// fine motion search + P-frame reconstruction (after launch_coarse_me); pi: intra quadrants
// (nullptr: inter only)
void launch_inter_frame(FrameSet src, FrameSet ref, const uint8_t* phase, FrameSet rec, DecisionSet dec,
                        const Geo& g, const RcTables* rc, int range, const MeBuffers& me, int B, hipStream_t s,
                        const PIntraBuffers* pi = nullptr);
// One list's fine-search result for a CTB of a B picture: the 21 ME blocks' cost (SAD +
// MV rate), rate part and vector (tv::me_ctb in the golden encoder).
struct CtbMeOut {
  int cost[21];
  int pen[21];
  int mv[21][2];
};
// B picture: fine search against both references (after both lists' launch_coarse_me), per
// block the best of L0 / L1 / their average, the CU split, then bi-predictive reconstruction.
// meout: scratch of 2 x B x nctu CtbMeOut.
void launch_inter_frame_b(FrameSet src, FrameSet ref0, const uint8_t* phase0, FrameSet ref1, const uint8_t* phase1,
                          FrameSet rec, DecisionSet dec, const Geo& g, const RcTables* rc, const int* range,
                          const MeBuffers& me0, const MeBuffers& me1, CtbMeOut* meout, int B, hipStream_t s);
// 16 quarter-pel phase planes (B x 16 x psz bytes) of the luma reference
void launch_phase_planes(FrameSet ref, uint8_t* phase, const Geo& g, int B, hipStream_t s);
void launch_deblock(FrameSet rec, DecisionSet dec, const Geo& g, int B, hipStream_t s);
// SAO: per-CTB statistics (source vs deblocked `deb`) + RD decision into `sao` (3 packed
// words per CTB, B x nctu x 3), then the filter from `deb` into `out` (every sample written).
void launch_sao(FrameSet src, FrameSet deb, FrameSet out, uint32_t* sao, const int8_t* qp, const RcTables* rc,
                const Geo& g, int B, hipStream_t s, unsigned long long* sse = nullptr);  // sse: + SSE vs src

// Compact (non-zero 4x4 groups only) level representation for the D2H transfer.
struct CompactSet {
  unsigned long long* mask_y;  // [B][nctu] luma groups (bit = sy*8 + sx within the CTB)
  unsigned* mask_c;            // [B][nctu] chroma groups (Cb bits 0..15, Cr bits 16..31)
  int* count;                  // [B][nctu]
  int* offset;                 // [B][nctu] exclusive scan of count (in groups)
  int* total;                  // [B]
  int16_t* packed;             // [B][cap] 16 levels per group
  long cap;                    // int16 capacity per segment
};
void launch_compact(DecisionSet dec, const Geo& g, CompactSet cs, int B, hipStream_t s);
// one byte per 8x8 unit for the D2H transfer: (cu_log2 - 3, or 3 for an RQT-split 32x32 CU) |
// intra << 2 | cbf << 3 | dir << 6 (dir = 1 when dec.dir is null)
void launch_pack_flags(DecisionSet dec, uint8_t* flags, const Geo& g, int B, hipStream_t s);

// ---- GPU CABAC (k_entropy.hip): WPP substreams of every slice of one picture -------------
constexpr int kEntCtx = 160;  // >= tv::CTX_COUNT (static_assert in k_entropy.hip)
// tokens per CTB region of the single binarisation pass (a CTB that needs more is binarised
// again straight into the picture's token list)
constexpr int kEntRegionTokens = 1024;
struct EntropyPic {
  int type;        // 2 I, 1 P, 0 B
  int init_type;   // cabac initType: 0 I, 1 P, 2 B
  int poc;         // B slices: POCs for the AMVP scaling
  int ref_poc[2];
  int sao, rqt, max_merge;
};
// context init states [initType][SliceQpY][ctx] (state | valMps << 6) and the coder tables
struct EntropyTables {
  uint8_t init[3][52][kEntCtx];
  uint8_t lps[256];   // rangeTabLps[state][(range >> 6) & 3]
  uint8_t tlps[64];   // transIdxLps
};
struct EntropyArgs {
  Geo g;
  EntropyPic pic;
  DecisionSet dec;      // the slot's decision planes (qp, cu_log2, intra, ipm, mv, cbf, dir, mv1, tu)
  CompactSet cs;        // the slot's compact levels (mask_y, mask_c, offset, total, packed)
  const uint32_t* sao;  // the slot's SAO parameters (nullptr: SAO off)
  // per-core binariser scratch (the entropy stream binarises one picture at a time)
  uint8_t* skip;        // [B][usz] cu_skip_flag of the unit's CU
  int8_t* midx;         // [B][usz] merge candidate matching the CU's motion (-1: none)
  int* ctb_cnt;         // [B][nctu] tokens of each CTB
  uint32_t* regions;    // [B][nctu][kEntRegionTokens] the CTBs' tokens as first written
  int* ctb_off;         // [B][nctu] exclusive scan of ctb_cnt within the segment
  int* seg_tok;         // [B] tokens of each segment
  uint32_t* tokens;     // token lists, segments back to back
  long tok_cap;
  uint8_t* stage;       // per row: 3 bytes per token + 20 (arithmetic coder output, bounded)
  int* wflag;           // [B][hc] WPP hand-off: 1 = row's contexts stored in wctx, 2 = aborted
  uint8_t* wctx;        // [B][hc][kEntCtx] contexts after CTB 1 of each row
  const EntropyTables* tab;
  // the slot's outputs (device -> host in one head copy + one payload copy)
  int* status;          // 0 ok; else the host codes this picture (capacity / consistency)
  int* seg_bytes;       // [B] payload bytes per slice
  int* row_bytes;       // [B][hc] bytes per WPP substream
  // the host slot (pinned, device-visible): the pack kernel writes the head (status,
  // seg_bytes, row_bytes -- the layout of status / seg_bytes / row_bytes above), the slice QPs
  // and the payload there directly
  int* hhead;
  int8_t* hqp;
  uint8_t* hout;
  long hout_cap;
  // TV_ENT_DEBUG: coder counters (k_ent_ac): rows, context bins, tokens, coding clocks, wait
  // ticks (100 MHz), max row span (nullptr: off)
  unsigned long long* dbg = nullptr;
};
// binarisation (merge/skip pre-pass, token count, scan, token write) and the arithmetic coder +
// payload packing, on separate streams (the second waits for the first)
void launch_entropy_bin(const EntropyArgs& a, int B, hipStream_t s);
void launch_entropy_ac(const EntropyArgs& a, int B, hipStream_t s);
void entropy_tables(EntropyTables& t);

}  // namespace gpu
}  // namespace tv
