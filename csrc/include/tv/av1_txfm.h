// av1_txfm.h — AV1 transform family as exact integer basis matrices (SURVEY.md §2.3 K16:
// "AV1 transforms (DCT/ADST/identity 4-64) via MFMA").
//
//   DCT-II   N = 4..64   B[k][n] = round(4096 * c_k * cos(pi (2n+1) k / 2N)), c_0 = 1/sqrt2
//   ADST     N = 4       B[k][n] = round(4096 * sqrt2 * 2/3 * sin(pi (k+1)... )   (AV1 sinpi:
//                        1321 2482 3344 3803 — the DST-VII of AV1's av1_fadst4)
//            N = 8, 16   B[k][n] = round(4096 * sin(pi (2n+1)(2k+1) / 4N))     (AV1 DST-IV-like)
//   FLIPADST            ADST of the mirrored input
//   IDTX                4096 * sqrt(N/2) on the diagonal
//
// Every basis row has norm ~4096 * sqrt(N/2).  The 2-D forward transform is two integer
// matrix stages (columns then rows) with rounding shifts; the inverse is the transposed
// pair.  The C++ golden model (av1_txfm_ref in av1_tools.cpp) and the gfx950 MFMA kernels
// (k_av1_txfm.hip) compute the same integers.  This is the AV1 basis, not libaom's butterfly
// rounding sequence (parity with libaom unpinned).
#pragma once
#include <cmath>
#include <cstdint>

namespace tv {
namespace av1 {

enum TxType1D { TX_DCT = 0, TX_ADST = 1, TX_FLIPADST = 2, TX_IDTX = 3 };

inline int32_t txfm_basis(int type, int N, int k, int n) {
  const double pi = 3.14159265358979323846;
  if (type == TX_FLIPADST) n = N - 1 - n;
  double v;
  switch (type) {
    case TX_DCT:
      v = std::cos(pi * (2 * n + 1) * k / (2.0 * N)) * (k == 0 ? std::sqrt(0.5) : 1.0);
      break;
    case TX_ADST:
    case TX_FLIPADST:
      if (N == 4) v = std::sqrt(2.0) * 2.0 / 3.0 * std::sin(pi * (n + 1) * (2 * k + 1) / 9.0);
      else v = std::sin(pi * (2 * n + 1) * (2 * k + 1) / (4.0 * N));
      break;
    default:
      v = k == n ? std::sqrt(N / 2.0) : 0.0;
      break;
  }
  return (int32_t)std::lround(4096.0 * v);
}

inline bool txfm_valid(int type, int N) {
  if (N != 4 && N != 8 && N != 16 && N != 32 && N != 64) return false;
  if (type == TX_ADST || type == TX_FLIPADST) return N <= 16;
  return type >= 0 && type <= TX_IDTX && (type != TX_IDTX || N <= 32);
}

// Rounding shifts of the two forward stages / two inverse stages for an N x N block.  The
// forward output is ~8x the orthonormal transform (3 guard bits, like AV1's 8-bit path);
// intermediates stay within 16 bits for 9-bit residuals.
inline void txfm_shifts(int log2N, int& f1, int& f2, int& i1, int& i2) {
  f1 = 12 + (log2N - 1) / 2 - 2;   // columns: keep 2 extra bits
  f2 = 12 + log2N / 2 - 1;         // rows
  i1 = 13 + log2N / 2;             // inverse rows
  i2 = 14 + (log2N - 1) / 2;       // inverse columns back to the residual scale (f1+f2+6)
}

}  // namespace av1
}  // namespace tv
