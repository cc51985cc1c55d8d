// qlin_gemv_tile.h — per-wave tile helpers shared by the GEMV kernels (qlin_gemv.hip: single
// decode launches; qlin_gemv_batched.hip: strided batches): a tile's packed codes + (scale, zero)
// words, a lane's raw x words, and the x hand-off through the wave's LDS slot into the MFMA A
// fragments.
#pragma once

#include "qlin_common.h"

namespace {

using namespace qlin;

constexpr int kGemvMaxM = 16;  // one MFMA row block

template <int BITS, int GPT>
struct WTile {
  Piece<BITS> pc;
  uint32_t sz[GPT];  // packed (scale, zero) of each group slot, decoded only at use
};

// raw x words of one tile for MT rows: lane l holds 2*MT halfs of row l / (64/MT)
template <int MT>
struct XRaw {
  uint32_t w[MT];
};

template <int MT>
__device__ __forceinline__ void park_x(h8 (&xa)[4], const XRaw<MT>& r, uint32_t* slot, int lane,
                                       int n_in) {
  if constexpr (MT == 1) {
    slot[lane] = r.w[0];
  } else if constexpr (MT == 2) {
    *reinterpret_cast<uint2*>(slot + 2 * lane) = make_uint2(r.w[0], r.w[1]);
  } else {
#pragma unroll
    for (int c = 0; c < MT / 4; ++c)
      reinterpret_cast<uint4*>(slot + MT * lane)[c] =
          make_uint4(r.w[4 * c], r.w[4 * c + 1], r.w[4 * c + 2], r.w[4 * c + 3]);
  }
  const int m = min(n_in, MT - 1);
  const uint4* b = reinterpret_cast<const uint4*>(slot + 64 * m) + (lane >> 4);
#pragma unroll
  for (int s = 0; s < 4; ++s) xa[s] = __builtin_bit_cast(h8, b[4 * s]);
}

inline bool valid_layout(int64_t N, int64_t K, int bits, int group) {
  return N >= 0 && N <= (1 << 30) && K > 0 && K % 32 == 0 && K <= (1 << 20) && group > 0 &&
         group % 32 == 0 && K % group == 0 && (bits == 2 || bits == 3 || bits == 4 || bits == 8);
}

}  // namespace
