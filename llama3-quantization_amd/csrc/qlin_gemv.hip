// qlin_gemv.hip — fused unpack + (scale, zero) dequant + GEMV for decode-sized M (1..4), gfx950,
// plus the standalone dequant kernel (parity / fake-quant eval mode).
//
// Replaces QuantLinear.forward -> F.linear(input, W_dq, bias) (quant/int_linear.py:48-65) on
// packed weights.  HBM-bound: per output row the kernel streams K*bits/8 bytes of codes plus
// K/group (fp16 scale, int zero) once, and nothing else from HBM.
//
// Decomposition (one 256-thread block = 4 waves; a wave owns RPW output rows):
//   lane l of a wave handles the lane chunks c = l + 64*j of each of its rows (chunk = 32 codes =
//   bits*4 contiguous bytes), so every weight load is a fully coalesced 64-lane x (bits*4)-byte
//   sweep of the packed row; 2 rounds (j) are kept in flight.
//   x is staged once per block into LDS (fp16, chunk-swizzled so the 16 lanes of a ds_read_b128
//   group hit 16 distinct 16-byte bank slots) and each lane reads its 64 bytes per round.
//   Dequant is the exact fp16 magic-number form (qlin_common.h); products accumulate in fp32 via
//   v_dot2_f32_f16; per-row totals by DPP row reduction + 4 readlanes.
#include "qlin_common.h"
#include "../../include/qlin_gfx950.h"

using namespace qlin;

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;

template <int BITS, bool WIDE>
struct RoundData {
  Chunk<BITS> c;
  _Float16 s;
  int z;
};

template <int BITS, bool WIDE>
__device__ __forceinline__ void load_round(RoundData<BITS, WIDE>& d, const uint32_t* __restrict__ qw,
                                           const _Float16* __restrict__ scales,
                                           const void* __restrict__ zeros, int64_t row, int c,
                                           int nch, int gpr, int cpg) {
  if (c < nch) {
    d.c = load_chunk<BITS>(qw + (row * nch + c) * BITS);
    const int64_t gi = row * gpr + c / cpg;
    d.s = scales[gi];
    if constexpr (WIDE) d.z = ((const int16_t*)zeros)[gi];
    else d.z = ((const int8_t*)zeros)[gi];
  } else {
#pragma unroll
    for (int i = 0; i < BITS; ++i) d.c.w[i] = 0;
    d.s = (_Float16)0.0f;
    d.z = 0;
  }
}

__device__ __forceinline__ int xswz(int c, int i) { return c * 64 + 16 * (i ^ ((c >> 2) & 3)); }

template <int BITS, bool WIDE, int M, int P>
__device__ __forceinline__ void dot_pair(const Chunk<BITS>& c, const GroupQ& g,
                                         const uint4 (&xv)[M][4], float (&acc)[M]) {
  const h2 w = dequant_pair<BITS, WIDE, P>(c, g);
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const uint32_t xu = (&xv[m][P >> 2].x)[P & 3];
    acc[m] = __builtin_amdgcn_fdot2(w, as_h2(xu), acc[m], false);
  }
}

template <int BITS, bool WIDE, int M>
__device__ __forceinline__ void dot_chunk(const RoundData<BITS, WIDE>& d, const uint4 (&xv)[M][4],
                                          float (&acc)[M]) {
  const GroupQ g = make_group<WIDE>(d.s, d.z);
  dot_pair<BITS, WIDE, M, 0>(d.c, g, xv, acc);
  dot_pair<BITS, WIDE, M, 1>(d.c, g, xv, acc);
  dot_pair<BITS, WIDE, M, 2>(d.c, g, xv, acc);
  dot_pair<BITS, WIDE, M, 3>(d.c, g, xv, acc);
  dot_pair<BITS, WIDE, M, 4>(d.c, g, xv, acc);
  dot_pair<BITS, WIDE, M, 5>(d.c, g, xv, acc);
  dot_pair<BITS, WIDE, M, 6>(d.c, g, xv, acc);
  dot_pair<BITS, WIDE, M, 7>(d.c, g, xv, acc);
  dot_pair<BITS, WIDE, M, 8>(d.c, g, xv, acc);
  dot_pair<BITS, WIDE, M, 9>(d.c, g, xv, acc);
  dot_pair<BITS, WIDE, M, 10>(d.c, g, xv, acc);
  dot_pair<BITS, WIDE, M, 11>(d.c, g, xv, acc);
  dot_pair<BITS, WIDE, M, 12>(d.c, g, xv, acc);
  dot_pair<BITS, WIDE, M, 13>(d.c, g, xv, acc);
  dot_pair<BITS, WIDE, M, 14>(d.c, g, xv, acc);
  dot_pair<BITS, WIDE, M, 15>(d.c, g, xv, acc);
}

template <int BITS, bool WIDE, int M, int RPW>
__global__ __launch_bounds__(kThreads) void gemv_kernel(
    const uint32_t* __restrict__ qw, const _Float16* __restrict__ scales,
    const void* __restrict__ zeros, const _Float16* __restrict__ x,
    const _Float16* __restrict__ bias, _Float16* __restrict__ y, int Mrt, int N, int K,
    int group) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int nch = K >> 5;
  const int nj = (nch + 63) >> 6;
  const int gpr = K / group;
  const int cpg = group >> 5;
  const int64_t rbase = ((int64_t)blockIdx.x * kWaves + wave) * RPW;

  // issue the first two rounds of weight loads before anything else
  RoundData<BITS, WIDE> b0[RPW], b1[RPW];
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int64_t row = min(rbase + r, (int64_t)N - 1);
    load_round<BITS, WIDE>(b0[r], qw, scales, zeros, row, lane, nch, gpr, cpg);
    load_round<BITS, WIDE>(b1[r], qw, scales, zeros, row, lane + 64, nch, gpr, cpg);
  }

  // stage x (M rows) into LDS, chunk-swizzled
  const int pieces = K >> 3;  // 16-byte pieces per x row
#pragma unroll
  for (int m = 0; m < M; ++m) {
    for (int q = tid; q < pieces; q += kThreads) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (m < Mrt) v = *reinterpret_cast<const uint4*>(x + (int64_t)m * K + q * 8);
      *reinterpret_cast<uint4*>(smem + (int64_t)m * K * 2 + xswz(q >> 2, q & 3)) = v;
    }
  }
  __syncthreads();

  float acc[RPW][M];
#pragma unroll
  for (int r = 0; r < RPW; ++r)
#pragma unroll
    for (int m = 0; m < M; ++m) acc[r][m] = 0.f;

  for (int j = 0; j < nj; j += 2) {
    {
      const int c = lane + 64 * j;
      uint4 xv[M][4];
      const int cx = min(c, nch - 1);
#pragma unroll
      for (int m = 0; m < M; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          xv[m][i] = *reinterpret_cast<const uint4*>(smem + (int64_t)m * K * 2 + xswz(cx, i));
      if (c < nch) {
#pragma unroll
        for (int r = 0; r < RPW; ++r) dot_chunk<BITS, WIDE, M>(b0[r], xv, acc[r]);
      }
#pragma unroll
      for (int r = 0; r < RPW; ++r) {
        const int64_t row = min(rbase + r, (int64_t)N - 1);
        if (j + 2 < nj) load_round<BITS, WIDE>(b0[r], qw, scales, zeros, row, lane + 64 * (j + 2), nch, gpr, cpg);
      }
    }
    if (j + 1 < nj) {
      const int c = lane + 64 * (j + 1);
      uint4 xv[M][4];
      const int cx = min(c, nch - 1);
#pragma unroll
      for (int m = 0; m < M; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          xv[m][i] = *reinterpret_cast<const uint4*>(smem + (int64_t)m * K * 2 + xswz(cx, i));
      if (c < nch) {
#pragma unroll
        for (int r = 0; r < RPW; ++r) dot_chunk<BITS, WIDE, M>(b1[r], xv, acc[r]);
      }
#pragma unroll
      for (int r = 0; r < RPW; ++r) {
        const int64_t row = min(rbase + r, (int64_t)N - 1);
        if (j + 3 < nj) load_round<BITS, WIDE>(b1[r], qw, scales, zeros, row, lane + 64 * (j + 3), nch, gpr, cpg);
      }
    }
  }

  // reduce and store
#pragma unroll
  for (int r = 0; r < RPW; ++r) {
    const int64_t row = rbase + r;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const float t = wave_sum(acc[r][m]);
      if (lane == 0 && row < N && m < Mrt) {
        const float b = bias ? (float)bias[row] : 0.f;
        y[(int64_t)m * N + row] = (_Float16)(t + b);
      }
    }
  }
}

// standalone dequant: one thread per lane chunk -> 32 fp16 values
template <int BITS, bool WIDE>
__global__ __launch_bounds__(kThreads) void dequant_kernel(
    const uint32_t* __restrict__ qw, const _Float16* __restrict__ scales,
    const void* __restrict__ zeros, _Float16* __restrict__ w, int64_t total_chunks, int K,
    int group) {
  const int64_t c = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (c >= total_chunks) return;
  const int nch = K >> 5;
  const int64_t row = c / nch;
  const int cc = (int)(c - row * nch);
  RoundData<BITS, WIDE> d;
  load_round<BITS, WIDE>(d, qw, scales, zeros, row, cc, nch, K / group, group >> 5);
  const GroupQ g = make_group<WIDE>(d.s, d.z);
  uint32_t o[16];
  o[0] = as_u32(dequant_pair<BITS, WIDE, 0>(d.c, g));
  o[1] = as_u32(dequant_pair<BITS, WIDE, 1>(d.c, g));
  o[2] = as_u32(dequant_pair<BITS, WIDE, 2>(d.c, g));
  o[3] = as_u32(dequant_pair<BITS, WIDE, 3>(d.c, g));
  o[4] = as_u32(dequant_pair<BITS, WIDE, 4>(d.c, g));
  o[5] = as_u32(dequant_pair<BITS, WIDE, 5>(d.c, g));
  o[6] = as_u32(dequant_pair<BITS, WIDE, 6>(d.c, g));
  o[7] = as_u32(dequant_pair<BITS, WIDE, 7>(d.c, g));
  o[8] = as_u32(dequant_pair<BITS, WIDE, 8>(d.c, g));
  o[9] = as_u32(dequant_pair<BITS, WIDE, 9>(d.c, g));
  o[10] = as_u32(dequant_pair<BITS, WIDE, 10>(d.c, g));
  o[11] = as_u32(dequant_pair<BITS, WIDE, 11>(d.c, g));
  o[12] = as_u32(dequant_pair<BITS, WIDE, 12>(d.c, g));
  o[13] = as_u32(dequant_pair<BITS, WIDE, 13>(d.c, g));
  o[14] = as_u32(dequant_pair<BITS, WIDE, 14>(d.c, g));
  o[15] = as_u32(dequant_pair<BITS, WIDE, 15>(d.c, g));
  uint4* dst = reinterpret_cast<uint4*>(w + c * 32);
  dst[0] = make_uint4(o[0], o[1], o[2], o[3]);
  dst[1] = make_uint4(o[4], o[5], o[6], o[7]);
  dst[2] = make_uint4(o[8], o[9], o[10], o[11]);
  dst[3] = make_uint4(o[12], o[13], o[14], o[15]);
}

bool valid_layout(int64_t N, int64_t K, int bits, int group, int zero_bits) {
  return N >= 0 && K > 0 && K % 32 == 0 && K <= (1 << 20) && group > 0 && group % 32 == 0 &&
         K % group == 0 && (bits == 2 || bits == 3 || bits == 4 || bits == 8) &&
         (zero_bits == 8 || zero_bits == 16);
}

template <int BITS, bool WIDE, int M>
int launch_gemv_m(const uint32_t* qw, const uint16_t* sc, const void* z, const uint16_t* x,
                  const uint16_t* bias, uint16_t* y, int Mrt, int N, int K, int group,
                  hipStream_t st) {
  constexpr int RPW = 2;
  const unsigned blocks = (unsigned)((N + kWaves * RPW - 1) / (kWaves * RPW));
  const size_t lds = (size_t)M * K * 2;
  if (lds > 65536) {
    static bool raised = false;  // opt in to > 64 KiB of dynamic LDS (160 KiB per CU on gfx950)
    if (!raised) {
      const hipError_t e = hipFuncSetAttribute(
          reinterpret_cast<const void*>(&gemv_kernel<BITS, WIDE, M, RPW>),
          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds > 65536 ? 163840 : 65536);
      if (e != hipSuccess) return (int)e;
      raised = true;
    }
  }
  hipLaunchKernelGGL((gemv_kernel<BITS, WIDE, M, RPW>), dim3(blocks), dim3(kThreads), lds, st, qw,
                     (const _Float16*)sc, z, (const _Float16*)x, (const _Float16*)bias,
                     (_Float16*)y, Mrt, N, K, group);
  return (int)hipGetLastError();
}

template <int BITS, bool WIDE>
int launch_gemv_b(const uint32_t* qw, const uint16_t* sc, const void* z, const uint16_t* x,
                  const uint16_t* bias, uint16_t* y, int M, int N, int K, int group,
                  hipStream_t st) {
  if (M == 1) return launch_gemv_m<BITS, WIDE, 1>(qw, sc, z, x, bias, y, M, N, K, group, st);
  if (M == 2) return launch_gemv_m<BITS, WIDE, 2>(qw, sc, z, x, bias, y, M, N, K, group, st);
  return launch_gemv_m<BITS, WIDE, 4>(qw, sc, z, x, bias, y, M, N, K, group, st);
}

}  // namespace

extern "C" int qlin_dequant_f16(const uint32_t* qweight, const uint16_t* scales,
                                const void* zeros, int zero_bits, int64_t N, int64_t K, int bits,
                                int group, uint16_t* w, void* stream) {
  if (!qweight || !scales || !zeros || !w || !valid_layout(N, K, bits, group, zero_bits))
    return QLIN_EINVAL;
  const int64_t chunks = N * (K / 32);
  if (chunks == 0) return QLIN_OK;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)((chunks + kThreads - 1) / kThreads));
#define QLIN_D(B, W)                                                                        \
  hipLaunchKernelGGL((dequant_kernel<B, W>), grid, dim3(kThreads), 0, st, qweight,          \
                     (const _Float16*)scales, zeros, (_Float16*)w, chunks, (int)K, group)
  const bool wide = zero_bits == 16;
  switch (bits) {
    case 2: if (wide) QLIN_D(2, true); else QLIN_D(2, false); break;
    case 3: if (wide) QLIN_D(3, true); else QLIN_D(3, false); break;
    case 4: if (wide) QLIN_D(4, true); else QLIN_D(4, false); break;
    default: if (wide) QLIN_D(8, true); else QLIN_D(8, false); break;
  }
#undef QLIN_D
  return (int)hipGetLastError();
}

extern "C" int qlin_gemv_f16(const uint32_t* qweight, const uint16_t* scales, const void* zeros,
                             int zero_bits, const uint16_t* x, const uint16_t* bias, uint16_t* y,
                             int64_t M, int64_t N, int64_t K, int bits, int group, void* stream) {
  if (!qweight || !scales || !zeros || !x || !y || M < 1 || M > 4 || N > (1 << 30) ||
      K > 16384 || !valid_layout(N, K, bits, group, zero_bits))
    return QLIN_EINVAL;
  if (N == 0) return QLIN_OK;
  hipStream_t st = (hipStream_t)stream;
  const bool wide = zero_bits == 16;
  const int m = (int)M, n = (int)N, k = (int)K;
#define QLIN_G(B)                                                                            \
  return wide ? launch_gemv_b<B, true>(qweight, scales, zeros, x, bias, y, m, n, k, group, st) \
              : launch_gemv_b<B, false>(qweight, scales, zeros, x, bias, y, m, n, k, group, st)
  switch (bits) {
    case 2: QLIN_G(2);
    case 3: QLIN_G(3);
    case 4: QLIN_G(4);
    default: QLIN_G(8);
  }
#undef QLIN_G
}
