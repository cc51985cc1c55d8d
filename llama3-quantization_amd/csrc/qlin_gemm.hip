// qlin_gemm.hip — fused dequant + MFMA GEMM for batched tokens (M > 4), gfx950.
//
// y[M, N] = x[M, K] @ W_dq[N, K]^T (+ bias): replaces F.linear at quant/int_linear.py:62 for the
// prefill / PPL-window shapes (M = 2048 per window, main.py:127-136; M = 65,536 for batch 32).
//
// v1 structure (one 256-thread block = 4 waves in a 2x2 grid, block tile 128(M) x 128(N), BK = 64):
//   - A = x tile [128][64] fp16 and B = W tile [128][64] fp16 live in LDS with the 16-byte piece
//     index XOR-swizzled by (row & 7) so a 32-row fragment read spreads over the bank row;
//   - each thread owns one 32-code lane chunk of the W tile: it loads bits*4 bytes of packed codes
//     and one (scale, zero), dequantizes bit-exactly (qlin_common.h) and writes 64 bytes of fp16;
//   - the next K-step's global loads are issued before this step's MFMAs (register prefetch);
//   - each wave computes a 64x64 sub-tile as 2x2 v_mfma_f32_32x32x16_f16 accumulators.
#include "qlin_common.h"
#include "../../include/qlin_gfx950.h"

using namespace qlin;

namespace {

constexpr int kThreads = 256;
constexpr int BM = 128, BN = 128, BK = 64;
constexpr int kRowBytes = BK * 2;  // 128 B per LDS row

__device__ __forceinline__ int swz(int row, int piece) {  // byte offset of 16-B piece in a tile
  return row * kRowBytes + 16 * (piece ^ (row & 7));
}

template <int BITS, bool WIDE>
struct BStage {
  Chunk<BITS> c;
  _Float16 s;
  int z;
};

template <int BITS, bool WIDE>
__device__ __forceinline__ void load_b(BStage<BITS, WIDE>& b, const uint32_t* __restrict__ qw,
                                       const _Float16* __restrict__ scales,
                                       const void* __restrict__ zeros, int64_t n, int N, int k0,
                                       int K, int group, int tid) {
  // tile row = tid / 2, chunk within BK = tid & 1
  const int r = tid >> 1;
  const int kc = (k0 >> 5) + (tid & 1);
  const int64_t row = min(n + r, (int64_t)N - 1);
  const int nch = K >> 5;
  b.c = load_chunk<BITS>(qw + (row * nch + kc) * BITS);
  const int64_t gi = row * (K / group) + (kc * 32) / group;
  b.s = scales[gi];
  if constexpr (WIDE) b.z = ((const int16_t*)zeros)[gi];
  else b.z = ((const int8_t*)zeros)[gi];
}

__device__ __forceinline__ void load_a(uint4 (&a)[4], const _Float16* __restrict__ x, int64_t m0,
                                       int64_t M, int k0, int K, int tid) {
  // 128 rows x 8 pieces = 1024 pieces; thread handles pieces tid + 256*i
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int p = tid + kThreads * i;
    const int r = p >> 3, pc = p & 7;
    const int64_t m = m0 + r;
    a[i] = m < M ? *reinterpret_cast<const uint4*>(x + m * K + k0 + pc * 8) : make_uint4(0, 0, 0, 0);
  }
}

template <int BITS, bool WIDE>
__device__ __forceinline__ void store_b(unsigned char* sB, const BStage<BITS, WIDE>& b, int tid) {
  const GroupQ g = make_group<WIDE>(b.s, b.z);
  const int r = tid >> 1;
  const int pbase = (tid & 1) * 4;  // 4 pieces of 8 halfs
  uint32_t o[16];
  o[0] = as_u32(dequant_pair<BITS, WIDE, 0>(b.c, g));
  o[1] = as_u32(dequant_pair<BITS, WIDE, 1>(b.c, g));
  o[2] = as_u32(dequant_pair<BITS, WIDE, 2>(b.c, g));
  o[3] = as_u32(dequant_pair<BITS, WIDE, 3>(b.c, g));
  o[4] = as_u32(dequant_pair<BITS, WIDE, 4>(b.c, g));
  o[5] = as_u32(dequant_pair<BITS, WIDE, 5>(b.c, g));
  o[6] = as_u32(dequant_pair<BITS, WIDE, 6>(b.c, g));
  o[7] = as_u32(dequant_pair<BITS, WIDE, 7>(b.c, g));
  o[8] = as_u32(dequant_pair<BITS, WIDE, 8>(b.c, g));
  o[9] = as_u32(dequant_pair<BITS, WIDE, 9>(b.c, g));
  o[10] = as_u32(dequant_pair<BITS, WIDE, 10>(b.c, g));
  o[11] = as_u32(dequant_pair<BITS, WIDE, 11>(b.c, g));
  o[12] = as_u32(dequant_pair<BITS, WIDE, 12>(b.c, g));
  o[13] = as_u32(dequant_pair<BITS, WIDE, 13>(b.c, g));
  o[14] = as_u32(dequant_pair<BITS, WIDE, 14>(b.c, g));
  o[15] = as_u32(dequant_pair<BITS, WIDE, 15>(b.c, g));
#pragma unroll
  for (int i = 0; i < 4; ++i)
    *reinterpret_cast<uint4*>(sB + swz(r, pbase + i)) =
        make_uint4(o[4 * i], o[4 * i + 1], o[4 * i + 2], o[4 * i + 3]);
}

__device__ __forceinline__ void store_a(unsigned char* sA, const uint4 (&a)[4], int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int p = tid + kThreads * i;
    *reinterpret_cast<uint4*>(sA + swz(p >> 3, p & 7)) = a[i];
  }
}

template <int BITS, bool WIDE>
__global__ __launch_bounds__(kThreads) void gemm_kernel(
    const uint32_t* __restrict__ qw, const _Float16* __restrict__ scales,
    const void* __restrict__ zeros, const _Float16* __restrict__ x,
    const _Float16* __restrict__ bias, _Float16* __restrict__ y, int64_t M, int N, int K,
    int group, int tiles_n) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * BM * kRowBytes];
  unsigned char* sA = smem;
  unsigned char* sB = smem + BM * kRowBytes;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // n-tile fastest: consecutive blocks share the x tile
  const int64_t tile_m = blockIdx.x / tiles_n;
  const int tile_n = blockIdx.x - (int)(tile_m * tiles_n);
  const int64_t m0 = tile_m * BM;
  const int64_t n0 = (int64_t)tile_n * BN;

  f16v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  uint4 a[4];
  BStage<BITS, WIDE> b;
  load_a(a, x, m0, M, 0, K, tid);
  load_b<BITS, WIDE>(b, qw, scales, zeros, n0, N, 0, K, group, tid);

  const int nk = K / BK;
  const int r32 = lane & 31, h = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    __syncthreads();
    store_a(sA, a, tid);
    store_b<BITS, WIDE>(sB, b, tid);
    __syncthreads();
    if (kt + 1 < nk) {
      load_a(a, x, m0, M, (kt + 1) * BK, K, tid);
      load_b<BITS, WIDE>(b, qw, scales, zeros, n0, N, (kt + 1) * BK, K, group, tid);
    }
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      h8 af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int ra = wm * 64 + i * 32 + r32;
        af[i] = *reinterpret_cast<const h8*>(sA + swz(ra, kk * 2 + h));
        const int rb = wn * 64 + i * 32 + r32;
        bf[i] = *reinterpret_cast<const h8*>(sB + swz(rb, kk * 2 + h));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af[i], bf[j], acc[i][j], 0, 0, 0);
    }
  }

  // epilogue: C/D layout col = lane & 31, row = (e & 3) + 8 * (e >> 2) + 4 * (lane >> 5)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int64_t n = n0 + wn * 64 + j * 32 + r32;
    if (n >= N) continue;
    const float bv = bias ? (float)bias[n] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t m = m0 + wm * 64 + i * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (m < M) y[m * N + n] = (_Float16)(acc[i][j][e] + bv);
      }
    }
  }
}

template <int BITS, bool WIDE>
int launch_gemm(const uint32_t* qw, const uint16_t* sc, const void* z, const uint16_t* x,
                const uint16_t* bias, uint16_t* y, int64_t M, int N, int K, int group,
                hipStream_t st) {
  const int tiles_n = (N + BN - 1) / BN;
  const int64_t tiles_m = (M + BM - 1) / BM;
  const int64_t blocks = tiles_m * tiles_n;
  if (blocks > 0x7fffffff) return QLIN_EINVAL;
  hipLaunchKernelGGL((gemm_kernel<BITS, WIDE>), dim3((unsigned)blocks), dim3(kThreads), 0, st, qw,
                     (const _Float16*)sc, z, (const _Float16*)x, (const _Float16*)bias,
                     (_Float16*)y, M, N, K, group, tiles_n);
  return (int)hipGetLastError();
}

bool valid(int64_t M, int64_t N, int64_t K, int bits, int group, int zero_bits) {
  return M >= 0 && N >= 0 && N <= (1 << 30) && K > 0 && K % BK == 0 && K <= (1 << 20) &&
         group > 0 && group % 32 == 0 && K % group == 0 &&
         (bits == 2 || bits == 3 || bits == 4 || bits == 8) && (zero_bits == 8 || zero_bits == 16);
}

}  // namespace

extern "C" int qlin_gemm_f16(const uint32_t* qweight, const uint16_t* scales, const void* zeros,
                             int zero_bits, const uint16_t* x, const uint16_t* bias, uint16_t* y,
                             int64_t M, int64_t N, int64_t K, int bits, int group,
                             void* workspace, void* stream) {
  (void)workspace;
  if (!qweight || !scales || !zeros || !x || !y || !valid(M, N, K, bits, group, zero_bits))
    return QLIN_EINVAL;
  if (M == 0 || N == 0) return QLIN_OK;
  hipStream_t st = (hipStream_t)stream;
  const bool wide = zero_bits == 16;
  const int n = (int)N, k = (int)K;
#define QLIN_M(B)                                                                            \
  return wide ? launch_gemm<B, true>(qweight, scales, zeros, x, bias, y, M, n, k, group, st) \
              : launch_gemm<B, false>(qweight, scales, zeros, x, bias, y, M, n, k, group, st)
  switch (bits) {
    case 2: QLIN_M(2);
    case 3: QLIN_M(3);
    case 4: QLIN_M(4);
    default: QLIN_M(8);
  }
#undef QLIN_M
}

extern "C" int qlin_linear_f16(const uint32_t* qweight, const uint16_t* scales, const void* zeros,
                               int zero_bits, const uint16_t* x, const uint16_t* bias,
                               uint16_t* y, int64_t M, int64_t N, int64_t K, int bits, int group,
                               void* stream) {
  if (M <= 4 && K <= 16384)
    return qlin_gemv_f16(qweight, scales, zeros, zero_bits, x, bias, y, M, N, K, bits, group,
                         stream);
  return qlin_gemm_f16(qweight, scales, zeros, zero_bits, x, bias, y, M, N, K, bits, group,
                       nullptr, stream);
}
