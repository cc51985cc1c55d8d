// qlin_gemm.hip — fused dequant + MFMA GEMM for batched tokens (M > 64 via qlin_linear_f16), gfx950.
//
// y[M, N] = x[M, K] @ W_dq[N, K]^T (+ bias): replaces F.linear at quant/int_linear.py:62 for the
// prefill / PPL-window shapes (M = 2048 per window, main.py:127-136; M = 65,536 for batch 32).
//
// v1 structure (one 256-thread block = 4 waves in a 2x2 grid, block tile 128(M) x 128(N), BK = 128
// = one k-tile of the packed layout):
//   - A = x tile [128][128] fp16 and B = W tile [128][128] fp16 live in LDS with the 16-byte piece
//     index XOR-swizzled by (row & 15) so a 32-row fragment read is bank-conflict-free;
//   - each thread stages two lane pieces of the 8 packed row tiles (coalesced 1 KB per wave),
//     dequantizes them bit-exactly (qlin_common.h) and writes 4 x 16 B of fp16 per piece;
//   - the next K-step's global loads are issued before this step's MFMAs (register prefetch);
//   - each wave computes a 64x64 sub-tile as 2x2 v_mfma_f32_32x32x16_f16 accumulators.
#include "qlin_common.h"
#include "../../include/qlin_gfx950.h"

using namespace qlin;

namespace {

constexpr int kThreads = 256;
constexpr int64_t kSkinnyMaxM = 64;  // qlin_linear_f16: M <= this runs the GEMV kernel
constexpr int BM = 128, BN = 128, BK = kTileK;  // one k-tile of the packed layout per K-step
constexpr int kRowBytes = BK * 2;                 // 256 B per LDS row = one LDS bank row

// byte offset of 16-B piece c (0..15) of LDS row r: piece index XOR (r & 15) spreads the 16 rows
// read by a ds_read_b128 lane group over all 16 bank slots (conflict-free)
__device__ __forceinline__ int swz(int r, int c) { return r * kRowBytes + 16 * (c ^ (r & 15)); }

// the two lane pieces a thread stages per K-step: pieces tid and tid + 256 of the 8 row tiles
template <int BITS, int GPT>
struct BStage {
  Piece<BITS> c[2];
  uint32_t sz[2][GPT];  // packed (scale, zero) words, decoded at use
};

template <int BITS, int GPT>
__device__ __forceinline__ void load_b(BStage<BITS, GPT>& b, const uint32_t* __restrict__ qw,
                                       const uint32_t* __restrict__ qsz, int64_t nt0, int kt,
                                       int Kt, int N, int K, int group, int tid) {
  const int G = K / group;
  const int64_t ntl = (N + kTileN - 1) / kTileN - 1;  // last row tile that exists
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int p = tid + kThreads * h;
    const int rt = p >> 6, lane = p & 63;
    const int64_t nt = min(nt0 + rt, ntl);
    b.c[h] = load_piece<BITS>(qw + piece_off(nt, kt, Kt, lane, BITS));
#pragma unroll
    for (int i = 0; i < GPT; ++i) {
      const int g = min((kt * kTileK + 32 * (i * 4 / GPT)) / group, G - 1);
      b.sz[h][i] = qsz[sz_index(nt, g, G, lane & 15)];
    }
  }
}

template <int BITS, int GPT, bool WIDE>
__device__ __forceinline__ void store_b(unsigned char* sB, const BStage<BITS, GPT>& b, int kt,
                                        int K, int tid) {
  const Magics mg = make_magics<BITS>();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int p = tid + kThreads * h;
    const int rt = p >> 6, lane = p & 63;
    const int r = rt * kTileN + (lane & 15), q = lane >> 4;
    auto one = [&](auto S_) {
      constexpr int S = decltype(S_)::value;
      uint32_t o[4] = {0u, 0u, 0u, 0u};
      if (kt * kTileK + 32 * S < K) {
        constexpr int slot = S * GPT / 4;
        const GroupQ g = make_group<BITS, WIDE>(sz_scale(b.sz[h][slot]), sz_zero(b.sz[h][slot]));
        dequant_step<BITS, WIDE, S>(b.c[h], mg, g, o);
      }
      *reinterpret_cast<uint4*>(sB + swz(r, 4 * S + q)) = make_uint4(o[0], o[1], o[2], o[3]);
    };
    one(std::integral_constant<int, 0>{});
    one(std::integral_constant<int, 1>{});
    one(std::integral_constant<int, 2>{});
    one(std::integral_constant<int, 3>{});
  }
}

// x tile [128 rows][128 k]: 2048 16-B pieces, 8 per thread; k >= K and m >= M read as zero
__device__ __forceinline__ void load_a(uint4 (&a)[8], const _Float16* __restrict__ x, int64_t m0,
                                       int64_t M, int k0, int K, int tid) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int p = tid + kThreads * i;
    const int r = p >> 4, c = p & 15;
    const int64_t m = m0 + r;
    const int k = k0 + 8 * c;
    a[i] = (m < M && k < K) ? *reinterpret_cast<const uint4*>(x + m * K + k) : make_uint4(0, 0, 0, 0);
  }
}

__device__ __forceinline__ void store_a(unsigned char* sA, const uint4 (&a)[8], int tid) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int p = tid + kThreads * i;
    *reinterpret_cast<uint4*>(sA + swz(p >> 4, p & 15)) = a[i];
  }
}

template <int BITS, int GPT, bool WIDE>
__global__ __launch_bounds__(kThreads) void gemm_kernel(
    const uint32_t* __restrict__ qw, const uint32_t* __restrict__ qsz,
    const _Float16* __restrict__ x, const _Float16* __restrict__ bias, _Float16* __restrict__ y,
    int64_t M, int N, int K, int group, int tiles_n) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[2 * BM * kRowBytes];
  unsigned char* sA = smem;
  unsigned char* sB = smem + BM * kRowBytes;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // n-tile fastest: consecutive blocks share the x tile in L2
  const int64_t tile_m = blockIdx.x / tiles_n;
  const int tile_n = blockIdx.x - (int)(tile_m * tiles_n);
  const int64_t m0 = tile_m * BM;
  const int64_t nt0 = (int64_t)tile_n * (BN / kTileN);
  const int Kt = (K + kTileK - 1) / kTileK;

  f16v acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  uint4 a[8];
  BStage<BITS, GPT> b;
  load_a(a, x, m0, M, 0, K, tid);
  load_b<BITS, GPT>(b, qw, qsz, nt0, 0, Kt, N, K, group, tid);

  const int r32 = lane & 31, h = lane >> 5;
  for (int kt = 0; kt < Kt; ++kt) {
    __syncthreads();
    store_a(sA, a, tid);
    store_b<BITS, GPT, WIDE>(sB, b, kt, K, tid);
    __syncthreads();
    if (kt + 1 < Kt) {
      load_a(a, x, m0, M, (kt + 1) * BK, K, tid);
      load_b<BITS, GPT>(b, qw, qsz, nt0, kt + 1, Kt, N, K, group, tid);
    }
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      h8 af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        af[i] = *reinterpret_cast<const h8*>(sA + swz(wm * 64 + i * 32 + r32, kk * 2 + h));
        bf[i] = *reinterpret_cast<const h8*>(sB + swz(wn * 64 + i * 32 + r32, kk * 2 + h));
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
    const int64_t n = nt0 * kTileN + wn * 64 + j * 32 + r32;
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

template <int BITS, int GPT, bool WIDE>
int launch_gemm(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, const uint16_t* bias,
                uint16_t* y, int64_t M, int N, int K, int group, hipStream_t st) {
  const int tiles_n = (N + BN - 1) / BN;
  const int64_t tiles_m = (M + BM - 1) / BM;
  const int64_t blocks = tiles_m * tiles_n;
  if (blocks > 0x7fffffff) return QLIN_EINVAL;
  hipLaunchKernelGGL((gemm_kernel<BITS, GPT, WIDE>), dim3((unsigned)blocks), dim3(kThreads), 0, st,
                     qw, qsz, (const _Float16*)x, (const _Float16*)bias, (_Float16*)y, M, N, K,
                     group, tiles_n);
  return (int)hipGetLastError();
}

template <int BITS, bool WIDE>
int launch_gemm_g(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, const uint16_t* bias,
                  uint16_t* y, int64_t M, int N, int K, int group, hipStream_t st) {
  if (group % 128 == 0) return launch_gemm<BITS, 1, WIDE>(qw, qsz, x, bias, y, M, N, K, group, st);
  if (group % 64 == 0) return launch_gemm<BITS, 2, WIDE>(qw, qsz, x, bias, y, M, N, K, group, st);
  return launch_gemm<BITS, 4, WIDE>(qw, qsz, x, bias, y, M, N, K, group, st);
}

bool valid(int64_t M, int64_t N, int64_t K, int bits, int group) {
  return M >= 0 && N >= 0 && N <= (1 << 30) && K > 0 && K % 32 == 0 && K <= (1 << 20) &&
         group > 0 && group % 32 == 0 && K % group == 0 &&
         (bits == 2 || bits == 3 || bits == 4 || bits == 8);
}

}  // namespace

extern "C" int qlin_gemm_f16(const uint32_t* qweight, const uint32_t* qsz, int flags,
                             const uint16_t* x, const uint16_t* bias, uint16_t* y, int64_t M,
                             int64_t N, int64_t K, int bits, int group, void* workspace,
                             void* stream) {
  (void)workspace;
  if (!qweight || !qsz || !x || !y || !valid(M, N, K, bits, group)) return QLIN_EINVAL;
  if (M == 0 || N == 0) return QLIN_OK;
  hipStream_t st = (hipStream_t)stream;
  const bool wide = flags & QLIN_WIDE_ZERO;
  const int n = (int)N, k = (int)K;
#define QLIN_M(B)                                                                     \
  return wide ? launch_gemm_g<B, true>(qweight, qsz, x, bias, y, M, n, k, group, st) \
              : launch_gemm_g<B, false>(qweight, qsz, x, bias, y, M, n, k, group, st)
  switch (bits) {
    case 2: QLIN_M(2);
    case 3: QLIN_M(3);
    case 4: QLIN_M(4);
    default: QLIN_M(8);
  }
#undef QLIN_M
}

extern "C" int qlin_linear_f16(const uint32_t* qweight, const uint32_t* qsz, int flags,
                               const uint16_t* x, const uint16_t* bias, uint16_t* y, int64_t M,
                               int64_t N, int64_t K, int bits, int group, void* stream) {
  if (M == 0) return QLIN_OK;
  if (M <= kSkinnyMaxM) {
    // skinny batches: the GEMV kernel in 16-row chunks (weights re-streamed per chunk, still far
    // better parallelised than 128-row GEMM tiles for these M)
    for (int64_t m0 = 0; m0 < M; m0 += 16) {
      const int64_t mc = M - m0 < 16 ? M - m0 : 16;
      const int rc = qlin_gemv_f16(qweight, qsz, flags, x + m0 * K, bias, y + m0 * N, mc, N, K,
                                   bits, group, stream);
      if (rc) return rc;
    }
    return QLIN_OK;
  }
  return qlin_gemm_f16(qweight, qsz, flags, x, bias, y, M, N, K, bits, group, nullptr, stream);
}
