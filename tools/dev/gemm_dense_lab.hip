// Dev lab (not product): the large-M GEMM as a bit-exact dequant pre-pass into the MFMA B-fragment
// layout plus a dense-B MFMA GEMM.  int4 g128 narrow zeros only.
//
// Pre-pass: W_dq fragments Wf[nt][ks][lane][8 halfs] (nt: 16-row tile, ks: 32-deep k-step) =
// exactly the B operand lane `lane` feeds v_mfma_f32_16x16x32_f16 for that tile and step, formed
// by the product's exact dequant (qlin_common.h dequant_step).
// GEMM: 256 x 256 block, BK = 64 (two k-steps), 8 waves as 2 (M) x 4 (N), wave tile 128 x 64,
// A (x) and B (fragments) by LDS-DMA into two stages, one barrier per k-step; each output is one
// MFMA chain in k order, as the fused kernel's: the same bits.
#include "../../llama3-quantization_amd/csrc/qlin_common.h"

#include <type_traits>

using namespace qlin;

namespace {

typedef __attribute__((address_space(3))) void* lds_ptr;
typedef __attribute__((address_space(1))) void* gbl_ptr;

__device__ __forceinline__ void glds16(const void* g, unsigned char* lds) {
  __builtin_amdgcn_global_load_lds((gbl_ptr)g, (lds_ptr)lds, 16, 0, 0);
}

template <int BITS, int ZM>
__global__ __launch_bounds__(256) void dequant_frag_kernel(const uint32_t* __restrict__ qw,
                                                           const uint32_t* __restrict__ qsz,
                                                           uint4* __restrict__ wf, int64_t pieces,
                                                           int Kt, int G) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;  // (nt, kt, lane)
  if (p >= pieces) return;
  const int lane = (int)(p & 63);
  const int64_t t = p >> 6;  // tile index nt * Kt + kt
  const int64_t nt = t / Kt;
  const int kt = (int)(t - nt * Kt);
  const Piece<BITS> pc = load_piece_nt<BITS>(qw + p * BITS);
  const uint32_t sw = qsz[(nt * G + kt) * kTileN + (lane & 15)];  // g128: group = kt
  const Magics mg = make_magics<BITS>();
  const GroupQ gq = make_group_w<BITS, ZM>(sw);
  uint4* out = wf + ((t * 4) * 64 + lane);
  auto step = [&](auto S_) {
    constexpr int S = decltype(S_)::value;
    uint32_t v[4];
    dequant_step<BITS, ZM, S>(pc, mg, gq, v);
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 val = {v[0], v[1], v[2], v[3]};
    __builtin_nontemporal_store(val, reinterpret_cast<u32x4*>(out + S * 64));
  };
  step(std::integral_constant<int, 0>{});
  step(std::integral_constant<int, 1>{});
  step(std::integral_constant<int, 2>{});
  step(std::integral_constant<int, 3>{});
}

constexpr int BM = 256, BN = 256, BKD = 64, NW = 8;
constexpr int A_BYTES = BM * BKD * 2;          // 32 KB
constexpr int B_BYTES = (BN / 16) * 2 * 1024;  // 32 KB: 16 tiles x 2 k-steps x 1 KB
constexpr int STAGE = A_BYTES + B_BYTES;
constexpr int MB = 8, NB = 4;                  // wave tile 128 x 64

struct DArgs {
  const _Float16* x;
  const uint4* wf;
  _Float16* y;
  int64_t M;
  int N, K, KS, Nt;  // KS: k-steps per row tile (K / 32)
  int tiles_m, tiles_n;
};

__device__ __forceinline__ void load_stage(unsigned char* st, const DArgs& a, int64_t m0,
                                           int nt0, int kk, int wave, int lane) {
  // A: 256 rows x 8 chunks of 16 B; one instruction = 8 rows; physical chunk p of row r holds
  // logical chunk p ^ (r & 7)
#pragma unroll
  for (int j = 0; j < BM / (8 * NW); ++j) {
    const int r = (BM / NW) * wave + 8 * j + (lane >> 3);
    const int c = (lane & 7) ^ (r & 7);
    const int64_t m = min(m0 + r, a.M - 1);
    glds16(a.x + m * a.K + (int64_t)kk * BKD + 8 * c, st + ((BM / NW) * wave + 8 * j) * 128);
  }
  // B: 16 tiles x 2 k-steps, 1 KB each, contiguous fragments
  unsigned char* bs = st + A_BYTES;
#pragma unroll
  for (int j = wave; j < 32; j += NW) {
    const int tl = j >> 1, s = j & 1;
    const int nt = min(nt0 + tl, a.Nt - 1);
    glds16(a.wf + ((int64_t)nt * a.KS + 2 * kk + s) * 64 + lane, bs + 1024 * j);
  }
}

__global__ __launch_bounds__(512) void gemm_dense_kernel(const DArgs a) {
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * STAGE];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, n_in = lane & 15, q = lane >> 4;
  const int nblk = a.tiles_m * a.tiles_n;
  const int b = blockIdx.x;
  int lb = b;
  if ((nblk & 7) == 0) lb = (b & 7) * (nblk >> 3) + (b >> 3);
  const int tile_m = lb / a.tiles_n, tile_n = lb - tile_m * a.tiles_n;
  const int64_t m0 = (int64_t)tile_m * BM;
  const int nt0 = tile_n * (BN / 16);
  const int wm = wave >> 2, wn = wave & 3;
  f4 acc[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  const int nk = a.K / BKD;
  load_stage(smem, a, m0, nt0, 0, wave, lane);
  for (int kk = 0; kk < nk; ++kk) {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (kk + 1 < nk) load_stage(smem + ((kk + 1) & 1) * STAGE, a, m0, nt0, kk + 1, wave, lane);
    const unsigned char* as = smem + (kk & 1) * STAGE;
    const unsigned char* bs = as + A_BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      h8 bf[NB], af[MB];
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
        bf[nb] = *reinterpret_cast<const h8*>(bs + (((wn * NB + nb) * 2 + s) * 64 + lane) * 16);
#pragma unroll
      for (int mb = 0; mb < MB; ++mb) {
        const int r = wm * 128 + mb * 16 + n_in;
        const int c = (4 * s + q) ^ (r & 7);
        af[mb] = *reinterpret_cast<const h8*>(as + r * 128 + c * 16);
      }
#pragma unroll
      for (int nb = 0; nb < NB; ++nb)
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
          acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[mb], bf[nb], acc[mb][nb], 0, 0, 0);
    }
  }
  // epilogue: plain fp16 output (lab)
  const int64_t wrow0 = m0 + wm * 128;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int n = (nt0 + wn * NB + nb) * 16 + n_in;
    if (n >= a.N) continue;
#pragma unroll
    for (int mb = 0; mb < MB; ++mb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t m = wrow0 + mb * 16 + 4 * q + i;
        if (m < a.M) a.y[m * a.N + n] = (_Float16)acc[mb][nb][i];
      }
  }
}

}  // namespace

extern "C" int lab_dequant_frag(const uint32_t* qw, const uint32_t* qsz, void* wf, int N, int K,
                                void* stream) {
  const int Nt = (N + 15) / 16, Kt = K / 128;
  const int64_t pieces = (int64_t)Nt * Kt * 64;
  (void)hipGetLastError();
  hipLaunchKernelGGL((dequant_frag_kernel<4, kZNarrow>), dim3((unsigned)((pieces + 255) / 256)),
                     dim3(256), 0, (hipStream_t)stream, qw, qsz, (uint4*)wf, pieces, Kt, K / 128);
  return (int)hipGetLastError();
}

extern "C" int lab_gemm_dense(const uint16_t* x, const void* wf, uint16_t* y, int64_t M, int N,
                              int K, void* stream) {
  if (K % 128) return -1;
  DArgs a;
  a.x = (const _Float16*)x;
  a.wf = (const uint4*)wf;
  a.y = (_Float16*)y;
  a.M = M;
  a.N = N;
  a.K = K;
  a.KS = K / 32;
  a.Nt = (N + 15) / 16;
  a.tiles_m = (int)((M + BM - 1) / BM);
  a.tiles_n = (N + BN - 1) / BN;
  (void)hipGetLastError();
  hipLaunchKernelGGL(gemm_dense_kernel, dim3((unsigned)(a.tiles_m * a.tiles_n)), dim3(512), 0,
                     (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

// ---- variant 3: 256 x 128 blocks, three LDS stages, one k-step of DMA in flight across the
// barrier (counted vmcnt, raw s_barrier), 8 waves as 4 (M) x 2 (N), wave tile 64 x 64
namespace {
constexpr int BM3 = 256, BN3 = 128;
constexpr int A3 = BM3 * BKD * 2;          // 32 KB
constexpr int B3 = (BN3 / 16) * 2 * 1024;  // 16 KB
constexpr int STAGE3 = A3 + B3;            // 48 KB
constexpr int MB3 = 4, NB3 = 4;
constexpr int LPS = BM3 / (8 * NW) + (BN3 / 16 * 2) / NW;  // glds per wave per stage: 4 + 2

__device__ __forceinline__ void load_stage3(unsigned char* st, const DArgs& a, int64_t m0, int nt0,
                                            int kk, int wave, int lane) {
#pragma unroll
  for (int j = 0; j < BM3 / (8 * NW); ++j) {
    const int r = (BM3 / NW) * wave + 8 * j + (lane >> 3);
    const int c = (lane & 7) ^ (r & 7);
    const int64_t m = min(m0 + r, a.M - 1);
    glds16(a.x + m * a.K + (int64_t)kk * BKD + 8 * c, st + ((BM3 / NW) * wave + 8 * j) * 128);
  }
  unsigned char* bs = st + A3;
#pragma unroll
  for (int j = wave; j < BN3 / 16 * 2; j += NW) {
    const int tl = j >> 1, s = j & 1;
    const int nt = min(nt0 + tl, a.Nt - 1);
    glds16(a.wf + ((int64_t)nt * a.KS + 2 * kk + s) * 64 + lane, bs + 1024 * j);
  }
}

__global__ __launch_bounds__(512) void gemm_dense3_kernel(const DArgs a) {
  __shared__ __attribute__((aligned(1024))) unsigned char smem[3 * STAGE3];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63, n_in = lane & 15, q = lane >> 4;
  const int nblk = a.tiles_m * a.tiles_n;
  const int b = blockIdx.x;
  int lb = b;
  if ((nblk & 7) == 0) lb = (b & 7) * (nblk >> 3) + (b >> 3);
  const int tile_m = lb / a.tiles_n, tile_n = lb - tile_m * a.tiles_n;
  const int64_t m0 = (int64_t)tile_m * BM3;
  const int nt0 = tile_n * (BN3 / 16);
  const int wm = wave >> 1, wn = wave & 1;
  f4 acc[MB3][NB3];
#pragma unroll
  for (int i = 0; i < MB3; ++i)
#pragma unroll
    for (int j = 0; j < NB3; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  const int nk = a.K / BKD;  // >= 2
  load_stage3(smem, a, m0, nt0, 0, wave, lane);
  load_stage3(smem + STAGE3, a, m0, nt0, 1, wave, lane);
  int buf = 0;
  for (int kk = 0; kk < nk; ++kk) {
    if (kk + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LPS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (kk + 2 < nk) {
      const int nb2 = buf == 0 ? 2 : buf - 1;  // (kk + 2) % 3
      load_stage3(smem + nb2 * STAGE3, a, m0, nt0, kk + 2, wave, lane);
    }
    const unsigned char* as = smem + buf * STAGE3;
    const unsigned char* bs = as + A3;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      h8 bf[NB3], af[MB3];
#pragma unroll
      for (int nb = 0; nb < NB3; ++nb)
        bf[nb] = *reinterpret_cast<const h8*>(bs + (((wn * NB3 + nb) * 2 + s) * 64 + lane) * 16);
#pragma unroll
      for (int mb = 0; mb < MB3; ++mb) {
        const int r = wm * 64 + mb * 16 + n_in;
        const int c = (4 * s + q) ^ (r & 7);
        af[mb] = *reinterpret_cast<const h8*>(as + r * 128 + c * 16);
      }
#pragma unroll
      for (int nb = 0; nb < NB3; ++nb)
#pragma unroll
        for (int mb = 0; mb < MB3; ++mb)
          acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[mb], bf[nb], acc[mb][nb], 0, 0, 0);
    }
    buf = buf == 2 ? 0 : buf + 1;
  }
  const int64_t wrow0 = m0 + wm * 64;
#pragma unroll
  for (int nb = 0; nb < NB3; ++nb) {
    const int n = (nt0 + wn * NB3 + nb) * 16 + n_in;
    if (n >= a.N) continue;
#pragma unroll
    for (int mb = 0; mb < MB3; ++mb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t m = wrow0 + mb * 16 + 4 * q + i;
        if (m < a.M) a.y[m * a.N + n] = (_Float16)acc[mb][nb][i];
      }
  }
}
}  // namespace

extern "C" int lab_gemm_dense3(const uint16_t* x, const void* wf, uint16_t* y, int64_t M, int N,
                               int K, void* stream) {
  if (K % 128) return -1;
  DArgs a;
  a.x = (const _Float16*)x;
  a.wf = (const uint4*)wf;
  a.y = (_Float16*)y;
  a.M = M;
  a.N = N;
  a.K = K;
  a.KS = K / 32;
  a.Nt = (N + 15) / 16;
  a.tiles_m = (int)((M + BM3 - 1) / BM3);
  a.tiles_n = (N + BN3 - 1) / BN3;
  (void)hipGetLastError();
  hipLaunchKernelGGL(gemm_dense3_kernel, dim3((unsigned)(a.tiles_m * a.tiles_n)), dim3(512), 0,
                     (hipStream_t)stream, a);
  return (int)hipGetLastError();
}
