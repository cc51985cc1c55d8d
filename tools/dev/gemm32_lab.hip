// Dev lab: the fused dequant GEMM on v_mfma_f32_32x32x16_f16 (an MFMA holds the SIMD's vector
// issue for 8 of its 32 cycles instead of 8 of 16 for 16x16x32: half the issue slots per flop, so
// the dequant VALU has room) with buffer LDS-DMA whose per-k-tile advance is an SGPR offset (no
// per-lane address VALU in the loop).  lab_gemm32(bn = 256 | 512), int4 / int3 / int2 narrow zeros,
// any group that is a multiple of 32, plain epilogue.
#include "../../llama3-quantization_amd/csrc/qlin_common.h"

#include <type_traits>

using namespace qlin;

namespace {

typedef __attribute__((address_space(3))) void* lds_ptr;
constexpr int BK = kTileK;

template <int BITS, int BN_, int GPT, int NW_ = 8> struct G32 {
  static constexpr int NW = NW_;
  static constexpr int BN = BN_, BM = 128;
  static constexpr int WN = BN / NW;   // 32 or 64 columns per wave
  static constexpr int NB = WN / 32;   // 32-column MFMA blocks per wave
  static constexpr int MB = BM / 32;   // 32-row MFMA blocks per wave
  static constexpr int RT = BN / kTileN;
  static constexpr int A_BYTES = BM * BK * 2;
  static constexpr int B_BYTES = RT * 256 * BITS;
  static constexpr int SZ_BYTES = RT * GPT * 64;
  static constexpr int STAGE = A_BYTES + B_BYTES + SZ_BYTES;
  static constexpr int XL = BM / (4 * NW);                 // x DMA instructions per wave
  static constexpr int QCH = RT * 16 * BITS / 64;          // code DMA instructions per block
  static constexpr int QL = (QCH + NW - 1) / NW;           // ... per wave (at most)
  static constexpr int SW = RT * GPT * 16 / 64;            // (scale, zero) DMA instructions
  static constexpr int SL = (SW + NW - 1) / NW;
};

__device__ __forceinline__ void bl16(__amdgpu_buffer_rsrc_t r, unsigned char* lds, uint32_t vo,
                                     uint32_t so) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr)lds, 16, vo, so, 0, 0);
}
__device__ __forceinline__ void bl4(__amdgpu_buffer_rsrc_t r, unsigned char* lds, uint32_t vo,
                                    uint32_t so) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr)lds, 4, vo, so, 0, 0);
}

// a buffer descriptor over [p, p + bytes) built from readfirstlane'd inputs, so the compiler sees
// it as wave-uniform (otherwise every buffer op becomes a waterfall loop)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t srd(const void* p, uint32_t bytes) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const uint32_t n = __builtin_amdgcn_readfirstlane(bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, (int)n,
                                           0x00020000);
}

template <int BITS, int BN, int GPT, int ZM, bool FULL, int NW = 8, int PRIO = 0>
__global__ __launch_bounds__(64 * NW) void gemm32_kernel(
    const uint32_t* __restrict__ qw, const uint32_t* __restrict__ qsz,
    const _Float16* __restrict__ x, _Float16* __restrict__ y, int64_t M, int N, int K, int group,
    int tiles_m, int tiles_n) {
  using C = G32<BITS, BN, GPT, NW>;
  __shared__ __attribute__((aligned(1024))) unsigned char smem[2 * C::STAGE];
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const int Kt = (K + BK - 1) / BK, G = K / group;
  const int nblk = tiles_m * tiles_n;
  const int b = blockIdx.x;
  int lb = b;
  if ((nblk & 7) == 0) lb = (b & 7) * (nblk >> 3) + (b >> 3);
  const int tile_m = lb / tiles_n, tile_n = lb - tile_m * tiles_n;
  const int64_t m0 = (int64_t)tile_m * C::BM;
  const int64_t nt0 = (int64_t)tile_n * C::RT;
  const int64_t ntiles = (N + kTileN - 1) / kTileN;
  const int tv = (int)min<int64_t>(C::RT, ntiles - nt0);   // row tiles inside N
  const int rv = (int)min<int64_t>(C::BM, M - m0);          // rows inside M

  const __amdgpu_buffer_rsrc_t rx =
      srd(x + m0 * K, (uint32_t)((int64_t)rv * K * 2));
  const __amdgpu_buffer_rsrc_t rq = srd(qw + nt0 * Kt * 64 * BITS, (uint32_t)(tv * Kt * 256 * BITS));
  const __amdgpu_buffer_rsrc_t rs = srd(qsz + nt0 * G * kTileN, (uint32_t)(tv * G * 64));

  // per-lane byte offsets, fixed for the whole K loop
  uint32_t xo[C::XL], qo[C::QL], so[C::SL];
  {
    const int sub = lane >> 4, p = lane & 15;
#pragma unroll
    for (int j = 0; j < C::XL; ++j) {
      const int r = (C::BM / C::NW) * wave + 4 * j + sub;
      const int c = p ^ (r & 15);
      xo[j] = (uint32_t)(min(r, rv - 1) * K * 2 + 16 * c);
    }
#pragma unroll
    for (int i = 0; i < C::QL; ++i) {
      const int c = 64 * (wave + C::NW * i) + lane;
      const int rt = c / (16 * BITS), o = c % (16 * BITS);
      qo[i] = (uint32_t)(min(rt, tv - 1) * Kt * 256 * BITS + 16 * o);
    }
#pragma unroll
    for (int i = 0; i < C::SL; ++i) {
      const int w = 64 * (wave + C::NW * i) + lane;
      const int rt = w / (16 * GPT), gi = (w / 16) % GPT, n = w & 15;
      so[i] = (uint32_t)(((min(rt, tv - 1) * G + gi) * kTileN + n) * 4);
    }
  }
  auto load = [&](unsigned char* st, int kt) {
#pragma unroll
    for (int j = 0; j < C::XL; ++j)
      bl16(rx, st + ((C::BM / C::NW) * wave + 4 * j) * 256, xo[j], kt * 256);
#pragma unroll
    for (int i = 0; i < C::QL; ++i)
      if (wave + C::NW * i < C::QCH)
        bl16(rq, st + C::A_BYTES + 1024 * (wave + C::NW * i), qo[i], kt * 256 * BITS);
    const int g0 = GPT == 1 ? (kt * BK) / group : kt * GPT;
#pragma unroll
    for (int i = 0; i < C::SL; ++i)
      if (wave + C::NW * i < C::SW)
        bl4(rs, st + C::A_BYTES + C::B_BYTES + 256 * (wave + C::NW * i), so[i], g0 * 64);
  };

  f16v acc[C::MB][C::NB];
#pragma unroll
  for (int i = 0; i < C::MB; ++i)
#pragma unroll
    for (int j = 0; j < C::NB; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int r = lane & 31, h = lane >> 5;
  const Magics mg = make_magics<BITS>();
  load(smem, 0);
  if (PRIO && wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  for (int kt = 0; kt < Kt; ++kt) {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (kt + 1 < Kt) load(smem + ((kt + 1) & 1) * C::STAGE, kt + 1);
    const unsigned char* st = smem + (kt & 1) * C::STAGE;
    const unsigned char* as = st;
    const uint32_t* bs = reinterpret_cast<const uint32_t*>(st + C::A_BYTES);
    const uint32_t* ss = reinterpret_cast<const uint32_t*>(st + C::A_BYTES + C::B_BYTES);
    Piece<BITS> pc[C::NB][2];
#pragma unroll
    for (int cb = 0; cb < C::NB; ++cb) {
      const int t = wave * 2 * C::NB + 2 * cb + (r >> 4);
#pragma unroll
      for (int q2 = 0; q2 < 2; ++q2)
        pc[cb][q2] = load_piece<BITS>(bs + (t * 64 + (r & 15) + 16 * (h + 2 * q2)) * BITS);
    }
    GroupQ gq[C::NB];
    auto read_groups = [&](int slot) {
#pragma unroll
      for (int cb = 0; cb < C::NB; ++cb) {
        const int t = wave * 2 * C::NB + 2 * cb + (r >> 4);
        gq[cb] = make_group_w<BITS, ZM>(ss[(t * GPT + slot) * 16 + (r & 15)]);
      }
    };
    h8 a[2][C::MB];
    auto read_a = [&](int s, h8 (&dst)[C::MB]) {
#pragma unroll
      for (int mb = 0; mb < C::MB; ++mb) {
        const int R = mb * 32 + r;
        const int c = (2 * s + h) ^ (R & 15);
        dst[mb] = *reinterpret_cast<const h8*>(as + R * 256 + c * 16);
      }
    };
    read_a(0, a[0]);
    auto step = [&](auto S_) {
      constexpr int S = decltype(S_)::value;
      if constexpr (S == 0 || (S * GPT / 8) != ((S - 1) * GPT / 8)) read_groups(S * GPT / 8);
      if constexpr (S < 7) read_a(S + 1, a[(S + 1) & 1]);
      if (!FULL && kt * BK + 16 * S >= K) return;
#pragma unroll
      for (int cb = 0; cb < C::NB; ++cb) {
        uint32_t v[4];
        dequant_step<BITS, ZM, (S >> 1)>(pc[cb][S & 1], mg, gq[cb], v);
        const h8 bf = __builtin_bit_cast(h8, make_uint4(v[0], v[1], v[2], v[3]));
#pragma unroll
        for (int mb = 0; mb < C::MB; ++mb)
          acc[mb][cb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[S & 1][mb], bf, acc[mb][cb], 0, 0, 0);
      }
    };
    step(std::integral_constant<int, 0>{});
    step(std::integral_constant<int, 1>{});
    step(std::integral_constant<int, 2>{});
    step(std::integral_constant<int, 3>{});
    step(std::integral_constant<int, 4>{});
    step(std::integral_constant<int, 5>{});
    step(std::integral_constant<int, 6>{});
    step(std::integral_constant<int, 7>{});
  }

  // lane (r, h) holds C[(e & 3) + 8 (e >> 2) + 4h][r] of each 32 x 32 block
#pragma unroll
  for (int cb = 0; cb < C::NB; ++cb) {
    const int64_t n = (nt0 + wave * 2 * C::NB + 2 * cb) * kTileN + r;
    if (n >= N) continue;
#pragma unroll
    for (int mb = 0; mb < C::MB; ++mb)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t m = m0 + mb * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (m < M) y[m * N + n] = (_Float16)acc[mb][cb][e];
      }
  }
}

template <int BITS, int BN, int GPT, int NW, int PRIO>
int launch_v(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, uint16_t* y, int64_t M,
             int N, int K, int group, hipStream_t st) {
  const int tiles_n = (N + BN - 1) / BN;
  const int tiles_m = (int)((M + 127) / 128);
  const dim3 grid((unsigned)(tiles_m * tiles_n));
  if (K % BK == 0)
    hipLaunchKernelGGL((gemm32_kernel<BITS, BN, GPT, kZNarrow, true, NW, PRIO>), grid, dim3(64 * NW),
                       0, st, qw, qsz, (const _Float16*)x, (_Float16*)y, M, N, K, group, tiles_m,
                       tiles_n);
  else
    hipLaunchKernelGGL((gemm32_kernel<BITS, BN, GPT, kZNarrow, false, NW, PRIO>), grid,
                       dim3(64 * NW), 0, st, qw, qsz, (const _Float16*)x, (_Float16*)y, M, N, K,
                       group, tiles_m, tiles_n);
  return (int)hipGetLastError();
}
int g_variant = 0;  // lab: 0 = 8 waves, 1 = 8 waves + setprio for waves 4-7, 2 = 4 waves (BN 512)
template <int BITS, int BN, int GPT>
int launch(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, uint16_t* y, int64_t M,
           int N, int K, int group, hipStream_t st) {
  if (g_variant == 1) return launch_v<BITS, BN, GPT, 8, 1>(qw, qsz, x, y, M, N, K, group, st);
  if (g_variant == 2 && BN == 512) return launch_v<BITS, BN, GPT, 4, 0>(qw, qsz, x, y, M, N, K, group, st);
  return launch_v<BITS, BN, GPT, 8, 0>(qw, qsz, x, y, M, N, K, group, st);
}

template <int BITS, int BN>
int launch_g(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, uint16_t* y, int64_t M,
             int N, int K, int group, hipStream_t st) {
  if (group % 128 == 0) return launch<BITS, BN, 1>(qw, qsz, x, y, M, N, K, group, st);
  if (group % 64 == 0) return launch<BITS, BN, 2>(qw, qsz, x, y, M, N, K, group, st);
  return launch<BITS, BN, 4>(qw, qsz, x, y, M, N, K, group, st);
}

}  // namespace

extern "C" void lab_gemm32_variant(int v) { g_variant = v; }

extern "C" int lab_gemm32(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, uint16_t* y,
                          int64_t M, int N, int K, int bits, int group, int bn, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (bits == 4)
    return bn == 512 ? launch_g<4, 512>(qw, qsz, x, y, M, N, K, group, st)
                     : launch_g<4, 256>(qw, qsz, x, y, M, N, K, group, st);
  if (bits == 3)
    return bn == 512 ? launch_g<3, 512>(qw, qsz, x, y, M, N, K, group, st)
                     : launch_g<3, 256>(qw, qsz, x, y, M, N, K, group, st);
  return bn == 512 ? launch_g<2, 512>(qw, qsz, x, y, M, N, K, group, st)
                   : launch_g<2, 256>(qw, qsz, x, y, M, N, K, group, st);
}
