// Development-only: does the order in which a block's tiles sit in HBM change how well the
// dequant VALU overlaps the weight stream?  int4 g128, M = 1, 16 waves x 2 tiles (K = 4096).
//   SC bit 0: a wave's two tiles are kt = w and w + 16 (16 KB apart) instead of 2w, 2w + 1
//   SC bit 1: wave w of block b streams row tile (b + 16 w) % Nt (a block's 16 waves read 16
//             different row tiles; output garbage, timing only)
//   MODE 0: exact dequant + MFMA; 1: loads only (xor); 2: dequant, no MFMA
#include "../../llama3-quantization_amd/csrc/qlin_common.h"
#include <type_traits>
using namespace qlin;

__device__ __forceinline__ uint64_t stamp() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

template <int SC, int MODE>
__global__ __launch_bounds__(1024) void lab2(const uint32_t* __restrict__ qw,
                                             const uint32_t* __restrict__ qsz,
                                             const _Float16* __restrict__ x,
                                             _Float16* __restrict__ y, int N, int K,
                                             uint64_t* __restrict__ stamps) {
  const uint64_t t0s = stamp();
  __shared__ __attribute__((aligned(16))) float red[16 * 16];
  __shared__ __attribute__((aligned(16))) uint32_t xs[16][2][64];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, n_in = lane & 15;
  const int Nt = N / 16, Kt = K / 128;
  int nt = blockIdx.x;
  if constexpr (SC & 2) nt = (nt + 16 * wave) % Nt;
  int kt[2];
  if constexpr (SC & 1) { kt[0] = wave; kt[1] = wave + 16; }
  else { kt[0] = 2 * wave; kt[1] = 2 * wave + 1; }
  typedef uint32_t u4v __attribute__((ext_vector_type(4)));
  Piece<4> pc[2];
  uint32_t sz[2], xr[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int64_t t = (int64_t)nt * Kt + kt[u];
    const u4v v = __builtin_nontemporal_load(reinterpret_cast<const u4v*>(qw + t * 256 + lane * 4));
    pc[u].w[0] = v.x; pc[u].w[1] = v.y; pc[u].w[2] = v.z; pc[u].w[3] = v.w;
    sz[u] = qsz[t * 16 + n_in];
    xr[u] = reinterpret_cast<const uint32_t*>(x + kt[u] * 128)[lane];
  }
  const Magics mg = make_magics<4>();
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  uint32_t xo = 0;
  uint64_t t1s = 0;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    xs[wave][u][lane] = xr[u];
    h8 xa[4];
    const uint4* b = reinterpret_cast<const uint4*>(&xs[wave][u][0]);
#pragma unroll
    for (int s = 0; s < 4; ++s) xa[s] = __builtin_bit_cast(h8, b[4 * s + (lane >> 4)]);
    if constexpr (MODE == 1) {
      xo ^= pc[u].w[0] ^ pc[u].w[1] ^ pc[u].w[2] ^ pc[u].w[3] ^ sz[u];
      xo ^= __builtin_bit_cast(uint4, xa[0]).x ^ __builtin_bit_cast(uint4, xa[3]).y;
    } else {
      const GroupQ gq = make_group_w<4, kZNarrow>(sz[u]);
      auto one = [&](auto S_) {
        constexpr int S = decltype(S_)::value;
        uint32_t v[4];
        dequant_step<4, kZNarrow, S>(pc[u], mg, gq, v);
        const h8 bb = __builtin_bit_cast(h8, make_uint4(v[0], v[1], v[2], v[3]));
        if constexpr (MODE == 0) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa[S], bb, acc, 0, 0, 0);
        else xo ^= v[0] ^ v[1] ^ v[2] ^ v[3];
      };
      one(std::integral_constant<int, 0>{});
      one(std::integral_constant<int, 1>{});
      one(std::integral_constant<int, 2>{});
      one(std::integral_constant<int, 3>{});
    }
    if (u == 0) t1s = stamp();
  }
  const uint64_t t2s = stamp();
  const float yt = MODE == 0 ? acc[0] : (float)(xo & 0xFF);
  if (lane < 16) red[n_in * 16 + wave] = yt;
  __syncthreads();
  if (tid < 16) {
    const f4* r = reinterpret_cast<const f4*>(red + tid * 16);
    const f4 a = r[0], bq = r[1], c = r[2], d = r[3];
    const f4 e = (a + bq) + (c + d);
    y[(int64_t)blockIdx.x * 16 + tid] = (_Float16)((e[0] + e[1]) + (e[2] + e[3]));
  }
  const uint64_t t3s = stamp();
  if (lane == 0 && stamps) {
    uint64_t* s = stamps + ((int64_t)blockIdx.x * 16 + wave) * 4;
    s[0] = t0s; s[1] = t1s; s[2] = t2s; s[3] = t3s;
  }
}

extern "C" int lab2_launch(const void* qw, const void* qsz, const void* x, void* y, int N, int K,
                           int SC, int MODE, void* stamps, void* st) {
  if (K != 4096 || N % 16) return 1;
#define L(S, M)                                                                                 \
  hipLaunchKernelGGL((lab2<S, M>), dim3(N / 16), dim3(1024), 0, (hipStream_t)st,               \
                     (const uint32_t*)qw, (const uint32_t*)qsz, (const _Float16*)x, (_Float16*)y, \
                     N, K, (uint64_t*)stamps)
#define LS(S) if (MODE == 0) L(S, 0); else if (MODE == 1) L(S, 1); else L(S, 2)
  if (SC == 0) { LS(0); } else if (SC == 1) { LS(1); } else if (SC == 2) { LS(2); } else { LS(3); }
#undef LS
#undef L
  return (int)hipGetLastError();
}
