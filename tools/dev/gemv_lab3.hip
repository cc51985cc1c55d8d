// Development-only: where the GEMV's compute sits against the weight stream.  int4 g128, M = 1,
// K = 4096, one block per 16-row tile, 16 waves x 2 tiles (kt = w and w + 16).
//   V 0: exact dequant + MFMA, per-tile sz / x loads (gemv_lab2 SC = 1)
//   V 1: as 0 with one sz load (lanes 0-31) and one 8-B x load per wave for both tiles
//   V 2: as 1, VALU v_dot2_f32_f16 instead of the MFMA (lane partials summed over q by DPP)
//   V 3: as 1, four independent MFMA accumulators per wave
//   V 4: as 1, scale after accumulate (NOT exact: (u - z) x summed per group, times s)
//   V 5: as 1, the dequant + MFMA run on constant codes while the loads are in flight; the loaded
//        words are only xor-folded at the end (what overlapping the compute with the wait costs)
//   V 6: as 1, loads only (the loaded words xor-folded; nothing else)
//   V 7 / 8 / 9: V 0 / 5 / 6 with s_setprio 3 until the wave's loads are issued, then 0
//   V 10: V 0 with s_setprio 3 around the load issue and 1 for the tile-1 compute
//   V 11: V 0 with the dequant + MFMA of both tiles run 3 times (a rolled loop: same code,
//         warm instruction cache, data already in registers for passes 2 and 3)
//   V 12: V 6 (loads only) with ~1000 bytes of never-executed code between its instructions
//   V 13: V 0 with the block's whole x row staged in LDS once (one 16-B load per thread of waves
//         0-7, one barrier) instead of one x load + LDS park per tile
#include "../../llama3-quantization_amd/csrc/qlin_common.h"
#include <type_traits>
using namespace qlin;

template <int V0>
__global__ __launch_bounds__(1024) void lab3(const uint32_t* __restrict__ qw,
                                             const uint32_t* __restrict__ qsz,
                                             const _Float16* __restrict__ x,
                                             _Float16* __restrict__ y, int N, int K) {
  constexpr int V = V0 == 7 || V0 == 10 || V0 == 11 || V0 == 13 ? 0 : V0 == 8 ? 5 : V0 == 9 || V0 == 12 ? 6 : V0;
  constexpr bool PRIO = V0 >= 7 && V0 <= 12;
  if constexpr (PRIO) __builtin_amdgcn_s_setprio(3);
  __shared__ __attribute__((aligned(16))) float red[16 * 16];
  __shared__ __attribute__((aligned(16))) uint32_t xs[16][2][64];
  __shared__ __attribute__((aligned(16))) _Float16 xall[4096];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, n_in = lane & 15;
  const int Kt = K / 128;
  const int nt = blockIdx.x;
  const int kt[2] = {wave, wave + 16};
  typedef uint32_t u4v __attribute__((ext_vector_type(4)));
  Piece<4> pc[2];
  uint32_t sz[2], xr[2];
  const int64_t t0 = (int64_t)nt * Kt;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const u4v v = __builtin_nontemporal_load(
        reinterpret_cast<const u4v*>(qw + (t0 + kt[u]) * 256 + lane * 4));
    pc[u].w[0] = v.x; pc[u].w[1] = v.y; pc[u].w[2] = v.z; pc[u].w[3] = v.w;
  }
  if constexpr (V0 == 13) {
#pragma unroll
    for (int u = 0; u < 2; ++u) sz[u] = qsz[(t0 + kt[u]) * 16 + n_in];
    if (tid < 512) reinterpret_cast<uint4*>(xall)[tid] = reinterpret_cast<const uint4*>(x)[tid];
    __syncthreads();
  } else if constexpr (V == 0) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      sz[u] = qsz[(t0 + kt[u]) * 16 + n_in];
      xr[u] = reinterpret_cast<const uint32_t*>(x + kt[u] * 128)[lane];
    }
  } else {
    // lanes 0-15: group kt0, 16-31: group kt1 (lanes 32-63 repeat them)
    const int h = (lane >> 4) & 1;
    const uint32_t s1 = qsz[(t0 + kt[h]) * 16 + n_in];
    sz[0] = __builtin_amdgcn_ds_bpermute(4 * n_in, s1);
    sz[1] = __builtin_amdgcn_ds_bpermute(4 * (16 + n_in), s1);
    // lanes 0-31: x of tile 0 (8 B each), 32-63: tile 1
    const uint2 xv = reinterpret_cast<const uint2*>(x + kt[lane >> 5] * 128)[lane & 31];
    xs[wave][lane >> 5][2 * (lane & 31)] = xv.x;
    xs[wave][lane >> 5][2 * (lane & 31) + 1] = xv.y;
  }
  if constexpr (PRIO) {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
  }
  const Magics mg = make_magics<4>();
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  f4 acc4[4] = {};
  float dacc = 0.f, ys = 0.f;
  uint32_t xo = 0;
  if constexpr (V0 == 12) {
    if (N < 0) {  // never taken (N > 0): code that is fetched only if the I-cache streams past it
      asm volatile(".rept 250\n\tv_nop\n\t.endr" ::: "memory");
    }
  }
  constexpr int REP = V0 == 11 ? 3 : 1;
#pragma unroll 1
  for (int rep = 0; rep < REP; ++rep)
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if constexpr (V0 == 10) {
      if (u == 1) __builtin_amdgcn_s_setprio(1);
    }
    h8 xa[4];
    if constexpr (V0 == 13) {
      const uint4* b = reinterpret_cast<const uint4*>(xall + kt[u] * 128);
#pragma unroll
      for (int s = 0; s < 4; ++s) xa[s] = __builtin_bit_cast(h8, b[4 * s + (lane >> 4)]);
    } else {
      if constexpr (V == 0) xs[wave][u][lane] = xr[u];
      const uint4* b = reinterpret_cast<const uint4*>(&xs[wave][u][0]);
#pragma unroll
      for (int s = 0; s < 4; ++s) xa[s] = __builtin_bit_cast(h8, b[4 * s + (lane >> 4)]);
    }
    if constexpr (V == 6) {
      xo ^= pc[u].w[0] ^ pc[u].w[1] ^ pc[u].w[2] ^ pc[u].w[3] ^ sz[u];
      xo ^= __builtin_bit_cast(uint4, xa[0]).x ^ __builtin_bit_cast(uint4, xa[3]).y;
      continue;
    }
    Piece<4> p = pc[u];
    uint32_t szu = sz[u];
    if constexpr (V == 5) {  // constant operands: no dependency on the loads
      p.w[0] = 0x12345678u + u; p.w[1] = 0x9abcdef0u; p.w[2] = 0x0f1e2d3cu; p.w[3] = 0x4b5a6978u;
      szu = 0x00032c00u;
    }
    if constexpr (V == 4) {
      const _Float16 sc = sz_scale(szu);
      const int zp = sz_zero(szu);
      h2 zz[4];
#pragma unroll
      for (int P = 0; P < 4; ++P) {
        const _Float16 z = (_Float16)(pair_off<4>(P) + zp);
        zz[P] = h2{z, z};
      }
      f4 a = {0.f, 0.f, 0.f, 0.f};
      auto one = [&](auto S_) {
        constexpr int S = decltype(S_)::value;
        uint32_t v[4];
        step_pairs<4, S>(p, mg, v);
#pragma unroll
        for (int P = 0; P < 4; ++P) v[P] = as_u32(as_h2(v[P]) - zz[P]);
        const h8 bb = __builtin_bit_cast(h8, make_uint4(v[0], v[1], v[2], v[3]));
        a = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa[S], bb, a, 0, 0, 0);
      };
      one(std::integral_constant<int, 0>{});
      one(std::integral_constant<int, 1>{});
      one(std::integral_constant<int, 2>{});
      one(std::integral_constant<int, 3>{});
      ys += (float)sc * a[0];
      continue;
    }
    const GroupQ gq = make_group_w<4, kZNarrow>(szu);
    auto one = [&](auto S_) {
      constexpr int S = decltype(S_)::value;
      uint32_t v[4];
      dequant_step<4, kZNarrow, S>(p, mg, gq, v);
      const h8 bb = __builtin_bit_cast(h8, make_uint4(v[0], v[1], v[2], v[3]));
      if constexpr (V == 2) {
#pragma unroll
        for (int P = 0; P < 4; ++P)
          dacc = __builtin_amdgcn_fdot2(as_h2(v[P]), h2{xa[S][2 * P], xa[S][2 * P + 1]}, dacc, false);
      } else if constexpr (V == 3) {
        acc4[S] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa[S], bb, acc4[S], 0, 0, 0);
      } else {
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa[S], bb, acc, 0, 0, 0);
      }
    };
    one(std::integral_constant<int, 0>{});
    one(std::integral_constant<int, 1>{});
    one(std::integral_constant<int, 2>{});
    one(std::integral_constant<int, 3>{});
  }
  float yt;
  if constexpr (V == 2) {  // lanes n, n + 16, n + 32, n + 48 hold row n's k quarters
    float v = dacc;
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    yt = v;
  } else if constexpr (V == 3) {
    yt = (acc4[0][0] + acc4[1][0]) + (acc4[2][0] + acc4[3][0]);
  } else if constexpr (V == 4) {
    yt = ys;
  } else if constexpr (V == 6) {
    yt = (float)(xo & 0xFF);
  } else {
    yt = acc[0];
  }
  if constexpr (V == 5) {  // fold the loaded words in
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      xo ^= pc[u].w[0] ^ pc[u].w[1] ^ pc[u].w[2] ^ pc[u].w[3] ^ sz[u];
      xo ^= xs[wave][u][lane];
    }
    yt += (float)(xo & 1);
  }
  if (lane < 16) red[n_in * 16 + wave] = yt;
  __syncthreads();
  if (tid < 16) {
    const f4* r = reinterpret_cast<const f4*>(red + tid * 16);
    const f4 a = r[0], bq = r[1], c = r[2], d = r[3];
    const f4 e = (a + bq) + (c + d);
    y[(int64_t)blockIdx.x * 16 + tid] = (_Float16)((e[0] + e[1]) + (e[2] + e[3]));
  }
}

extern "C" int lab3_launch(const void* qw, const void* qsz, const void* x, void* y, int N, int K,
                           int V, void* st) {
  if (K != 4096 || N % 16) return 1;
#define L(v)                                                                                    \
  hipLaunchKernelGGL((lab3<v>), dim3(N / 16), dim3(1024), 0, (hipStream_t)st,                  \
                     (const uint32_t*)qw, (const uint32_t*)qsz, (const _Float16*)x, (_Float16*)y, \
                     N, K)
  switch (V) {
    case 0: L(0); break;
    case 1: L(1); break;
    case 2: L(2); break;
    case 3: L(3); break;
    case 4: L(4); break;
    case 5: L(5); break;
    case 6: L(6); break;
    case 7: L(7); break;
    case 8: L(8); break;
    case 9: L(9); break;
    case 10: L(10); break;
    case 11: L(11); break;
    case 12: L(12); break;
    default: L(13); break;
  }
#undef L
  return (int)hipGetLastError();
}
