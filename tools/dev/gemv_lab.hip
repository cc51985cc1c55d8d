// Development-only GEMV laboratory (not part of the product library): the product GEMV's
// structure (int4, g128, M = 1, exact dequant) with knobs and per-wave s_memrealtime stamps.
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

template <bool NT>
__device__ __forceinline__ Piece<4> ld_piece(const uint32_t* p) {
  Piece<4> c;
  typedef uint32_t u4v __attribute__((ext_vector_type(4)));
  u4v v;
  if constexpr (NT) v = __builtin_nontemporal_load(reinterpret_cast<const u4v*>(p));
  else v = *reinterpret_cast<const u4v*>(p);
  c.w[0] = v.x; c.w[1] = v.y; c.w[2] = v.z; c.w[3] = v.w;
  return c;
}

struct WT { Piece<4> pc; uint32_t sz; };

// MODE 0: full exact GEMV; 1: loads only (xor); 2: loads + dequant, no MFMA;
// 3: (u - z) exact in fp16, MFMA per group, y += s * acc (scale after accumulate)
// RED 0: serial W-loop reduction by 16 threads; 1: [n][w] layout, 4 x ds_read_b128 per thread
template <int PF, bool NT, int MODE, int RED, bool XL = false>
__global__ __launch_bounds__(1024) void lab_gemv(const uint32_t* __restrict__ qw,
                                                 const uint32_t* __restrict__ qsz,
                                                 const _Float16* __restrict__ x,
                                                 _Float16* __restrict__ y, int N, int K, int tpw,
                                                 uint64_t* __restrict__ stamps) {
  const uint64_t t0s = stamp();
  __shared__ float red[16 * 16];
  __shared__ __attribute__((aligned(16))) uint32_t xs[16][2][64];  // per wave, per x slot: 256 B
  const int W = blockDim.x >> 6;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, n_in = lane & 15;
  const int nt = blockIdx.x;
  const int Kt = K / 128, G = K / 128;
  const uint32_t* qw_nt = qw + (int64_t)nt * Kt * 256;
  const uint32_t* sz_nt = qsz + (int64_t)nt * G * 16;
  const int xoff = 8 * (lane >> 4);
  const int kt0 = wave * tpw;
  const int nts = max(0, min(tpw, Kt - kt0));
  const int ktl = max(0, min(Kt - 1, kt0 + nts - 1));
  // MODE 4: weights only; 5: weights + sz; 6: weights + x (all as MODE 1 otherwise)
  constexpr bool LSZ = MODE != 4 && MODE != 6;
  constexpr bool LX = MODE != 4 && MODE != 5;
  auto load_w = [&](WT& t, int kt) {
    t.pc = ld_piece<NT>(qw_nt + kt * 256 + lane * 4);
    if constexpr (LSZ) t.sz = sz_nt[kt * 16 + n_in];
    else t.sz = kt;
  };
  auto load_x = [&](h8 (&xa)[4], int kt) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      if constexpr (LX) xa[s] = *reinterpret_cast<const h8*>(x + kt * 128 + 32 * s + xoff);
      else xa[s] = h8{};
    }
  };
  // XL: one dword per lane per tile (x[kt*128 + 2 lane .. +1]), parked in LDS at use
  auto load_xr = [&](uint32_t& r, int kt) {
    r = reinterpret_cast<const uint32_t*>(x + kt * 128)[lane];
  };
  auto park_x = [&](h8 (&xa)[4], uint32_t r, int slot) {
    xs[wave][slot][lane] = r;
    const uint4* b = reinterpret_cast<const uint4*>(&xs[wave][slot][0]);
#pragma unroll
    for (int s = 0; s < 4; ++s) xa[s] = __builtin_bit_cast(h8, b[4 * s + (lane >> 4)]);
  };
  const Magics mg = make_magics<4>();
  h8 boff = {};
#pragma unroll
  for (int P = 0; P < 4; ++P) {
    const _Float16 o = n_in == 0 ? (_Float16)pair_off<4>(P) : n_in == 1 ? (_Float16)1.0f : (_Float16)0.0f;
    boff[2 * P] = o;
    boff[2 * P + 1] = o;
  }
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  f4 acc4[4] = {};
  float ys = 0.f;
  uint32_t xr = 0;
  uint64_t t1s = 0;
  auto tile = [&](const WT& t, const h8 (&xa)[4]) {
    if constexpr (MODE == 10) {
      // offset trick: MFMA on (off + u), offset-column MFMA gives S1 = sum off x, S2 = sum x
      f4 a = {0.f, 0.f, 0.f, 0.f}, ao = {0.f, 0.f, 0.f, 0.f};
      auto one = [&](auto S_) {
        constexpr int S = decltype(S_)::value;
        uint32_t v[4];
        step_pairs<4, S>(t.pc, mg, v);
        const h8 b = __builtin_bit_cast(h8, make_uint4(v[0], v[1], v[2], v[3]));
        a = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa[S], b, a, 0, 0, 0);
        ao = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa[S], boff, ao, 0, 0, 0);
      };
      one(std::integral_constant<int, 0>{});
      one(std::integral_constant<int, 1>{});
      one(std::integral_constant<int, 2>{});
      one(std::integral_constant<int, 3>{});
      const float sc = (float)sz_scale(t.sz), zf = (float)sz_zero(t.sz);
      const int ab = __builtin_bit_cast(int, ao[0]);
      const float s1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(ab, 0));
      const float s2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(ab, 1));
      ys += sc * (a[0] - (s1 + zf * s2));
    } else if constexpr (MODE == 7 || MODE == 8) {
      // VALU dot path (M = 1): lane (n, q) accumulates row n over its k subset; q-reduce at end
      const _Float16 sc = sz_scale(t.sz);
      const int zp = sz_zero(t.sz);
      GroupQ gq;
      h2 zz[4];
      if constexpr (MODE == 7) {
        gq = make_group<4, false>(sc, zp);
      } else {
#pragma unroll
        for (int P = 0; P < 4; ++P) {
          const _Float16 z = (_Float16)(pair_off<4>(P) + zp);
          zz[P] = h2{z, z};
        }
      }
      float a = 0.f;
      auto one = [&](auto S_) {
        constexpr int S = decltype(S_)::value;
        uint32_t v[4];
        if constexpr (MODE == 7) {
          dequant_step<4, false, S>(t.pc, mg, gq, v);
        } else {
          step_pairs<4, S>(t.pc, mg, v);
#pragma unroll
          for (int P = 0; P < 4; ++P) v[P] = as_u32(as_h2(v[P]) - zz[P]);
        }
        const h8 xv = xa[S];
#pragma unroll
        for (int P = 0; P < 4; ++P)
          a = __builtin_amdgcn_fdot2(as_h2(v[P]), h2{xv[2 * P], xv[2 * P + 1]}, a, false);
      };
      one(std::integral_constant<int, 0>{});
      one(std::integral_constant<int, 1>{});
      one(std::integral_constant<int, 2>{});
      one(std::integral_constant<int, 3>{});
      if constexpr (MODE == 7) ys += a;
      else ys += (float)sc * a;
    } else if constexpr (MODE == 3) {
      const _Float16 sc = sz_scale(t.sz);
      const int zp = sz_zero(t.sz);
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
        step_pairs<4, S>(t.pc, mg, v);
#pragma unroll
        for (int P = 0; P < 4; ++P) v[P] = as_u32(as_h2(v[P]) - zz[P]);
        const h8 b = __builtin_bit_cast(h8, make_uint4(v[0], v[1], v[2], v[3]));
        a = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa[S], b, a, 0, 0, 0);
      };
      one(std::integral_constant<int, 0>{});
      one(std::integral_constant<int, 1>{});
      one(std::integral_constant<int, 2>{});
      one(std::integral_constant<int, 3>{});
      ys += (float)sc * a[0];
    } else if constexpr (MODE == 1 || (MODE >= 4 && MODE <= 6)) {
      xr ^= t.pc.w[0] ^ t.pc.w[1] ^ t.pc.w[2] ^ t.pc.w[3] ^ t.sz;
      xr ^= __builtin_bit_cast(uint4, xa[0]).x ^ __builtin_bit_cast(uint4, xa[3]).y;
    } else {
      const GroupQ gq = make_group<4, false>(sz_scale(t.sz), sz_zero(t.sz));
      auto one = [&](auto S_) {
        constexpr int S = decltype(S_)::value;
        uint32_t v[4];
        dequant_step<4, false, S>(t.pc, mg, gq, v);
        const h8 b = __builtin_bit_cast(h8, make_uint4(v[0], v[1], v[2], v[3]));
        if constexpr (MODE == 0) acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa[S], b, acc, 0, 0, 0);
        else if constexpr (MODE == 9) acc4[S] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa[S], b, acc4[S], 0, 0, 0);
        else xr ^= v[0] ^ v[1] ^ v[2] ^ v[3];
      };
      one(std::integral_constant<int, 0>{});
      one(std::integral_constant<int, 1>{});
      one(std::integral_constant<int, 2>{});
      one(std::integral_constant<int, 3>{});
    }
  };
  WT wt[PF];
  h8 xa[2][4];
  uint32_t xq[PF];
  if constexpr (XL) {
    load_xr(xq[0], min(kt0, ktl));
    load_w(wt[0], min(kt0, ktl));
#pragma unroll
    for (int u = 1; u < PF; ++u) {
      load_xr(xq[u], min(kt0 + u, ktl));
      load_w(wt[u], min(kt0 + u, ktl));
    }
  } else {
    load_x(xa[0], min(kt0, ktl));
    load_w(wt[0], min(kt0, ktl));
    load_w(wt[1], min(kt0 + 1, ktl));
    load_x(xa[1], min(kt0 + 1, ktl));
#pragma unroll
    for (int u = 2; u < PF; ++u) load_w(wt[u], min(kt0 + u, ktl));
  }
  int t0 = 0;
  for (; t0 + PF < nts; t0 += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int kt = kt0 + t0 + u;
      if constexpr (XL) {
        park_x(xa[u & 1], xq[u], u & 1);
        tile(wt[u], xa[u & 1]);
        load_xr(xq[u], min(kt + PF, ktl));
      } else {
        tile(wt[u], xa[u & 1]);
        load_x(xa[u & 1], min(kt + 2, ktl));
      }
      if (t0 == 0 && u == 0) t1s = stamp();
      load_w(wt[u], min(kt + PF, ktl));
    }
  }
#pragma unroll
  for (int u = 0; u < PF; ++u) {
    if (t0 + u < nts) {
      if constexpr (XL) {
        park_x(xa[u & 1], xq[u], u & 1);
        tile(wt[u], xa[u & 1]);
      } else {
        tile(wt[u], xa[u & 1]);
        if (u + 2 < PF) load_x(xa[u & 1], min(kt0 + t0 + u + 2, ktl));
      }
      if (t0 == 0 && u == 0) t1s = stamp();
    }
  }
  const uint64_t t2s = stamp();
  float yt = acc[0];
  if constexpr (MODE == 9) yt = (acc4[0][0] + acc4[1][0]) + (acc4[2][0] + acc4[3][0]);
  if constexpr (MODE == 1 || MODE == 2 || (MODE >= 4 && MODE <= 6)) yt = (float)(xr & 0xFF);
  if constexpr (MODE == 3 || MODE == 10) yt = ys;
  if constexpr (MODE == 7 || MODE == 8) {  // sum the 4 k-quarters (lanes n, n+16, n+32, n+48)
    float v = ys;
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    yt = v;
  }
  if constexpr (RED == 0) {
    if (lane < 16) red[wave * 16 + n_in] = yt;
    __syncthreads();
    if (tid < 16) {
      float t = 0.f;
      for (int w = 0; w < W; ++w) t += red[w * 16 + tid];
      y[(int64_t)nt * 16 + tid] = (_Float16)t;
    }
  } else {
    if (lane < 16) red[n_in * 16 + wave] = yt;
    if (wave == 0 && lane < 16) {  // zero-fill the partials of absent waves
      for (int w = W; w < 16; ++w) red[n_in * 16 + w] = 0.f;
    }
    __syncthreads();
    if (tid < 16) {
      const f4* r = reinterpret_cast<const f4*>(red + tid * 16);
      const f4 a = r[0], b = r[1], c = r[2], d = r[3];
      const f4 e = (a + b) + (c + d);
      y[(int64_t)nt * 16 + tid] = (_Float16)((e[0] + e[1]) + (e[2] + e[3]));
    }
  }
  const uint64_t t3s = stamp();
  if (lane == 0 && stamps) {
    uint64_t* s = stamps + ((int64_t)blockIdx.x * W + wave) * 4;
    s[0] = t0s; s[1] = t1s; s[2] = t2s; s[3] = t3s;
  }
}

extern "C" int lab_gemv_launch(const void* qw, const void* qsz, const void* x, void* y, int N,
                               int K, int W, int PF, int NT, int MODE, int RED, void* stamps,
                               void* st, int XLv) {
  const int Kt = K / 128;
  const int tpw = (Kt + W - 1) / W;
  const int Wr = (Kt + tpw - 1) / tpw;
#define L(P, T, M)                                                                            \
  if (XLv) hipLaunchKernelGGL((lab_gemv<P, T, M, 1, true>), dim3(N / 16), dim3(64 * Wr), 0, (hipStream_t)st, \
                     (const uint32_t*)qw, (const uint32_t*)qsz, (const _Float16*)x,            \
                     (_Float16*)y, N, K, tpw, (uint64_t*)stamps); else \
  if (RED) hipLaunchKernelGGL((lab_gemv<P, T, M, 1>), dim3(N / 16), dim3(64 * Wr), 0, (hipStream_t)st, \
                     (const uint32_t*)qw, (const uint32_t*)qsz, (const _Float16*)x,            \
                     (_Float16*)y, N, K, tpw, (uint64_t*)stamps); else \
  hipLaunchKernelGGL((lab_gemv<P, T, M, 0>), dim3(N / 16), dim3(64 * Wr), 0, (hipStream_t)st,    \
                     (const uint32_t*)qw, (const uint32_t*)qsz, (const _Float16*)x,            \
                     (_Float16*)y, N, K, tpw, (uint64_t*)stamps)
#define LM(P, T) if (MODE == 0) { L(P, T, 0); } else if (MODE == 1) { L(P, T, 1); } else if (MODE == 2) { L(P, T, 2); } else if (MODE == 3) { L(P, T, 3); } else if (MODE == 4) { L(P, T, 4); } else if (MODE == 5) { L(P, T, 5); } else if (MODE == 6) { L(P, T, 6); } else if (MODE == 7) { L(P, T, 7); } else if (MODE == 8) { L(P, T, 8); } else if (MODE == 9) { L(P, T, 9); } else { L(P, T, 10); }
  if (PF == 2) { if (NT) { LM(2, true); } else { LM(2, false); } }
  else { if (NT) { LM(4, true); } else { LM(4, false); } }
  return (int)hipGetLastError();
}

// stamped pure stream read: 16 B per lane per load, 4 loads per thread
__global__ __launch_bounds__(256) void lab_stream(const uint4* __restrict__ p, int64_t n16,
                                                  uint32_t* out, uint64_t* stamps) {
  const uint64_t t0s = stamp();
  int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x;
  uint4 v[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) v[j] = p[min(i + j * 256, n16 - 1)];
  uint32_t acc = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) acc ^= v[j].x ^ v[j].y ^ v[j].z ^ v[j].w;
  const uint64_t t1s = stamp();
  if (acc == 0x12345678u) out[0] = acc;
  if ((threadIdx.x & 63) == 0 && stamps) {
    uint64_t* s = stamps + ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 4;
    s[0] = t0s; s[1] = t1s; s[2] = t1s; s[3] = t1s;
  }
}
extern "C" int lab_stream_launch(const void* p, int64_t bytes, void* out, void* stamps, void* st) {
  const int64_t n16 = bytes / 16;
  hipLaunchKernelGGL(lab_stream, dim3((unsigned)((n16 + 1023) / 1024)), dim3(256), 0,
                     (hipStream_t)st, (const uint4*)p, n16, (uint32_t*)out, (uint64_t*)stamps);
  return (int)hipGetLastError();
}
