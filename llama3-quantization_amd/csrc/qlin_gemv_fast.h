// qlin_gemv_fast.h — the decode fast GEMV (M <= 4, at most 4 k-tiles per wave) as a device body,
// shared by its own launch (qlin_gemv.hip gemv_fast_kernel) and by the fused q/k/v + decode
// attention launch (qlin_decode_fused.hip), plus the host geometry both use.
#pragma once

#include <type_traits>

#include "qlin_common.h"
#include "qlin_gemv_tile.h"

namespace qlin_gv {

using namespace qlin;

constexpr int kMaxWaves = 16;

// NRM (the fused RMSNorm of one token row): 0 none, kNwF32 an fp32 norm weight, kNwF16 the
// module's fp16 weight (half the bytes; every fp16 is exact in fp32, so the normed x is the same)
constexpr int kNwF32 = 1, kNwF16 = 2;
// two norm weights (k, k + 1) as loaded: raw until used, so no wait is scheduled at the load
template <int NRM>
using NwPair = std::conditional_t<NRM == kNwF16, uint32_t, float2>;
template <int NRM>
__device__ __forceinline__ NwPair<NRM> load_nw_pair(const void* nw, int k) {
  if constexpr (NRM == kNwF16) return *reinterpret_cast<const uint32_t*>((const _Float16*)nw + k);
  else return *reinterpret_cast<const float2*>((const float*)nw + k);
}
template <int NRM>
__device__ __forceinline__ float2 nw_pair_f32(NwPair<NRM> w) {
  if constexpr (NRM == kNwF16) {
    const h2 v = as_h2(w);
    return float2{(float)v.x, (float)v.y};
  } else {
    return w;
  }
}

// ---------------------------------------------------------------------------------------------
// Decode fast path: M <= 4, K % 128 == 0, group % 128 == 0 or group in {32, 64}, no activation
// fake-quant, at most 4 k-tiles per wave.  Same arithmetic as gemv_kernel (exact W_dq, one MFMA
// per k-step), built for the few microseconds a decode launch lasts (tools/dev/gemv_lab2.hip,
// gemv_lab3.hip):
//   - everything the general kernel derives by integer division (tiles, groups, strides) comes
//     precomputed from the host, so the first weight load issues a few scalar ops after the
//     kernel arguments land; the epilogue is a template parameter, so the executed code is one
//     short straight line;
//   - wave w streams tiles kt = w, w + W, w + 2W, ... (4096^2: 3.89 -> 3.74 us);
//   - all of a wave's tiles are loaded up front; a slot past the wave's tiles repeats its last
//     tile on x zeroed instead of branching (a load under a branch is waited for at the join).
// NRM (M = 1): x is the decoder layer's hidden state before its RMSNorm (OmniLlamaRMSNorm,
// quant/omni_norm.py:52-63 of the reference) and the kernel applies the norm at the reference's
// rounding point: each wave sums the squares of the x words it loads anyway (its own tiles;
// together the waves cover the row once), the block combines the W sums through LDS behind a bare
// s_barrier (no vmcnt drain), and every x word becomes RN16(weight * (x * rsqrt(mean + eps)))
// (fp32 inside) before it is parked.  The x words and norm weights are issued before the codes
// (in-order completion: the statistics wait for them, not for the weights).
// ---------------------------------------------------------------------------------------------
struct FastArgs {
  const uint32_t* qw;   // row tile 0 of qweight
  const uint32_t* qsz;  // row tile 0 of qsz
  const _Float16* x;
  const _Float16* bias;
  const _Float16* res;
  _Float16* y;
  int M, N, K, Kt, G;
  int W, lw;            // waves per block (power of two), log2 W
  uint32_t cmagic;      // GPT == 1: kt / (group / 128) = (kt * cmagic) >> 31
  const void* nw;       // NRM: RMSNorm weight [K] (fp32 / fp16) applied to x first
  float eps;
};

// The fast kernel's body for row tile `nt` (one block; blockDim = 64 * a.W).  HO (hand-off): the
// block's outputs also leave with agent-scope (sc1) stores of fp16 pairs, drained, and then one
// agent-scope add to *ready announces them — the producer side of a same-launch consumer
// (qlin_decode_fused.hip: q/k/v -> decode attention; MI355X_MICROARCH.md hand-off table, row 1).
template <int BITS, int MT, int GPT, int ZM, int EP, int PF, int NRM = 0, bool HO = false>
__device__ __forceinline__ void gemv_fast_body(const FastArgs& a, const int nt, int* ready = nullptr) {
  __shared__ __attribute__((aligned(16))) float red[MT * kTileN * kMaxWaves];
  __shared__ __attribute__((aligned(16))) uint32_t xs[kMaxWaves][64 * MT];
  __shared__ float nss[NRM ? kMaxWaves : 1];  // NRM: per-wave sums of squares
  static_assert(!NRM || MT == 1, "the fused RMSNorm serves one token row");
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, n_in = lane & 15;
  const _Float16* ax = a.x;
  const _Float16* abias = a.bias;
  _Float16* ay = a.y;
  const uint32_t* qw = a.qw + (int64_t)nt * a.Kt * (64 * BITS) + lane * BITS;
  const uint32_t* sz = a.qsz + (int64_t)nt * a.G * kTileN + n_in;
  constexpr int LPR = 64 / MT;  // lanes per x row
  const _Float16* xr = ax + (int64_t)min(lane / LPR, a.M - 1) * a.K + 2 * MT * (lane % LPR);
  const int nts = (a.Kt - wave + a.W - 1) >> a.lw;  // >= 1: W <= Kt
  const int ktl = wave + ((nts - 1) << a.lw);        // the wave's last tile
  auto kt_of = [&](int i) { return min(wave + (i << a.lw), ktl); };
  auto group_of_tile = [&](int kt) {
    return GPT == 1 ? (int)(((uint64_t)(uint32_t)kt * a.cmagic) >> 31) : kt * GPT;
  };
  WTile<BITS, GPT> wt[PF];
  XRaw<MT> xq[PF];
  NwPair<NRM> nwv[NRM ? PF : 1];  // NRM: norm weights of the lane's two x halves per tile
  auto load_codes = [&](int u, int kt) { wt[u].pc = load_piece_nt<BITS>(qw + kt * (64 * BITS)); };
  auto load_sz = [&](int u, int kt) {
    const int g0 = group_of_tile(kt);
#pragma unroll
    for (int s = 0; s < GPT; ++s) wt[u].sz[s] = sz[(g0 + s) * kTileN];
  };
  auto load_x = [&](int u, int kt) {
    const _Float16* p = xr + kt * kTileK;
    if constexpr (MT == 1) {
      xq[u].w[0] = *reinterpret_cast<const uint32_t*>(p);
    } else if constexpr (MT == 2) {
      const uint2 v = *reinterpret_cast<const uint2*>(p);
      xq[u].w[0] = v.x; xq[u].w[1] = v.y;
    } else {
      const uint4 v = *reinterpret_cast<const uint4*>(p);
      xq[u].w[0] = v.x; xq[u].w[1] = v.y; xq[u].w[2] = v.z; xq[u].w[3] = v.w;
    }
  };
  if constexpr (NRM) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      load_x(u, kt_of(u));
      nwv[u] = load_nw_pair<NRM>(a.nw, kt_of(u) * kTileK + 2 * lane);
    }
#pragma unroll
    for (int u = 0; u < PF; ++u) load_codes(u, kt_of(u));
#pragma unroll
    for (int u = 0; u < PF; ++u) load_sz(u, kt_of(u));
  } else {
#pragma unroll
    for (int u = 0; u < PF; ++u) load_codes(u, kt_of(u));
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      load_sz(u, kt_of(u));
      load_x(u, kt_of(u));
    }
  }
  // the epilogue's bias / residual operands, fetched while the weights stream (fetched after the
  // reduction they would cost one more round trip).  Only wave 0's lanes use them, but every wave
  // loads (clamped, L2-resident): a load under a branch is waited for at the branch's join
  constexpr int NO = EP == kEpSiluMul ? MT * 8 : MT * kTileN;  // outputs per block
  const int om = min(tid / (NO / MT), a.M - 1), on = tid % (NO / MT);  // output (row m, column n)
  const int64_t orow = (int64_t)nt * kTileN + on;
  const bool oval = tid < NO && tid / (NO / MT) < a.M && orow + (EP == kEpSiluMul ? 8 : 0) < a.N;
  const _Float16* bsrc = abias ? abias + min(orow, (int64_t)a.N - 1) : ax;
  const _Float16 ob0 = bsrc[0];
  const _Float16 ob1 = EP == kEpSiluMul ? bsrc[abias ? 8 : 0] : ob0;
  _Float16 ores = 0;
  if constexpr (EP == kEpResidual) ores = a.res[(int64_t)om * a.N + min(orow, (int64_t)a.N - 1)];

  float rn = 1.f;  // NRM: rsqrt(mean(x^2) + eps)
  if constexpr (NRM) {
#pragma clang fp contract(off)
    float ss = 0.f;
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      if (u < nts) {  // wave-uniform: slots past the wave's tiles repeat its last tile
        const h2 v = as_h2(xq[u].w[0]);
        const float f0 = (float)v.x, f1 = (float)v.y;
        ss = ss + f0 * f0;
        ss = ss + f1 * f1;
      }
    }
    ss = wave_sum(ss);
    if (lane == 0) nss[wave] = ss;
    // a bare s_barrier after the LDS store: __syncthreads() would also drain vmcnt, i.e. wait for
    // the weight words still in flight; the waves only need each other's sums
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    float tot = 0.f;
    for (int w = 0; w < a.W; ++w) tot += nss[w];
    rn = rsqrtf(tot / (float)a.K + a.eps);
  }

  const Magics mg = make_magics<BITS>();
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  uint32_t* slot = &xs[wave][0];
  auto tile = [&](int u) {
    h8 xa[4];
    if constexpr (NRM) {
#pragma clang fp contract(off)
      const h2 v = as_h2(xq[u].w[0]);
      const float2 w = nw_pair_f32<NRM>(nwv[u]);
      const float n0 = w.x * ((float)v.x * rn);
      const float n1 = w.y * ((float)v.y * rn);
      xq[u].w[0] = as_u32(h2{(_Float16)n0, (_Float16)n1});
    }
    park_x<MT>(xa, xq[u], slot, lane, n_in);
    auto step = [&](auto S_) {
      constexpr int S = decltype(S_)::value;
      uint32_t v[4];
      const GroupQ gq = make_group_w<BITS, ZM>(wt[u].sz[S * GPT / 4]);
      dequant_step<BITS, ZM, S>(wt[u].pc, mg, gq, v);
      const h8 b = __builtin_bit_cast(h8, make_uint4(v[0], v[1], v[2], v[3]));
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa[S], b, acc, 0, 0, 0);
    };
    step(std::integral_constant<int, 0>{});
    step(std::integral_constant<int, 1>{});
    step(std::integral_constant<int, 2>{});
    step(std::integral_constant<int, 3>{});
  };
  // every slot is computed — a slot past the wave's tiles (a repeat of its last tile) with x
  // zeroed — so the compiler cannot sink those slots' loads behind a branch
  tile(0);  // nts >= 1
#pragma unroll
  for (int u = 1; u < PF; ++u) {
    if (u >= nts) {  // wave-uniform
#pragma unroll
      for (int c = 0; c < MT; ++c) xq[u].w[c] = 0u;
    }
    tile(u);
  }

  // combine the W partials of (row m, column n): C row m = 4q + e sits in lane n + 16q, element e
  const int q4 = 4 * (lane >> 4);
  if (q4 < MT) {
#pragma unroll
    for (int e = 0; e < 4 && e < MT; ++e) red[((q4 + e) * kTileN + n_in) * kMaxWaves + wave] = acc[e];
    if (wave == 0)
      for (int w = a.W; w < kMaxWaves; ++w)
#pragma unroll
        for (int e = 0; e < 4 && e < MT; ++e) red[((q4 + e) * kTileN + n_in) * kMaxWaves + w] = 0.f;
  }
  __syncthreads();
  auto total = [&](int o, _Float16 b) {
    const f4* r = reinterpret_cast<const f4*>(red + o * kMaxWaves);
    const f4 p = r[0], q = r[1], c = r[2], d = r[3];
    const f4 e = (p + q) + (c + d);
    float t = (e[0] + e[1]) + (e[2] + e[3]);
    if (abias) t += (float)b;
    return (float)(_Float16)t;  // F.linear's fp16 output
  };
  if constexpr (HO) {  // M = 1, no epilogue, N % 16 == 0 (host): wave 0 hands the 16 outputs off
    static_assert(MT == 1 && EP == kEpNone, "hand-off: one token row, plain outputs");
    if (wave == 0) {
      const float t = total(min(lane, kTileN - 1), ob0);
      const uint32_t h = (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)t);
      const uint32_t h1 = (uint32_t)__shfl_xor((int)h, 1);
      if (lane < kTileN && !(lane & 1))
        __hip_atomic_store(reinterpret_cast<uint32_t*>(ay + orow), h | (h1 << 16),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the pairs acknowledged before the add
      if (lane == 0) __hip_atomic_fetch_add(ready, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  if (oval) {  // wave 0 only (tid < NO <= 64)
    if constexpr (EP == kEpSiluMul) {  // 8 outputs per tile and row
      const float g = total(om * kTileN + on, ob0), u = total(om * kTileN + on + 8, ob1);
      ay[(int64_t)om * (a.N >> 1) + nt * 8 + on] = (_Float16)(silu_rn16(g) * u);
    } else {
      float t = total(om * kTileN + on, ob0);
      if constexpr (EP == kEpResidual) t += (float)ores;
      ay[(int64_t)om * a.N + orow] = (_Float16)t;
    }
  }
}

static inline uint32_t tile_group_magic(int group) {  // GPT == 1: kt / (group / 128) = (kt * magic) >> 31
  const uint64_t c = group % kTileK == 0 ? (uint64_t)(group / kTileK) : 1;
  return (uint32_t)(((1ull << 31) + c - 1) / c);
}

// waves per block: grow W until the grid holds ~32 waves for each of the 256 CUs; on grids of
// >= 512 row tiles keep >= 4 tiles per wave (measured on the decode layer's shapes,
// tools/dev/gemv_geo.py: 28,672 x 4,096 W = 8 12.6 us vs W = 4 13.3 us; 14,336 x 4,096 W = 8
// 8.9 us vs W = 16 9.3 us; 4096 x 4096 and 6144 x 4096 keep W = 16)
constexpr int64_t kWaveTarget = 8192;
static inline int pick_waves(int Nt, int Kt, int& tpw) {
  int W = 1;
  while (W < kMaxWaves && (int64_t)Nt * W < kWaveTarget && (Nt < 512 || Kt >= 8 * W)) W *= 2;
  W = min(W, Kt);
  tpw = (Kt + W - 1) / W;
  return (Kt + tpw - 1) / tpw;
}

static inline bool group_fast(int K, int group) {  // whole-tile or 32 / 64-wide groups on whole k-tiles
  return K % kTileK == 0 && (group % kTileK == 0 || group == 32 || group == 64);
}

// fast-path geometry: pick_waves rounded down to a power of two, then halved while the grid holds
// more than 16 waves per CU (all blocks resident in one round: q/k/v, 384 row tiles, W = 16 ran in
// two rounds, round-4 stamp builds); the fast path takes launches whose waves stream at most 4
// tiles (tools/dev/fast_geo.py)
static inline bool fast_geometry(int Nt, int Kt, int& W, int& lw, int& tpw) {
  W = pick_waves(Nt, Kt, tpw);
  lw = 0;
  while ((2 << lw) <= W) ++lw;  // round W down to a power of two (W <= Kt)
  const int64_t cus = device_cu_count();
  while (lw > 0 && (int64_t)Nt * (1 << lw) > kMaxWaves * cus && (Kt + (1 << lw) / 2 - 1) / ((1 << lw) / 2) <= 4)
    --lw;
  W = 1 << lw;
  tpw = (Kt + W - 1) / W;
  return tpw <= 4;
}

}  // namespace qlin_gv
