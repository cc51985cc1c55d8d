// qlin_gemv.hip — fused unpack + group dequant + GEMV for decode-sized M (1..4) on the matrix
// cores, gfx950, plus the standalone exact dequant kernel.
//
// Replaces QuantLinear.forward -> F.linear(input, W_dq, bias) (quant/int_linear.py:48-65) on
// packed weights.  HBM-bound: every weight byte is read exactly once, with one coalesced
// 64 x (4*bits)-byte load per 16-row x 128-k tile and one 64-byte (scale, zero) load per tile and
// group slot (qlin_common.h layout).
//
// Per wave, per k-step of 32: one v_and_or_b32 per code pair (+1 shift per word) turns the lane's
// codes into the fp16 pairs (off_j + u_j); the default (exact) path then forms W_dq bit-exactly
// ((off + u) - (off + z), times s: v_pk_add/v_pk_mul) — already the B operand of
// v_mfma_f32_16x16x32_f16 — and the MFMA contracts it with x, so the result is the reference's
// F.linear(x, W_dq) up to fp32 summation order.  x (A operand) is fetched per k-step straight from
// L2 (16 B per lane; lanes whose A row is >= M re-read row M-1, whose C rows are never stored).
// No LDS staging and no barrier precede the first MFMA.  (QLIN_GEMV_FAST=1 selects the variant
// that feeds (off + u) directly and removes offsets / zero point / scale once per group with an
// offset-column MFMA: ~5 VALU per 8 codes instead of ~13, at a ~3e-4 max-relative deviation from
// F.linear(W_dq).)
//
// Every load is issued unconditionally from a wave-uniform base plus a per-lane offset and its
// value is consumed only later, so hipcc keeps PF tiles in flight with counted vmcnt(N) waits; a
// "load or zero" select on a lane condition makes it wait vmcnt(0) at the join (measured: the
// whole prefetch serialised).
//
// Decomposition: block = one 16-row tile row (grid = ceil(N/16)); its W <= 16 waves split K (tpw
// tiles each, PF = 2 or 4 weight tiles in flight per wave) and combine their 16 x M partials
// through LDS.
#include "qlin_common.h"
#include "../../include/qlin_gfx950.h"

#include <stdlib.h>

#include <type_traits>

using namespace qlin;

namespace {

constexpr int kMaxWaves = 16;

template <int BITS, int GPT>
struct WTile {
  Piece<BITS> pc;
  uint32_t sz[GPT];  // packed (scale, zero) of each group slot, decoded only at use
};

struct Geo {
  const uint32_t* qw_nt;  // this block's tile row of qweight (uniform)
  const uint32_t* sz_nt;  // this block's row tile of qsz (uniform)
  const _Float16* x;
  int K, G, group, gshift, lane, n_in, xoff;
};

__device__ __forceinline__ int group_of(const Geo& g, int k) {
  const int gi = g.gshift >= 0 ? (k >> g.gshift) : k / g.group;
  return min(gi, g.G - 1);
}

template <int BITS, int GPT>
__device__ __forceinline__ void load_w(WTile<BITS, GPT>& t, const Geo& g, int kt) {
  t.pc = load_piece<BITS>(g.qw_nt + kt * 64 * BITS + g.lane * BITS);
#pragma unroll
  for (int i = 0; i < GPT; ++i)
    t.sz[i] = g.sz_nt[group_of(g, kt * kTileK + 32 * (i * 4 / GPT)) * kTileN + g.n_in];
}

__device__ __forceinline__ void load_x(h8 (&xa)[4], const Geo& g, int kt) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int k = min(kt * kTileK + 32 * s, g.K - 32);  // uniform; + 8q + 7 stays < K
    xa[s] = *reinterpret_cast<const h8*>(g.x + k + g.xoff);
  }
}

template <int BITS, int MT, int GPT, bool WIDE, bool EXACT, int PF>
__device__ __forceinline__ void gemv_body(const Geo& g, int kt0, int nts, int ktl, f4& acc,
                                          float (&yt)[4]) {
  const Magics mg = make_magics<BITS>();
  // fast path: offset column MFMA (column 0: off_k, column 1: 1) gives S1 = sum off x, S2 = sum x
  f4 aoff = {0.f, 0.f, 0.f, 0.f};
  h8 boff = {};
  if constexpr (!EXACT) {
#pragma unroll
    for (int P = 0; P < 4; ++P) {
      const _Float16 o = g.n_in == 0 ? (_Float16)pair_off<BITS>(P)
                                     : g.n_in == 1 ? (_Float16)1.0f : (_Float16)0.0f;
      boff[2 * P] = o;
      boff[2 * P + 1] = o;
    }
  }
  int gend = (group_of(g, kt0 * kTileK) + 1) * g.group;  // k at which the current group ends

  // FULL: the tile is not the matrix's last (only that one can hold fewer than 4 k-steps)
  auto step = [&](const WTile<BITS, GPT>& t, const h8 (&xa)[4], int kt, auto S_, auto FULL_) {
    constexpr int S = decltype(S_)::value;
    constexpr bool FULL = decltype(FULL_)::value;
    constexpr int slot = S * GPT / 4;
    const int k0 = kt * kTileK + 32 * S;
    if (FULL || k0 < g.K) {  // wave-uniform
      uint32_t v[4];
      if constexpr (EXACT) {
        const GroupQ gq = make_group<BITS, WIDE>(sz_scale(t.sz[slot]), sz_zero(t.sz[slot]));
        dequant_step<BITS, WIDE, S>(t.pc, mg, gq, v);
      } else {
        step_pairs<BITS, S>(t.pc, mg, v);
      }
      const h8 b = __builtin_bit_cast(h8, make_uint4(v[0], v[1], v[2], v[3]));
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa[S], b, acc, 0, 0, 0);
      if constexpr (!EXACT) {
        aoff = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa[S], boff, aoff, 0, 0, 0);
        if (k0 + 32 == gend) {  // group ends: y += s * (acc - S1 - z * S2)
          const float sc = (float)sz_scale(t.sz[slot]), zf = (float)sz_zero(t.sz[slot]);
#pragma unroll
          for (int i = 0; i < MT && i < 4; ++i) {
            // rows m < 4 live in lanes 0..15: column 0 holds S1_m, column 1 holds S2_m
            const int ab = __builtin_bit_cast(int, aoff[i]);
            const float s1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(ab, 0));
            const float s2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(ab, 1));
            yt[i] += sc * (acc[i] - (s1 + zf * s2));
          }
          acc = f4{0.f, 0.f, 0.f, 0.f};
          aoff = f4{0.f, 0.f, 0.f, 0.f};
          gend += g.group;
        }
      }
    }
  };
  auto tile = [&](const WTile<BITS, GPT>& t, const h8 (&xa)[4], int kt, auto FULL_) {
    step(t, xa, kt, std::integral_constant<int, 0>{}, FULL_);
    step(t, xa, kt, std::integral_constant<int, 1>{}, FULL_);
    step(t, xa, kt, std::integral_constant<int, 2>{}, FULL_);
    step(t, xa, kt, std::integral_constant<int, 3>{}, FULL_);
  };

  // prologue: PF weight tiles and 2 x tiles in flight, tile index clamped to the wave's last
  WTile<BITS, GPT> wt[PF];
  h8 xa[2][4];
  load_x(xa[0], g, min(kt0, ktl));
  load_w(wt[0], g, min(kt0, ktl));
  load_w(wt[1], g, min(kt0 + 1, ktl));
  load_x(xa[1], g, min(kt0 + 1, ktl));
#pragma unroll
  for (int u = 2; u < PF; ++u) load_w(wt[u], g, min(kt0 + u, ktl));

  // full rounds of PF tiles: compute tile t, refill its x slot with t + 2, its weight slot with
  // t + PF (invariant at the top of a round: wt[u] = tile t0 + u, xa[0/1] = tiles t0, t0 + 1)
  int t0 = 0;
  for (; t0 + PF < nts; t0 += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int kt = kt0 + t0 + u;
      tile(wt[u], xa[u & 1], kt, std::true_type{});
      load_x(xa[u & 1], g, min(kt + 2, ktl));
      load_w(wt[u], g, min(kt + PF, ktl));
    }
  }
  // last round (1..PF tiles): compute only, plus the x refills its tiles 2, 3 need
#pragma unroll
  for (int u = 0; u < PF; ++u) {
    if (t0 + u < nts) {
      const int kt = kt0 + t0 + u;
      tile(wt[u], xa[u & 1], kt, std::false_type{});
      if (u + 2 < PF) load_x(xa[u & 1], g, min(kt + 2, ktl));
    }
  }
}

template <int BITS, int MT, int GPT, bool WIDE, bool EXACT, int PF>
__global__ __launch_bounds__(1024) void gemv_kernel(
    const uint32_t* __restrict__ qw, const uint32_t* __restrict__ qsz,
    const _Float16* __restrict__ x, const _Float16* __restrict__ bias, _Float16* __restrict__ y,
    int M, int N, int K, int group, int gshift, int tpw) {
  __shared__ float red[kMaxWaves * MT * kTileN];
  const int W = blockDim.x >> 6;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably wave-uniform
  const int nt = blockIdx.x;
  const int Kt = (K + kTileK - 1) / kTileK;
  Geo g;
  g.K = K;
  g.G = K / group;
  g.group = group;
  g.gshift = gshift;
  g.lane = tid & 63;
  g.n_in = g.lane & 15;
  g.qw_nt = qw + (int64_t)nt * Kt * 64 * BITS;
  g.sz_nt = qsz + (int64_t)nt * g.G * kTileN;
  g.x = x;
  // A operand: lane (m = n_in, q) supplies x row m at k = 32s + 8q + j
  g.xoff = min(g.n_in, M - 1) * K + 8 * (g.lane >> 4);
  const int kt0 = wave * tpw;
  const int nts = max(0, min(tpw, Kt - kt0));
  const int ktl = max(0, min(Kt - 1, kt0 + nts - 1));

  f4 acc = {0.f, 0.f, 0.f, 0.f};
  float yt[4] = {0.f, 0.f, 0.f, 0.f};
  gemv_body<BITS, MT, GPT, WIDE, EXACT, PF>(g, kt0, nts, ktl, acc, yt);
  if constexpr (EXACT) {
#pragma unroll
    for (int i = 0; i < 4; ++i) yt[i] = acc[i];
  }

  // combine the W partials of each (row m < MT, column n): C rows m < 4 live in lanes 0..15
  if (g.lane < kTileN) {
#pragma unroll
    for (int i = 0; i < MT && i < 4; ++i) red[(wave * MT + i) * kTileN + g.n_in] = yt[i];
  }
  __syncthreads();
  if (tid < MT * kTileN) {
    const int m = tid / kTileN, n = tid - m * kTileN;
    const int64_t row = (int64_t)nt * kTileN + n;
    float t = 0.f;
    for (int w = 0; w < W; ++w) t += red[(w * MT + m) * kTileN + n];
    if (m < M && row < N) {
      if (bias) t += (float)bias[row];
      y[(int64_t)m * N + row] = (_Float16)t;
    }
  }
}

// standalone exact dequant: one thread per lane piece -> 4 x 8 fp16 values of one row
template <int BITS, bool WIDE>
__global__ __launch_bounds__(256) void dequant_kernel(
    const uint32_t* __restrict__ qw, const uint32_t* __restrict__ qsz, _Float16* __restrict__ w,
    int64_t total_pieces, int N, int K, int group) {
  const int64_t pc = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (pc >= total_pieces) return;
  const int Kt = (K + kTileK - 1) / kTileK;
  const int lane = (int)(pc & 63);
  const int64_t tt = pc >> 6;
  const int kt = (int)(tt % Kt);
  const int64_t nt = tt / Kt;
  const int n_in = lane & 15, q = lane >> 4;
  const int64_t row = nt * kTileN + n_in;
  if (row >= N) return;
  const Piece<BITS> c = load_piece<BITS>(qw + pc * BITS);
  const Magics mg = make_magics<BITS>();
  const int G = K / group;
  auto one = [&](auto S_) {
    constexpr int S = decltype(S_)::value;
    const int k0 = kt * kTileK + 32 * S + 8 * q;
    if (k0 >= K) return;
    const uint32_t sw = qsz[sz_index(nt, k0 / group, G, n_in)];
    const GroupQ g = make_group<BITS, WIDE>(sz_scale(sw), sz_zero(sw));
    uint32_t o[4];
    dequant_step<BITS, WIDE, S>(c, mg, g, o);
    *reinterpret_cast<uint4*>(w + row * K + k0) = make_uint4(o[0], o[1], o[2], o[3]);
  };
  one(std::integral_constant<int, 0>{});
  one(std::integral_constant<int, 1>{});
  one(std::integral_constant<int, 2>{});
  one(std::integral_constant<int, 3>{});
}

bool valid_layout(int64_t N, int64_t K, int bits, int group) {
  return N >= 0 && N <= (1 << 30) && K > 0 && K % 32 == 0 && K <= (1 << 20) && group > 0 &&
         group % 32 == 0 && K % group == 0 && (bits == 2 || bits == 3 || bits == 4 || bits == 8);
}

int log2_or_neg(int v) {
  if (v <= 0 || (v & (v - 1))) return -1;
  int s = 0;
  while ((1 << s) < v) ++s;
  return s;
}

// waves per block: grow W until the grid holds ~16 waves for each of the 256 CUs
int pick_waves(int Nt, int Kt, int& tpw) {
  int W = 1;
  while (W < kMaxWaves && (int64_t)Nt * W < 4096) W *= 2;
  W = min(W, Kt);
  tpw = (Kt + W - 1) / W;
  return (Kt + tpw - 1) / tpw;
}

bool gemv_fast() {
  static const int fast = [] {
    const char* e = getenv("QLIN_GEMV_FAST");
    return (e && e[0] == '1') ? 1 : 0;
  }();
  return fast != 0;
}

template <int BITS, int MT, int GPT, bool WIDE, bool EXACT>
int launch_gemv_e(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, const uint16_t* bias,
                  uint16_t* y, int M, int N, int K, int group, hipStream_t st) {
  const int Nt = (N + kTileN - 1) / kTileN;
  const int Kt = (K + kTileK - 1) / kTileK;
  int tpw = 0;
  const int W = pick_waves(Nt, Kt, tpw);
  const int gs = log2_or_neg(group);
#define QLIN_GV(PF)                                                                        \
  hipLaunchKernelGGL((gemv_kernel<BITS, MT, GPT, WIDE, EXACT, PF>), dim3(Nt), dim3(64 * W), \
                     0, st, qw, qsz, (const _Float16*)x, (const _Float16*)bias,             \
                     (_Float16*)y, M, N, K, group, gs, tpw)
  if (tpw <= 2) QLIN_GV(2);
  else QLIN_GV(4);
#undef QLIN_GV
  return (int)hipGetLastError();
}

template <int BITS, int MT, int GPT, bool WIDE>
int launch_gemv(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, const uint16_t* bias,
                uint16_t* y, int M, int N, int K, int group, hipStream_t st) {
  if (gemv_fast())
    return launch_gemv_e<BITS, MT, GPT, WIDE, false>(qw, qsz, x, bias, y, M, N, K, group, st);
  return launch_gemv_e<BITS, MT, GPT, WIDE, true>(qw, qsz, x, bias, y, M, N, K, group, st);
}

template <int BITS, int MT, bool WIDE>
int launch_gemv_g(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, const uint16_t* bias,
                  uint16_t* y, int M, int N, int K, int group, hipStream_t st) {
  if (group % 128 == 0)
    return launch_gemv<BITS, MT, 1, WIDE>(qw, qsz, x, bias, y, M, N, K, group, st);
  if (group % 64 == 0)
    return launch_gemv<BITS, MT, 2, WIDE>(qw, qsz, x, bias, y, M, N, K, group, st);
  return launch_gemv<BITS, MT, 4, WIDE>(qw, qsz, x, bias, y, M, N, K, group, st);
}

template <int BITS, bool WIDE>
int launch_gemv_m(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, const uint16_t* bias,
                  uint16_t* y, int M, int N, int K, int group, hipStream_t st) {
  if (M == 1) return launch_gemv_g<BITS, 1, WIDE>(qw, qsz, x, bias, y, M, N, K, group, st);
  if (M == 2) return launch_gemv_g<BITS, 2, WIDE>(qw, qsz, x, bias, y, M, N, K, group, st);
  return launch_gemv_g<BITS, 4, WIDE>(qw, qsz, x, bias, y, M, N, K, group, st);
}

}  // namespace

extern "C" int qlin_dequant_f16(const uint32_t* qweight, const uint32_t* qsz, int flags, int64_t N,
                                int64_t K, int bits, int group, uint16_t* w, void* stream) {
  if (!qweight || !qsz || !w || !valid_layout(N, K, bits, group)) return QLIN_EINVAL;
  const int64_t pieces = ((N + kTileN - 1) / kTileN) * ((K + kTileK - 1) / kTileK) * 64;
  if (pieces == 0) return QLIN_OK;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)((pieces + 255) / 256));
  const bool wide = flags & QLIN_WIDE_ZERO;
#define QLIN_D(B)                                                                              \
  if (wide)                                                                                    \
    hipLaunchKernelGGL((dequant_kernel<B, true>), grid, dim3(256), 0, st, qweight, qsz,        \
                       (_Float16*)w, pieces, (int)N, (int)K, group);                           \
  else                                                                                         \
    hipLaunchKernelGGL((dequant_kernel<B, false>), grid, dim3(256), 0, st, qweight, qsz,       \
                       (_Float16*)w, pieces, (int)N, (int)K, group);                           \
  break
  switch (bits) {
    case 2: QLIN_D(2);
    case 3: QLIN_D(3);
    case 4: QLIN_D(4);
    default: QLIN_D(8);
  }
#undef QLIN_D
  return (int)hipGetLastError();
}

extern "C" int qlin_gemv_f16(const uint32_t* qweight, const uint32_t* qsz, int flags,
                             const uint16_t* x, const uint16_t* bias, uint16_t* y, int64_t M,
                             int64_t N, int64_t K, int bits, int group, void* stream) {
  if (!qweight || !qsz || !x || !y || M < 1 || M > 4 || !valid_layout(N, K, bits, group))
    return QLIN_EINVAL;
  if (N == 0) return QLIN_OK;
  hipStream_t st = (hipStream_t)stream;
  const int m = (int)M, n = (int)N, k = (int)K;
#define QLIN_G(B)                                                                   \
  return (flags & QLIN_WIDE_ZERO)                                                   \
             ? launch_gemv_m<B, true>(qweight, qsz, x, bias, y, m, n, k, group, st) \
             : launch_gemv_m<B, false>(qweight, qsz, x, bias, y, m, n, k, group, st)
  switch (bits) {
    case 2: QLIN_G(2);
    case 3: QLIN_G(3);
    case 4: QLIN_G(4);
    default: QLIN_G(8);
  }
#undef QLIN_G
}
