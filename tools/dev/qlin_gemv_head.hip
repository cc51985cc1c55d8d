// qlin_gemv.hip — fused unpack + group dequant + GEMV for decode-sized M (1..4) on the matrix
// cores (M = 1..16: the A operand's 16 rows), gfx950, plus the standalone exact dequant kernel.
//
// Replaces QuantLinear.forward -> F.linear(input, W_dq, bias) (quant/int_linear.py:48-65) on
// packed weights.  HBM-bound: every weight byte is read exactly once, with one coalesced
// 64 x (4*bits)-byte non-temporal load per 16-row x 128-k tile and one 64-byte (scale, zero) load
// per tile and group slot (qlin_common.h layout).
//
// Per wave, per k-step of 32: one v_and_or_b32 per code pair (+1 shift per word) turns the lane's
// codes into the fp16 pairs (off_j + u_j); the default (exact) path then forms W_dq bit-exactly
// ((off + u) - (off + z), times s: v_pk_add/v_pk_mul) — already the B operand of
// v_mfma_f32_16x16x32_f16 — and the MFMA contracts it with x, so the result is the reference's
// F.linear(x, W_dq) up to fp32 summation order.  (Scale-after-accumulate variants that skip the
// W_dq rounding save ~8 VALU per 8 codes but measured at most 5 % faster per launch and deviate
// ~2e-4 of the output scale from F.linear(W_dq); not kept — DESIGN.md §4.)
//
// x (A operand): one 4*MT-byte load per lane per tile brings the tile's 128 k of all M rows
// (64 lanes x 4*MT B); the wave parks it in its private LDS slot and reads the MFMA fragments
// back with ds_read_b128 — 4x fewer vector-memory instructions than fetching each k-step's
// fragment from L2 (measured -0.24 us per launch).
//
// Every global load is issued unconditionally from a wave-uniform base plus a per-lane offset
// and consumed only later, so hipcc keeps PF tiles in flight with counted vmcnt(N) waits; a
// "load or zero" select on a lane condition makes it wait vmcnt(0) at the join (measured: the
// whole prefetch serialised).
//
// Decomposition: block = one 16-row tile row (grid = ceil(N/16)); its W <= 16 waves split K (tpw
// tiles each, PF = 2 or 4 tiles in flight per wave) and combine their 16 x M partials through
// LDS.  Design measurements: tools/dev/gemv_lab.hip, DESIGN.md §4.
#include "qlin_common.h"
#include "qlin_gemv_tile.h"
#include "../../include/qlin_gfx950.h"

#include <type_traits>

using namespace qlin;

namespace qlin_gv {

constexpr int kMaxWaves = 16;

// per-token activation fake-quant of x fused into the GEMV (UniformAffineQuantizer with
// dynamic_method="per_token", quant/quantizer.py:132-159 + :94-115, as QuantLinear.forward's
// act_quantizer(input) at quant/int_linear.py:59-60): every block recomputes each row's min / max
// over K (x is L2-resident: 2 B x K per row) and fake-quantizes the x values it parks
struct ActQ {
  int on, bits, flags;
  float qmin, qmax;
};

struct Ep {  // output epilogue (qlin_common.h kEp*) and fused activation fake-quant
  const uint16_t* res;
  int ep;
  ActQ aq;
};

struct Geo {
  const uint32_t* qw_nt;  // this block's first tile row of qweight (uniform)
  const uint32_t* sz_nt;  // this block's first row tile of qsz (uniform)
  int64_t wstride, szstride;  // words between consecutive row tiles of qweight / qsz
  int jmax;                   // last valid row tile of the block, relative to its first
  const _Float16* xrow;   // x row this lane loads (row min(lane / (64/MT), M-1))
  int K, G, group, lane, n_in, xk;  // xk: the lane's first k inside a tile
  uint32_t gmagic;                   // ceil(2^31 / (group / 32)): branch-free k / group
};

// k / group for k, group multiples of 32 (k < 2^20): q = (k/32 * ceil(2^31/d)) >> 31 with
// d = group/32 is exact because the rounding term stays below 1/d (d < 2^15)
__device__ __forceinline__ int group_of(const Geo& g, int k) {
  const int gi = (int)(((uint64_t)(uint32_t)(k >> 5) * g.gmagic) >> 31);
  return min(gi, g.G - 1);
}

// row tile j of the block (clamped to its last valid tile: those loads feed outputs never stored)
template <int NTB, int BITS, int GPT>
__device__ __forceinline__ void load_w(WTile<BITS, GPT>& t, const Geo& g, int kt, int j) {
  const int jj = NTB == 1 ? 0 : min(j, g.jmax);
  t.pc = load_piece_nt<BITS>(g.qw_nt + jj * g.wstride + kt * 64 * BITS + g.lane * BITS);
#pragma unroll
  for (int i = 0; i < GPT; ++i)
    t.sz[i] = g.sz_nt[jj * g.szstride +
                      group_of(g, kt * kTileK + 32 * (i * 4 / GPT)) * kTileN + g.n_in];
}

template <int MT>
__device__ __forceinline__ void load_x(XRaw<MT>& r, const Geo& g, int kt) {
  // k clamped into the row: lanes past K (last tile only) feed k-steps that are skipped
  const int k = min(kt * kTileK + g.xk, g.K - 2 * MT);
  const _Float16* p = g.xrow + k;
  if constexpr (MT == 1) {
    r.w[0] = *reinterpret_cast<const uint32_t*>(p);
  } else if constexpr (MT == 2) {
    const uint2 v = *reinterpret_cast<const uint2*>(p);
    r.w[0] = v.x; r.w[1] = v.y;
  } else {
#pragma unroll
    for (int c = 0; c < MT / 4; ++c) {
      const uint4 v = reinterpret_cast<const uint4*>(p)[c];
      r.w[4 * c] = v.x; r.w[4 * c + 1] = v.y; r.w[4 * c + 2] = v.z; r.w[4 * c + 3] = v.w;
    }
  }
}

// park a tile's x in the wave's LDS slot (row m at words 64m .. 64m+63), read back the A
// fragments of its 4 k-steps: lane (m = n_in, q) takes row min(m, MT-1) at k = 32s + 8q .. +7
// fake-quantize the 2*MT halfs of a lane's raw x words (row `row` of x), the reference's fp16
// arithmetic (qlin_common.h fq)
template <int MT>
__device__ __forceinline__ void fake_quant_x(XRaw<MT>& r, const ActQ& aq, float sc, float zp) {
  QP P;
  P.bits = aq.bits;
  P.flags = aq.flags;
  P.qmin = aq.qmin;
  P.qmax = aq.qmax;
  const bool has_zp = !(aq.flags & QLIN_DISABLE_ZERO_POINT);
#pragma unroll
  for (int i = 0; i < MT; ++i) {
    const h2 v = as_h2(r.w[i]);
    float xi;
    const float lo = fq<_Float16>((float)v.x, sc, zp, has_zp, P, xi);
    const float hi = fq<_Float16>((float)v.y, sc, zp, has_zp, P, xi);
    r.w[i] = as_u32(h2{(_Float16)lo, (_Float16)hi});
  }
}

// NTB row tiles per block share each parked x tile (x is re-read from L2 once per block, so
// for M >= 8 a block of several row tiles cuts the x traffic that otherwise dominates)
template <int BITS, int MT, int GPT, int ZM, int PF, int NTB>
__device__ __forceinline__ void gemv_body(const Geo& g, uint32_t* xslot, int kt0, int nts,
                                          int ktl, f4 (&acc)[NTB], const ActQ& aq, float aq_sc,
                                          float aq_zp) {
  const Magics mg = make_magics<BITS>();

  // FULL: the tile is not the matrix's last (only that one can hold fewer than 4 k-steps)
  auto step = [&](const WTile<BITS, GPT>& t, f4& ac, const h8 (&xa)[4], int kt, auto S_,
                  auto FULL_) {
    constexpr int S = decltype(S_)::value;
    constexpr bool FULL = decltype(FULL_)::value;
    constexpr int slot = S * GPT / 4;
    const int k0 = kt * kTileK + 32 * S;
    if (FULL || k0 < g.K) {  // wave-uniform
      uint32_t v[4];
      const GroupQ gq = make_group_w<BITS, ZM>(t.sz[slot]);
      dequant_step<BITS, ZM, S>(t.pc, mg, gq, v);
      const h8 b = __builtin_bit_cast(h8, make_uint4(v[0], v[1], v[2], v[3]));
      ac = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa[S], b, ac, 0, 0, 0);
    }
  };
  // live == false: a slot past the wave's tiles (a repeat of its last tile), computed on x zeroed
  auto tile = [&](const WTile<BITS, GPT> (&t)[NTB], XRaw<MT>& xr, int kt, auto FULL_, bool live) {
    h8 xa[4];
    if (aq.on) fake_quant_x<MT>(xr, aq, aq_sc, aq_zp);  // wave-uniform
    if (!live) {  // wave-uniform
#pragma unroll
      for (int c = 0; c < MT; ++c) xr.w[c] = 0u;
    }
    park_x<MT>(xa, xr, xslot, g.lane, g.n_in);
#pragma unroll
    for (int j = 0; j < NTB; ++j) {
      step(t[j], acc[j], xa, kt, std::integral_constant<int, 0>{}, FULL_);
      step(t[j], acc[j], xa, kt, std::integral_constant<int, 1>{}, FULL_);
      step(t[j], acc[j], xa, kt, std::integral_constant<int, 2>{}, FULL_);
      step(t[j], acc[j], xa, kt, std::integral_constant<int, 3>{}, FULL_);
    }
  };

  // prologue: PF tiles (codes, (scale, zero), x) in flight, tile index clamped to the wave's last
  WTile<BITS, GPT> wt[PF][NTB];
  XRaw<MT> xq[PF];
#pragma unroll
  for (int u = 0; u < PF; ++u) {
    load_x<MT>(xq[u], g, min(kt0 + u, ktl));
#pragma unroll
    for (int j = 0; j < NTB; ++j) load_w<NTB>(wt[u][j], g, min(kt0 + u, ktl), j);
  }

  // full rounds of PF tiles: compute tile t, refill its slot with tile t + PF
  int t0 = 0;
  for (; t0 + PF < nts; t0 += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const int kt = kt0 + t0 + u;
      tile(wt[u], xq[u], kt, std::true_type{}, true);
      load_x<MT>(xq[u], g, min(kt + PF, ktl));
#pragma unroll
      for (int j = 0; j < NTB; ++j) load_w<NTB>(wt[u][j], g, min(kt + PF, ktl), j);
    }
  }
  // last round (1..PF tiles): compute only; a tile short of K (the matrix's last) takes the
  // per-k-step checks, every other one the straight-line body.  Slots past the wave's tiles are
  // computed too (their clamped repeat on x zeroed): under an `if (live)` the compiler sinks
  // their loads into the branch, i.e. behind the earlier slots' dequant
#pragma unroll
  for (int u = 0; u < PF; ++u) {
    const int kt = kt0 + t0 + u;
    const bool live = t0 + u < nts;  // wave-uniform
    if (!live || (kt + 1) * kTileK <= g.K) tile(wt[u], xq[u], kt, std::true_type{}, live);
    else tile(wt[u], xq[u], kt, std::false_type{}, true);
  }

}

template <int BITS, int MT, int GPT, int ZM, int PF, int NTB = 1>
__global__ __launch_bounds__(1024) void gemv_kernel(
    const uint32_t* __restrict__ qw, const uint32_t* __restrict__ qsz,
    const _Float16* __restrict__ x, const _Float16* __restrict__ bias, _Float16* __restrict__ y,
    int M, int N, int K, int group, uint32_t gmagic, int tpw, const _Float16* __restrict__ res,
    int ep, ActQ aq) {
  __shared__ __attribute__((aligned(16))) float red[NTB * MT * kTileN * kMaxWaves];
  __shared__ __attribute__((aligned(16))) uint32_t xs[kMaxWaves][64 * MT];
  __shared__ float aq_s[2][MT];
  const int W = blockDim.x >> 6;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // provably wave-uniform
  const int nt = blockIdx.x * NTB;  // first row tile of the block
  const int Kt = (K + kTileK - 1) / kTileK;
  Geo g;
  g.K = K;
  g.G = K / group;
  g.group = group;
  g.gmagic = gmagic;
  g.lane = tid & 63;
  g.n_in = g.lane & 15;
  g.qw_nt = qw + (int64_t)nt * Kt * 64 * BITS;
  g.sz_nt = qsz + (int64_t)nt * g.G * kTileN;
  g.wstride = (int64_t)Kt * 64 * BITS;
  g.szstride = (int64_t)g.G * kTileN;
  g.jmax = min(NTB, (N + kTileN - 1) / kTileN - nt) - 1;
  constexpr int LPR = 64 / MT;  // lanes per x row
  g.xrow = x + (int64_t)min(g.lane / LPR, M - 1) * K;
  g.xk = 2 * MT * (g.lane % LPR);
  const int kt0 = wave * tpw;
  const int nts = max(0, min(tpw, Kt - kt0));
  const int ktl = max(0, min(Kt - 1, kt0 + nts - 1));

  float aq_sc = 0.f, aq_zp = 0.f;
  if (aq.on) {  // per-row (token) min / max over K, then the reference's calibration
#pragma clang fp contract(off)
    float* mm = red;  // [MT][2][kMaxWaves] scratch, free until the partial sums
    const int nch = K >> 3;
    for (int m = 0; m < M; ++m) {
      float mn = __builtin_inff(), mx = -__builtin_inff();
      for (int c = tid; c < nch; c += blockDim.x) {
        const h8 v = __builtin_bit_cast(h8, reinterpret_cast<const uint4*>(x + (int64_t)m * K)[c]);
#pragma unroll
        for (int j = 0; j < 8; ++j) { mn = min_nan(mn, (float)v[j]); mx = max_nan(mx, (float)v[j]); }
      }
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        mn = min_nan(mn, __shfl_xor(mn, o));
        mx = max_nan(mx, __shfl_xor(mx, o));
      }
      if (g.lane == 0) { mm[(m * 2) * kMaxWaves + wave] = mn; mm[(m * 2 + 1) * kMaxWaves + wave] = mx; }
    }
    __syncthreads();
    if (tid < M) {
      float mn = mm[(tid * 2) * kMaxWaves], mx = mm[(tid * 2 + 1) * kMaxWaves];
      for (int w = 1; w < W; ++w) {
        mn = min_nan(mn, mm[(tid * 2) * kMaxWaves + w]);
        mx = max_nan(mx, mm[(tid * 2 + 1) * kMaxWaves + w]);
      }
      QP P;
      P.bits = aq.bits;
      P.flags = aq.flags;
      P.qmin = aq.qmin;
      P.qmax = aq.qmax;
      float sc, zp;
      calib<_Float16>((float)(_Float16)mn, (float)(_Float16)mx, 1.f, 1.f, P, sc, zp);
      aq_s[0][tid] = sc;
      aq_s[1][tid] = zp;
    }
    __syncthreads();
    const int r = min(g.lane / (64 / MT), M - 1);  // the x row this lane parks
    aq_sc = aq_s[0][r];
    aq_zp = aq_s[1][r];
  }

  f4 acc[NTB];
#pragma unroll
  for (int j = 0; j < NTB; ++j) acc[j] = f4{0.f, 0.f, 0.f, 0.f};
  gemv_body<BITS, MT, GPT, ZM, PF, NTB>(g, &xs[wave][0], kt0, nts, ktl, acc, aq, aq_sc, aq_zp);

  // combine the W partials of each (row m < MT, column n): C row m = 4q + i sits in lane
  // n + 16q, element i; layout [m][n][wave] so one thread reads its 16 partials with 4
  // ds_read_b128
  // (row tile j of the block: [j][m][n][wave])
  const int q4 = 4 * (g.lane >> 4);
  if (q4 < MT) {
#pragma unroll
    for (int j = 0; j < NTB; ++j) {
      float* rj = red + j * MT * kTileN * kMaxWaves;
#pragma unroll
      for (int i = 0; i < 4 && i < MT; ++i)
        rj[((q4 + i) * kTileN + g.n_in) * kMaxWaves + wave] = acc[j][i];
      if (wave == 0) {
        for (int w = W; w < kMaxWaves; ++w)
#pragma unroll
          for (int i = 0; i < 4 && i < MT; ++i)
            rj[((q4 + i) * kTileN + g.n_in) * kMaxWaves + w] = 0.f;
      }
    }
  }
  __syncthreads();
  // MT * 16 outputs; a block of W < MT / 4 waves (short K) loops
  auto total = [&](int o, int64_t row) {
    const f4* r = reinterpret_cast<const f4*>(red + o * kMaxWaves);
    const f4 a = r[0], b = r[1], c = r[2], d = r[3];
    const f4 e = (a + b) + (c + d);
    float t = (e[0] + e[1]) + (e[2] + e[3]);
    if (bias) t += (float)bias[row];
    return (float)(_Float16)t;  // F.linear's fp16 output
  };
  if (ep == kEpSiluMul) {  // N even, interleaved halves: 8 outputs per tile and row m
    for (int o = tid; o < NTB * MT * 8; o += blockDim.x) {
      const int j = o / (MT * 8), oo = o - j * MT * 8;
      const int m = oo >> 3, n = oo & 7;
      const int64_t ntj = (int64_t)nt + j;
      const int64_t row = ntj * kTileN + n;
      const int b = j * MT * kTileN;
      if (m < M && row + 8 < N) {
        const float g = total(b + m * kTileN + n, row), u = total(b + m * kTileN + n + 8, row + 8);
        y[(int64_t)m * (N >> 1) + ntj * 8 + n] = (_Float16)(silu_rn16(g) * u);
      }
    }
    return;
  }
  for (int o = tid; o < NTB * MT * kTileN; o += blockDim.x) {
    const int j = o / (MT * kTileN), oo = o - j * MT * kTileN;
    const int m = oo / kTileN, n = oo - m * kTileN;
    const int64_t row = ((int64_t)nt + j) * kTileN + n;
    if (m < M && row < N) {
      float t = total(o, row);
      if (ep == kEpResidual) t += (float)res[(int64_t)m * N + row];
      y[(int64_t)m * N + row] = (_Float16)t;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Decode path, one token row (M == 1): the persistent "rows" kernel.
//
// QuantLinear.forward -> F.linear(x, W_dq) (quant/int_linear.py:62 of the reference) for one
// token, optionally with the decoder layer's RMSNorm in front (OmniLlamaRMSNorm,
// quant/omni_norm.py:52-63: input_layernorm -> q/k/v, post_attention_layernorm -> gate/up) and
// its glue behind (residual add, SiLU * up; models/int_llama_layer.py:44-45, :241-257).
//
// Decomposition (the single-launch analogue of the batched streaming kernel,
// qlin_gemv_batched.hip): block b owns the 16-row tile rows b, b + nb, b + 2 nb, ...; its W waves
// split K, wave w taking the same TPW k-tiles of every row (W * TPW == Kt).  A wave therefore
// loads its x words ONCE per launch (parked in its LDS slots, read back as MFMA A fragments for
// every row) and streams its weight tiles row after row with PF tiles in flight across row
// boundaries: no block ever waits between rows, and a grid of one block per CU keeps every CU
// streaming until the matrix is done (gate/up, 1,792 tile rows: 7 rows per block).  Each row's
// W partial 16-vectors meet in LDS behind a bare s_barrier (no vmcnt drain: the next rows' tiles
// stay in flight) and one wave applies the epilogue.  Row r's output is sum_w (MFMA chain of
// wave w over its k-tiles), the W partials added in a fixed tree order: deterministic.
//
// RMSNorm (nrm): each wave sums the squares of its own x words (the waves cover the row once), the
// W sums meet in LDS (bare s_barrier, fixed order), and every x word is normalised as the
// reference rounds it — x_hat = RN16(weight * (x * rsqrt(mean(x^2) + eps))), fp32 inside — before
// it is parked: the linear then multiplies exactly the reference's normed fp16 row (up to the
// fp32 ulp of the statistics' summation order).  The norm runs once per block, not per row.
//
// Every global load is unconditional (clamped indices) except the last round's refills, so the
// compiler counts them with vmcnt(N): x words first, then the first PF tiles' codes and
// (scale, zero) words; the x wait does not wait for the weights.
// ---------------------------------------------------------------------------------------------
// Measured and not kept (round-4 dev builds): (scale, zero) words issued before each tile's
// codes; __syncthreads() at the row barrier (drains vmcnt); a dynamic-LDS floor admitting one
// block per CU.  Wave w streams k-tiles w*TPW .. (w+1)*TPW - 1 when TPW = 8 (down 8.25 vs 8.39 us
// strided), else k-tiles w, w + W, ... (4096^2 3.86 vs 4.02 us contiguous).
constexpr int kRowsBpc = 2;  // resident blocks per CU of a persistent (multi-row) launch
constexpr int kRowsMaxTPW = 8;  // k-tiles per wave and row

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

struct RowsArgs {
  const uint32_t* qw;   // tile row 0 of qweight
  const uint32_t* qsz;  // tile row 0 of qsz
  const _Float16* x;
  const _Float16* bias;
  const _Float16* res;  // kEpResidual
  _Float16* y;
  const void* nw;       // NRM: RMSNorm weight [K], fp32 or fp16 (kNwF32 / kNwF16)
  float eps;
  int ep, has_bias;     // bias / res always readable (the host points absent ones at y)
  int64_t nres;         // readable elements at res
  int N, K, Kt, G;
  int W;                // waves per block (W * TPW == Kt)
  int nb, rpb, extra;   // blocks; block b owns rpb + (b < extra) tile rows b, b + nb, ...
  int64_t wstep, sstep; // qweight / qsz words between two rows of a block (nb tile rows)
  uint32_t cmagic;      // GPT == 1: kt / (group / 128) = (kt * cmagic) >> 31
};

template <int BITS, int GPT, int ZM, int TPW, int PF, int NRM>
__global__ __launch_bounds__(1024) void gemv_rows_kernel(const RowsArgs a) {
  __shared__ __attribute__((aligned(16))) uint32_t xs[kMaxWaves][TPW * 64];  // the wave's x words
  __shared__ __attribute__((aligned(16))) float red[2][kTileN][kMaxWaves];   // row partials
  __shared__ float nss[NRM ? kMaxWaves : 1];                                 // sums of squares
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, n_in = lane & 15;
  const int b = blockIdx.x;
  const int nrows = a.rpb + (b < a.extra ? 1 : 0);
  const int T = nrows * TPW;  // tiles this wave streams (host: T >= PF)
  constexpr bool kContig = TPW >= 8;
  const int kt0 = kContig ? wave * TPW : wave;
  const int kts = kContig ? 1 : a.W;
  auto group_of_tile = [&](int kt) {
    return GPT == 1 ? (int)(((uint64_t)(uint32_t)kt * a.cmagic) >> 31) : kt * GPT;
  };

  // x words of this wave's k-tiles (lane l: k = 128 kt + 2l, 2l + 1), the same for every row;
  // issued first (in-order completion: their wait does not wait for the weights)
  const _Float16* xp = a.x + kt0 * kTileK + 2 * lane;
  uint32_t xw[TPW];
  NwPair<NRM> nwv[NRM ? TPW : 1];
#pragma unroll
  for (int i = 0; i < TPW; ++i) xw[i] = *reinterpret_cast<const uint32_t*>(xp + i * kts * kTileK);
  if constexpr (NRM) {
#pragma unroll
    for (int i = 0; i < TPW; ++i)
      nwv[i] = load_nw_pair<NRM>(a.nw, (kt0 + i * kts) * kTileK + 2 * lane);
  }

  // the epilogue operands of the first row this wave finishes (the epilogue of a block's j-th row
  // runs on wave j % W: wave w's first is row w): loaded unconditionally (the host points absent
  // operands at a readable buffer, never used) ahead of the weights, so no tile waits for them
  const int NO = a.ep == kEpSiluMul ? 8 : kTileN;  // outputs per row
  const int on = min(lane, NO - 1);
  _Float16 ob0, ob1, ores;
  auto load_epi = [&](int j) {
    const int64_t row = (int64_t)(b + min(j, nrows - 1) * a.nb) * kTileN + on;
    const int64_t nb_ = a.has_bias ? (int64_t)a.N : a.nres;  // readable bias elements
    ob0 = a.bias[min(row, nb_ - 1)];
    ob1 = a.bias[min(row + 8, nb_ - 1)];
    ores = a.res[min(row, a.nres - 1)];
  };
  load_epi(wave);

  // weight stream: the load cursor (row offset lq / ls, k-tile il) runs PF tiles ahead
  WTile<BITS, GPT> wt[PF];
  const uint32_t* qwp = a.qw + ((int64_t)b * a.Kt + kt0) * (64 * BITS) + lane * BITS;
  const uint32_t* szp = a.qsz + (int64_t)b * a.G * kTileN + n_in;
  int il = 0;
  int64_t lq = 0, ls = 0;
  auto load = [&](int u) {
    const int ki = il * kts;  // k-tile offset from kt0
    const int g0 = group_of_tile(kt0 + ki);
    wt[u].pc = load_piece_nt<BITS>(qwp + lq + ki * (64 * BITS));
#pragma unroll
    for (int s = 0; s < GPT; ++s) wt[u].sz[s] = szp[ls + (g0 + s) * kTileN];
    if (++il == TPW) {
      il = 0;
      lq += a.wstep;
      ls += a.sstep;
    }
  };
#pragma unroll
  for (int u = 0; u < PF; ++u) load(u);


  if constexpr (NRM) {
#pragma clang fp contract(off)
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const h2 v = as_h2(xw[i]);
      const float f0 = (float)v.x, f1 = (float)v.y;
      ss = ss + f0 * f0;
      ss = ss + f1 * f1;
    }
    ss = wave_sum(ss);
    if (lane == 0) nss[wave] = ss;
    // a bare s_barrier: __syncthreads() would also wait for the weight tiles in flight
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    float tot = 0.f;
    for (int w = 0; w < a.W; ++w) tot += nss[w];
    const float rn = rsqrtf(tot / (float)a.K + a.eps);
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const h2 v = as_h2(xw[i]);
      const float2 w = nw_pair_f32<NRM>(nwv[i]);
      const float n0 = w.x * ((float)v.x * rn);
      const float n1 = w.y * ((float)v.y * rn);
      xw[i] = as_u32(h2{(_Float16)n0, (_Float16)n1});
    }
  }
  uint32_t* xsl = &xs[wave][0];
#pragma unroll
  for (int i = 0; i < TPW; ++i) xsl[i * 64 + lane] = xw[i];

  const Magics mg = make_magics<BITS>();
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  int ic = 0, jc = 0, ew = 0, par = 0;  // compute cursor, epilogue wave, partial buffer
  auto epilogue = [&]() {
    if (lane < kTileN) red[par][lane][wave] = acc[0];
    acc = f4{0.f, 0.f, 0.f, 0.f};
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (wave == ew) {  // wave-uniform
      const int64_t r = (int64_t)b + (int64_t)jc * a.nb;
      auto total = [&](int n, _Float16 bv) {  // the W partials in a fixed tree order
        const f4* p = reinterpret_cast<const f4*>(&red[par][n][0]);
        f4 q[4] = {p[0], p[1], p[2], p[3]};
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int e = 0; e < 4; ++e) q[c][e] = 4 * c + e < a.W ? q[c][e] : 0.f;  // absent waves
        const f4 e4 = (q[0] + q[1]) + (q[2] + q[3]);
        float t = (e4[0] + e4[1]) + (e4[2] + e4[3]);
        if (a.has_bias) t += (float)bv;
        return (float)(_Float16)t;  // F.linear's fp16 output
      };
      if (lane < NO) {
        if (a.ep == kEpSiluMul) {
          if (r * kTileN + lane + 8 < a.N)
            a.y[r * 8 + lane] = (_Float16)(silu_rn16(total(lane, ob0)) * total(lane + 8, ob1));
        } else if (r * kTileN + lane < a.N) {
          float t = total(lane, ob0);
          if (a.ep == kEpResidual) t += (float)ores;
          a.y[r * kTileN + lane] = (_Float16)t;
        }
      }
      if (jc + a.W < nrows) load_epi(jc + a.W);  // this wave's next epilogue row (multi-row)
    }
    if (++ew == a.W) ew = 0;
    par ^= 1;
  };
  auto compute = [&](int u) {
    const uint4* xb = reinterpret_cast<const uint4*>(xsl + ic * 64) + (lane >> 4);
    h8 xa[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) xa[s] = __builtin_bit_cast(h8, xb[4 * s]);
    auto step = [&](auto S_) {
      constexpr int S = decltype(S_)::value;
      uint32_t v[4];
      const GroupQ gq = make_group_w<BITS, ZM>(wt[u].sz[S * GPT / 4]);
      dequant_step<BITS, ZM, S>(wt[u].pc, mg, gq, v);
      const h8 bb = __builtin_bit_cast(h8, make_uint4(v[0], v[1], v[2], v[3]));
      acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa[S], bb, acc, 0, 0, 0);
    };
    step(std::integral_constant<int, 0>{});
    step(std::integral_constant<int, 1>{});
    step(std::integral_constant<int, 2>{});
    step(std::integral_constant<int, 3>{});
    if (++ic == TPW) {  // block-uniform: the row is complete in every wave
      epilogue();
      ic = 0;
      ++jc;
    }
  };

  // rounds of PF tiles; every refill of all but the last full round is in range
  const int Q = T / PF;  // >= 1
  for (int q = 0; q + 1 < Q; ++q) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      compute(u);
      load(u);
    }
  }
  const int rem = T - Q * PF;  // tiles after the last full round (< PF)
#pragma unroll
  for (int u = 0; u < PF; ++u) {
    compute(u);
    if (u < rem) load(u);
  }
#pragma unroll
  for (int u = 0; u < PF; ++u)
    if (u < rem) compute(u);
}

// ---------------------------------------------------------------------------------------------
// Decode path for wide matrices (one token row, >= 4 tile rows per CU): the work-queue kernel.
//
// One 8-wave block per CU owns the tile rows b, b + nb, b + 2 nb, ... (gate/up: 1,792 rows, 7 per
// CU).  Their tiles form chunks of kWqC = 4 consecutive k-tiles of one row; the waves take chunks
// from a counter in LDS (the first kWqD each statically), keep kWqD chunks of loads in flight
// (codes nt-loaded to registers, the chunk's (scale, zero) words with ONE load per chunk), and
// store each chunk's 16 partial sums in LDS; after one block barrier every row's chunks are added
// in k order (deterministic: the same order whatever wave ran which chunk) and the epilogue is
// applied.  Why a queue: with whole rows per wave (round 4's kernel) the second wave of each SIMD
// finished ~3 us after the first — the CU serves its waves' requests oldest first, so statically
// equal shares end unequally; waves that are served sooner now simply take more chunks
// (tools/dev/wq_lab.hip: gate/up + norm + SiLU 17.0 -> 14.3-15.3 us per launch, one box).
//
// x is staged once per block in LDS (16-B chunks; with the RMSNorm normalised there at the
// reference's rounding point after one block reduction of the sum of squares), and every A
// fragment is a broadcast ds_read_b128 of it.  A chunk's (scale, zero) words go through a per-wave
// LDS slot (one ds_write, then one ds_read_b32 per tile and group slot).
// ---------------------------------------------------------------------------------------------
constexpr int kWqWaves = 8;  // waves per block (one block per CU)
constexpr int kWqC = 4;      // k-tiles per chunk
constexpr int kWqD = 2;      // chunks in flight per wave

struct WrowArgs {
  const uint32_t* qw;
  const uint32_t* qsz;
  const _Float16* x;
  const _Float16* bias;
  const _Float16* res;
  _Float16* y;
  const void* nw;       // NRM: RMSNorm weight [K], fp32 or fp16 (kNwF32 / kNwF16)
  float eps;
  int ep, has_bias;     // bias / res always readable (the host points absent ones at y)
  int64_t nres;         // readable elements at res
  int N, K, Kt, G, Nt;
  int nb, CPR;          // blocks (block b: rows b, b + nb, ...); chunks per row (Kt / kWqC)
  int part_off, sz_off, misc_off;  // LDS byte offsets (x staging at 0)
  uint32_t cmagic;
};

// LDS bytes of a launch: x (fp16 [K]) | partials [rows x CPR][16] fp32 | (scale, zero) slots
// [waves][kWqD][64 GPT] words | the wave sums of squares [8] and the chunk counter
inline void wq_lds_layout(int K, int max_rows, int CPR, int GPT, int& part_off, int& sz_off,
                          int& misc_off, int& total) {
  part_off = (K * 2 + 15) / 16 * 16;
  sz_off = part_off + max_rows * CPR * kTileN * 4;
  misc_off = sz_off + kWqWaves * kWqD * 64 * GPT * 4;
  total = misc_off + (kWqWaves + 4) * 4;
}

template <int BITS, int GPT, int ZM, int NRM, int XI>
__global__ __launch_bounds__(64 * kWqWaves) void gemv_wq_kernel(const WrowArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];  // ONE LDS object
  uint4* xs4 = reinterpret_cast<uint4*>(lds);
  float* part = reinterpret_cast<float*>(lds + a.part_off);
  uint32_t* szs = reinterpret_cast<uint32_t*>(lds + a.sz_off);
  float* nss = reinterpret_cast<float*>(lds + a.misc_off);
  int* ctr = reinterpret_cast<int*>(lds + a.misc_off) + kWqWaves;
  constexpr int nthr = 64 * kWqWaves, C = kWqC, D = kWqD;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, n_in = lane & 15, q = lane >> 4;
  const int b = blockIdx.x;
  const int nrows = b < a.Nt ? (a.Nt - 1 - b) / a.nb + 1 : 0;
  const int CPR = a.CPR;
  const int NC = nrows * CPR;  // chunks of this block
  auto group_of_tile = [&](int kt) {
    return GPT == 1 ? (int)(((uint64_t)(uint32_t)kt * a.cmagic) >> 31) : kt * GPT;
  };

  // x chunks of this thread (clamped: repeats are never stored) and their norm weights, issued
  // first
  const int nch = a.K >> 3;
  uint4 xc[XI];
  float4 nc[NRM ? 2 * XI : 1];  // two float4 (fp32 weights) or one uint4 of fp16 (kNwF16)
#pragma unroll
  for (int i = 0; i < XI; ++i) {
    const int c = min(tid + i * nthr, nch - 1);
    xc[i] = reinterpret_cast<const uint4*>(a.x)[c];
    if constexpr (NRM == kNwF16) {
      nc[2 * i] = __builtin_bit_cast(float4, reinterpret_cast<const uint4*>(a.nw)[c]);
    } else if constexpr (NRM) {
      nc[2 * i] = reinterpret_cast<const float4*>(a.nw)[2 * c];
      nc[2 * i + 1] = reinterpret_cast<const float4*>(a.nw)[2 * c + 1];
    }
  }
  // the epilogue operands of this thread's first output (output o = tid: row o / 16, column
  // o % 16; SiLU: o / 8, o % 8), loaded unconditionally ahead of the weights
  const int NO = a.ep == kEpSiluMul ? 8 : kTileN;  // outputs per row
  auto out_row = [&](int o) { return (int64_t)b + (int64_t)(o / NO) * a.nb; };
  const int64_t nbias = a.has_bias ? (int64_t)a.N : a.nres;  // readable bias elements
  _Float16 ob0, ob1, ores;
  auto load_epi = [&](int o) {
    const int64_t row = min(out_row(o), (int64_t)a.Nt - 1) * kTileN + o % NO;
    ob0 = a.bias[min(row, nbias - 1)];
    ob1 = a.bias[min(row + 8, nbias - 1)];
    ores = a.res[min(row, a.nres - 1)];
  };
  load_epi(tid);
  asm volatile("" ::: "memory");  // the x / norm-weight / epilogue requests go out first

  // chunk loads: (scale, zero) words first (GPT per lane: lane l holds words GPT l .. GPT l + GPT
  // - 1 of the chunk's 64 GPT), then the C tiles' codes; a chunk past the block's last (a wave's
  // final prefetches) reads the block's first chunk again (L2-hot, never used)
  const int64_t wrow = (int64_t)a.Kt * (64 * BITS), srow = (int64_t)a.G * kTileN;
  Piece<BITS> wt[D][C];
  uint32_t szc[D][GPT];
  int gb[D];  // GPT == 1: the chunk's first group
  auto load_chunk = [&](auto SET_, int c) {
    constexpr int d = decltype(SET_)::value;
    if (c >= NC) c = 0;
    const int j = c / CPR, kt0 = (c - j * CPR) * C;
    const int64_t r = (int64_t)b + (int64_t)j * a.nb;
    const uint32_t* sp = a.qsz + r * srow;
    if constexpr (GPT == 1) {
      gb[d] = group_of_tile(kt0);
      szc[d][0] = sp[min(gb[d] + (lane >> 4), a.G - 1) * kTileN + n_in];
    } else if constexpr (GPT == 2) {
      const uint2 v = *reinterpret_cast<const uint2*>(sp + (int64_t)kt0 * GPT * kTileN + 2 * lane);
      szc[d][0] = v.x;
      szc[d][1] = v.y;
    } else {
      const uint4 v = *reinterpret_cast<const uint4*>(sp + (int64_t)kt0 * GPT * kTileN + 4 * lane);
      szc[d][0] = v.x;
      szc[d][1] = v.y;
      szc[d][2] = v.z;
      szc[d][3] = v.w;
    }
    const uint32_t* qp = a.qw + r * wrow + (int64_t)kt0 * (64 * BITS) + lane * BITS;
#pragma unroll
    for (int u = 0; u < C; ++u) wt[d][u] = load_piece_nt<BITS>(qp + u * (64 * BITS));
  };
  load_chunk(std::integral_constant<int, 0>{}, wave);
  load_chunk(std::integral_constant<int, 1>{}, wave + kWqWaves);
  if (tid == 0) *ctr = D * kWqWaves;

  // stage x (normed) in LDS: one block reduction for the statistics, one barrier
  if constexpr (NRM) {
#pragma clang fp contract(off)
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const h8 v = __builtin_bit_cast(h8, xc[i]);
      float s8 = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) s8 = s8 + (float)v[e] * (float)v[e];
      ss = ss + (tid + i * nthr < nch ? s8 : 0.f);
    }
    ss = wave_sum(ss);
    if (lane == 0) nss[wave] = ss;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    float tot = 0.f;
#pragma unroll
    for (int w = 0; w < kWqWaves; ++w) tot += nss[w];
    const float rn = rsqrtf(tot / (float)a.K + a.eps);
#pragma unroll
    for (int i = 0; i < XI; ++i) {
      const h8 v = __builtin_bit_cast(h8, xc[i]);
      float w8[8];
      if constexpr (NRM == kNwF16) {
        const h8 h = __builtin_bit_cast(h8, nc[2 * i]);
#pragma unroll
        for (int e = 0; e < 8; ++e) w8[e] = (float)h[e];
      } else {
        const float t8[8] = {nc[2 * i].x, nc[2 * i].y, nc[2 * i].z, nc[2 * i].w,
                             nc[2 * i + 1].x, nc[2 * i + 1].y, nc[2 * i + 1].z, nc[2 * i + 1].w};
#pragma unroll
        for (int e = 0; e < 8; ++e) w8[e] = t8[e];
      }
      h8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (_Float16)(w8[e] * ((float)v[e] * rn));
      xc[i] = __builtin_bit_cast(uint4, o);
    }
  }
#pragma unroll
  for (int i = 0; i < XI; ++i)
    if (tid + i * nthr < nch) xs4[tid + i * nthr] = xc[i];
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

  const Magics mg = make_magics<BITS>();
  uint32_t* wsz = szs + wave * (D * 64 * GPT);  // this wave's (scale, zero) slots
  int cs[D] = {wave, wave + kWqWaves};
  // compute the chunk in set d, prefetching the next chunk from the queue into the same set
  auto run = [&](auto SET_) {
    constexpr int d = decltype(SET_)::value;
    const int c = cs[d];
    if (c >= NC) return false;  // wave-uniform
    int cn = 0;
    if (lane == 0)
      cn = __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    cn = __builtin_amdgcn_readfirstlane(cn);
    const int j = c / CPR, kc = c - j * CPR;
    const int g0 = GPT == 1 ? gb[d] : 0;
    uint32_t* slot = wsz + d * (64 * GPT);
#pragma unroll
    for (int i = 0; i < GPT; ++i) slot[GPT * lane + i] = szc[d][i];
    f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int u = 0; u < C; ++u) {
      const int kt = kc * C + u;
      h8 xa[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) xa[s] = __builtin_bit_cast(h8, xs4[kt * 16 + 4 * s + q]);
      uint32_t sw[GPT];
#pragma unroll
      for (int i = 0; i < GPT; ++i)
        sw[i] = GPT == 1 ? slot[(group_of_tile(kt) - g0) * kTileN + n_in]
                         : slot[(GPT * u + i) * kTileN + n_in];
      auto step = [&](auto S_) {
        constexpr int S = decltype(S_)::value;
        uint32_t v[4];
        const GroupQ gq = make_group_w<BITS, ZM>(sw[S * GPT / 4]);
        dequant_step<BITS, ZM, S>(wt[d][u], mg, gq, v);
        const h8 bb = __builtin_bit_cast(h8, make_uint4(v[0], v[1], v[2], v[3]));
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa[S], bb, acc, 0, 0, 0);
      };
      step(std::integral_constant<int, 0>{});
      step(std::integral_constant<int, 1>{});
      step(std::integral_constant<int, 2>{});
      step(std::integral_constant<int, 3>{});
    }
    load_chunk(SET_, cn);  // the set's registers are free again
    cs[d] = cn;
    if (lane < kTileN) part[(j * CPR + kc) * kTileN + lane] = acc[0];  // C row 0, column lane
    return true;
  };
  for (;;) {
    if (!run(std::integral_constant<int, 0>{})) break;
    if (!run(std::integral_constant<int, 1>{})) break;
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

  // every row: its chunks' partials in k order, then F.linear's fp16 output and the epilogue
  for (int o = tid; o < nrows * NO; o += nthr) {
    if (o != tid) load_epi(o);
    const int64_t r = out_row(o);
    const int n = o % NO;
    auto total = [&](int nn, _Float16 bv) {
      const float* p = part + (int64_t)(o / NO) * CPR * kTileN + nn;
      float t = 0.f;
      for (int kc = 0; kc < CPR; ++kc) t += p[kc * kTileN];
      if (a.has_bias) t += (float)bv;
      return (float)(_Float16)t;
    };
    if (a.ep == kEpSiluMul) {
      if (r * kTileN + n + 8 < a.N) a.y[r * 8 + n] = (_Float16)(silu_rn16(total(n, ob0)) * total(n + 8, ob1));
    } else if (r * kTileN + n < a.N) {
      float t = total(n, ob0);
      if (a.ep == kEpResidual) t += (float)ores;
      a.y[r * kTileN + n] = (_Float16)t;
    }
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

template <int BITS, int MT, int GPT, int ZM, int EP, int PF, int NRM = 0>
__global__ __launch_bounds__(1024) void gemv_fast_kernel(const FastArgs a) {
  __shared__ __attribute__((aligned(16))) float red[MT * kTileN * kMaxWaves];
  __shared__ __attribute__((aligned(16))) uint32_t xs[kMaxWaves][64 * MT];
  __shared__ float nss[NRM ? kMaxWaves : 1];  // NRM: per-wave sums of squares
  static_assert(!NRM || MT == 1, "the fused RMSNorm serves one token row");
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, n_in = lane & 15;
  const int nt = blockIdx.x;
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

// standalone exact dequant: one thread per lane piece -> 4 x 8 fp16 values of one row
template <int BITS, int ZM>
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
    const GroupQ g = make_group_w<BITS, ZM>(sw);
    uint32_t o[4];
    dequant_step<BITS, ZM, S>(c, mg, g, o);
    *reinterpret_cast<uint4*>(w + row * K + k0) = make_uint4(o[0], o[1], o[2], o[3]);
  };
  one(std::integral_constant<int, 0>{});
  one(std::integral_constant<int, 1>{});
  one(std::integral_constant<int, 2>{});
  one(std::integral_constant<int, 3>{});
}

static inline uint32_t group_magic(int group) {
  const uint64_t d = (uint64_t)(group / 32);
  return (uint32_t)(((1ull << 31) + d - 1) / d);
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

template <int BITS, int MT, int GPT, int ZM>
int launch_gemv(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, const uint16_t* bias,
                  uint16_t* y, int M, int N, int K, int group, hipStream_t st, const Ep& e) {
  const int Nt = (N + kTileN - 1) / kTileN;
  const int Kt = (K + kTileK - 1) / kTileK;
  // 8-16 token rows on a wide matrix: two row tiles per block share each parked x tile (x is
  // re-read from L2 per block); measured (tools/dev/gemv_geo.py) 14336 x 4096, M = 16: 24.5 ->
  // 15.7 us, M = 8: 12.0 -> 10.2 us; no gain at N = 4096 and for M <= 4, so those keep one
  const int ntb = (MT >= 8 && Nt >= 512) ? 2 : 1;
  const int blocks = (Nt + ntb - 1) / ntb;
  int tpw = 0;
  const int W = pick_waves(blocks, Kt, tpw);
  const uint32_t gs = group_magic(group);
#define QLIN_GV(PF, T)                                                                     \
  hipLaunchKernelGGL((gemv_kernel<BITS, MT, GPT, ZM, PF, T>), dim3(blocks), dim3(64 * W), \
                     0, st, qw, qsz, (const _Float16*)x, (const _Float16*)bias,             \
                     (_Float16*)y, M, N, K, group, gs, tpw, (const _Float16*)e.res, e.ep, e.aq)
  if constexpr (MT >= 8) {  // x registers of 4 tiles in flight would spill
    if (ntb == 2) QLIN_GV(2, 2);
    else QLIN_GV(2, 1);
  } else {
    // four tiles in flight where the wave's tiles come in whole rounds of four (or many of
    // them): 4096 x 14,336 (tpw 7) PF = 2 7.95 us vs PF = 4 8.46 us; 28,672 x 4,096 (tpw 4)
    // and tpw 14 prefer four
    if (tpw % 4 == 0 || tpw >= 12) QLIN_GV(4, 1);
    else QLIN_GV(2, 1);
  }
#undef QLIN_GV
  return (int)hipGetLastError();
}

static inline bool group_fast(int K, int group) {  // whole-tile or 32 / 64-wide groups on whole k-tiles
  return K % kTileK == 0 && (group % kTileK == 0 || group == 32 || group == 64);
}

// ---- M == 1, wide matrices: the work-queue kernel ------------------------------------------------
struct WrowGeo {
  int nb, CPR, max_rows, part_off, sz_off, misc_off, lds;
};
// one block per CU for matrices of >= 4 tile rows per CU with whole chunks of k-tiles; the LDS
// image (x, the partials of every row's chunks, the waves' (scale, zero) slots) within 64 KB
static inline bool wrow_geometry(int64_t Nt, int Kt, int K, int group, WrowGeo& g) {
  const int64_t cus = device_cu_count();
  if (Nt < 4 * cus || Kt % kWqC || K > 64 * kWqWaves * 8 * 4) return false;
  g.nb = (int)std::min<int64_t>(cus, Nt);
  g.CPR = Kt / kWqC;
  g.max_rows = (int)((Nt + g.nb - 1) / g.nb);
  const int GPT = group % kTileK == 0 ? 1 : group == 64 ? 2 : 4;
  wq_lds_layout(K, g.max_rows, g.CPR, GPT, g.part_off, g.sz_off, g.misc_off, g.lds);
  return g.lds <= 64 * 1024;
}

template <int BITS, int GPT, int ZM, int NRM>
int launch_wrow(const WrowArgs& a, const WrowGeo& g, hipStream_t st) {
  const int xi = (a.K / 8 + 64 * kWqWaves - 1) / (64 * kWqWaves);
#define QLIN_WQ(XI)                                                                             \
  hipLaunchKernelGGL((gemv_wq_kernel<BITS, GPT, ZM, NRM, XI>), dim3((unsigned)g.nb),            \
                     dim3(64 * kWqWaves), (size_t)g.lds, st, a)
  if (xi <= 1) QLIN_WQ(1);
  else QLIN_WQ(4);
#undef QLIN_WQ
  return (int)hipGetLastError();
}

template <int BITS, int ZM>
int launch_wrow_g(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, const uint16_t* bias,
                  uint16_t* y, int N, int K, int group, hipStream_t st, int ep,
                  const uint16_t* res, const void* nw, bool nw16, float eps, const WrowGeo& g) {
  WrowArgs a;
  a.qw = qw;
  a.qsz = qsz;
  a.x = (const _Float16*)x;
  a.has_bias = bias != nullptr;
  a.bias = (const _Float16*)(bias ? bias : y);
  a.res = (const _Float16*)(ep == kEpResidual ? res : y);
  a.nres = ep == kEpSiluMul ? N / 2 : N;
  a.y = (_Float16*)y;
  a.nw = nw;
  a.eps = eps;
  a.ep = ep;
  a.N = N;
  a.K = K;
  a.Kt = K / kTileK;
  a.G = K / group;
  a.Nt = (N + kTileN - 1) / kTileN;
  a.nb = g.nb;
  a.CPR = g.CPR;
  a.part_off = g.part_off;
  a.sz_off = g.sz_off;
  a.misc_off = g.misc_off;
  a.cmagic = tile_group_magic(group);
#define QLIN_WG(GPT)                                                                            \
  return !nw  ? launch_wrow<BITS, GPT, ZM, 0>(a, g, st)                                         \
         : nw16 ? launch_wrow<BITS, GPT, ZM, kNwF16>(a, g, st)                                  \
                : launch_wrow<BITS, GPT, ZM, kNwF32>(a, g, st)
  if (group % kTileK == 0) QLIN_WG(1);
  if (group == 64) QLIN_WG(2);
  QLIN_WG(4);
#undef QLIN_WG
}

// ---- M == 1: the rows kernel ------------------------------------------------------------------
struct RowsGeo {
  int W, TPW, nb, pf;
};

// W * TPW == Kt with TPW the smallest of {2, 4, 8} that keeps W <= 16 (the most waves per row);
// one row per block up to 2 rows per CU (PF = the wave's whole row), else a persistent grid of
// kRowsBpc blocks per CU streaming 8 tiles ahead across rows
constexpr int kRowsMinTPW = 2;   // smallest k-tiles per wave and row
constexpr int kRowsOneRowCU = 2; // grids of up to this many rows per CU run one row per block
static inline bool rows_geometry(int64_t Nt, int Kt, RowsGeo& g) {
  const int64_t cus = device_cu_count();
  // one-row grids: few enough waves that every block is resident at once (16 waves per CU: the
  // register budget of these kernels admits at least that); measured qkv (384 rows) W = 16: two
  // rounds of blocks, 7.4 us; W = 8: 6.1 us (round-4 stamp builds)
  const bool onerow = Nt <= kRowsOneRowCU * cus;
  g.TPW = 0;
  for (int t = kRowsMinTPW; t <= kRowsMaxTPW; t *= 2)
    if (Kt % t == 0 && Kt / t <= kMaxWaves && (!onerow || t == kRowsMaxTPW ||
                                               Nt * (Kt / t) <= kMaxWaves * cus)) {
      g.TPW = t;
      break;
    }
  if (!g.TPW || Nt < 1 || Nt > (1 << 26)) return false;
  g.W = Kt / g.TPW;
  g.nb = onerow ? (int)Nt : (int)(cus * kRowsBpc);
  g.pf = (g.nb < Nt && (Nt / g.nb) * g.TPW >= 8) ? 8 : g.TPW;
  return true;
}


template <int BITS, int GPT, int ZM, int NRM>
int launch_rows(const RowsArgs& a, const RowsGeo& g, hipStream_t st) {
  const size_t lds = 0;
#define QLIN_GR(T, P)                                                                          \
  hipLaunchKernelGGL((gemv_rows_kernel<BITS, GPT, ZM, T, P, NRM>), dim3((unsigned)g.nb),        \
                     dim3(64 * g.W), lds, st, a)
  if (g.TPW == 2) {
    if (g.pf == 8) QLIN_GR(2, 8);
    else QLIN_GR(2, 2);
  } else if (g.TPW == 4) {
    if (g.pf == 8) QLIN_GR(4, 8);
    else QLIN_GR(4, 4);
  } else {
    QLIN_GR(8, 8);
  }
#undef QLIN_GR
  return (int)hipGetLastError();
}

template <int BITS, int ZM>
int launch_rows_g(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, const uint16_t* bias,
                  uint16_t* y, int N, int K, int group, hipStream_t st, int ep,
                  const uint16_t* res, const void* nw, bool nw16, float eps, const RowsGeo& g) {
  const int64_t Nt = (N + kTileN - 1) / kTileN;
  RowsArgs a;
  a.qw = qw;
  a.qsz = qsz;
  a.x = (const _Float16*)x;
  // absent epilogue operands point at y (read before it is written, never used)
  const int ny = ep == kEpSiluMul ? N / 2 : N;
  a.has_bias = bias != nullptr;
  a.bias = (const _Float16*)(bias ? bias : y);
  a.res = (const _Float16*)(ep == kEpResidual ? res : y);
  a.nres = ny;
  a.y = (_Float16*)y;
  a.nw = nw;
  a.eps = eps;
  a.ep = ep;
  a.N = N;
  a.K = K;
  a.Kt = K / kTileK;
  a.G = K / group;
  a.W = g.W;
  a.nb = g.nb;
  a.rpb = (int)(Nt / g.nb);
  a.extra = (int)(Nt % g.nb);
  a.wstep = (int64_t)g.nb * a.Kt * 64 * BITS;
  a.sstep = (int64_t)g.nb * a.G * kTileN;
  a.cmagic = tile_group_magic(group);
#define QLIN_RG(GPT)                                                                            \
  return !nw  ? launch_rows<BITS, GPT, ZM, 0>(a, g, st)                                         \
         : nw16 ? launch_rows<BITS, GPT, ZM, kNwF16>(a, g, st)                                  \
                : launch_rows<BITS, GPT, ZM, kNwF32>(a, g, st)
  if (group % kTileK == 0) QLIN_RG(1);
  if (group == 64) QLIN_RG(2);
  QLIN_RG(4);
#undef QLIN_RG
}

// ---- M <= 4: the fast kernel -----------------------------------------------------------------
template <int BITS, int MT, int GPT, int ZM, int EP>
int launch_fast_t(const FastArgs& a, bool nw16, int Nt, int tpw, hipStream_t st) {
#define QLIN_GF(PF, NR)                                                                      \
  hipLaunchKernelGGL((gemv_fast_kernel<BITS, MT, GPT, ZM, EP, PF, NR>), dim3(Nt),          \
                     dim3(64 * a.W), 0, st, a)
  if constexpr (MT == 1) {
    if (a.nw && nw16) {
      if (tpw <= 2) QLIN_GF(2, kNwF16);
      else QLIN_GF(4, kNwF16);
      return (int)hipGetLastError();
    }
    if (a.nw) {
      if (tpw <= 2) QLIN_GF(2, kNwF32);
      else QLIN_GF(4, kNwF32);
      return (int)hipGetLastError();
    }
  }
  if (tpw <= 2) QLIN_GF(2, 0);
  else QLIN_GF(4, 0);
#undef QLIN_GF
  return (int)hipGetLastError();
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

static inline bool fast_ok(int M, int K, int group, const Ep& e) {
  return M <= 4 && !e.aq.on && group_fast(K, group);
}

template <int BITS, int MT, int ZM>
int launch_fast(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, const uint16_t* bias,
                uint16_t* y, int M, int N, int K, int group, int W, int lw, int tpw,
                hipStream_t st, int ep, const uint16_t* res, const void* nw = nullptr,
                bool nw16 = false, float eps = 0.f) {
  const int Nt = (N + kTileN - 1) / kTileN;
  FastArgs a;
  a.qw = qw;
  a.qsz = qsz;
  a.x = (const _Float16*)x;
  a.bias = (const _Float16*)bias;
  a.res = (const _Float16*)res;
  a.y = (_Float16*)y;
  a.M = M;
  a.N = N;
  a.K = K;
  a.Kt = K / kTileK;
  a.G = K / group;
  a.W = W;
  a.lw = lw;
  a.cmagic = tile_group_magic(group);
  a.nw = nw;
  a.eps = eps;
#define QLIN_FE(GPT)                                                                           \
  return ep == kEpResidual  ? launch_fast_t<BITS, MT, GPT, ZM, kEpResidual>(a, nw16, Nt, tpw, st)  \
         : ep == kEpSiluMul ? launch_fast_t<BITS, MT, GPT, ZM, kEpSiluMul>(a, nw16, Nt, tpw, st)   \
                            : launch_fast_t<BITS, MT, GPT, ZM, kEpNone>(a, nw16, Nt, tpw, st)
  if (group % kTileK == 0) QLIN_FE(1);
  if (group == 64) QLIN_FE(2);
  QLIN_FE(4);
#undef QLIN_FE
}

// ---- M == 1 routing: each decode shape on the kernel measured fastest for it
// (tools/dev/rows_sweep.py: gate/up 28,672 x 4,096 whole-row 15.3 us vs fast 15.4 / rows 15.6;
// down 4,096 x 14,336 rows 8.25 us vs gemv_kernel 8.7; 4096^2 and q/k/v fast 3.7 / 5.7 us vs rows
// 3.8-4.2 / 6.1)
enum { kM1None = 0, kM1Wrow, kM1Fast, kM1Rows };
static inline int m1_route(int64_t N, int K, int group, const void* x, const void* nw, WrowGeo& wg,
                           int& W, int& lw, int& tpw, RowsGeo& rg) {
  if (!group_fast(K, group)) return kM1None;
  const int64_t Nt = (N + kTileN - 1) / kTileN;
  const int Kt = K / kTileK;
  const bool aligned = ((uintptr_t)x & 15) == 0 && ((uintptr_t)nw & 15) == 0 && K % 8 == 0;
  if (aligned && wrow_geometry(Nt, Kt, K, group, wg)) return kM1Wrow;
  if (Nt <= (1 << 26) && fast_geometry((int)Nt, Kt, W, lw, tpw)) return kM1Fast;
  if (rows_geometry(Nt, Kt, rg)) return kM1Rows;
  return kM1None;
}

template <int BITS, int ZM>
int launch_m1(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, const uint16_t* bias,
              uint16_t* y, int N, int K, int group, hipStream_t st, int ep, const uint16_t* res,
              const void* nw, bool nw16, float eps) {
  WrowGeo wg;
  RowsGeo rg;
  int W = 0, lw = 0, tpw = 0;
  switch (m1_route(N, K, group, x, nw, wg, W, lw, tpw, rg)) {
    case kM1Wrow:
      return launch_wrow_g<BITS, ZM>(qw, qsz, x, bias, y, N, K, group, st, ep, res, nw, nw16, eps,
                                      wg);
    case kM1Fast:
      return launch_fast<BITS, 1, ZM>(qw, qsz, x, bias, y, 1, N, K, group, W, lw, tpw, st, ep,
                                      res, nw, nw16, eps);
    case kM1Rows:
      return launch_rows_g<BITS, ZM>(qw, qsz, x, bias, y, N, K, group, st, ep, res, nw, nw16, eps,
                                      rg);
    default:
      return QLIN_EINVAL;
  }
}

template <int BITS, int MT, int ZM>
int launch_gemv_g(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, const uint16_t* bias,
                  uint16_t* y, int M, int N, int K, int group, hipStream_t st, const Ep& e) {
  if (group % 128 == 0)
    return launch_gemv<BITS, MT, 1, ZM>(qw, qsz, x, bias, y, M, N, K, group, st, e);
  if (group % 64 == 0)
    return launch_gemv<BITS, MT, 2, ZM>(qw, qsz, x, bias, y, M, N, K, group, st, e);
  return launch_gemv<BITS, MT, 4, ZM>(qw, qsz, x, bias, y, M, N, K, group, st, e);
}

template <int BITS, int ZM>
int launch_gemv_m(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, const uint16_t* bias,
                  uint16_t* y, int M, int N, int K, int group, hipStream_t st, const Ep& e) {
  if (M == 1 && !e.aq.on) {
    WrowGeo wg;
    RowsGeo rg;
    int W = 0, lw = 0, tpw = 0;
    if (m1_route(N, K, group, x, nullptr, wg, W, lw, tpw, rg) != kM1None)
      return launch_m1<BITS, ZM>(qw, qsz, x, bias, y, N, K, group, st, e.ep, e.res, nullptr, false,
                                 0.f);
  }
  int W = 0, lw = 0, tpw = 0;
  if (M > 1 && fast_ok(M, K, group, e) &&
      fast_geometry((N + kTileN - 1) / kTileN, K / kTileK, W, lw, tpw)) {
    if (M == 2)
      return launch_fast<BITS, 2, ZM>(qw, qsz, x, bias, y, M, N, K, group, W, lw, tpw, st, e.ep, e.res);
    return launch_fast<BITS, 4, ZM>(qw, qsz, x, bias, y, M, N, K, group, W, lw, tpw, st, e.ep, e.res);
  }
  if (M == 1) return launch_gemv_g<BITS, 1, ZM>(qw, qsz, x, bias, y, M, N, K, group, st, e);
  if (M == 2) return launch_gemv_g<BITS, 2, ZM>(qw, qsz, x, bias, y, M, N, K, group, st, e);
  if (M <= 4) return launch_gemv_g<BITS, 4, ZM>(qw, qsz, x, bias, y, M, N, K, group, st, e);
  if (M <= 8) return launch_gemv_g<BITS, 8, ZM>(qw, qsz, x, bias, y, M, N, K, group, st, e);
  return launch_gemv_g<BITS, 16, ZM>(qw, qsz, x, bias, y, M, N, K, group, st, e);
}

}  // namespace qlin_gv

// The kernel instances of each bit width are compiled in a translation unit of their own (the
// Makefile builds this file once per width with -DQLIN_GEMV_BITS=b, and once without it for the
// entry points), so they compile in parallel.
#define QLIN_GV_INST(EXT, B, Z)                                                                  \
  EXT template int qlin_gv::launch_gemv_m<B, Z>(const uint32_t*, const uint32_t*, const uint16_t*, \
                                                const uint16_t*, uint16_t*, int, int, int, int,    \
                                                hipStream_t, const qlin_gv::Ep&);                \
  EXT template int qlin_gv::launch_m1<B, Z>(const uint32_t*, const uint32_t*, const uint16_t*,  \
                                            const uint16_t*, uint16_t*, int, int, int,           \
                                            hipStream_t, int, const uint16_t*, const void*,      \
                                            bool, float)
#define QLIN_GV_INST_B(EXT, B)           \
  QLIN_GV_INST(EXT, B, kZNarrow);        \
  QLIN_GV_INST(EXT, B, kZWide);          \
  QLIN_GV_INST(EXT, B, kZFloat)
#ifdef QLIN_GEMV_BITS
QLIN_GV_INST_B(, QLIN_GEMV_BITS);
#else
QLIN_GV_INST_B(extern, 2);
QLIN_GV_INST_B(extern, 3);
QLIN_GV_INST_B(extern, 4);
QLIN_GV_INST_B(extern, 8);

using namespace qlin_gv;

extern "C" int qlin_dequant_f16(const uint32_t* qweight, const uint32_t* qsz, int flags, int64_t N,
                                int64_t K, int bits, int group, uint16_t* w, void* stream) {
  if (!qweight || !qsz || !w || !valid_layout(N, K, bits, group)) return QLIN_EINVAL;
  const int64_t pieces = ((N + kTileN - 1) / kTileN) * ((K + kTileK - 1) / kTileK) * 64;
  if (pieces == 0) return QLIN_OK;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)((pieces + 255) / 256));
  const int zm = zero_mode(flags);
#define QLIN_D1(B, Z)                                                                          \
  hipLaunchKernelGGL((dequant_kernel<B, Z>), grid, dim3(256), 0, st, qweight, qsz,             \
                     (_Float16*)w, pieces, (int)N, (int)K, group)
#define QLIN_D(B)                                                                              \
  if (zm == kZFloat) QLIN_D1(B, kZFloat);                                                      \
  else if (zm == kZWide) QLIN_D1(B, kZWide);                                                   \
  else QLIN_D1(B, kZNarrow);                                                                   \
  break
  switch (bits) {
    case 2: QLIN_D(2);
    case 3: QLIN_D(3);
    case 4: QLIN_D(4);
    default: QLIN_D(8);
  }
#undef QLIN_D
#undef QLIN_D1
  return (int)hipGetLastError();
}

// GEMV with an output epilogue (qlin_linear_ep_f16's M <= 16 leg)
int qlin::gemv_ep(const uint32_t* qweight, const uint32_t* qsz, int flags, const uint16_t* x,
                  const uint16_t* bias, const uint16_t* residual, uint16_t* y, int64_t M,
                  int64_t N, int64_t K, int bits, int group, int epilogue, int act_bits,
                  int act_flags, void* stream) {
  if (!qweight || !qsz || !x || !y || M < 1 || M > kGemvMaxM || !valid_layout(N, K, bits, group))
    return QLIN_EINVAL;
  if (act_bits && (act_bits < 2 || act_bits > 8 || K % 8 || ((uintptr_t)x & 15))) return QLIN_EINVAL;
  if (N == 0) return QLIN_OK;
  ActQ aq{act_bits != 0, act_bits, act_flags, 0.f, 0.f};
  if (aq.on) {
    const bool has_zp = !(act_flags & QLIN_DISABLE_ZERO_POINT);
    aq.qmin = has_zp ? 0.f : -(float)(1 << (act_bits - 1));
    aq.qmax = has_zp ? (float)((1 << act_bits) - 1) : (float)((1 << (act_bits - 1)) - 1);
  }
  const Ep e{residual, epilogue, aq};
  hipStream_t st = (hipStream_t)stream;
  const int m = (int)M, n = (int)N, k = (int)K;
  const int zm = zero_mode(flags);
#define QLIN_G(B)                                                                           \
  return zm == kZFloat  ? launch_gemv_m<B, kZFloat>(qweight, qsz, x, bias, y, m, n, k, group, st, e) \
         : zm == kZWide ? launch_gemv_m<B, kZWide>(qweight, qsz, x, bias, y, m, n, k, group, st, e)  \
                        : launch_gemv_m<B, kZNarrow>(qweight, qsz, x, bias, y, m, n, k, group, st, e)
  switch (bits) {
    case 2: QLIN_G(2);
    case 3: QLIN_G(3);
    case 4: QLIN_G(4);
    default: QLIN_G(8);
  }
#undef QLIN_G
}

namespace qlin_gv {
// the fused RMSNorm + linear serves one token row on the rows kernel (M = 1, K % 128 == 0, whole /
// 32 / 64-wide groups, Kt = W * TPW with W <= 16, TPW in {2, 4, 8})
bool rmsnorm_linear_ok(int64_t M, int64_t N, int64_t K, int bits, int group) {
  if (M != 1 || N < 1 || !valid_layout(N, K, bits, group)) return false;
  WrowGeo wg;
  RowsGeo rg;
  int W = 0, lw = 0, tpw = 0;
  return m1_route(N, (int)K, group, nullptr, nullptr, wg, W, lw, tpw, rg) != kM1None;
}
}  // namespace

extern "C" int qlin_rmsnorm_linear_supported(int64_t M, int64_t N, int64_t K, int bits,
                                             int group) {
  return rmsnorm_linear_ok(M, N, K, bits, group) ? 1 : 0;
}

extern "C" int qlin_gemv_m1_route(int64_t N, int64_t K, int bits, int group) {
  if (N < 1 || !valid_layout(N, K, bits, group)) return -1;
  WrowGeo wg;
  RowsGeo rg;
  int W = 0, lw = 0, tpw = 0;
  return m1_route(N, (int)K, group, nullptr, nullptr, wg, W, lw, tpw, rg);
}

extern "C" int qlin_rmsnorm_linear_ep_f16(const uint32_t* qweight, const uint32_t* qsz, int flags,
                                          const uint16_t* x, const void* norm_weight, float eps,
                                          const uint16_t* bias, const uint16_t* residual,
                                          uint16_t* y, int64_t M, int64_t N, int64_t K, int bits,
                                          int group, int epilogue, void* stream) {
  const bool nw16 = (flags & QLIN_NORM_W16) != 0;
  if (!qweight || !qsz || !x || !norm_weight || !y || !rmsnorm_linear_ok(M, N, K, bits, group) ||
      ((uintptr_t)norm_weight & (nw16 ? 3 : 7)) || ((uintptr_t)x & 3) || !(eps >= 0.f) ||
      epilogue < kEpNone || epilogue > kEpSiluMul || (epilogue == kEpResidual && !residual) ||
      (epilogue == kEpSiluMul && N % kTileN))
    return QLIN_EINVAL;
  hipStream_t st = (hipStream_t)stream;
  const int n = (int)N, k = (int)K;
  const int zm = zero_mode(flags);
#define QLIN_N(B)                                                                              \
  return zm == kZFloat ? launch_m1<B, kZFloat>(qweight, qsz, x, bias, y, n, k, group, st,  \
                                               epilogue, residual, norm_weight, nw16, eps)       \
         : zm == kZWide ? launch_m1<B, kZWide>(qweight, qsz, x, bias, y, n, k, group, st,  \
                                               epilogue, residual, norm_weight, nw16, eps)       \
                        : launch_m1<B, kZNarrow>(qweight, qsz, x, bias, y, n, k, group, st, \
                                                 epilogue, residual, norm_weight, nw16, eps)
  switch (bits) {
    case 2: QLIN_N(2);
    case 3: QLIN_N(3);
    case 4: QLIN_N(4);
    default: QLIN_N(8);
  }
#undef QLIN_N
}

extern "C" int qlin_gemv_f16(const uint32_t* qweight, const uint32_t* qsz, int flags,
                             const uint16_t* x, const uint16_t* bias, uint16_t* y, int64_t M,
                             int64_t N, int64_t K, int bits, int group, void* stream) {
  return qlin::gemv_ep(qweight, qsz, flags, x, bias, nullptr, y, M, N, K, bits, group,
                               kEpNone, 0, 0, stream);
}
#endif  // QLIN_GEMV_BITS
