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

namespace {

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
  float* sq_out = nullptr;  // M == 1, kEpResidual: per-tile sums of squares of y
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

// the sum of squares of the 16 outputs one tile row's block writes (lanes 0..15 of wave 0 hold
// them; every other lane 0) in a fixed butterfly order -> sq_out[nt]: the statistics of the
// RMSNorm that reads this output next (qlin_rmsnorm_linear_ep_f16's sumsq_in), precomputed
__device__ __forceinline__ void sq_tile_out(float v, float* sq_out, int64_t nt) {
#pragma clang fp contract(off)
  v = v + __shfl_xor(v, 8);
  v = v + __shfl_xor(v, 4);
  v = v + __shfl_xor(v, 2);
  v = v + __shfl_xor(v, 1);
  if ((threadIdx.x & 63) == 0) sq_out[nt] = v;
}

template <int BITS, int MT, int GPT, int ZM, int PF, int NTB = 1>
__global__ __launch_bounds__(1024) void gemv_kernel(
    const uint32_t* __restrict__ qw, const uint32_t* __restrict__ qsz,
    const _Float16* __restrict__ x, const _Float16* __restrict__ bias, _Float16* __restrict__ y,
    int M, int N, int K, int group, uint32_t gmagic, int tpw, const _Float16* __restrict__ res,
    int ep, ActQ aq, float* __restrict__ sq_out) {
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
  float sqv = 0.f;  // sq_out: this thread's output squared
  for (int o = tid; o < NTB * MT * kTileN; o += blockDim.x) {
    const int j = o / (MT * kTileN), oo = o - j * MT * kTileN;
    const int m = oo / kTileN, n = oo - m * kTileN;
    const int64_t row = ((int64_t)nt + j) * kTileN + n;
    if (m < M && row < N) {
      float t = total(o, row);
      if (ep == kEpResidual) t += (float)res[(int64_t)m * N + row];
      y[(int64_t)m * N + row] = (_Float16)t;
      const float f = (float)(_Float16)t;
      sqv = f * f;
    }
  }
  if (sq_out && wave == 0) sq_tile_out(sqv, sq_out, nt);  // M == 1, NTB == 1 (host)
}

// ---------------------------------------------------------------------------------------------
// Decode fast path: M <= 4, K % 128 == 0, group % 128 == 0 or group in {32, 64}, no activation
// fake-quant.  Same arithmetic as gemv_kernel (exact W_dq, one MFMA per k-step), built for the
// ~3-4 us a 4096 x 4096 launch lasts (tools/dev/gemv_lab2.hip, gemv_lab3.hip):
//   - everything the general kernel derives by integer division (tiles, groups, strides) comes
//     precomputed from the host, so the first weight load issues a few scalar ops after the
//     kernel arguments land; the epilogue is a template parameter, so the executed code is one
//     short straight line (the weights arrive ~1 us after the start: code fetched late, or work
//     queued in front of the loads, shows up 1:1 in the launch time);
//   - wave w streams tiles kt = w, w + W, w + 2W, ...: the tiles in flight on a CU at one time
//     are W tiles (W x 1 KB for int4) apart in HBM instead of adjacent (4096^2: 3.89 -> 3.74 us);
//   - all codes of the prefetch window are issued before their (scale, zero) words and x, so the
//     first tile only waits for its own three loads.
// ---------------------------------------------------------------------------------------------
#ifndef GEMV_NRM_XFIRST  // dev switch: the fused norm's x words issued before the codes
#define GEMV_NRM_XFIRST 1
#endif
#ifndef GEMV_NRM_LATE  // 1 (round 3): the norm's rsqrt is applied to the accumulators in the
#define GEMV_NRM_LATE 1  // epilogue (x words rounded as RN16(w * x)): the first MFMAs wait for no
#endif                   // statistics; 0: the round-2 form (statistics behind a barrier first)
// qlin_rmsnorm_linear_ep_f16's optional inputs (precomputed statistics, RoPE row gather)
struct NormIn {
  const float* sq_in;
  int sq_n;
  const int64_t* rope_pos;
  const float* rope_cos;
  const float* rope_sin;
  int64_t rope_rows;
  float* rope_out;
};

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
  const float* nw;      // NRM: RMSNorm weight (fp32 [K]) applied to x first
  float eps;
  const float* sq_in;   // NRM: precomputed statistics (sq_n partial sums of squares of x), or null
  int sq_n;
  float* sq_out;        // EP == kEpResidual, M == 1: per-tile sums of squares of y, or null
  const int64_t* rope_pos;  // block 0, wave 0: copy cos / sin row rope_pos[0] to rope_out
  const float* rope_cos;
  const float* rope_sin;
  int64_t rope_rows;
  float* rope_out;      // [2][128] fp32, or null
};
constexpr int kSqMaxPerLane = 8;  // sumsq_in partials per lane (K <= 64 * 8 * 16 = 8192)

// every wave streams at most PF tiles, all of them loaded up front (no refill loop: a launch whose
// waves need more tiles takes gemv_kernel, whose contiguous tile runs stream better then).
// NRM (M = 1): x is the decoder layer's hidden state before its RMSNorm (OmniLlamaRMSNorm,
// quant/omni_norm.py:52-63 of the reference) and the kernel applies the norm itself: each wave
// sums the squares of the x words it loads anyway (its own tiles; together the waves cover the
// row once), the block combines the W wave sums through LDS behind a bare s_barrier (no vmcnt
// drain), and every x word is normalised (weight * (x * rsqrt(mean + eps)), fp32, rounded to fp16
// as the norm's output) before it is parked.  One launch instead of two (the separate
// qlin_rmsnorm_f16); the sum of squares runs in another order than that kernel's, so the normed
// x can differ from it by an fp16 ulp.
template <int BITS, int MT, int GPT, int ZM, int EP, int PF, bool NRM = false>
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

  // precomputed norm statistics: issued before every other load (in-order completion: the norm
  // then waits for these alone, not for the weights)
  float sqp[NRM ? kSqMaxPerLane : 1];
  if constexpr (NRM && !GEMV_NRM_LATE) {
    if (a.sq_in) {
#pragma unroll
      for (int i = 0; i < kSqMaxPerLane; ++i) sqp[i] = a.sq_in[min(lane + 64 * i, a.sq_n - 1)];
    }
  }
  if (a.rope_out && nt == 0 && wave == 0) {
    // the step's RoPE cos / sin row for the attention launch that follows (it then skips the
    // position -> row round trip); tiny, and only block 0's wave 0 pays it
    const int64_t p = min(max(a.rope_pos[0], (int64_t)0), a.rope_rows - 1);
    const float* src = (lane < 32 ? a.rope_cos : a.rope_sin) + p * 128 + 4 * (lane & 31);
    *reinterpret_cast<float4*>(a.rope_out + 4 * lane) = *reinterpret_cast<const float4*>(src);
  }
  auto kt_of = [&](int i) { return min(wave + (i << a.lw), ktl); };
  auto group_of_tile = [&](int kt) {
    return GPT == 1 ? (int)(((uint64_t)(uint32_t)kt * a.cmagic) >> 31) : kt * GPT;
  };
  WTile<BITS, GPT> wt[PF];
  XRaw<MT> xq[PF];
  float2 nwv[NRM ? PF : 1];  // NRM: norm weights of the lane's two x halves per tile
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
#if GEMV_NRM_XFIRST
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      load_x(u, kt_of(u));
      nwv[u] = *reinterpret_cast<const float2*>(a.nw + kt_of(u) * kTileK + 2 * lane);
    }
#pragma unroll
    for (int u = 0; u < PF; ++u) load_codes(u, kt_of(u));
#else
#pragma unroll
    for (int u = 0; u < PF; ++u) load_codes(u, kt_of(u));
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      load_x(u, kt_of(u));
      nwv[u] = *reinterpret_cast<const float2*>(a.nw + kt_of(u) * kTileK + 2 * lane);
    }
#endif
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
  float ss_late = 0.f;  // GEMV_NRM_LATE: this wave's sum of squares of its x words
  if constexpr (NRM && GEMV_NRM_LATE) {
#pragma clang fp contract(off)
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      if (u < nts) {
        const h2 v = as_h2(xq[u].w[0]);
        const float f0 = (float)v.x, f1 = (float)v.y;
        ss_late = ss_late + f0 * f0;
        ss_late = ss_late + f1 * f1;
      }
    }
  } else if constexpr (NRM) {
   if (a.sq_in) {
#pragma clang fp contract(off)
    // sum of partial i over i = lane + 64 j (j in order), then the wave butterfly: the same
    // order in every wave and block, and no barrier
    float ss = 0.f;
#pragma unroll
    for (int i = 0; i < kSqMaxPerLane; ++i)
      if (lane + 64 * i < a.sq_n) ss = ss + sqp[i];
    ss = wave_sum(ss);
    rn = rsqrtf(ss / (float)a.K + a.eps);
   } else {
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
    // the sz words still in flight; the waves only need each other's sums
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    float tot = 0.f;
    for (int w = 0; w < a.W; ++w) tot += nss[w];
    rn = rsqrtf(tot / (float)a.K + a.eps);
   }
  }

  const Magics mg = make_magics<BITS>();
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  uint32_t* slot = &xs[wave][0];
  auto tile = [&](int u) {
    h8 xa[4];
    if constexpr (NRM) {
#pragma clang fp contract(off)
      const h2 v = as_h2(xq[u].w[0]);
      const float n0 = GEMV_NRM_LATE ? nwv[u].x * (float)v.x : nwv[u].x * ((float)v.x * rn);
      const float n1 = GEMV_NRM_LATE ? nwv[u].y * (float)v.y : nwv[u].y * ((float)v.y * rn);
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
  // zeroed — so the compiler cannot sink those slots' loads behind a branch (which it does for
  // `if (u < nts) tile(u)`: the loads then issue only after the earlier tiles' compute, one
  // extra HBM round trip per launch)
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
  if constexpr (NRM && GEMV_NRM_LATE) {
    const float ssw = wave_sum(ss_late);
    if (lane == 0) nss[wave] = ssw;
  }
  __syncthreads();
  if constexpr (NRM && GEMV_NRM_LATE) {
    if (wave == 0) {  // the outputs are formed by wave 0
#pragma clang fp contract(off)
      float tot = 0.f;
      if (a.sq_in) {  // precomputed statistics (fixed order: every block forms the same value)
        for (int i = 0; i < a.sq_n; ++i) tot += a.sq_in[i];
      } else {
        for (int w = 0; w < a.W; ++w) tot += nss[w];
      }
      rn = rsqrtf(tot / (float)a.K + a.eps);
    }
  }
  auto total = [&](int o, _Float16 b) {
    const f4* r = reinterpret_cast<const f4*>(red + o * kMaxWaves);
    const f4 p = r[0], q = r[1], c = r[2], d = r[3];
    const f4 e = (p + q) + (c + d);
    float t = (e[0] + e[1]) + (e[2] + e[3]);
    if (NRM && GEMV_NRM_LATE) t = t * rn;
    if (abias) t += (float)b;
    return (float)(_Float16)t;  // F.linear's fp16 output
  };
  float sqv = 0.f;  // sq_out: this thread's output squared
  if (oval) {  // wave 0 only (tid < NO <= 64)
    if constexpr (EP == kEpSiluMul) {  // 8 outputs per tile and row
      const float g = total(om * kTileN + on, ob0), u = total(om * kTileN + on + 8, ob1);
      ay[(int64_t)om * (a.N >> 1) + nt * 8 + on] = (_Float16)(silu_rn16(g) * u);
    } else {
      float t = total(om * kTileN + on, ob0);
      if constexpr (EP == kEpResidual) t += (float)ores;
      ay[(int64_t)om * a.N + orow] = (_Float16)t;
      const float f = (float)(_Float16)t;
      sqv = f * f;
    }
  }
  if constexpr (EP == kEpResidual && MT == 1) {
    if (a.sq_out && wave == 0) sq_tile_out(sqv, a.sq_out, nt);
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

uint32_t group_magic(int group) {
  const uint64_t d = (uint64_t)(group / 32);
  return (uint32_t)(((1ull << 31) + d - 1) / d);
}

// waves per block: grow W until the grid holds ~32 waves for each of the 256 CUs; on grids of
// >= 512 row tiles keep >= 4 tiles per wave (measured on the decode layer's shapes,
// tools/dev/gemv_geo.py: 28,672 x 4,096 W = 8 12.6 us vs W = 4 13.3 us; 14,336 x 4,096 W = 8
// 8.9 us vs W = 16 9.3 us; 4096 x 4096 and 6144 x 4096 keep W = 16)
#ifndef GEMV_WAVE_TARGET  // dev sweep knob (tools/dev/Makefile libgv*.so)
#define GEMV_WAVE_TARGET 8192
#endif
int pick_waves(int Nt, int Kt, int& tpw) {
  int W = 1;
  while (W < kMaxWaves && (int64_t)Nt * W < GEMV_WAVE_TARGET && (Nt < 512 || Kt >= 8 * W)) W *= 2;
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
                     (_Float16*)y, M, N, K, group, gs, tpw, (const _Float16*)e.res, e.ep, e.aq,   \
                     e.sq_out)
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

// the decode fast path (gemv_fast_kernel): M <= 4, K % 128 == 0, whole or 32 / 64-wide groups
bool fast_ok(int M, int K, int group, const Ep& e) {
  return M <= 4 && K % kTileK == 0 && !e.aq.on &&
         (group % kTileK == 0 || group == 32 || group == 64);
}

template <int BITS, int MT, int GPT, int ZM, int EP>
int launch_fast_t(const FastArgs& a, int Nt, int tpw, hipStream_t st) {
#define QLIN_GF(PF, NR)                                                                      \
  hipLaunchKernelGGL((gemv_fast_kernel<BITS, MT, GPT, ZM, EP, PF, NR>), dim3(Nt),          \
                     dim3(64 * a.W), 0, st, a)
  if constexpr (MT == 1) {
    if (a.nw) {
      if (tpw <= 2) QLIN_GF(2, true);
      else if (tpw <= 4) QLIN_GF(4, true);
      else QLIN_GF(8, true);
      return (int)hipGetLastError();
    }
  }
  if (tpw <= 2) QLIN_GF(2, false);
  else if (tpw <= 4) QLIN_GF(4, false);
  else QLIN_GF(8, false);
#undef QLIN_GF
  return (int)hipGetLastError();
}

// fast-path geometry: pick_waves rounded down to a power of two; the fast path takes launches
// whose waves stream at most 4 tiles (tools/dev/fast_geo.py, M = 1: 4096 x 4096 W = 16 x 2 tiles
// 4.30 -> 3.76 us, 6144 x 4096 5.48 -> 5.02, 28672 x 4096 W = 8 x 4 13.55 -> 12.67; the
// LLaMA down projection 4096 x 14336, 7 tiles per wave, stays on gemv_kernel: 7.8 vs 8.3 us)
#ifndef GEMV_FAST_MAX_TPW  // dev sweep knob: tiles per wave the fast path takes (4 or 8)
#define GEMV_FAST_MAX_TPW 4
#endif
bool fast_geometry(int Nt, int Kt, int& W, int& lw, int& tpw) {
  W = pick_waves(Nt, Kt, tpw);
  lw = 0;
  while ((2 << lw) <= W) ++lw;  // round W down to a power of two (W <= Kt)
  W = 1 << lw;
  tpw = (Kt + W - 1) / W;
  return tpw <= GEMV_FAST_MAX_TPW;
}

template <int BITS, int MT, int ZM>
int launch_fast(const uint32_t* qw, const uint32_t* qsz, const uint16_t* x, const uint16_t* bias,
                uint16_t* y, int M, int N, int K, int group, int W, int lw, int tpw,
                hipStream_t st, const Ep& e, const float* nw = nullptr, float eps = 0.f,
                const NormIn* ni = nullptr) {
  const int Nt = (N + kTileN - 1) / kTileN;
  FastArgs a;
  a.nw = nw;
  a.eps = eps;
  a.sq_out = e.sq_out;
  a.sq_in = ni ? ni->sq_in : nullptr;
  a.sq_n = ni ? ni->sq_n : 0;
  a.rope_pos = ni ? ni->rope_pos : nullptr;
  a.rope_cos = ni ? ni->rope_cos : nullptr;
  a.rope_sin = ni ? ni->rope_sin : nullptr;
  a.rope_rows = ni ? ni->rope_rows : 0;
  a.rope_out = ni ? ni->rope_out : nullptr;
  a.qw = qw;
  a.qsz = qsz;
  a.x = (const _Float16*)x;
  a.bias = (const _Float16*)bias;
  a.res = (const _Float16*)e.res;
  a.y = (_Float16*)y;
  a.M = M;
  a.N = N;
  a.K = K;
  a.Kt = K / kTileK;
  a.G = K / group;
  a.W = W;
  a.lw = lw;
  const uint64_t c = group % kTileK == 0 ? (uint64_t)(group / kTileK) : 1;
  a.cmagic = (uint32_t)(((1ull << 31) + c - 1) / c);
#define QLIN_FE(GPT)                                                                           \
  return e.ep == kEpResidual  ? launch_fast_t<BITS, MT, GPT, ZM, kEpResidual>(a, Nt, tpw, st)  \
         : e.ep == kEpSiluMul ? launch_fast_t<BITS, MT, GPT, ZM, kEpSiluMul>(a, Nt, tpw, st)   \
                              : launch_fast_t<BITS, MT, GPT, ZM, kEpNone>(a, Nt, tpw, st)
  if (group % kTileK == 0) QLIN_FE(1);
  if (group == 64) QLIN_FE(2);
  QLIN_FE(4);
#undef QLIN_FE
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
  int W = 0, lw = 0, tpw = 0;
  if (fast_ok(M, K, group, e) &&
      fast_geometry((N + kTileN - 1) / kTileN, K / kTileK, W, lw, tpw)) {
#define QLIN_F(MT) \
  return launch_fast<BITS, MT, ZM>(qw, qsz, x, bias, y, M, N, K, group, W, lw, tpw, st, e)
    if (M == 1) QLIN_F(1);
    if (M == 2) QLIN_F(2);
    QLIN_F(4);
#undef QLIN_F
  }
  if (M == 1) return launch_gemv_g<BITS, 1, ZM>(qw, qsz, x, bias, y, M, N, K, group, st, e);
  if (M == 2) return launch_gemv_g<BITS, 2, ZM>(qw, qsz, x, bias, y, M, N, K, group, st, e);
  if (M <= 4) return launch_gemv_g<BITS, 4, ZM>(qw, qsz, x, bias, y, M, N, K, group, st, e);
  if (M <= 8) return launch_gemv_g<BITS, 8, ZM>(qw, qsz, x, bias, y, M, N, K, group, st, e);
  return launch_gemv_g<BITS, 16, ZM>(qw, qsz, x, bias, y, M, N, K, group, st, e);
}

}  // namespace

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
                  int act_flags, void* stream, float* sq_out) {
  if (!qweight || !qsz || !x || !y || M < 1 || M > kGemvMaxM || !valid_layout(N, K, bits, group))
    return QLIN_EINVAL;
  if (sq_out && (M != 1 || epilogue != kEpResidual)) return QLIN_EINVAL;
  if (act_bits && (act_bits < 2 || act_bits > 8 || K % 8 || ((uintptr_t)x & 15))) return QLIN_EINVAL;
  if (N == 0) return QLIN_OK;
  ActQ aq{act_bits != 0, act_bits, act_flags, 0.f, 0.f};
  if (aq.on) {
    const bool has_zp = !(act_flags & QLIN_DISABLE_ZERO_POINT);
    aq.qmin = has_zp ? 0.f : -(float)(1 << (act_bits - 1));
    aq.qmax = has_zp ? (float)((1 << act_bits) - 1) : (float)((1 << (act_bits - 1)) - 1);
  }
  const Ep e{residual, epilogue, aq, sq_out};
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

namespace {
// the fused RMSNorm + linear serves one token row on the fast path (M = 1, K % 128 == 0, whole /
// 32 / 64-wide groups, <= 4 tiles per wave)
bool rmsnorm_linear_ok(int64_t M, int64_t N, int64_t K, int bits, int group) {
  if (M != 1 || N < 1 || !valid_layout(N, K, bits, group)) return false;
  const Ep e{nullptr, kEpNone, ActQ{false, 0, 0, 0.f, 0.f}};
  int W = 0, lw = 0, tpw = 0;
  return fast_ok(1, (int)K, group, e) &&
         fast_geometry((int)((N + kTileN - 1) / kTileN), (int)(K / kTileK), W, lw, tpw);
}
}  // namespace

extern "C" int qlin_rmsnorm_linear_supported(int64_t M, int64_t N, int64_t K, int bits,
                                             int group) {
  return rmsnorm_linear_ok(M, N, K, bits, group) ? 1 : 0;
}

extern "C" int qlin_rmsnorm_linear_ep_f16(const uint32_t* qweight, const uint32_t* qsz, int flags,
                                          const uint16_t* x, const float* norm_weight, float eps,
                                          const uint16_t* bias, const uint16_t* residual,
                                          uint16_t* y, int64_t M, int64_t N, int64_t K, int bits,
                                          int group, int epilogue, const float* sumsq_in,
                                          int64_t sumsq_n, const int64_t* rope_pos,
                                          const float* rope_cos, const float* rope_sin,
                                          int64_t rope_rows, float* rope_out, void* stream) {
  if (!qweight || !qsz || !x || !norm_weight || !y || !rmsnorm_linear_ok(M, N, K, bits, group) ||
      ((uintptr_t)norm_weight & 7) || ((uintptr_t)x & 3) || !(eps >= 0.f) ||
      epilogue < kEpNone || epilogue > kEpSiluMul || (epilogue == kEpResidual && !residual) ||
      (epilogue == kEpSiluMul && N % kTileN))
    return QLIN_EINVAL;
  // precomputed statistics: one partial per 16 elements of x (the producing launch's tiles)
  if (sumsq_in && (sumsq_n != (K + kTileN - 1) / kTileN || sumsq_n > 64 * kSqMaxPerLane))
    return QLIN_EINVAL;
  if (rope_out && (!rope_pos || !rope_cos || !rope_sin || rope_rows < 1 ||
                   ((uintptr_t)rope_out & 15) || ((uintptr_t)rope_cos & 15) ||
                   ((uintptr_t)rope_sin & 15)))
    return QLIN_EINVAL;
  const Ep e{residual, epilogue, ActQ{false, 0, 0, 0.f, 0.f}};
  const NormIn ni{sumsq_in, (int)sumsq_n, rope_pos, rope_cos, rope_sin, rope_rows, rope_out};
  hipStream_t st = (hipStream_t)stream;
  const int n = (int)N, k = (int)K;
  int W = 0, lw = 0, tpw = 0;
  fast_geometry((n + kTileN - 1) / kTileN, k / kTileK, W, lw, tpw);
  const int zm = zero_mode(flags);
#define QLIN_N(B)                                                                             \
  return zm == kZFloat                                                                        \
             ? launch_fast<B, 1, kZFloat>(qweight, qsz, x, bias, y, 1, n, k, group, W, lw, tpw, \
                                          st, e, norm_weight, eps, &ni)                       \
         : zm == kZWide                                                                       \
             ? launch_fast<B, 1, kZWide>(qweight, qsz, x, bias, y, 1, n, k, group, W, lw, tpw,  \
                                         st, e, norm_weight, eps, &ni)                        \
             : launch_fast<B, 1, kZNarrow>(qweight, qsz, x, bias, y, 1, n, k, group, W, lw,     \
                                           tpw, st, e, norm_weight, eps, &ni)
  switch (bits) {
    case 2: QLIN_N(2);
    case 3: QLIN_N(3);
    case 4: QLIN_N(4);
    default: QLIN_N(8);
  }
#undef QLIN_N
}

extern "C" int qlin_linear_res_sumsq_f16(const uint32_t* qweight, const uint32_t* qsz, int flags,
                                         const uint16_t* x, const uint16_t* bias,
                                         const uint16_t* residual, uint16_t* y, int64_t N,
                                         int64_t K, int bits, int group, float* sumsq_out,
                                         void* stream) {
  if (!residual || !sumsq_out) return QLIN_EINVAL;
  return qlin::gemv_ep(qweight, qsz, flags, x, bias, residual, y, 1, N, K, bits, group,
                       kEpResidual, 0, 0, stream, sumsq_out);
}

extern "C" int qlin_gemv_f16(const uint32_t* qweight, const uint32_t* qsz, int flags,
                             const uint16_t* x, const uint16_t* bias, uint16_t* y, int64_t M,
                             int64_t N, int64_t K, int bits, int group, void* stream) {
  return qlin::gemv_ep(qweight, qsz, flags, x, bias, nullptr, y, M, N, K, bits, group,
                               kEpNone, 0, 0, stream);
}
