// qlin_attn_prefill.hip — fused fp32 attention for prefill / PPL windows (many query tokens), gfx950.
//
// Replaces, for q_len > 1, the attention core of QuantLlamaAttention.forward
// (models/int_llama_layer.py:137-165 of the reference; QuantMatMul qkt_matmul / pv_matmul of
// quant/int_matmul.py at A16): repeat_kv, the fp32 QK^T matmul, / sqrt(head_dim), + mask, the
// finfo(fp32).min clamp, the fp32 softmax and the fp32 PV matmul.  The reference materialises the
// [B, Hq, S, L] fp32 score tensor (512 MB per layer for one 2048-token window) and passes over it
// five times; this kernel streams K / V once per query block and keeps the scores on chip
// (online softmax).
//
// Arithmetic: the fp32 operands (q, the probabilities P) enter the fp16 matrix cores as unevaluated
// fp16 pairs x = hi + lo (|x - hi - lo| <= 2^-22 |x|; P scaled by 2^12 first so small
// probabilities keep their pair out of the subnormals), K / V are fp16 exactly, every product is
// exact and v_mfma_f32_16x16x32_f16 accumulates in fp32 — the reference's fp32 matmuls to within
// a few fp32 ulps, at 8x the rate of the fp32 matrix instructions (two fp16 MFMAs per product
// block).  The scores get the reference's scaling (x the fp32 reciprocal of sqrt(d), as torch
// divides by a scalar), additive mask and clamp; the softmax is the online form (running max m,
// sum l, output rescaled by exp(m_old - m_new)).  Results agree with the reference to fp32
// rounding (summation order, exp(a) exp(b) vs exp(a + b)), not bit for bit.
//
// Decomposition: a 256-thread block = 4 waves = (hw query heads of one KV head) x (4 / hw 16-row
// query sub-blocks), hw = min(Hq / Hkv, 4), so each staged K / V block serves hw heads (GQA: K / V
// are read once per KV head, never expanded).  Per 64-key block: K [64][128] and V^T [128][64]
// (fp16) are staged in LDS by all 256 threads, every wave computes its 16 x 64 score tile (32
// MFMAs over d), the online softmax in registers (row reductions over the 16 lanes of a row by
// DPP), parks P in its LDS slot (the C fragment's row / column roles are the A operand's
// transposed) and accumulates O += P V (32 MFMAs).  The next block's K / V rows and mask tile are
// fetched into registers while a block computes.  Lane (n, j) of an MFMA holds A[n][8j ..],
// B[8j ..][n] and C rows 4j + e, column n — the scores and the output share the row layout, so
// the rescale factors stay in registers.
//
// Causal windows (mask verified causal on the host): key blocks past a query block's last
// diagonal position are skipped — their mask entries are <= -1e4, so exp() underflows to exactly
// 0 in the reference too.  Query row i sits at key position L - S + i (a cached prefix of L - S
// keys precedes the window).
#include "qlin_common.h"
#include "../../include/qlin_gfx950.h"

namespace {

constexpr int kD = 128;       // head_dim
constexpr int kKB = 64;       // keys per block
constexpr int kKS = kD + 8;   // K row stride in LDS (halves): 272 B, conflict-free row reads
constexpr int kVS = kKB + 8;  // V^T row stride (halves): 144 B
constexpr int kPS = kKB + 4;  // P row stride (floats): 272 B
constexpr int kMaxG = 8;      // query heads per KV head

struct PrefillArgs {
  const float* q;      // [B, Hq, S, D]
  const _Float16* k;   // [B, Hkv, L, D]
  const _Float16* v;
  const void* mask;    // [B', 1, S, L] additive (fp16 / fp32), batch b at mask + b * mask_bs, or null
  int64_t mask_bs;
  void* out;           // [B, S, Hq, D]
  int mask_f32, out_f16, causal;
  int Hq, Hkv, S, L;
  int hw, lhw;         // query heads per block (power of two <= 4) and its log2
  int nrb;             // query row blocks per (b, KV head, head group)
  float inv;           // fp32 1 / sqrt(d)
};

typedef float f4v __attribute__((ext_vector_type(4)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));

template <int CTRL>
__device__ __forceinline__ float dpp_max_step(float v) {
  return fmaxf(v, qlin::dpp_f<CTRL>(v));
}
// max / sum over the 16 lanes of each 16-lane row (every lane ends with its row's total)
__device__ __forceinline__ float row16_max(float v) {
  v = dpp_max_step<0xB1>(v);
  v = dpp_max_step<0x4E>(v);
  v = dpp_max_step<0x141>(v);
  v = dpp_max_step<0x140>(v);
  return v;
}

// fp32 value as an unevaluated pair of fp16 (hi = RN16(x), lo = RN16(x - hi)): |x - hi - lo| <=
// 2^-22 |x| in the normal range
__device__ __forceinline__ void split16(float x, _Float16& hi, _Float16& lo) {
#pragma clang fp contract(off)
  hi = (_Float16)x;
  lo = (_Float16)(x - (float)hi);
}

__global__ __launch_bounds__(256) void attn_prefill_kernel(const PrefillArgs a) {
  __shared__ __attribute__((aligned(16))) _Float16 ks[kKB * kKS];   // 17,408 B
  __shared__ __attribute__((aligned(16))) _Float16 vt[kD * kVS];    // 18,432 B
  __shared__ __attribute__((aligned(16))) float ps[4][16 * kPS];    // 17,408 B

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63, n = lane & 15, j = lane >> 4;
  const int RB = 64 >> a.lhw;  // query rows per block (16 per wave sub-block)
  // heaviest (last) row blocks first: causal work grows with the row index
  int bid = blockIdx.x;
  const int rb = a.nrb - 1 - bid % a.nrb;
  bid /= a.nrb;
  const int G = a.Hq / a.Hkv;
  const int ngrp = G >> a.lhw;  // head groups per KV head
  const int hg = bid % ngrp;
  bid /= ngrp;
  const int hkv = bid % a.Hkv;
  const int b = bid / a.Hkv;
  const int hq = hkv * G + hg * a.hw + (wave & (a.hw - 1));
  const int row0 = rb * RB + (wave >> a.lhw) * 16;  // the wave's first query row
  const int L = a.L, S = a.S, off = L - S;         // query row i <-> key position off + i
  const bool wave_rows = row0 < S;                 // wave-uniform

  // the block's key range and the wave's own (causal: up to the last row's diagonal)
  int kend = L, kend_w = L;
  if (a.causal) {
    kend = min(L, off + min(rb * RB + RB, S));
    kend_w = min(L, off + min(row0 + 16, S));
  }
  const int nkb = (kend + kKB - 1) / kKB;

  // q as fp16 pairs in the A-operand layout of v_mfma_f32_16x16x32_f16: lane (n, j), d-step t
  // holds q[row0 + n][32 t + 8 j .. + 7]
  qlin::h8 qh[4], ql[4];
  {
    const float* qp = a.q + (((int64_t)b * a.Hq + hq) * S + min(row0 + n, S - 1)) * kD + 8 * j;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float4 x0 = reinterpret_cast<const float4*>(qp + 32 * t)[0];
      const float4 x1 = reinterpret_cast<const float4*>(qp + 32 * t)[1];
      const float xv[8] = {x0.x, x0.y, x0.z, x0.w, x1.x, x1.y, x1.z, x1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        _Float16 h, l;
        split16(xv[e], h, l);
        qh[t][e] = h;
        ql[t][e] = l;
      }
    }
  }
  f4v o[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) o[c] = f4v{0.f, 0.f, 0.f, 0.f};
  float m[4], l[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) { m[e] = -INFINITY; l[e] = 0.f; }

  const _Float16* kbase = a.k + ((int64_t)b * a.Hkv + hkv) * L * kD;
  const _Float16* vbase = a.v + ((int64_t)b * a.Hkv + hkv) * L * kD;
  const char* mrow = nullptr;
  if (a.mask) {
    const int64_t esz = a.mask_f32 ? 4 : 2;
    mrow = reinterpret_cast<const char*>(a.mask) + (int64_t)b * a.mask_bs * esz;
  }
  float* pw = ps[wave];

  // next block's K / V rows and the wave's mask tile, in registers while this block computes
  u4v kr[4], vr[4];
  float mk[4][4];
  auto fetch = [&](int k0) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {  // K: chunk c = tid + 256 u -> key c / 16, d 8 (c % 16)
      const int c = tid + 256 * u, key = c >> 4, d8 = (c & 15) * 8;
      kr[u] = *reinterpret_cast<const u4v*>(kbase + (int64_t)min(k0 + key, L - 1) * kD + d8);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)  // V: lane = key, d 8 (wave + 4 u)
      vr[u] = *reinterpret_cast<const u4v*>(vbase + (int64_t)min(k0 + lane, L - 1) * kD +
                                             (wave + 4 * u) * 8);
#pragma unroll
    for (int sb = 0; sb < 4; ++sb)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        mk[sb][e] = 0.f;
        if (mrow) {
          const int64_t idx =
              (int64_t)min(row0 + 4 * j + e, S - 1) * L + min(k0 + 16 * sb + n, L - 1);
          mk[sb][e] = a.mask_f32 ? reinterpret_cast<const float*>(mrow)[idx]
                                 : (float)reinterpret_cast<const _Float16*>(mrow)[idx];
        }
      }
  };
  fetch(0);

  for (int kb = 0; kb < nkb; ++kb) {
    const int k0 = kb * kKB;
    __syncthreads();  // every wave is done with the previous block's K / V^T
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = tid + 256 * u, key = c >> 4, d8 = (c & 15) * 8;
      *reinterpret_cast<u4v*>(ks + key * kKS + d8) = kr[u];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {  // V^T: each instruction writes 64 consecutive keys of 8 rows
      const int d8 = (wave + 4 * u) * 8;
      const qlin::h8 h = __builtin_bit_cast(qlin::h8, vr[u]);
#pragma unroll
      for (int e = 0; e < 8; ++e) vt[(d8 + e) * kVS + lane] = h[e];
    }
    float mc[4][4];
#pragma unroll
    for (int sb = 0; sb < 4; ++sb)
#pragma unroll
      for (int e = 0; e < 4; ++e) mc[sb][e] = mk[sb][e];
    __syncthreads();
    fetch(k0 + kKB);  // lands while this block computes (past the last block: clamped, unused)
    if (!wave_rows || k0 >= kend_w) continue;  // wave-uniform; the wave still stages and syncs

    // scores S = Q K^T (fp32 accumulate of q_hi k + q_lo k): C rows 4 j + e, key 16 sb + n
    f4v sc[4];
#pragma unroll
    for (int sb = 0; sb < 4; ++sb) sc[sb] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int sb = 0; sb < 4; ++sb) {
        const qlin::h8 kf = *reinterpret_cast<const qlin::h8*>(ks + (16 * sb + n) * kKS + 32 * t + 8 * j);
        sc[sb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(qh[t], kf, sc[sb], 0, 0, 0);
        sc[sb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ql[t], kf, sc[sb], 0, 0, 0);
      }
    // scale, mask, clamp (the reference's order), keys past L masked out
    float mloc[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
    for (int sb = 0; sb < 4; ++sb) {
      const bool kin = k0 + 16 * sb + n < L;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
#pragma clang fp contract(off)
        float sv = sc[sb][e] * a.inv;
        if (mrow) {
          sv = sv + mc[sb][e];
          sv = (sv != sv) ? sv : fmaxf(sv, -3.402823466e38f);  // torch.max(w, finfo(fp32).min)
        }
        sv = kin ? sv : -INFINITY;
        sc[sb][e] = sv;
        mloc[e] = fmaxf(mloc[e], sv);
      }
    }
    // online softmax: row max over the 64 keys, rescale, P = exp(s - m)
    float alpha[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float mb = row16_max(mloc[e]);
      const float mn = fmaxf(m[e], mb);
      alpha[e] = (mn == -INFINITY) ? 1.f : expf(m[e] - mn);
      m[e] = mn;
      float rs = 0.f;
#pragma unroll
      for (int sb = 0; sb < 4; ++sb) {
        const float pv = (mn == -INFINITY) ? 0.f : expf(sc[sb][e] - mn);
        sc[sb][e] = pv;
        rs += pv;
      }
      l[e] = l[e] * alpha[e] + qlin::row16_sum(rs);
    }
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) o[c][e] *= alpha[e];
    // park P x 2^12 (P <= 1: its fp16 pair stays out of the subnormals down to 2^-26) as
    // P[row][key], rows 4 j + e, key 16 sb + n; lane (n, j) of key step t reads P[n][32 t + 8 j ..]
#pragma unroll
    for (int sb = 0; sb < 4; ++sb)
#pragma unroll
      for (int e = 0; e < 4; ++e) pw[(4 * j + e) * kPS + 16 * sb + n] = sc[sb][e] * 4096.f;
    // O += P V (fp32 accumulate of p_hi v + p_lo v): d block c, lane (n, j) of key step t takes
    // V[32 t + 8 j ..][16 c + n] = V^T[16 c + n][32 t + 8 j ..]
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      qlin::h8 ph, pl;
      {
        const float4 p0 = reinterpret_cast<const float4*>(pw + n * kPS + 32 * t + 8 * j)[0];
        const float4 p1 = reinterpret_cast<const float4*>(pw + n * kPS + 32 * t + 8 * j)[1];
        const float pvv[8] = {p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          _Float16 h, lo;
          split16(pvv[e], h, lo);
          ph[e] = h;
          pl[e] = lo;
        }
      }
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const qlin::h8 vf = *reinterpret_cast<const qlin::h8*>(vt + (16 * c + n) * kVS + 32 * t + 8 * j);
        o[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ph, vf, o[c], 0, 0, 0);
        o[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(pl, vf, o[c], 0, 0, 0);
      }
    }
  }

  if (!wave_rows) return;
  // O / (l 2^12) -> out[b][row][hq][d] (the layer's transpose(1, 2) layout; fp16 = its .to(fp16))
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int row = row0 + 4 * j + e;
    if (row >= S) continue;
    const float rl = l[e] * 4096.f;
    const int64_t base = (((int64_t)b * S + row) * a.Hq + hq) * kD + n;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const float val = o[c][e] / rl;
      if (a.out_f16) reinterpret_cast<_Float16*>(a.out)[base + 16 * c] = (_Float16)val;
      else reinterpret_cast<float*>(a.out)[base + 16 * c] = val;
    }
  }
}

}  // namespace

extern "C" int qlin_attn_prefill(const float* q, const uint16_t* k, const uint16_t* v,
                                 const void* mask, int mask_dtype, int64_t mask_batch_stride,
                                 int causal, void* out, int out_dtype, int64_t B, int Hq, int Hkv,
                                 int64_t S, int64_t L, int D, float scale_div, void* stream) {
  if (!q || !k || !v || !out || (out_dtype != QLIN_F32 && out_dtype != QLIN_F16) || B < 0 ||
      Hq <= 0 || Hkv <= 0 || Hq % Hkv || S <= 0 || L < S || L > (1 << 20) || D != kD ||
      !(scale_div > 0.f) || (mask && mask_dtype != QLIN_F16 && mask_dtype != QLIN_F32) ||
      mask_batch_stride < 0 || (causal && !mask))
    return QLIN_EINVAL;
  const int G = Hq / Hkv;
  if (G > kMaxG || (G & (G - 1))) return QLIN_EINVAL;
  if (B == 0) return QLIN_OK;
  PrefillArgs a;
  a.q = q;
  a.k = (const _Float16*)k;
  a.v = (const _Float16*)v;
  a.mask = mask;
  a.mask_bs = mask_batch_stride;
  a.out = out;
  a.mask_f32 = mask_dtype == QLIN_F32;
  a.out_f16 = out_dtype == QLIN_F16;
  a.causal = causal != 0;
  a.Hq = Hq;
  a.Hkv = Hkv;
  a.S = (int)S;
  a.L = (int)L;
  a.hw = G < 4 ? G : 4;
  a.lhw = a.hw == 1 ? 0 : a.hw == 2 ? 1 : 2;
  const int RB = 64 >> a.lhw;
  a.nrb = (int)((S + RB - 1) / RB);
  a.inv = 1.0f / scale_div;
  const int64_t blocks = B * Hkv * (G / a.hw) * (int64_t)a.nrb;
  if (blocks > 0x7fffffff) return QLIN_EINVAL;
  hipLaunchKernelGGL(attn_prefill_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     (hipStream_t)stream, a);
  return (int)hipGetLastError();
}
