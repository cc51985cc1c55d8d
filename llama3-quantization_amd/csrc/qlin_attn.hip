// qlin_attn.hip — fused decode attention (one query token) for the quantized LLaMA layer, gfx950.
//
// Replaces, for q_len == 1, the attention core of QuantLlamaAttention.forward
// (models/int_llama_layer.py:137-165 of the reference): repeat_kv of the fp16 K/V cache, the fp32
// QK^T bmm, the division by sqrt(head_dim), the additive mask with the finfo.min clamp, the fp32
// softmax and the fp32 PV bmm — six PyTorch kernels plus two K/V expansions and two fp16 -> fp32
// copies of the whole cache per layer and token — with one kernel that reads each K/V row once
// for all the query heads of its group (GQA) and keeps scores in LDS.
//
// Arithmetic: fp32 throughout, as the reference (q is fp32, K/V are upcast exactly); the dot
// products and sums run in a different order than hipBLASLt's bmm, so results agree to fp32
// rounding, not bit for bit.
#include "qlin_common.h"  // QLIN_OK / QLIN_EINVAL
#include "../../include/qlin_gfx950.h"

namespace {

constexpr int kD = 128;             // head_dim
constexpr int kThreads = 256;
constexpr int kMaxGroup = 8;        // query heads per KV head
constexpr int kMaxL = 4096;         // scores live in LDS: kMaxGroup * kMaxL fp32 = 128 KB
static_assert(kMaxGroup * kMaxL * 4 <= 128 * 1024, "scores must fit the LDS budget");

__device__ __forceinline__ float block_max(float v, float* red) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float r = red[0];
  for (int i = 1; i < kThreads / 64; ++i) r = fmaxf(r, red[i]);
  return r;
}

__device__ __forceinline__ float block_sum(float v, float* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  __syncthreads();
  if (l == 0) red[w] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < kThreads / 64; ++i) r += red[i];
  return r;
}

// one block per (batch, KV head); GRP query heads share the K/V rows
template <int GRP>
__global__ __launch_bounds__(kThreads) void attn_decode_kernel(
    const float* __restrict__ q, const _Float16* __restrict__ k, const _Float16* __restrict__ v,
    const _Float16* __restrict__ mask, float* __restrict__ out, int Hq, int Hkv, int L,
    float scale_div) {
  __shared__ float qs[GRP][kD];
  __shared__ float sc[GRP][kMaxL];
  __shared__ float red[kThreads / 64];
  const int b = blockIdx.x / Hkv, hk = blockIdx.x % Hkv;
  const int tid = threadIdx.x;
  const float* qb = q + ((int64_t)b * Hq + (int64_t)hk * GRP) * kD;
  for (int i = tid; i < GRP * kD; i += kThreads) qs[i / kD][i % kD] = qb[i];
  __syncthreads();
  const _Float16* kb = k + ((int64_t)b * Hkv + hk) * (int64_t)L * kD;
  const _Float16* vb = v + ((int64_t)b * Hkv + hk) * (int64_t)L * kD;
  const _Float16* mb = mask ? mask + (int64_t)b * L : nullptr;

  // scores: one K row per thread (16 x 16-byte loads), GRP dot products
  for (int t = tid; t < L; t += kThreads) {
    float acc[GRP];
#pragma unroll
    for (int g = 0; g < GRP; ++g) acc[g] = 0.f;
    const uint4* kr = reinterpret_cast<const uint4*>(kb + (int64_t)t * kD);
#pragma unroll 4
    for (int c = 0; c < kD / 8; ++c) {
      const uint4 w = kr[c];
      const _Float16* hv = reinterpret_cast<const _Float16*>(&w);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float kf = (float)hv[j];
#pragma unroll
        for (int g = 0; g < GRP; ++g) acc[g] = fmaf(qs[g][8 * c + j], kf, acc[g]);
      }
    }
    const float mv = mb ? (float)mb[t] : 0.f;
#pragma unroll
    for (int g = 0; g < GRP; ++g) {
      float s = acc[g] / scale_div + mv;
      s = (s != s) ? s : fmaxf(s, -3.402823466e38f);  // torch.max(w, finfo(fp32).min)
      sc[g][t] = s;
    }
  }
  __syncthreads();

  // softmax per query head (fp32)
#pragma unroll 1
  for (int g = 0; g < GRP; ++g) {
    float m = -INFINITY;
    for (int t = tid; t < L; t += kThreads) m = fmaxf(m, sc[g][t]);
    m = block_max(m, red);
    float s = 0.f;
    for (int t = tid; t < L; t += kThreads) {
      const float e = expf(sc[g][t] - m);
      sc[g][t] = e;
      s += e;
    }
    s = block_sum(s, red);
    const float inv = 1.f / s;
    for (int t = tid; t < L; t += kThreads) sc[g][t] *= inv;
  }
  __syncthreads();

  // PV: thread (g, pair of dims) accumulates over t; V rows read once per (group, dim pair)
  for (int o = tid; o < GRP * (kD / 2); o += kThreads) {
    const int g = o / (kD / 2), dp = o % (kD / 2);
    float a0 = 0.f, a1 = 0.f;
    const uint32_t* vr = reinterpret_cast<const uint32_t*>(vb) + dp;
    for (int t = 0; t < L; ++t) {
      const uint32_t w = vr[(int64_t)t * (kD / 2)];
      const float p = sc[g][t];
      a0 = fmaf(p, (float)__builtin_bit_cast(_Float16, (uint16_t)(w & 0xFFFFu)), a0);
      a1 = fmaf(p, (float)__builtin_bit_cast(_Float16, (uint16_t)(w >> 16)), a1);
    }
    float* ob = out + ((int64_t)b * Hq + (int64_t)hk * GRP + g) * kD + 2 * dp;
    ob[0] = a0;
    ob[1] = a1;
  }
}

}  // namespace

extern "C" int qlin_attn_decode(const float* q, const uint16_t* k, const uint16_t* v,
                                const uint16_t* mask, float* out, int64_t B, int Hq, int Hkv,
                                int64_t L, int D, float scale_div, void* stream) {
  if (!q || !k || !v || !out || B < 0 || Hq <= 0 || Hkv <= 0 || Hq % Hkv || L <= 0 ||
      L > kMaxL || D != kD || B * Hkv > 0x7fffffff)
    return QLIN_EINVAL;
  const int grp = Hq / Hkv;
  if (grp > kMaxGroup) return QLIN_EINVAL;
  if (B == 0) return QLIN_OK;
  const dim3 grid((unsigned)(B * Hkv));
  hipStream_t st = (hipStream_t)stream;
#define QLIN_A(G)                                                                          \
  hipLaunchKernelGGL((attn_decode_kernel<G>), grid, dim3(kThreads), 0, st, q,              \
                     (const _Float16*)k, (const _Float16*)v, (const _Float16*)mask, out, Hq, \
                     Hkv, (int)L, scale_div)
  switch (grp) {
    case 1: QLIN_A(1); break;
    case 2: QLIN_A(2); break;
    case 4: QLIN_A(4); break;
    case 8: QLIN_A(8); break;
    default: return QLIN_EINVAL;
  }
#undef QLIN_A
  return (int)hipGetLastError();
}
