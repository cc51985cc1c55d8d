// qlin_layer.hip — the decoder layer's elementwise glue around the quantized linears, gfx950:
// RMSNorm and rotary position embedding, one launch each (the reference runs each as 5-14
// PyTorch kernels per layer and token; at batch-1 decode they cost more than the 7 packed
// linears' HBM time).
//
// qlin_rmsnorm_f16 replaces OmniLlamaRMSNorm.forward (quant/omni_norm.py:52-63 of the reference):
//   var = mean(x.float()^2); h = x * rsqrt(var + eps) (fp32); y = (weight * h).to(fp16).
// One block per row; the sum of squares runs in a different order than torch's reduction, so y
// can differ from the reference by one fp16 ulp where var's last bit differs.
//
// qlin_rope_f16 replaces, in QuantLlamaAttention.forward (models/int_llama_layer.py:116-125),
// the q/k reshape + transpose, q's cast to fp32, rotary_emb(cos/sin cache slice, cast to fp16)
// and apply_rotary_pos_emb (index by position_ids, q*cos + rotate_half(q)*sin in fp32 for q,
// the same in fp16 for k: every product and the sum rounded to fp16 as torch's fp16 ops do).
// Elementwise with the reference's op order and roundings: bit-exact.
//
// qlin_attn_scores_f32 replaces, for prefill windows, the three fp32 passes over the
// [B, H, T, L] score tensor after QK^T (models/int_llama_layer.py:143-157: / sqrt(head_dim),
// + attention_mask, torch.max(w, finfo.min)) with one in-place pass, bit-exact.
#include "qlin_common.h"
#include "../../include/qlin_gfx950.h"

namespace {

using qlin::h2;
using qlin::h8;

constexpr int kNormThreads = 256;
constexpr int kNormCPT = 4;  // 8-half chunks a thread keeps in registers: H <= 8192

// block sum of a per-thread float (every thread gets the total)
__device__ __forceinline__ float block_sum(float v, float* part) {
  v = qlin::row16_sum(v);
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = v;
  __syncthreads();
  float tot = 0.f;
#pragma unroll
  for (int i = 0; i < kNormThreads / 64; ++i) tot += part[i];
  return tot;
}

// H % 8 == 0 and H <= 8 * kNormThreads * kNormCPT: x read once with 16-B loads, kept in registers
__global__ __launch_bounds__(kNormThreads) void rmsnorm_vec_kernel(
    const _Float16* __restrict__ x, const float* __restrict__ w, _Float16* __restrict__ y,
    int H, float eps) {
#pragma clang fp contract(off)
  __shared__ float part[kNormThreads / 64];
  const int64_t row = blockIdx.x;
  const uint4* xr = reinterpret_cast<const uint4*>(x + row * H);
  const int nch = H >> 3;
  uint4 xv[kNormCPT];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < kNormCPT; ++c) {
    const int ch = c * kNormThreads + threadIdx.x;
    xv[c] = ch < nch ? xr[ch] : make_uint4(0u, 0u, 0u, 0u);
    const h8 v = __builtin_bit_cast(h8, xv[c]);
#pragma unroll
    for (int j = 0; j < 8; ++j) ss += (float)v[j] * (float)v[j];
  }
  const float var = block_sum(ss, part) / (float)H;
  const float r = rsqrtf(var + eps);
  uint4* yr = reinterpret_cast<uint4*>(y + row * H);
  const float4* wr = reinterpret_cast<const float4*>(w);
#pragma unroll
  for (int c = 0; c < kNormCPT; ++c) {
    const int ch = c * kNormThreads + threadIdx.x;
    if (ch >= nch) break;
    const h8 v = __builtin_bit_cast(h8, xv[c]);
    const float4 w0 = wr[2 * ch], w1 = wr[2 * ch + 1];
    const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
    h8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (_Float16)(wv[j] * ((float)v[j] * r));
    yr[ch] = __builtin_bit_cast(uint4, o);
  }
}

// any H: two passes over the row
__global__ __launch_bounds__(kNormThreads) void rmsnorm_kernel(
    const _Float16* __restrict__ x, const float* __restrict__ w, _Float16* __restrict__ y,
    int64_t H, float eps) {
#pragma clang fp contract(off)
  __shared__ float part[kNormThreads / 64];
  const int64_t row = blockIdx.x;
  const _Float16* xr = x + row * H;
  float ss = 0.f;
  for (int64_t i = threadIdx.x; i < H; i += kNormThreads) {
    const float v = (float)xr[i];
    ss += v * v;
  }
  const float var = block_sum(ss, part) / (float)H;
  const float r = rsqrtf(var + eps);
  _Float16* yr = y + row * H;
  for (int64_t i = threadIdx.x; i < H; i += kNormThreads) {
    const float h = (float)xr[i] * r;
    yr[i] = (_Float16)(w[i] * h);
  }
}

// one thread per (b, s, head, d) of q (Hq heads) and k (Hkv heads)
__global__ __launch_bounds__(256) void rope_kernel(
    const _Float16* __restrict__ q, int64_t q_rs, const _Float16* __restrict__ k, int64_t k_rs,
    const float* __restrict__ cosc, const float* __restrict__ sinc, int64_t cache_rows,
    const int64_t* __restrict__ pos, int64_t pos_bs, float* __restrict__ q_out,
    _Float16* __restrict__ k_out, int64_t B, int64_t S, int Hq, int Hkv, int D) {
#pragma clang fp contract(off)
  const int64_t total = B * S * (int64_t)(Hq + Hkv) * D;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int d = (int)(i % D);
  int64_t t = i / D;
  const int h = (int)(t % (Hq + Hkv));
  t /= (Hq + Hkv);
  const int64_t s = t % S, b = t / S;
  // positions outside the cache are clamped (never read out of bounds; the reference raises)
  const int64_t p = min(max(pos[b * pos_bs + s], (int64_t)0), cache_rows - 1);
  // the reference's cos/sin: the fp32 cache sliced and cast to the activation dtype (fp16)
  const float c = (float)(_Float16)cosc[p * D + d];
  const float sn = (float)(_Float16)sinc[p * D + d];
  const int half = D / 2;
  const int dr = d < half ? d + half : d - half;  // rotate_half partner
  if (h < Hq) {
    const _Float16* qr = q + (b * S + s) * q_rs + (int64_t)h * D;
    const float v = (float)qr[d];
    const float rv = d < half ? -(float)qr[dr] : (float)qr[dr];
    q_out[((b * Hq + h) * S + s) * D + d] = v * c + rv * sn;  // fp32, each op rounded once
  } else {
    const int hk = h - Hq;
    const _Float16* kr = k + (b * S + s) * k_rs + (int64_t)hk * D;
    const float v = (float)kr[d];
    const float rv = d < half ? -(float)kr[dr] : (float)kr[dr];
    const float a = (float)(_Float16)(v * c), bb = (float)(_Float16)(rv * sn);
    k_out[((b * Hkv + hk) * S + s) * D + d] = (_Float16)(a + bb);
  }
}

// attention scores of a prefill window, in place: w = max(w / scale + mask, finfo(fp32).min)
// (w / scale alone without a mask)
// with torch's scalar division (multiplication by the fp32 reciprocal), one pass instead of three
template <bool MASK32>
__global__ __launch_bounds__(256) void attn_scores_kernel(float* __restrict__ w,
                                                          const void* __restrict__ mask,
                                                          int64_t n4, int64_t L, int64_t rows_per_b,
                                                          int64_t T, int64_t mask_bs, float inv) {
#pragma clang fp contract(off)
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n4) return;
  const int64_t e = 4 * i;             // L % 4 == 0: the four elements share a row
  const int64_t row = e / L, l = e - row * L;
  const int64_t b = row / rows_per_b;  // rows_per_b = H * T
  const int64_t t = row % T;
  float4 v = reinterpret_cast<float4*>(w)[i];
  float m[4] = {0.f, 0.f, 0.f, 0.f};
  if (mask) {
    const int64_t mo = b * mask_bs + t * L + l;
    if constexpr (MASK32) {
      const float4 mm = *reinterpret_cast<const float4*>((const float*)mask + mo);
      m[0] = mm.x; m[1] = mm.y; m[2] = mm.z; m[3] = mm.w;
    } else {
      const uint2 mm = *reinterpret_cast<const uint2*>((const _Float16*)mask + mo);
      const h2 a = __builtin_bit_cast(h2, mm.x), c = __builtin_bit_cast(h2, mm.y);
      m[0] = (float)a.x; m[1] = (float)a.y; m[2] = (float)c.x; m[3] = (float)c.y;
    }
  }
  float* vv = reinterpret_cast<float*>(&v);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float s = vv[j] * inv;
    if (mask) {  // the reference clamps only after adding a mask
      s = s + m[j];
      s = (s != s) ? s : fmaxf(s, -3.402823466e38f);  // torch.max(w, finfo.min): NaN stays
    }
    vv[j] = s;
  }
  reinterpret_cast<float4*>(w)[i] = v;
}

}  // namespace

extern "C" int qlin_attn_scores_f32(float* scores, const void* mask, int mask_dtype, int64_t B,
                                    int64_t H, int64_t T, int64_t L, int64_t mask_batch_stride,
                                    float scale_div, void* stream) {
  if (!scores || B < 0 || H < 0 || T < 0 || L <= 0 || L % 4 || mask_batch_stride < 0 ||
      (mask && mask_dtype != QLIN_F16 && mask_dtype != QLIN_F32) || !(scale_div > 0.f) ||
      ((uintptr_t)scores & 15))
    return QLIN_EINVAL;
  const int64_t n4 = B * H * T * L / 4;
  if (n4 == 0) return QLIN_OK;
  if ((n4 + 255) / 256 > 0x7fffffff) return QLIN_EINVAL;
  const float inv = 1.0f / scale_div;
  const dim3 grid((unsigned)((n4 + 255) / 256));
  if (mask_dtype == QLIN_F32)
    hipLaunchKernelGGL(attn_scores_kernel<true>, grid, dim3(256), 0, (hipStream_t)stream, scores,
                       mask, n4, L, H * T, T, mask_batch_stride, inv);
  else
    hipLaunchKernelGGL(attn_scores_kernel<false>, grid, dim3(256), 0, (hipStream_t)stream, scores,
                       mask, n4, L, H * T, T, mask_batch_stride, inv);
  return (int)hipGetLastError();
}

extern "C" int qlin_rmsnorm_f16(const uint16_t* x, const float* weight, uint16_t* y, int64_t rows,
                                int64_t H, float eps, void* stream) {
  if (!x || !weight || !y || rows < 0 || H <= 0 || rows > 0x7fffffff) return QLIN_EINVAL;
  if (rows == 0) return QLIN_OK;
  const bool vec = H % 8 == 0 && H <= 8 * kNormThreads * kNormCPT &&
                   ((uintptr_t)x | (uintptr_t)y) % 16 == 0 && (uintptr_t)weight % 16 == 0;
  if (vec)
    hipLaunchKernelGGL(rmsnorm_vec_kernel, dim3((unsigned)rows), dim3(kNormThreads), 0,
                       (hipStream_t)stream, (const _Float16*)x, weight, (_Float16*)y, (int)H, eps);
  else
    hipLaunchKernelGGL(rmsnorm_kernel, dim3((unsigned)rows), dim3(kNormThreads), 0,
                       (hipStream_t)stream, (const _Float16*)x, weight, (_Float16*)y, H, eps);
  return (int)hipGetLastError();
}

extern "C" int qlin_rope_f16(const uint16_t* q, int64_t q_row_stride, const uint16_t* k,
                             int64_t k_row_stride, const float* cos_cache, const float* sin_cache,
                             int64_t cache_rows, const int64_t* position_ids,
                             int64_t pos_batch_stride, float* q_out, uint16_t* k_out, int64_t B,
                             int64_t S, int Hq, int Hkv, int D, void* stream) {
  if (!q || !k || !cos_cache || !sin_cache || !position_ids || !q_out || !k_out || B < 0 ||
      S < 0 || Hq <= 0 || Hkv <= 0 || D <= 0 || D % 2 || q_row_stride < (int64_t)Hq * D ||
      k_row_stride < (int64_t)Hkv * D || pos_batch_stride < 0 || cache_rows <= 0)
    return QLIN_EINVAL;
  const int64_t total = B * S * (int64_t)(Hq + Hkv) * D;
  if (total == 0) return QLIN_OK;
  if ((total + 255) / 256 > 0x7fffffff) return QLIN_EINVAL;
  hipLaunchKernelGGL(rope_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, (const _Float16*)q, q_row_stride, (const _Float16*)k,
                     k_row_stride, cos_cache, sin_cache, cache_rows, position_ids,
                     pos_batch_stride, q_out, (_Float16*)k_out, B, S, Hq, Hkv, D);
  return (int)hipGetLastError();
}
