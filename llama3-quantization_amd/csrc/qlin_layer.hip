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
// Elementwise with the reference's op order and roundings: bit-exact.  One block per token row
// (the position and the cos / sin rows read once per block), each thread rotating four
// (d, d + D/2) pairs with 8-B / 16-B accesses; qlin_rope_kv_f16 also writes the rotated k and
// the v row straight into a KV cache at row kv0 + s (the reference's torch.cat of the cache,
// models/int_llama_layer.py:130-135, without re-copying the cache).  A 2048-token window:
// 50 us (one thread per element, 64-bit index math) -> see DESIGN.md §4.
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

struct RopeArgs {
  const _Float16* q;
  int64_t q_rs;
  const _Float16* k;
  int64_t k_rs;
  const _Float16* v;  // nullptr: no v copy
  int64_t v_rs;
  const float* cosc;
  const float* sinc;
  int64_t cache_rows;
  const int64_t* pos;
  int64_t pos_bs;
  float* q_out;      // [B, Hq, S, D]
  _Float16* k_out;   // [B, Hkv, kv_rows, D], rows kv0 .. kv0 + S - 1 written
  _Float16* v_out;
  int64_t kv_rows, kv0;
  int S, Hq, Hkv, D;
};

// one block per (b, s); D % 8 == 0, q / k / v rows and strides 4-element aligned, outputs 16-B
// aligned (checked on the host)
__global__ __launch_bounds__(256) void rope_rows_kernel(RopeArgs a) {
#pragma clang fp contract(off)
  typedef _Float16 h4 __attribute__((ext_vector_type(4)));
  const int64_t bs = blockIdx.x;
  const int64_t b = bs / a.S;
  const int s = (int)(bs - b * a.S);
  const int64_t p = min(max(a.pos[b * a.pos_bs + s], (int64_t)0), a.cache_rows - 1);
  const int D = a.D, half = D >> 1, nq = half >> 2;
  const float* cr = a.cosc + p * D;
  const float* sr = a.sinc + p * D;
  const int items = (a.Hq + a.Hkv) * nq;
  for (int it = threadIdx.x; it < items; it += 256) {
    const int h = it / nq, d0 = (it - h * nq) * 4;
    const float4 cl4 = *reinterpret_cast<const float4*>(cr + d0);
    const float4 ch4 = *reinterpret_cast<const float4*>(cr + d0 + half);
    const float4 sl4 = *reinterpret_cast<const float4*>(sr + d0);
    const float4 sh4 = *reinterpret_cast<const float4*>(sr + d0 + half);
    // the reference's cos / sin: the fp32 cache cast to the activation dtype (fp16)
    const float cl[4] = {(float)(_Float16)cl4.x, (float)(_Float16)cl4.y, (float)(_Float16)cl4.z,
                         (float)(_Float16)cl4.w};
    const float chh[4] = {(float)(_Float16)ch4.x, (float)(_Float16)ch4.y, (float)(_Float16)ch4.z,
                          (float)(_Float16)ch4.w};
    const float sl[4] = {(float)(_Float16)sl4.x, (float)(_Float16)sl4.y, (float)(_Float16)sl4.z,
                         (float)(_Float16)sl4.w};
    const float shh[4] = {(float)(_Float16)sh4.x, (float)(_Float16)sh4.y, (float)(_Float16)sh4.z,
                          (float)(_Float16)sh4.w};
    if (h < a.Hq) {
      const _Float16* qr = a.q + (b * a.S + s) * a.q_rs + (int64_t)h * D;
      const h4 lo = *reinterpret_cast<const h4*>(qr + d0);
      const h4 hi = *reinterpret_cast<const h4*>(qr + d0 + half);
      float ol[4], oh[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        // fp32: q * cos + rotate_half(q) * sin, rotate_half = (-q[d + D/2], q[d - D/2])
        ol[j] = (float)lo[j] * cl[j] + (-(float)hi[j]) * sl[j];
        oh[j] = (float)hi[j] * chh[j] + (float)lo[j] * shh[j];
      }
      float* qo = a.q_out + ((b * a.Hq + h) * a.S + s) * (int64_t)D;
      *reinterpret_cast<float4*>(qo + d0) = make_float4(ol[0], ol[1], ol[2], ol[3]);
      *reinterpret_cast<float4*>(qo + d0 + half) = make_float4(oh[0], oh[1], oh[2], oh[3]);
    } else {
      const int hk = h - a.Hq;
      const _Float16* kr = a.k + (b * a.S + s) * a.k_rs + (int64_t)hk * D;
      const h4 lo = *reinterpret_cast<const h4*>(kr + d0);
      const h4 hi = *reinterpret_cast<const h4*>(kr + d0 + half);
      h4 ol, oh;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        // fp16 ops: every product and the sum rounded to fp16
        const float a0 = (float)(_Float16)((float)lo[j] * cl[j]);
        const float b0 = (float)(_Float16)((-(float)hi[j]) * sl[j]);
        ol[j] = (_Float16)(a0 + b0);
        const float a1 = (float)(_Float16)((float)hi[j] * chh[j]);
        const float b1 = (float)(_Float16)((float)lo[j] * shh[j]);
        oh[j] = (_Float16)(a1 + b1);
      }
      _Float16* ko = a.k_out + ((b * a.Hkv + hk) * a.kv_rows + a.kv0 + s) * (int64_t)D;
      *reinterpret_cast<h4*>(ko + d0) = ol;
      *reinterpret_cast<h4*>(ko + d0 + half) = oh;
    }
  }
  if (a.v) {  // the v row into the cache (8 halves per thread and step)
    const int nv = a.Hkv * (D >> 3);
    for (int it = threadIdx.x; it < nv; it += 256) {
      const int hk = it / (D >> 3), d0 = (it - hk * (D >> 3)) * 8;
      const _Float16* vr = a.v + (b * a.S + s) * a.v_rs + (int64_t)hk * D + d0;
      typedef _Float16 h4v __attribute__((ext_vector_type(4)));
      const h4v v0 = *reinterpret_cast<const h4v*>(vr);
      const h4v v1 = *reinterpret_cast<const h4v*>(vr + 4);
      _Float16* vo = a.v_out + ((b * a.Hkv + hk) * a.kv_rows + a.kv0 + s) * (int64_t)D + d0;
      *reinterpret_cast<h4v*>(vo) = v0;
      *reinterpret_cast<h4v*>(vo + 4) = v1;
    }
  }
}

// the vector kernel's alignment / shape conditions
bool rope_rows_ok(const RopeArgs& a) {
  const auto al = [](const void* p, uintptr_t n) { return ((uintptr_t)p % n) == 0; };
  return a.D % 8 == 0 && a.q_rs % 4 == 0 && a.k_rs % 4 == 0 && al(a.q, 8) && al(a.k, 8) &&
         al(a.cosc, 16) && al(a.sinc, 16) && al(a.q_out, 16) && al(a.k_out, 8) &&
         (!a.v || (a.v_rs % 4 == 0 && al(a.v, 8) && al(a.v_out, 8)));
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
  const RopeArgs ra{(const _Float16*)q, q_row_stride, (const _Float16*)k, k_row_stride, nullptr, 0,
                    cos_cache, sin_cache, cache_rows, position_ids, pos_batch_stride, q_out,
                    (_Float16*)k_out, nullptr, S, 0, (int)S, Hq, Hkv, D};
  if (rope_rows_ok(ra) && B * S <= 0x7fffffff && S <= 0x7fffffff) {
    hipLaunchKernelGGL(rope_rows_kernel, dim3((unsigned)(B * S)), dim3(256), 0,
                       (hipStream_t)stream, ra);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(rope_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, (const _Float16*)q, q_row_stride, (const _Float16*)k,
                     k_row_stride, cos_cache, sin_cache, cache_rows, position_ids,
                     pos_batch_stride, q_out, (_Float16*)k_out, B, S, Hq, Hkv, D);
  return (int)hipGetLastError();
}

extern "C" int qlin_rope_kv_f16(const uint16_t* q, int64_t q_row_stride, const uint16_t* k,
                                int64_t k_row_stride, const uint16_t* v, int64_t v_row_stride,
                                const float* cos_cache, const float* sin_cache, int64_t cache_rows,
                                const int64_t* position_ids, int64_t pos_batch_stride,
                                float* q_out, uint16_t* k_cache, uint16_t* v_cache,
                                int64_t kv_rows, int64_t kv0, int64_t B, int64_t S, int Hq,
                                int Hkv, int D, void* stream) {
  if (!q || !k || !v || !cos_cache || !sin_cache || !position_ids || !q_out || !k_cache ||
      !v_cache || B < 0 || S < 0 || Hq <= 0 || Hkv <= 0 || D <= 0 ||
      q_row_stride < (int64_t)Hq * D || k_row_stride < (int64_t)Hkv * D ||
      v_row_stride < (int64_t)Hkv * D || pos_batch_stride < 0 || cache_rows <= 0 || kv0 < 0 ||
      kv0 + S > kv_rows || B * S > 0x7fffffff || S > 0x7fffffff)
    return QLIN_EINVAL;
  const RopeArgs ra{(const _Float16*)q, q_row_stride, (const _Float16*)k, k_row_stride,
                    (const _Float16*)v, v_row_stride, cos_cache, sin_cache, cache_rows,
                    position_ids, pos_batch_stride, q_out, (_Float16*)k_cache,
                    (_Float16*)v_cache, kv_rows, kv0, (int)S, Hq, Hkv, D};
  if (!rope_rows_ok(ra)) return QLIN_EINVAL;
  if (B * S == 0) return QLIN_OK;
  hipLaunchKernelGGL(rope_rows_kernel, dim3((unsigned)(B * S)), dim3(256), 0, (hipStream_t)stream,
                     ra);
  return (int)hipGetLastError();
}
