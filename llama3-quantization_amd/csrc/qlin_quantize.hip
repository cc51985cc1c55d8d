// qlin_quantize.hip — fused RTN quantizer (calibrate + fake-quant + pack) and the real-quant
// packer, gfx950.
//
// Replaces UniformAffineQuantizer.forward (quant/quantizer.py:118-130): per-group amin/amax
// (:141-142), optional LWC clipping (:143-145), symmetric / asymmetric scale and zero point
// (:146-159), then fake_quant (:94-115) — every op rounded to the element dtype exactly as the
// reference's fp16/fp32 torch ops round (oracle/quant_oracle.py restates the same arithmetic).
//
// Work decomposition: a block of 256 threads owns RPB whole rows.  Phase 1 reduces the min/max of
// each 32-element chunk into LDS; phase 2 reduces one group per thread (a group never crosses a
// row) and computes (scale, zp); phase 3 walks the rows' lane pieces (qlin_common.h tiled layout:
// 4 x 8 elements of one row), re-reads them (L2-hot), fake-quantizes, and writes x_dq and/or the
// packed piece.
#include "qlin_common.h"
#include "../../include/qlin_gfx950.h"

using namespace qlin;

namespace {

constexpr int kThreads = 256;
constexpr int kMaxChunks = 1024;  // chunks per block: K <= 32768


template <typename T>
__device__ __forceinline__ void load32(const T* __restrict__ p, float (&v)[32]) {
  if constexpr (sizeof(T) == 2) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const h8 h = *reinterpret_cast<const h8*>(p + 8 * i);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[8 * i + j] = (float)h[j];
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float4 f = *reinterpret_cast<const float4*>(p + 4 * i);
      v[4 * i] = f.x; v[4 * i + 1] = f.y; v[4 * i + 2] = f.z; v[4 * i + 3] = f.w;
    }
  }
}

// 8 consecutive elements <-> float
template <typename T>
__device__ __forceinline__ void load8(const T* __restrict__ p, float* v) {
  if constexpr (sizeof(T) == 2) {
    const h8 h = *reinterpret_cast<const h8*>(p);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (float)h[j];
  } else {
    const float4 a = *reinterpret_cast<const float4*>(p);
    const float4 b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
}
template <typename T>
__device__ __forceinline__ void store8(T* __restrict__ p, const float* v) {
  if constexpr (sizeof(T) == 2) {
    h8 h;
#pragma unroll
    for (int j = 0; j < 8; ++j) h[j] = (_Float16)v[j];
    *reinterpret_cast<h8*>(p) = h;
  } else {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
}

// pack the 32 codes u[8s + j] of one lane piece (step s, element j) — qlin_common.h layout
template <int BITS>
__device__ __forceinline__ void pack_piece(const uint32_t (&u)[32], uint32_t* __restrict__ out) {
  uint32_t w[BITS];
#pragma unroll
  for (int i = 0; i < BITS; ++i) w[i] = 0;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t c = u[8 * s + j];
      const int h = j & 1, p = j >> 1;
      if constexpr (BITS == 4) {
        w[s] |= c << (16 * h + 4 * p);
      } else if constexpr (BITS == 8) {
        w[2 * s + (j >> 2)] |= c << (16 * h + 8 * ((j & 3) >> 1));
      } else {
        w[s >> 1] |= (c & 3u) << (16 * h + 8 * (s & 1) + 2 * p);
        if constexpr (BITS == 3)
          w[2] |= ((c >> 2) & 1u) << ((16 * h + 2 * p + 2 + rho3(s)) & 31);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < BITS; ++i) out[i] = w[i];
}

template <typename T, int BITS>  // BITS == 0: no packed output
__global__ __launch_bounds__(kThreads) void quantize_kernel(
    const T* __restrict__ x, QP P, const T* __restrict__ up, const T* __restrict__ low,
    T* __restrict__ x_dq, T* __restrict__ scale_out, T* __restrict__ zp_out,
    uint32_t* __restrict__ qweight, uint32_t* __restrict__ qsz) {
  __shared__ float s_min[kMaxChunks];
  __shared__ float s_max[kMaxChunks];
  __shared__ float s_scale[kMaxChunks];
  __shared__ float s_zp[kMaxChunks];
  const int tid = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * P.rpb;
  const int nrows = (int)min((int64_t)P.rpb, P.rows - row0);
  const int nch = nrows * P.cpr;
  const bool has_zp = !(P.flags & QLIN_DISABLE_ZERO_POINT);
  const T* xb = x + row0 * P.K;

  // phase 1: chunk min / max
  for (int c = tid; c < nch; c += kThreads) {
    float v[32];
    load32<T>(xb + (int64_t)c * 32, v);
    float mn = v[0], mx = v[0];
#pragma unroll
    for (int i = 1; i < 32; ++i) { mn = min_nan(mn, v[i]); mx = max_nan(mx, v[i]); }
    s_min[c] = mn;
    s_max[c] = mx;
  }
  __syncthreads();

  // phase 2: per group, min / max over its chunks, then the calibration
  const int ngr = nch / P.cpg;
  const int64_t g0 = row0 * (P.K / P.group);
  auto finish_group = [&](int gi, float mn, float mx) {
    float upf = 1.f, lowf = 1.f;
    if (P.flags & QLIN_LWC) { upf = (float)up[g0 + gi]; lowf = (float)low[g0 + gi]; }
    float scale, zp;
    calib<T>(mn, mx, upf, lowf, P, scale, zp);
    s_scale[gi] = scale;
    s_zp[gi] = zp;
    if (scale_out) scale_out[g0 + gi] = (T)scale;
    if (zp_out && has_zp) zp_out[g0 + gi] = (T)zp;
    if constexpr (BITS > 0) {
      const int Gr = P.K / P.group;
      const int64_t row = row0 + gi / Gr;
      const int g = gi - (gi / Gr) * Gr;
      qsz[sz_index(row >> 4, g, Gr, (int)(row & 15))] =
          sz_pack((_Float16)scale, has_zp ? (int)zp : (1 << (BITS - 1)));
    }
  };
  if (P.cpg <= 8) {  // small groups (g <= 256): one group per thread
    for (int gi = tid; gi < ngr; gi += kThreads) {
      float mn = s_min[gi * P.cpg], mx = s_max[gi * P.cpg];
      for (int j = 1; j < P.cpg; ++j) {
        mn = min_nan(mn, s_min[gi * P.cpg + j]);
        mx = max_nan(mx, s_max[gi * P.cpg + j]);
      }
      finish_group(gi, mn, mx);
    }
  } else {  // long groups (per-channel weights, per-token activations): one group per wave
    const int wave = tid >> 6, lane = tid & 63;
    for (int gi = wave; gi < ngr; gi += kThreads / 64) {
      float mn = __builtin_inff(), mx = -__builtin_inff();
      for (int j = lane; j < P.cpg; j += 64) {
        mn = min_nan(mn, s_min[gi * P.cpg + j]);
        mx = max_nan(mx, s_max[gi * P.cpg + j]);
      }
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        mn = min_nan(mn, __shfl_xor(mn, o));
        mx = max_nan(mx, __shfl_xor(mx, o));
      }
      if (lane == 0) finish_group(gi, mn, mx);
    }
  }
  __syncthreads();

  // phase 3: fake-quant (+ pack), one lane piece (row, k-tile, q) per thread iteration
  const int Kt = (P.K + kTileK - 1) / kTileK;
  const int npc = nrows * Kt * 4;
  for (int pc = tid; pc < npc; pc += kThreads) {
    const int r = pc / (Kt * 4);
    const int rem = pc - r * Kt * 4;
    const int kt = rem >> 2, q = rem & 3;
    const int64_t row = row0 + r;
    uint32_t u[32];
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      const int k0 = kt * kTileK + 32 * st + 8 * q;
      if (k0 < P.K) {
        float v[8], o[8];
        load8<T>(x + row * P.K + k0, v);
        const int gi = r * (P.K / P.group) + k0 / P.group;
        const float sc = s_scale[gi], zp = s_zp[gi];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float xi;
          o[j] = fq<T>(v[j], sc, zp, has_zp, P, xi);
          if (!has_zp) xi += (float)(1 << (P.bits - 1));
          u[8 * st + j] = (xi == xi) ? (uint32_t)(int)xi : 0u;  // NaN (x/s overflow): code 0
        }
        if (x_dq) store8<T>(x_dq + row * P.K + k0, o);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) u[8 * st + j] = 0u;
      }
    }
    if constexpr (BITS > 0)
      pack_piece<BITS>(u, qweight + piece_off(row >> 4, kt, Kt, (int)(row & 15) + 16 * q, BITS));
  }
}

// fake_quant with given (scale, zp) — quant/quantizer.py:94-115 — optionally packing the codes.
// Applied to W_dq with its registered (scales, zeros) it is the real-quant packer
// (quant/omniquant.py:315-335): the codes are recovered with the quantizer's own arithmetic.
template <typename T, int BITS>  // BITS == 0: no packed output
__global__ __launch_bounds__(kThreads) void fq_kernel(
    const T* __restrict__ x, const T* __restrict__ sref, const T* __restrict__ zref,
    int64_t total_pieces, int K, int group, int bits, int flags, T* __restrict__ x_dq,
    uint32_t* __restrict__ qweight, uint32_t* __restrict__ qsz) {
  const int64_t pc = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (pc >= total_pieces) return;
  const int Kt = (K + kTileK - 1) / kTileK;
  const int64_t row = pc / (Kt * 4);
  const int rem = (int)(pc - row * Kt * 4);
  const int kt = rem >> 2, q = rem & 3;
  const bool has_zp = !(flags & QLIN_DISABLE_ZERO_POINT);
  QP P;
  P.bits = bits;
  P.qmin = has_zp ? 0.f : -(float)(1 << (bits - 1));
  P.qmax = has_zp ? (float)((1 << bits) - 1) : (float)((1 << (bits - 1)) - 1);
  uint32_t u[32];
#pragma unroll
  for (int st = 0; st < 4; ++st) {
    const int k0 = kt * kTileK + 32 * st + 8 * q;
    if (k0 < K) {
      const int64_t gidx = row * (K / group) + k0 / group;
      const float sc = (float)sref[gidx];
      const float zp = has_zp ? (float)zref[gidx] : 0.f;
      float v[8], o[8];
      load8<T>(x + row * K + k0, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float xi;
        o[j] = fq<T>(v[j], sc, zp, has_zp, P, xi);
        if (!has_zp) xi += (float)(1 << (bits - 1));
        u[8 * st + j] = (xi == xi) ? (uint32_t)(int)xi : 0u;
      }
      if (x_dq) store8<T>(x_dq + row * K + k0, o);
      if constexpr (BITS > 0) {
        if (k0 % group == 0)
          qsz[sz_index(row >> 4, k0 / group, K / group, (int)(row & 15))] =
              sz_pack((_Float16)sc, has_zp ? (int)zp : (1 << (BITS - 1)));
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) u[8 * st + j] = 0u;
    }
  }
  if constexpr (BITS > 0)
    pack_piece<BITS>(u, qweight + piece_off(row >> 4, kt, Kt, (int)(row & 15) + 16 * q, BITS));
}

// integer codes -> tiled qweight: one thread per lane piece gathers its 32 codes (four 8-byte
// runs of one row) and packs them (converters whose zero points are not integral, e.g. HQQ's
// fp16 zeros, cannot recover codes from W_dq as qlin_pack_f16 does)
template <int BITS>
__global__ __launch_bounds__(kThreads) void pack_codes_kernel(const uint8_t* __restrict__ codes,
                                                              int64_t pieces, int N, int K,
                                                              uint32_t* __restrict__ qweight) {
  const int64_t pc = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  if (pc >= pieces) return;
  const int Kt = (K + kTileK - 1) / kTileK;
  const int lane = (int)(pc & 63);
  const int64_t tt = pc >> 6;
  const int kt = (int)(tt % Kt);
  const int64_t row = (tt / Kt) * kTileN + (lane & 15);
  const int q = lane >> 4;
  constexpr uint32_t mask = (1u << BITS) - 1u;
  uint32_t u[32];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int k = kt * kTileK + 32 * s + 8 * q;  // K % 32 == 0: a run is wholly in or out
    uint2 r = make_uint2(0u, 0u);
    if (row < N && k < K) r = *reinterpret_cast<const uint2*>(codes + row * K + k);
#pragma unroll
    for (int j = 0; j < 8; ++j) u[8 * s + j] = ((j < 4 ? r.x : r.y) >> (8 * (j & 3))) & mask;
  }
  pack_piece<BITS>(u, qweight + pc * BITS);
}

// one group per row of any length K (per-token activations, per-channel weights) without packing:
// QuantMatMul's per-token operands have K = the key count L, not a multiple of 32.  One wave per
// row: min / max (order-free, NaN-propagating: bit-exact), the reference calibration, fake-quant.
template <typename T>
__global__ __launch_bounds__(kThreads) void rowq_kernel(const T* __restrict__ x, QP P,
                                                        const T* __restrict__ up,
                                                        const T* __restrict__ low,
                                                        T* __restrict__ x_dq,
                                                        T* __restrict__ scale_out,
                                                        T* __restrict__ zp_out) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * (kThreads / 64) + wave;
  if (row >= P.rows) return;
  const T* xr = x + row * P.K;
  float mn = __builtin_inff(), mx = -__builtin_inff();
  for (int k = lane; k < P.K; k += 64) {
    const float v = (float)xr[k];
    mn = min_nan(mn, v);
    mx = max_nan(mx, v);
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    mn = min_nan(mn, __shfl_xor(mn, o));
    mx = max_nan(mx, __shfl_xor(mx, o));
  }
  float upf = 1.f, lowf = 1.f;
  if (P.flags & QLIN_LWC) { upf = (float)up[row]; lowf = (float)low[row]; }
  float scale, zp;
  calib<T>(mn, mx, upf, lowf, P, scale, zp);
  const bool has_zp = !(P.flags & QLIN_DISABLE_ZERO_POINT);
  if (lane == 0) {
    if (scale_out) scale_out[row] = (T)scale;
    if (zp_out && has_zp) zp_out[row] = (T)zp;
  }
  if (!x_dq) return;
  for (int k = lane; k < P.K; k += 64) {
    float xi;
    x_dq[row * P.K + k] = (T)fq<T>((float)xr[k], scale, zp, has_zp, P, xi);
  }
}

template <typename T>
int launch_quantize(const void* x, int64_t rows, int64_t K, int bits, int group, int flags,
                    const void* up, const void* low, void* x_dq, void* scale_out, void* zp_out,
                    uint32_t* qweight, uint32_t* qsz, hipStream_t st) {
  QP P;
  P.rows = rows;
  P.K = (int)K;
  P.group = group;
  P.cpr = (int)(K / 32);
  P.cpg = group / 32;
  P.rpb = P.cpr >= kThreads ? 1 : kThreads / (P.cpr > 0 ? P.cpr : 1);
  P.bits = bits;
  P.flags = flags;
  const bool has_zp = !(flags & QLIN_DISABLE_ZERO_POINT);
  P.qmin = has_zp ? 0.f : -(float)(1 << (bits - 1));
  P.qmax = has_zp ? (float)((1 << bits) - 1) : (float)((1 << (bits - 1)) - 1);
  const bool pack = qweight != nullptr;
  const T* xx = (const T*)x;
  if (K % 32 || K / 32 > kMaxChunks) {  // one whole-row group, no packing (checked by the caller)
    hipLaunchKernelGGL((rowq_kernel<T>), dim3((unsigned)((rows + 3) / 4)), dim3(kThreads), 0, st,
                       xx, P, (const T*)up, (const T*)low, (T*)x_dq, (T*)scale_out, (T*)zp_out);
    return (int)hipGetLastError();
  }
  const dim3 grid((unsigned)((rows + P.rpb - 1) / P.rpb));
#define QLIN_Q(B)                                                                            \
  hipLaunchKernelGGL((quantize_kernel<T, B>), grid, dim3(kThreads), 0, st, xx, P,            \
                     (const T*)up, (const T*)low, (T*)x_dq, (T*)scale_out, (T*)zp_out,       \
                     qweight, qsz)
  if (!pack) QLIN_Q(0);
  else if (bits == 2) QLIN_Q(2);
  else if (bits == 3) QLIN_Q(3);
  else if (bits == 4) QLIN_Q(4);
  else QLIN_Q(8);
#undef QLIN_Q
  return (int)hipGetLastError();
}

}  // namespace

extern "C" int qlin_abi_version(void) { return QLIN_ABI_VERSION; }

extern "C" const char* qlin_error_string(int code) {
  if (code == QLIN_OK) return "ok";
  if (code == QLIN_EINVAL) return "invalid argument";
  return hipGetErrorString((hipError_t)code);
}

extern "C" int qlin_quantize(const void* x, int dtype, int64_t rows, int64_t K, int bits,
                             int group, int flags, const void* lwc_up_sig,
                             const void* lwc_low_sig, void* x_dq, void* scale_out, void* zp_out,
                             uint32_t* qweight, uint32_t* qsz, void* stream) {
  const bool pack = qweight || qsz;
  // K % 32 != 0 (or K > 32768): only one group per row and no packing (rowq_kernel)
  const bool rowwise = K > 0 && (K % 32 || K / 32 > kMaxChunks);
  if (!x || rows < 0 || K <= 0 || K > (1 << 24) || group <= 0 || K % group || bits < 2 ||
      bits > 8 || (dtype != QLIN_F16 && dtype != QLIN_F32) ||
      (rowwise ? (group != K || pack) : group % 32 != 0))
    return QLIN_EINVAL;
  if ((flags & QLIN_LWC) && (!lwc_up_sig || !lwc_low_sig)) return QLIN_EINVAL;
  if (pack && (!qweight || !qsz || dtype != QLIN_F16 ||
               !(bits == 2 || bits == 3 || bits == 4 || bits == 8)))
    return QLIN_EINVAL;
  if (rows == 0) return QLIN_OK;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == QLIN_F16)
    return launch_quantize<_Float16>(x, rows, K, bits, group, flags, lwc_up_sig, lwc_low_sig,
                                     x_dq, scale_out, zp_out, qweight, qsz, st);
  return launch_quantize<float>(x, rows, K, bits, group, flags, lwc_up_sig, lwc_low_sig, x_dq,
                                scale_out, zp_out, nullptr, nullptr, st);
}

extern "C" int qlin_fake_quant(const void* x, int dtype, const void* scale, const void* zp,
                               int64_t rows, int64_t K, int bits, int group, int flags,
                               void* x_dq, uint32_t* qweight, uint32_t* qsz, void* stream) {
  const bool has_zp = !(flags & QLIN_DISABLE_ZERO_POINT);
  const bool pack = qweight || qsz;
  if (!x || !scale || (has_zp && !zp) || rows < 0 || K <= 0 || K % 32 || group <= 0 ||
      group % 32 || K % group || bits < 2 || bits > 8 || (dtype != QLIN_F16 && dtype != QLIN_F32))
    return QLIN_EINVAL;
  if (pack && (!qweight || !qsz || dtype != QLIN_F16 ||
               !(bits == 2 || bits == 3 || bits == 4 || bits == 8)))
    return QLIN_EINVAL;
  const int64_t pieces = rows * ((K + kTileK - 1) / kTileK) * 4;
  if (pieces == 0) return QLIN_OK;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)((pieces + kThreads - 1) / kThreads));
  if (dtype == QLIN_F32) {
    hipLaunchKernelGGL((fq_kernel<float, 0>), grid, dim3(kThreads), 0, st, (const float*)x,
                       (const float*)scale, (const float*)zp, pieces, (int)K, group, bits, flags,
                       (float*)x_dq, nullptr, nullptr);
    return (int)hipGetLastError();
  }
#define QLIN_P(B)                                                                            \
  hipLaunchKernelGGL((fq_kernel<_Float16, B>), grid, dim3(kThreads), 0, st, (const _Float16*)x, \
                     (const _Float16*)scale, (const _Float16*)zp, pieces, (int)K, group, bits,  \
                     flags, (_Float16*)x_dq, qweight, qsz)
  if (!pack) QLIN_P(0);
  else if (bits == 2) QLIN_P(2);
  else if (bits == 3) QLIN_P(3);
  else if (bits == 4) QLIN_P(4);
  else QLIN_P(8);
#undef QLIN_P
  return (int)hipGetLastError();
}

extern "C" int qlin_pack_f16(const uint16_t* w_dq, const uint16_t* scales_ref,
                             const uint16_t* zeros_ref, int64_t N, int64_t K, int bits, int group,
                             int flags, uint32_t* qweight, uint32_t* qsz, void* stream) {
  if (!w_dq || !qweight || !qsz) return QLIN_EINVAL;
  return qlin_fake_quant(w_dq, QLIN_F16, scales_ref, zeros_ref, N, K, bits, group, flags, nullptr,
                         qweight, qsz, stream);
}

extern "C" int qlin_pack_codes(const uint8_t* codes, int64_t N, int64_t K, int bits,
                               uint32_t* qweight, void* stream) {
  if (!codes || !qweight || N < 0 || N > (1 << 30) || K <= 0 || K % 32 || K > (1 << 20) ||
      !(bits == 2 || bits == 3 || bits == 4 || bits == 8))
    return QLIN_EINVAL;
  const int64_t pieces = ((N + kTileN - 1) / kTileN) * ((K + kTileK - 1) / kTileK) * 64;
  if (pieces == 0) return QLIN_OK;
  hipStream_t st = (hipStream_t)stream;
  const dim3 grid((unsigned)((pieces + kThreads - 1) / kThreads));
#define QLIN_PC(B)                                                                             \
  hipLaunchKernelGGL((pack_codes_kernel<B>), grid, dim3(kThreads), 0, st, codes, pieces,       \
                     (int)N, (int)K, qweight);                                                 \
  break
  switch (bits) {
    case 2: QLIN_PC(2);
    case 3: QLIN_PC(3);
    case 4: QLIN_PC(4);
    default: QLIN_PC(8);
  }
#undef QLIN_PC
  return (int)hipGetLastError();
}
