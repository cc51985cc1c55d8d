// qlin_common.h — device helpers shared by the gfx950 quantized-linear kernels.
//
// Written for CDNA4 (gfx950, wave64) only.
//
// Packed layout ("qlin tiled", include/qlin_gfx950.h): qweight is a grid of 16-row x 128-k tiles;
// a tile is 64 lane pieces of BITS uint32.  Lane l = n + 16q holds the 32 codes (s, j), s < 4,
// j < 8, of tile row n at k = 32s + 8q + j, i.e. exactly the B operand that lane feeds to k-step s
// of v_mfma_f32_16x16x32_f16 (B[k = 8q + j][col n]).  A GEMV wave therefore streams one fully
// coalesced 64 x (4*BITS)-byte load per tile and needs no shuffles.
//
// Unpack: codes sit in each 16-bit half so that ONE v_and_or_b32 with an fp16 exponent "magic"
// (1024, 256, 64 or 16, chosen so the code's weight in the mantissa is exactly 1) turns a pair of
// codes into the fp16 pair (off + u_j, off + u_j+1).  Two uses:
//   exact dequant: (off + u) - (off + zp) is the exact integer u - zp, and one v_pk_mul_f16 by the
//     group scale rounds once — bit-identical to the reference's fp16
//     x_dequant.sub(round_zero_point).mul(scale) (quant/quantizer.py:107-110);
//   GEMV: the MFMA consumes (off + u) directly; sum_k (off_k + u_k - off_k - zp) x_k * s is
//     recovered per group from two per-group x sums (S1 = sum off_k x_k, S2 = sum x_k).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/qlin_gfx950.h"

namespace qlin {

typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

constexpr int kTileN = 16;
constexpr int kTileK = 128;

__device__ __forceinline__ h2 as_h2(uint32_t u) { return __builtin_bit_cast(h2, u); }
__device__ __forceinline__ uint32_t as_u32(h2 v) { return __builtin_bit_cast(uint32_t, v); }

// round a float32 value to the element dtype and back (the reference's per-op rounding)
template <typename T> struct Elt;
template <> struct Elt<_Float16> {
  static __device__ __forceinline__ float rn(float v) { return (float)(_Float16)v; }
};
template <> struct Elt<float> {
  static __device__ __forceinline__ float rn(float v) { return v; }
};

// torch.clamp semantics: NaN propagates (fminf/fmaxf would drop it)
__device__ __forceinline__ float clamp_nan(float v, float lo, float hi) {
  return (v != v) ? v : fminf(fmaxf(v, lo), hi);
}
// torch.amin / amax semantics: NaN propagates
__device__ __forceinline__ float min_nan(float a, float b) { return (a != a || b != b) ? __builtin_nanf("") : fminf(a, b); }
__device__ __forceinline__ float max_nan(float a, float b) { return (a != a || b != b) ? __builtin_nanf("") : fmaxf(a, b); }

// ---------------------------------------------------------------------------------------------
// tiled layout
// ---------------------------------------------------------------------------------------------
template <int BITS> struct Piece { uint32_t w[BITS]; };

// word offset of lane piece (nt, kt, lane)
__device__ __forceinline__ int64_t piece_off(int64_t nt, int kt, int Kt, int lane, int bits) {
  return ((nt * Kt + kt) * 64 + lane) * bits;
}

template <int BITS>
__device__ __forceinline__ Piece<BITS> load_piece(const uint32_t* __restrict__ p) {
  Piece<BITS> c;
  if constexpr (BITS == 4) {
    const uint4 v = *reinterpret_cast<const uint4*>(p);
    c.w[0] = v.x; c.w[1] = v.y; c.w[2] = v.z; c.w[3] = v.w;
  } else if constexpr (BITS == 8) {
    const uint4 a = *reinterpret_cast<const uint4*>(p);
    const uint4 b = *reinterpret_cast<const uint4*>(p + 4);
    c.w[0] = a.x; c.w[1] = a.y; c.w[2] = a.z; c.w[3] = a.w;
    c.w[4] = b.x; c.w[5] = b.y; c.w[6] = b.z; c.w[7] = b.w;
  } else if constexpr (BITS == 2) {
    const uint2 v = *reinterpret_cast<const uint2*>(p);
    c.w[0] = v.x; c.w[1] = v.y;
  } else {  // 3: 12 bytes, 4-byte aligned -> global_load_dwordx3
    struct U3 { uint32_t a, b, c; };
    const U3 v = *reinterpret_cast<const U3*>(p);
    c.w[0] = v.a; c.w[1] = v.b; c.w[2] = v.c;
  }
  return c;
}

// the same with the non-temporal hint on the streamed (read-once) weight bytes: measured
// -5 % per 4096 x 4096 GEMV launch (tools/dev/gemv_lab.hip)
template <int BITS>
__device__ __forceinline__ Piece<BITS> load_piece_nt(const uint32_t* __restrict__ p) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  Piece<BITS> c;
  if constexpr (BITS == 4) {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    c.w[0] = v.x; c.w[1] = v.y; c.w[2] = v.z; c.w[3] = v.w;
  } else if constexpr (BITS == 8) {
    const u32x4 a = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    const u32x4 b = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p + 4));
    c.w[0] = a.x; c.w[1] = a.y; c.w[2] = a.z; c.w[3] = a.w;
    c.w[4] = b.x; c.w[5] = b.y; c.w[6] = b.z; c.w[7] = b.w;
  } else if constexpr (BITS == 2) {
    const u32x2 v = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p));
    c.w[0] = v.x; c.w[1] = v.y;
  } else {  // 12 B: a 3-dword vector load (global_load_dwordx3 nt; only 4-byte alignment needed)
    typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
    const u32x3 v = __builtin_nontemporal_load(reinterpret_cast<const u32x3*>(p));
    c.w[0] = v.x; c.w[1] = v.y; c.w[2] = v.z;
  }
  return c;
}

// int3 high-bit word rotation per k-step (oracle/quant_oracle.py RHO3)
__host__ __device__ constexpr int rho3(int s) { return s == 0 ? 0 : s == 1 ? 1 : s == 2 ? 8 : 9; }

// fp16 offset of pair P (codes j = 2P, 2P+1) of a k-step
template <int BITS> __host__ __device__ constexpr int pair_off(int P) {
  return BITS == 8 ? 1024 : BITS == 4 ? ((P & 1) ? 64 : 1024)
                                      : (P == 0 ? 1024 : P == 1 ? 256 : P == 2 ? 64 : 16);
}

// An fp16-pair constant kept in a VGPR.  gfx9 VOP3 has no literal operand, so with the constant
// opaque to the optimiser `(w & mask) | magic` selects ONE v_and_or_b32 (mask from an SGPR).  The
// value is pinned by an EMPTY asm with a VGPR constraint: no instruction comes from asm, so the
// compiler's hazard recognizer sees every instruction it schedules (an asm-emitted VALU write is
// opaque to it -- e.g. the wait states before overwriting an in-flight MFMA's source registers).
__device__ __forceinline__ uint32_t pin_v(uint32_t x) {
  asm("" : "+v"(x));
  return x;
}
template <uint32_t C>
__device__ __forceinline__ uint32_t vreg() {
  return pin_v(C);
}
struct Magics {
  uint32_t m1024, m256, m64, m16;
};
template <int BITS>
__device__ __forceinline__ Magics make_magics() {
  Magics g;
  g.m1024 = vreg<0x64006400u>();
  g.m64 = (BITS != 8) ? vreg<0x54005400u>() : 0u;
  g.m256 = (BITS == 2 || BITS == 3) ? vreg<0x5C005C00u>() : 0u;
  g.m16 = (BITS == 2 || BITS == 3) ? vreg<0x4C004C00u>() : 0u;
  return g;
}

// raw (off + u) fp16 pairs of k-step S of a lane piece: v[P] = pair (j = 2P, 2P+1)
template <int BITS, int S>
__device__ __forceinline__ void step_pairs(const Piece<BITS>& c, const Magics& g, uint32_t (&v)[4]) {
  if constexpr (BITS == 4) {
    const uint32_t w = c.w[S];
    const uint32_t w8 = w >> 8;
    v[0] = (w & 0x000F000Fu) | g.m1024;
    v[1] = (w & 0x00F000F0u) | g.m64;
    v[2] = (w8 & 0x000F000Fu) | g.m1024;
    v[3] = (w8 & 0x00F000F0u) | g.m64;
  } else if constexpr (BITS == 8) {
    const uint32_t a = c.w[2 * S], b = c.w[2 * S + 1];
    v[0] = (a & 0x00FF00FFu) | g.m1024;
    v[1] = ((a >> 8) & 0x00FF00FFu) | g.m1024;
    v[2] = (b & 0x00FF00FFu) | g.m1024;
    v[3] = ((b >> 8) & 0x00FF00FFu) | g.m1024;
  } else if constexpr (BITS == 2) {
    const uint32_t w = (S & 1) ? (c.w[S >> 1] >> 8) : c.w[S >> 1];
    v[0] = (w & 0x00030003u) | g.m1024;
    v[1] = (w & 0x000C000Cu) | g.m256;
    v[2] = (w & 0x00300030u) | g.m64;
    v[3] = (w & 0x00C000C0u) | g.m16;
  } else {
    // int3: the (rotated) high-bit word h holds pair P's third bit at bit 2P + 2 of each half,
    // right above its 2-bit field in w.  Pairs 0 and 2 (fields at bits 0-1, 4-5) and pairs 1 and 3
    // (2-3, 6-7) each take their fields from w and their high bits from h in ONE bitfield insert
    // (v_bfi_b32: the bits outside the mask come from h; those no field reads are masked away
    // below), then one v_and_or_b32 per pair: 6 VALU per k-step instead of 8.  The merged words
    // are pinned so the masks are not pushed back into AND / AND / OR3.
    const uint32_t w = (S & 1) ? (c.w[S >> 1] >> 8) : c.w[S >> 1];
    const uint32_t h = (rho3(S) == 0) ? c.w[2] : __builtin_amdgcn_alignbit(c.w[2], c.w[2], rho3(S));
    const uint32_t w02 = pin_v((w & 0x00330033u) | (h & ~0x00330033u));
    const uint32_t w13 = pin_v((w & 0x00CC00CCu) | (h & ~0x00CC00CCu));
    v[0] = (w02 & 0x00070007u) | g.m1024;
    v[1] = (w13 & 0x001C001Cu) | g.m256;
    v[2] = (w02 & 0x00700070u) | g.m64;
    v[3] = (w13 & 0x01C001C0u) | g.m16;
  }
}

// packed (scale, zero) word of the qsz array [ceil(N/16), G, 16]: fp16 scale in bits 0..15,
// int16 zero point in bits 16..31
__device__ __forceinline__ int64_t sz_index(int64_t nt, int g, int G, int n) {
  return (nt * G + g) * kTileN + n;
}
__device__ __forceinline__ _Float16 sz_scale(uint32_t w) {
  return __builtin_bit_cast(_Float16, (uint16_t)(w & 0xFFFFu));
}
__device__ __forceinline__ int sz_zero(uint32_t w) { return (int)(int16_t)(w >> 16); }
__device__ __forceinline__ uint32_t sz_pack(_Float16 s, int z) {
  return (uint32_t)__builtin_bit_cast(uint16_t, s) | ((uint32_t)(uint16_t)(int16_t)z << 16);
}

// zero-point modes of a packed matrix (layout flags, include/qlin_gfx950.h):
//   kZNarrow  int16 zero, |zp| <= 1024: (off + u) - (off + zp) is the exact integer u - zp
//   kZWide    int16 zero, |zp| > 1024 somewhere (QLIN_WIDE_ZERO): u - zp formed in fp32
//   kZFloat   fp16 zero (QLIN_FLOAT_ZERO, HQQ checkpoints): u - zp rounded once in fp16, as
//             hqq's ((W_q - zero) * scale) in the compute dtype
constexpr int kZNarrow = 0;
constexpr int kZWide = 1;
constexpr int kZFloat = 2;

// per-group dequant constants for the exact path
struct GroupQ {
  h2 ss;     // (s, s)
  h2 zz[4];  // (off_P + zp) pairs, narrow zeros; (zp, zp) in zz[0], float zeros
  float zf;  // zp, wide zeros
};

template <int BITS, int ZM>
__device__ __forceinline__ GroupQ make_group(_Float16 s, int zp) {
  GroupQ g;
  g.ss = h2{s, s};
  if constexpr (ZM == kZNarrow) {
#pragma unroll
    for (int P = 0; P < 4; ++P) {
      const _Float16 z = (_Float16)(pair_off<BITS>(P) + zp);  // exact: |zp| <= 1024
      g.zz[P] = h2{z, z};
    }
  } else {
    g.zf = (float)zp;
  }
  return g;
}

// the same straight from a qsz word, in fp16 arithmetic: int16 -> fp16 is exact for |zp| <= 2048
// and off + zp is exact for |zp| <= 1024 (narrow), so no int -> fp32 -> fp16 round trip
template <int BITS, int ZM>
__device__ __forceinline__ GroupQ make_group_w(uint32_t w) {
  if constexpr (ZM == kZWide) return make_group<BITS, kZWide>(sz_scale(w), sz_zero(w));
  GroupQ g;
  const _Float16 s = sz_scale(w);
  g.ss = h2{s, s};
  if constexpr (ZM == kZFloat) {
    const _Float16 z = __builtin_bit_cast(_Float16, (uint16_t)(w >> 16));
    g.zz[0] = h2{z, z};
  } else {
    const _Float16 z = (_Float16)(int16_t)(w >> 16);
#pragma unroll
    for (int P = 0; P < 4; ++P)
      g.zz[P] = h2{z, z} + h2{(_Float16)pair_off<BITS>(P), (_Float16)pair_off<BITS>(P)};
  }
  return g;
}

// exact dequantized fp16 values of k-step S: out[P] = (w_2P, w_2P+1) = RN16(RN16(u - zp) * s)
template <int BITS, int ZM, int S>
__device__ __forceinline__ void dequant_step(const Piece<BITS>& c, const Magics& mg, const GroupQ& g,
                                             uint32_t (&out)[4]) {
#pragma clang fp contract(off)
  uint32_t v[4];
  step_pairs<BITS, S>(c, mg, v);
#pragma unroll
  for (int P = 0; P < 4; ++P) {
    const h2 q = as_h2(v[P]);
    h2 d;
    if constexpr (ZM == kZNarrow) {
      d = q - g.zz[P];  // exact integer u - zp
    } else if constexpr (ZM == kZFloat) {
      // (off + u) - off is the exact code u; minus the fp16 zero rounds once (hqq: W_q - zero)
      const _Float16 off = (_Float16)pair_off<BITS>(P);
      d = (q - h2{off, off}) - g.zz[0];
    } else {
      // |zp| > 1024 (up to 1e4, QLIN_WIDE_ZERO): u - zp formed exactly in fp32, rounded once to
      // fp16 as the reference's fp16 x_int.sub(round_zero_point) does
      const float off = (float)pair_off<BITS>(P);
      const float lo = ((float)q.x - off) - g.zf;
      const float hi = ((float)q.y - off) - g.zf;
      d = h2{(_Float16)lo, (_Float16)hi};
    }
    out[P] = as_u32(d * g.ss);
  }
}

// ---------------------------------------------------------------------------------------------
// the reference quantizer's arithmetic (quant/quantizer.py), shared by the quantizer kernels and
// the GEMV's fused per-token activation fake-quant
// ---------------------------------------------------------------------------------------------
struct QP {
  int64_t rows;
  int K, group, cpr, cpg, rpb, bits, flags;
  float qmin, qmax;
};

// (scale, zp) of one group — quant/quantizer.py:141-159
template <typename T>
__device__ __forceinline__ void calib(float xmin, float xmax, float up, float low, const QP& P,
                                      float& scale, float& zp) {
#pragma clang fp contract(off)
  using E = Elt<T>;
  if (P.flags & QLIN_LWC) {
    xmax = E::rn(up * xmax);
    xmin = E::rn(low * xmin);
  }
  if (P.flags & QLIN_SYMMETRIC) {
    const float am = max_nan(fabsf(xmax), fabsf(xmin));
    scale = E::rn(am / (float)((1 << (P.bits - 1)) - 1));
    scale = E::rn(clamp_nan(scale, 1e-5f, 1e4f));
    zp = (float)((1 << (P.bits - 1)) - 1);
  } else {
    const float range = E::rn(xmax - xmin);
    scale = E::rn(range / (float)((1 << P.bits) - 1));
    scale = E::rn(clamp_nan(scale, 1e-5f, 1e4f));
    zp = E::rn(-xmin / scale);
  }
  zp = rintf(E::rn(clamp_nan(zp, -1e4f, 1e4f)));
}

// fake_quant of one element — quant/quantizer.py:103-110 (round_ste forward = (r - v) + v)
template <typename T>
__device__ __forceinline__ float fq(float x, float s, float zp, bool has_zp, const QP& P,
                                    float& xi_out) {
#pragma clang fp contract(off)
  using E = Elt<T>;
  const float v = E::rn(x / s);
  const float r = rintf(v);
  float xi = E::rn(E::rn(r - v) + v);
  if (has_zp) xi = E::rn(xi + zp);
  xi = clamp_nan(xi, P.qmin, P.qmax);
  xi_out = xi;
  float d = xi;
  if (has_zp) d = E::rn(d - zp);
  return E::rn(d * s);
}

// ---------------------------------------------------------------------------------------------
// wave64 reductions (DPP within 16-lane rows, then the four row totals)
// ---------------------------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                                              0xF, 0xF, false));
}

// every lane of each 16-lane row ends with that row's total
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);  // row_half_mirror
  v += dpp_f<0x140>(v);  // row_mirror
  return v;
}

// v_permlane32_swap / v_permlane16_swap (gfx950): x <-> y exchanges across the wave halves / the
// odd and even 16-lane rows, VALU only (no LDS round trip).  With both operands the same value
// hipcc (ROCm 7.2) folds the builtin's two results into one, so y is an opaque copy (pin_v, an
// empty asm: the swap itself and its hazard wait states come from the compiler).
// After permlane32_swap(x, y) with x = y = v: x = v[l % 32], y = v[l % 32 + 32]; after
// permlane16_swap likewise for the even / odd row of each pair of 16-lane rows.
__device__ __forceinline__ void permlane32_swap(float& x, float& y) {
  const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(uint32_t, x),
                                                  pin_v(__builtin_bit_cast(uint32_t, y)), false, false);
  x = __builtin_bit_cast(float, (uint32_t)r[0]);
  y = __builtin_bit_cast(float, (uint32_t)r[1]);
}
__device__ __forceinline__ void permlane16_swap(float& x, float& y) {
  const auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(uint32_t, x),
                                                  pin_v(__builtin_bit_cast(uint32_t, y)), false, false);
  x = __builtin_bit_cast(float, (uint32_t)r[0]);
  y = __builtin_bit_cast(float, (uint32_t)r[1]);
}
// sum over lanes n, n + 16, n + 32, n + 48 (every lane gets its column's total)
__device__ __forceinline__ float cols4_sum(float v) {
  float x = v, y = v;
  permlane32_swap(x, y);
  v = x + y;
  x = v;
  y = v;
  permlane16_swap(x, y);
  return x + y;
}
// sum over all 64 lanes, every lane gets it (16-lane rows by DPP, then the row exchanges)
__device__ __forceinline__ float wave_sum(float v) { return cols4_sum(row16_sum(v)); }

// output epilogues of the packed linear (qlin_linear_ep_f16); the accumulator (+ bias) is first
// rounded to fp16 exactly as F.linear's output, then
//   kEpResidual  y = RN16(residual + that)           (the decoder layer's `residual + h`)
//   kEpSiluMul   rows interleaved in 8-row halves (gate rows 8j..8j+7 at tile rows 0-7, up rows
//                at 8-15 of output tile j): y[:, 8j + n] = RN16(RN16(silu(gate)) * up), N/2 cols
//                (QuantLlamaMLP's act_fn(gate_proj(x)) * up_proj(x))
constexpr int kEpNone = 0;
constexpr int kEpResidual = 1;
constexpr int kEpSiluMul = 2;

// the GEMV kernel with an output epilogue (qlin_gemv.hip), for qlin_linear_ep_f16
// (act_bits != 0: per-token activation fake-quant of x with the quantizer flags act_flags)
int gemv_ep(const uint32_t* qweight, const uint32_t* qsz, int flags, const uint16_t* x,
            const uint16_t* bias, const uint16_t* residual, uint16_t* y, int64_t M, int64_t N,
            int64_t K, int bits, int group, int epilogue, int act_bits, int act_flags,
            void* stream);

// CUs of the current device, cached per device id (qlin_gemm.hip; used by the GEMM's block-width
// picker and the batched GEMV's resident-grid size)
int device_cu_count();

// torch's fp32 silu (x / (1 + exp(-x))) on an fp16 value, rounded to fp16
__device__ __forceinline__ float silu_rn16(float g) {
#pragma clang fp contract(off)
  return (float)(_Float16)(g / (1.0f + expf(-g)));
}

}  // namespace qlin

// zero mode from the layout flags (QLIN_FLOAT_ZERO wins: an fp16 zero is never "wide")
__host__ __device__ inline int zero_mode(int flags) {
  return (flags & QLIN_FLOAT_ZERO) ? qlin::kZFloat
         : (flags & QLIN_WIDE_ZERO) ? qlin::kZWide : qlin::kZNarrow;
}
