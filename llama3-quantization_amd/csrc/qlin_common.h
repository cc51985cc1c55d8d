// qlin_common.h — device helpers shared by the gfx950 quantized-linear kernels.
//
// Written for CDNA4 (gfx950, wave64) only.  The fp16 unpack uses the "magic number" form: a code u
// placed in the low mantissa bits of 0x6400 (= 1024.0h) gives the fp16 value 1024 + u exactly, so
// (1024 + u) - (1024 + zp) is the exact integer u - zp in fp16 (Sterbenz), and one v_pk_mul_f16 by
// the group scale rounds once — bit-identical to the reference's fp16
// x_dequant.sub(round_zero_point).mul(scale) (quant/quantizer.py:107-110).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace qlin {

typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

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
// canonical layout: one 32-element lane chunk = BITS uint32 words
// ---------------------------------------------------------------------------------------------
template <int BITS> struct Chunk { uint32_t w[BITS]; };

template <int BITS>
__device__ __forceinline__ Chunk<BITS> load_chunk(const uint32_t* __restrict__ p) {
  Chunk<BITS> c;
  if constexpr (BITS == 4) {
    uint4 v = *reinterpret_cast<const uint4*>(p);
    c.w[0] = v.x; c.w[1] = v.y; c.w[2] = v.z; c.w[3] = v.w;
  } else if constexpr (BITS == 8) {
    uint4 a = *reinterpret_cast<const uint4*>(p);
    uint4 b = *reinterpret_cast<const uint4*>(p + 4);
    c.w[0] = a.x; c.w[1] = a.y; c.w[2] = a.z; c.w[3] = a.w;
    c.w[4] = b.x; c.w[5] = b.y; c.w[6] = b.z; c.w[7] = b.w;
  } else if constexpr (BITS == 2) {
    uint2 v = *reinterpret_cast<const uint2*>(p);
    c.w[0] = v.x; c.w[1] = v.y;
  } else {  // BITS == 3: 12 bytes, 4-byte aligned
    struct U3 { uint32_t a, b, c; };
    U3 v = *reinterpret_cast<const U3*>(p);
    c.w[0] = v.a; c.w[1] = v.b; c.w[2] = v.c;
  }
  return c;
}

// 0x64006400 (fp16 pair 1024, 1024) held in a VGPR: gfx9 VOP3 cannot encode a literal, so with
// the constant opaque to the optimiser (w & mask) | magic selects ONE v_and_or_b32 (mask in an
// SGPR) instead of a v_and_b32 + v_or_b32 literal pair.
__device__ __forceinline__ uint32_t magic_vgpr() {
  uint32_t m;
  asm("v_mov_b32 %0, 0x64006400" : "=v"(m));
  return m;
}

// fp16 pair (1024 + u[2p], 1024 + u[2p+1]) of pair index p (0..15) of a chunk, as raw bits
template <int BITS, int P>
__device__ __forceinline__ uint32_t magic_pair(const Chunk<BITS>& c, uint32_t magic) {
  static_assert(P >= 0 && P < 16, "pair index");
  if constexpr (BITS == 4) {
    return ((c.w[P >> 2] >> (4 * (P & 3))) & 0x000F000Fu) | magic;
  } else if constexpr (BITS == 8) {
    return ((c.w[P >> 1] >> (8 * (P & 1))) & 0x00FF00FFu) | magic;
  } else if constexpr (BITS == 2) {
    return ((c.w[P >> 3] >> (2 * (P & 7))) & 0x00030003u) | magic;
  } else {
    const uint32_t lo = ((c.w[P >> 3] >> (2 * (P & 7))) & 0x00030003u) | magic;
    uint32_t hi;
    if constexpr (P >= 2) hi = c.w[2] >> (P - 2);
    else hi = c.w[2] << (2 - P);
    return (hi & 0x00040004u) | lo;
  }
}

// per-group dequant constants
struct GroupQ {
  uint32_t magic;  // 0x64006400 in a VGPR
  h2 ss;    // (s, s)
  h2 zz;    // (1024 + zp, 1024 + zp)   narrow zeros
  float zf; // zp                       wide zeros
};

template <bool WIDE>
__device__ __forceinline__ GroupQ make_group(_Float16 s, int zp) {
  GroupQ g;
  g.magic = magic_vgpr();
  g.ss = h2{s, s};
  if constexpr (!WIDE) {
    const _Float16 z = (_Float16)(1024 + zp);  // exact: |zp| <= 128
    g.zz = h2{z, z};
  } else {
    g.zf = (float)zp;
  }
  return g;
}

// dequantized fp16 pair P of a chunk: RN16(RN16(u - zp) * s), bit-exact with the reference
template <int BITS, bool WIDE, int P>
__device__ __forceinline__ h2 dequant_pair(const Chunk<BITS>& c, const GroupQ& g) {
#pragma clang fp contract(off)
  const h2 q = as_h2(magic_pair<BITS, P>(c, g.magic));
  h2 d;
  if constexpr (!WIDE) {
    d = q - g.zz;  // exact integer u - zp
  } else {
    // |zp| up to 1e4: u - zp is formed exactly in fp32 and rounded once to fp16, as the
    // reference's fp16 x_int.sub(round_zero_point) does
    const float lo = ((float)q.x - 1024.0f) - g.zf;
    const float hi = ((float)q.y - 1024.0f) - g.zf;
    d = h2{(_Float16)lo, (_Float16)hi};
  }
  return d * g.ss;
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

// wave-uniform total over all 64 lanes (requires EXEC all ones)
__device__ __forceinline__ float wave_sum(float v) {
  v = row16_sum(v);
  const int b = __builtin_bit_cast(int, v);
  return (__builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 0)) +
          __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 16))) +
         (__builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 32)) +
          __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 48)));
}

}  // namespace qlin

// error codes (hipError_t values)
#define QLIN_OK 0
#define QLIN_EINVAL 1
